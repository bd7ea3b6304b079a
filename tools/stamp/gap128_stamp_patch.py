"""Writes a stamp copy of csrc/fa_fwd_f16_gap128.hip (the one-wave D = 128 gap-stream forward,
FA_FWD_VARIANT 2700): s_memtime of every wave of workgroups 0 and gridDim/2 at six edges of each of the first
64 key steps of the first block (step start, after the barrier, after segment A, after block B's check and
block A's mask, after segment B, after block A's check) and, with 'gaps', after every second gap statement of
every step (kept for step GAP_STEP of wave 0, workgroup 0).  The stamps are written over the last slice's Q
(outputs WRONG).  Measurement only: never built into the product or diagnostic library.
Usage: python tools/stamp/gap128_stamp_patch.py PKG_DIR [gaps]"""
import sys

GAPS = len(sys.argv) > 2 and sys.argv[2] == "gaps"
p = f"{sys.argv[1]}/csrc/fa_fwd_f16_gap128.hip"
s = open(p).read()


def sub(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)


sub("""  Blk A, B;
""", """  constexpr int kGapStep = 20, kNStep = 64;
  constexpr bool GAPS = """ + ("true" if GAPS else "false") + """;
  uint64_t* dbg = reinterpret_cast<uint64_t*>(const_cast<void*>(a.Q)) + (a.b - 1) * (int64_t)d * nq / 4;
  const int sel = blockIdx.x == 0 ? 0 : (blockIdx.x == gridDim.x / 2 ? 1 : -1);
  uint32_t gst[16];  // one segment's stamps, every second gap (low halves)
  int npass_done = 0;
  auto stamp = [&](int it, int k) __attribute__((always_inline)) {
    if (sel >= 0 && it < kNStep && npass_done == 0) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      if (lane == 0) dbg[((sel * kNW + w) * kNStep + it) * 6 + k] = t;
    }
  };
  // (unconditional in every wave and step: a per-gap branch on the step number costs ~30 cycles)
  auto gstamp = [&](int j) __attribute__((always_inline)) {
    if (GAPS) gst[j] = (uint32_t)__builtin_amdgcn_s_memtime();
  };
  auto gstore = [&](int base, int it) __attribute__((always_inline)) {
    if (GAPS && sel == 0 && w == 0 && it == kGapStep && npass_done == 0 && lane == 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) dbg[2 * kNW * kNStep * 6 + base + j] = gst[j];
    }
  };
  Blk A, B;
""")
assert s.count("""          gap(A, B, G_);
""") == 2
s = s.replace("""          gap(A, B, G_);
""", """          gap(A, B, G_);
          if constexpr (g % 2 == 1) gstamp(g >> 1);
""")
sub("""        gap(B, A, G_);
""", """        gap(B, A, G_);
        if constexpr (g % 2 == 1) gstamp(g >> 1);
""")
sub("""      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      {
        const int cls = tcls(B, it);
        if (cls != 2) mask(B, it, cls);
      }
      seg_a(C_);
      check(B);
      {
        const int cls = tcls(A, it + 1);
        if (cls != 2) mask(A, it + 1, cls);
      }
      seg_b(C_, it);
      check(A);""", """      stamp(it, 0);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      stamp(it, 1);
      {
        const int cls = tcls(B, it);
        if (cls != 2) mask(B, it, cls);
      }
      seg_a(C_);
      stamp(it, 2);
      gstore(0, it);
      check(B);
      {
        const int cls = tcls(A, it + 1);
        if (cls != 2) mask(A, it + 1, cls);
      }
      stamp(it, 3);
      seg_b(C_, it);
      stamp(it, 4);
      gstore(16, it);
      check(A);
      stamp(it, 5);""")
sub("""    finish(A, 0);
    finish(B, 1);
""", """    finish(A, 0);
    finish(B, 1);
    npass_done = 1;
""")
open(p, "w").write(s)
