"""Writes a stamp copy of csrc/diag/fa_fwd_f16_gap.hip (the one-wave gap-stream c2 forward, FA_FWD_VARIANT
2600): s_memtime of every wave of workgroups 0 and gridDim/2 at six edges of each key step (before / after
the step barrier, after segment A, after block B's rebase check, after segment B, after block A's check),
and — wave 0 of workgroup 0, step GAP_STEP only — after every one of the step's 32 gap statements.  The
stamps are written over the last slice's Q (outputs WRONG).  Measurement only: never built into the product
or diagnostic library (tools/stamp/gap_stamp.sh builds a separate copy).
Usage: python tools/stamp/gap_stamp_patch.py PKG_DIR [gaps]   (gaps: the per-gap stamps too; they keep 32 SGPRs
live across the loop, which spills SGPRs, so the step timeline is read from the build without them)"""
import sys

GAPS = len(sys.argv) > 2 and sys.argv[2] == "gaps"

p = f"{sys.argv[1]}/csrc/diag/fa_fwd_f16_gap.hip"
s = open(p).read()


def sub(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)


# stamp state: the buffer, which workgroup / wave records, the per-gap stamps of one step (SGPR pairs)
sub("""  Blk A, B;
  auto init_blk""", """  constexpr int kGapStep = 20, kNStep = 64;
  constexpr bool GAPS = """ + ("true" if GAPS else "false") + """;
  uint64_t* dbg = reinterpret_cast<uint64_t*>(const_cast<void*>(a.Q)) + (a.b - 1) * (int64_t)d * nq / 4;
  const int sel = blockIdx.x == 0 ? 0 : (blockIdx.x == gridDim.x / 2 ? 1 : -1);
  uint32_t gst[16];  // one segment's gaps (low halves)
  int cur_it = 0;
  auto stamp = [&](int it, int k) __attribute__((always_inline)) {
    if (sel >= 0 && it < kNStep) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      if (lane == 0) dbg[((sel * kNW + w) * kNStep + it) * 6 + k] = t;
    }
  };
  auto gstamp = [&](int j) __attribute__((always_inline)) {
    // (defined in every segment, stored after it: the stamps are not live across the loop)
    // (unconditional in every wave and step: a per-gap branch on the step number cost ~30 cycles a gap)
    if (GAPS) gst[j & 15] = (uint32_t)__builtin_amdgcn_s_memtime();
  };
  Blk A, B;
  auto init_blk""")
# per-gap stamps
sub("""      gap(A, B, IC<0>{}, G_);
      if constexpr (g < 2""", """      gap(A, B, IC<0>{}, G_);
      gstamp(g);
      if constexpr (g < 2""")
sub("""      gap(B, A, IC<1>{}, G_);
""", """      gap(B, A, IC<1>{}, G_);
      gstamp(16 + g);
""")
# step edges
sub("""    if constexpr (!(ABL & kANoBar)) __builtin_amdgcn_s_barrier();
    const int k0 = it * kBN;
    if (k0 + kBN > nk) mask(B, k0);
    seg_a(C_);
    check(B, IC<1>{});
    if (k0 + 2 * kBN > nk) mask(A, k0 + kBN);
    seg_b(C_, it);
    check(A, IC<0>{});""", """    cur_it = it;
    stamp(it, 0);
    if constexpr (!(ABL & kANoBar)) __builtin_amdgcn_s_barrier();
    stamp(it, 1);
    const int k0 = it * kBN;
    if (k0 + kBN > nk) mask(B, k0);
    seg_a(C_);
    stamp(it, 2);
    if (GAPS && sel == 0 && w == 0 && it == kGapStep && lane == 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) dbg[2 * kNW * kNStep * 6 + j] = gst[j];
    }
    check(B, IC<1>{});
    stamp(it, 3);
    if (k0 + 2 * kBN > nk) mask(A, k0 + kBN);
    seg_b(C_, it);
    stamp(it, 4);
    if (GAPS && sel == 0 && w == 0 && it == kGapStep && lane == 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) dbg[2 * kNW * kNStep * 6 + 16 + j] = gst[j];
    }
    check(A, IC<0>{});
    stamp(it, 5);
""")
open(p, "w").write(s)
