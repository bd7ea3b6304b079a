"""Writes a stamp copy of fa_fwd_f16_band.hip (tools/stamp/build/): s_memtime of waves 0 and 4 of
workgroup 0 at the four phase edges of every position of its first four items, written over the last
slice's Q (outputs WRONG).  Measurement only: never built into the product or diagnostic library.
Usage: python tools/stamp/band_stamp_patch.py SRC_DIR OUT_DIR"""
import shutil
import sys

src, out = sys.argv[1], sys.argv[2]
shutil.copytree(src, out, dirs_exist_ok=True)
p = f"{out}/fa_fwd_f16_band.hip"
s = open(p).read()
old = """    __builtin_amdgcn_s_barrier();
    mfma_phase(IT_);
    __builtin_amdgcn_s_barrier();
    valu_phase(IT_);
  };"""
new = """    auto stamp = [&](int k) __attribute__((always_inline)) {
      if (blockIdx.x == 0 && (w == 0 || w == 4) && lane == 0 && n < 4) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        uint64_t* dbg = reinterpret_cast<uint64_t*>(const_cast<void*>(a.Q)) + (a.b - 1) * (int64_t)d * nq / 4;
        dbg[((n * T + it) * 4 + k) * 2 + (w >> 2)] = t;
      }
    };
    __builtin_amdgcn_s_barrier();
    stamp(0);
    mfma_phase(IT_);
    stamp(1);
    __builtin_amdgcn_s_barrier();
    stamp(2);
    valu_phase(IT_);
    stamp(3);
  };"""
assert s.count(old) == 1
s = s.replace(old, new)
open(p, "w").write(s)
