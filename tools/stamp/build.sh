#!/bin/bash
# Builds tools/stamp/build/libfa_hip_stamp.so: the product sources with the band kernel's phase stamps
# (tools/stamp/band_stamp_patch.py).  Run on the CPU container; the .so travels with the tree.
set -e
cd "$(dirname "$0")"
rm -rf build && mkdir -p build
python3 band_stamp_patch.py ../../tf_flash_attention_amd/csrc build/pkg/csrc
cp -r ../../include build/include  # (csrc includes ../../include/fa_api.h)
cd build/pkg
for f in csrc/*.hip; do
  extra=""
  case $(basename $f) in fa_bwd_f16_fast.hip|fa_fwd_f16_fast.hip|fa_fwd_f16_wide.hip|fa_fwd_f32_wide.hip|fa_bwd_f32_wide.hip) extra="-mllvm -amdgpu-mfma-vgpr-form=1";; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -fno-honor-nans -w $extra \
    -DFA_SRC_HASH=\"stamp\" -I../include -c $f -o ${f%.hip}.o || exit 1 &
  while [ $(jobs -r | wc -l) -ge 8 ]; do sleep 1; done
done
wait
[ $(ls csrc/*.o | wc -l) -eq $(ls csrc/*.hip | wc -l) ] || { echo 'stamp build: a source failed'; exit 1; }
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 csrc/*.o -o ../libfa_hip_stamp.so
ls -la ../libfa_hip_stamp.so
