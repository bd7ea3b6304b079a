#!/bin/bash
# Builds ablation variants of the fp16 forward into tools/ablate_out/libfa_<mask>.so
# (profiling only; never the product).  Usage: tools/ablate.sh 0 1 2 4 8 ...
set -e
cd "$(dirname "$0")/../tf_flash_attention_amd"
make -j8 >/dev/null
mkdir -p ../tools/ablate_out
for m in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -DFA_ABLATE=$m -c csrc/fa_fwd_f16.hip -o ../tools/ablate_out/fwd_$m.o &
done
wait
for m in "$@"; do
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared build/fa_api.o build/fa_generic.o build/fa_f16_stub.o ../tools/ablate_out/fwd_$m.o -o ../tools/ablate_out/libfa_$m.so
done
rm -f ../tools/ablate_out/*.o
