#!/bin/bash
# Builds the diagnostic library with the one-wave D = 128 gap-stream forward's stamps
# (tools/stamp/gap128_stamp_patch.py; outputs of variant 2700 WRONG), twice: tools/stamp/build_gap128/libfa_hip_diag.so (step edges only) and
# libfa_hip_diag_gaps.so (plus the per-gap stamps of one step).  Run on the CPU container; the .so files
# travel with the tree.  Read with tools/stamp/gap128_stamps.py [gaps] on the GPU.
set -e
cd "$(dirname "$0")"
rm -rf build_gap128 && mkdir -p build_gap128/pkg
cp -r ../../include build_gap128/include
cp -r ../../tf_flash_attention_amd/csrc ../../tf_flash_attention_amd/Makefile build_gap128/pkg/
cp ../../tf_flash_attention_amd/csrc/fa_fwd_f16_gap128.hip build_gap128/gap128_orig.hip
python3 gap128_stamp_patch.py build_gap128/pkg
make -s -C build_gap128/pkg -j8 diag 2>&1 | grep -v -i warning | grep -E 'error|Error' && exit 1 || true
mv build_gap128/pkg/libfa_hip_diag.so build_gap128/libfa_hip_diag.so
cp build_gap128/gap128_orig.hip build_gap128/pkg/csrc/fa_fwd_f16_gap128.hip
python3 gap128_stamp_patch.py build_gap128/pkg gaps
make -s -C build_gap128/pkg -j8 diag 2>&1 | grep -v -i warning | grep -E 'error|Error' && exit 1 || true
mv build_gap128/pkg/libfa_hip_diag.so build_gap128/libfa_hip_diag_gaps.so
rm -rf build_gap128/pkg/build_diag
ls -la build_gap128/*.so
