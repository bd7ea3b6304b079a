#!/bin/bash
# Builds the diagnostic library with the one-wave gap-stream forward's stamps (tools/stamp/gap_stamp_patch.py;
# outputs of variant 2600 WRONG), twice: tools/stamp/build_gap/libfa_hip_diag.so (step edges only) and
# libfa_hip_diag_gaps.so (plus the per-gap stamps of one step).  Run on the CPU container; the .so files
# travel with the tree.  Read with tools/stamp/gap_stamps.py [gaps] on the GPU.
set -e
cd "$(dirname "$0")"
rm -rf build_gap && mkdir -p build_gap/pkg
cp -r ../../include build_gap/include
cp -r ../../tf_flash_attention_amd/csrc ../../tf_flash_attention_amd/Makefile build_gap/pkg/
cp ../../tf_flash_attention_amd/csrc/diag/fa_fwd_f16_gap.hip build_gap/gap_orig.hip
python3 gap_stamp_patch.py build_gap/pkg
make -s -C build_gap/pkg -j8 diag 2>&1 | grep -v -i warning | grep -E 'error|Error' && exit 1 || true
mv build_gap/pkg/libfa_hip_diag.so build_gap/libfa_hip_diag.so
cp build_gap/gap_orig.hip build_gap/pkg/csrc/diag/fa_fwd_f16_gap.hip
python3 gap_stamp_patch.py build_gap/pkg gaps
make -s -C build_gap/pkg -j8 diag 2>&1 | grep -v -i warning | grep -E 'error|Error' && exit 1 || true
mv build_gap/pkg/libfa_hip_diag.so build_gap/libfa_hip_diag_gaps.so
rm -rf build_gap/pkg/build_diag
ls -la build_gap/*.so
