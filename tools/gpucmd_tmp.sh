set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "wide_channels_mfma_backward" > gpurun_out/gpu_w4.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_w4.log; [ $rc -eq 0 ] || exit $rc
FA_HIP_LIB=$PWD/tf_flash_attention_amd/libfa_hip_diag.so timeout -k 10 400 python tools/bwd_variants.py w256b -1 1421 > gpurun_out/r05/w4_ab.txt 2>&1; rc=$?; tail -5 gpurun_out/r05/w4_ab.txt; exit $rc
