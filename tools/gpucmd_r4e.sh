# wide-channel backward: its parity cases first, then the whole -m gpu suite, then forward / backward timing at d = 256
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "wide_channels_mfma_backward" > gpurun_out/r04/wide_bwd_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r04/wide_bwd_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python tools/wide_time.py > gpurun_out/r04/wide_time.json 2> gpurun_out/r04/wide_time.err
rc=$?; cat gpurun_out/r04/wide_time.json; tail -3 gpurun_out/r04/wide_time.err; exit $rc
