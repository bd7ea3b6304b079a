# fp32 forward past 128 channels: its parity cases and the other wide-channel cases, then the d = 256 timings
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "wide_channels" > gpurun_out/r04/wide_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r04/wide_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python tools/wide_time.py > gpurun_out/r04/wide_time.json 2> gpurun_out/r04/wide_time.err
rc=$?; cat gpurun_out/r04/wide_time.json; tail -3 gpurun_out/r04/wide_time.err; exit $rc
