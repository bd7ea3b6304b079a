set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "wide" > gpurun_out/t_wide.log 2>&1
rc=$?; tail -3 gpurun_out/t_wide.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/wide_time.py > gpurun_out/wide_time.txt 2>&1; rc=$?; cat gpurun_out/wide_time.txt
