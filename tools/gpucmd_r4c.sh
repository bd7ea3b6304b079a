set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -k "band or local or c4" > gpurun_out/t_band.log 2>&1
rc=$?; tail -2 gpurun_out/t_band.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=4 timeout -k 10 300 python -u tools/fwd_variants.py c4 -1 2424 > gpurun_out/var_c4.txt 2>&1; rc=$?; cat gpurun_out/var_c4.txt
