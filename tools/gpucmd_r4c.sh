set -o pipefail
ROUNDS=4 timeout -k 10 300 python -u tools/fwd_variants.py c4 -1 2424 2422 > gpurun_out/var_c4.txt 2>&1; rc=$?; cat gpurun_out/var_c4.txt; [ $rc -eq 0 ] || exit $rc
FA_FWD_VARIANT=2424 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "band_forward_persistent or local_band" > gpurun_out/t_band.log 2>&1
rc=$?; tail -2 gpurun_out/t_band.log
