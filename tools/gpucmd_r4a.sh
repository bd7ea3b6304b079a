set -o pipefail
timeout -k 10 120 ./tools/rotation_probe > gpurun_out/rot.txt 2>&1 || exit 1
cat gpurun_out/rot.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "trio" > gpurun_out/t_trio.log 2>&1
rc=$?; tail -5 gpurun_out/t_trio.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=4 timeout -k 10 200 python -u tools/fwd_variants.py c2 -1 2501 2504 2505 2507 2508 > gpurun_out/var.txt 2>&1; rc=$?; cat gpurun_out/var.txt; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 timeout -k 10 150 python -u tools/fwd_variants.py d32 -1 2501 2505 2507 2508 > gpurun_out/var32.txt 2>&1; rc=$?; cat gpurun_out/var32.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -u tools/trio_stamps.py c2 2509 > gpurun_out/stamps.txt 2>&1; rc=$?; cat gpurun_out/stamps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "backward_read_placement or band" > gpurun_out/t1.log 2>&1; tail -3 gpurun_out/t1.log
