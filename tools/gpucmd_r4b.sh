set -o pipefail
ROUNDS=3 timeout -k 10 200 python -u tools/fwd_variants.py c2 -1 2501 2510 2511 2512 2500 > gpurun_out/var.txt 2>&1; rc=$?; cat gpurun_out/var.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -u tools/trio_stamps.py c2 2513 > gpurun_out/stamps.txt 2>&1; rc=$?; cat gpurun_out/stamps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -u tools/trio_stamps.py c2 2514 > gpurun_out/stamps2.txt 2>&1; rc=$?; cat gpurun_out/stamps2.txt
