set -o pipefail
cd $GRAFT_REPO_ROOT
ROUNDS=4 timeout -k 10 200 python tools/fwd_variants.py c2 -1 2000 > gpurun_out/r5_c2_pp_ab.txt 2>&1 && \
timeout -k 10 100 python tools/pp_stamps.py c2 2132 > gpurun_out/r5_pp_stamps.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "forward_structures and not d128" > gpurun_out/r5_pp_tests.log 2>&1
