set -o pipefail
cd $GRAFT_REPO_ROOT
ROUNDS=3 timeout -k 10 300 python tools/fwd_variants.py c2 -1 2000 2101 2102 2104 2108 2116 2164 2111 2175 > gpurun_out/r5_pp_abl.txt 2>&1
