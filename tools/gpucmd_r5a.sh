set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/shape_probe > gpurun_out/r5_shape_probe.txt 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r5_bench_c2_start.json 2> gpurun_out/r5_bench_c2_start.err
