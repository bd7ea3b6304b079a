set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/sw_probe > gpurun_out/r5_sw_probe.txt 2>&1 && \
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "reference_shapes or wide_channels_mfma_forward or d128 or config3 or mfma_shapes" > gpurun_out/r5_tests_b.log 2>&1 && \
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 > gpurun_out/r5_bench_c3_pair.json 2> gpurun_out/r5_bench_c3_pair.err
