set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/trans_probe > gpurun_out/r5_trans_probe.txt 2>&1 && \
timeout -k 10 120 ./tools/shape_probe > gpurun_out/r5_shape_probe2.txt 2>&1 && \
ROUNDS=6 timeout -k 10 200 python tools/fwd_variants.py c2 -1 2240 2241 > gpurun_out/r5_c2_asm_ab.txt 2>&1 && \
ROUNDS=4 timeout -k 10 200 python tools/fwd_variants.py c4 -1 2440 > gpurun_out/r5_c4_asm_ab.txt 2>&1 && \
timeout -k 10 100 python tools/pingpong_stamps.py c2 2299 > gpurun_out/r5_c2_stamps.txt 2>&1 && \
timeout -k 10 100 python tools/pingpong_stamps.py c2 2242 >> gpurun_out/r5_c2_stamps.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "reference_shapes or wide_channels_mfma_forward or d128 or config3 or mfma_shapes" > gpurun_out/r5_tests_b.log 2>&1 && \
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 > gpurun_out/r5_bench_c3_pair.json 2> gpurun_out/r5_bench_c3_pair.err
