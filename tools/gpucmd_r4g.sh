# fp32 backward past 128 channels (parity), then the inline-asm LDS-DMA c2 variants (parity, timing)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "wide_channels" > gpurun_out/r04/wide_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04/wide_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/variant_parity.py c2 -1 2230 2231 2232 > gpurun_out/r04/dma_par2.json 2>&1
rc=$?; cat gpurun_out/r04/dma_par2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/fwd_variants.py c2 -1 2218 2230 2231 2232 > gpurun_out/r04/dma_c2b.json 2>&1
rc=$?; cat gpurun_out/r04/dma_c2b.json; exit $rc
