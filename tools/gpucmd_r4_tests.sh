# round-4 GPU check: the whole -m gpu suite, smoke(), and the 2-rank batch-shard rehearsal of bench.py
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/r04
timeout -k 10 300 python bench.py --gpus 2 --config c2 --steps 20 > gpurun_out/r04/c2_bench_2ranks_1gpu.json 2> gpurun_out/r04/shard.err
rc=$?; cat gpurun_out/r04/c2_bench_2ranks_1gpu.json; exit $rc
