# round-4 final measurement, part 2: SQ counters (c2, c3, c4), the d = 256 configs' traces and traffic,
# and the 2-rank batch-shard rehearsal of bench.py on this one GPU
set -o pipefail
CONFIGS="c2 c3 c4" bash tools/pmc_round.sh || exit 1
ROUND=r04 CONFIGS="w256 w256b" bash tools/profile_round.sh || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 300 python bench.py --gpus 2 --config c2 --steps 20 > gpurun_out/r04/c2_bench_2ranks_1gpu.json 2> gpurun_out/r04/shard.err
rc=$?; cat gpurun_out/r04/c2_bench_2ranks_1gpu.json; exit $rc
