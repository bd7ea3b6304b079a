# Round-end measurement, part 2: SQ counters (c2, c3, c4), the d = 256 configs' traces and traffic, and
# the 2-rank batch-shard rehearsal of bench.py on one GPU.  Usage: ROUND=r05 bash tools/round_end2.sh
set -o pipefail
ROUND=${ROUND:?set ROUND, e.g. r05}
CONFIGS="c2 c3 c4" bash tools/pmc_round.sh || exit 1
ROUND=$ROUND CONFIGS="w256 w256b" bash tools/profile_round.sh || exit 1
mkdir -p gpurun_out/$ROUND
timeout -k 10 300 python bench.py --gpus 2 --config c2 --steps 20 > gpurun_out/$ROUND/c2_bench_2ranks_1gpu.json 2> gpurun_out/$ROUND/shard.err
rc=$?; cat gpurun_out/$ROUND/c2_bench_2ranks_1gpu.json; exit $rc
