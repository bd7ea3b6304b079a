# Round-end measurement, part 1: the whole -m gpu suite, smoke(), then kernel traces + PMC traffic +
# bench lines for the headline configs (tools/profile_round.sh), all from one box and one commit.
# Usage (on the GPU box): ROUND=r05 bash tools/round_end.sh
set -o pipefail
ROUND=${ROUND:?set ROUND, e.g. r05}
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
ROUND=$ROUND CONFIGS="${CONFIGS:-c2 c3 c4 c5 d32}" bash tools/profile_round.sh
