# end-of-session check: the whole -m gpu suite and smoke() at this commit, then the default bench line
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r04/bench_end.json 2> gpurun_out/r04/bench_end.err
rc=$?; cat gpurun_out/r04/bench_end.json; exit $rc
