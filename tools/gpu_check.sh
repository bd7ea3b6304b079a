#!/bin/bash
# GPU validation run: parity tests, smoke, short bench.  Stops at the first
# step that faults / aborts / times out (exit codes other than 0 or 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local c=$1; [ "$c" -eq 0 ] || [ "$c" -eq 1 ]; }
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu -q"}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest $PYTEST_ARGS > gpurun_out/pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -5 gpurun_out/pytest.log
ok $c || exit $c
if [ -z "$SKIP_SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  c=$?; echo "smoke exit $c"; tail -3 gpurun_out/smoke.log
  ok $c || exit $c
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --cpu-budget 8} > gpurun_out/bench.log 2>&1
  c=$?; echo "bench exit $c"; tail -3 gpurun_out/bench.log
fi
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py ${PROFILE_ARGS:---steps 10 --warmup 3 --no-cpu-baseline} > gpurun_out/prof.log 2>&1
  c=$?; echo "profile exit $c"; tail -3 gpurun_out/prof.log
fi
exit 0
