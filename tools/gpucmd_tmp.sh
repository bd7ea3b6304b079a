set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "f64 or wide_channels or tiny or masked or odd_channels" > gpurun_out/gpu_f64.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_f64.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/f64trace -o run -- python3 $GRAFT_REPO_ROOT/tools/dispatch_trace.py f64 > $GRAFT_REPO_ROOT/gpurun_out/f64trace.log 2>&1
rc=$?; tail -2 $GRAFT_REPO_ROOT/gpurun_out/f64trace.log; exit $rc
