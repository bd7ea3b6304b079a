#!/bin/bash
# GPU side: time each ablation variant with bench.py (c2 forward), interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2; do
  for so in tools/ablate_out/libfa_*.so; do
    v=$(basename $so .so)
    r=$(FA_HIP_LIB=$PWD/$so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${ABL_ARGS} 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['event_ms_per_launch'], d['value'])")
    c=$?
    echo "round $round $v: $r"
    [ $c -eq 0 ] || exit $c
  done
done
