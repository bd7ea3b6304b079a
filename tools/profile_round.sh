#!/bin/bash
# Per-round profiling evidence for bench.py configs (run on the GPU box).  For each config:
#   1. rocprofv3 --kernel-trace --stats of the bench command
#   2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE: the TCC block can't hold both)
#      -> traffic_<cfg>.json (tools/pmc_traffic.py applies the gfx950 corrections)
#   3. the bench line itself, with roofline.traffic filled from that json
# Everything lands in gpurun_out/<ROUND>/ (the only directory gpurun merges back);
# copy it into profiles/ afterwards with:  bash tools/profile_round.sh --collect
# Usage: ROUND=r01 CONFIGS="c2 c5" bash tools/profile_round.sh
# Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:-r01}
OUT=gpurun_out/$ROUND
if [ "$1" == "--collect" ]; then   # local: keep the summaries, drop the raw traces
  for f in $OUT/*_kernel_stats.csv $OUT/*_bench*.json $OUT/traffic_*.json; do
    [ -f "$f" ] || continue
    case $(basename $f) in traffic_*) cp $f profiles/ ;; *) cp $f profiles/${ROUND}_$(basename $f) ;; esac
  done
  ls -la profiles; exit 0
fi
export TMPDIR=/tmp
mkdir -p $OUT
declare -A REGEX=([c2]=fwd_f16 [c3]="fwd_f16|bwd_dkdv|bwd_dq|bwd_prep" [c4]=fwd_f16 [c5]=fwd_f32_kernel [d32]=fwd_f16 [w256]="fwd_f16|generic" [w256b]="fwd_f16|bwd_dkdv|bwd_dq|bwd_prep|generic")
for cfg in ${CONFIGS:-c2}; do
  rx=${REGEX[$cfg]}
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$cfg -o run \
      -- python3 bench.py --config $cfg --no-cpu-baseline > $OUT/prof_$cfg.log 2>&1
  c=$?; echo "[$cfg] kernel-trace exit $c"; [ $c -eq 0 ] || exit $c
  cp "$(find $OUT/prof_$cfg -name '*kernel_stats.csv' | head -1)" $OUT/${cfg}_kernel_stats.csv
  grep -h '^{' $OUT/prof_$cfg.log > $OUT/${cfg}_bench_under_rocprof.json || true
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv \
        -d $OUT/pmc_$cfg/$ctr -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline \
        > $OUT/pmc_${cfg}_$ctr.log 2>&1
    c=$?; echo "[$cfg] pmc $ctr exit $c"; [ $c -eq 0 ] || exit $c
  done
  python3 tools/pmc_traffic.py $cfg "$rx" $OUT/pmc_$cfg --out $OUT/traffic_$cfg.json > $OUT/traffic_$cfg.log 2>&1
  echo "[$cfg] traffic: $(cat $OUT/traffic_$cfg.log)"
  cp $OUT/traffic_$cfg.json profiles/ 2>/dev/null
  timeout -k 10 600 python3 bench.py --config $cfg ${BENCH_EXTRA} > $OUT/${cfg}_bench.json 2> $OUT/bench_$cfg.err
  c=$?; echo "[$cfg] bench exit $c: $(cat $OUT/${cfg}_bench.json)"; [ $c -eq 0 ] || exit $c
done
exit 0
