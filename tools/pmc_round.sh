#!/bin/bash
# SQ / GRBM counter passes (one rocprofv3 --pmc run per group, counters only: no trace domains)
# over bench.py configs.  Output: gpurun_out/pmc_<cfg>/p<i>/ ; summarise per kernel with
#   python tools/pmc_summary.py --by-kernel <regex> gpurun_out/pmc_<cfg> --json profiles/<round>_pmc_<cfg>.json
# Usage (GPU box): CONFIGS="c2 c3" bash tools/pmc_round.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
declare -A REGEX=([c2]=fwd_f16 [c3]="fwd_f16|bwd_dkdv|bwd_dq|bwd_prep" [c4]=fwd_f16 [c5]=fwd_f32_kernel [d32]=fwd_f16)
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
G2="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
G3="SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAVES"
for cfg in ${CONFIGS:-c2}; do
  out=gpurun_out/pmc_$cfg; mkdir -p $out
  i=0
  for group in "$G1" "$G2" "$G3"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $group --kernel-include-regex "${REGEX[$cfg]}" --output-format csv \
        -d $out/p$i -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --warmup-s 0 --no-cpu-baseline \
        > $out/p$i.log 2>&1
    c=$?; echo "[$cfg] pass $i exit $c"; [ $c -eq 0 ] || exit $c
  done
done
exit 0
