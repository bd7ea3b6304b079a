#!/bin/bash
# PMC passes over the bench (c2 forward by default), one counter group per pass.
# Output: gpurun_out/pmc/<pass>/..._counter_collection.csv ; summarise with tools/pmc_summary.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS=${PMC_ARGS:---steps 3 --warmup 1 --no-cpu-baseline}
REGEX=${PMC_REGEX:-fwd_f16}
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
while IFS= read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --kernel-include-regex "$REGEX" --output-format csv \
      -d gpurun_out/pmc/p$i -o run -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  c=$?; echo "pass $i ($group) exit $c"
  [ $c -eq 0 ] || exit $c
done <<GROUPS
${PMC_GROUPS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU
SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
WRITE_SIZE}
GROUPS
