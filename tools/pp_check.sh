#!/bin/bash
# paired-block forward: parity (default dispatch, then forced for every rule it takes) + A/B timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/pp_pytest.log 2>&1
c=$?; echo "pytest default exit $c"; tail -3 gpurun_out/pp_pytest.log; [ $c -eq 0 ] || exit $c
FA_HIP_LIB=$PWD/tf_flash_attention_amd/libfa_hip_diag.so FA_FWD_VARIANT=${FORCE:-2000} timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/pp_pytest2000.log 2>&1
c=$?; echo "pytest forced exit $c"; tail -3 gpurun_out/pp_pytest2000.log; [ $c -eq 0 ] || exit $c
timeout -k 10 300 python -u tools/fwd_variants.py ${CFG:-c2} ${VARIANTS:-1814 -1} > gpurun_out/pp_var.log 2>&1
c=$?; echo "variants exit $c"; cat gpurun_out/pp_var.log; exit $c
