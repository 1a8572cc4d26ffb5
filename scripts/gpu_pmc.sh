#!/bin/bash
# PMC passes over the GEMM arms (each counter set in its own rocprofv3 run,
# kernel-trace + pmc only). Stops at any crash/timeout exit status.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
N=${N:-16384}
KS=${KS:-auto}
pass() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace "$@" --output-format csv -d $OUT/$name -o run -- \
      python3 scripts/prof_gemm_arms.py --n $N --reps ${REPS:-3} --kernels $KS --dtype ${DT:-bfloat16} \
      ${SHAPE:+--shape $SHAPE} > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
pass trace
pass p1 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU
pass p2 --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES
pass p3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
if [ -n "$MIX" ]; then  # instruction mix per MFMA (MIX=1; pmc_summary.py prints the second table)
  pass mix --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVES
fi
find $OUT -name "*.csv" | head -50
