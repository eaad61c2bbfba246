#!/bin/bash
# PMC passes (one counter group per pass, no tracing domains besides kernel
# trace) over tools/prof_target.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out/pmc; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1; echo "list rc=$?"
n=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  n=$((n+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d "$R/gpurun_out/pmc/p$n" -o p -- python "$R/tools/prof_target.py" --reps 2 > "gpurun_out/pmc/p$n.log" 2>&1
  rc=$?; echo "pass $n [$ctrs] rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping"; exit $rc; fi
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64
LIST
