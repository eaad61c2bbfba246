#!/bin/bash
# fused-step kernel breakdown + PMC of the int8 score kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/step_trace" -o s -- python "$R/tools/prof_step.py" --chains 16 --reps 5 > gpurun_out/step_trace.log 2>&1 || { tail gpurun_out/step_trace.log; exit 1; }
tail -2 gpurun_out/step_trace.log
NEMO_PROF_PATH=2 NEMO_PROF_BATCH=512 NEMO_PROF_GROUPS=1 PMC_OUT=gpurun_out/pmc_i8 timeout -k 10 900 bash tools/gpu_pmc.sh tools/pmc_factored.txt
