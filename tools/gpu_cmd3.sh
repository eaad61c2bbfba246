#!/bin/bash
# quick tests + sweep, then PMC passes of the int8 score kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SWEEP_CONFIGS=C3 bash tools/gpu_quick.sh || exit 1
NEMO_PROF_PATH=2 NEMO_PROF_BATCH=512 NEMO_PROF_GROUPS=1 PMC_OUT=gpurun_out/pmc_i8b timeout -k 10 600 bash tools/gpu_pmc.sh tools/pmc_i8.txt
