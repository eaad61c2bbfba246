#!/bin/bash
# PMC record of the capped lookup-table kernel (C5, B = 2048): two counter
# passes (tools/pmc_win.txt) over tools/prof_target.py, then profiles/valu.json
# key C5:win:b2048 via tools/make_valu.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export NEMO_PROF_CONFIGS=C5 NEMO_PROF_BATCH=2048 PMC_OUT=gpurun_out/pmc_win
bash tools/gpu_pmc.sh tools/pmc_win.txt || exit 1
for f in gpurun_out/pmc_win/p*/p_counter_collection.csv; do
  python tools/make_valu.py "$f" "C5:{kind}:b2048" gpurun_out/pmc_win/valu_win.json > /dev/null || exit 1
done
cat gpurun_out/pmc_win/valu_win.json
