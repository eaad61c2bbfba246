#!/bin/bash
# round 6 pass l: the local-optimum kernel's PMC at 16 and 128 chains on the slot-form build
# (auto: the slot form at both; each counter set in its own pass)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); P=gpurun_out/r6l; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1

for ch in 16 128; do
  for cs in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
    tag=$(echo $cs | cut -d' ' -f1)
    timeout -s KILL 240 rocprofv3 --pmc $cs --kernel-include-regex "local_opt_exact" --output-format csv -d "$R/$P/c${ch}_$tag" -o p -- python "$R/tools/step_probe.py" $ch > "$P/c${ch}_$tag.log" 2>&1 || { echo "pmc $ch $tag failed"; tail -3 "$P/c${ch}_$tag.log"; exit 1; }
    python tools/exact_pmc.py "$P/c${ch}_$tag/p_counter_collection.csv" | tail -2
  done
done
