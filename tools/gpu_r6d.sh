#!/bin/bash
# round 6 pass d: the bench (local_opt roofline fields) and the local-optimum kernel's PMC at
# 16 and 128 chains (each counter set in its own pass)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); P=gpurun_out/r6d; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python bench.py --no-cpu-baseline > $P/bench.log 2>&1 || { tail -5 $P/bench.log; exit 1; }
grep '^{' $P/bench.log > $P/bench.json
python -c "
import json; d=json.load(open('$P/bench.json'))
print(json.dumps(d.get('local_opt'))[:1500]); print(d['value'], d['c4_chains']['chain_steps_per_s'], d['mcmc_fused_step']['ms_per_step'])"
for ch in 16 128; do
  for cs in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
    tag=$(echo $cs | cut -d' ' -f1)
    timeout -s KILL 240 rocprofv3 --pmc $cs --kernel-include-regex "local_opt_exact" --output-format csv -d "$R/$P/c${ch}_$tag" -o p -- python "$R/tools/step_probe.py" $ch > "$P/c${ch}_$tag.log" 2>&1 || { echo "pmc $ch $tag failed"; tail -3 "$P/c${ch}_$tag.log"; exit 1; }
    python tools/exact_pmc.py "$P/c${ch}_$tag/p_counter_collection.csv" | tail -2
  done
done
