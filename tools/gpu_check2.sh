#!/bin/bash
# GPU tests, the C3 per-step weights dump, and a short bench for the extras
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PROF_DIR:-gpurun_out/check2}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$P/pytest_gpu.log" 2>&1; rc=$?
tail -4 "$P/pytest_gpu.log"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/diag_traj_c3_steps.py > "$P/diag.log" 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$P/bench.log" 2>&1 || exit 1
python - "$P/bench.log" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("value", r["value"], "roof", r["roofline"]["bound"], r["roofline"]["frac"])
for k in ("single_chain", "mcmc_fused_step", "mcmc_end_to_end", "c4_chains"):
    print(k, json.dumps({a: b for a, b in r[k].items() if a not in ("includes", "workload", "best_order")})[:400])
PY
