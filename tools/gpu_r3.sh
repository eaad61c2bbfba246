#!/bin/bash
# Round-3 GPU pass: smoke, GPU tests, parity statistics, bench (with C4).
# Every GPU step has its own time limit; a test failure (rc 1) does not stop
# the pass, anything else (fault, abort, timeout) ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PROF_DIR:-gpurun_out/r3}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "$P/$name.log"; return $rc; }
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; ok $rc || exit $rc
TAILN=30 step pytest_gpu 1200 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS}; rc=$?; ok $rc || exit $rc
step parity_stats 300 python tools/parity_stats.py; rc=$?; ok $rc || exit $rc
[ -n "$NO_BENCH" ] && exit 0
TAILN=2 step bench 400 python bench.py --steps 50 --warmup 5 --cpu-seconds 10; rc=$?; ok $rc || exit $rc
python - "$P/bench.log" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
r = json.loads(line)
print(json.dumps({k: r[k] for k in ("value", "ms_per_step", "dtype", "ll_error_bound")}))
print(json.dumps({k: v for k, v in r["roofline"].items() if k not in ("kernel", "note", "fp64_equivalent")})[:1500])
for k in ("c4_chains", "single_chain", "mcmc_fused_step", "mcmc_end_to_end"):
    print(k, json.dumps({a: b for a, b in r.get(k, {}).items() if a not in ("includes", "workload", "best_order")}))
PY
