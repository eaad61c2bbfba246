#!/bin/bash
# Iteration pass on one MI355X: GPU tests, a score-kernel A/B sweep (C3),
# the bench line.  Each GPU step has its own limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PROF_DIR:-gpurun_out/iter}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "$P/$name.log"; return $rc; }
TAILN=8 step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread || exit 1
TAILN=40 step sweep 300 python tools/sweep.py --rounds 3 --steps 10 --configs C3 --batches ${SWEEP_B:-512,2048} --fks ${SWEEP_FKS:-8,10,11} --out "$P/sweep.json" || exit 1
step bench 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 3 --no-extras || exit 1
