#!/bin/bash
# the fused step: GPU tests, then the one-chain and 16-chain step probes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PROF_DIR:-gpurun_out/step}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-6} "$P/$name.log"; return $rc; }
TAILN=8 step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS} || exit 1
step probe1 200 python tools/step_probe.py 1 || exit 1
AB_OPT=local_split AB_VALS=1,3,2 step probe1ab 400 python tools/step_probe.py 1 || exit 1
AB_OPT=local_split AB_VALS=1,3 step probe4ab 400 python tools/step_probe.py 4 || exit 1
step probe16 200 python tools/step_probe.py 16 || exit 1
