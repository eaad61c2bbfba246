#!/bin/bash
# kernel 10's small-batch form (16-wave blocks, one set per wave) against its
# 8-wave split form (fact_kernel 21): bits, a batch sweep, the one-chain and
# 16-chain fused step, then the GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); P=${PROF_DIR:-gpurun_out/small}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-12} "$P/$name.log"; return $rc; }
step bits 300 python tools/ab_bits.py 21 || exit 1
TAILN=14 step sweep 300 python tools/sweep.py --configs C3 --batches 1,8,32,128,255,512 --fks 10,21 --rounds 5 --no-fused --no-stream --out "$P/sweep_small.json" || exit 1
step probe1 200 python tools/step_probe.py 1 || exit 1
step probe16 200 python tools/step_probe.py 16 || exit 1
TAILN=8 step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread || exit 1
