#!/bin/bash
# quick loop: GPU tests + sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/sweep.py --rounds 3 --steps 10 --configs ${SWEEP_CONFIGS:-C3,C5} > gpurun_out/sweep.log 2>&1; rc=$?
cat gpurun_out/sweep.log | grep -v amdgpu.ids; exit $rc
