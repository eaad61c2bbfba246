#!/bin/bash
# GPU tests, then bench + kernel trace + FETCH/WRITE passes (tools/gpu_bench_prof.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
bash tools/gpu_bench_prof.sh
