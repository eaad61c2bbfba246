#!/bin/bash
# round 6 pass e: the GPU suite, then pass d (bench + local-optimum PMC)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gpurun_out/r6e; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $P/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r6d.sh
