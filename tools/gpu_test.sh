#!/bin/bash
# GPU tests on the box: pytest -m gpu (optionally a subset: $1 = pytest args)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PROF_DIR:-gpurun_out/t}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread ${1:-} > "$P/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$P/pytest_gpu.log"; exit $rc
