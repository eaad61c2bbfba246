#!/bin/bash
# round 6 pass b: GPU tests, then the local-optimum forms A/B at 16 and 128 chains
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gpurun_out/r6b; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 $P/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
AB_OPT=exact_form AB_VALS=1,2,4 timeout -k 10 300 python tools/step_probe.py 16 > $P/ab16.log 2>&1 || exit 1
grep AB $P/ab16.log
AB_OPT=exact_form AB_VALS=2,4 timeout -k 10 400 python tools/step_probe.py 128 > $P/ab128.log 2>&1 || exit 1
grep AB $P/ab128.log
