#!/bin/bash
# round 6 pass c: the exact forms' bits, then forms A/B at 16 and 128 chains
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gpurun_out/r6c; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -q -rf --timeout 300 --timeout-method thread > $P/pytest_exact.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $P/pytest_exact.log; [ $rc -eq 0 ] || exit $rc
AB_OPT=exact_form AB_VALS=1,4,5 timeout -k 10 300 python tools/step_probe.py 16 > $P/ab16.log 2>&1 || exit 1
grep AB $P/ab16.log
AB_OPT=exact_form AB_VALS=2,5 timeout -k 10 400 python tools/step_probe.py 128 > $P/ab128.log 2>&1 || exit 1
grep AB $P/ab128.log
