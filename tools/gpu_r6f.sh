#!/bin/bash
# round 6 pass f: the exact forms' bits, then the forms A/B per chain count (policy sweep)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gpurun_out/r6f; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_parity.py -x -q -rf --timeout 300 --timeout-method thread > $P/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
for ch in 1 4 16 32 64 128; do
  vals=1,2,4; [ $ch -ge 64 ] && vals=2,4
  AB_OPT=exact_form AB_VALS=$vals timeout -k 10 400 python tools/step_probe.py $ch > $P/ab$ch.log 2>&1 || exit 1
  echo "chains $ch"; grep AB $P/ab$ch.log | cut -c1-70
done
