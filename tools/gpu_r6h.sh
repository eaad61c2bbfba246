#!/bin/bash
# round 6 pass h: the slot form (exact_form 7) -- its bits, then A/B against the throughput form per chain count
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gpurun_out/r6h; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -q -rf --timeout 300 --timeout-method thread \
  -k "forms_give_the_same_bits or more_slots" > $P/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
for ch in 16 32 128; do
  vals=1,2,7; [ $ch -ge 64 ] && vals=2,7
  AB_OPT=exact_form AB_VALS=$vals timeout -k 10 400 python tools/step_probe.py $ch > $P/ab$ch.log 2>&1 || exit 1
  echo "chains $ch"; grep AB $P/ab$ch.log | cut -c1-70
done
