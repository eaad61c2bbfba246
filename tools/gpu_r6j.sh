#!/bin/bash
# round 6 pass j: latency form (1) against the slot form (7) per chain count, for the auto policy
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gpurun_out/r6j; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
for ch in 1 2 4 8 12 16 24 64; do
  vals=1,7; [ $ch -ge 64 ] && vals=2,7
  AB_OPT=exact_form AB_VALS=$vals timeout -k 10 400 python tools/step_probe.py $ch > $P/ab$ch.log 2>&1 || exit 1
  echo "chains $ch"; grep AB $P/ab$ch.log | cut -c1-70
done
