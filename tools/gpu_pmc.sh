#!/bin/bash
# PMC passes over tools/prof_target.py, one counter group per pass (read from
# the file given as $1, one line per pass; env NEMO_PROF_* selects variants).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=${PMC_OUT:-gpurun_out/pmc}; mkdir -p "$OUT"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
n=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d "$R/$OUT/p$n" -o p -- python "$R/tools/prof_target.py" --reps 2 > "$OUT/p$n.log" 2>&1
  rc=$?; echo "pass $n [$ctrs] rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping"; exit $rc; fi
done < "$1"
