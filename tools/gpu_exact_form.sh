#!/bin/bash
# exact tests, then the exact local-optimum kernel's two forms A/B (option
# exact_form 1 = latency, 2 = throughput) at 1, 4 and 16 chains
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PROF_DIR:-gpurun_out/exact_form}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
NO_AB=1 TESTS="${TESTS:-exact or raises}" bash tools/gpu_exact.sh || exit 1
for n in 1 4 16; do
  timeout -k 10 180 env AB_OPT=exact_form AB_VALS=1,2 python tools/step_probe.py $n > "$P/n$n.log" 2>&1 || { tail "$P/n$n.log"; exit 1; }
  echo "n=$n"; grep "^AB" "$P/n$n.log"
done
