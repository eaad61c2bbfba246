#!/bin/bash
# kernel trace of the fused step for 1 and 16 chains (tools/step_probe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); P=${PROF_DIR:-gpurun_out/step_trace}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
for n in ${CHAINS:-1 16}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$R/$P/n$n" -o t -- python tools/step_probe.py $n > "$P/n$n.log" 2>&1 || exit 1
  echo "== n=$n"; python tools/trace_filter.py "$P/n$n/t_kernel_trace.csv" ""
done
