#!/bin/bash
# A/B of two builds on the fused step (tools/step_probe.py): ROUNDS x (new,
# alt) for 1 and 16 chains, then the GPU tests on the new build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ALT=${ALT:-nem-mcmc-optimization_amd/nemo/libnemo_old.so}
P=${PROF_DIR:-gpurun_out/ab_step}; mkdir -p "$P"; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in $(seq ${ROUNDS:-3}); do
  for v in new alt; do
    lib=""; [ $v = alt ] && lib="$(pwd)/$ALT"
    for n in ${CHAINS:-1 16}; do
      NEMO_LIBRARY=$lib timeout -k 10 200 python tools/step_probe.py $n > "$P/${v}_${n}_$r.log" 2>&1 || exit 1
      echo "$v n=$n r=$r $(grep -E 'raw ctypes|dev x10' "$P/${v}_${n}_$r.log" | tr '\n' ' ')"
    done
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$P/pytest_gpu.log" 2>&1; rc=$?
tail -4 "$P/pytest_gpu.log"; exit $rc
