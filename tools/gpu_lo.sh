#!/bin/bash
# local-optimum kernel change: the GPU parity tests that exercise it, then the
# fused step timed with libnemo.so and with libnemo_old.so (1 and 16 chains)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/lo; export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lo/pt.log 2>&1; rc=$?; tail -3 gpurun_out/lo/pt.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in new old; do for n in 1 16; do
  lib=""; [ $v = old ] && lib="$(pwd)/nem-mcmc-optimization_amd/nemo/libnemo_old.so"
  NEMO_LIBRARY=$lib timeout -k 10 120 python tools/step_probe.py $n > gpurun_out/lo/$v$n.log 2>&1 || exit 1
  echo "$v chains=$n $(grep -v amdgpu gpurun_out/lo/$v$n.log | tr '\n' ' ')"
done; done; done
