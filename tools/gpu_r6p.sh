#!/bin/bash
# round 6 pass p: the slot form's row set in element pairs (NEMO_EXACT_SLOT_PAIRS) -- bits, then
# the fused step against the previous build, interleaved, 16 and 128 chains
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gpurun_out/r6p; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_parity.py -x -q --timeout 300 \
  --timeout-method thread > $P/pytest.log 2>&1 || { echo "bits failed"; tail -5 $P/pytest.log; exit 1; }
echo "bits: $(tail -1 $P/pytest.log)"
for r in 1 2; do
  for ch in 16 128; do
    for v in new old; do
      lib=nem-mcmc-optimization_amd/nemo/libnemo.so; [ $v = old ] && lib=tools/var/libnemo_old.so
      NEMO_LIBRARY=$lib timeout -k 10 300 python tools/step_probe.py $ch > $P/$v.$ch.$r.log 2>&1 || exit 1
      echo "r$r chains $ch $v $(grep -E '^raw ctypes' $P/$v.$ch.$r.log)"
    done
  done
done
