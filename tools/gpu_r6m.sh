#!/bin/bash
# round 6 pass m: slot-form variants -- hybrid (slot 0 recomputed: half the row set's L2 footprint)
# and the paired log -- bits (forms test on each variant), then the fused step at 16 / 128 chains
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gpurun_out/r6m; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in hy lp; do
  NEMO_LIBRARY=tools/var/libnemo_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 240 \
    --timeout-method thread -k "forms_give_the_same_bits or more_slots" > $P/pytest_$v.log 2>&1 || { echo "bits $v failed"; tail -5 $P/pytest_$v.log; exit 1; }
  echo "bits $v: $(tail -1 $P/pytest_$v.log)"
done
for ch in 16 128; do
  for v in base hy lp; do
    lib=nem-mcmc-optimization_amd/nemo/libnemo.so; [ $v != base ] && lib=tools/var/libnemo_$v.so
    NEMO_LIBRARY=$lib EXACT_FORM=7 timeout -k 10 300 python tools/step_probe.py $ch > $P/$v.$ch.log 2>&1 || exit 1
    echo "chains $ch $v $(grep -E '^raw ctypes' $P/$v.$ch.log)"
  done
done
