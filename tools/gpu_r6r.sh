#!/bin/bash
# round 6 pass r: the paired slot form with 4 (this build) or 8 (NEMO_EXACT_SLOT_GROUP=8) pair loads
# in flight: bits of both, then the fused step at 16 / 128 chains, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gpurun_out/r6r; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in g4 g8; do
  lib=nem-mcmc-optimization_amd/nemo/libnemo.so; [ $v = g8 ] && lib=tools/var/libnemo_g8.so
  NEMO_LIBRARY=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 240 \
    --timeout-method thread -k "forms_give_the_same_bits or more_slots" > $P/pytest_$v.log 2>&1 || { echo "bits $v failed"; tail -5 $P/pytest_$v.log; exit 1; }
  echo "bits $v: $(tail -1 $P/pytest_$v.log)"
done
for r in 1 2; do
  for ch in 16 128; do
    for v in g4 g8; do
      lib=nem-mcmc-optimization_amd/nemo/libnemo.so; [ $v = g8 ] && lib=tools/var/libnemo_g8.so
      NEMO_LIBRARY=$lib timeout -k 10 300 python tools/step_probe.py $ch > $P/$v.$ch.$r.log 2>&1 || exit 1
      echo "r$r chains $ch $v $(grep -E '^raw ctypes' $P/$v.$ch.$r.log)"
    done
  done
done
