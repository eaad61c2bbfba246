#!/bin/bash
# round 6 pass q: the paired slot form with 2 or 4 pair loads in flight (g2 = this build, g4 =
# NEMO_EXACT_SLOT_GROUP=4, old = unpaired), bits of g4, then the fused step per chain count,
# and the latency form at 4 / 8 chains for the auto crossover
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gpurun_out/r6q; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
NEMO_LIBRARY=tools/var/libnemo_g4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 240 \
  --timeout-method thread -k "forms_give_the_same_bits or more_slots" > $P/pytest_g4.log 2>&1 || { echo "bits g4 failed"; tail -5 $P/pytest_g4.log; exit 1; }
echo "bits g4: $(tail -1 $P/pytest_g4.log)"
for ch in 4 8 16 128; do
  for v in g2 g4 old; do
    lib=nem-mcmc-optimization_amd/nemo/libnemo.so; [ $v = g4 ] && lib=tools/var/libnemo_g4.so; [ $v = old ] && lib=tools/var/libnemo_old.so
    NEMO_LIBRARY=$lib EXACT_FORM=7 timeout -k 10 300 python tools/step_probe.py $ch > $P/$v.$ch.log 2>&1 || exit 1
    echo "chains $ch slot $v $(grep -E '^raw ctypes' $P/$v.$ch.log)"
  done
  if [ $ch -le 16 ]; then
    EXACT_FORM=1 timeout -k 10 300 python tools/step_probe.py $ch > $P/lat.$ch.log 2>&1 || exit 1
    echo "chains $ch latency $(grep -E '^raw ctypes' $P/lat.$ch.log)"
  fi
done
