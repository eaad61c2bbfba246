#!/bin/bash
# round 6 pass i: slot form variants (waves per SIMD x pipelined c loads), fused step time at 16 / 128 chains
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=gpurun_out/r6i; mkdir -p $P; export TMPDIR=/tmp PYTHONUNBUFFERED=1
for ch in 16 128; do
  for v in base s41 s30 s31; do
    lib=nem-mcmc-optimization_amd/nemo/libnemo.so; [ $v != base ] && lib=tools/var/libnemo_$v.so
    NEMO_LIBRARY=$lib EXACT_FORM=7 timeout -k 10 300 python tools/step_probe.py $ch > $P/$v.$ch.log 2>&1 || exit 1
    echo "chains $ch $v $(grep -E '^raw ctypes' $P/$v.$ch.log)"
  done
  EXACT_FORM=2 timeout -k 10 300 python tools/step_probe.py $ch > $P/f2.$ch.log 2>&1 || exit 1
  echo "chains $ch form2 $(grep -E '^raw ctypes' $P/f2.$ch.log)"
done
