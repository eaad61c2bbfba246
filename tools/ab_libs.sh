#!/bin/bash
# A/B of two builds of the library on one box: ROUNDS x (sweep with
# libnemo.so, sweep with $ALT), same configs; prints the score-kernel lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ALT=${ALT:-nem-mcmc-optimization_amd/nemo/libnemo_old.so}
OUT=${AB_OUT:-gpurun_out/ab}; mkdir -p "$OUT"; export PYTHONUNBUFFERED=1
for r in $(seq ${ROUNDS:-2}); do
  for v in new alt; do
    lib=""; [ $v = alt ] && lib="$(pwd)/$ALT"
    NEMO_LIBRARY=$lib timeout -k 10 200 python tools/sweep.py --rounds ${SW_ROUNDS:-3} --steps ${SW_STEPS:-20} \
      --configs ${AB_CONFIGS:-C3} --batches ${AB_B:-512,2048} --fks ${AB_FKS:-10} --out "$OUT/$v$r.json" > "$OUT/$v$r.log" 2>&1 || exit 1
    grep "path=factored" "$OUT/$v$r.log" | sed "s/^/$v /"
  done
done
