#!/bin/bash
# A/B of two builds on the whole sampler (tools/mcmc_e2e.py, inversion pool):
# ROUNDS x (new, alt) for each chain count in CHAINS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ALT=${ALT:-nem-mcmc-optimization_amd/nemo/libnemo_old.so}
P=${PROF_DIR:-gpurun_out/ab_e2e}; mkdir -p "$P"; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in $(seq ${ROUNDS:-3}); do
  for v in new alt; do
    lib=""; [ $v = alt ] && lib="$(pwd)/$ALT"
    for n in ${CHAINS:-16 128}; do
      NEMO_LIBRARY=$lib timeout -k 10 300 python tools/mcmc_e2e.py --chains $n --steps ${STEPS:-30} --inv-workers ${WORKERS:-8} > "$P/${v}_${n}_$r.log" 2>&1 || exit 1
      echo "$v n=$n r=$r $(grep -E "chains x" "$P/${v}_${n}_$r.log" | tail -1 | tr '\n' ' ')"
    done
  done
done
