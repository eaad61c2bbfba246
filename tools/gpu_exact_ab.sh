#!/bin/bash
# A/B of exact-kernel builds: the default library and variants built on the
# CPU host beforehand into nem-mcmc-optimization_amd/nemo/libnemo_abl_*.so
# (python -c "from nemo import build; build.build(out=..., defines=[...])"),
# each timed by tools/step_probe.py at 1 and 16 chains, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PROF_DIR:-gpurun_out/exact_ab}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
L=nem-mcmc-optimization_amd/nemo
for round in 1 2; do
  for lib in $L/libnemo.so $L/libnemo_abl_*.so; do
    for n in 1 16; do
      timeout -k 10 120 env NEMO_LIBRARY=$(pwd)/$lib python tools/step_probe.py $n > "$P/x.log" 2>&1 || { cat "$P/x.log"; exit 1; }
      echo "$round $(basename $lib) n=$n $(grep 'raw ctypes' "$P/x.log")"
    done
  done
done
