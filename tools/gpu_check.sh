#!/bin/bash
# GPU pass: smoke, GPU parity tests, variant sweep, bench, rocprof kernel
# trace.  Each GPU step has its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-8} "gpurun_out/$name.log"; return $rc; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
TAILN=6 step pytest_gpu 900 python -m pytest tests -m gpu -q -rf; rc=$?; [ $rc -le 1 ] || exit $rc
TAILN=60 step sweep 600 python tools/sweep.py --rounds 3 --steps 10 || exit 1
step bench 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 10 || exit 1
R=$(pwd)
export TMPDIR=/tmp
TAILN=3 step prof_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o trace -- python "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline || exit 1
TAILN=3 step prof_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o fetch -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline || exit 1
TAILN=3 step prof_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write" -o write -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline || exit 1
find gpurun_out -name "*.csv" | head -20
