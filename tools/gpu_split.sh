#!/bin/bash
# fact_kernel 20 (prep-only launch + walk-only launch) against 10 (one launch):
# bits, an interleaved burst sweep, and a kernel trace of both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); P=${PROF_DIR:-gpurun_out/split}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-12} "$P/$name.log"; return $rc; }
step bits 300 python tools/ab_bits.py 20 || exit 1
step sweep 300 python tools/sweep.py --configs C3 --batches 512,2048,8192 --fks 10,20 --rounds 5 --no-fused --no-stream --out "$P/sweep_split.json" || exit 1
TAILN=3 step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$P/trace" -o t -- python tools/sweep.py --configs C3 --batches 2048 --fks 20 --rounds 2 --no-fused --no-stream --out "$P/sweep_trace.json" || exit 1
cut -c1-160 "$P"/trace/*kernel_stats.csv | head -12
