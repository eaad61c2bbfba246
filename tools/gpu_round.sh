#!/bin/bash
# Round pass on one MI355X: smoke, GPU tests, bench (C3, B=2048), rocprofv3
# kernel trace of the same command, FETCH/WRITE_SIZE passes (traffic) and a
# VALU pass.  Every GPU step has its own limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); P=${PROF_DIR:-gpurun_out/round}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "$P/$name.log"; return $rc; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
TAILN=6 step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread || exit 1
step bench 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 10 || exit 1
B=${NEMO_BENCH_BATCH:-2048}
TAILN=2 step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$P/trace" -o t -- python "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --batch $B || exit 1
TAILN=2 step fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$P/fetch" -o f -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-extras --warmup-seconds 0 --batch $B || exit 1
TAILN=2 step write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$P/write" -o w -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-extras --warmup-seconds 0 --batch $B || exit 1
TAILN=2 step valu 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d "$R/$P/valu" -o v -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-extras --warmup-seconds 0 --batch $B || exit 1
cut -c1-150 "$P/trace/t_kernel_stats.csv"
