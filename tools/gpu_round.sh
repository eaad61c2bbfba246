#!/bin/bash
# Round pass on one MI355X: smoke, GPU tests, the default bench under a
# rocprofv3 kernel trace (the bench line and the trace of the same process,
# so the dominant kernel's trace mean sits beside its ms_per_step), a plain
# bench run, and with PMC=1 the FETCH/WRITE_SIZE (traffic) and VALU passes.
# Every GPU step has its own limit; stop at the first failure.
#   SKIP_TESTS=1: no smoke / pytest;  PMC=1: the counter passes too
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); P=${PROF_DIR:-gpurun_out/round}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "$P/$name.log"; return $rc; }
if [ -z "$SKIP_TESTS" ]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
  TAILN=6 step pytest_gpu 1000 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread ${PYTEST_ARGS} || exit 1
fi
B=${NEMO_BENCH_BATCH:-2048}
TAILN=2 step bench_traced 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$P/trace" -o t -- python "$R/bench.py" || exit 1
grep '^{' "$P/bench_traced.log" > "$P/bench_traced.json"
TAILN=1 step bench 300 python bench.py || exit 1
grep '^{' "$P/bench.log" > "$P/bench.json"
if [ -n "$PMC" ]; then
  TAILN=2 step fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$P/fetch" -o f -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-extras --warmup-seconds 0 --batch $B || exit 1
  TAILN=2 step write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$P/write" -o w -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-extras --warmup-seconds 0 --batch $B || exit 1
  TAILN=2 step valu 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d "$R/$P/valu" -o v -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-extras --warmup-seconds 0 --batch $B || exit 1
fi
cut -c1-150 "$P/trace/t_kernel_stats.csv" | head -12
