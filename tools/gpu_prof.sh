#!/bin/bash
# rocprofv3 passes over bench.py for the records bench.py attaches to its
# roofline (profiles/traffic.json, profiles/valu.json; tools/make_traffic.py,
# tools/make_valu.py stamp them with the build id): a kernel trace of the
# bench command, then FETCH_SIZE, WRITE_SIZE and the SQ / GRBM counters, each
# in a pass of its own (counters never share a pass with a trace domain).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); P=${PROF_DIR:-gpurun_out/prof}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
B=${NEMO_BENCH_BATCH:-2048}; CFG=${CONFIG:-C3}
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-2} "$P/$name.log"; return $rc; }
BENCH="$R/bench.py --config $CFG --batch $B --no-cpu-baseline ${BENCH_ARGS}"
step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$P/trace" -o t -- python $BENCH --steps 20 --warmup 3 ${TRACE_ARGS:---no-extras} || exit 1
step fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$P/fetch" -o f -- python $BENCH --steps 5 --warmup 1 --no-extras --warmup-seconds 0 || exit 1
step write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$P/write" -o w -- python $BENCH --steps 5 --warmup 1 --no-extras --warmup-seconds 0 || exit 1
step valu 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d "$R/$P/valu" -o v -- python $BENCH --steps 5 --warmup 1 --no-extras --warmup-seconds 0 || exit 1
if [ -n "$STALLS" ]; then
step stalls 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d "$R/$P/stalls" -o s -- python $BENCH --steps 5 --warmup 1 --no-extras --warmup-seconds 0 || exit 1
fi
find "$P" -name "*.csv" | head -20
