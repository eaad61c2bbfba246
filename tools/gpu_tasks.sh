#!/bin/bash
# The one-off GPU passes of rounds 3-4 in one place (DESIGN.md cites them as
# `tools/gpu_tasks.sh <task>`); the round pass is tools/gpu_round.sh, the final
# pass tools/gpu_final.sh.  Every GPU step runs under its own time limit and a
# task stops at its first failure.
#   bash tools/gpu_tasks.sh <task> [args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp PYTHONUNBUFFERED=1
task=$1; shift

# ---- ab: A/B of libnemo.so against libnemo_old.so (another build): ll bits of both on
# the same inputs, the fact_kernel variants' bits, then interleaved sweeps
task_ab() (
O=${AB_OUT:-gpurun_out/ab2}; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/ab_bits_libs.py $O/new.npy > $O/bits_new.log 2>&1 || exit 1
NEMO_LIBRARY=$(pwd)/nem-mcmc-optimization_amd/nemo/libnemo_old.so timeout -k 10 200 python tools/ab_bits_libs.py $O/old.npy > $O/bits_old.log 2>&1 || exit 1
python -c "import numpy as np; a=np.load('$O/new.npy'); b=np.load('$O/old.npy'); print('bits equal:', np.array_equal(a,b), a.shape, 'max diff', np.max(np.abs(a-b)))"
[ -n "$AB_SKIP_VARIANTS" ] || timeout -k 10 200 python tools/ab_bits.py 10 14 16 12 11 | grep -c True || exit 1
ROUNDS=${ROUNDS:-3} AB_B=${AB_B:-512,2048} AB_OUT=$O bash tools/ab_libs.sh
)

# ---- ab_step: A/B of two builds on the fused step (tools/step_probe.py): ROUNDS x (new,
# alt) for 1 and 16 chains, then the GPU tests on the new build.
task_ab_step() (
ALT=${ALT:-nem-mcmc-optimization_amd/nemo/libnemo_old.so}
P=${PROF_DIR:-gpurun_out/ab_step}; mkdir -p "$P"; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in $(seq ${ROUNDS:-3}); do
  for v in new alt; do
    lib=""; [ $v = alt ] && lib="$(pwd)/$ALT"
    for n in ${CHAINS:-1 16}; do
      NEMO_LIBRARY=$lib timeout -k 10 200 python tools/step_probe.py $n > "$P/${v}_${n}_$r.log" 2>&1 || exit 1
      echo "$v n=$n r=$r $(grep -E 'raw ctypes|dev x10' "$P/${v}_${n}_$r.log" | tr '\n' ' ')"
    done
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$P/pytest_gpu.log" 2>&1; rc=$?
tail -4 "$P/pytest_gpu.log"; exit $rc
)

# ---- batch: bench.py's headline line at several batch sizes / step counts / warm-up
# lengths (score kernel only): the fixed part of a launch and the clock ramp
task_batch() (
mkdir -p gpurun_out/batch; export PYTHONUNBUFFERED=1
for cfg in ${BATCH_CFGS:-"2048 50 0" "2048 50 0.5" "2048 50 2" "2048 1000 0.5" "4096 50 0.5" "8192 50 0.5" "2048 50 0.5"}; do
  set -- $(echo $cfg | tr ',' ' ')
  timeout -k 10 120 python bench.py --batch $1 --steps $2 --warmup 5 --warmup-seconds $3 --no-extras --no-cpu-baseline > gpurun_out/batch/b$1_s$2_w$3.json 2>gpurun_out/batch/err.log || exit 1
  python -c "import json,sys; r=json.load(open('gpurun_out/batch/b$1_s$2_w$3.json')); print('B=$1 K=$2 warm=$3s', round(r['value']/1e6,3), 'M evals/s', 'ms/step', round(r['ms_per_step'],4), 'kernel', round(r['roofline']['kernel_avg_ms'],4))"
done
)

# ---- c4_rehearsal: BASELINE C4 rehearsal on one GPU: bench.py at N = 1 (all 128 chains on the
# GPU) and N = 2 gloo ranks sharing it (64 chains each, one all-gather):
# n_gathered must be 128 and the gathered scores (sha) identical.
task_c4_rehearsal() (
P=${PROF_DIR:-gpurun_out/c4}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --c4-steps 10 > "$P/n1.json" 2> "$P/n1.err" || exit $?
NEMO_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 2 --c4-steps 10 \
    > "$P/n2.json" 2> "$P/n2.err" || exit $?
python - "$P" <<'PY'
import json, sys
r = {}
for n in ("n1", "n2"):
    line = [l for l in open(f"{sys.argv[1]}/{n}.json") if l.startswith("{")][-1]
    r[n] = json.loads(line)
    c = r[n]["c4_chains"]
    print(n, "value", round(r[n]["value"]), {k: c[k] for k in ("n_ranks", "chains_per_rank", "inv_workers_per_rank",
          "n_gathered", "best_score", "best_chain", "scores_sha256", "chain_steps_per_s", "collective")})
print("same gathered scores:", r["n1"]["c4_chains"]["scores_sha256"] == r["n2"]["c4_chains"]["scores_sha256"])
PY
)

# ---- exact: Exact-arithmetic pass: the bit-exact GPU tests, then the fused step's time
# with the reference's arithmetic against the fast kernels (interleaved A/B,
# 1 and 16 chains) and a kernel trace of the exact step.
task_exact() (
P=${PROF_DIR:-gpurun_out/exact}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "$P/$name.log"; return $rc; }
TAILN=30 step tests 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_parity.py -k "${TESTS:-exact or trajectory or raises}" -v -s --timeout 300 --timeout-method thread
[ -n "$NO_AB" ] && exit 0
TAILN=8 step ab1 300 env AB_OPT=exact python tools/step_probe.py 1 || exit 1
TAILN=8 step ab16 300 env AB_OPT=exact python tools/step_probe.py 16 || exit 1
for n in ${TRACE:-1 16}; do
  TAILN=2 step trace$n 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$P/trace$n" -o t -- python "$R/tools/step_probe.py" $n || exit 1
  cut -c1-140 "$P/trace$n/t_kernel_stats.csv" | head -8
done
)

# ---- exact_ab: A/B of exact-kernel builds: the default library and variants built on the
# CPU host beforehand into nem-mcmc-optimization_amd/nemo/libnemo_abl_*.so
# (python -c "from nemo import build; build.build(out=..., defines=[...])"),
# each timed by tools/step_probe.py at 1 and 16 chains, interleaved.
task_exact_ab() (
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
)

# ---- exact_form: exact tests, then the exact local-optimum kernel's two forms A/B (option
# exact_form 1 = latency, 2 = throughput) at 1, 4 and 16 chains
task_exact_form() (
P=${PROF_DIR:-gpurun_out/exact_form}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
NO_AB=1 TESTS="${TESTS:-exact or raises}" bash tools/gpu_tasks.sh exact || exit 1
for n in ${CHAINS:-1 2 4 16}; do
  timeout -k 10 180 env AB_OPT=exact_form AB_VALS=${FORMS:-1,2,3} python tools/step_probe.py $n > "$P/n$n.log" 2>&1 || { tail "$P/n$n.log"; exit 1; }
  echo "n=$n"; grep "^AB" "$P/n$n.log"
done
)

# ---- exact_prof: The exact local optimum's cost split: the objective alone (tools/ubench/
# exact_obj, built beforehand on the CPU host) and PMC passes over the exact
# fused step at 16 chains (tools/step_probe.py).
task_exact_prof() (
P=${PROF_DIR:-gpurun_out/exactprof}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "$P/$name.log"; return $rc; }
step obj32k 120 tools/ubench/exact_obj 32256 5 || exit 1
step obj2k 120 tools/ubench/exact_obj 2016 5 || exit 1
step obj2k22 120 tools/ubench/exact_obj 2016 22 || exit 1
N=${CHAINS:-16}
TAILN=1 step pmc_valu 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-include-regex "exact" --output-format csv -d "$R/$P/valu" -o v -- python "$R/tools/step_probe.py" $N || exit 1
TAILN=1 step pmc_wait 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "exact" --output-format csv -d "$R/$P/wait" -o w -- python "$R/tools/step_probe.py" $N || exit 1
)

# ---- lo: local-optimum kernel change: the GPU parity tests that exercise it, then the
# fused step timed with libnemo.so and with libnemo_old.so (1 and 16 chains)
task_lo() (
mkdir -p gpurun_out/lo; export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lo/pt.log 2>&1; rc=$?; tail -3 gpurun_out/lo/pt.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in new old; do for n in 1 16; do
  lib=""; [ $v = old ] && lib="$(pwd)/nem-mcmc-optimization_amd/nemo/libnemo_old.so"
  NEMO_LIBRARY=$lib timeout -k 10 120 python tools/step_probe.py $n > gpurun_out/lo/$v$n.log 2>&1 || exit 1
  echo "$v chains=$n $(grep -v amdgpu gpurun_out/lo/$v$n.log | tr '\n' ' ')"
done; done; done
)

# ---- prof: rocprofv3 passes over bench.py for the records bench.py attaches to its
# roofline (profiles/traffic.json, profiles/valu.json; tools/make_traffic.py,
# tools/make_valu.py stamp them with the build id): a kernel trace of the
# bench command, then FETCH_SIZE, WRITE_SIZE and the SQ / GRBM counters, each
# in a pass of its own (counters never share a pass with a trace domain).
task_prof() (
P=${PROF_DIR:-gpurun_out/prof}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
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
)

# ---- small: kernel 10's small-batch form (16-wave blocks, one set per wave) against its
# 8-wave split form (fact_kernel 21): bits, a batch sweep, the one-chain and
# 16-chain fused step, then the GPU tests.
task_small() (
P=${PROF_DIR:-gpurun_out/small}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-12} "$P/$name.log"; return $rc; }
step bits 300 python tools/ab_bits.py 21 || exit 1
TAILN=14 step sweep 300 python tools/sweep.py --configs C3 --batches 1,8,32,128,255,512 --fks 10,21 --rounds 5 --no-fused --no-stream --out "$P/sweep_small.json" || exit 1
step probe1 200 python tools/step_probe.py 1 || exit 1
step probe16 200 python tools/step_probe.py 16 || exit 1
TAILN=8 step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread || exit 1
)

# ---- split: fact_kernel 20 (prep-only launch + walk-only launch) against 10 (one launch):
# bits, an interleaved burst sweep, and a kernel trace of both.
task_split() (
P=${PROF_DIR:-gpurun_out/split}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-12} "$P/$name.log"; return $rc; }
step bits 300 python tools/ab_bits.py 20 || exit 1
step sweep 300 python tools/sweep.py --configs C3 --batches 512,2048,8192 --fks 10,20 --rounds 5 --no-fused --no-stream --out "$P/sweep_split.json" || exit 1
TAILN=3 step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$P/trace" -o t -- python tools/sweep.py --configs C3 --batches 2048 --fks 20 --rounds 2 --no-fused --no-stream --out "$P/sweep_trace.json" || exit 1
cut -c1-160 "$P"/trace/*kernel_stats.csv | head -12
)

# ---- exact_dev: batched order scores in the reference's arithmetic (option exact_dev):
# the GPU test, tools/exact_score_probe.py (ms per call by batch, bits against the host
# exact path), and its kernel trace
task_exact_dev() (
P=${PROF_DIR:-gpurun_out/exact_dev}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "$P/$name.log"; return $rc; }
TAILN=6 step tests 600 python -u -m pytest tests/test_gpu_exact.py -k "${TESTS:-score_dev or scores_equal}" -v --timeout 300 --timeout-method thread || exit 1
TAILN=6 step probe 300 python tools/exact_score_probe.py ${SIZES:-16 128 2048} || exit 1
if [ -f nem-mcmc-optimization_amd/nemo/libnemo_old.so ]; then   # interleaved A/B against another build
  for r in $(seq ${ROUNDS:-2}); do
    TAILN=3 step "probe_old_$r" 300 env NEMO_LIBRARY=$R/nem-mcmc-optimization_amd/nemo/libnemo_old.so python tools/exact_score_probe.py ${SIZES:-16 128 2048} || exit 1
    TAILN=3 step "probe_new_$r" 300 python tools/exact_score_probe.py ${SIZES:-16 128 2048} || exit 1
  done
fi
TAILN=2 step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$P/trace" -o t -- python "$R/tools/exact_score_probe.py" ${SIZES:-16 128 2048} || exit 1
cut -c1-140 "$P/trace/t_kernel_stats.csv" | head -8
)

# ---- exact_pmc: VALU / LDS counters of the exact kernels: the batched exact scores
# (tools/exact_score_probe.py 2048) and the fused step at 1 and 16 chains (tools/step_probe.py)
task_exact_pmc() (
P=${PROF_DIR:-gpurun_out/exact_pmc}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
C=${COUNTERS:-"SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"}
if [ -z "$NO_SCORE" ]; then
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$R/$P/score" -o p -- python "$R/tools/exact_score_probe.py" 2048 > "$P/score.log" 2>&1 || exit 1
  python tools/exact_pmc.py "$P/score/p_counter_collection.csv"
fi
for n in ${CHAINS:-1 16}; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$R/$P/step$n" -o p -- python "$R/tools/step_probe.py" $n > "$P/step$n.log" 2>&1 || exit 1
  echo "== step n=$n"; python tools/exact_pmc.py "$P/step$n/p_counter_collection.csv"
done
)

# ---- step_trace: kernel trace of the fused step for 1 and 16 chains (tools/step_probe.py)
task_step_trace() (
P=${PROF_DIR:-gpurun_out/step_trace}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
for n in ${CHAINS:-1 16}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$R/$P/n$n" -o t -- python tools/step_probe.py $n > "$P/n$n.log" 2>&1 || exit 1
  echo "== n=$n"; python tools/trace_filter.py "$P/n$n/t_kernel_trace.csv" ""
done
)

# ---- cform: the exact local optima's c stored per optimum (exact_cform 0) against recomputed
# from the parent's a rows (1), and the XCD-contiguous optimum order (exact_xcd): the bit-exact
# GPU tests on the default, interleaved step A/Bs, then FETCH_SIZE / L2 / VALU / wait counters of
# the local-optimum kernel at 16 chains for both forms (each counter set in its own pass)
task_cform() (
P=${PROF_DIR:-gpurun_out/cform}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "$P/$name.log"; return $rc; }
if [ -z "$NO_TESTS" ]; then   # an assertion failure does not stop the A/B; a fault, abort or time limit does
  TAILN=12 step tests 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_parity.py tests/test_gpu_rehearsal.py -q -rf -k "${TESTS:-exact or trajectory or raises or replica or rehearsal or ranks}" --timeout 300 --timeout-method thread; rc=$?
  [ $rc -le 1 ] || exit $rc
fi
for n in ${CHAINS:-1 16 128}; do
  TAILN=3 step ab_cform_$n 300 env AB_OPT=exact_cform AB_VALS=0,1 python tools/step_probe.py $n || exit 1
done
for n in ${XCD_CHAINS:-16 128}; do
  TAILN=3 step ab_xcd_$n 300 env AB_OPT=exact_xcd AB_VALS=0,1 python tools/step_probe.py $n || exit 1
done
[ -n "$NO_PMC" ] && exit 0
for f in 0 1; do
  for cs in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
    tag=$(echo $cs | cut -d' ' -f1)
    timeout -s KILL 180 env EXACT_CFORM=$f rocprofv3 --pmc $cs --kernel-include-regex "local_opt_exact" --output-format csv -d "$R/$P/pmc_${f}_$tag" -o p -- python "$R/tools/step_probe.py" 16 > "$P/pmc_${f}_$tag.log" 2>&1 || { echo "pmc $f $tag failed"; tail -3 "$P/pmc_${f}_$tag.log"; exit 1; }
  done
done
echo "pmc done"
)

# ---- lo_pmc: the local-optimum kernel's counters at 16 chains on the default build
# (FETCH_SIZE, WRITE_SIZE, L2 hit / miss, VALU, waits; each set in its own pass)
task_lo_pmc() (
P=${PROF_DIR:-gpurun_out/lo_pmc}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
for cs in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  tag=$(echo $cs | cut -d' ' -f1)
  timeout -s KILL 180 rocprofv3 --pmc $cs --kernel-include-regex "local_opt_exact" --output-format csv -d "$R/$P/lo_$tag" -o p -- python "$R/tools/step_probe.py" ${CHAINS:-16} > "$P/lo_$tag.log" 2>&1 || { echo "pmc $tag failed"; tail -3 "$P/lo_$tag.log"; exit 1; }
done
echo "lo pmc done"
)

# ---- i8l_valu: SQ_INSTS_VALU of score_i8l_kernel (C3, B = 2048) for the default build and
# the prep-only instrumented build (libnemo_abl32.so, NEMO_I8_ABLATE=32: no tiles walked), so
# the walk's share is the difference (DESIGN.md 3.1h's per-cell accounting)
task_i8l_valu() (
P=${PROF_DIR:-gpurun_out/i8l_valu}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
L=$R/nem-mcmc-optimization_amd/nemo
for v in default abl32; do
  lib=""; [ $v = abl32 ] && lib=$L/libnemo_abl32.so
  timeout -s KILL 180 env NEMO_LIBRARY=$lib rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex "score_i8l" --output-format csv -d "$R/$P/$v" -o p -- python "$R/tools/i8l_probe.py" > "$P/$v.log" 2>&1 || { tail -3 "$P/$v.log"; exit 1; }
  echo "== $v"; python tools/exact_pmc.py "$P/$v/p_counter_collection.csv"
done
)

case "$task" in
  ab|ab_step|batch|c4_rehearsal|cform|i8l_valu|exact|exact_ab|exact_dev|exact_pmc|exact_form|exact_prof|lo|lo_pmc|prof|small|split|step_trace) "task_$task" "$@" ;;
  *) echo "tasks: ab ab_step batch c4_rehearsal cform i8l_valu exact exact_ab exact_dev exact_pmc exact_form exact_prof lo lo_pmc prof small split step_trace"; exit 2 ;;
esac
