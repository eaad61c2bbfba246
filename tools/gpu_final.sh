#!/bin/bash
# Final pass: tools/gpu_round.sh (smoke, GPU tests, the traced bench, PMC), then the
# rocprofv3 kernel traces and PMC passes whose records bench.py attaches
# (C3 with stall counters, W128, C5, and the streaming kernel at B = 128).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PROF_DIR:-gpurun_out/final}
PROF_DIR=$P PMC=1 bash tools/gpu_round.sh || exit 1
PROF_DIR=$P/c3 STALLS=1 bash tools/gpu_tasks.sh prof || exit 1
PROF_DIR=$P/w128 CONFIG=W128 bash tools/gpu_tasks.sh prof || exit 1
PROF_DIR=$P/c5 CONFIG=C5 bash tools/gpu_tasks.sh prof || exit 1
PROF_DIR=$P/stream NEMO_BENCH_BATCH=128 BENCH_ARGS="--path stream" bash tools/gpu_tasks.sh prof || exit 1
