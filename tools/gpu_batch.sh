#!/bin/bash
# bench.py's headline line at several batch sizes / step counts / warm-up
# lengths (score kernel only): the fixed part of a launch and the clock ramp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/batch; export PYTHONUNBUFFERED=1
for cfg in ${BATCH_CFGS:-"2048 50 0" "2048 50 0.5" "2048 50 2" "2048 1000 0.5" "4096 50 0.5" "8192 50 0.5" "2048 50 0.5"}; do
  set -- $(echo $cfg | tr ',' ' ')
  timeout -k 10 120 python bench.py --batch $1 --steps $2 --warmup 5 --warmup-seconds $3 --no-extras --no-cpu-baseline > gpurun_out/batch/b$1_s$2_w$3.json 2>gpurun_out/batch/err.log || exit 1
  python -c "import json,sys; r=json.load(open('gpurun_out/batch/b$1_s$2_w$3.json')); print('B=$1 K=$2 warm=$3s', round(r['value']/1e6,3), 'M evals/s', 'ms/step', round(r['ms_per_step'],4), 'kernel', round(r['roofline']['kernel_avg_ms'],4))"
done
