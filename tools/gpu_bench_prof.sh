#!/bin/bash
# bench + rocprofv3 kernel trace + FETCH/WRITE_SIZE passes of the same command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); P=${PROF_DIR:-gpurun_out/prof}; mkdir -p "$P"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
B=${NEMO_BENCH_BATCH:-512}
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > "$P/bench.json" 2> "$P/bench.err" || { tail "$P/bench.err"; exit 1; }
cat "$P/bench.json"
for path in factored stream; do
  NB=$B; [ $path = stream ] && NB=128
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$P/trace_$path" -o t -- python "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-extras --path $path --batch $NB > "$P/trace_$path.log" 2>&1 || { echo "trace $path failed"; tail "$P/trace_$path.log"; exit 1; }
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$P/fetch_$path" -o f -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-extras --path $path --batch $NB > "$P/fetch_$path.log" 2>&1 || { echo "fetch $path failed"; exit 1; }
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$P/write_$path" -o w -- python "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-extras --path $path --batch $NB > "$P/write_$path.log" 2>&1 || { echo "write $path failed"; exit 1; }
  echo "== $path"; cat "$P/trace_$path/t_kernel_stats.csv" | cut -c1-160
done
