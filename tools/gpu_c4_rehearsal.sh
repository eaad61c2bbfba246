#!/bin/bash
# BASELINE C4 rehearsal on one GPU: bench.py at N = 1 (all 128 chains on the
# GPU) and N = 2 gloo ranks sharing it (64 chains each, one all-gather):
# n_gathered must be 128 and the gathered scores (sha) identical.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
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
