#!/bin/bash
# bench lines for the parity configs (C2) and a 2-rank rehearsal of the N > 1
# path on one GPU (gloo; the driver's multi-GPU runs use RCCL)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/cfg; export PYTHONUNBUFFERED=1
timeout -k 10 120 python bench.py --config C2 --steps 50 --no-extras --cpu-seconds 5 > gpurun_out/cfg/c2.json 2>gpurun_out/cfg/c2.err || exit 1
tail -c 600 gpurun_out/cfg/c2.json; echo
NEMO_BENCH_BACKEND=gloo timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 5 --no-extras \
  > gpurun_out/cfg/n2_gloo.json 2>gpurun_out/cfg/n2_gloo.err || exit 1
head -c 400 gpurun_out/cfg/n2_gloo.json; echo
