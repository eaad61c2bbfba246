# sampler throughput A/B on the GPU box: bash tools/gpu_e2e.sh [out dir]
# env ARGS_LIST: newline-separated tools/mcmc_e2e.py argument sets
set -e
O=${1:-gpurun_out/e2e}
mkdir -p "$O"
: "${ARGS_LIST:=--chains 16
--chains 128}"
while IFS= read -r args; do
  [ -n "$args" ] || continue
  timeout -k 10 240 python tools/mcmc_e2e.py $args --steps 20 --inv-workers 8 >> "$O/runs.txt" 2>&1
done <<< "$ARGS_LIST"
grep chain-steps "$O/runs.txt"
