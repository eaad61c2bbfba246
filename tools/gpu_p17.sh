#!/bin/bash
# fact_kernel 17 (persistent, pipelined prep) against 10: bits, then sweeps
# over the prep point (after walk iteration w * MUL + ADD) and blocks per CU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/p17; export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/ab_bits.py 17 > gpurun_out/p17/bits.log 2>&1; rc=$?; grep -c True gpurun_out/p17/bits.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${P17_CFGS:-"2 1 0" "3 1 0" "3 0 0" "3 0 99" "2 0 99" "3 0 4"}; do
set -- $cfg
NEMO_I8P_BLOCKS_PER_CU=$1 NEMO_I8P_STAG_MUL=$2 NEMO_I8P_STAG_ADD=$3 timeout -k 10 300 python tools/sweep.py --rounds 2 --steps 20 --configs C3 --batches 2048 --fks 10,17 > gpurun_out/p17/sweep.log 2>&1 || exit 1
grep "path=factored" gpurun_out/p17/sweep.log | sed "s/^/per_cu=$1 mul=$2 add=$3 /; s/\"min_ms.*//; s/remap=1 path=factored //"
done
