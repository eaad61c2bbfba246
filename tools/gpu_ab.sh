#!/bin/bash
# A/B of libnemo.so against libnemo_old.so (another build): ll bits of both on
# the same inputs, the fact_kernel variants' bits, then interleaved sweeps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=${AB_OUT:-gpurun_out/ab2}; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/ab_bits_libs.py $O/new.npy > $O/bits_new.log 2>&1 || exit 1
NEMO_LIBRARY=$(pwd)/nem-mcmc-optimization_amd/nemo/libnemo_old.so timeout -k 10 200 python tools/ab_bits_libs.py $O/old.npy > $O/bits_old.log 2>&1 || exit 1
python -c "import numpy as np; a=np.load('$O/new.npy'); b=np.load('$O/old.npy'); print('bits equal:', np.array_equal(a,b), a.shape, 'max diff', np.max(np.abs(a-b)))"
[ -n "$AB_SKIP_VARIANTS" ] || timeout -k 10 200 python tools/ab_bits.py 10 14 16 12 11 | grep -c True || exit 1
ROUNDS=${ROUNDS:-3} AB_B=${AB_B:-512,2048} AB_OUT=$O bash tools/ab_libs.sh
