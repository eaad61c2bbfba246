cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/ab2; export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/ab_bits_libs.py gpurun_out/ab2/new.npy > gpurun_out/ab2/bits_new.log 2>&1 || exit 1
NEMO_LIBRARY=$(pwd)/nem-mcmc-optimization_amd/nemo/libnemo_old.so timeout -k 10 200 python tools/ab_bits_libs.py gpurun_out/ab2/old.npy > gpurun_out/ab2/bits_old.log 2>&1 || exit 1
python -c "import numpy as np; a=np.load('gpurun_out/ab2/new.npy'); b=np.load('gpurun_out/ab2/old.npy'); print('bits equal:', np.array_equal(a,b), a.shape)"
timeout -k 10 200 python tools/ab_bits.py 10 14 16 12 11 || exit 1
ROUNDS=3 AB_B=512,2048 AB_OUT=gpurun_out/ab2 bash tools/ab_libs.sh
