#!/bin/bash
# Cost breakdown of the int8 score kernel: kernel time (C3, 512 evals) of
# instrumented builds with the exps (1), the MFMAs (2) or the digit prep (8)
# removed (bits combine).  Build the variants here (CPU container) with
# `bash tools/ablate.sh build`, then run `bash tools/ablate.sh` on the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARIANTS="${VARIANTS:-1 2 8 9}"
if [ "$1" = build ]; then
  for v in $VARIANTS; do
    python -c "import sys; sys.path.insert(0,'nem-mcmc-optimization_amd'); from nemo import build; print(build.build(out='nem-mcmc-optimization_amd/nemo/libnemo_abl$v.so', defines=['NEMO_I8_ABLATE=$v']))"
  done
  exit 0
fi
mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
for round in $(seq ${ROUNDS:-1}); do for v in 0 $VARIANTS; do
  lib=""; [ $v -gt 0 ] && lib="$(pwd)/nem-mcmc-optimization_amd/nemo/libnemo_abl$v.so"
  NEMO_LIBRARY=$lib timeout -k 10 300 python - <<PY || exit 1
import sys, numpy as np
sys.path.insert(0, "nem-mcmc-optimization_amd")
import torch
from scipy.special import expit
from nemo import generator
from nemo.engine import Engine
m = generator.config_nem("C3"); eng = Engine.for_nem(m); B = int("${ABL_B:-512}"); eng.reserve(B)
eng.set_option("fact_kernel", int("${FK:-0}"))
rng = np.random.default_rng(5)
pos = torch.from_numpy(np.array([rng.permutation(64) for _ in range(B)], dtype=np.int32)).cuda()
w01 = torch.from_numpy(expit(rng.uniform(-3, 3, (B, 64, 64)))).cuda()
ll = torch.zeros(B, dtype=torch.float64, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for _ in range(5): eng.score_dev(B, pos.data_ptr(), w01.data_ptr(), ll.data_ptr(), stream=st)
torch.cuda.synchronize(); eng.timing(True)
for _ in range(20): eng.score_dev(B, pos.data_ptr(), w01.data_ptr(), ll.data_ptr(), stream=st)
torch.cuda.synchronize(); ms, n = eng.timing_read()
print(f"ablate=$v kernel {ms / n * 1e3:.1f} us per {B} evals")
PY
done; done
