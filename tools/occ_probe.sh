cd $GRAFT_REPO_ROOT
for lib in "" "$(pwd)/nem-mcmc-optimization_amd/nemo/libnemo_abl3w.so"; do
NEMO_LIBRARY=$lib timeout -k 10 300 python - <<PY || exit 1
import sys, numpy as np
sys.path.insert(0, "nem-mcmc-optimization_amd")
import torch
from scipy.special import expit
from nemo import generator
from nemo.engine import Engine
m = generator.config_nem("C3"); eng = Engine.for_nem(m)
for B in (128, 512, 2048):
    eng.reserve(B)
    rng = np.random.default_rng(5)
    pos = torch.from_numpy(np.array([rng.permutation(64) for _ in range(B)], dtype=np.int32)).cuda()
    w01 = torch.from_numpy(expit(rng.uniform(-3, 3, (B, 64, 64)))).cuda()
    ll = torch.zeros(B, dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(5): eng.score_dev(B, pos.data_ptr(), w01.data_ptr(), ll.data_ptr(), stream=st)
    torch.cuda.synchronize(); eng.timing(True)
    for _ in range(20): eng.score_dev(B, pos.data_ptr(), w01.data_ptr(), ll.data_ptr(), stream=st)
    torch.cuda.synchronize(); ms, n = eng.timing_read(); eng.timing(False)
    print(f"lib={'$lib'[-14:]} B={B} kernel {ms / n * 1e3:.1f} us -> {B / (ms / n) * 1e3 / 1e6:.2f} M evals/s")
PY
done
