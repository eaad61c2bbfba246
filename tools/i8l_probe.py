"""score_i8l_kernel alone at C3, B = 2048 (bench.py's headline batch): 5 launches
on device inputs, for a PMC pass (tools/gpu_tasks.sh i8l_valu)."""
import sys

import numpy as np
import torch
from scipy.special import expit

sys.path.insert(0, "nem-mcmc-optimization_amd")
from nemo import generator  # noqa: E402
from nemo.engine import Engine  # noqa: E402

m = generator.config_nem("C3")
eng = Engine.for_nem(m)
B = 2048
eng.reserve(B)
rng = np.random.default_rng(5)
pos = torch.from_numpy(np.array([rng.permutation(64) for _ in range(B)], dtype=np.int32)).cuda()
w01 = torch.from_numpy(expit(rng.uniform(-3, 3, (B, 64, 64)))).cuda()
ll = torch.zeros(B, dtype=torch.float64, device="cuda")
st = torch.cuda.current_stream().cuda_stream
assert eng.score_kernel(0, True)[0] == 10
for _ in range(5):
    eng.score_dev(B, pos.data_ptr(), w01.data_ptr(), ll.data_ptr(), stream=st)
torch.cuda.synchronize()
print("ll[0]", float(ll[0]))
