"""Shader cycles per phase of the ancestor kernel (csrc/nemo_ancestor.hip) from
its instrumented build (NEMO_ANC_PROFILE=1, nemo/libnemo_ancprof.so):
    NEMO_LIBRARY=.../libnemo_ancprof.so python tools/anc_phases.py [chains=16]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nem-mcmc-optimization_amd"))
from nemo import _lib, generator  # noqa: E402
from nemo.engine import Engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    eng = Engine.for_nem(generator.config_nem("C3"))
    rng = np.random.default_rng(1)
    pos = np.array([rng.permutation(64) for _ in range(n)], dtype=np.int32)
    w = np.where(pos[:, None, :] < pos[:, :, None], rng.uniform(-3, 3, (n, 64, 64)), 0.0)
    dpos, dw = torch.from_numpy(pos).cuda(), torch.from_numpy(w).cuda()
    d01, danc = torch.empty_like(dw), torch.empty_like(dw)
    dfl = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    rows = []
    for _ in range(5):
        _lib.check(_lib.load().nemo_ancestor_dev(eng._ctx, n, dpos.data_ptr(), dw.data_ptr(), 0, d01.data_ptr(),
                                                 danc.data_ptr(), dfl.data_ptr(), st))
        torch.cuda.synchronize()
        rows.append(danc[-1, 0, :8].cpu().numpy())
    r = np.median(np.array(rows), axis=0)
    names = ["getrf", "trti2", "getri gemv", "swaps+clip", "  getf2", "  laswp", "  trsm", "  gemm"]
    for k, v in zip(names, r):
        print(f"{k:12s} {v:10.0f} cycles")


if __name__ == "__main__":
    main()
