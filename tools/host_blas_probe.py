"""Which OpenBLAS kernels the host's scipy / numpy run, and the bits they
give: sha256 of scipy.linalg.inv of fixed matrices (the ancestor_x inputs'
shape, 64 x 64 and 11 x 11), of np.log / np.exp / expit / logaddexp over
fixed inputs, and of small dpotrf / dtrtrs calls.  Run here and on the GPU
box: equal hashes mean the box's host arithmetic is this container's."""
import hashlib
import json
import platform

import numpy as np
from scipy.linalg import inv, lapack
from scipy.special import expit


def h(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()[:16]


def main():
    from threadpoolctl import threadpool_info
    rng = np.random.default_rng(7)
    out = {"cpu": platform.processor(), "pools": [(p.get("prefix"), p.get("architecture"), p.get("version"))
                                                  for p in threadpool_info()]}
    for s in (11, 64):
        w = np.triu(rng.uniform(0, 1, (s, s)), 1) * (rng.random((s, s)) < 0.5)
        out[f"inv{s}"] = h(inv(np.identity(s) - expit(w) * (w > 0)))
    x = rng.uniform(0.5, 4.0, 100000)
    out["log"] = h(np.log(x))
    out["exp"] = h(np.exp(rng.uniform(-30, 5, 100000)))
    out["expit"] = h(expit(rng.normal(0, 3, 100000)))
    a, b = rng.normal(-50, 20, 100000), rng.normal(-50, 20, 100000)
    out["logaddexp"] = h(np.logaddexp(a, b))
    m = rng.normal(size=(13, 10))
    c, _ = lapack.dpotrf(np.asfortranarray(m.T @ m), lower=0, clean=1)
    out["potrf10"] = h(c)
    out["trtrs"] = h(lapack.dtrtrs(c, rng.normal(size=(10, 7)), lower=0, trans=1)[0])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
