"""Small profiling target: a few launches of each score-kernel variant at C3
(and C5), for rocprofv3 PMC passes.  python tools/prof_target.py [--reps 3]"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "nem-mcmc-optimization_amd"))
import numpy as np  # noqa: E402


def main():
    import torch
    from scipy.special import expit

    from nemo import generator
    from nemo.engine import Engine
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 3
    cfgs = os.environ.get("NEMO_PROF_CONFIGS", "C3").split(",")
    groups = [int(g) for g in os.environ.get("NEMO_PROF_GROUPS", "1,4").split(",")]
    B = int(os.environ.get("NEMO_PROF_BATCH", "128"))
    for cfg in cfgs:
        S, E, seed, cap, dtype = generator.CONFIGS[cfg]
        m = generator.config_nem(cfg)
        eng = Engine.for_nem(m, dtype=dtype)
        eng.set_option("score_path", int(os.environ.get("NEMO_PROF_PATH", "0")))
        eng.set_option("fact_kernel", int(os.environ.get("NEMO_PROF_FK", "0")))
        eng.reserve(B)
        rng = np.random.default_rng(5)
        pos = torch.from_numpy(np.array([rng.permutation(S) for _ in range(B)], dtype=np.int32)).cuda()
        w01 = torch.from_numpy(expit(rng.uniform(-3, 3, (B, S, S)))).cuda()
        ll = torch.zeros(B, dtype=torch.float64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        for g in (groups if cap == 0 else [1]):
            for _ in range(reps):
                eng.score_dev(B, pos.data_ptr(), w01.data_ptr(), ll.data_ptr(), cap=cap, stream=st, group=g)
        torch.cuda.synchronize()
        eng.close()
    print("done")


if __name__ == "__main__":
    main()
