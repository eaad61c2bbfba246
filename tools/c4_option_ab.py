"""A/B of engine options on the C4 sampler itself (run_c4 at one GPU: the
sampler's own inputs, not the bench's random W): rounds of interleaved runs,
ms per MCMC step and the gathered-scores sha of each (equal shas: same bits).

    python tools/c4_option_ab.py NAME=V1,V2 [chains=128] [steps=10] [rounds=2]   (GPU box)
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "nem-mcmc-optimization_amd"))
from nemo import generator  # noqa: E402
from nemo.chains import run_c4  # noqa: E402
from nemo.engine import Engine  # noqa: E402


def main():
    name, vals = sys.argv[1].split("=")
    vals = [int(v) for v in vals.split(",")]
    chains = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    m = generator.config_nem("C3")
    eng = Engine.for_nem(m)
    base = eng.get_option(name)
    for r in range(rounds):
        for v in vals:
            eng.set_option(name, v)
            out = run_c4(m, eng, n_chains=chains, steps=steps, warmup_steps=1)
            print(f"round {r} {name}={v}: {out['ms_per_step']:.3f} ms/step, sha {out['scores_sha256']}", flush=True)
    eng.set_option(name, base)


if __name__ == "__main__":
    main()
