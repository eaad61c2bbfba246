"""End-to-end MCMC throughput: ChainBatch (host state machines + one fused
device call per step) at C3, chain-steps per second, with a cProfile of the
host side.   python tools/mcmc_e2e.py [--chains 16] [--steps 20] [--profile]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "nem-mcmc-optimization_amd"))
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=16)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--local-prod", type=int, default=1)
    ap.add_argument("--seed-base", type=int, default=1234)
    ap.add_argument("--on-fail", default="continue", choices=["raise", "continue"])
    ap.add_argument("--inv-workers", type=int, default=0, help="InvPool worker processes (0: serial inv)")
    ap.add_argument("--timeline", action="store_true", help="print per-phase timestamps of 3 steps")
    ap.add_argument("--groups", type=int, default=0, help="pipeline chain groups (0: ChainBatch default)")
    a = ap.parse_args()
    from nemo import generator, utils
    from nemo.chains import ChainBatch
    m = generator.config_nem(a.config)
    from nemo.invpool import InvPool
    order = utils.initial_order_guess(m.observed_knockdown_mat)
    pool = InvPool(m.num_s, a.chains, a.inv_workers) if a.inv_workers else None
    cb = ChainBatch(m, [order] * a.chains, seeds=[a.seed_base + c for c in range(a.chains)],
                    on_fail=a.on_fail, inv_pool=pool)
    cb.engine.set_option("local_prod", a.local_prod)
    cb.run(2)  # warm-up
    cb = ChainBatch(m, [order] * a.chains, seeds=[a.seed_base + c for c in range(a.chains)], engine=cb.engine,
                    on_fail=a.on_fail, inv_pool=pool, groups=a.groups or None)
    marks = []
    if a.timeline:
        import threading
        from nemo import chains as ch

        def wrap(name, f):
            def g(*args, **kw):
                t = time.perf_counter()
                try:
                    return f(*args, **kw)
                finally:
                    marks.append((t, time.perf_counter(), name, threading.get_ident()))
            return g
        from nemo import engine as en
        for nm in ("_prepare_start", "_prepare_end", "_finish"):
            setattr(ch, nm, wrap(nm, getattr(ch, nm)))
        en._OptimalWeightsCall.begin = wrap("step_begin", en._OptimalWeightsCall.begin)
        en._OptimalWeightsCall.end = wrap("step_end_wait", en._OptimalWeightsCall.end)
        NM = type(cb.chains[0])
        NM.reset = wrap("reset", NM.reset)
        NM.accepting = wrap("accepting", NM.accepting)
    prof = cProfile.Profile() if a.profile else None
    t0 = time.perf_counter()
    if prof:
        prof.enable()
    best, _ = cb.run(a.steps)
    if prof:
        prof.disable()
    dt = time.perf_counter() - t0
    print(f"{a.config}: groups {a.groups or 'default'}, {a.chains} chains x {a.steps} steps in {dt:.3f} s: "
          f"{1e3 * dt / a.steps:.2f} ms/step, {a.chains * a.steps / dt:.0f} chain-steps/s; best {best.max():.3f}")
    if marks:
        marks.sort()
        base = marks[len(marks) // 2][0]
        main_tid = marks[0][3]
        agg = []
        for t0_, t1_, nm, tid in marks:
            if not 0 <= t0_ - base < 3 * dt / a.steps:
                continue
            if agg and agg[-1][2] == nm and nm in ("reset", "accepting"):
                agg[-1][1], agg[-1][3] = t1_, agg[-1][3] + 1
                continue
            agg.append([t0_, t1_, nm, 1, tid])
        print(f"timeline base (perf_counter ns): {int(base * 1e9)}")
        for t0_, t1_, nm, cnt, tid in agg:
            print(f"{1e6 * (t0_ - base):9.1f} us {1e6 * (t1_ - t0_):8.1f} us  {'main' if tid == main_tid else 'dev '} {nm} x{cnt}")
    if prof:
        pstats.Stats(prof).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
