"""Nondeterminism probe for the fused step under two processes sharing one
GPU (the N = 2 rehearsal of tests/test_gpu_rehearsal.py): every fused call
of the chain batches is run twice and the two results compared bit for bit;
a difference is printed with the chains, pairs and values it touches.

    python tools/race_probe.py [repeats=2] [NAME=VALUE engine options ...]   (GPU box)
"""
import hashlib
import os
import random
import socket
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "nem-mcmc-optimization_amd"))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _patch(tag, opts):
    """Wrap chains.optimal_weights_batch: each call's step recomputed and compared."""
    from nemo import chains
    from nemo.nem_order_mcmc import SIG0, SIG1
    orig = chains.optimal_weights_batch
    stats = {"calls": 0, "bad": 0}

    def wrapped(cs, engine, use_nem=False, cap=0, raise_on_fail=True, pool=None):
        for k, v in opts.items():
            engine.set_option(k, v)
        pos = np.stack([c._pos for c in cs]).astype(np.int32)
        w = np.stack([c.parent_weights for c in cs]).copy()
        out = orig(cs, engine, use_nem=use_nem, cap=cap, raise_on_fail=raise_on_fail, pool=pool)
        if engine.S < 64 or np.any(np.asarray(out) > 0):
            print(f"[{tag}] step S={engine.S} n={len(cs)} lld {np.round(np.asarray(out), 3).tolist()}", flush=True)
        if pool is None and engine.device_ancestor:
            a = engine.bind_optimal_weights_w(pos, w, SIG0, SIG1, cap=cap, want_prep=False)
            a.run()
            b = engine.bind_optimal_weights_w(pos, w, SIG0, SIG1, cap=cap, want_prep=False)
            b.run()
            stats["calls"] += 1
            for name in ("w_new", "ll1", "lld", "info"):
                x, y = getattr(a, name), getattr(b, name)
                if not np.array_equal(x.view(np.uint8), y.view(np.uint8)):
                    stats["bad"] += 1
                    d = np.argwhere(x != y)
                    print(f"[{tag}] call {stats['calls']} n={len(cs)} S={engine.S}: {name} differs at {len(d)} "
                          f"entries, first {d[:6].tolist()}", flush=True)
                    for idx in d[:4]:
                        t = tuple(idx)
                        print(f"    {t}: {x[t]!r} vs {y[t]!r}", flush=True)
            eq = np.array_equal(a.lld, np.asarray(out))
            if not eq:
                print(f"[{tag}] call {stats['calls']}: the sampler's lld {np.asarray(out)} vs recomputed {a.lld}",
                      flush=True)
        return out

    chains.optimal_weights_batch = wrapped

    from nemo.engine import Engine
    oscore = Engine.score

    def score(self, pos, w01, cap=0, **kw):
        ra = oscore(self, pos, w01, cap=cap, **kw)
        rb = oscore(self, pos, w01, cap=cap, **kw)
        a, b = (ra["ll"], rb["ll"]) if isinstance(ra, dict) else (ra, rb)
        stats["scores"] = stats.get("scores", 0) + 1
        if not np.array_equal(np.asarray(a), np.asarray(b)) or np.any(np.asarray(a) > 0):
            stats["bad_scores"] = stats.get("bad_scores", 0) + 1
            print(f"[{tag}] score call {stats['scores']} S={self.S} n={len(np.atleast_2d(pos))}: {a} vs {b}",
                  flush=True)
        return ra

    Engine.score = score
    return stats


def _rank_main(rank, world, port, q, opts):
    import torch.distributed as dist

    from nemo import generator, utils
    from nemo.chains import run_c4
    from nemo.engine import Engine
    from nemo.replicas import ReplicaExchange
    stats = _patch(f"rank{rank}", opts)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = generator.config_nem("C3")
        eng = Engine.for_nem(m)
        run_c4(m, eng, n_chains=32, steps=3, warmup_steps=0, inv_workers=1)
        m2 = generator.config_nem("C2")
        rx = ReplicaExchange(m2, utils.initial_order_guess(m2.observed_knockdown_mat), n_replicas=6,
                             rng=random.Random(2025), rank=rank, world=world)
        rounds = []
        for k in range(2):
            rx.step(2, k % 2 == 0)
            rounds.append(rx.scores.copy())
        q.put((rank, stats, [r.tolist() for r in rounds]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    opts = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[2:]}
    ctx = mp.get_context("spawn")
    for r in range(reps):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_rank_main, args=(k, 2, port, q, opts)) for k in range(2)]
        for p in procs:
            p.start()
        got = []
        for _ in range(2):
            while True:
                try:
                    got.append(q.get(timeout=20))
                    break
                except Exception:
                    if any(p.exitcode not in (None, 0) for p in procs):
                        for p in procs:
                            p.kill()
                        raise SystemExit("a rank failed")
                    print("waiting", flush=True)
        for p in procs:
            p.join(timeout=120)
        for rank, st, rounds in sorted(got, key=lambda g: g[0]):
            print(f"rep {r} rank {rank}: {st}; scores {hashlib.sha256(str(rounds).encode()).hexdigest()[:12]} "
                  f"{np.round(rounds[0], 3).tolist()}", flush=True)


if __name__ == "__main__":
    main()
