"""Inputs of the golden order-score evaluations (tests/golden/eval_*.npz).

Evaluation k of a model with S S-genes takes (perm, raw W):
  k < 20      random_chain_inputs(S, k): a random order, W ~ U(-3, 3)
              (the only kind the first goldens held)
  20 ... 23   W ~ U(-30, 30): weights saturated at expit ~ 1e-13 / 1 - 1e-13
  24 / 25     W = -inf / +inf: every weight exactly 0 / exactly 1
  26          W = 0: every weight 1/2
  27 / 28     the identity order / its reverse, W ~ U(-3, 3)
  29 / 30     W = +30 / -30 everywhere
  31          W = +inf or -inf per entry (weights 0 and 1 mixed)
The raw W goes through expit as in the reference (nem_order_mcmc.py:84-86);
the last node of every order has S - 1 permissible parents.
"""
import numpy as np

KINDS = ["random"] * 20 + ["saturated"] * 4 + ["zero", "one", "half", "identity", "reverse",
                                                "plus30", "minus30", "mixed01"]


def eval_inputs(s, k):
    from nemo import generator
    if k < 20:
        perm, _pos, w = generator.random_chain_inputs(s, k)
        return perm, w
    rng = np.random.default_rng(5000 + k)
    perm = rng.permutation(s)
    kind = KINDS[k]
    if kind == "saturated":
        return perm, rng.uniform(-30, 30, (s, s))
    if kind in ("identity", "reverse"):
        perm = np.arange(s) if kind == "identity" else np.arange(s)[::-1].copy()
        return perm, rng.uniform(-3, 3, (s, s))
    const = {"zero": -np.inf, "one": np.inf, "half": 0.0, "plus30": 30.0, "minus30": -30.0}
    if kind in const:
        return perm, np.full((s, s), const[kind])
    return perm, np.where(rng.random((s, s)) < 0.5, np.inf, -np.inf)
