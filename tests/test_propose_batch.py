"""The group-wide proposal of nemo.chains (propose_batch) against the
per-chain ``get_new_order`` + ``reset`` (nem_order_mcmc.py:231-255, :50-77,
restated in NEMOrderMCMC), on the CPU: same random draws, same orders,
same weights after the reset quirks, same positions and masks."""
import copy
import random

import numpy as np
import pytest

from nemo.chains import propose_batch
from nemo.nem_order_mcmc import NEMOrderMCMC


def _bare_chain(s, cap, seed, rng):
    c = object.__new__(NEMOrderMCMC)
    c.num_s, c.cap = s, cap
    c.parent_weights = rng.choice([0.0, 0.5, 1.0, -2.0, 3.7], size=(s, s))
    c.rng = random.Random(seed)
    return c


@pytest.mark.parametrize("s,cap,swap_prob", [(8, 0, 0.95), (13, 3, 0.5), (64, 0, 0.5), (40, 6, 0.0), (2, 0, 1.0)])
def test_propose_batch_equals_per_chain_reset(s, cap, swap_prob):
    rng = np.random.default_rng(s * 100 + cap)
    n = 7
    batch = [_bare_chain(s, cap, 1000 + k, rng) for k in range(n)]
    single = [copy.deepcopy(c) for c in batch]
    curr = [rng.permutation(s) for _ in range(n)]
    curr_b = [p.copy() for p in curr]
    wb = None
    for _step in range(12):
        props = []
        for c, p in zip(single, curr):
            perm, i1, i2 = c.get_new_order(p, swap_prob=swap_prob)
            c.reset(perm_order=perm, i1=i1, i2=i2)
            props.append(perm)
        perms, (pos, w, mask) = propose_batch(batch, curr_b, swap_prob, w=wb if _step % 2 else None)
        for k in range(n):
            a, b = single[k], batch[k]
            assert np.array_equal(perms[k], props[k]) and perms[k].dtype == props[k].dtype
            assert np.array_equal(b.parent_weights, a.parent_weights)
            assert np.array_equal(b._pos, a._pos) and b._pos.dtype == a._pos.dtype
            assert np.array_equal(b._mask, a._mask)
            assert b._parents is None and b.ll == 0.0
            assert a.rng.getstate() == b.rng.getstate()
            assert all(np.array_equal(x, y) for x, y in zip(a.parents_list, b.parents_list))
            assert np.shares_memory(b.parent_weights, w) and np.shares_memory(b._mask, mask)
        # accept about half of the proposals (the caller's curr_perm update)
        for k in range(n):
            if (k + _step) % 2:
                curr[k], curr_b[k] = props[k], perms[k]
        # the device step hands back fresh weights (one stack: updated in
        # place by the next proposal when passed as ``w``)
        wb = rng.normal(size=(n, s, s))
        for k, (a, b) in enumerate(zip(single, batch)):
            a.parent_weights, b.parent_weights = wb[k].copy(), wb[k]
