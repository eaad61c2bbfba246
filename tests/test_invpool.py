"""InvPool (nemo/invpool.py): the ancestor_x inversions of ChainBatch in
worker processes give the bits of chains.inv_stack (= scipy.linalg.inv) and
scipy's errors for singular or non-finite matrices."""
import numpy as np
import pytest
from scipy.linalg import inv

from nemo.chains import inv_stack
from nemo.invpool import InvPool


@pytest.fixture(scope="module")
def pool():
    p = InvPool(16, 12, n_workers=3)
    yield p
    p.close()


def _mats(n, s, seed):
    rng = np.random.default_rng(seed)
    w = rng.uniform(0, 1, (n, s, s)) * np.tril(np.ones((s, s)), -1)
    return np.identity(s) - w


def test_pool_bits_equal_serial(pool):
    for n in (1, 2, 5, 12):
        a = _mats(n, 16, n)
        pool.start(a)
        out = pool.finish()
        assert np.array_equal(out, inv_stack(a))
        assert np.array_equal(out[0], inv(a[0]))


def test_pool_errors_and_capacity(pool):
    a = _mats(4, 16, 9)
    a[2][:] = 0.0
    pool.start(a)
    with pytest.raises(np.linalg.LinAlgError):
        pool.finish()
    a = _mats(3, 16, 10)
    a[1][0, 0] = np.nan
    pool.start(a)
    with pytest.raises(ValueError):
        pool.finish()
    with pytest.raises(ValueError):
        pool.start(_mats(13, 16, 0))
    # a start whose finish never ran (the caller raised in between) is drained
    pool.start(_mats(5, 16, 1))
    b = _mats(6, 16, 2)
    pool.start(b)
    assert np.array_equal(pool.finish(), inv_stack(b))


def test_pool_prepare_bits_equal(pool):
    """start_prepare / finish_prepare: W~ and ancestor_x of chains._prepare."""
    from scipy.special import expit
    rng = np.random.default_rng(3)
    n, s = 7, 16
    ws = [rng.uniform(-3, 3, (s, s)) for _ in range(n)]
    masks = []
    for _ in range(n):
        pos = rng.permutation(s)
        masks.append(pos[None, :] < pos[:, None])   # (child, parent): parent earlier in the order
    pool.start_prepare(ws, masks)
    sig, anc = pool.finish_prepare()
    eye = np.identity(s)
    for k in range(n):
        ref = ws[k].copy()
        ref[masks[k]] = expit(ws[k][masks[k]])
        assert np.array_equal(sig[k], ref)
        assert np.array_equal(anc[k], np.clip(inv_stack((eye - ref)[None])[0] - eye, 0, 1))
    with pytest.raises(RuntimeError):
        pool.start(_mats(2, 16, 0))
        pool.finish_prepare()


def test_default_workers_under_local_world_size(monkeypatch):
    """default_workers: the cores this rank may use, shared by the node's
    LOCAL_WORLD_SIZE ranks, one left for the rank itself, at least 1, capped
    at 8 -- e.g. the 8-rank C4 run on a 256-core host gets 8 workers per rank
    (64 helpers in all), on a 64-core host 7, on 16 cores 1."""
    import os

    from nemo import invpool
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    for cores, want in ((256, 8), (64, 7), (16, 1), (8, 1), (4, 1)):
        monkeypatch.setattr(os, "sched_getaffinity", lambda pid, n=cores: set(range(n)))
        assert invpool.default_workers() == want, cores
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(12)))
    assert invpool.default_workers() == 8
    assert invpool.default_workers(cap=4) == 4
    assert invpool.default_workers(local_world=3) == 3
