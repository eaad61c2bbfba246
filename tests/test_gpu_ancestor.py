"""GPU: the step's W~ and ancestor_x made on the device (csrc/nemo_ancestor.hip:
getrf + getri of scipy's OpenBLAS restated) against scipy's expit and
scipy.linalg.inv -- the reference's own calls (nem_order_mcmc.py:98-103,
:185) -- to the bit, for every S up to 64, with and without a cap and with the
stale entries the sampler leaves outside the permissible set; the fused step
from W against the fused step from the host's W~ / ancestor_x; scipy's own
errors for a singular or non-finite I - W~; chain batches with the device's
ancestor_x against the host's (InvPool) step for step."""
import numpy as np
import pytest
from scipy.linalg import LinAlgError, inv
from scipy.special import expit

from nemo import _lib, generator
from nemo.chains import ChainBatch
from nemo.engine import Engine
from nemo.invpool import InvPool
from nemo.nem_order_mcmc import SIG0, SIG1, permissible_batch

pytestmark = pytest.mark.gpu


def _bits_equal(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))


def _host(pos, w, cap=0):
    """chains._prepare's host computation: scipy's expit and inv."""
    mask = permissible_batch(pos, cap)
    sig = w.copy()
    sig[mask] = expit(w[mask])
    eye = np.identity(w.shape[-1])
    return sig, np.stack([np.clip(inv(eye - s) - eye, 0, 1) for s in sig])


def _weights(rng, pos, stale, diag=False):
    n, s = pos.shape
    mask = permissible_batch(pos)
    w = np.where(mask, rng.uniform(-4, 4, (n, s, s)), 0.0)
    if stale:   # left by earlier orders: expit(x*) values outside today's parents
        w = np.where(~mask & (rng.random((n, s, s)) < 0.15), rng.uniform(0, 1, (n, s, s)), w)
    for k in range(n):
        np.fill_diagonal(w[k], rng.uniform(-0.5, 0.5, s) if diag else 0.0)
    return w


def _device(eng, pos, w, cap=0):
    import torch
    n = w.shape[0]
    dpos = torch.from_numpy(np.ascontiguousarray(pos, dtype=np.int32)).cuda()
    dw = torch.from_numpy(np.ascontiguousarray(w)).cuda()
    d01, danc = torch.empty_like(dw), torch.empty_like(dw)
    dfl = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    _lib.check(_lib.load().nemo_ancestor_dev(eng._ctx, n, dpos.data_ptr(), dw.data_ptr(), int(cap), d01.data_ptr(),
                                             danc.data_ptr(), dfl.data_ptr(), st))
    torch.cuda.synchronize()
    return d01.cpu().numpy(), danc.cpu().numpy(), dfl.cpu().numpy()


@pytest.mark.parametrize("s", [2, 3, 5, 11, 16, 17, 33, 48, 63, 64])
def test_ancestor_equals_scipy_bit_for_bit(s):
    eng = Engine.for_nem(generator.synthetic_nem(s, 40, 0))
    rng = np.random.default_rng(100 + s)
    n = 24
    pos = np.array([rng.permutation(s) for _ in range(n)], dtype=np.int32)
    for stale, diag in ((False, False), (True, False), (True, True)):
        w = _weights(rng, pos, stale, diag)
        for cap in ((0, 3) if s >= 5 else (0,)):
            sig, anc = _host(pos, w, cap)
            d01, danc, fl = _device(eng, pos, w, cap)
            assert np.array_equal(fl, np.zeros(n)), fl
            assert _bits_equal(d01, sig), (stale, diag, cap)
            assert _bits_equal(danc, anc), (stale, diag, cap)
    eng.close()


def test_ancestor_flags_and_scipys_errors():
    m = generator.synthetic_nem(16, 40, 0)
    eng = Engine.for_nem(m)
    rng = np.random.default_rng(4)
    pos = np.array([rng.permutation(16) for _ in range(3)], dtype=np.int32)
    w = _weights(rng, pos, True)
    i = int(np.argmin(pos[1]))        # first in chain 1's order: no permissible parents
    w[1, i, :] = 0.0
    w[1, i, i] = 1.0                  # row i of I - W~ all zero: singular
    w[2, 5, 5] = np.inf               # I - W~ not finite
    _, _, fl = _device(eng, pos, w)
    assert fl[0] == 0 and fl[1] == 1 and fl[2] & 2
    with pytest.raises(LinAlgError):
        eng.optimal_weights_w(pos[:2], w[:2], SIG0, SIG1)
    with pytest.raises(ValueError):
        eng.optimal_weights_w(pos[2:], w[2:], SIG0, SIG1)
    # the host's own calls raise the same
    with pytest.raises(LinAlgError):
        _host(pos[1:2], w[1:2])
    with pytest.raises(ValueError):
        _host(pos[2:], w[2:])
    # the engine still steps afterwards
    out = eng.optimal_weights_w(pos[:1], w[:1], SIG0, SIG1, raise_on_fail=False)
    assert np.isfinite(out[3]).all()
    eng.close()


@pytest.mark.parametrize("cap,overlap", [(0, 1), (3, 1), (0, 0)])
def test_step_from_w_equals_step_from_host_ancestor(cap, overlap):
    """nemo_optimal_weights_w (W in) against nemo_optimal_weights with the
    host's W~ / ancestor_x: every output to the bit, direct and queued, with
    ancestor_x beside eval #1 on a second stream (option anc_overlap 1, the
    default) or in line."""
    m = generator.config_nem("C3")
    eng = Engine.for_nem(m)
    eng.set_option("anc_overlap", overlap)
    rng = np.random.default_rng(21 + cap)
    n = 16
    pos = np.array([rng.permutation(64) for _ in range(n)], dtype=np.int32)
    w = _weights(rng, pos, True)
    sig, anc = _host(pos, w, cap)
    ref = eng.optimal_weights(pos, sig, anc, w, SIG0, SIG1, cap=cap, raise_on_fail=False)
    got = eng.optimal_weights_w(pos, w, SIG0, SIG1, cap=cap, raise_on_fail=False)
    assert _bits_equal(got[0], sig) and _bits_equal(got[1], anc)
    for a, b in zip(got[2:5], ref[:3]):
        assert _bits_equal(a, b)
    assert np.array_equal(got[5], ref[3])
    # queued: two calls in flight, ended in order
    calls = [eng.bind_optimal_weights_w(pos[h::2], w[h::2], SIG0, SIG1, cap=cap) for h in (0, 1)]
    for c in calls:
        c.begin()
    for h, c in enumerate(calls):
        c.end()
        wn, ll1, lld, info = c.result(raise_on_fail=False)
        assert _bits_equal(c.anc, anc[h::2]) and _bits_equal(wn, ref[0][h::2])
        assert _bits_equal(ll1, ref[1][h::2]) and _bits_equal(lld, ref[2][h::2])
    eng.close()


def test_chain_batch_device_ancestor_equals_host_pool():
    """ChainBatch with the device's ancestor_x (the default at S <= 64) and
    with the host's (InvPool workers), pipelined in two groups: the same
    proposals, scores, accepts, weights and ancestor_x, step for step."""
    m = generator.config_nem("C3")
    eng = Engine.for_nem(m)
    from nemo import utils
    order = utils.initial_order_guess(m.observed_knockdown_mat)
    res = []
    pool = InvPool(64, 8, n_workers=1)
    try:
        for pl in (None, pool):
            cb = ChainBatch(m, [order] * 8, seeds=list(range(40, 48)), engine=eng, on_fail="continue",
                            inv_pool=pl, groups=2)
            best, orders = cb.run(6)
            res.append((best, orders, cb.accepted, [c.parent_weights.copy() for c in cb.chains],
                        [c.ancestor_x.copy() for c in cb.chains],
                        [np.array(c.all_score_list) for c in cb.chains]))
    finally:
        pool.close()
    (b1, o1, a1, w1, x1, s1), (b2, o2, a2, w2, x2, s2) = res
    assert _bits_equal(b1, b2) and np.array_equal(o1, o2) and np.array_equal(a1, a2)
    for u, v in zip(w1 + x1 + s1, w2 + x2 + s2):
        assert _bits_equal(u, v)
    eng.close()
