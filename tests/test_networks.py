"""The bundled networks 0-19: CSV parsing, the
knockdown data the NEM constructor draws, DOT output, and (for the small
networks) the oracle's MCMC run -- against the reference's own data files
(tests/golden/networks/, copied from DAGs/networks) and the runs captured from
the reference (networks_mcmc.npz, tests/golden/make_goldens.py
--only-networks)."""
import os
import random

import numpy as np
import pytest
from conftest import GOLDEN, golden

import nemo_oracle as no
from nemo import NEM, dot, utils

NET = os.path.join(GOLDEN, "networks")
Z = golden("networks_mcmc.npz")


def _csv(i, red=False):
    return os.path.join(NET, f"network{i}{'_red' if red else ''}.csv")


@pytest.mark.parametrize("i", range(20))
def test_csv_knockdown_and_dot(i, tmp_path):
    adj, end, err, s, e = utils.read_csv_to_adj(_csv(i))
    assert adj.shape == (s, s) and len(end) == e and len(err) == 2
    m = NEM(adj, end, err, s, e)
    d = np.unpackbits(Z[f"n{i}_D_packed"])[: s * e].reshape(s, e)
    assert np.array_equal(m.observed_knockdown_mat.astype(np.uint8), d)
    assert np.array_equal(utils.initial_order_guess(m.observed_knockdown_mat), Z[f"n{i}_order0"])
    # DAGs/dot.py:4-26 made the bundled .dot files from the CSVs
    for red in (False, True):
        out = tmp_path / f"n{i}{red}.dot"
        dot.generate_dot_language(_csv(i, red), str(out))
        with open(os.path.join(NET, f"network{i}{'_red' if red else ''}.dot")) as fh:
            assert out.read_text() == fh.read()
    # the reduced network's closure is the network (the bundled _red files are
    # reductions, not necessarily minimal ones)
    red_adj = utils.read_csv_to_adj(_csv(i, True))[0]
    assert np.array_equal((utils.ancestor(red_adj) > 0).astype(int), adj)


@pytest.mark.parametrize("i", range(20))
def test_output_dot_of_best_dag(i, tmp_path):
    """main.py:44-53: DOT of ancestor(best_dag) and of its transitive
    reduction, byte-equal to what the reference wrote for its best DAG."""
    from nemo.main import output_handling
    paths = output_handling(Z[f"n{i}_best_dag"], None, str(tmp_path / "output"))
    assert open(paths["infer_closed"]).read() == str(Z[f"n{i}_closed_dot"])
    assert open(paths["infer_red"]).read() == str(Z[f"n{i}_red_dot"])


@pytest.mark.parametrize("i", [0, 8, 9])
def test_oracle_mcmc_matches_reference(i):
    """The oracle's sampler on main.py's configuration (gamma 2S/E, swap 0.90)
    reproduces the reference run: every score, accept and the best order."""
    adj, end, err, s, e = utils.read_csv_to_adj(_csv(i))
    m = NEM(adj, end, err, s, e)
    t = m.get_score_tensor()
    smp = no.OracleSampler(m.U, t, Z[f"n{i}_order0"])
    best = smp.method(swap_prob=0.90, gamma=2.0 * s / e, n_iterations=int(Z["n_iter"]))
    assert np.max(np.abs(np.array(smp.all_scores) - Z[f"n{i}_all_scores"])) <= 1e-9
    assert smp.traj["acc"] == Z[f"n{i}_acc"].tolist()
    assert best == pytest.approx(float(Z[f"n{i}_best_score"]), abs=1e-9)
    assert np.array_equal(smp.best_order, Z[f"n{i}_best_order"])
    random.seed()
