"""End-to-end runs on the bundled networks 0-19 on the GPU (SURVEY.md 8(f)
rank 4): ``nemo.main.run_network`` with main.py's MCMC configuration against
the reference's runs (networks_mcmc.npz): every step's score within 1e-6, the
same accept decisions, best score, best order and best DAG, and the DOT
output of the best DAG byte for byte."""
import os

import numpy as np
import pytest
from conftest import GOLDEN, golden

from nemo.main import run_network

pytestmark = pytest.mark.gpu
Z = golden("networks_mcmc.npz")


@pytest.mark.parametrize("i", range(20))
def test_network_mcmc_matches_reference(i, tmp_path):
    r = run_network(os.path.join(GOLDEN, "networks", f"network{i}.csv"), method="mcmc",
                    n_iterations=int(Z["n_iter"]), out_dir=str(tmp_path / "output"))
    assert np.array_equal(r["order0"], Z[f"n{i}_order0"])
    assert np.max(np.abs(r["all_scores"] - Z[f"n{i}_all_scores"])) <= 1e-6
    assert np.array_equal(r["accepted"], Z[f"n{i}_acc"])
    assert abs(r["score"] - float(Z[f"n{i}_best_score"])) <= 1e-6
    assert np.array_equal(r["best_order"], Z[f"n{i}_best_order"])
    assert np.array_equal(r["best_dag"], Z[f"n{i}_best_dag"])
    assert open(r["paths"]["infer_closed"]).read() == str(Z[f"n{i}_closed_dot"])
    assert open(r["paths"]["infer_red"]).read() == str(Z[f"n{i}_red_dot"])
