"""End-to-end runs on a bundled network (reference main.py).

The reference's ``main()`` (main.py:56-121) reads ``DAGs/networks/networkN``,
builds the NEM, guesses an initial order, runs one optimizer and writes the
inferred DAG as DOT files (``output_handling``, main.py:44-53).  This module
keeps those steps and names; the optimizer is one of the three the reference
wires up, each on the GPU:

* ``"inverse"`` -- ``InverseMethod(...).optimize()``, main()'s active path
  (main.py:115-116);
* ``"mcmc"``    -- ``NEMOrderMCMC.method`` with main()'s settings (gamma =
  2S/E, swap_prob 0.90, main.py:62-70, 88-91);
* ``"replica"`` -- ``replica_exchange_method`` (main.py:98).

Not reproduced: PDF rendering (graphviz, DAGs/graph.py; not installed here)
and wandb logging.  ``output_handling`` copies the network's bundled PDFs
when they exist, as the reference does.

    python -m nemo.main --network path/to/network11.csv --method inverse --out DIR
"""
from __future__ import annotations

import argparse
import os
import shutil

import numpy as np

from . import dot, utils
from .nem import NEM

OUTPUT_FILES = ["output.pdf", "output.dot", "output.gv", "infer_closed.dot", "infer_closed.pdf",
                "infer_closed.gv", "infer_red.dot", "infer_red.pdf", "infer_red.gv", "real_red.dot",
                "real_red.pdf", "real_red.gv", "real_closed.pdf"]   # main.py:27-30


def initial_order_guess(observed_knockdown_mat):
    """main.py:16-24 (the same function as utils.initial_order_guess)."""
    return utils.initial_order_guess(observed_knockdown_mat)


def remove_old_output(out_dir="output") -> None:
    """main.py:26-36: delete the previous run's files, create the directory."""
    for name in OUTPUT_FILES:
        path = os.path.join(out_dir, name)
        if os.path.exists(path):
            os.remove(path)
    os.makedirs(out_dir, exist_ok=True)


def output_handling(best_dag, network_path=None, out_dir="output") -> dict:
    """main.py:44-53: DOT of the transitive closure (``utils.ancestor``) and of
    the transitive reduction of ``best_dag``; the network's real PDFs are
    copied next to them when present.  Returns the written paths."""
    remove_old_output(out_dir)
    best_nem = utils.ancestor(best_dag)
    paths = {"infer_closed": os.path.join(out_dir, "infer_closed.dot"),
             "infer_red": os.path.join(out_dir, "infer_red.dot")}
    dot.generate_dot_from_matrix(best_nem, paths["infer_closed"])
    best_red = utils.transitive_reduction(best_dag)
    dot.generate_dot_from_matrix(best_red, paths["infer_red"])
    if network_path is not None:
        for src, name in ((network_path + ".pdf", "real_closed.pdf"), (network_path + "_red.pdf", "real_red.pdf")):
            if os.path.exists(src):
                shutil.copy(src, os.path.join(out_dir, name))
    return paths


def run_network(csv_path, method="inverse", n_iterations=500, swap_prob=0.90, n_exchange=20,
                replica_iters=300, out_dir=None, device=0, engine=None, verbose=False) -> dict:
    """main.py:56-121 for one network CSV.  Returns the best DAG, its score,
    the Hamming distances main() prints and (with ``out_dir``) the DOT
    paths.  The random stream is the global ``random`` one, left where the
    NEM constructor puts it (reseeded 42, then S*E draws), as in main()."""
    from .engine import Engine
    adj_matrix, end_nodes, errors, num_s, num_e = utils.read_csv_to_adj(csv_path)
    my_nem = NEM(adj_matrix, end_nodes, errors, num_s, num_e)
    order = initial_order_guess(my_nem.observed_knockdown_mat)
    gamma = 2.0 * float(my_nem.num_s) / float(my_nem.num_e)
    eng = engine if engine is not None else Engine.for_nem(my_nem, device=device)
    result = {"num_s": num_s, "num_e": num_e, "order0": order, "method": method}
    if method == "inverse":
        from .methods import InverseMethod
        inv = InverseMethod(order, num_s, num_e, my_nem.U,
                            my_nem.get_score_tables(my_nem.observed_knockdown_mat), engine=eng)
        best_dag, score = inv.optimize()
        result["ll_list"] = inv.ll_list
    elif method == "mcmc":
        from .nem_order_mcmc import NEMOrderMCMC
        smp = NEMOrderMCMC(my_nem, order, engine=eng)
        score, best_dag = smp.method(n_iterations=n_iterations, gamma=gamma, swap_prob=swap_prob,
                                     verbose=verbose)
        result.update(best_order=np.asarray(smp.best_order), all_scores=np.array(smp.all_score_list),
                      accepted=np.array(smp.accepted))
    elif method == "replica":
        from .nem_order_mcmc import replica_exchange_method
        score, best = replica_exchange_method(my_nem, n_exchange, replica_iters, order, device=device)
        best_dag = best.best_dag
        result["best_order"] = np.asarray(best.best_order)
    else:
        raise ValueError(f"unknown method {method!r}: inverse, mcmc or replica")
    best_dag = np.asarray(best_dag)
    result.update(score=float(score), best_dag=best_dag,
                  hamming=int(utils.hamming_distance(best_dag, adj_matrix)),
                  hamming_ancestor=int(utils.hamming_distance(utils.ancestor(best_dag), adj_matrix)))
    if verbose:
        print(f"Hamming Distance: {result['hamming']}")
        print(f"Hamming Distance to Ancestor: {result['hamming_ancestor']}")
    if out_dir is not None:
        base = os.path.splitext(csv_path)[0]
        result["paths"] = output_handling(best_dag, base, out_dir)
    return result


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--network", required=True, help="network CSV (DAGs/networks/networkN/networkN.csv)")
    ap.add_argument("--method", default="inverse", choices=["inverse", "mcmc", "replica"])
    ap.add_argument("--iterations", type=int, default=500)
    ap.add_argument("--out", default="output")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    r = run_network(a.network, a.method, n_iterations=a.iterations, out_dir=a.out, device=a.device,
                    verbose=True)
    print(f"Score: {r['score']}")


if __name__ == "__main__":
    main()
