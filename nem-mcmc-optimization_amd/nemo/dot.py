"""DOT output of DAGs (reference DAGs/dot.py).

Pure host text I/O around the hot path: the reference writes the bundled
networks' ``.dot`` files from their CSVs (``generate_dot_language``) and the
inferred DAGs of a run from adjacency matrices (``generate_dot_from_matrix``,
called by main.py:44-53).  Same names, arguments, output bytes and console
lines as the reference.

One deliberate difference: the reference's ``generate_dot_from_matrix``
changes the process's working directory to ``'../'`` before writing
(DAGs/dot.py:39), so a relative ``output_file`` lands one level up and every
later relative path of the caller shifts.  Here the file is written where
``output_file`` points and the working directory is left alone.
"""
from __future__ import annotations

import csv

import numpy as np


def _dot_text(edges) -> str:
    """``digraph {`` + one ``    a -> b;`` line per edge + ``}`` (no newline
    after the brace), the layout of DAGs/dot.py:15-21 and :30-36."""
    return "digraph {\n" + "".join(f"    {a} -> {b};\n" for a, b in edges) + "}"


def generate_dot_language(csv_file_path, output_file_path) -> None:
    """DOT of a network CSV's edges, in file order.  Reference: DAGs/dot.py:4-26
    (the header line and the last two lines -- end nodes and errors -- are
    dropped; every other row is an edge)."""
    with open(csv_file_path, "r") as f:
        print(f"Reading {csv_file_path}")
        rows = list(csv.reader(f))
    rows = rows[1:-2]
    with open(output_file_path, "w") as fh:
        fh.write(_dot_text((r[0], r[1]) for r in rows))
    print(f"Generated {output_file_path}")


def generate_dot_from_matrix(adj_matrix, output_file) -> None:
    """DOT of every non-zero entry (i, j) of ``adj_matrix`` as ``i -> j``, row
    major.  Reference: DAGs/dot.py:28-42 (see the module note on its
    ``os.chdir``)."""
    adj = np.asarray(adj_matrix)
    n = len(adj)
    edges = [(i, j) for i in range(n) for j in range(n) if adj[i][j] != 0]
    with open(output_file, "w") as fh:
        fh.write(_dot_text(edges))
    print(f"Generated {output_file}")


__all__ = ["generate_dot_language", "generate_dot_from_matrix"]
