"""Where the sampler's step keeps the reference's bits: one table of limits.

The default step (option ``exact``) computes in the reference's own arithmetic
(DESIGN.md 3.5b): numpy's SVML log / exp, numpy's pairwise sum, scipy's
compact-form L-BFGS-B, and -- when the device makes them -- W~ and ancestor_x
in scipy.linalg.inv's bits.  Each row below is one limit of
that arithmetic on the device, the model's value, and what the sampler does
outside it.  ``Engine.exact_status()`` and ``Engine.exact_limits()`` read the
same rows; INTEGRATION.md prints the table.

Nothing here touches the GPU: the rows are computed from the model's shape,
its table form and the host's BLAS, so the CPU suite walks every limit.
"""
from __future__ import annotations

from dataclasses import dataclass

# the exact local optima's wave plan: one leaf block result per lane, the
# leaves of numpy's pairwise recursion of one buffer of E (csrc/nemo_host.h
# build_pairwise_plan; one plan per numpy buffer of 8192 terms)
MAX_LEAVES = 64
# the device's getrf / getri restatement (csrc/nemo_ancestor.hip)
MAX_S_DEVICE_ANCESTOR = 64
# the fast local optima (option exact 0)
MAX_E_FAST_LOCAL_OPT = 80 * 64


NUMPY_BUFSIZE = 8192      # np.getbufsize(): np.sum adds buffer-sized chunks in order
MAX_PARTS = 64            # csrc/nemo_internal.h kExactMaxParts


def pairwise_parts(E: int):
    """The wave plans the exact local optima sum E terms in, as numpy's np.sum
    does (csrc/nemo_host.h build_pairwise_parts): one per numpy buffer of
    8192 terms, each summed pairwise, the chunks added in order; None past
    MAX_PARTS buffers."""
    if E < 1:
        return None
    parts = [min(NUMPY_BUFSIZE, E - k) for k in range(0, E, NUMPY_BUFSIZE)]
    return parts if len(parts) <= MAX_PARTS else None


def pairwise_leaves(E: int) -> int:
    """Leaf blocks of numpy's pairwise sum of E terms (pairwise_sum in
    numpy/_core/src/umath/loops_utils.h: n <= 128 sums directly, else n / 2
    rounded down to a multiple of 8 and the rest)."""
    if E < 1:
        return 0
    stack, leaves = [E], 0
    while stack:
        n = stack.pop()
        if n <= 128:
            leaves += 1
            continue
        n2 = n // 2
        n2 -= n2 % 8
        stack += [n2, n - n2]
    return leaves


@dataclass(frozen=True)
class Limit:
    name: str          # what is limited
    bound: str         # the limit
    value: str         # this model's value
    covered: bool      # within the limit
    outside: str       # what the sampler does outside it
    bits: bool         # True: outside it the step still gives the reference's bits


def exact_limits(S: int, E: int, factored: bool, cap: int = 0, host_blas: str | None = "SkylakeX",
                 exact_option: bool = True) -> list[Limit]:
    """The exact path's limits for a model of S S-genes and E effects."""
    leaves = pairwise_leaves(E)
    parts = pairwise_parts(E)
    rows = [
        Limit("option exact", "1 (default)", "1" if exact_option else "0", bool(exact_option),
              "the fast kernels: scores within ~1e-9, a local optimum may take another line-search path",
              False),
        Limit("table form", "factored: every off-diagonal row T[.][j] shared by all children, two-valued "
              "(every table nem.py builds)", "factored" if factored else "generic", bool(factored),
              "ExactArithmeticWarning (strict=True: RuntimeError); the fast kernels", False),
        Limit("E (effects)", f"np.sum of E terms in <= {MAX_PARTS} numpy buffers of {NUMPY_BUFSIZE} (E <= "
              f"{MAX_PARTS * NUMPY_BUFSIZE}; each buffer summed pairwise in <= {MAX_LEAVES} leaf blocks, the "
              "buffers in order) -- with numpy's default np.getbufsize()",
              f"E={E}: {leaves} leaves" + (f", {len(parts)} buffers" if parts and len(parts) > 1 else ""),
              parts is not None,
              "ExactArithmeticWarning (strict=True: RuntimeError); the fast kernels"
              + ("" if E <= MAX_E_FAST_LOCAL_OPT else f" -- which take E <= {MAX_E_FAST_LOCAL_OPT}: the step fails"),
              False),
        Limit("parent cap", "any (0 = the reference; 1..S-1 the build-defined C5 extension)", f"cap={cap}", True,
              "-", True),
        Limit("S (S-genes), ancestor_x on the device",
              f"S <= {MAX_S_DEVICE_ANCESTOR} and scipy's OpenBLAS running its SkylakeX kernels on this host",
              f"S={S}, host BLAS {host_blas or 'unknown'}",
              S <= MAX_S_DEVICE_ANCESTOR and host_blas in ("SkylakeX", None),
              "W~ and ancestor_x made on the host by scipy itself (chain batches: InvPool workers); the "
              "reference's bits", True),
    ]
    return rows


def exact_status_from(rows: list[Limit]) -> tuple[bool, str]:
    """(True, "") when the step keeps the reference's bits, else (False, the
    first limit that breaks it and what happens instead)."""
    for r in rows:
        if not r.covered and not r.bits:
            return False, f"{r.name}: {r.value} is outside {r.bound}; {r.outside}"
    return True, ""


def limits_table_markdown(rows: list[Limit]) -> str:
    out = ["| limit | bound | this model | covered | outside it |", "|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| {r.name} | {r.bound} | {r.value} | {'yes' if r.covered else 'no'} | {r.outside} |")
    return "\n".join(out)
