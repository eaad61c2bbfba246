"""Benchmark: order-score evaluations/s on the synthetic 64 S-gene x 2000
effect NEM (BASELINE.json metric, config C3; C4 = the same per GPU at N > 1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--path auto|stream|factored]

A step is one batched pass of the hot path over B = 2048 (pos, W)
evaluations whose inputs are already resident in HBM, enqueued on one HIP
stream through the C-ABI: for the default path (the staged C3 model has the
NEM structure) that is ONE kernel, score_i8l_kernel: per evaluation the
fixed-point digits of Delta in LDS, the int8 MFMA contraction and the fp64
log-sum-exp, with the effect sum finalized in-kernel.
With N > 1 (torchrun, one rank per GPU) every rank evaluates its own B
evaluations (weak scaling, no data-path collective); the only collective is
one RCCL all-gather of per-chain best scores at the end of the timed region
(C4).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "nem-mcmc-optimization_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
F64_MFMA_PEAK_TF = 78.6  # v_mfma_f64_16x16x4_f64: 2048 FLOP / 64 busy cycles / SIMD (PMC-checked)
I8_MFMA_PEAK_TOPS = 5000.0  # dense int8 MFMA (MI355X_MICROARCH.md: 2x the ~2.5 PF BF16 rate)
# VALU issue: 256 CUs x 4 SIMDs, one VALU instruction in flight per SIMD per
# cycle at the 2.4 GHz max clock (MI355X_MICROARCH.md chip table); PMC
# SQ_ACTIVE_INST_VALU counts the busy cycles in quad-cycles
N_SIMD = 1024
CLOCK_MAX_GHZ = 2.4
L2_PEAK_GBS = 34500.0   # aggregate L2 read rate over the 8 XCDs (MI355X_MICROARCH.md L2)
LDS_PEAK_TBS = 150.0   # ds_read_b64/b128, every CU streaming (MI355X_MICROARCH.md LDS)
PATHS = {"auto": 0, "stream": 1, "factored": 2}


def n_pairs(S, cap):
    return sum(min(q, cap) if cap else q for q in range(S))


def algorithmic_bytes_per_eval(S, E, cap, b):
    """P*E*b (table rows) + (S+1)*E*b (U) + S^2*b (W) + 4S (pos) + b (ll)."""
    return n_pairs(S, cap) * E * b + (S + 1) * E * b + S * S * b + 4 * S + b


def factored_bytes_per_launch(S, E, B):
    """Algorithmic HBM bytes of one launch of the factored kernels (DESIGN.md
    3.1, 5): what they must read and write at least -- per evaluation its
    weights (S^2 f64), order (S int32) and ll (f64), and once per launch the
    model: U ((S+1) x E f64) and the D1 bit rows (S x ceil(E/64) u64).  They
    never read the S x S x E table T, so SURVEY.md 8(d)'s T-streaming bytes
    do not describe them (that model prices the streaming kernel)."""
    return B * (S * S * 8 + 4 * S + 8) + (S + 1) * E * 8 + S * ((E + 63) // 64) * 8


def algorithmic_flops_per_eval(S, E, cap):
    """Factored form: cell = U + G + Delta.D1 over the permissible (i, j):
    2 FLOP per (pair, effect)."""
    return 2 * n_pairs(S, cap) * E


def host_cpu():
    """The host CPU's model name (/proc/cpuinfo): the same oracle loop runs
    ~2x faster on the GPU box's host than in the build container (SURVEY.md
    6 was measured there), so every CPU figure names its CPU."""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(m, seconds=10.0, config="C3"):
    """The oracle (numpy restatement of the reference's compute_cell_ratios +
    calculate_ll, nem_order_mcmc.py:79-93, same operation order) timed on
    this host, one thread."""
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import nemo_oracle as no
    from scipy.special import expit
    t = m.get_score_tensor()
    rng = np.random.default_rng(77)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        perm = rng.permutation(m.num_s)
        w01 = expit(rng.uniform(-3, 3, (m.num_s, m.num_s)))
        no.order_score(m.U, t, perm, w01)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "evals/s", "cores": 1, "kind": "port",
            "sample": f"{n} order-score evals of the {m.num_s}x{m.num_e} {config} model in {dt:.1f} s: oracle numpy "
                      "loop form (reference operation order), one thread, this host"}


_CPU_CHILD = r"""
import sys, time
import numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import nemo_oracle as no
from scipy.special import expit
from nemo import generator
m = generator.config_nem(sys.argv[3]); t = m.get_score_tensor()
rng = np.random.default_rng(int(sys.argv[5]))
sys.stdout.write("ready\n"); sys.stdout.flush()
sys.stdin.readline()
n, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < float(sys.argv[4]):
    no.order_score(m.U, t, rng.permutation(m.num_s), expit(rng.uniform(-3, 3, (m.num_s, m.num_s))))
    n += 1
print(n, time.perf_counter() - t0)
"""


def cpu_baseline_procs(config, nproc=8, seconds=10.0):
    """the same oracle loop in nproc independent processes
    (one thread each, independent chains), started together; the rate is the
    sum of the processes' own rates.  Children are plain subprocesses that
    never touch the GPU."""
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    args = [os.path.join(HERE, "oracle"), os.path.join(HERE, "nem-mcmc-optimization_amd"), config, str(seconds)]
    procs = [subprocess.Popen([sys.executable, "-c", _CPU_CHILD] + args + [str(100 + k)], stdin=subprocess.PIPE,
                              stdout=subprocess.PIPE, text=True, env=env) for k in range(nproc)]
    try:
        for p in procs:  # every child has built its model before any starts timing
            if p.stdout.readline().strip() != "ready":
                raise RuntimeError("cpu baseline child failed to start")
        for p in procs:
            p.stdin.write("go\n")
            p.stdin.flush()
        res = [p.communicate(timeout=seconds + 120)[0].split() for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    rates = [int(n) / float(dt) for n, dt in res]
    n = sum(int(r[0]) for r in res)
    return {"value": sum(rates), "unit": "evals/s", "cores": nproc, "kind": "port",
            "sample": f"{n} order-score evals of the {config} model by {nproc} independent one-thread "
                      f"processes in ~{seconds:.0f} s each: oracle numpy loop form (reference operation "
                      "order), this host"}


def load_record(name, key, build_id):
    """A PMC record (profiles/valu.json: VALU / MFMA / LDS busy;
    profiles/traffic.json: HBM bytes per launch) of the score kernel --
    only if it was measured on THIS build of libnemo.so (its build id: a hash
    of the sources and flags, nemo_build_id()); a record of another build is
    stale and dropped."""
    p = os.path.join(HERE, "profiles", name)
    if not os.path.exists(p):
        return None
    with open(p) as fh:
        rec = json.load(fh).get(key)
    if not rec:
        return None
    if rec.get("build_id") == build_id:
        return dict(rec, matched_by="build_id")
    # a record of another build still holds when the kernel's own translation
    # unit is unchanged (its code id) and the loaded library is the one this
    # tree builds (so that unit's machine code is the one measured)
    from nemo import build as nb
    tu = nb.KERNEL_TU.get(key.split(":")[1])
    if tu and rec.get("code_id") and rec["code_id"] == nb.code_id(tu) and build_id == nb.build_id():
        return dict(rec, matched_by="code_id")
    return None


def stream_roofline(B, bpe, kern_ms, tr):
    """Roofline of the generic streaming kernel (score_kernel): every
    algorithmic byte (the masked exp(T) rows, U, W, pos)
    is a vector load served by the L2 (or the L1 above it), so the bound is
    the chip's L2 read rate (MI355X_MICROARCH.md: ~34.5 TB/s over the 8
    XCDs).  The 65.5 MB table at C3 stays in the Infinity Cache and the batch
    re-reads each row from the L2, so HBM carries far fewer bytes: those come
    from the PMC record of this kernel's code (FETCH_SIZE x2 + WRITE_SIZE) as a
    fraction of the 8 TB/s HBM peak."""
    ach = B * bpe / (kern_ms / 1e3) / 1e9
    roof = {"bound": "l2", "achieved": ach, "peak": L2_PEAK_GBS, "unit": "GB/s", "frac": ach / L2_PEAK_GBS,
            "bytes_per_eval": bpe, "evals_per_launch": B,
            "traffic": tr["bytes_per_launch"] if tr else None,
            "note": ("algorithmic bytes (every vector load) against the aggregate L2 read rate; the "
                     "exp(T) table is Infinity-Cache resident at C3 and re-read across the batch, so "
                     "HBM bytes (traffic, PMC) are a fraction of them")}
    if tr:
        hbm = tr["bytes_per_launch"] / (kern_ms / 1e3) / 1e9
        roof["secondary"] = {"hbm": {"achieved": hbm, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": hbm / HBM_PEAK_GBS}}
    return roof


def timed_steps(eng, torch, B, cap, steps, warmup, d_pos, d_w01, d_ll, stream, world, dist,
                warmup_s=0.0, collective=None):
    """``collective``: run the barriers and the best-score all-gather on the
    default process group (default: world > 1; rank-0-only extras pass
    world = 1 and run none)."""
    coll = world > 1 if collective is None else collective
    def step():
        eng.score_dev(B, d_pos.data_ptr(), d_w01.data_ptr(), d_ll.data_ptr(), cap=cap, stream=stream)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    # the engine clock ramps up over the first tens of ms of load (a 20-step
    # run measures ~10% slower per launch than a 200-step one): untimed steps
    # until warmup_s of load have passed, so the K timed steps see the
    # sustained clock whatever W is
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warmup_s:
        for _ in range(10):
            step()
        torch.cuda.synchronize()
    if coll:
        dist.barrier()
    torch.cuda.synchronize()
    # kernel time = HIP events recorded on the launch stream around the K
    # back-to-back launches, divided by K (an upper bound on the kernel's own
    # duration: it includes any gap between launches).  The library's
    # per-launch events would add ~6 us of stream work per step inside the
    # timed region, so they run after it, on 20 more launches, as a cross-check
    ts = torch.cuda.current_stream()  # the stream every kernel is launched on
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(ts)
    for _ in range(steps):
        step()
    ev1.record(ts)
    if coll:
        # C4: gather every rank's per-chain best score (tiny, latency-bound)
        best = d_ll.max().reshape(1)
        if dist.get_backend() != "nccl":
            best = best.cpu()
        allb = [torch.empty_like(best) for _ in range(dist.get_world_size())]
        dist.all_gather(allb, best)
    torch.cuda.synchronize()
    if coll:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / steps
    eng.timing(True)
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    lt_ms, launches = eng.timing_read()
    eng.timing(False)
    return wall, kern_ms, lt_ms / max(launches, 1)


def c5_capped(torch, dist, stream, batch=2048, steps=10, warmup_s=0.3):
    """BASELINE config C5 (S=128, E=5000, parent cap 6): evals/s of the capped
    lookup-table kernel (fact_kernel 9, what auto takes for capped calls), of
    its round-1 form (fact_kernel 15) and of the fp64 MFMA factored kernel
    (fact_kernel 1) on the same resident inputs; kernel time per launch from
    the library's HIP events."""
    from scipy.special import expit

    from nemo import generator
    from nemo.engine import Engine
    S, E, _seed, cap, dtype = generator.CONFIGS["C5"]
    eng = Engine.for_nem(generator.config_nem("C5"), dtype=dtype)
    eng.reserve(batch)
    rng = np.random.default_rng(78)
    d_pos = torch.from_numpy(np.array([rng.permutation(S) for _ in range(batch)], dtype=np.int32)).cuda()
    d_w01 = torch.from_numpy(expit(rng.uniform(-3, 3, (batch, S, S)))).cuda()
    d_ll = torch.zeros(batch, dtype=torch.float64, device="cuda")
    staged = bool(eng.get_option("win"))
    out = {"workload": f"C5: S={S} E={E} cap={cap} {dtype} tables, {batch} evaluations per launch",
           "lookup_table_staged": staged}
    lls = {}
    runs = ((("lookup_table_kernel", 9), ("lookup_table_kernel_r1", 15)) if staged else ()) + \
        (("f64_mfma_factored_kernel", 1),)
    for name, fk in runs:
        eng.set_option("fact_kernel", fk)
        wall, kms, _ = timed_steps(eng, torch, batch, cap, steps, 2, d_pos, d_w01, d_ll, stream, 1, dist,
                                   warmup_s=warmup_s)
        lls[name] = d_ll.cpu().numpy()
        out[name] = {"evals_per_s": batch * steps / wall, "kernel_avg_ms": kms,
                     "cells_per_s": batch * S * E / (kms / 1e3)}
    if staged:
        out["lookup_table_kernel"]["kernel"] = (
            "score_window2_kernel (row bits transposed into registers, 7-bit window per row by one "
            "funnel shift; two table reads + one FMA per cell)")
        out["lookup_table_kernel_r1"]["kernel"] = "score_window_kernel (round 1: row bits re-read from LDS)"
        # the walk reads two f64 table entries per cell from LDS: priced
        # against the chip's ds_read_b64 rate (MI355X_MICROARCH.md, LDS table:
        # 256 B/clk/CU, ~150 TB/s with every CU streaming)
        kms = out["lookup_table_kernel"]["kernel_avg_ms"]
        lds_tbs = batch * S * E * 16 / (kms / 1e3) / 1e12
        out["lookup_table_kernel"]["roofline"] = {
            "bound": "lds", "achieved": lds_tbs, "peak": 150.0, "unit": "TB/s", "frac": lds_tbs / 150.0,
            "bytes_per_eval": S * E * 16, "note": "2 x 8 B of LDS reads per cell (S*E cells per evaluation)"}
        out["max_abs_ll_diff"] = float(np.max(np.abs(lls["lookup_table_kernel"] -
                                                     lls["f64_mfma_factored_kernel"])))
        out["max_abs_ll_diff_r1"] = float(np.max(np.abs(lls["lookup_table_kernel"] -
                                                        lls["lookup_table_kernel_r1"])))
    eng.close()
    return out


KERNEL_NAMES = {
    "i8w": "score_i8w_kernel (score_i8l_kernel's arithmetic for 64 < S <= 128: K = 128 as two K = 64 "
           "halves per row block, two tiles per iteration)",
    "i8l": "score_i8l_kernel (x / ln 2 = Delta.D1 + U' + G exact in int8 fixed point on "
           "v_mfma_i32_16x16x64_i8, 7 digit slices; e^x assembled from the integer accumulators + "
           "table + degree-2 series; log-sum-exp offset by the null row; two 16-effect tiles per "
           "iteration share the A fragments)",
    "i8o": "score_i8o_kernel (Delta.D1 + U - U[S] exact in int8 fixed point on v_mfma_i32_16x16x64_i8, "
           "fp64 cells, log-sum-exp offset by the null row)",
    "i8": "score_i8_kernel (Delta.D1 exact in int8 fixed point on v_mfma_i32_16x16x64_i8, fp64 cells + "
          "fused log-sum-exp)",
    "factored": "score_factored_kernel (fp64 MFMA 16x16x4 + fused log-sum-exp)",
    "pipe": "score_factored_pipe_kernel (fp64 MFMA 16x16x4, U as the C-init, fused log-sum-exp)",
    "win2": "score_window2_kernel (capped lookup tables walked from registers)",
    "win": "score_window_kernel (capped lookup tables, round-1 form: row bits re-read from LDS)",
}
ARITH = {
    "i8l": "int8 fixed point 2^-38/ln2 + fp64 LSE",
    "i8w": "int8 fixed point 2^-38/ln2 + fp64 LSE",
    "i8o": "int8 fixed point 2^-44 + fp64 LSE",
    "i8": "int8 fixed point 2^-44 + fp64 LSE",
}


def kernel_tag(fk):
    """profiles/*.json key tag of the kernel fact_kernel ``fk`` launches."""
    if fk in (18, 19):
        return "i8w"
    if fk in (10, 11, 12, 14, 16, 17, 20):
        return "i8l"
    if fk == 13:
        return "i8s"
    if fk in (7, 8):
        return "i8o"
    if fk in (4, 5, 6):
        return "i8"
    if fk == 9:
        return "win2"
    if fk == 15:
        return "win"
    if fk in (2, 3):
        return "pipe"
    return "factored"


def score_roofline(config, S, E, cap, B, fk, kern_ms, launch_ev_ms, bid):
    """The dominant kernel's roofline: the unit that binds it, priced against
    that unit's peak, with the other units beside it as fractions <= 1."""
    tag = kernel_tag(fk)
    kern_s = kern_ms / 1e3
    valu = load_record("valu.json", f"{config}:{tag}:b{B}", bid)
    traffic = load_record("traffic.json", f"{config}:{tag}:b{B}", bid)
    fpe = algorithmic_flops_per_eval(S, E, cap)
    f64eq = B * fpe / kern_s / 1e12
    secondary = {}
    if tag in ("i8l", "i8o", "i8s", "i8w"):
        # the MFMAs the kernel issues: 7 (log2) or 8 v_mfma_i32_16x16x64_i8
        # (2*16*16*64 ops each) per 16-child row block per 16-effect tile
        # (per K = 64 half: two halves for 64 < S <= 128)
        nslice = 7 if tag != "i8o" else 8
        nr = 8 if S > 64 else 4 if S > 32 else 2 if S > 16 else 1
        ops = ((E + 15) // 16) * nr * nslice * (2 if S > 64 else 1) * 32768
        a = B * ops / kern_s / 1e12
        secondary["int8_mfma"] = {"achieved": a, "peak": I8_MFMA_PEAK_TOPS, "unit": "TOPS",
                                  "frac": a / I8_MFMA_PEAK_TOPS, "ops_per_eval": ops}
    fbytes = factored_bytes_per_launch(S, E, B)
    hbm_alg = fbytes / kern_s / 1e9
    secondary["hbm"] = {"algorithmic_bytes_per_launch": fbytes, "achieved": hbm_alg, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": hbm_alg / HBM_PEAK_GBS,
                        "note": "algorithmic bytes of the factored form (weights, orders and lls of the batch + "
                                "U and the D1 bits once; bench.factored_bytes_per_launch) / this run's launch time"}
    if traffic:
        hbm = traffic["bytes_per_launch"] / kern_s / 1e9
        secondary["hbm"].update({"pmc_bytes_per_launch": traffic["bytes_per_launch"], "pmc_achieved": hbm,
                                 "pmc_frac": hbm / HBM_PEAK_GBS,
                                 "pmc_over_algorithmic": traffic["bytes_per_launch"] / fbytes,
                                 "pmc_note": "PMC bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, the kernel's code as built here) / "
                                             "this run's launch time"})
    if valu and "SQ_LDS_IDX_ACTIVE" in valu:
        lds = valu["SQ_LDS_IDX_ACTIVE"] / kern_s / 1e12
        peak = 256 * CLOCK_MAX_GHZ / 1e3
        secondary["lds"] = {"achieved": lds, "peak": peak, "unit": "T LDS-busy CU-cycles/s", "frac": lds / peak,
                            "bank_conflict_share": valu.get("SQ_LDS_BANK_CONFLICT", 0.0) / valu["SQ_LDS_IDX_ACTIVE"]}
    roof = {"kernel": KERNEL_NAMES.get(tag, tag), "fact_kernel": fk, "kernel_avg_ms": kern_ms,
            "kernel_avg_ms_launch_events": launch_ev_ms,
            "traffic": traffic["bytes_per_launch"] if traffic else None,
            "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE of the kernel's code as built "
                            "here)" if traffic else None,
            "evals_per_launch": B}
    if valu and "SQ_ACTIVE_INST_VALU" in valu:
        busy = 4.0 * valu["SQ_ACTIVE_INST_VALU"]        # SIMD-cycles with a VALU instruction issuing
        a = busy / kern_s / 1e12
        peak = N_SIMD * CLOCK_MAX_GHZ / 1e3
        roof.update({"bound": "valu", "achieved": a, "peak": peak, "unit": "T VALU-busy SIMD-cycles/s",
                     "frac": a / peak, "valu_busy_cycles_per_launch": busy,
                     "pmc": {k: valu[k] for k in ("valu_busy", "mfma_busy", "lds_busy", "mfma_coexec_frac",
                                                  "GRBM_GUI_ACTIVE", "SQ_INSTS_VALU", "SQ_INSTS_MFMA") if k in valu}})
        if tag == "i8l":
            # the formulation's own work: the epilogue's 11 VALU per cell, S x E
            # cells per evaluation, one wave instruction per 64 cells at 4 SIMD-cycles each, priced
            # at the same max-clock issue rate; the rest of the 16.6 per 64 cells is 3.1i's table
            alg = 4.0 * 11.0 * S * E / 64.0 * B
            roof["algorithmic_frac"] = alg / kern_s / (N_SIMD * CLOCK_MAX_GHZ * 1e9)
            roof["algorithmic_valu_per_64_cells"] = 11.0
            if "SQ_INSTS_VALU" in valu:
                roof["valu_per_64_cells"] = valu["SQ_INSTS_VALU"] / (B * S * E / 64.0)
        roof["note"] = ("bound = the SIMD's VALU issue (the exp epilogue: S*E cells per evaluation): achieved = "
                        "PMC VALU-busy SIMD-cycles per launch (4 x SQ_ACTIVE_INST_VALU; the record of the kernel's "
                        f"code as built here, matched by its {valu.get('matched_by', 'build_id')}) / this run's "
                        "HIP-event launch time, against 1024 SIMDs x 2.4 GHz (the max clock, so frac <= the PMC "
                        "valu_busy at the clock the chip held); the other units in secondary")
    elif "int8_mfma" in secondary:
        roof.update({"bound": "mfma", **{k: secondary["int8_mfma"][k] for k in ("achieved", "peak", "unit", "frac")},
                     "note": "no PMC record of the kernel's code as built here (profiles/valu.json): the int8 "
                             "matrix-core fraction; "
                             "the VALU issue binds in every profiled build (DESIGN.md 3.1e)"})
    else:
        roof.update({"bound": "mfma", "achieved": f64eq, "peak": F64_MFMA_PEAK_TF, "unit": "TFLOP/s",
                     "frac": f64eq / F64_MFMA_PEAK_TF, "note": "fp64 MFMA contraction 2*P*E FLOP per evaluation"})
    roof["secondary"] = secondary
    if tag in ("i8l", "i8o", "i8s", "i8", "i8w"):
        roof["fp64_equivalent"] = {
            "achieved": f64eq, "unit": "TFLOP/s", "flops_per_eval": fpe, "vs_f64_mfma_peak": f64eq / F64_MFMA_PEAK_TF,
            "note": "the contraction Delta.D1 priced as fp64 work (2*P*E FLOP/eval) against the fp64 MFMA peak: "
                    "how far the int8 fixed-point reformulation is past an fp64 matrix-core roofline; not a "
                    "hardware fraction"}
    return roof


# The exact local optima's kernel (local_opt_exact_kernel, nemo_exact.hip): where the sampler's
# step spends its time.  Priced on the SIMDs' VALU issue: its unit of work is one
# f-evaluation of the reference's objective (nem_order_mcmc.py:18-23), E terms log(c e + 1)
# summed, at LOG_VALU wave instructions per 64 terms -- svml_log as restated (refmath.h: 14 for
# the reduction and the table row, 16 for the polynomial and the reconstruction) plus the product,
# the + 1 and the sum's add -- each 4 SIMD cycles.  The f-evaluations of a launch
# are the optima's nfev (the info array); the kernel's time from HIP events around its launch
# (option timing_kernel 1).  The control of L-BFGS-B and the tree of the pairwise sum are not
# priced: the fraction says how far the launch is from the objective's own VALU work.
LOG_VALU = 33
SIMD_CYCLES_PER_S = 1024 * 2.4e9


def local_opt_roofline(eng, S, E, cap, chains, reps=5):
    from scipy.special import expit

    from nemo.nem_order_mcmc import SIG0, SIG1
    rng = np.random.default_rng(11 + chains)
    pos = np.array([rng.permutation(S) for _ in range(chains)], dtype=np.int32)
    w = rng.uniform(-3, 3, (chains, S, S))
    w01 = expit(w)
    anc = np.clip(rng.random((chains, S, S)) - 0.5, 0, 1)
    eng.optimal_weights(pos, w01, anc, w, SIG0, SIG1, cap=cap, raise_on_fail=False)
    eng.set_option("timing_kernel", 1)
    eng.timing(True)
    try:
        for _ in range(reps):
            _, _, _, info = eng.optimal_weights(pos, w01, anc, w, SIG0, SIG1, cap=cap, raise_on_fail=False)
        ms, n = eng.timing_read()
    finally:
        eng.timing(False)
        eng.set_option("timing_kernel", 0)
    kern_ms = ms / max(n, 1)
    inf = info[info != -1]
    nfev = int(((inf >> 16) & 0x7fff).sum())
    work = nfev * E * LOG_VALU / 64.0 * 4.0          # VALU-busy SIMD cycles of the objective
    achieved = work / (kern_ms * 1e-3) / 1e12
    peak = SIMD_CYCLES_PER_S / 1e12
    return {"chains": chains, "optima": int(inf.size), "f_evaluations": nfev, "kernel_avg_ms": kern_ms,
            "launches_timed": n, "exact_form": eng.get_option("exact_form"),
            "roofline": {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "T VALU-busy SIMD-cycles/s",
                         "frac": achieved / peak, "traffic": None,
                         "work": f"f-evaluations x E x {LOG_VALU} VALU / 64 lanes x 4 cycles"}}


def c3_fp64(eng, torch, dist, B, cap, d_pos, d_w01, stream, S, E, ll_ref, steps=10, warmup_s=0.3):
    """The headline workload (same model, same resident inputs, same B) in
    fp64 arithmetic: the fp64 MFMA factored kernels (fact_kernel 2: pipelined,
    U as the C-init; 1: chunked), priced against the fp64 matrix-core peak
    (2*P*E FLOP of the contraction per evaluation), next to the fixed-point
    headline kernel's lls."""
    fk0 = eng.get_option("fact_kernel")
    d_ll = torch.zeros(B, dtype=torch.float64, device="cuda")
    out = {"workload": f"C3: S={S} E={E}, {B} evaluations per launch, fp64 arithmetic throughout"}
    try:
        for name, fk in (("f64_mfma_pipelined_kernel", 2), ("f64_mfma_chunked_kernel", 1)):
            eng.set_option("fact_kernel", fk)
            wall, kms, _ = timed_steps(eng, torch, B, cap, steps, 2, d_pos, d_w01, d_ll, stream, 1, dist,
                                       warmup_s=warmup_s)
            fl = B * algorithmic_flops_per_eval(S, E, cap) / (kms / 1e3) / 1e12
            out[name] = {"fact_kernel": fk, "evals_per_s": B * steps / wall, "kernel_avg_ms": kms,
                         "roofline": {"bound": "mfma", "achieved": fl, "peak": F64_MFMA_PEAK_TF, "unit": "TFLOP/s",
                                      "frac": fl / F64_MFMA_PEAK_TF,
                                      "flops_per_eval": algorithmic_flops_per_eval(S, E, cap)},
                         "max_abs_ll_diff_vs_headline": float(np.max(np.abs(d_ll.cpu().numpy() - ll_ref)))}
    finally:
        eng.set_option("fact_kernel", fk0)
    best = max((k for k in out if k.endswith("_kernel")), key=lambda k: out[k]["evals_per_s"])
    out["best"] = best
    out["evals_per_s"] = out[best]["evals_per_s"]
    return out


def c3_exact(eng, torch, dist, B, cap, d_pos, d_w01, stream, S, E, pos, w01, ll_ref, steps=5, warmup_s=0.3):
    """The headline workload (same model, same resident inputs, same B) in
    the reference's own arithmetic (option exact_dev: numpy's SVML log / exp,
    glibc's exp / log1p in logaddexp.reduce, Python's left fold; the
    nemo_exact.hip kernels), with its first evaluations checked bit for bit
    against the host-pointer exact path."""
    d_ll = torch.zeros(B, dtype=torch.float64, device="cuda")
    eng.set_option("exact_dev", 1)
    try:
        wall, kms, _ = timed_steps(eng, torch, B, cap, steps, 1, d_pos, d_w01, d_ll, stream, 1, dist,
                                   warmup_s=warmup_s)
    finally:
        eng.set_option("exact_dev", 0)
    got = d_ll.cpu().numpy()
    nchk = min(B, 8)
    host = eng.score(pos[:nchk], w01[:nchk], cap=cap)
    return {"workload": f"C3: S={S} E={E}, {B} evaluations per launch, the reference's arithmetic (bits of "
                        "numpy's calculate_ll)",
            "kernels": "exact_cells_kernel, exact_fold_kernel, exact_seq_sum_kernel (nemo_exact.hip)",
            "evals_per_s": B * steps / wall, "kernel_avg_ms": kms,
            "bits_equal_host_exact_first": int(nchk) if np.array_equal(got[:nchk].view(np.uint64),
                                                                       host.view(np.uint64)) else 0,
            "max_abs_ll_diff_vs_headline": float(np.max(np.abs(got - ll_ref)))}


def wide_uncapped(torch, dist, stream, batch=2048, steps=5, warmup_s=0.3):
    """Uncapped 64 < S <= 128 (generator config W128: 128 x 2000): the int8
    log2 kernel for wide models (fact_kernel 18, what auto takes within the
    error budget) next to the fp64 MFMA kernel it replaces (fact_kernel 1),
    on the same resident inputs; kernel time per launch from HIP events."""
    from scipy.special import expit

    from nemo import generator
    from nemo.engine import Engine
    S, E, _seed, cap, dtype = generator.CONFIGS["W128"]
    eng = Engine.for_nem(generator.config_nem("W128"), dtype=dtype)
    eng.reserve(batch)
    rng = np.random.default_rng(79)
    d_pos = torch.from_numpy(np.array([rng.permutation(S) for _ in range(batch)], dtype=np.int32)).cuda()
    d_w01 = torch.from_numpy(expit(rng.uniform(-3, 3, (batch, S, S)))).cuda()
    d_ll = torch.zeros(batch, dtype=torch.float64, device="cuda")
    fk_auto, bound = eng.score_kernel(0)
    out = {"workload": f"W128: S={S} E={E} uncapped {dtype}, {batch} evaluations per launch",
           "auto_fact_kernel": fk_auto, "ll_error_bound": bound}
    lls = {}
    for name, fk in (("int8_log2_wide_kernel", 18), ("f64_mfma_factored_kernel", 1)):
        eng.set_option("fact_kernel", fk)
        wall, kms, _ = timed_steps(eng, torch, batch, cap, steps, 1, d_pos, d_w01, d_ll, stream, 1, dist,
                                   warmup_s=warmup_s)
        lls[name] = d_ll.cpu().numpy()
        out[name] = {"evals_per_s": batch * steps / wall, "kernel_avg_ms": kms,
                     "cells_per_s": batch * S * E / (kms / 1e3)}
    out["int8_log2_wide_kernel"]["kernel"] = ("score_i8w_kernel (score_i8l_kernel's arithmetic over K = 128 as "
                                              "two K = 64 halves; two tiles per iteration)")
    out["speedup_vs_f64"] = (out["f64_mfma_factored_kernel"]["kernel_avg_ms"] /
                             out["int8_log2_wide_kernel"]["kernel_avg_ms"])
    out["max_abs_ll_diff"] = float(np.max(np.abs(lls["int8_log2_wide_kernel"] - lls["f64_mfma_factored_kernel"])))
    eng.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--warmup-seconds", type=float, default=0.5,
                    help="untimed load after the W warmup steps (clock ramp); 0: W steps only")
    ap.add_argument("--batch", type=int, default=int(os.environ.get("NEMO_BENCH_BATCH", 2048)))
    ap.add_argument("--path", default=os.environ.get("NEMO_BENCH_PATH", "auto"), choices=list(PATHS))
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the stream-kernel, MCMC and C4 lines")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=8,
                    help="processes of the multi-process CPU baseline (1: off)")
    ap.add_argument("--c4-chains", type=int, default=128, help="C4: chains over all ranks (0: off)")
    ap.add_argument("--c4-steps", type=int, default=30, help="C4: timed MCMC steps (after 2 untimed ones)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # NEMO_BENCH_BACKEND=gloo rehearses the N > 1 path with several ranks on
    # one GPU (device = local rank modulo the visible GPUs); the driver's
    # multi-GPU runs use RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("NEMO_BENCH_BACKEND", "nccl")
    local = local % max(torch.cuda.device_count(), 1) if backend != "nccl" else local
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from scipy.special import expit

    from nemo import _lib, generator
    from nemo.engine import Engine

    bid = _lib.build_id()
    S, E, seed, cap, dtype = generator.CONFIGS[args.config]
    m = generator.config_nem(args.config)
    eng = Engine.for_nem(m, device=local, dtype=dtype)
    eng.set_option("score_path", PATHS[args.path])
    factored = eng.factored and args.path != "stream"
    fk, err_bound = eng.score_kernel(cap) if factored else (-1, 0.0)
    B = args.batch
    eng.reserve(B)
    rng = np.random.default_rng(1000 + rank)
    pos = np.array([rng.permutation(S) for _ in range(B)], dtype=np.int32)
    w01 = expit(rng.uniform(-3, 3, (B, S, S)))
    d_pos = torch.from_numpy(pos).cuda()
    d_w01 = torch.from_numpy(w01).cuda()
    d_ll = torch.zeros(B, dtype=torch.float64, device="cuda")
    side = torch.cuda.Stream()          # the stream every kernel is launched on
    torch.cuda.set_stream(side)
    stream = side.cuda_stream

    wall, kern_ms, launch_ev_ms = timed_steps(eng, torch, B, cap, args.steps, args.warmup, d_pos, d_w01,
                                              d_ll, stream, world, dist, warmup_s=args.warmup_seconds)
    t_max = torch.tensor([wall], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    t_max = float(t_max.item())
    ll = d_ll.cpu().numpy()

    extras = {}
    if not args.no_extras and args.c4_chains > 0 and args.config == "C3":
        # BASELINE C4 on every rank: the chains sharded over the ranks, one
        # ChainBatch per rank, one all-gather of (best score, best order) --
        # over RCCL with device tensors at N > 1 on GPUs
        from nemo.chains import run_c4
        dev = torch.device("cuda", local) if backend == "nccl" and world > 1 else None
        r = run_c4(m, eng, n_chains=args.c4_chains, steps=args.c4_steps, device=dev, repeats=3)
        extras["c4_chains"] = {
            **{k: v for k, v in r.items() if k not in ("scores", "orders")},
            "workload": f"C4: {args.c4_chains} chains of the C3 model sharded over {world} rank(s), "
                        f"{args.c4_steps} MCMC steps (reference method() loop per chain, one fused device "
                        "step per MCMC step per rank), one all-gather of (best score, best order)",
            "collective": (f"all_gather over {'RCCL' if backend == 'nccl' else backend}"
                           if world > 1 else None),
            "accepted": None,
            "reference_cpu_s_per_chain_step": 1.2}

    if rank == 0 and not args.no_extras:
        # the generic streaming kernel on the same model (HBM-priced roofline)
        eng.set_option("score_path", 1)
        Bs = min(B, 128)
        w_s, k_s, _ = timed_steps(eng, torch, Bs, cap, 10, 2, d_pos, d_w01, d_ll, stream, 1, dist,
                                  warmup_s=min(args.warmup_seconds, 0.3))
        bpe = algorithmic_bytes_per_eval(S, E, cap, 8 if dtype == "f64" else 4)
        tr = load_record("traffic.json", f"{args.config}:stream:b{Bs}", bid)
        extras["stream_kernel"] = {
            "evals_per_s": Bs * 10 / w_s, "batch": Bs, "kernel_avg_ms": k_s,
            "roofline": stream_roofline(Bs, bpe, k_s, tr)}
        eng.set_option("score_path", PATHS[args.path])
        if factored and args.config in ("C3", "C2"):
            # the same workload in fp64 arithmetic (the headline's dtype is fixed point)
            extras["c3_fp64"] = c3_fp64(eng, torch, dist, B, cap, d_pos, d_w01, stream, S, E, ll,
                                        warmup_s=min(args.warmup_seconds, 0.3))
            if eng.get_option("exact_ok"):
                extras["c3_exact"] = c3_exact(eng, torch, dist, B, cap, d_pos, d_w01, stream, S, E, pos, w01, ll,
                                              warmup_s=min(args.warmup_seconds, 0.3))
        # fused per-step scorer of the sampler: 16 chains (C4 share of one GPU)
        from nemo.nem_order_mcmc import SIG0, SIG1
        nch = 16
        pos_h = pos[:nch]
        w_h = rng.uniform(-3, 3, (nch, S, S))
        anc = np.clip(rng.random((nch, S, S)) - 0.5, 0, 1)
        def fused_ms(nc, reps, given_anc=False):
            """one nemo_optimal_weights_w call (W in: W~ and ancestor_x made on
            the device), or with given_anc the host's W~ / ancestor_x handed in"""
            def call():
                if given_anc:
                    eng.optimal_weights(pos_h[:nc], expit(w_h[:nc]), anc[:nc], w_h[:nc], SIG0, SIG1, cap=cap,
                                        raise_on_fail=False)
                else:   # as the chain batch calls it: W~ / ancestor_x stay on the device
                    eng.optimal_weights_w(pos_h[:nc], w_h[:nc], SIG0, SIG1, cap=cap, raise_on_fail=False,
                                          want_prep=False)
            call()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                call()
                ts.append(time.perf_counter() - t0)
            return float(np.median(ts))

        # the default step computes in the reference's own arithmetic ("exact":
        # the same bits as numpy / scipy); the fast kernels
        # beside it (scores within ~1e-9, a few optima per C3 step on another
        # line-search path)
        exact_on = bool(eng.get_option("exact")) and bool(eng.get_option("exact_ok"))
        fs = fused_ms(nch, 5)
        fs_given = fused_ms(nch, 5, given_anc=True)
        eng.set_option("exact", 0)
        fs_fast = fused_ms(nch, 5)
        fs1_fast = fused_ms(1, 20)
        eng.set_option("exact", 1)
        if exact_on:
            extras["local_opt"] = {
                "kernel": "local_opt_exact_kernel (scipy's L-BFGS-B per (chain, parent pair), the reference's bits)",
                "c16": local_opt_roofline(eng, S, E, cap, nch),
                "c128": local_opt_roofline(eng, S, E, cap, 128, reps=3)}
        extras["mcmc_fused_step"] = {
            "chains": nch, "ms_per_step": 1e3 * fs, "chain_steps_per_s": nch / fs,
            "arithmetic": "exact (the reference's bits)" if exact_on else "fast",
            "fast_kernels_ms_per_step": 1e3 * fs_fast,
            "ms_per_step_given_ancestor": 1e3 * fs_given,
            "includes": "nemo_optimal_weights_w: H2D of pos/W, W~ and ancestor_x (getrf/getri in scipy's bits) "
                        "on the device, eval#1 with order weights, 2016 L-BFGS-B local optima per chain, eval#2 "
                        "on binarised weights, D2H (ms_per_step_given_ancestor: the host's W~ / ancestor_x "
                        "handed in instead)"}
        # BASELINE C3 names ONE chain: what one chain sees per call -- a
        # synchronous host-pointer order score (B = 1: the calculate_ll path of
        # one sampler, H2D + kernel + D2H) and the fused step of one chain
        lat = []
        for _ in range(50):
            t0 = time.perf_counter()
            eng.score(pos[:1], w01[:1], cap=cap)
            lat.append(time.perf_counter() - t0)
        eng.set_option("exact", 0)
        lat_fast = []
        for _ in range(50):
            t0 = time.perf_counter()
            eng.score(pos[:1], w01[:1], cap=cap)
            lat_fast.append(time.perf_counter() - t0)
        eng.set_option("exact", 1)
        ts1 = []
        for _ in range(20):
            t0 = time.perf_counter()
            eng.optimal_weights_w(pos_h[:1], w_h[:1], SIG0, SIG1, cap=cap, raise_on_fail=False)   # as the sampler
            ts1.append(time.perf_counter() - t0)
        extras["single_chain"] = {
            "score_call_us": 1e6 * float(np.median(lat)), "evals_per_s_sequential": 1.0 / float(np.median(lat)),
            "fused_step_ms": 1e3 * float(np.median(ts1)), "chain_steps_per_s": 1.0 / float(np.median(ts1)),
            "fused_step_ms_fast_kernels": 1e3 * fs1_fast,
            "score_call_us_fast_kernels": 1e6 * float(np.median(lat_fast)),
            "arithmetic": "exact (the reference's bits)" if exact_on else "fast",
            "reference_cpu_s_per_chain_step": 1.2,
            "includes": "score_call_us: one synchronous nemo_score call for one (pos, W) from host "
                        "arrays; fused_step_ms: nemo_optimal_weights_w for one chain (W~ and ancestor_x, "
                        "eval#1 with order weights, 2016 local optima, eval#2, transfers)"}
        # the whole sampler: 16 chains' host state machines (reference call order,
        # Python random) + one fused device call per step
        from nemo import utils as nutils
        from nemo.chains import ChainBatch
        from nemo.invpool import InvPool, default_workers
        order0 = nutils.initial_order_guess(m.observed_knockdown_mat)
        seeds = [1234 + c for c in range(nch)]
        # ancestor_x on the device (the default at S <= 64); an InvPool of host
        # worker processes (scipy's getrf / getri) beside it for the A/B
        nw = default_workers()
        pool = InvPool(S, nch, n_workers=nw)
        # the host side (Python) is noisy run to run: three timed runs, the
        # median reported
        n_it = 30
        e2e = {}
        # the fused calls the sampler itself makes, timed in place (its own
        # inputs: the step's cost depends on them), so the host's share is the
        # run's wall time minus these
        from nemo import engine as nengine
        call_run = nengine._OptimalWeightsWCall.run
        in_call = []

        def timed_run(self):
            t0 = time.perf_counter()
            call_run(self)
            in_call[-1] += time.perf_counter() - t0

        for tag, pl, reps in (("device", None, 3), ("pool", pool, 1)):
            ChainBatch(m, [order0] * nch, seeds=seeds, engine=eng, on_fail="continue", inv_pool=pl).run(2)
            walls = []
            for _ in range(reps):
                cb = ChainBatch(m, [order0] * nch, seeds=seeds, engine=eng, on_fail="continue", inv_pool=pl)
                if pl is None:
                    in_call.append(0.0)
                    nengine._OptimalWeightsWCall.run = timed_run
                try:
                    t0 = time.perf_counter()
                    cb.run(n_it)
                    walls.append(time.perf_counter() - t0)
                finally:
                    nengine._OptimalWeightsWCall.run = call_run
            e2e[tag] = (float(np.median(walls)), cb.best_scores, walls)
        # the same sampler with the fast kernels (the host's share of a step)
        eng.set_option("exact", 0)
        ChainBatch(m, [order0] * nch, seeds=seeds, engine=eng, on_fail="continue").run(2)
        cbf = ChainBatch(m, [order0] * nch, seeds=seeds, engine=eng, on_fail="continue")
        t0 = time.perf_counter()
        cbf.run(n_it)
        e2e_fast = time.perf_counter() - t0
        eng.set_option("exact", 1)
        pool.close()
        dt = e2e["device"][0]
        extras["mcmc_end_to_end"] = {
            "chains": nch, "steps": n_it, "ms_per_step": 1e3 * dt / n_it,
            "ms_per_step_runs": [1e3 * w / n_it for w in e2e["device"][2]],
            "chain_steps_per_s": nch * n_it / dt,
            "over_fused_step": (dt / n_it) / fs,
            # the sampler's own fused calls (its inputs), timed in place: the
            # step's device + transfer share and the host's share of the wall
            "fused_calls_ms_per_step": 1e3 * float(np.median(in_call)) / n_it,
            "host_ms_per_step": 1e3 * (dt - float(np.median(in_call))) / n_it,
            "over_own_fused_calls": dt / float(np.median(in_call)) if in_call and min(in_call) > 0 else None,
            "includes": "ChainBatch.run: proposals, reset quirks and accept per chain on the host + the fused "
                        "device step from W (W~ and ancestor_x on the device, in scipy's bits)",
            "ms_per_step_host_pool": 1e3 * e2e["pool"][0] / n_it,
            "host_pool_workers": nw,
            "arithmetic": "exact (the reference's bits)" if exact_on else "fast",
            "ms_per_step_fast_kernels": 1e3 * e2e_fast / n_it,
            "device_bits_equal_host_pool": bool(np.array_equal(e2e["device"][1], e2e["pool"][1])),
            "reference_cpu_s_per_chain_step": 1.2}
        if args.config == "C3":
            # BASELINE config C5 (128 x 5000, parent cap 6): the capped
            # lookup-table kernel next to the fp64 MFMA factored kernel
            extras["c5_capped"] = c5_capped(torch, dist, stream, warmup_s=min(args.warmup_seconds, 0.3))
            # uncapped 64 < S <= 128: the wide int8 kernel next to the fp64 one
            extras["wide_uncapped"] = wide_uncapped(torch, dist, stream, warmup_s=min(args.warmup_seconds, 0.3))

    if rank == 0:
        if factored:
            roof = score_roofline(args.config, S, E, cap, B, fk, kern_ms, launch_ev_ms, bid)
        else:
            bpe = algorithmic_bytes_per_eval(S, E, cap, 8 if dtype == "f64" else 4)
            tr = load_record("traffic.json", f"{args.config}:stream:b{B}", bid)
            roof = stream_roofline(B, bpe, kern_ms, tr)
            roof.update({"kernel": "score_kernel (streams exp(T) rows)", "kernel_avg_ms": kern_ms,
                         "kernel_avg_ms_launch_events": launch_ev_ms})
        roof["build_id"] = bid
        tag = kernel_tag(fk) if factored else "stream"
        path = "factored" if factored else "stream"
        rec = {
            "metric": "order-score evals/sec (64 S-genes x 2000 effects); HBM GB/s fraction",
            "value": world * B * args.steps / t_max,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * t_max / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ARITH.get(tag, "f64" if dtype == "f64" else "f32"),
            "ll_error_bound": err_bound,
            "ll_error_bound_note": ("worst-case |ll error| of the kernel's fixed-point arithmetic for this "
                                    "model (nemo_score_kernel; DESIGN.md 3.5a); auto keeps it within the "
                                    "err_budget option (1e-7)"),
            "data": "synthetic (build-defined generator, SURVEY.md 8(d)); random orders, W~U(-3,3)",
            "config": {"workload": f"{args.config}: S={S} E={E} cap={cap} {dtype} tables, {B} order-score "
                                   f"evaluations per step per GPU, {path} kernel",
                       "S": S, "E": E, "cap": cap, "batch_per_gpu": B, "path": path,
                       "parallelism": f"independent evaluations/chains sharded over {world} GPU(s); "
                                      "one RCCL all-gather of best scores"},
            "roofline": roof,
            "ll_sample": float(ll[0]),
        }
        rec.update(extras)
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(m, args.cpu_seconds, args.config)
            rec["cpu_baseline"]["host_nproc"] = os.cpu_count()
            rec["cpu_baseline"]["host_cpu"] = host_cpu()
            if args.cpu_procs > 1:  # also all the host cores the round budget allows
                rec["cpu_baseline_procs"] = cpu_baseline_procs(args.config, args.cpu_procs, args.cpu_seconds)
                rec["cpu_baseline_procs"]["host_nproc"] = os.cpu_count()
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
