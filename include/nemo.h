/*
 * nemo.h -- C-ABI of the MI355X order-score engine for Nested Effects Model
 * order MCMC (drop-in for the per-step scorer of MrGreyPanda/NEM-MCMC-optimization).
 *
 * The reference has no FFI layer: its boundary is the Python method surface of
 * NEMOrderMCMC.  Each entry point below replaces one of those
 * methods; the Python host (nemo.nem_order_mcmc) keeps the reference's names
 * and signatures and delegates here through ctypes.
 *
 * Conventions
 *   - plain pointers and sizes; host buffers are caller-owned and only borrowed
 *     for the call; device buffers are owned by the context;
 *   - every call returns NEMO_OK (0) or a negative code, and nemo_last_error()
 *     (thread-local) explains it; the Python host raises RuntimeError with it;
 *   - host-pointer calls are synchronous (the context stream is synchronised
 *     before return); *_dev calls take device pointers and only enqueue work on
 *     the given stream (hipStream_t passed as void*; NULL = HIP's null stream);
 *   - one context per (device, model); calls on one context must not overlap.
 *     Different contexts may be driven from different threads: graph capture
 *     and the calls that allocate or use the legacy stream (create, destroy,
 *     stage, reserve, the probes) serialise on one process-wide lock.
 *
 * Layouts (row-major, C order):
 *   T    [S][S][E]  score table, T[i][j][e]: child i, candidate parent j
 *   U    [S+1][E]   node LR table, row S = "effect attached to nothing"
 *   pos  [batch][S] int32 position of every S-gene in the order (inverse of pi)
 *   w01  [batch][S][S] parent weights already mapped to [0,1]
 *        (the reference maps with expit inside compute_cell_ratios,
 *         nem_order_mcmc.py:84-86; methods.py:52-57 passes them unmapped)
 *   Only entries (i, j) with pos[j] < pos[i] (and, with cap > 0,
 *   pos[i] - pos[j] <= cap) are read: these are the permissible parents.
 */
#ifndef NEMO_H
#define NEMO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nemo_ctx nemo_ctx;

/* table storage / elementwise arithmetic type */
enum { NEMO_F64 = 0, NEMO_F32 = 1 };

/* return codes */
enum {
  NEMO_OK = 0,
  NEMO_ERR_ARG = -1,     /* bad argument (shape, pointer, range)          */
  NEMO_ERR_HIP = -2,     /* HIP runtime error (no device, OOM, launch)    */
  NEMO_ERR_STATE = -3,   /* tables not staged / capacity not reserved     */
  NEMO_ERR_OPT = -5,     /* a local optimisation did not converge         */
  NEMO_ERR_LINALG = -6   /* ancestor_x: I - W~ singular or not finite      */
};

/* per-problem termination codes of the local optimiser (scipy task names) */
enum {
  NEMO_LBFGSB_CONV_PGTOL = 0,  /* CONVERGENCE: NORM_OF_PROJECTED_GRADIENT_<=_PGTOL */
  NEMO_LBFGSB_CONV_REL = 1,    /* CONVERGENCE: REL_REDUCTION_OF_F_<=_FACTR*EPSMCH  */
  NEMO_LBFGSB_ABNORMAL = 2,    /* ABNORMAL_TERMINATION_IN_LNSRCH                  */
  NEMO_LBFGSB_MAXITER = 3      /* STOP: TOTAL NO. of ITERATIONS REACHED LIMIT     */
};

const char* nemo_last_error(void);
int nemo_version(void);
/* identity of this build: a hash of the sources and compile flags it was
 * built from (bench.py matches profiler records against it) */
const char* nemo_build_id(void);
/* number of visible HIP devices (0 on a host without GPU; never an error) */
int nemo_device_count(int* count);

/* ---- context lifetime (replaces NEMOrderMCMC.__init__'s table setup,
 *      nem_order_mcmc.py:40-46) ------------------------------------------ */
int nemo_ctx_create(int device, int num_s, int num_e, int dtype, nemo_ctx** out);
void nemo_ctx_destroy(nemo_ctx* ctx);
/* grow per-batch scratch so *_dev calls with up to max_batch evaluations
 * (and max_chains chains for nemo_optimal_weights_dev) never allocate: with a
 * model staged (before or after this call) that covers the exact step's
 * buffers as well, so such a _dev call only enqueues and may be captured into
 * the caller's graph.  Without the reservation the first _dev call with more
 * chains allocates and synchronises the context's stream (not capturable). */
int nemo_reserve(nemo_ctx* ctx, int max_batch, int max_chains);

/* ---- A1/A2: stage the model once (nem.py:25-64 outputs) ---------------- */
int nemo_stage_tables(nemo_ctx* ctx, const double* U, const double* T);
/* the same model built on the device from the observed knockdown matrix
 * (nem.py:25-64, the tables NEM.__init__ derives, nem_order_mcmc.py:44):
 *   D [S][E] bytes in {0,1} (NEM.observed_knockdown_mat), A = log(alpha/(1-beta)),
 *   B = log(beta/(1-alpha)) (NEM.A, NEM.B, nem.py:17-18).
 * T[i][j] = where(D[j]==0, B, -A) off the diagonal, T[i][i] = U[i] with
 * U[i] = where(D[i]==1, 0, B) + A per other 1 in the column, U[S] = A per 1.
 * Stages bit-for-bit what nemo_stage_tables stages for those U and T, with
 * no S*S*E host table (655 MB at C5 in fp64). */
int nemo_stage_knockdown(nemo_ctx* ctx, const uint8_t* D, double A, double B);

/* ---- A4+A5: batched order-score evaluation --------------------------------
 * Replaces NEMOrderMCMC.compute_cell_ratios + calculate_ll
 * (nem_order_mcmc.py:79-93) and utils.compute_ll (utils.py:84-94).
 *   ll_out    [batch]           sum_e logsumexp_i cell[i][e]
 *   cs_out    [batch][E]        per-effect log-sum-exp (nullable)
 *   cells_out [batch][S+1][E]   cell ratios (nullable)
 *   ow_out    [batch][S+1][E]   order weights exp(cell - cs) (nullable)
 * cap = 0: every predecessor is a permissible parent (the reference);
 * cap > 0: only the `cap` nearest predecessors (build-defined C5 extension). */
int nemo_score(nemo_ctx* ctx, int batch, const int32_t* pos, const double* w01, int cap,
               double* ll_out, double* cs_out, double* cells_out, double* ow_out);
int nemo_score_dev(nemo_ctx* ctx, int batch, const int32_t* d_pos, const double* d_w01, int cap,
                   double* d_ll, double* d_cs, double* d_cells, double* d_ow, void* stream);

/* reuse-batched variant: `group` evaluations share every table row read
 * (group in {1,4,8,16}); same results as nemo_score_dev */
int nemo_score_group_dev(nemo_ctx* ctx, int batch, int group, const int32_t* d_pos, const double* d_w01,
                         int cap, double* d_ll, void* stream);

/* ---- utils.compute_ll / calculate_ll on a given cell matrix ------------- */
int nemo_lse(nemo_ctx* ctx, int rows, const double* cells, double* ll_out, double* cs_out, double* ow_out);

/* ---- A8 core: batch of penalised 1-D local problems -----------------------
 * Replaces scipy.optimize.minimize(local_ll_sum_penalized, x0,
 * bounds=[(-inf, inf)], args=(c, x_anc), method='L-BFGS-B', tol=0.01)
 * (nem_order_mcmc.py:18-23, 167): f(x) = -sum_e log(c_e*expit(x) + 1)
 *   + |expit(x) - x_anc| + expit(x)*(1 - expit(x)), forward-difference
 * gradient with absolute step 1e-8, L-BFGS-B 3.0 logic for n = 1.
 *   c [n][E], anc [n], x0 [n] -> xstar, fstar [n]; nit, nfev, status [n] */
int nemo_local_opt(nemo_ctx* ctx, int n, const double* c, const double* anc, const double* x0,
                   double* xstar, double* fstar, int32_t* nit, int32_t* nfev, int32_t* status);

/* ---- A6 fused per-step scorer (get_optimal_weights(init=True, max_iter=1),
 *      nem_order_mcmc.py:172-208) for a batch of chains --------------------
 * per chain: eval#1 on w01 (order weights kept on device), the local optimum
 * of every permissible (i, k) pair (c built from T[i][k], order weights row k,
 * w01[i][k]; x0 = w01[i][k]; anc[i][k]), then eval#2 on the binarised weights
 * (sigma(x*) > 0.5 ? sig1 : sig0, sig0 = expit(0), sig1 = expit(1)).
 *   anc    [nchains][S][S]  clip(inv(I - expit_parent_weights(W)) - I, 0, 1)
 *   w_new  [nchains][S][S]  expit(x*) at permissible entries (others untouched)
 *   info   [nchains][S][S]  nullable; status | nit << 4 | nfev << 16 per pair,
 *                           -1 at entries that are not a permissible pair
 *   ll1, ll_dag [nchains]
 * Returns NEMO_ERR_OPT (results still written) if any pair ended abnormally.
 * _dev: the same on device pointers, queued on `stream` (null: the context's),
 * without the NEMO_ERR_OPT check (read it from d_info). */
int nemo_optimal_weights(nemo_ctx* ctx, int nchains, const int32_t* pos, const double* w01,
                         const double* anc, double sig0, double sig1, int cap, double* w_new,
                         double* ll1, double* ll_dag, int32_t* info);
int nemo_optimal_weights_dev(nemo_ctx* ctx, int nchains, const int32_t* d_pos, const double* d_w01,
                             const double* d_anc, double sig0, double sig1, int cap, double* d_w_new,
                             double* d_ll1, double* d_ll_dag, int32_t* d_info, void* stream);
/* nemo_optimal_weights as a queued call: _begin checks the context and
 * pointers and returns at once; a library thread runs the queued calls in
 * order (transfers, launches, the NEMO_ERR_OPT check), two in flight at a
 * time: it stages and queues the next call's device work before it waits for
 * the previous one, so the device runs them back to back; _end waits for the
 * oldest call not yet ended and returns its result code (nemo_last_error()
 * then holds its message).  The caller keeps every buffer alive and untouched
 * until the matching _end, and makes no other call on ctx in between except
 * further _begin / _end.  Replaces, like nemo_optimal_weights,
 * get_optimal_weights(init=True) (nem_order_mcmc.py:172-208) for a caller
 * that runs chain groups in a pipeline (nemo/chains.py). */
int nemo_optimal_weights_begin(nemo_ctx* ctx, int nchains, const int32_t* pos, const double* w01,
                               const double* anc, double sig0, double sig1, int cap, double* w_new,
                               double* ll1, double* ll_dag, int32_t* info);
int nemo_optimal_weights_end(nemo_ctx* ctx);
/* nemo_optimal_weights from the weights themselves, as the reference's step
 * starts (nem_order_mcmc.py:172-208 with :98-103 and :185): the device makes
 * each chain's W~ = expit(W) on the permissible entries (cap as below; the
 * other entries W's own) and ancestor_x = clip(inv(I - W~) - I, 0, 1) in
 * scipy.linalg.inv's bits (LAPACK getrf + getri of scipy's OpenBLAS 0.3.28,
 * restated in csrc/nemo_ancestor.hip), then runs the step on them.  S <= 64.
 *   w        [nchains][S][S]  the weights W (after the proposal's reset)
 *   w01_out, anc_out [nchains][S][S]  nullable: W~ and ancestor_x (both null:
 *                             neither leaves the device)
 *   anc_flag [nchains]        nullable: 0, or 1 singular / 2 not finite /
 *                             4 non-finite factors (recompute on the host)
 * Returns NEMO_ERR_LINALG when a flag is set (the step's results are then
 * not meaningful: scipy.linalg.inv raises LinAlgError / ValueError for 1 / 2),
 * else as nemo_optimal_weights.  _begin: the queued form (ended by
 * nemo_optimal_weights_end, in submission order with the other _begin). */
int nemo_optimal_weights_w(nemo_ctx* ctx, int nchains, const int32_t* pos, const double* w, double sig0,
                           double sig1, int cap, double* w01_out, double* anc_out, double* w_new,
                           double* ll1, double* ll_dag, int32_t* info, int32_t* anc_flag);
int nemo_optimal_weights_w_begin(nemo_ctx* ctx, int nchains, const int32_t* pos, const double* w,
                                 double sig0, double sig1, int cap, double* w01_out, double* anc_out,
                                 double* w_new, double* ll1, double* ll_dag, int32_t* info,
                                 int32_t* anc_flag);
/* the same W~ / ancestor_x / flags on device buffers, queued on `stream`
 * (null: HIP's null stream); feeds nemo_optimal_weights_dev.  S <= 64. */
int nemo_ancestor_dev(nemo_ctx* ctx, int nchains, const int32_t* d_pos, const double* d_w, int cap,
                      double* d_w01, double* d_anc, int32_t* d_flag, void* stream);
/* order weights of chain `chain` from the last eval#1 of nemo_optimal_weights:
 * (S+1)*E doubles (NEMOrderMCMC.order_weights after get_optimal_weights) */
int nemo_fetch_order_weights(nemo_ctx* ctx, int chain, double* ow_out);
/* diagnostic (option "exact_trace" 1): the last exact fused step's local
 * optima, [*n][4]: start / end times (wall_clock64, 100 MHz ticks) and the
 * shader cycles spent in the objective / the optimiser's control, in launch
 * order (chain-major, each chain's pair list); out may be NULL to query *n.
 * No reference counterpart: profiling of the scheduling only. */
int nemo_fetch_exact_trace(nemo_ctx* ctx, int* n, long long* out);

/* ---- fixed-order optimizers of methods.py ---------
 * Every call handles nprob independent problems (one order each) with host
 * buffers; w / w_out are [nprob][S][S] (w_out = w with every permissible pair
 * replaced by its optimum), ll_out [nprob] is the sweep's evaluation, info
 * (nullable) as for nemo_optimal_weights.  NEMO_ERR_OPT (results written)
 * when a local optimisation fails, where the reference raises
 * (methods.py:115, :394).
 *
 * Method.opt_gamma (methods.py:397-405): evaluation on the raw weights in
 * [0, 1], then per pair minimize(local_ll_sum_gamma (:8-9), x0 = w[i][k],
 * bounds [(0, 1)], jac=True, tol=0.01) with c from exp(T[i][k]) and order
 * weights row k (:385-395).  cap as for nemo_score (0 = the reference). */
int nemo_gamma_sweep(nemo_ctx* ctx, int nprob, const int32_t* pos, const double* w, int cap,
                     double* w_out, double* ll_out, int32_t* info);
/* InverseMethod (methods.py:21-172): w holds log-weights (-5000 off the
 * parents).  out = unorder_arr(order, B / (1 + B)) with B =
 * solve_triangular(I - order_arr(order, exp(w)), I, lower=True)
 * (:118-121, :160-164). */
int nemo_inverse_ancestral(nemo_ctx* ctx, int nprob, const int32_t* pos, const double* w, double* out);
/* InverseMethod.opt_b (:117-129): evaluation on B/(1+B), then every pair
 * in the reference's loop order minimises local_ll_sum_b_inv (:73-82),
 * bounds [(-5000, 500)], eps 1e-3, tol 0.1, each pair seeing the optima of
 * the pairs before it (levels of independent pairs on the device). */
int nemo_inverse_sweep(nemo_ctx* ctx, int nprob, const int32_t* pos, const double* w, double* w_out,
                       double* ll_out, int32_t* info);

/* ---- options -------------------------------------------------------------
 *   "xcd_remap"  1 (default) XCD-aware block order; speed only
 *   "score_path" 0 (default) auto: the factored MFMA kernel when the staged
 *                table has the NEM structure (every off-diagonal row T[.][j]
 *                shared by all children and two-valued), else the streaming
 *                kernel; 1 = always stream; 2 = always factored
 *   "fact_kernel" 0 (default) auto: ll-only calls with S <= 64 take the
 *                int8 fixed-point factored kernel, the rest the chunked fp64
 *                one; 1 = chunked; 2 / 3 = fp64 pipelined with 4 / 8 waves
 *                per block; 4 / 5 = int8 with 4 / 5 digit pairs; 6 = int8
 *                with 8 waves per block; 7 / 8 = int8 with the offset
 *                log-sum-exp (4 / 8 waves), which auto prefers when the
 *                staged model passes its range checks (option "i8o");
 *                9 = the banded lookup-table kernel for capped calls
 *                (1 <= cap <= 6), which auto prefers for ll-only capped
 *                calls when the model passes its checks (option "win");
 *                10 / 11 = the offset kernel in log2 fixed point (8 / 4
 *                waves), which auto prefers over 7 / 8 when staged
 *                (option "i8l"; 10 walks two 16-effect tiles per
 *                iteration); 12 = the same with 16 waves per block,
 *                13 = its register-stationary variant, 14 = 8 waves with
 *                one tile per iteration compiled for 6 waves per SIMD,
 *                16 = 8 waves with one tile per iteration (11, 12, 14 and
 *                16 give one another's bits, within 1e-11 of 10's);
 *                15 = the round-1 form of 9 (row bits re-read from LDS);
 *                17 = 10's walk in persistent blocks that prep the next
 *                evaluation's digits during the walk (10's bits);
 *                18 = the log2 kernel for 64 < S <= 128 (two K = 64 halves,
 *                two tiles per iteration), which auto takes for uncapped
 *                ll-only calls there within the error budget; 19 = the same
 *                with one tile per iteration; 20 = 10 as two launches, a
 *                prep-only one writing each evaluation's digits to HBM and a
 *                walk-only one reading them (10's bits; an experiment,
 *                measured slower)
 *   "factored"   (get only) 1 if the staged table is factorable
 *   "win"        (get only) 1 if the capped lookup-table kernel is staged
 *                (U - U[S] two-valued per row, partial sums in range)
 *   "i8o"        (get only) 0: no offset int8 kernel for this model; 1: it
 *                reads U - U[S] per cell; 2: U - U[S] is two-valued per row
 *                and rides in the contraction (no U reads)
 *   "i8o_nodiag" 1 = keep the U reads even when 2 is available (testing)
 *   "i8l"        (get only) 1 if the log2 fixed-point offset kernel is staged
 *                (i8o = 2 and |Delta|, |U - U[S]| / ln 2 within its digit range)
 *   "i8w"        (get only) 1 if the same is staged for 64 < S <= 128 (18 / 19)
 *   "graphs"     1 (default): nemo_optimal_weights replays its device work
 *                as a hipGraph per (nchains, cap); 0 = direct launches
 *   "step_host_sum" 1 (default): nemo_optimal_weights (and _begin / _end)
 *                copy eval #2's per-evaluation partials out with the other
 *                outputs and sum them on the host in the device's fixed
 *                order (same bits, one launch fewer); 0 = the device sums
 *                them (as nemo_optimal_weights_dev always does)
 *   "local_split" 2 = run each local optimum of a fused step on a 4-wave
 *                block (the objective's products split over the waves; same
 *                bits; measured slower for one chain, so 0 = auto never
 *                takes it), 1 = never, 3 = the same on a 2-wave block
 *   "exact"      1 (default): nemo_optimal_weights, nemo_local_opt and the
 *                ll-only host-pointer nemo_score (any batch; with
 *                "fact_kernel" 0 -- an explicitly chosen kernel runs as
 *                chosen -- and no effective cap) compute in the
 *                reference's own arithmetic -- numpy's SVML log / exp, glibc's
 *                exp / log1p, numpy's pairwise sum and scipy's compact-form
 *                L-BFGS-B with OpenBLAS's small kernels, restated bit for bit
 *                (csrc/refmath.h, csrc/lbfgsb_exact.h, csrc/nemo_exact.hip):
 *                the same order scores, order weights, local optima and
 *                weights as nem_order_mcmc.py, to the bit, when "exact_ok";
 *                0 = the fast kernels (scores within ~1e-9)
 *   "exact_dev"  0 (default): nemo_score_dev runs the fast kernels; 1 = the
 *                same conditions as "exact" on nemo_score, on device buffers
 *                (cells built in d_ow -- then order weights in place -- or in
 *                d_cells, not both)
 *   "exact_ok"   (get only) 1 if the staging supports "exact" (factored
 *                tables, any parent cap, E <= 524288: numpy's np.sum adds
 *                buffers of 8192 terms in order, each summed pairwise, and
 *                the local optima run one wave plan per buffer)
 *   "exact_form" the exact local-optimum kernel's form (same bits): 0 auto
 *                (default: the latency form while chains x pairs <=
 *                "exact_lat_waves", 20000 by default ~ 10 C3 chains, the slot
 *                form beyond; the pair form while chains x pairs <=
 *                "exact_pair_waves", 0 by default), 1 latency (one wave per
 *                optimum, two per SIMD, the optimum's c values held in
 *                registers), 2 throughput (four per SIMD, c recomputed each
 *                evaluation), 3 pair (two waves per optimum, the objective's
 *                slots split between them; E > 1024), 4 cached throughput
 *                (three per SIMD, the cache partly in scratch), 5 dual (two
 *                optima per wave, one per half; measured slower, DESIGN.md
 *                3.5e), 7 slot (four per SIMD, c made once per optimum into
 *                the resident wave's own row set in device memory, read at
 *                each evaluation; needs "exact_cform" 1 and "exact_persist",
 *                else the throughput form); E > 8192 always runs the
 *                throughput form
 *   "timing_kernel" 0 (default): nemo_timing_enable / _read time the score
 *                kernels; 1: the exact local optima's kernel (bench.py)
 *   "anc_overlap" 1 (default): nemo_optimal_weights_w makes ancestor_x on a
 *                second stream beside eval #1 (same bits); 0 = in line */
int nemo_set_option(nemo_ctx* ctx, const char* name, int value);
int nemo_get_option(nemo_ctx* ctx, const char* name, int* value);

/* ---- the fixed-point kernels' error budget ---------------------------------
 * The int8 kernels round every entry of their contraction once (Delta of each
 * permissible parent, the diagonal U entry, the row constant G); the roundings
 * repeat over the effects, so their worst-case ll error grows with E:
 *   |d ll| <= eps * sum_e (min(colbits_e, k) + 1) + E * series
 * (colbits_e = staged rows whose D1 bit is set at effect e, k = S or cap + 1;
 * eps = 2^-39 ln 2 for the log2 kernels 10-14, 16, 17, 2^(c - 49) for 4-8;
 * DESIGN.md 3.5a).  Auto (fact_kernel 0) takes an int8 kernel only while that
 * bound stays within "err_budget", else the next more precise one, down to
 * the fp64 MFMA kernels.
 *   f64 options: "err_budget" (get / set; default 1e-7, the north star's
 *                1e-6 ll tolerance with a 10x margin);
 *                "i8l_bound", "i8o_bound" (get only): the bound of the log2 /
 *                natural-units kernels for an uncapped call on the staged model */
int nemo_set_option_f64(nemo_ctx* ctx, const char* name, double value);

/* Test hook: refmath.h's restatements evaluated on the current device, for
 * the tests that compare them with numpy / scipy bit for bit.  fn: 0 np.log
 * (SVML), 1 np.exp (SVML), 2 scipy.special.expit, 3 np.logaddexp(x, y),
 * 4 glibc exp, 5 glibc log1p, 6 sqrt, 7 x / y (the optimiser's IEEE operations),
 * 8 glibc log1p on [0, 1] as logaddexp evaluates it.
 * Host arrays of n doubles (y only for fn 3 and 7). */
int nemo_refmath_probe(int fn, int n, const double* x, const double* y, double* out);
int nemo_get_option_f64(nemo_ctx* ctx, const char* name, double* value);
/* which fact_kernel a factored score call with this cap takes (ll_only: no
 * cs / cells / order-weight outputs), with the worst-case |ll error| bound of
 * its fixed-point arithmetic (0 for the fp64 kernels); *fact_kernel = -1 when
 * the call takes the streaming kernel or the requested kernel cannot serve it */
int nemo_score_kernel(nemo_ctx* ctx, int cap, int ll_only, int* fact_kernel, double* bound);

/* ---- timing of the dominant (score) kernel, for bench.py ---------------- */
int nemo_timing_enable(nemo_ctx* ctx, int enable);
/* total milliseconds and number of score-kernel launches since enable/reset */
int nemo_timing_read(nemo_ctx* ctx, double* total_ms, int* launches);

#ifdef __cplusplus
}
#endif

#endif /* NEMO_H */
