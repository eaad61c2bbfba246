// nemo_internal.h -- context and launcher declarations shared by the C-ABI
// (nemo_abi.cpp) and the HIP kernels (nemo_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "nemo_host.h"

namespace nemo {

constexpr int kWave = 64;
constexpr int kMaxS = 256;         // one prep block covers all S-genes
constexpr int kScoreWaves = 4;     // waves per score block (child split)
constexpr int kTileCols = kWave;   // effects per score block
constexpr int kFactWaves = 8;      // waves per factored-score block (16 effects each)
constexpr int kI8MaxPairs = 5;     // digit-slice pairs of the int8 factored kernel
constexpr int kWinMaxCap = 6;      // capped lookup-table kernel: parents per child
constexpr int kWinMaxS = kMaxS;    // ... and S (LDS: ~356 S bytes per block)
constexpr int kExactMaxSlots = 8;  // exact local optima: numpy's pairwise sum of E in <= 64 leaf blocks per part
constexpr int kExactMaxParts = 64; // ... per numpy buffer of 8192 terms, 64 of them (E <= 524288)

// Device state of one staged model on one GPU.
struct Ctx {
  int device = 0;
  int S = 0, E = 0, dtype = 0;     // dtype: 0 f64, 1 f32
  hipStream_t stream = nullptr;
  // nemo_optimal_weights_w: ancestor_x on stream2 beside eval #1 (option
  // "anc_overlap"), forked and joined through these events
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  int anc_overlap = 1;
  bool staged = false;
  int xcd_remap = 1;               // option "xcd_remap": XCD-aware block order
  double table_absmax = 0.0;       // max |T| over off-diagonal rows
  bool local_prod = true;          // option "local_prod": local optima sum logs as one log of a product
  int local_split = 0;             // option "local_split": 0 auto, 1 never, 2 always (4 waves per problem)
  void* d_eT = nullptr;            // exp(T) [S][S][E] (dtype)
  void* d_U = nullptr;             // U [S+1][E] (dtype)

  // per-batch scratch (grown by reserve)
  int cap_batch = 0, cap_chains = 0;
  int32_t* d_pos = nullptr;        // [cap][S]
  double* d_w01 = nullptr;         // [cap][S][S]
  double* d_anc = nullptr;         // [chains][S][S]
  int32_t* d_rows = nullptr;       // [cap][S][S]   parent list per child
  double* d_sw = nullptr;          // [cap][S][S]   weight per list entry
  int32_t* d_cnt = nullptr;        // [cap][S]
  int32_t* d_pairs = nullptr;      // [chains][S*S] (child << 16 | list index)
  double* d_partial = nullptr;     // [cap][ntiles]
  double* d_ll = nullptr;          // [cap]
  double* d_ll2 = nullptr;         // [chains]
  double* d_cs = nullptr;          // [cap][E]
  double* d_ow = nullptr;          // [max(cap, chains)][S+1][E]
  double* d_wnew = nullptr;        // [chains][S][S]
  double* d_wdag = nullptr;        // [chains][S][S]
  int32_t* d_info = nullptr;       // [chains][S][S]
  double* d_c = nullptr;           // generic local-opt inputs [n][E] (grown on demand)
  size_t c_capacity = 0;
  int ow_chains = 0;               // chains whose order weights d_ow holds

  // factored (MFMA) path: available when every off-diagonal table row is
  // shared by all children and two-valued (all tables nem.py builds)
  int score_path = 0;              // option "score_path": 0 auto, 1 stream, 2 factored
  int fact_kernel = 0;             // option "fact_kernel": 0 auto, 1 chunked, 2/3 f64 pipelined
                                   // (4/8 waves), 4/5 int8 (4/5 digit pairs), 6 int8 x 8 waves,
                                   // 7/8 int8 offset LSE (4/8 waves), 9 capped lookup tables,
                                   // 10/11 int8 offset LSE in log2 fixed point (8/4 waves)
  bool factored = false;
  int fspad = 0;                   // S rounded up to the MFMA row-block size
  int nwords = 0;                  // 64-bit words per D1 row
  uint64_t* d_D1w = nullptr;       // [S][nwords] bit D1[j][e]: T row j takes its "hi" value
  double* d_elo = nullptr;         // [S] exp(lo_j)
  double* d_ehi = nullptr;         // [S] exp(hi_j)
  double* d_U64 = nullptr;         // U in fp64 [S+1][E]
  double* d_fDp = nullptr;         // [cap][fspad][fspad] Delta in order positions
  double* d_fG = nullptr;          // [cap][fspad]
  int32_t* d_fperm = nullptr;      // [cap][fspad]
  double* d_fpartial = nullptr;    // [cap][factored_partials]
  // where the score kernels write their per-evaluation partials when set
  // (fpartial()): the fused step's staged path points eval #2's at its
  // staging block, so they ride in the one D2H copy and the host sums them
  double* part_out = nullptr;
  // int8 matrix-core variant (S <= 64): fixed-point Delta digits
  int i8_cexp = 0;                 // per-model scale: 2^(c-1) >= max_j |hi_j - lo_j|
  uint8_t* d_B8 = nullptr;         // [2][KH][ceil(E/16)][64 lanes][16] D1 bytes in B-fragment order
                                   // (KH = 1 K half for S <= 64, 2 for S <= 128),
                                   // then the same x 64
  // offset log-sum-exp variant (score_i8o_kernel), staged by stage_i8o
  bool i8o_ok = false;             // staging bounds hold: |cell - U[S]| <= 690
  double i8o_padg = 0.0;           // G of padding rows
  double* d_Uoff = nullptr;        // [fspad + 1][E] + 16: U - U[S], zero past row S-1
  double* d_nullsum = nullptr;     // [nsets] sum of U[S][e] over each 8-tile set
  void* d_i8o_tabs = nullptr;      // exp table [2048] uint2 + log table [128] double2
  bool i8o_diag = false;           // U' = u0 + du D1 per row: folded into the contraction
  bool i8o_nodiag = false;         // option "i8o_nodiag": keep the U' loads (testing)
  int8_t* d_udig = nullptr;        // [S][8] digits of du_i (the diagonal A entries)
  // log2 fixed-point epilogue of the same kernel (stage_i8o): Delta, G and U'
  // digits in units of 2^-20 / ln 2, so the contraction yields y = x / ln 2
  // and 2^y is assembled from the integer accumulators (no f64 range reduction)
  bool i8l_ok = false;             // diagonal form and the fixed-point ranges hold
  int8_t* d_udig2 = nullptr;       // [S][8] digits of du_i / ln 2
  double* d_u0 = nullptr;          // [S] u0_i, added to G
  // fact_kernel 20 (experiment): the prep's LDS image of each evaluation
  // (G split, perm, digits) written by a prep-only launch, read by a walk-only one
  int32_t* d_i8img = nullptr;      // [i8img_cap][i8l image]
  int i8img_cap = 0;
  // the same for 64 < S <= 128 (score_i8w_kernel; d_B8 then holds two K halves)
  bool i8w_ok = false;
  double* d_nullsum_w = nullptr;   // [ceil(ntiles / 2)] sum of U[S][e] per 32 effects
  // capped lookup-table variant (score_window_kernel), staged by stage_window
  bool win_ok = false;             // U - U[S] two-valued per row, partial sums in range
  double* d_wuw = nullptr;         // [S][2] U - U[S] of row i at D1 bit 0 / 1
  double* d_wnull = nullptr;       // [nwords] sum of U[S][e] over each 64-effect word

  // the reference's own arithmetic in the fused step and the sampler's ll-only
  // calls (nemo_exact.hip): option "exact" (1 default), available when the
  // staged model is factored and numpy's pairwise sum of E fits the wave plan
  int exact = 1;
  // the local-optimum kernel's form: 0 auto (the pair form up to
  // exact_pair_waves optima, none by default; the latency form -- its c values
  // held in registers -- up to exact_lat_waves, ~10 C3 chains, measured best
  // from 1 to 8 chains; the slot form beyond, best from 12), 1 latency, 2
  // throughput, 3 pair, 4 cached throughput, 5 dual, 7 slot
  int exact_form = 0;
  int exact_lat_waves = 20000;
  int exact_pair_waves = 0;
  bool exact_ok = false;
  double* d_xlo = nullptr;         // [S] numpy's exp(lo_j) (refmath::svml_exp)
  double* d_xhi = nullptr;         // [S] numpy's exp(hi_j)
  int32_t* d_pwplan = nullptr;     // host::PairwisePlan of E (pw_parts of them, pw_ns slots each), device layout
  int32_t* d_pwmeta = nullptr;     // [pw_parts][2]: each part's tree height and largest trailing count
  int pw_ns = 0, pw_nh = 0, pw_maxrem = 0, pw_parts = 1;
  double* d_xcs = nullptr;         // [2][chains][E] cs of the step's two evaluations
  double* d_xcells2 = nullptr;     // [chains][S+1][E] eval #2's cells (allocated on first use)
  size_t cap_xcells2 = 0;          // its chains
  double* d_xcbuf = nullptr;       // [chains * pairs][exact_plan_doubles] the local optima's c, plan order
  size_t cap_xcbuf = 0;            // its size in doubles (allocated on first use of the stored form)
  // the local optima's c: option "exact_cform" 0 = stored (c = a / b written
  // once per optimum into d_xcbuf, read at every evaluation), 1 = recomputed at
  // every evaluation from the parent's plan-ordered a = (lv - 1) ow (d_xa,
  // written by eval #1's order-weight launch) and lv's bit (d_xbits)
  int exact_cform = 1;
  // the slot form (exact_form 7): one c row set per resident wave of its
  // kernel, [waves][exact_plan_doubles] (allocated with d_xa, one plan part)
  double* d_xsbuf = nullptr;
  size_t cap_xsbuf = 0;
  int exact_xcd = 1;               // option "exact_xcd": XCD-contiguous optimum ranges
  double* d_xa = nullptr;          // [chains][S][exact_plan_doubles]
  size_t cap_xa = 0;               // its size in doubles
  uint32_t* d_xbits = nullptr;     // [S][pw_ns][64] lv bit of parent row k per (slot, lane): bit m, 16 = remainder
  int32_t* d_pwpos = nullptr;      // [E] plan position (u * 17 + m) * 64 + lane of element e
  int exact_persist = 1;           // option "exact_persist": resident waves take optima from a counter
  int* d_xqueue = nullptr;         // its counter (allocated at staging)
  // option "exact_sched": 1 = hand the optima out longest-first by each pair's
  // evaluation count in the chain's previous step (d_xcost [chains][S][S],
  // written by the kernel; d_xorder [optima] built per launch)
  int exact_sched = 1;
  int32_t* d_xcost = nullptr;
  int32_t* d_xorder = nullptr;
  int* d_xhist = nullptr;          // [chains][64] the schedule's per-chain histograms
  size_t cap_xorder = 0;           // optima d_xorder holds (d_xcost: cap_xcells2 chains)
  // option "exact_trace" (diagnostic): each exact local optimum records its
  // start and end time (wall_clock64, 100 MHz) into d_xtrace [optima][2]
  int exact_trace = 0;
  long long* d_xtrace = nullptr;
  size_t cap_xtrace = 0;           // its optima
  int xtrace_n = 0;                // optima the last traced launch recorded

  // worst-case |ll error| of the fixed-point kernels (nemo_host.h):
  // fx_colsum[k] = sum_e min(colbits_e, k) over the staged D1 bits; auto takes
  // a fixed-point kernel only while its bound stays within err_budget
  std::vector<double> fx_colsum;
  double err_budget = 1e-7;        // option "err_budget" (nemo_set_option_f64)

  // InverseMethod pair schedule (levels), cached per batch of orders
  host::InverseSchedule inv;
  int32_t* d_inv_list = nullptr;
  size_t inv_list_cap = 0;

  // grouped (reuse) evaluation scratch
  int cap_group_batch = 0;
  int32_t* d_grows = nullptr;
  double* d_gsw = nullptr;
  int32_t* d_gcnt = nullptr;

  // pinned host staging of the host-pointer entry points (hipHostMalloc):
  // pageable hipMemcpyAsync blocks the host ~0.1 ms per 512 KB, a memcpy into
  // pinned memory plus a DMA copy costs a fraction of that
  // slot 0: the synchronous nemo_optimal_weights; slots 1 and 2: the queued
  // calls (nemo_optimal_weights_begin), two in flight so the library thread
  // stages the next call while the device runs the previous one
  static constexpr int kStepSlots = 3;
  void* h_stage[kStepSlots] = {};
  size_t h_stage_bytes[kStepSlots] = {};
  // device mirror of the staging layout of nemo_optimal_weights (one copy each way)
  void* d_step[kStepSlots] = {};
  size_t d_step_bytes[kStepSlots] = {};
  hipEvent_t step_done[kStepSlots] = {};  // recorded after a slot's D2H copy
  int step_np2[kStepSlots] = {};   // the slot's queued step: eval #2's partials per chain (host sums)

  // hipGraphs of nemo_optimal_weights' device work (one H2D copy, the
  // launches, one D2H copy) per (nchains, cap, sig0, sig1); graph_epoch moves
  // whenever a captured argument may change (buffers, options, staging)
  struct StepGraph {
    int nchains = -1, cap = -1, slot = -1;
    int np2 = 0;                   // eval #2's partials per chain left for the host (0: ll_dag on device)
    double sig0 = 0.0, sig1 = 0.0;
    bool from_w = false;           // nemo_optimal_weights_w: ancestor_x made on the device
    bool want_prep = false;        // ... and W~ / ancestor_x copied back
    uint64_t epoch = 0;
    hipGraphExec_t exec = nullptr;
  };
  int graphs = 1;                  // option "graphs": replay the fused step as a hipGraph
  int step_host_sum = 1;           // option "step_host_sum": the staged step sums eval #2's partials on the host
  uint64_t graph_epoch = 1;
  static constexpr int kStepGraphs = 8;
  StepGraph step_graph[kStepGraphs];
  int step_graph_next = 0;

  // timing of the score kernel (timing_kernel 0) or of the exact local
  // optima's kernel (1; option "timing_kernel")
  bool timing = false;
  int timing_kernel = 0;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  int launches = 0;
  double timed_ms = 0.0;

  int ntiles() const { return (E + kTileCols - 1) / kTileCols; }
};

// A staging copy on the context's own stream, finished on return (so the host
// buffer may be freed or read): never on HIP's legacy stream, whose
// operations HIP refuses while a blocking stream of the process captures, and
// ordered with the staging kernels on c.stream
inline hipError_t copy_sync(const Ctx& c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
  const hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, c.stream);
  return e != hipSuccess ? e : hipStreamSynchronize(c.stream);
}

// the partial buffer the score kernels write (Ctx::part_out over d_fpartial)
inline double* fpartial(const Ctx& c) { return c.part_out ? c.part_out : c.d_fpartial; }

// fact_kernel 20: bytes of one evaluation's prep image (G split [2][SPAD]
// int, perm [SPAD] int, digits [7][SPAD][64] bytes) and its buffer for the
// reserved batch (allocated when the option is set or the batch grows)
inline size_t i8img_bytes(int spad) { return (size_t)spad * 460; }
hipError_t i8img_reserve(Ctx& c);

// ---- launchers (nemo_kernels.hip); all enqueue on `st` and never allocate ----
// exp() of the staged table (in place conversion from fp64 host layout)
hipError_t launch_exp_table(Ctx& c, const double* d_T64, hipStream_t st);
// staging from the knockdown matrix (nemo_stage.hip): d_D [S][E] bytes in
// {0,1}, d_chains [2][S+1] = (0 + k A, B + k A); writes d_U64 (S+1 rows), d_U
// and d_eT
hipError_t launch_knockdown_tables(Ctx& c, const uint8_t* d_D, const double* d_chains, double A,
                                   double B, hipStream_t st);
hipError_t launch_prep(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                       int32_t* d_rows, double* d_sw, int32_t* d_cnt, int32_t* d_pairs,
                       hipStream_t st, int32_t* d_info = nullptr);
hipError_t launch_score(Ctx& c, int batch, const int32_t* d_rows, const double* d_sw,
                        const int32_t* d_cnt, double* d_ll, double* d_cs, double* d_cells,
                        double* d_ow, hipStream_t st);
hipError_t launch_prep_group(Ctx& c, int batch, int group, int cap, const int32_t* d_pos,
                             const double* d_w01, hipStream_t st);
hipError_t launch_score_group(Ctx& c, int batch, int group, double* d_ll, hipStream_t st);
hipError_t launch_lse(Ctx& c, int rows, const double* d_cells, double* d_ll, double* d_cs,
                      double* d_ow, hipStream_t st);
// fin: when fin_ll is set, the launch also sums the fin_n partials per
// evaluation of fin_batch evaluations into fin_ll (finalize_factored_kernel's
// work, in blocks appended to the grid: one launch less in the fused step)
struct FinalizeArgs {
  const double* partial = nullptr;
  int n = 0, batch = 0;
  double* ll = nullptr;
};
hipError_t launch_local_opt_pairs(Ctx& c, int nchains, int npairs, const int32_t* d_pairs,
                                  const int32_t* d_rows, const double* d_w01, const double* d_anc,
                                  const double* d_ow, double sig0, double sig1, double* d_wnew,
                                  double* d_wdag, int32_t* d_info, hipStream_t st,
                                  FinalizeArgs fin = FinalizeArgs{});
// prod: the objective as one log of a product per lane (every factor 1 + c e,
// e in (0, 1), within [1e-30, 1e30]; the caller checks)
hipError_t launch_local_opt_generic(Ctx& c, int n, const double* d_c, const double* d_anc,
                                    const double* d_x0, double* d_out, bool prod, hipStream_t st);

// the reference's arithmetic (nemo_exact.hip): supported for this staging?
bool exact_supported(const Ctx& c);
size_t exact_plan_doubles(const Ctx& c);   // one plan-ordered row set (per optimum / per parent row)
size_t exact_slot_doubles(const Ctx& c);   // the slot form's row sets: its resident waves x one row set
// the local optima recompute c from the parents' a rows (option exact_cform 1,
// and always for a plan in two parts, which the stored rows do not serve)
inline bool exact_rc(const Ctx& c) { return c.exact_cform == 1 || c.pw_parts > 1; }
// eval in the reference's order: cells into d_cells [batch][S+1][E] (with
// want_ow: replaced by the order weights), cs into d_cs [batch][E], ll into
// d_ll (nullable: left to the caller)
// d_xa (with want_ow): also a = (lv - 1) ow of rows 0..S-1 in plan order
// (cap: the parent-set cap, 0 none, as the score kernels)
hipError_t launch_exact_eval(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01, double* d_cells,
                             double* d_cs, double* d_ll, bool want_ow, hipStream_t st, double* d_xa = nullptr);
// every permissible pair's exact local optimum; the appended blocks sum d_cs1
// into d_ll1 (eval #1's ll) when d_ll1 is set
hipError_t launch_local_opt_exact(Ctx& c, int nchains, int npairs, const int32_t* d_pairs, const double* d_w01,
                                  const double* d_anc, const double* d_ow, double sig0, double sig1, double* d_wnew,
                                  double* d_wdag, int32_t* d_info, const double* d_cs1, double* d_ll1,
                                  hipStream_t st);

// nemo_local_opt in the reference's arithmetic (out [n][3] as local_opt_generic)
hipError_t launch_local_opt_exact_generic(Ctx& c, int n, const double* d_c, const double* d_anc, const double* d_x0,
                                          double* d_out, hipStream_t st);
// refmath.h on the device, for the tests (nemo_refmath_probe)
hipError_t launch_refmath_probe(int fn, int n, const double* d_x, const double* d_y, double* d_out, hipStream_t st);

// number of (child, parent) pairs per chain for a given cap
int pairs_per_chain(int S, int cap);

// factored MFMA path (nemo_factored.hip)
int factored_spad(int S);
int factored_partials(const Ctx& c);
// the partials per evaluation the kernel fact_kernel `fk` (resolved) writes:
// each launcher's own formula, known before anything is launched, so a
// caller that redirects them (Ctx::part_out) checks its buffer first
int score_partials(const Ctx& c, int fk);
// 16-effect tiles per partial of score_i8w_kernel
constexpr int kWideSetT = 2;
// int8 matrix-core factored path (nemo_factored_i8.hip), S <= 64, ll only:
// one kernel (digits of Delta built in LDS + score); partials per 8-tile set
// (*finalized: ll already written -- one block per evaluation -- else the
// caller sums the nparts partials per evaluation with sum_partials' order)
hipError_t launch_score_i8(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                           double* d_ll, int np, int waves, hipStream_t st, int* nparts,
                           bool* finalized);
// the same with the offset log-sum-exp (c.i8o_ok), waves 4 or 8 per block;
// l2: the log2 fixed-point epilogue (c.i8l_ok)
hipError_t launch_score_i8o(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                            double* d_ll, int waves, bool l2, hipStream_t st, int* nparts,
                            bool* finalized);
// the log2 kernel for 64 < S <= 128 (c.i8w_ok): one block per evaluation,
// ll written in-kernel (*finalized)
hipError_t launch_score_i8w(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                            double* d_ll, bool two, hipStream_t st, int* nparts, bool* finalized);
hipError_t stage_i8o(Ctx& c, const std::vector<double>& elo, const std::vector<double>& ehi,
                     const std::vector<uint64_t>& d1);
// capped lookup-table kernel (nemo_window.hip): ll only, 1 <= cap <= kWinMaxCap,
// S <= kWinMaxS; one partial per 64-effect word (*nparts = nwords)
hipError_t launch_score_window(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                               double* d_ll, hipStream_t st, int* nparts, bool* finalized,
                               bool walk_lds = false);
hipError_t stage_window(Ctx& c, const std::vector<double>& elo, const std::vector<double>& ehi,
                        const std::vector<uint64_t>& d1);

// log(x) for finite x > 0 (normal): x = 2^k m, m in [1, 2); table entry j
// (top 7 fraction bits) holds inv_j ~ 1/(1 + (j + 0.5)/128) and L_j =
// -log(inv_j), so log x = k ln2 + L_j + log1p(m inv_j - 1), |m inv_j - 1| <
// 1/254, degree-6 series.  Within ~1 ulp of max(|log x|, 0.5) (restated and
// checked against a 120-bit reference in tests/test_numerics.py); 11 f64 + 5
// integer VALU and one LDS read, against ~45 VALU for the general log.
__device__ __forceinline__ double log_fast(double x, const double2* __restrict__ ltab) {
  constexpr double kLn2Hi = 0x1.62e42fefa3800p-1;  // 42 bits: k * kLn2Hi exact
  constexpr double kLn2Lo = 5.4956039718945254e-14;
  const uint64_t bits = __builtin_bit_cast(uint64_t, x);
  const uint32_t hi = (uint32_t)(bits >> 32);
  const int k = (int)((hi >> 20) & 0x7ff) - 1023;
  const double m = __builtin_bit_cast(double, (bits & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
  const double2 tj = ltab[(hi >> 13) & 127];
  const double r = fma(m, tj.x, -1.0);
  double p = fma(r, -1.0 / 6.0, 0.2);
  p = fma(r, p, -0.25);
  p = fma(r, p, 1.0 / 3.0);
  p = fma(r, p, -0.5);
  p = fma(r, p, 1.0);
  p *= r;
  const double kd = (double)k;
  return fma(kd, kLn2Hi, tj.y) + fma(kd, kLn2Lo, p);
}

// Cross-lane sums of a double without the LDS (DPP moves and permlane swaps are
// VALU; __shfl_xor goes through ds_bpermute).
// DPP move of a double (both dwords), dpp_ctrl CTRL over all rows / banks
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)b, CTRL, 0xf, 0xf, false);
  const uint32_t hi = __builtin_amdgcn_update_dpp(0u, (uint32_t)(b >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// sum over the four 16-lane rows (lanes col, col+16, col+32, col+48), in
// every lane: v_permlane16_swap then v_permlane32_swap (both outputs kept)
__device__ __forceinline__ double rowsum4(double v) {
  uint64_t b = __builtin_bit_cast(uint64_t, v);
  auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)b, (uint32_t)b, false, false);
  auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
  double a0 = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
  double a1 = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
  v = a0 + a1;
  b = __builtin_bit_cast(uint64_t, v);
  lo = __builtin_amdgcn_permlane32_swap((uint32_t)b, (uint32_t)b, false, false);
  hi = __builtin_amdgcn_permlane32_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
  a0 = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
  a1 = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
  return a0 + a1;
}

// the column sums of two 16 x 16 tiles at once (lane = column + 16 row
// group; a and b: each lane's sum over its rows of tile a / tile b): after
// it, rows 0 and 2 of the wave hold tile a's sum over the four row groups
// and rows 1 and 3 tile b's.  v_permlane16_swap(a, b) exchanges a's odd rows
// with b's even rows, so out[0] + out[1] = (a0 + a1, b0 + b1, a2 + a3, b2 + b3)
// by row; one v_permlane32_swap adds rows 0 + 2 and 1 + 3.  Six VALU for two
// tiles against ten per tile for rowsum4.
__device__ __forceinline__ double rowsum_pair(double a, double b) {
  const uint64_t x = __builtin_bit_cast(uint64_t, a), y = __builtin_bit_cast(uint64_t, b);
  auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)x, (uint32_t)y, false, false);
  auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(x >> 32), (uint32_t)(y >> 32), false, false);
  const double v = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]) +
                   __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
  const uint64_t z = __builtin_bit_cast(uint64_t, v);
  lo = __builtin_amdgcn_permlane32_swap((uint32_t)z, (uint32_t)z, false, false);
  hi = __builtin_amdgcn_permlane32_swap((uint32_t)(z >> 32), (uint32_t)(z >> 32), false, false);
  return __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]) +
         __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
}

// sum over the wave in every lane, all VALU: quad xor 1 and 2 (quad_perm),
// the 8-lane and 16-lane mirrors, then the permlane swaps across rows
__device__ __forceinline__ double wsum_dpp(double v) {
  v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);  // row_half_mirror
  v += dpp_d<0x140>(v);  // row_mirror
  return rowsum4(v);
}

// sum over each 16-lane row, in every lane of the row (wsum_dpp's first four
// stages): 12 VALU against ~50 for a 64-lane ds_bpermute tree
__device__ __forceinline__ double rowsum16(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  v += dpp_d<0x141>(v);
  v += dpp_d<0x140>(v);
  return v;
}

// the 128-entry table of log_fast (2 KB of LDS), filled by a block
__device__ __forceinline__ void fill_log_table(double2* ltab, int tid, int nthreads) {
  for (int k = tid; k < 128; k += nthreads) {
    const double inv = 1.0 / (1.0 + ((double)k + 0.5) * (1.0 / 128.0));
    ltab[k] = double2{inv, -log(inv)};
  }
}

// ---- the per-evaluation prep shared by prep_kernel and step_prep_kernel ----
// the evaluation's order in LDS (block of >= S threads): perm[p] = the node
// at position p; with want_scan, scan[i] = inclusive prefix sum of the list
// lengths of children 0..i (Hillis-Steele).  Malformed positions are clamped
// (they must not fault; the host rejects them first).
__device__ __forceinline__ void prep_order_lds(int S, int cap, const int32_t* __restrict__ pb, int* perm,
                                               int* scan, bool want_scan) {
  const int tid = threadIdx.x;
  if (tid < S) perm[tid] = 0;
  __syncthreads();
  if (tid < S) {
    int p = pb[tid];
    p = p < 0 ? 0 : (p >= S ? S - 1 : p);
    perm[p] = tid;
    const int lo = (cap > 0 && p > cap) ? p - cap : 0;
    scan[tid] = p - lo;  // list length of child tid
  }
  __syncthreads();
  if (want_scan) {
    for (int o = 1; o < S; o <<= 1) {
      const int v = (tid < S && tid >= o) ? scan[tid - o] : 0;
      __syncthreads();
      if (tid < S) scan[tid] += v;
      __syncthreads();
    }
  }
}

// one wave: child i's permissible parents in pi order (nem_order_mcmc.py:
// 62-65; with cap, the last `cap` of them), their weights, the list length,
// the child's slots of the flat pair list (when pairs: i << 16 | parent
// node, in list order), and -1 in every entry
// of its info row (when info: "not a permissible pair"; the local optima
// overwrite theirs)
__device__ __forceinline__ void prep_child_list(int S, int cap, const int32_t* __restrict__ pb,
                                                const double* __restrict__ w01, int32_t* __restrict__ rows,
                                                double* __restrict__ sw, int32_t* __restrict__ cnt,
                                                int32_t* __restrict__ pairs, int32_t* __restrict__ info, int b,
                                                int i, const int* perm, const int* scan, int lane) {
  int pi = pb[i];
  pi = pi < 0 ? 0 : (pi >= S ? S - 1 : pi);
  const int lo = (cap > 0 && pi > cap) ? pi - cap : 0;
  const int n = pi - lo;
  const size_t row = ((size_t)b * S + i) * S;
  int32_t* r = rows + row;
  double* w = sw + row;
  const double* wr = w01 + row;
  int32_t* pr = pairs ? pairs + (size_t)b * S * S + (scan[i] - n) : nullptr;
  if (info)
    for (int t = lane; t < S; t += kWave) info[row + t] = -1;
  for (int t = lane; t < n; t += kWave) {
    const int j = perm[lo + t];
    r[t] = j;
    w[t] = wr[j];
    if (pr) pr[t] = (i << 16) | j;  // the parent node itself: no rows[] lookup in the consumers
  }
  if (lane == 0) cnt[(size_t)b * S + i] = n;
}

// fixed-order sum of n partials by one wave: strided lane sums, then an xor
// tree (finalize_factored_kernel and the int8 kernel's own finalize share it,
// so both paths give identical bits)
__device__ __forceinline__ double sum_partials(const double* __restrict__ p, int n, int lane) {
  double s = 0.0;
  for (int t = lane; t < n; t += kWave) s += p[t];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, kWave);
  return s;
}
// fixed-order optimizers of methods.py (nemo_methods.hip)
hipError_t launch_gamma_pairs(Ctx& c, int nprob, int npairs, const int32_t* d_pairs, const int32_t* d_rows,
                              const double* d_w, const double* d_ow, double* d_wout, int32_t* d_info,
                              hipStream_t st);
hipError_t launch_ancestral(Ctx& c, int nprob, const int32_t* d_pos, const double* d_w, double* d_out,
                            hipStream_t st);
// one level of InverseMethod.opt_b's pair loop (list entries prob << 16 | i << 8 | k),
// then the commit of the level's optima into d_w
hipError_t launch_inverse_level(Ctx& c, int n, const int32_t* d_list, const int32_t* d_pos, double* d_w,
                                const double* d_ow, double* d_xout, int32_t* d_info, hipStream_t st);
// prepped: Delta / G / perm of the batch are already staged (step_prep_kernel);
// defer_np: when set, the per-evaluation partials are left unsummed and
// *defer_np = their count (0 if the kernel summed them itself)
hipError_t launch_score_factored(Ctx& c, int batch, int cap, const int32_t* d_pos,
                                 const double* d_w01, double* d_ll, double* d_cs, double* d_cells,
                                 double* d_ow, hipStream_t st, bool prepped = false,
                                 int* defer_np = nullptr);
// the fused step's prep in ONE launch: prep_kernel's parent and pair lists
// with the info rows preset to -1, and prep_factored_kernel's Delta / G / perm
hipError_t launch_step_prep(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                            int32_t* d_info, hipStream_t st);
// the fact_kernel value a factored call takes (the option, or what auto
// resolves to for this cap / output set), with the worst-case |ll error| of
// its fixed-point arithmetic (0 for the fp64 kernels); -1 if none applies
int resolve_fact_kernel(const Ctx& c, int cap, bool ll_only, double* bound);
// the step's W~ and ancestor_x from W on the device, in scipy's bits
// (nemo_ancestor.hip; S <= 64): d_w01 = expit on the permissible entries (cap
// as for the step), d_anc = clip(inv(I - W~) - I, 0, 1), d_flag [nchains]: 1
// singular, 2 non-finite I - W~, 4 non-finite factors (the host recomputes)
bool ancestor_supported(const Ctx& c);
hipError_t launch_ancestor(Ctx& c, int nchains, int cap, const int32_t* d_pos, const double* d_w, double* d_w01,
                           double* d_anc, int32_t* d_flag, hipStream_t st);
// W~ alone (d_w01), for a step whose ancestor_x runs on a second stream
// (launch_ancestor with d_w01 null)
hipError_t launch_w01(Ctx& c, int nchains, int cap, const int32_t* d_pos, const double* d_w, double* d_w01,
                      hipStream_t st);

}  // namespace nemo
