// nemo_abi.cpp -- the C-ABI (include/nemo.h): context lifetime, staging,
// argument checking, host<->device transfers and launch sequencing.
// No arithmetic of the hot path lives here; it is all in nemo_kernels.hip.
#include "nemo.h"
#include "nemo_internal.h"
#include "refmath.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

using nemo::Ctx;

// one queued nemo_optimal_weights call (nemo_optimal_weights_begin)
struct StepJob {
  int nchains, cap;
  const int32_t* pos;
  const double *w01, *anc;
  double sig0, sig1;
  double *w_new, *ll1, *ll_dag;
  int32_t* info;
  // nemo_optimal_weights_w_begin: W in, W~ / ancestor_x / flags out
  const double* w_in = nullptr;
  double *w01_out = nullptr, *anc_out = nullptr;
  int32_t* aflag = nullptr;
  int rc = 0;
  std::string err;
  int slot = 0;  // staging slot while in flight
};

struct nemo_ctx {
  Ctx c;
  // the asynchronous fused step: a library thread runs the queued calls in
  // submission order; the caller collects them in the same order
  // (nemo_host.h StepQueue; created on the first _begin)
  std::unique_ptr<nemo::host::StepQueue<StepJob>> steps;
  // option "exact_dev": nemo_score_dev in the reference's arithmetic
  int exact_dev = 0;
};

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

// A HIP failure's message, with the process's FIRST HIP failure beside it when
// this one differs: an asynchronous fault sticks and is then reported by every
// later call under its own name (a capture conflict resurfaced as "invalid
// device ordinal"), so the first failure is what names the cause
int fail_hip(const char* what, hipError_t e) {
  static std::mutex mu;
  static std::string first;
  std::string cur = std::string(what) + " failed: " + hipGetErrorString(e);
  {
    std::lock_guard<std::mutex> g(mu);
    if (first.empty()) first = cur;
    else if (first != cur) cur += " (the first HIP error in this process: " + first + ")";
  }
  return fail(NEMO_ERR_HIP, "%s", cur.c_str());
}

#define HIPCHK(expr)                                    \
  do {                                                  \
    hipError_t e_ = (expr);                             \
    if (e_ != hipSuccess) return fail_hip(#expr, e_);   \
  } while (0)

// One process-wide lock around graph capture and the calls that still use the
// legacy stream or resize a context's buffers under a running step (reserve,
// context create / destroy, the probes): HIP refuses a legacy-stream operation
// while a stream captures ("would make the legacy stream depend on a
// capturing blocking stream"), and the error then sticks to the next launch.
// Staging holds no lock: its transfers run on the context's own stream
// (tests/test_gpu_parity.py::test_staging_while_another_engine_captures)
std::recursive_mutex& api_mutex() {
  static std::recursive_mutex m;
  return m;
}
#define NEMO_API_LOCK std::lock_guard<std::recursive_mutex> nemo_api_lock_(api_mutex())

template <class T>
hipError_t dalloc(T** p, size_t n) {
  if (*p) {
    hipError_t fe = hipFree(*p);
    *p = nullptr;
    if (fe != hipSuccess) return fe;
  }
  if (n == 0) n = 1;
  return hipMalloc((void**)p, n * sizeof(T));
}

int check_ctx(nemo_ctx* ctx, bool need_staged) {
  if (!ctx) return fail(NEMO_ERR_ARG, "null context");
  if (need_staged && !ctx->c.staged) return fail(NEMO_ERR_STATE, "tables not staged");
  HIPCHK(hipSetDevice(ctx->c.device));
  return NEMO_OK;
}

// every row of pos must be a permutation of 0..S-1
int check_pos(const int32_t* pos, int batch, int S) {
  const int b = nemo::host::first_bad_pos_row(pos, batch, S);
  if (b >= 0) return fail(NEMO_ERR_ARG, "pos[%d] is not a permutation of 0..%d", b, S - 1);
  return NEMO_OK;
}

// *_dev entry points run on the caller's stream verbatim: NULL is HIP's null
// stream (torch's default stream), as in the HIP API itself
hipStream_t pick(nemo_ctx*, void* stream) { return (hipStream_t)stream; }

bool step_exact(const Ctx& c, int);
int exact_reserve(Ctx& c, int nchains);

}  // namespace

extern "C" {

const char* nemo_last_error(void) { return g_err.c_str(); }

int nemo_version(void) { return 10000; }

int nemo_device_count(int* count) {
  if (!count) return fail(NEMO_ERR_ARG, "null count");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return NEMO_OK;
}

int nemo_ctx_create(int device, int num_s, int num_e, int dtype, nemo_ctx** out) {
  NEMO_API_LOCK;
  if (!out) return fail(NEMO_ERR_ARG, "null out");
  *out = nullptr;
  if (num_s < 2 || num_s > nemo::kMaxS)
    return fail(NEMO_ERR_ARG, "num_s=%d outside [2, %d]", num_s, nemo::kMaxS);
  if (num_e < 1) return fail(NEMO_ERR_ARG, "num_e=%d < 1", num_e);
  if (dtype != NEMO_F64 && dtype != NEMO_F32) return fail(NEMO_ERR_ARG, "dtype=%d", dtype);
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return fail(NEMO_ERR_HIP, "no HIP device visible (the engine has no CPU fallback)");
  if (device < 0 || device >= n) return fail(NEMO_ERR_ARG, "device %d of %d", device, n);
  HIPCHK(hipSetDevice(device));
  nemo_ctx* ctx = new nemo_ctx();
  ctx->c.device = device;
  ctx->c.S = num_s;
  ctx->c.E = num_e;
  ctx->c.dtype = dtype;
  hipError_t e = hipStreamCreateWithFlags(&ctx->c.stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete ctx;
    return fail(NEMO_ERR_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  *out = ctx;
  return NEMO_OK;
}

void nemo_ctx_destroy(nemo_ctx* ctx) {
  if (!ctx) return;
  // every queued step still runs (its caller's buffers are written), then the
  // step thread ends; steps not collected with _end are dropped
  if (ctx->steps) ctx->steps->shutdown();
  NEMO_API_LOCK;
  Ctx& c = ctx->c;
  // teardown is best effort: a failure here has no caller left to report to
  (void)hipSetDevice(c.device);
  (void)hipStreamSynchronize(c.stream);
  void* bufs[] = {c.d_eT,   c.d_U,    c.d_pos,  c.d_w01,  c.d_anc,     c.d_rows, c.d_sw,
                  c.d_cnt,  c.d_pairs, c.d_partial, c.d_ll, c.d_ll2, c.d_cs, c.d_ow,
                  c.d_wnew, c.d_wdag, c.d_info, c.d_c,    c.d_grows, c.d_gsw,  c.d_gcnt,
                  c.d_D1w,  c.d_elo,  c.d_ehi,  c.d_U64,  c.d_fDp,  c.d_fG,  c.d_fperm,
                  c.d_fpartial, c.d_B8, c.d_inv_list, c.d_Uoff, c.d_nullsum, c.d_i8o_tabs,
                  c.d_udig, c.d_udig2, c.d_u0, c.d_wuw, c.d_wnull, c.d_nullsum_w, c.d_i8img,
                  c.d_xlo,  c.d_xhi,  c.d_pwplan, c.d_xcs, c.d_xcells2, c.d_xcbuf,
                  c.d_xa,   c.d_xbits, c.d_pwpos, c.d_pwmeta, c.d_xtrace, c.d_xqueue,
                  c.d_xcost, c.d_xorder, c.d_xhist, c.d_xsbuf};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  for (int k = 0; k < Ctx::kStepSlots; ++k) {
    if (c.h_stage[k]) (void)hipHostFree(c.h_stage[k]);
    if (c.d_step[k]) (void)hipFree(c.d_step[k]);
    if (c.step_done[k]) (void)hipEventDestroy(c.step_done[k]);
  }
  for (hipEvent_t ev : c.ev_pool) (void)hipEventDestroy(ev);
  for (auto& g : c.step_graph)
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
  (void)hipStreamDestroy(c.stream);
  if (c.stream2) (void)hipStreamDestroy(c.stream2);
  if (c.ev_fork) (void)hipEventDestroy(c.ev_fork);
  if (c.ev_join) (void)hipEventDestroy(c.ev_join);
  delete ctx;
}

int nemo_reserve(nemo_ctx* ctx, int max_batch, int max_chains) {
  NEMO_API_LOCK;
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  if (max_batch < 0 || max_chains < 0) return fail(NEMO_ERR_ARG, "negative capacity");
  Ctx& c = ctx->c;
  const size_t S = c.S, E = c.E;
  const int nb = std::max({max_batch, max_chains, 1});
  if (nb > c.cap_batch) {
    ++c.graph_epoch;
    HIPCHK(hipStreamSynchronize(c.stream));
    HIPCHK(dalloc(&c.d_pos, nb * S));
    HIPCHK(dalloc(&c.d_w01, nb * S * S));
    HIPCHK(dalloc(&c.d_rows, nb * S * S));
    HIPCHK(dalloc(&c.d_sw, nb * S * S));
    HIPCHK(dalloc(&c.d_cnt, nb * S));
    HIPCHK(dalloc(&c.d_partial, nb * (size_t)c.ntiles()));
    HIPCHK(dalloc(&c.d_ll, nb));
    HIPCHK(dalloc(&c.d_cs, nb * E));
    HIPCHK(dalloc(&c.d_ow, nb * (S + 1) * E));
    const size_t sp = nemo::factored_spad(c.S);
    HIPCHK(dalloc(&c.d_fDp, nb * sp * sp));
    HIPCHK(dalloc(&c.d_fG, nb * sp));
    HIPCHK(dalloc(&c.d_fperm, nb * sp));
    HIPCHK(dalloc(&c.d_fpartial, nb * (size_t)nemo::factored_partials(c)));
    c.cap_batch = nb;
    if (c.fact_kernel == 20) HIPCHK(nemo::i8img_reserve(c));
  }
  const int nc = std::max(max_chains, 1);
  if (nc > c.cap_chains) {
    ++c.graph_epoch;
    HIPCHK(hipStreamSynchronize(c.stream));
    HIPCHK(dalloc(&c.d_anc, nc * S * S));
    HIPCHK(dalloc(&c.d_pairs, nc * S * S));
    HIPCHK(dalloc(&c.d_ll2, nc));
    HIPCHK(dalloc(&c.d_wnew, nc * S * S));
    HIPCHK(dalloc(&c.d_wdag, nc * S * S));
    HIPCHK(dalloc(&c.d_info, nc * S * S));
    HIPCHK(dalloc(&c.d_xcs, 2 * nc * E));
    c.cap_chains = nc;
  }
  // the exact step's own buffers too, so nemo_optimal_weights_dev never
  // allocates (or synchronises) once this returned -- a caller may capture it
  if (max_chains > 0 && c.staged && step_exact(c, 0)) return exact_reserve(c, nc);
  return NEMO_OK;
}

}  // extern "C"

namespace {

// grow staging slot `slot` (pinned host buffer and its device mirror) to at
// least `bytes`
int step_stage(Ctx& c, int slot, size_t bytes) {
  if (!c.step_done[slot]) HIPCHK(hipEventCreateWithFlags(&c.step_done[slot], hipEventDisableTiming));
  if (bytes <= c.h_stage_bytes[slot] && bytes <= c.d_step_bytes[slot]) return NEMO_OK;
  NEMO_API_LOCK;
  ++c.graph_epoch;
  HIPCHK(hipStreamSynchronize(c.stream));
  if (c.h_stage[slot]) HIPCHK(hipHostFree(c.h_stage[slot]));
  if (c.d_step[slot]) HIPCHK(hipFree(c.d_step[slot]));
  c.h_stage[slot] = c.d_step[slot] = nullptr;
  c.h_stage_bytes[slot] = c.d_step_bytes[slot] = 0;
  HIPCHK(hipHostMalloc(&c.h_stage[slot], bytes, hipHostMallocDefault));
  c.h_stage_bytes[slot] = bytes;
  HIPCHK(hipMalloc(&c.d_step[slot], bytes));
  c.d_step_bytes[slot] = bytes;
  return NEMO_OK;
}

// (re)allocate the table buffers of a staging: exp(T) and U in the table
// dtype, U in fp64 padded to the factored row blocking (the int8 kernel reads
// padding rows unclamped, their G hides them) plus one zeroed 16-effect tile
// (the factored kernels read whole tiles; lanes past E are masked out)
int alloc_tables(Ctx& c) {
  const size_t S = c.S, E = c.E;
  ++c.graph_epoch;
  const size_t esz = c.dtype == NEMO_F64 ? 8 : 4;
  HIPCHK(hipStreamSynchronize(c.stream));
  c.staged = false;
  void** bufs[] = {&c.d_eT, &c.d_U, (void**)&c.d_U64};
  for (void** p : bufs)
    if (*p) {
      HIPCHK(hipFree(*p));
      *p = nullptr;
    }
  HIPCHK(hipMalloc(&c.d_eT, S * S * E * esz));
  HIPCHK(hipMalloc(&c.d_U, (S + 1) * E * esz));
  const size_t urows = std::max(S + 1, (size_t)std::max(nemo::factored_spad(c.S), 0));
  HIPCHK(hipMalloc((void**)&c.d_U64, (urows * E + 16) * 8));
  // on the context's stream, finished before the staging kernels run: c.stream
  // is non-blocking, so a null-stream hipMemset is not ordered before them (it
  // can land after the knockdown kernels wrote U, seen under a shared GPU)
  HIPCHK(hipMemsetAsync(c.d_U64, 0, (urows * E + 16) * 8, c.stream));
  HIPCHK(hipStreamSynchronize(c.stream));
  return NEMO_OK;
}

// the factored form once T's structure is known: every off-diagonal row j is
// shared by all children and takes lo_j or hi_j (bit d1[j][e] = 1: hi_j)
int stage_factored(nemo_ctx* ctx, bool fact, const std::vector<uint64_t>& d1,
                   const std::vector<double>& elo, const std::vector<double>& ehi,
                   const std::vector<double>& tlo, const std::vector<double>& thi) {
  Ctx& c = ctx->c;
  const size_t S = c.S, E = c.E;
  const int nwords = (int)((E + 63) / 64);
  ++c.graph_epoch;
  c.factored = fact;
  c.i8o_ok = false;
  c.win_ok = false;
  c.fspad = nemo::factored_spad(c.S);
  c.nwords = nwords;
  c.fx_colsum.clear();
  if (fact) {
    c.fx_colsum = nemo::host::fixed_point_colsums(c.S, c.E, d1.data(), nwords);
    HIPCHK(dalloc(&c.d_D1w, d1.size()));
    HIPCHK(dalloc(&c.d_elo, S));
    HIPCHK(dalloc(&c.d_ehi, S));
    HIPCHK(nemo::copy_sync(c, c.d_D1w, d1.data(), d1.size() * 8, hipMemcpyHostToDevice));
    HIPCHK(nemo::copy_sync(c, c.d_elo, elo.data(), S * 8, hipMemcpyHostToDevice));
    HIPCHK(nemo::copy_sync(c, c.d_ehi, ehi.data(), S * 8, hipMemcpyHostToDevice));
    // int8 variants (S <= 128): per-model fixed-point scale and the D1 bytes in
    // v_mfma_i32_16x16x64_i8 B-fragment order: K half h (parents 64 h .. 64 h
    // + 63; one half for S <= 64, two for S <= 128), tile t, lane l (effect
    // 16t + (l & 15), parents 64 h + 16 (l >> 4) .. + 15), byte j = parent
    // 64 h + 16 (l >> 4) + j
    if (c.d_B8) HIPCHK(hipFree(c.d_B8));
    c.d_B8 = nullptr;
    if (S <= 128) {
      double dmax = 0.0;
      for (size_t j = 0; j < S; ++j) dmax = std::max(dmax, fabs(log(ehi[j]) - log(elo[j])));
      int ex = 0;
      if (dmax > 0.0) frexp(dmax * (1.0 + 1e-9), &ex);  // dmax * (1 + 1e-9) <= 2^ex
      c.i8_cexp = dmax > 0.0 ? ex + 1 : 0;              // |Delta| <= 2^(c - 1)
      const size_t nt = (E + 15) / 16, kh = S > 64 ? 2 : 1;
      std::vector<uint8_t> b8(kh * nt * 64 * 16, 0);
      for (size_t h = 0; h < kh; ++h)
        for (size_t t = 0; t < nt; ++t)
          for (int l = 0; l < 64; ++l) {
            const size_t e = 16 * t + (l & 15);
            if (e >= E) continue;
            for (int jj = 0; jj < 16; ++jj) {
              const size_t k = 64 * h + 16 * (l >> 4) + jj;
              if (k < S)
                b8[((h * nt + t) * 64 + l) * 16 + jj] = (uint8_t)((d1[k * nwords + e / 64] >> (e % 64)) & 1ull);
            }
          }
      // a second copy scaled by 64 follows (the B operand of the high digit of
      // each pair; the log2 kernels load it instead of shifting per tile)
      const size_t nb = b8.size();
      b8.resize(2 * nb);
      for (size_t k = 0; k < nb; ++k) b8[nb + k] = (uint8_t)(b8[k] << 6);
      HIPCHK(hipMalloc((void**)&c.d_B8, b8.size()));
      HIPCHK(nemo::copy_sync(c, c.d_B8, b8.data(), b8.size(), hipMemcpyHostToDevice));
    }
    HIPCHK(nemo::stage_i8o(c, elo, ehi, d1));
    HIPCHK(nemo::stage_window(c, elo, ehi, d1));
    // the exact path (nemo_exact.hip): numpy's exp of the two values of each
    // row (the reference's local_vec = np.exp(T[i][k]), restated bit for bit)
    // and the wave layout of numpy's pairwise sum of E terms
    c.exact_ok = false;
    c.pw_parts = 1;
    // numpy's pairwise sum of E as wave plans: one, or the two halves of its
    // top split when E needs more than 64 leaf blocks (E > 8192)
    std::vector<nemo::host::PairwisePlan> parts;
    bool plan_ok = nemo::host::build_pairwise_parts(c.E, parts) && parts.size() <= (size_t)nemo::kExactMaxParts;
    for (const auto& p : parts) plan_ok = plan_ok && p.ns <= nemo::kExactMaxSlots && p.nh <= 8;
    if (plan_ok) {
      std::vector<double> xlo(S), xhi(S);
      for (size_t j = 0; j < S; ++j) {
        xlo[j] = nemo::refmath::svml_exp(tlo[j]);
        xhi[j] = nemo::refmath::svml_exp(thi[j]);
      }
      std::vector<int32_t> dev, meta;
      nemo::host::parts_device_rows(parts, dev, meta);
      // the recompute form's element -> plan position map and lv bits per
      // (parent row, slot, lane)
      std::vector<int32_t> ppos;
      std::vector<uint32_t> bits;
      nemo::host::parts_positions(parts, c.E, ppos);
      nemo::host::parts_lv_bits(parts, c.S, d1.data(), nwords, bits);
      HIPCHK(dalloc(&c.d_xlo, S));
      HIPCHK(dalloc(&c.d_xhi, S));
      HIPCHK(dalloc(&c.d_pwplan, dev.size()));
      HIPCHK(dalloc(&c.d_pwmeta, meta.size()));
      HIPCHK(dalloc(&c.d_pwpos, ppos.size()));
      if (!c.d_xqueue) HIPCHK(dalloc(&c.d_xqueue, 1));
      HIPCHK(dalloc(&c.d_xbits, bits.size()));
      HIPCHK(nemo::copy_sync(c, c.d_xlo, xlo.data(), S * 8, hipMemcpyHostToDevice));
      HIPCHK(nemo::copy_sync(c, c.d_xhi, xhi.data(), S * 8, hipMemcpyHostToDevice));
      HIPCHK(nemo::copy_sync(c, c.d_pwplan, dev.data(), dev.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(nemo::copy_sync(c, c.d_pwmeta, meta.data(), meta.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(nemo::copy_sync(c, c.d_pwpos, ppos.data(), ppos.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(nemo::copy_sync(c, c.d_xbits, bits.data(), bits.size() * 4, hipMemcpyHostToDevice));
      c.pw_ns = nemo::host::parts_slots(parts);
      c.pw_parts = (int)parts.size();
      c.pw_nh = parts[0].nh;
      c.pw_maxrem = parts[0].maxrem;
      c.exact_ok = true;
    }
  }
  // grow the factored scratch if a batch was reserved before staging
  if (c.cap_batch > 0) {
    const int nb = c.cap_batch;
    c.cap_batch = 0;
    int rc2 = nemo_reserve(ctx, nb, 0);
    if (rc2) return rc2;
  }
  c.staged = true;
  // a chain reservation made before this staging covers the exact step too
  if (c.cap_chains > 0 && step_exact(c, 0)) return exact_reserve(c, c.cap_chains);
  return NEMO_OK;
}

}  // namespace

extern "C" {

// Staging takes no process-wide lock: its copies and fills run on the
// context's own non-blocking stream (nemo::copy_sync), so they neither touch
// the legacy stream nor wait for another engine's capture
// (tests/test_gpu_parity.py::test_staging_while_another_engine_captures)
int nemo_stage_tables(nemo_ctx* ctx, const double* U, const double* T) {
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  if (!U || !T) return fail(NEMO_ERR_ARG, "null table");
  Ctx& c = ctx->c;
  const size_t S = c.S, E = c.E, n = S * S * E;
  // range of the off-diagonal rows (the ones the score reads)
  double amax = 0.0;
  for (size_t i = 0; i < S; ++i)
    for (size_t j = 0; j < S; ++j) {
      if (i == j) continue;
      const double* r = T + (i * S + j) * E;
      for (size_t e = 0; e < E; ++e) {
        const double v = r[e];
        if (!isfinite(v)) return fail(NEMO_ERR_ARG, "T[%zu][%zu][%zu] is not finite", i, j, e);
        amax = std::max(amax, fabs(v));
      }
    }
  const double lim = c.dtype == NEMO_F64 ? 170.0 : 20.0;
  if (amax > lim)
    return fail(NEMO_ERR_ARG, "|T| up to %g exceeds the %s product range (%g)", amax,
                c.dtype == NEMO_F64 ? "f64" : "f32", lim);
  for (size_t k = 0; k < (S + 1) * E; ++k)
    if (isnan(U[k])) return fail(NEMO_ERR_ARG, "U has NaN");
  if ((rc = alloc_tables(c))) return rc;
  double* d_t64 = nullptr;
  HIPCHK(hipMalloc((void**)&d_t64, n * sizeof(double)));
  HIPCHK(hipMemcpyAsync(d_t64, T, n * sizeof(double), hipMemcpyHostToDevice, c.stream));
  HIPCHK(nemo::launch_exp_table(c, d_t64, c.stream));
  if (c.dtype == NEMO_F64) {
    HIPCHK(hipMemcpyAsync(c.d_U, U, (S + 1) * E * 8, hipMemcpyHostToDevice, c.stream));
  } else {
    std::vector<float> u32((S + 1) * E);
    for (size_t k = 0; k < u32.size(); ++k) u32[k] = (float)U[k];
    HIPCHK(hipMemcpyAsync(c.d_U, u32.data(), u32.size() * 4, hipMemcpyHostToDevice, c.stream));
    HIPCHK(hipStreamSynchronize(c.stream));
  }
  HIPCHK(hipStreamSynchronize(c.stream));
  HIPCHK(hipFree(d_t64));
  HIPCHK(nemo::copy_sync(c, c.d_U64, U, (S + 1) * E * 8, hipMemcpyHostToDevice));
  c.table_absmax = amax;

  // factored form: every off-diagonal row T[.][j] identical for all children
  // and two-valued (nem.py:44-46 builds exactly that); lo_j = its first value
  std::vector<uint64_t> d1;
  std::vector<double> elo, ehi, tlo, thi;
  bool fact = nemo::host::detect_factored(c.S, c.E, T, d1, elo, ehi, &tlo, &thi);
  if (!fact) d1.assign((size_t)S * ((E + 63) / 64), 0ull);
  // the factored kernels' exp takes finite arguments: U must be finite too
  for (size_t k = 0; k < (S + 1) * E && fact; ++k)
    if (!isfinite(U[k]) || fabs(U[k]) > 1e9) fact = false;
  return stage_factored(ctx, fact, d1, elo, ehi, tlo, thi);
}

int nemo_stage_knockdown(nemo_ctx* ctx, const uint8_t* D, double A, double B) {
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  if (!D) return fail(NEMO_ERR_ARG, "null knockdown matrix");
  Ctx& c = ctx->c;
  const size_t S = c.S, E = c.E;
  if (!isfinite(A) || !isfinite(B)) return fail(NEMO_ERR_ARG, "A=%g B=%g must be finite", A, B);
  // the values present in the off-diagonal rows (S >= 2: every row j is one)
  bool has0 = false, has1 = false;
  std::vector<int> colsum(E, 0);
  for (size_t j = 0; j < S; ++j)
    for (size_t e = 0; e < E; ++e) {
      const uint8_t d = D[j * E + e];
      if (d > 1) return fail(NEMO_ERR_ARG, "D[%zu][%zu] = %d is not 0 or 1", j, e, (int)d);
      has0 |= d == 0;
      has1 |= d == 1;
      colsum[e] += d;
    }
  const double amax = std::max(has0 ? fabs(B) : 0.0, has1 ? fabs(A) : 0.0);
  const double lim = c.dtype == NEMO_F64 ? 170.0 : 20.0;
  if (amax > lim)
    return fail(NEMO_ERR_ARG, "|T| up to %g exceeds the %s product range (%g)", amax,
                c.dtype == NEMO_F64 ? "f64" : "f32", lim);
  // the addition chains of compute_scores (nem.py:25-34), in its order
  const std::vector<double> chains = nemo::host::knockdown_chains(c.S, A, B);
  // U's entries are chain elements: the ones indexed must be finite (NaN
  // cannot arise from finite A, B) and, for the factored kernels, <= 1e9
  bool ufin = true;
  for (size_t e = 0; e < E; ++e) {
    const int k = colsum[e];
    const double vs[3] = {chains[k], k > 0 ? chains[k - 1] : 0.0, chains[S + 1 + k]};
    for (double v : vs) ufin &= isfinite(v) && fabs(v) <= 1e9;
  }
  if ((rc = alloc_tables(c))) return rc;
  uint8_t* d_D = nullptr;
  double* d_chains = nullptr;
  HIPCHK(hipMalloc((void**)&d_D, S * E));
  HIPCHK(hipMalloc((void**)&d_chains, chains.size() * 8));
  HIPCHK(hipMemcpyAsync(d_D, D, S * E, hipMemcpyHostToDevice, c.stream));
  HIPCHK(hipMemcpyAsync(d_chains, chains.data(), chains.size() * 8, hipMemcpyHostToDevice, c.stream));
  HIPCHK(nemo::launch_knockdown_tables(c, d_D, d_chains, A, B, c.stream));
  HIPCHK(hipStreamSynchronize(c.stream));
  HIPCHK(hipFree(d_D));
  HIPCHK(hipFree(d_chains));
  c.table_absmax = amax;

  // factored form straight from D, with nemo_stage_tables' conventions:
  // lo_j = row j's first value, bit = "not lo_j"
  std::vector<uint64_t> d1;
  std::vector<double> elo, ehi, tlo, thi;
  nemo::host::knockdown_factored(c.S, c.E, D, A, B, d1, elo, ehi, &tlo, &thi);
  return stage_factored(ctx, ufin, d1, elo, ehi, tlo, thi);
}

static bool use_factored(const Ctx& c) {
  if (c.score_path == 1) return false;
  return c.factored;
}

// ---------------------------------------------------------------------------
// A4+A5
// ---------------------------------------------------------------------------
}  // extern "C"

// nemo_score_dev; allow_exact: the option exact_dev may route the call to the
// exact kernels (nemo_score's own fall-through passes false: it takes the
// exact path itself when option exact asks for it)
static int score_dev(nemo_ctx* ctx, int batch, const int32_t* d_pos, const double* d_w01, int cap, double* d_ll,
                     double* d_cs, double* d_cells, double* d_ow, void* stream, bool allow_exact) {
  int rc = check_ctx(ctx, true);
  if (rc) return rc;
  Ctx& c = ctx->c;
  if (batch < 0 || cap < 0) return fail(NEMO_ERR_ARG, "batch=%d cap=%d", batch, cap);
  if (batch == 0) return NEMO_OK;
  if (batch > c.cap_batch) return fail(NEMO_ERR_STATE, "batch %d > reserved %d", batch, c.cap_batch);
  if (!d_pos || !d_w01 || !d_ll) return fail(NEMO_ERR_ARG, "null device pointer");
  hipStream_t st = pick(ctx, stream);
  if (c.score_path == 2 && !c.factored)
    return fail(NEMO_ERR_STATE, "score_path=2 (factored) but the staged table is not factorable");
  if (allow_exact && ctx->exact_dev && use_factored(c) && c.fact_kernel == 0 && nemo::exact_supported(c)) {
    // nemo_score's exact path on device buffers: the cells are built in the
    // caller's d_ow (turned into order weights in place) or d_cells, else in
    // the context's scratch
    if (d_cells && d_ow) return fail(NEMO_ERR_ARG, "exact_dev: cells and order weights share one buffer");
    double* cells = d_ow ? d_ow : d_cells ? d_cells : c.d_ow;
    HIPCHK(nemo::launch_exact_eval(c, batch, cap, d_pos, d_w01, cells, d_cs ? d_cs : c.d_cs, d_ll, d_ow != nullptr,
                                   st));
    if (cells == c.d_ow) c.ow_chains = 0;  // d_ow no longer holds fused-step order weights
    return NEMO_OK;
  }
  if (use_factored(c)) {
    HIPCHK(nemo::launch_score_factored(c, batch, cap, d_pos, d_w01, d_ll, d_cs, d_cells, d_ow, st));
    return NEMO_OK;
  }
  HIPCHK(nemo::launch_prep(c, batch, cap, d_pos, d_w01, c.d_rows, c.d_sw, c.d_cnt, nullptr, st));
  HIPCHK(nemo::launch_score(c, batch, c.d_rows, c.d_sw, c.d_cnt, d_ll, d_cs, d_cells, d_ow, st));
  return NEMO_OK;
}

extern "C" {

int nemo_score_dev(nemo_ctx* ctx, int batch, const int32_t* d_pos, const double* d_w01, int cap,
                   double* d_ll, double* d_cs, double* d_cells, double* d_ow, void* stream) {
  return score_dev(ctx, batch, d_pos, d_w01, cap, d_ll, d_cs, d_cells, d_ow, stream, true);
}

int nemo_score(nemo_ctx* ctx, int batch, const int32_t* pos, const double* w01, int cap,
               double* ll_out, double* cs_out, double* cells_out, double* ow_out) {
  int rc = check_ctx(ctx, true);
  if (rc) return rc;
  if (batch < 0 || cap < 0) return fail(NEMO_ERR_ARG, "batch=%d cap=%d", batch, cap);
  if (batch == 0) return NEMO_OK;
  if (!pos || !w01 || !ll_out) return fail(NEMO_ERR_ARG, "null host pointer");
  Ctx& c = ctx->c;
  if ((rc = check_pos(pos, batch, c.S))) return rc;
  if ((rc = nemo_reserve(ctx, batch, 0))) return rc;
  const size_t S = c.S, E = c.E;
  hipStream_t st = c.stream;
  if (use_factored(c) && c.exact && c.fact_kernel == 0 && nemo::exact_supported(c)) {
    // the reference's arithmetic (nemo_exact.hip) whatever the batch, so a
    // score never depends on how many orders share the call: ll and, when
    // asked, the column sums cs, the cells and the order weights
    // (calculate_ll's ow; written over the cells, so a call that wants both
    // gets the cells from a first pass); pos and W in one copy.  An
    // explicitly chosen kernel (option fact_kernel) runs as chosen; the
    // batched device entry (nemo_score_dev) keeps the fixed-point kernels
    // unless option exact_dev is set.
    auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t n = batch, o_w01 = up(n * S * 4), o_ll = o_w01 + up(n * S * S * 8), total = o_ll + up(n * 8);
    if ((rc = step_stage(c, 0, total))) return rc;
    char* hs = (char*)c.h_stage[0];
    char* ds = (char*)c.d_step[0];
    memcpy(hs, pos, n * S * 4);
    memcpy(hs + o_w01, w01, n * S * S * 8);
    HIPCHK(hipMemcpyAsync(ds, hs, o_ll, hipMemcpyHostToDevice, st));
    if (cells_out && ow_out) {   // the cells first, then the pass below writes the order weights over them
      HIPCHK(nemo::launch_exact_eval(c, batch, cap, (const int32_t*)ds, (const double*)(ds + o_w01), c.d_ow,
                                     c.d_cs, nullptr, false, st));
      HIPCHK(hipMemcpyAsync(cells_out, c.d_ow, n * (S + 1) * E * 8, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(nemo::launch_exact_eval(c, batch, cap, (const int32_t*)ds, (const double*)(ds + o_w01), c.d_ow, c.d_cs,
                                   (double*)(ds + o_ll), ow_out != nullptr, st));
    HIPCHK(hipMemcpyAsync(hs + o_ll, ds + o_ll, n * 8, hipMemcpyDeviceToHost, st));
    if (cs_out) HIPCHK(hipMemcpyAsync(cs_out, c.d_cs, n * E * 8, hipMemcpyDeviceToHost, st));
    if (ow_out || cells_out)
      HIPCHK(hipMemcpyAsync(ow_out ? ow_out : cells_out, c.d_ow, n * (S + 1) * E * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    memcpy(ll_out, hs + o_ll, n * 8);
    c.ow_chains = 0;  // d_ow no longer holds fused-step order weights
    return NEMO_OK;
  }
  if (!cs_out && !cells_out && !ow_out && use_factored(c) && c.step_host_sum && batch <= 64) {
    // ll only (one sampler's calculate_ll): the fused step's transfer pattern --
    // pos and W staged in the pinned slot 0 and sent in ONE copy, the kernel's
    // per-evaluation partials (or its own sums) back in ONE copy, summed on the
    // host in the device's fixed order (sum_partials_host: the same bits as the
    // finalize launch this saves); pageable copies cost ~10 us each
    auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t n = batch, npart = (size_t)nemo::factored_partials(c);
    const size_t o_w01 = up(n * S * 4), o_part = o_w01 + up(n * S * S * 8), o_ll = o_part + up(n * npart * 8);
    const size_t total = o_ll + up(n * 8);
    if ((rc = step_stage(c, 0, total))) return rc;
    char* hs = (char*)c.h_stage[0];
    char* ds = (char*)c.d_step[0];
    memcpy(hs, pos, n * S * 4);
    memcpy(hs + o_w01, w01, n * S * S * 8);
    HIPCHK(hipMemcpyAsync(ds, hs, o_part, hipMemcpyHostToDevice, st));
    int np = 0;
    c.part_out = (double*)(ds + o_part);
    const hipError_t e = nemo::launch_score_factored(c, batch, cap, (const int32_t*)ds, (const double*)(ds + o_w01),
                                                     (double*)(ds + o_ll), nullptr, nullptr, nullptr, st, false, &np);
    c.part_out = nullptr;
    HIPCHK(e);  // np <= npart: launch_score_factored checks score_partials before launching
    HIPCHK(hipMemcpyAsync(hs + o_part, ds + o_part, total - o_part, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (np > 0) {
      const double* part = (const double*)(hs + o_part);
      for (size_t b = 0; b < n; ++b) ll_out[b] = nemo::host::sum_partials_host(part + b * (size_t)np, np);
    } else {
      memcpy(ll_out, hs + o_ll, n * 8);
    }
    c.ow_chains = 0;
    return NEMO_OK;
  }
  double* d_cells = nullptr;
  if (cells_out) HIPCHK(hipMallocAsync((void**)&d_cells, batch * (S + 1) * E * 8, st));
  HIPCHK(hipMemcpyAsync(c.d_pos, pos, batch * S * 4, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(c.d_w01, w01, batch * S * S * 8, hipMemcpyHostToDevice, st));
  rc = score_dev(ctx, batch, c.d_pos, c.d_w01, cap, c.d_ll, cs_out ? c.d_cs : nullptr, d_cells,
                 ow_out ? c.d_ow : nullptr, st, false);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(ll_out, c.d_ll, batch * 8, hipMemcpyDeviceToHost, st));
  if (cs_out) HIPCHK(hipMemcpyAsync(cs_out, c.d_cs, batch * E * 8, hipMemcpyDeviceToHost, st));
  if (ow_out)
    HIPCHK(hipMemcpyAsync(ow_out, c.d_ow, batch * (S + 1) * E * 8, hipMemcpyDeviceToHost, st));
  if (cells_out) {
    HIPCHK(hipMemcpyAsync(cells_out, d_cells, batch * (S + 1) * E * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipFreeAsync(d_cells, st));
  }
  HIPCHK(hipStreamSynchronize(st));
  c.ow_chains = 0;  // d_ow no longer holds fused-step order weights
  return NEMO_OK;
}

int nemo_score_group_dev(nemo_ctx* ctx, int batch, int group, const int32_t* d_pos,
                         const double* d_w01, int cap, double* d_ll, void* stream) {
  int rc = check_ctx(ctx, true);
  if (rc) return rc;
  Ctx& c = ctx->c;
  if (group != 1 && group != 4 && group != 8 && group != 16)
    return fail(NEMO_ERR_ARG, "group=%d not in {1,4,8,16}", group);
  if (group == 1) return nemo_score_dev(ctx, batch, d_pos, d_w01, cap, d_ll, nullptr, nullptr, nullptr, stream);
  if (batch < 0 || cap < 0) return fail(NEMO_ERR_ARG, "batch=%d cap=%d", batch, cap);
  if (batch == 0) return NEMO_OK;
  if (batch > c.cap_batch) return fail(NEMO_ERR_STATE, "batch %d > reserved %d", batch, c.cap_batch);
  const int ng = (batch + group - 1) / group;
  const size_t need = (size_t)ng * c.S * c.S * 16;  // sized for the largest group
  if ((size_t)c.cap_group_batch < need) {
    // first use only: callers reserve by calling once before timing/capture
    HIPCHK(hipStreamSynchronize(pick(ctx, stream)));
    HIPCHK(dalloc(&c.d_grows, (size_t)ng * c.S * c.S));
    HIPCHK(dalloc(&c.d_gsw, need));
    HIPCHK(dalloc(&c.d_gcnt, (size_t)ng * c.S));
    c.cap_group_batch = (int)std::min(need, (size_t)0x7fffffff);
  }
  hipStream_t st = pick(ctx, stream);
  HIPCHK(nemo::launch_prep_group(c, batch, group, cap, d_pos, d_w01, st));
  HIPCHK(nemo::launch_score_group(c, batch, group, d_ll, st));
  return NEMO_OK;
}

int nemo_lse(nemo_ctx* ctx, int rows, const double* cells, double* ll_out, double* cs_out,
             double* ow_out) {
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  if (rows < 1 || !cells || !ll_out) return fail(NEMO_ERR_ARG, "rows=%d / null pointer", rows);
  if ((rc = nemo_reserve(ctx, 1, 0))) return rc;
  Ctx& c = ctx->c;
  const size_t E = c.E;
  hipStream_t st = c.stream;
  double *d_cells = nullptr, *d_ow = nullptr;
  HIPCHK(hipMallocAsync((void**)&d_cells, rows * E * 8, st));
  if (ow_out) HIPCHK(hipMallocAsync((void**)&d_ow, rows * E * 8, st));
  HIPCHK(hipMemcpyAsync(d_cells, cells, rows * E * 8, hipMemcpyHostToDevice, st));
  HIPCHK(nemo::launch_lse(c, rows, d_cells, c.d_ll, cs_out ? c.d_cs : nullptr, d_ow, st));
  HIPCHK(hipMemcpyAsync(ll_out, c.d_ll, 8, hipMemcpyDeviceToHost, st));
  if (cs_out) HIPCHK(hipMemcpyAsync(cs_out, c.d_cs, E * 8, hipMemcpyDeviceToHost, st));
  if (ow_out) HIPCHK(hipMemcpyAsync(ow_out, d_ow, rows * E * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipFreeAsync(d_cells, st));
  if (d_ow) HIPCHK(hipFreeAsync(d_ow, st));
  HIPCHK(hipStreamSynchronize(st));
  return NEMO_OK;
}

// ---------------------------------------------------------------------------
// A8 core: generic batch of 1-D problems
// ---------------------------------------------------------------------------
int nemo_local_opt(nemo_ctx* ctx, int n, const double* cvec, const double* anc, const double* x0,
                   double* xstar, double* fstar, int32_t* nit, int32_t* nfev, int32_t* status) {
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  if (n < 0 || (n > 0 && (!cvec || !anc || !x0 || !xstar)))
    return fail(NEMO_ERR_ARG, "n=%d / null pointer", n);
  if (n == 0) return NEMO_OK;
  Ctx& c = ctx->c;
  if (!(c.exact && nemo::exact_supported(c)) && c.E > 80 * 64)
    return fail(NEMO_ERR_ARG, "E=%d > 5120 not supported by the fast local optima (option exact 0)", c.E);
  const size_t E = c.E;
  hipStream_t st = c.stream;
  double *d_c = nullptr, *d_a = nullptr, *d_x = nullptr, *d_o = nullptr;
  HIPCHK(hipMallocAsync((void**)&d_c, n * E * 8, st));
  HIPCHK(hipMallocAsync((void**)&d_a, n * 8, st));
  HIPCHK(hipMallocAsync((void**)&d_x, n * 8, st));
  HIPCHK(hipMallocAsync((void**)&d_o, n * 3 * 8, st));
  HIPCHK(hipMemcpyAsync(d_c, cvec, n * E * 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(d_a, anc, n * 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(d_x, x0, n * 8, hipMemcpyHostToDevice, st));
  // the product form needs each factor 1 + c e (e in (0, 1)) in [1e-30, 1e30]
  double cmin = 0.0, cmax = 0.0;
  for (size_t k = 0; k < (size_t)n * E; ++k) {
    cmin = std::min(cmin, cvec[k]);
    cmax = std::max(cmax, cvec[k]);
  }
  const bool prod = c.local_prod && 1.0 + cmin >= 1e-30 && 1.0 + cmax <= 1e30;
  if (c.exact && nemo::exact_supported(c)) HIPCHK(nemo::launch_local_opt_exact_generic(c, n, d_c, d_a, d_x, d_o, st));
  else HIPCHK(nemo::launch_local_opt_generic(c, n, d_c, d_a, d_x, d_o, prod, st));
  std::vector<double> o((size_t)n * 3);
  HIPCHK(hipMemcpyAsync(o.data(), d_o, n * 3 * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipFreeAsync(d_c, st));
  HIPCHK(hipFreeAsync(d_a, st));
  HIPCHK(hipFreeAsync(d_x, st));
  HIPCHK(hipFreeAsync(d_o, st));
  HIPCHK(hipStreamSynchronize(st));
  for (int k = 0; k < n; ++k) {
    const int32_t info = (int32_t)o[(size_t)k * 3 + 2];
    xstar[k] = o[(size_t)k * 3];
    if (fstar) fstar[k] = o[(size_t)k * 3 + 1];
    if (status) status[k] = info & 15;
    if (nit) nit[k] = (info >> 4) & 4095;
    if (nfev) nfev[k] = (info >> 16) & 32767;
  }
  return NEMO_OK;
}

// ---------------------------------------------------------------------------
// A6 fused per-step scorer
// ---------------------------------------------------------------------------
}  // extern "C"

namespace {

// the fused step takes the reference's arithmetic for this call (option
// exact and a factored model the exact kernels cover; any parent cap)
bool step_exact(const Ctx& c, int) { return use_factored(c) && c.exact && nemo::exact_supported(c); }

// the exact fused step's buffers for nchains chains, allocated on first use
// (never captured: step_start and nemo_optimal_weights_dev call this before
// any launch): eval #2's cells and either the recompute form's a rows
// (d_xa, chains x S x plan: 1.1 MB per chain at C3) or the stored form's c
// rows (d_xcbuf, chains x pairs x plan: 35 MB per chain at C3).  A failed
// allocation is the call's error -- the step never drops to other arithmetic
int exact_reserve(Ctx& c, int nchains) {
  NEMO_API_LOCK;
  const size_t S = c.S, E = c.E, plan = nemo::exact_plan_doubles(c), nc = (size_t)std::max(nchains, 1);
  bool grew = false;
  if (!c.d_xcells2 || c.cap_xcells2 < nc) {
    grew = true;
    ++c.graph_epoch;
    HIPCHK(hipStreamSynchronize(c.stream));
    HIPCHK(dalloc(&c.d_xcells2, nc * (S + 1) * E));
    // the persistent form's schedule: each pair's last evaluation count (0:
    // none yet) and the hand-out order
    HIPCHK(dalloc(&c.d_xcost, nc * S * S));
    HIPCHK(hipMemsetAsync(c.d_xcost, 0, nc * S * S * 4, c.stream));   // stream-ordered (see alloc_tables)
    HIPCHK(dalloc(&c.d_xorder, nc * (size_t)nemo::pairs_per_chain(c.S, 0)));
    HIPCHK(dalloc(&c.d_xhist, nc * 64));
    c.cap_xorder = nc * (size_t)nemo::pairs_per_chain(c.S, 0);
    c.cap_xcells2 = nc;
  }
  if (c.exact_trace) {
    const size_t need = nc * (size_t)nemo::pairs_per_chain(c.S, 0);
    if (need > c.cap_xtrace) {
      ++c.graph_epoch;
      HIPCHK(hipStreamSynchronize(c.stream));
      HIPCHK(dalloc(&c.d_xtrace, 4 * need));
      c.cap_xtrace = need;
    }
  }
  if (nemo::exact_rc(c)) {
    const size_t need = nc * S * plan;
    if (need > c.cap_xa) {
      ++c.graph_epoch;
      HIPCHK(hipStreamSynchronize(c.stream));
      HIPCHK(dalloc(&c.d_xa, need));
      // positions without an element stay 0 (the order-weight launch writes
      // only real elements): their c is 0 / b = 0, as in a stored row
      HIPCHK(hipMemsetAsync(c.d_xa, 0, need * 8, c.stream));
      c.cap_xa = need;
      grew = true;
    }
    // the slot form's row sets (one plan part; a fixed size: its resident waves)
    const size_t sneed = c.pw_parts == 1 ? nemo::exact_slot_doubles(c) : 0;
    if (sneed > c.cap_xsbuf) {
      ++c.graph_epoch;
      HIPCHK(hipStreamSynchronize(c.stream));
      HIPCHK(dalloc(&c.d_xsbuf, sneed));
      c.cap_xsbuf = sneed;
    }
  } else {
    const size_t need = nc * (size_t)nemo::pairs_per_chain(c.S, 0) * plan;
    if (need > c.cap_xcbuf) {
      ++c.graph_epoch;
      HIPCHK(hipStreamSynchronize(c.stream));
      HIPCHK(dalloc(&c.d_xcbuf, need));
      c.cap_xcbuf = need;
    }
  }
  // the zero fills above ran on c.stream (non-blocking): finish them before
  // any other stream -- the caller's of a _dev call, the null stream included
  // -- queues the step that reads them (a late d_xa fill would wipe real a
  // rows; unfilled d_xcost would give sched_bucket negative costs)
  if (grew) HIPCHK(hipStreamSynchronize(c.stream));
  return NEMO_OK;
}

// the fused step's device work on `stream`.  d_part2 null: eval #2's ll is
// summed on the device into d_ll_dag.  Set (the staged host path): eval #2's
// per-evaluation partials go to d_part2 (stride *np2) and are left for the
// host (sum_partials_host, same bits), *np2 = their count -- one launch
// fewer; *np2 = 0 when the kernel summed them itself (ll_dag written).
int optimal_weights_enqueue(nemo_ctx* ctx, int nchains, const int32_t* d_pos, const double* d_w01,
                            const double* d_anc, double sig0, double sig1, int cap, double* d_w_new,
                            double* d_ll1, double* d_ll_dag, int32_t* d_info, void* stream, double* d_part2,
                            int* np2, hipEvent_t anc_ready = nullptr) {
  if (np2) *np2 = 0;
  int rc = check_ctx(ctx, true);
  if (rc) return rc;
  Ctx& c = ctx->c;
  if (nchains < 0 || cap < 0) return fail(NEMO_ERR_ARG, "nchains=%d cap=%d", nchains, cap);
  if (nchains == 0) return NEMO_OK;
  if (nchains > c.cap_chains || nchains > c.cap_batch)
    return fail(NEMO_ERR_STATE, "nchains %d > reserved %d", nchains, c.cap_chains);
  if (!step_exact(c, cap) && c.E > 80 * 64)
    return fail(NEMO_ERR_ARG, "E=%d > 5120 not supported by the fast local optima (option exact 0)", c.E);
  if (!d_pos || !d_w01 || !d_anc || !d_w_new || !d_ll1 || !d_ll_dag)
    return fail(NEMO_ERR_ARG, "null device pointer");
  hipStream_t st = pick(ctx, stream);
  if (step_exact(c, cap)) {
    // the reference's own arithmetic (nemo_exact.hip): eval #1's cells and
    // order weights in d_ow (and the local optima's a rows), the local optima
    // (eval #1's ll summed by the launch's appended blocks), eval #2 summed on
    // the device.  With a cap, the capped parent lists throughout (the prep's
    // pair lists, both evaluations' cells)
    if (c.cap_xcells2 < (size_t)nchains || (nemo::exact_rc(c) ? !c.d_xa : !c.d_xcbuf))
      return fail(NEMO_ERR_STATE, "exact step buffers not reserved for %d chains", nchains);
    double* cs1 = c.d_xcs;
    double* cs2 = c.d_xcs + (size_t)nchains * c.E;
    HIPCHK(nemo::launch_step_prep(c, nchains, cap, d_pos, d_w01, d_info, st));
    HIPCHK(nemo::launch_exact_eval(c, nchains, cap, d_pos, d_w01, c.d_ow, cs1, nullptr, true, st,
                                   nemo::exact_rc(c) ? c.d_xa : nullptr));
    if (anc_ready) HIPCHK(hipStreamWaitEvent(st, anc_ready, 0));  // ancestor_x from the second stream
    HIPCHK(nemo::launch_local_opt_exact(c, nchains, nemo::pairs_per_chain(c.S, cap), c.d_pairs, d_w01, d_anc, c.d_ow,
                                        sig0, sig1, d_w_new,
                                        c.d_wdag, d_info, cs1, d_ll1, st));
    HIPCHK(nemo::launch_exact_eval(c, nchains, cap, d_pos, c.d_wdag, c.d_xcells2, cs2, d_ll_dag, false, st));
    c.ow_chains = nchains;
    return NEMO_OK;
  }
  const int npairs = nemo::pairs_per_chain(c.S, cap);
  // eval #1 with order weights (nem_order_mcmc.py:181-182).  Factored: one
  // prep launch for the pair lists (info rows preset to -1) and eval #1's
  // Delta, and eval #1's partial sums ride in the local-optimum launch -- two
  // launches fewer per step (a graph node costs ~5 us however small its kernel)
  nemo::FinalizeArgs fin;
  if (use_factored(c)) {
    HIPCHK(nemo::launch_step_prep(c, nchains, cap, d_pos, d_w01, d_info, st));
    int np = 0;
    HIPCHK(nemo::launch_score_factored(c, nchains, cap, d_pos, d_w01, d_ll1, nullptr, nullptr, c.d_ow, st,
                                       true, &np));
    if (np > 0) fin = nemo::FinalizeArgs{c.d_fpartial, np, nchains, d_ll1};
  } else {
    HIPCHK(nemo::launch_prep(c, nchains, cap, d_pos, d_w01, c.d_rows, c.d_sw, c.d_cnt, c.d_pairs, st, d_info));
    HIPCHK(nemo::launch_score(c, nchains, c.d_rows, c.d_sw, c.d_cnt, d_ll1, nullptr, nullptr, c.d_ow, st));
  }
  // every permissible pair's local optimum (nem_order_mcmc.py:186-189)
  if (anc_ready) HIPCHK(hipStreamWaitEvent(st, anc_ready, 0));
  HIPCHK(nemo::launch_local_opt_pairs(c, nchains, npairs, c.d_pairs, c.d_rows, d_w01, d_anc, c.d_ow,
                                      sig0, sig1, d_w_new, c.d_wdag, d_info, st, fin));
  // eval #2 on the binarised weights (nem_order_mcmc.py:205-207)
  if (use_factored(c) && d_part2) {
    c.part_out = d_part2;
    const hipError_t e = nemo::launch_score_factored(c, nchains, cap, d_pos, c.d_wdag, d_ll_dag, nullptr, nullptr,
                                                     nullptr, st, false, np2);
    c.part_out = nullptr;
    HIPCHK(e);
  } else if (use_factored(c)) {
    HIPCHK(nemo::launch_score_factored(c, nchains, cap, d_pos, c.d_wdag, d_ll_dag, nullptr, nullptr, nullptr, st));
  } else {
    HIPCHK(nemo::launch_prep(c, nchains, cap, d_pos, c.d_wdag, c.d_rows, c.d_sw, c.d_cnt, nullptr, st));
    HIPCHK(nemo::launch_score(c, nchains, c.d_rows, c.d_sw, c.d_cnt, d_ll_dag, nullptr, nullptr, nullptr, st));
  }
  c.ow_chains = nchains;
  return NEMO_OK;
}

}  // namespace

extern "C" {

int nemo_optimal_weights_dev(nemo_ctx* ctx, int nchains, const int32_t* d_pos, const double* d_w01,
                             const double* d_anc, double sig0, double sig1, int cap,
                             double* d_w_new, double* d_ll1, double* d_ll_dag, int32_t* d_info,
                             void* stream) {
  int rc = check_ctx(ctx, true);
  if (rc) return rc;
  if (nchains > 0 && nchains <= ctx->c.cap_chains && cap >= 0 && step_exact(ctx->c, cap) &&
      (rc = exact_reserve(ctx->c, nchains)))
    return rc;
  return optimal_weights_enqueue(ctx, nchains, d_pos, d_w01, d_anc, sig0, sig1, cap, d_w_new, d_ll1, d_ll_dag,
                                 d_info, stream, nullptr, nullptr);
}

}  // extern "C"

namespace {

// every transfer of a fused step goes through a pinned staging slot: [W |
// pos | w01 | anc | w_new | info | ll1 | ll_dag | ancestor flags | eval #2's
// partials], each part 256-B aligned, and a device block with the same
// layout.  Given W~ and ancestor_x (nemo_optimal_weights): one H2D of [pos ..
// anc], one D2H of [w_new .. partials].  Given W (nemo_optimal_weights_w):
// one H2D of [W | pos], the device computes W~ and ancestor_x in place, one
// D2H of [w01 .. partials].  info is preset to -1 (= not a permissible pair)
// by the step's prep; the host hands back w_new at the entries info marks
// (the caller's values stay everywhere else) and sums eval #2's partials
// (npart: the most any score kernel writes per evaluation)
struct StepLayout {
  size_t o_pos, o_w01, o_anc, o_wn, o_inf, o_ll1, o_lld, o_flag, o_part, total;
  // from_w: the W segment leads the slot; the W~ / ancestor_x calls have none
  StepLayout(size_t S, size_t n, size_t npart, bool from_w) {
    auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
    o_pos = from_w ? up(n * S * S * 8) : 0;
    o_w01 = o_pos + up(n * S * 4);
    o_anc = o_w01 + up(n * S * S * 8);
    o_wn = o_anc + up(n * S * S * 8);
    o_inf = o_wn + up(n * S * S * 8);
    o_ll1 = o_inf + up(n * S * S * 4);
    o_lld = o_ll1 + up(n * 8);
    o_flag = o_lld + up(n * 8);
    o_part = o_flag + up(n * 4);
    total = o_part + up(n * npart * 8);
  }
};

size_t step_npart(const Ctx& c) { return use_factored(c) ? (size_t)nemo::factored_partials(c) : 0; }

}  // namespace

extern "C" {

// first half of nemo_optimal_weights: validate, fill staging slot `slot`,
// queue the device work (one H2D copy, the launches, one D2H copy) and record
// the slot's event; returns without waiting
static int step_start(nemo_ctx* ctx, int slot, int nchains, const int32_t* pos, const double* w01,
                      const double* anc, const double* w_in, double sig0, double sig1, int cap,
                      const double* w_new, bool want_prep = false) {
  int rc = check_ctx(ctx, true);
  if (rc) return rc;
  if (nchains < 0) return fail(NEMO_ERR_ARG, "nchains=%d", nchains);
  if (nchains == 0) return NEMO_OK;
  const bool from_w = w_in != nullptr;
  if (!pos || (!from_w && (!w01 || !anc)) || !w_new) return fail(NEMO_ERR_ARG, "null host pointer");
  Ctx& c = ctx->c;
  if (from_w && !nemo::ancestor_supported(c))
    return fail(NEMO_ERR_ARG, "S=%d > 64: ancestor_x on the device covers S <= 64 (give W~ and ancestor_x)", c.S);
  if (from_w && c.anc_overlap && !c.stream2) {  // created before any capture
    NEMO_API_LOCK;
    HIPCHK(hipStreamCreateWithFlags(&c.stream2, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&c.ev_fork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c.ev_join, hipEventDisableTiming));
  }
  if ((rc = check_pos(pos, nchains, c.S))) return rc;
  if ((rc = nemo_reserve(ctx, nchains, nchains))) return rc;
  if (cap >= 0 && step_exact(c, cap) && (rc = exact_reserve(c, nchains))) return rc;
  const size_t S = c.S, n = nchains;
  hipStream_t st = c.stream;
  const StepLayout L(S, n, step_npart(c), from_w);
  if ((rc = step_stage(c, slot, L.total))) return rc;
  char* hs = (char*)c.h_stage[slot];
  char* ds = (char*)c.d_step[slot];
  memcpy(hs + L.o_pos, pos, n * S * 4);
  if (from_w) {
    memcpy(hs, w_in, n * S * S * 8);
  } else {
    memcpy(hs + L.o_w01, w01, n * S * S * 8);
    memcpy(hs + L.o_anc, anc, n * S * S * 8);
  }
  // replayed as a hipGraph per (nchains, cap, slot) while no captured
  // argument changes (the staging buffers, options and tables bump
  // graph_epoch), so a step costs one graph launch instead of ~10 API calls
  int np2 = 0;
  auto enqueue = [&]() -> int {
    const int32_t* d_pos = (const int32_t*)(ds + L.o_pos);
    hipEvent_t anc_ready = nullptr;
    if (from_w) {  // [W | pos] in; W~ and ancestor_x made in place
      HIPCHK(hipMemcpyAsync(ds, hs, L.o_w01, hipMemcpyHostToDevice, st));
      const double* d_w = (const double*)ds;
      double* d_w01 = (double*)(ds + L.o_w01);
      double* d_anc = (double*)(ds + L.o_anc);
      int32_t* d_flag = (int32_t*)(ds + L.o_flag);
      if (c.anc_overlap) {
        // W~ on the step's stream for eval #1; ancestor_x on stream2 beside
        // it, joined before the local optima
        HIPCHK(nemo::launch_w01(c, nchains, cap, d_pos, d_w, d_w01, st));
        HIPCHK(hipEventRecord(c.ev_fork, st));
        HIPCHK(hipStreamWaitEvent(c.stream2, c.ev_fork, 0));
        HIPCHK(nemo::launch_ancestor(c, nchains, cap, d_pos, d_w, nullptr, d_anc, d_flag, c.stream2));
        HIPCHK(hipEventRecord(c.ev_join, c.stream2));
        anc_ready = c.ev_join;
      } else {
        HIPCHK(nemo::launch_ancestor(c, nchains, cap, d_pos, d_w, d_w01, d_anc, d_flag, st));
      }
    } else {  // info: preset by the prep
      HIPCHK(hipMemcpyAsync(ds + L.o_pos, hs + L.o_pos, L.o_wn - L.o_pos, hipMemcpyHostToDevice, st));
    }
    int r = optimal_weights_enqueue(ctx, nchains, d_pos, (const double*)(ds + L.o_w01),
                                    (const double*)(ds + L.o_anc), sig0, sig1, cap, (double*)(ds + L.o_wn),
                                    (double*)(ds + L.o_ll1), (double*)(ds + L.o_lld), (int32_t*)(ds + L.o_inf), st,
                                    c.step_host_sum && L.o_part < L.total ? (double*)(ds + L.o_part) : nullptr,
                                    &np2, anc_ready);
    if (r) return r;  // np2 <= step_npart: checked by launch_score_factored before it launched
    // W~ and ancestor_x go back only when the caller asked for them
    const size_t o_out = from_w && want_prep ? L.o_w01 : L.o_wn;
    HIPCHK(hipMemcpyAsync(hs + o_out, ds + o_out, L.total - o_out, hipMemcpyDeviceToHost, st));
    return NEMO_OK;
  };
  Ctx::StepGraph* sg = nullptr;
  bool graphs_off = false;  // the capture failed: decided after the direct launch below
  if (c.graphs && !c.timing) {
    for (auto& g : c.step_graph)
      if (g.exec && g.epoch == c.graph_epoch && g.nchains == nchains && g.cap == cap && g.slot == slot &&
          g.sig0 == sig0 && g.sig1 == sig1 && g.from_w == from_w && g.want_prep == want_prep)
        sg = &g;
    if (!sg) {  // capture once
      NEMO_API_LOCK;
      Ctx::StepGraph& g = c.step_graph[c.step_graph_next];
      c.step_graph_next = (c.step_graph_next + 1) % Ctx::kStepGraphs;
      if (g.exec) {
        // the evicted exec may be the one the other staging slot launched and
        // is still running: every step runs on st, so draining it is enough
        HIPCHK(hipStreamSynchronize(st));
        (void)hipGraphExecDestroy(g.exec);
        g.exec = nullptr;
      }
      hipGraph_t graph = nullptr;
      if (hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) == hipSuccess) {
        const int r = enqueue();
        const hipError_t ee = hipStreamEndCapture(st, &graph);
        if (r != NEMO_OK && r != NEMO_ERR_HIP) {
          // a call error (argument, state, unsupported kernel): the caller's,
          // not the capture's -- graphs stay on
          if (graph) (void)hipGraphDestroy(graph);
          (void)hipGetLastError();
          return r;
        }
        if (r == NEMO_OK && ee == hipSuccess && graph &&
            hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0) == hipSuccess) {
          g.nchains = nchains;
          g.cap = cap;
          g.slot = slot;
          g.sig0 = sig0;
          g.sig1 = sig1;
          g.from_w = from_w;
          g.want_prep = want_prep;
          g.epoch = c.graph_epoch;
          g.np2 = np2;
          sg = &g;
        } else {
          g.exec = nullptr;
          graphs_off = true;
        }
        if (graph) (void)hipGraphDestroy(graph);
        (void)hipGetLastError();
      } else {
        graphs_off = true;
      }
    }
  }
  if (sg) {
    HIPCHK(hipGraphLaunch(sg->exec, st));
    c.ow_chains = nchains;  // nemo_optimal_weights_dev's host-side effect
    np2 = sg->np2;
  } else if ((rc = enqueue())) {
    return rc;  // the direct launch fails as well: the call's error, graphs stay on
  }
  // the step ran without the graph the capture could not make: this runtime
  // does not capture it, so launch directly from now on
  if (graphs_off) c.graphs = 0;
  c.step_np2[slot] = np2;
  HIPCHK(hipEventRecord(c.step_done[slot], st));
  return NEMO_OK;
}

// second half: wait for the slot's device work, hand the outputs back and
// raise the reference's error for a failed local optimisation
static int step_finish(nemo_ctx* ctx, int slot, int nchains, double* w_new, double* ll1, double* ll_dag,
                       int32_t* info, bool from_w = false, double* w01_out = nullptr, double* anc_out = nullptr,
                       int32_t* aflag = nullptr) {
  Ctx& c = ctx->c;
  if (nchains == 0) return NEMO_OK;
  const size_t S = c.S, n = nchains;
  const StepLayout L(S, n, step_npart(c), from_w);
  HIPCHK(hipEventSynchronize(c.step_done[slot]));
  const char* hs = (const char*)c.h_stage[slot];
  if (from_w) {
    if (w01_out) memcpy(w01_out, hs + L.o_w01, n * S * S * 8);
    if (anc_out) memcpy(anc_out, hs + L.o_anc, n * S * S * 8);
    const int32_t* fl = (const int32_t*)(hs + L.o_flag);
    if (aflag) memcpy(aflag, fl, n * 4);
    for (size_t b = 0; b < n; ++b)
      if (fl[b])
        return fail(NEMO_ERR_LINALG, "ancestor_x of chain %zu: %s", b,
                    (fl[b] & 2) ? "I - W~ is not finite" : (fl[b] & 1) ? "singular matrix"
                                                                      : "non-finite factors (recompute on the host)");
  }
  memcpy(ll1, hs + L.o_ll1, n * 8);
  if (const int np2 = c.step_np2[slot]) {  // eval #2's partials: the device's fixed-order sum, on the host
    const double* part = (const double*)(hs + L.o_part);
    for (size_t b = 0; b < n; ++b) ll_dag[b] = nemo::host::sum_partials_host(part + b * (size_t)np2, np2);
  } else {
    memcpy(ll_dag, hs + L.o_lld, n * 8);
  }
  if (info) memcpy(info, hs + L.o_inf, n * S * S * 4);
  const int32_t* inf = (const int32_t*)(hs + L.o_inf);
  const double* wn = (const double*)(hs + L.o_wn);
  const size_t nn = n * S * S;
  // branch-free blend (vectorised): the caller's value stays where info is -1
  for (size_t k = 0; k < nn; ++k) w_new[k] = inf[k] != -1 ? wn[k] : w_new[k];
  size_t bad = SIZE_MAX;  // first failed pair in index order
  for (size_t k = 0; k < nn; ++k)
    if (inf[k] != -1 && (inf[k] & 15) >= NEMO_LBFGSB_ABNORMAL) {
      bad = k;
      break;
    }
  if (bad != SIZE_MAX) {
    const size_t b = bad / (S * S), i = (bad / S) % S, j = bad % S;
    return fail(NEMO_ERR_OPT, "Minimization not successful, Reason: %s (chain %zu, pair %zu<-%zu)",
                (inf[bad] & 15) == NEMO_LBFGSB_ABNORMAL ? "ABNORMAL_TERMINATION_IN_LNSRCH"
                                                       : "STOP: TOTAL NO. of ITERATIONS REACHED LIMIT",
                b, i, j);
  }
  return NEMO_OK;
}

int nemo_optimal_weights(nemo_ctx* ctx, int nchains, const int32_t* pos, const double* w01,
                         const double* anc, double sig0, double sig1, int cap, double* w_new,
                         double* ll1, double* ll_dag, int32_t* info) {
  if (!ll1 || !ll_dag) return fail(NEMO_ERR_ARG, "null host pointer");
  int rc = step_start(ctx, 0, nchains, pos, w01, anc, nullptr, sig0, sig1, cap, w_new);
  if (rc) return rc;
  return step_finish(ctx, 0, nchains, w_new, ll1, ll_dag, info);
}

int nemo_optimal_weights_w(nemo_ctx* ctx, int nchains, const int32_t* pos, const double* w, double sig0,
                           double sig1, int cap, double* w01_out, double* anc_out, double* w_new, double* ll1,
                           double* ll_dag, int32_t* info, int32_t* anc_flag) {
  if (!ll1 || !ll_dag || !w) return fail(NEMO_ERR_ARG, "null host pointer");
  int rc = step_start(ctx, 0, nchains, pos, nullptr, nullptr, w, sig0, sig1, cap, w_new, w01_out || anc_out);
  if (rc) return rc;
  return step_finish(ctx, 0, nchains, w_new, ll1, ll_dag, info, true, w01_out, anc_out, anc_flag);
}

// asynchronous form: the library thread runs each call's transfers, launches
// and checks; the caller's thread only queues and, later, collects.  Two calls
// are in flight at once (staging slots 1 and 2): the thread stages and queues
// the next call while the device still runs the previous one, then waits for
// that one (nemo_host.h StepQueue)
static int steps_submit(nemo_ctx* ctx, std::unique_ptr<StepJob> j);

int nemo_optimal_weights_begin(nemo_ctx* ctx, int nchains, const int32_t* pos, const double* w01,
                               const double* anc, double sig0, double sig1, int cap, double* w_new,
                               double* ll1, double* ll_dag, int32_t* info) {
  int rc = check_ctx(ctx, true);
  if (rc) return rc;
  if (nchains < 0) return fail(NEMO_ERR_ARG, "nchains=%d", nchains);
  if (!pos || !w01 || !anc || !w_new || !ll1 || !ll_dag) return fail(NEMO_ERR_ARG, "null host pointer");
  return steps_submit(
      ctx, std::unique_ptr<StepJob>(new StepJob{nchains, cap, pos, w01, anc, sig0, sig1, w_new, ll1, ll_dag, info}));
}

int nemo_optimal_weights_w_begin(nemo_ctx* ctx, int nchains, const int32_t* pos, const double* w, double sig0,
                                 double sig1, int cap, double* w01_out, double* anc_out, double* w_new,
                                 double* ll1, double* ll_dag, int32_t* info, int32_t* anc_flag) {
  int rc = check_ctx(ctx, true);
  if (rc) return rc;
  if (nchains < 0) return fail(NEMO_ERR_ARG, "nchains=%d", nchains);
  if (!pos || !w || !w_new || !ll1 || !ll_dag) return fail(NEMO_ERR_ARG, "null host pointer");
  std::unique_ptr<StepJob> j(
      new StepJob{nchains, cap, pos, nullptr, nullptr, sig0, sig1, w_new, ll1, ll_dag, info});
  j->w_in = w;
  j->w01_out = w01_out;
  j->anc_out = anc_out;
  j->aflag = anc_flag;
  return steps_submit(ctx, std::move(j));
}

static int steps_submit(nemo_ctx* ctx, std::unique_ptr<StepJob> j) {
  std::string err;
  try {
    if (!ctx->steps) {
      auto next_slot = std::make_shared<int>(1);
      ctx->steps.reset(new nemo::host::StepQueue<StepJob>(
          [ctx, next_slot](StepJob& j) {  // start: true = in flight
            j.slot = *next_slot;
            j.rc = step_start(ctx, j.slot, j.nchains, j.pos, j.w01, j.anc, j.w_in, j.sig0, j.sig1, j.cap,
                              j.w_new, j.w01_out || j.anc_out);
            if (j.rc) {
              j.err = g_err;
              (void)hipStreamSynchronize(ctx->c.stream);  // nothing of it left running in its slot
              return false;
            }
            if (j.nchains == 0) return false;
            *next_slot = 3 - *next_slot;
            return true;
          },
          [ctx](StepJob& j) { return hipEventQuery(ctx->c.step_done[j.slot]) != hipErrorNotReady; },
          [ctx](StepJob& j) {
            j.rc = step_finish(ctx, j.slot, j.nchains, j.w_new, j.ll1, j.ll_dag, j.info, j.w_in != nullptr,
                               j.w01_out, j.anc_out, j.aflag);
            if (j.rc) j.err = g_err;
          },
          2));
    }
    if (ctx->steps->submit(std::move(j), &err)) return NEMO_OK;
  } catch (const std::exception& e) {
    err = e.what();
  }
  return fail(NEMO_ERR_STATE, "nemo_optimal_weights_begin: %s", err.c_str());
}

int nemo_optimal_weights_end(nemo_ctx* ctx) {
  if (!ctx) return fail(NEMO_ERR_ARG, "null context");
  std::unique_ptr<StepJob> j = ctx->steps ? ctx->steps->collect() : nullptr;
  if (!j) return fail(NEMO_ERR_STATE, "no nemo_optimal_weights_begin to end");
  if (j->rc) g_err = j->err;
  return j->rc;
}

int nemo_ancestor_dev(nemo_ctx* ctx, int nchains, const int32_t* d_pos, const double* d_w, int cap,
                      double* d_w01, double* d_anc, int32_t* d_flag, void* stream) {
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  Ctx& c = ctx->c;
  if (nchains < 0 || cap < 0) return fail(NEMO_ERR_ARG, "nchains=%d cap=%d", nchains, cap);
  if (!nemo::ancestor_supported(c)) return fail(NEMO_ERR_ARG, "S=%d > 64", c.S);
  if (nchains == 0) return NEMO_OK;
  if (!d_pos || !d_w || !d_w01 || !d_anc || !d_flag) return fail(NEMO_ERR_ARG, "null device pointer");
  HIPCHK(nemo::launch_ancestor(c, nchains, cap, d_pos, d_w, d_w01, d_anc, d_flag, pick(ctx, stream)));
  return NEMO_OK;
}

int nemo_fetch_exact_trace(nemo_ctx* ctx, int* n, long long* out) {
  NEMO_API_LOCK;
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  if (!n) return fail(NEMO_ERR_ARG, "null n");
  Ctx& c = ctx->c;
  HIPCHK(hipStreamSynchronize(c.stream));
  *n = c.xtrace_n;
  if (out && c.xtrace_n > 0)
    HIPCHK(nemo::copy_sync(c, out, c.d_xtrace, (size_t)c.xtrace_n * 4 * sizeof(long long), hipMemcpyDeviceToHost));
  return NEMO_OK;
}

int nemo_fetch_order_weights(nemo_ctx* ctx, int chain, double* ow_out) {
  int rc = check_ctx(ctx, true);
  if (rc) return rc;
  Ctx& c = ctx->c;
  if (chain < 0 || chain >= c.ow_chains || !ow_out)
    return fail(NEMO_ERR_STATE, "no order weights for chain %d (have %d)", chain, c.ow_chains);
  const size_t n = (size_t)(c.S + 1) * c.E;
  HIPCHK(hipMemcpyAsync(ow_out, c.d_ow + (size_t)chain * n, n * 8, hipMemcpyDeviceToHost, c.stream));
  HIPCHK(hipStreamSynchronize(c.stream));
  return NEMO_OK;
}

// ---------------------------------------------------------------------------
// fixed-order optimizers (methods.py)
// ---------------------------------------------------------------------------
}  // extern "C"

namespace {

int opt_status(const Ctx& c, const std::vector<int32_t>& inf, int nprob) {
  const size_t S = c.S;
  for (size_t k = 0; k < inf.size(); ++k) {
    if (inf[k] == -1) continue;  // not a permissible pair
    const int status = inf[k] & 15;
    if (status >= NEMO_LBFGSB_ABNORMAL) {
      const size_t b = k / (S * S), i = (k / S) % S, j = k % S;
      return fail(NEMO_ERR_OPT, "Minimization not successful, Reason: %s (problem %zu, pair %zu<-%zu)",
                  status == NEMO_LBFGSB_ABNORMAL ? "ABNORMAL_TERMINATION_IN_LNSRCH"
                                                 : "STOP: TOTAL NO. of ITERATIONS REACHED LIMIT",
                  b, i, j);
    }
  }
  (void)nprob;
  return NEMO_OK;
}

// eval with order weights of nprob problems on device weights d_w (cap 0 or
// a cap), into c.d_ll and c.d_ow; leaves prep's pair lists in c.d_pairs
int eval_with_ow(Ctx& c, int nprob, int cap, const double* d_w, hipStream_t st) {
  HIPCHK(nemo::launch_prep(c, nprob, cap, c.d_pos, d_w, c.d_rows, c.d_sw, c.d_cnt, c.d_pairs, st));
  if (c.score_path != 1 && c.factored)
    HIPCHK(nemo::launch_score_factored(c, nprob, cap, c.d_pos, d_w, c.d_ll, nullptr, nullptr, c.d_ow, st));
  else
    HIPCHK(nemo::launch_score(c, nprob, c.d_rows, c.d_sw, c.d_cnt, c.d_ll, nullptr, nullptr, c.d_ow, st));
  c.ow_chains = nprob;
  return NEMO_OK;
}

int methods_prologue(nemo_ctx* ctx, int nprob, const int32_t* pos, const double* w) {
  int rc = check_ctx(ctx, true);
  if (rc) return rc;
  Ctx& c = ctx->c;
  if (nprob < 0) return fail(NEMO_ERR_ARG, "nprob=%d", nprob);
  if (nprob > 0 && (!pos || !w)) return fail(NEMO_ERR_ARG, "null host pointer");
  if (nprob > 32767) return fail(NEMO_ERR_ARG, "nprob=%d > 32767", nprob);
  if (c.E > 80 * 64) return fail(NEMO_ERR_ARG, "E=%d > 5120 not supported by local optima", c.E);
  if ((rc = check_pos(pos, nprob, c.S))) return rc;
  if ((rc = nemo_reserve(ctx, nprob, nprob))) return rc;
  const size_t S = c.S;
  HIPCHK(hipMemcpyAsync(c.d_pos, pos, nprob * S * 4, hipMemcpyHostToDevice, c.stream));
  HIPCHK(hipMemcpyAsync(c.d_wnew, w, nprob * S * S * 8, hipMemcpyHostToDevice, c.stream));
  HIPCHK(hipMemsetAsync(c.d_info, 0xff, nprob * S * S * 4, c.stream));
  return NEMO_OK;
}

}  // namespace

extern "C" {

int nemo_gamma_sweep(nemo_ctx* ctx, int nprob, const int32_t* pos, const double* w, int cap,
                     double* w_out, double* ll_out, int32_t* info) {
  int rc = methods_prologue(ctx, nprob, pos, w);
  if (rc || nprob == 0) return rc;
  if (cap < 0) return fail(NEMO_ERR_ARG, "cap=%d", cap);
  if (!w_out || !ll_out) return fail(NEMO_ERR_ARG, "null host pointer");
  Ctx& c = ctx->c;
  const size_t S = c.S;
  hipStream_t st = c.stream;
  // opt_gamma: the evaluation takes the raw weights (methods.py:398)
  HIPCHK(hipMemcpyAsync(c.d_w01, c.d_wnew, nprob * S * S * 8, hipMemcpyDeviceToDevice, st));
  if ((rc = eval_with_ow(c, nprob, cap, c.d_w01, st))) return rc;
  HIPCHK(nemo::launch_gamma_pairs(c, nprob, nemo::pairs_per_chain(c.S, cap), c.d_pairs, c.d_rows, c.d_w01,
                                  c.d_ow, c.d_wnew, c.d_info, st));
  std::vector<int32_t> inf((size_t)nprob * S * S);
  HIPCHK(hipMemcpyAsync(w_out, c.d_wnew, nprob * S * S * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(ll_out, c.d_ll, nprob * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(inf.data(), c.d_info, inf.size() * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (info) memcpy(info, inf.data(), inf.size() * 4);
  return opt_status(c, inf, nprob);
}

int nemo_inverse_ancestral(nemo_ctx* ctx, int nprob, const int32_t* pos, const double* w, double* out) {
  NEMO_API_LOCK;
  int rc = methods_prologue(ctx, nprob, pos, w);
  if (rc || nprob == 0) return rc;
  if (!out) return fail(NEMO_ERR_ARG, "null host pointer");
  Ctx& c = ctx->c;
  const size_t S = c.S;
  HIPCHK(nemo::launch_ancestral(c, nprob, c.d_pos, c.d_wnew, c.d_w01, c.stream));
  HIPCHK(hipMemcpyAsync(out, c.d_w01, nprob * S * S * 8, hipMemcpyDeviceToHost, c.stream));
  HIPCHK(hipStreamSynchronize(c.stream));
  return NEMO_OK;
}

int nemo_inverse_sweep(nemo_ctx* ctx, int nprob, const int32_t* pos, const double* w, double* w_out,
                       double* ll_out, int32_t* info) {
  int rc = methods_prologue(ctx, nprob, pos, w);
  if (rc || nprob == 0) return rc;
  if (!w_out || !ll_out) return fail(NEMO_ERR_ARG, "null host pointer");
  Ctx& c = ctx->c;
  const size_t S = c.S;
  hipStream_t st = c.stream;
  // levels of independent pairs that keep the reference's loop semantics
  // (nemo_host.h build_inverse_schedule)
  nemo::host::build_inverse_schedule(c.inv, c.S, nprob, pos);
  if (c.inv.list.size() > c.inv_list_cap) {
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(dalloc(&c.d_inv_list, c.inv.list.size()));
    c.inv_list_cap = c.inv.list.size();
  }
  if (!c.inv.list.empty())
    HIPCHK(hipMemcpyAsync(c.d_inv_list, c.inv.list.data(), c.inv.list.size() * 4, hipMemcpyHostToDevice, st));
  // evaluation weights B/(1+B) (methods.py:118-121), evaluation (:122-123)
  HIPCHK(nemo::launch_ancestral(c, nprob, c.d_pos, c.d_wnew, c.d_w01, st));
  if ((rc = eval_with_ow(c, nprob, 0, c.d_w01, st))) return rc;
  // the pair loop (:125-127), level by level, optima committed into d_wnew
  for (size_t l = 0; l + 1 < c.inv.level_off.size(); ++l) {
    const int o0 = c.inv.level_off[l], o1 = c.inv.level_off[l + 1];
    HIPCHK(nemo::launch_inverse_level(c, o1 - o0, c.d_inv_list + o0, c.d_pos, c.d_wnew, c.d_ow, c.d_wdag,
                                      c.d_info, st));
  }
  std::vector<int32_t> inf((size_t)nprob * S * S);
  HIPCHK(hipMemcpyAsync(w_out, c.d_wnew, nprob * S * S * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(ll_out, c.d_ll, nprob * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(inf.data(), c.d_info, inf.size() * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  // pairs outside the lower triangle: B[a][b] = 0 whatever x, so the
  // objective is flat and L-BFGS-B stops at the clipped start (nit 0, 2 f-evals)
  for (int32_t ent : c.inv.skip) {
    const size_t idx = ((size_t)(ent >> 16) * S + ((ent >> 8) & 0xff)) * S + (ent & 0xff);
    w_out[idx] = std::min(std::max(w[idx], -5000.0), 500.0);
    inf[idx] = NEMO_LBFGSB_CONV_PGTOL | (2 << 16);
  }
  if (info) memcpy(info, inf.data(), inf.size() * 4);
  return opt_status(c, inf, nprob);
}

int nemo_set_option(nemo_ctx* ctx, const char* name, int value) {
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  if (!name) return fail(NEMO_ERR_ARG, "null option name");
  ++ctx->c.graph_epoch;  // any option may change what a captured step launches
  if (strcmp(name, "exact") == 0) {
    ctx->c.exact = value ? 1 : 0;
    return NEMO_OK;
  }
  if (strcmp(name, "exact_dev") == 0) {
    ctx->exact_dev = value ? 1 : 0;
    return NEMO_OK;
  }
  if (strcmp(name, "exact_form") == 0) {
    if (value < 0 || value > 7 || value == 6)
      return fail(NEMO_ERR_ARG,
                  "exact_form %d (0 auto, 1 latency, 2 throughput, 3 pair, 4 cached throughput, 5 dual, 7 slot)",
                  value);
    ctx->c.exact_form = value;
    return NEMO_OK;
  }
  if (strcmp(name, "exact_cform") == 0) {
    if (value < 0 || value > 1) return fail(NEMO_ERR_ARG, "exact_cform %d (0 stored, 1 recomputed)", value);
    ctx->c.exact_cform = value;
    return NEMO_OK;
  }
  if (strcmp(name, "exact_xcd") == 0) {
    ctx->c.exact_xcd = value ? 1 : 0;
    return NEMO_OK;
  }
  if (strcmp(name, "exact_sched") == 0) {
    ctx->c.exact_sched = value ? 1 : 0;
    return NEMO_OK;
  }
  if (strcmp(name, "anc_overlap") == 0) {
    ctx->c.anc_overlap = value ? 1 : 0;
    return NEMO_OK;
  }
  if (strcmp(name, "timing_kernel") == 0) {
    if (value < 0 || value > 1) return fail(NEMO_ERR_ARG, "timing_kernel %d (0 score kernels, 1 exact local optima)", value);
    ctx->c.timing_kernel = value;
    return NEMO_OK;
  }
  if (strcmp(name, "exact_persist") == 0) {
    ctx->c.exact_persist = value ? 1 : 0;
    return NEMO_OK;
  }
  if (strcmp(name, "exact_trace") == 0) {
    ctx->c.exact_trace = value ? 1 : 0;
    return NEMO_OK;
  }
  if (strcmp(name, "exact_lat_waves") == 0) {
    if (value < 0) return fail(NEMO_ERR_ARG, "exact_lat_waves %d", value);
    ctx->c.exact_lat_waves = value;
    return NEMO_OK;
  }
  if (strcmp(name, "exact_pair_waves") == 0) {
    if (value < 0) return fail(NEMO_ERR_ARG, "exact_pair_waves %d", value);
    ctx->c.exact_pair_waves = value;
    return NEMO_OK;
  }
  if (strcmp(name, "graphs") == 0) {
    ctx->c.graphs = value ? 1 : 0;
    return NEMO_OK;
  }
  if (strcmp(name, "step_host_sum") == 0) {
    ctx->c.step_host_sum = value ? 1 : 0;
    return NEMO_OK;
  }
  if (strcmp(name, "xcd_remap") == 0) {
    ctx->c.xcd_remap = value ? 1 : 0;
    return NEMO_OK;
  }
  if (strcmp(name, "fact_kernel") == 0) {
    if (value < 0 || value > 20) return fail(NEMO_ERR_ARG, "fact_kernel=%d not in 0..20", value);
    ctx->c.fact_kernel = value;
    if (value == 20) return nemo::i8img_reserve(ctx->c) == hipSuccess ? NEMO_OK
                                                                      : fail(NEMO_ERR_HIP, "fact_kernel 20: image buffer");
    return NEMO_OK;
  }
  if (strcmp(name, "local_prod") == 0) {
    ctx->c.local_prod = value != 0;
    return NEMO_OK;
  }
  if (strcmp(name, "i8o_nodiag") == 0) {
    ctx->c.i8o_nodiag = value != 0;
    return NEMO_OK;
  }
  if (strcmp(name, "local_split") == 0) {
    if (value < 0 || value > 3) return fail(NEMO_ERR_ARG, "local_split=%d not in {0,1,2,3}", value);
    ctx->c.local_split = value;
    return NEMO_OK;
  }
  if (strcmp(name, "score_path") == 0) {
    if (value < 0 || value > 2) return fail(NEMO_ERR_ARG, "score_path=%d not in {0,1,2}", value);
    ctx->c.score_path = value;
    return NEMO_OK;
  }
  return fail(NEMO_ERR_ARG, "unknown option '%s'", name);
}

int nemo_get_option(nemo_ctx* ctx, const char* name, int* value) {
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  if (!name || !value) return fail(NEMO_ERR_ARG, "null argument");
  const Ctx& c = ctx->c;
  if (strcmp(name, "xcd_remap") == 0) *value = c.xcd_remap;
  else if (strcmp(name, "score_path") == 0) *value = c.score_path;
  else if (strcmp(name, "factored") == 0) *value = c.factored ? 1 : 0;
  else if (strcmp(name, "fact_kernel") == 0) *value = c.fact_kernel;
  else if (strcmp(name, "i8o") == 0) *value = c.i8o_ok ? (c.i8o_diag ? 2 : 1) : 0;
  else if (strcmp(name, "i8o_nodiag") == 0) *value = c.i8o_nodiag ? 1 : 0;
  else if (strcmp(name, "i8l") == 0) *value = c.i8l_ok && c.fspad <= 64 ? 1 : 0;
  else if (strcmp(name, "i8w") == 0) *value = c.i8w_ok ? 1 : 0;
  else if (strcmp(name, "local_split") == 0) *value = c.local_split;
  else if (strcmp(name, "graphs") == 0) *value = c.graphs;
  else if (strcmp(name, "exact") == 0) *value = c.exact;
  else if (strcmp(name, "exact_dev") == 0) *value = ctx->exact_dev;
  else if (strcmp(name, "exact_form") == 0) *value = c.exact_form;
  else if (strcmp(name, "exact_cform") == 0) *value = c.exact_cform;
  else if (strcmp(name, "exact_xcd") == 0) *value = c.exact_xcd;
  else if (strcmp(name, "exact_trace") == 0) *value = c.exact_trace;
  else if (strcmp(name, "exact_persist") == 0) *value = c.exact_persist;
  else if (strcmp(name, "timing_kernel") == 0) *value = c.timing_kernel;
  else if (strcmp(name, "exact_sched") == 0) *value = c.exact_sched;
  else if (strcmp(name, "anc_overlap") == 0) *value = c.anc_overlap;
  else if (strcmp(name, "exact_lat_waves") == 0) *value = c.exact_lat_waves;
  else if (strcmp(name, "exact_pair_waves") == 0) *value = c.exact_pair_waves;
  else if (strcmp(name, "exact_ok") == 0) *value = nemo::exact_supported(c) ? 1 : 0;
  else if (strcmp(name, "step_host_sum") == 0) *value = c.step_host_sum;
  else if (strcmp(name, "win") == 0) *value = c.win_ok ? 1 : 0;
  else if (strcmp(name, "local_prod") == 0) *value = c.local_prod && c.table_absmax <= 40.0 ? 1 : 0;
  else return fail(NEMO_ERR_ARG, "unknown option '%s'", name);
  return NEMO_OK;
}

int nemo_refmath_probe(int fn, int n, const double* x, const double* y, double* out) {
  NEMO_API_LOCK;
  if (n < 0 || fn < 0 || fn > 8 || (n > 0 && (!x || !out || ((fn == 3 || fn == 7) && !y))))
    return fail(NEMO_ERR_ARG, "fn=%d n=%d / null pointer", fn, n);
  if (n == 0) return NEMO_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(NEMO_ERR_HIP, "no HIP device visible");
  double *dx = nullptr, *dy = nullptr, *dout = nullptr;
  HIPCHK(hipMalloc((void**)&dx, (size_t)n * 8));
  HIPCHK(hipMalloc((void**)&dout, (size_t)n * 8));
  if (fn == 3 || fn == 7) HIPCHK(hipMalloc((void**)&dy, (size_t)n * 8));
  HIPCHK(hipMemcpy(dx, x, (size_t)n * 8, hipMemcpyHostToDevice));
  if (dy) HIPCHK(hipMemcpy(dy, y, (size_t)n * 8, hipMemcpyHostToDevice));
  HIPCHK(nemo::launch_refmath_probe(fn, n, dx, dy, dout, nullptr));
  HIPCHK(hipMemcpy(out, dout, (size_t)n * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipFree(dx));
  HIPCHK(hipFree(dout));
  if (dy) HIPCHK(hipFree(dy));
  return NEMO_OK;
}

int nemo_set_option_f64(nemo_ctx* ctx, const char* name, double value) {
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  if (!name) return fail(NEMO_ERR_ARG, "null option name");
  if (strcmp(name, "err_budget") == 0) {
    if (!(value >= 0.0)) return fail(NEMO_ERR_ARG, "err_budget=%g must be >= 0", value);
    ++ctx->c.graph_epoch;
    ctx->c.err_budget = value;
    return NEMO_OK;
  }
  return fail(NEMO_ERR_ARG, "unknown f64 option '%s'", name);
}

int nemo_get_option_f64(nemo_ctx* ctx, const char* name, double* value) {
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  if (!name || !value) return fail(NEMO_ERR_ARG, "null argument");
  const Ctx& c = ctx->c;
  if (strcmp(name, "err_budget") == 0) {
    *value = c.err_budget;
    return NEMO_OK;
  }
  const bool l2 = strcmp(name, "i8l_bound") == 0, nat = strcmp(name, "i8o_bound") == 0;
  if (l2 || nat) {
    if (!c.staged || c.fx_colsum.empty()) return fail(NEMO_ERR_STATE, "no factored model staged");
    *value = nemo::host::fixed_point_bound(l2 ? nemo::host::kFxLog2 : nemo::host::kFxNatural, c.i8_cexp,
                                           c.fx_colsum, c.S, c.E, 0);
    return NEMO_OK;
  }
  return fail(NEMO_ERR_ARG, "unknown f64 option '%s'", name);
}

int nemo_score_kernel(nemo_ctx* ctx, int cap, int ll_only, int* fact_kernel, double* bound) {
  int rc = check_ctx(ctx, true);
  if (rc) return rc;
  if (cap < 0 || !fact_kernel) return fail(NEMO_ERR_ARG, "cap=%d / null fact_kernel", cap);
  const Ctx& c = ctx->c;
  double b = 0.0;
  *fact_kernel = use_factored(c) ? nemo::resolve_fact_kernel(c, cap, ll_only != 0, &b) : -1;
  if (bound) *bound = b;
  return NEMO_OK;
}

const char* nemo_build_id(void) {
#ifdef NEMO_BUILD_ID
  return NEMO_BUILD_ID;
#else
  return "unversioned";
#endif
}

// ---------------------------------------------------------------------------
// timing
// ---------------------------------------------------------------------------
int nemo_timing_enable(nemo_ctx* ctx, int enable) {
  NEMO_API_LOCK;
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  Ctx& c = ctx->c;
  HIPCHK(hipStreamSynchronize(c.stream));
  ++c.graph_epoch;
  c.timing = enable != 0;
  c.ev_used = 0;
  c.launches = 0;
  c.timed_ms = 0.0;
  if (c.timing && c.ev_pool.empty()) {
    c.ev_pool.resize(8192);
    for (auto& ev : c.ev_pool) HIPCHK(hipEventCreate(&ev));
  }
  return NEMO_OK;
}

int nemo_timing_read(nemo_ctx* ctx, double* total_ms, int* launches) {
  int rc = check_ctx(ctx, false);
  if (rc) return rc;
  Ctx& c = ctx->c;
  double tot = 0.0;
  for (size_t k = 0; k + 1 < c.ev_used; k += 2) {
    HIPCHK(hipEventSynchronize(c.ev_pool[k + 1]));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, c.ev_pool[k], c.ev_pool[k + 1]));
    tot += ms;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = c.launches;
  return NEMO_OK;
}

}  // extern "C"
