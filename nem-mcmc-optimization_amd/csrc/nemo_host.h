// nemo_host.h -- the host logic of the C-ABI that needs no HIP: argument
// checks, the worst-case error bounds of the fixed-point score kernels, the
// level schedule of InverseMethod's pair loop and the queue of asynchronous
// fused steps.  Header-only so that tests/host/host_check.cpp builds it with
// plain g++ under AddressSanitizer, UndefinedBehaviorSanitizer and
// ThreadSanitizer (tests/test_host_sanitizers.py); nemo_abi.cpp is its only
// product user.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

namespace nemo {
namespace host {

// index of the first row of pos [batch][S] that is not a permutation of
// 0..S-1, or -1 (nemo_score / nemo_optimal_weights / methods argument check)
inline int first_bad_pos_row(const int32_t* pos, int batch, int S) {
  std::vector<char> seen((size_t)std::max(S, 1));
  for (int b = 0; b < batch; ++b) {
    std::fill(seen.begin(), seen.end(), 0);
    for (int i = 0; i < S; ++i) {
      const int p = pos[(size_t)b * S + i];
      if (p < 0 || p >= S || seen[p]) return b;
      seen[p] = 1;
    }
  }
  return -1;
}

// ---------------------------------------------------------------------------
// Staging validation: the factored form of a score table
// ---------------------------------------------------------------------------
// Every table nem.py builds (nem.py:44-46) has off-diagonal rows T[i][j]
// shared by all children i != j and two-valued: lo_j = the row's first value,
// bit d1[j][e] = 1 where it takes the other value hi_j.  T [S][S][E];
// d1 [S][nwords] (nwords = ceil(E / 64)), elo / ehi [S] = exp(lo_j), exp(hi_j).
// Returns false (outputs unspecified) when T lacks that structure.
inline bool detect_factored(int S, int E, const double* T, std::vector<uint64_t>& d1, std::vector<double>& elo,
                            std::vector<double>& ehi, std::vector<double>* tlo = nullptr,
                            std::vector<double>* thi = nullptr) {
  const int nwords = (E + 63) / 64;
  d1.assign((size_t)S * nwords, 0ull);
  elo.assign(S, 0.0);
  ehi.assign(S, 0.0);
  if (tlo) tlo->assign(S, 0.0);
  if (thi) thi->assign(S, 0.0);
  for (int j = 0; j < S; ++j) {
    const int i0 = (j == 0) ? 1 : 0;
    const double* L = T + ((size_t)i0 * S + j) * E;
    for (int i = 0; i < S; ++i)
      if (i != j && i != i0 && !std::equal(L, L + E, T + ((size_t)i * S + j) * E)) return false;
    const double lo = L[0];
    double hi = lo;
    bool have_hi = false;
    for (int e = 0; e < E; ++e) {
      const double v = L[e];
      if (v == lo) continue;
      if (!have_hi) {
        hi = v;
        have_hi = true;
      }
      if (v != hi) return false;
      d1[(size_t)j * nwords + e / 64] |= 1ull << (e % 64);
    }
    elo[j] = std::exp(lo);
    ehi[j] = std::exp(hi);
    if (tlo) (*tlo)[j] = lo;
    if (thi) (*thi)[j] = hi;
  }
  return true;
}

// the same from the knockdown matrix D [S][E] in {0,1} (nem.py:25-64): row j
// of T is where(D[j] == 0, B, -A), so lo_j = (D[j][0] ? -A : B)
inline void knockdown_factored(int S, int E, const uint8_t* D, double A, double B, std::vector<uint64_t>& d1,
                               std::vector<double>& elo, std::vector<double>& ehi,
                               std::vector<double>* tlo = nullptr, std::vector<double>* thi = nullptr) {
  const int nwords = (E + 63) / 64;
  d1.assign((size_t)S * nwords, 0ull);
  elo.assign(S, 0.0);
  ehi.assign(S, 0.0);
  if (tlo) tlo->assign(S, 0.0);
  if (thi) thi->assign(S, 0.0);
  const double negA = -A;
  for (int j = 0; j < S; ++j) {
    const uint8_t* r = D + (size_t)j * E;
    const double lo = r[0] ? negA : B;
    double hi = lo;
    for (int e = 0; e < E; ++e) {
      const double v = r[e] ? negA : B;
      if (v == lo) continue;
      hi = v;
      d1[(size_t)j * nwords + e / 64] |= 1ull << (e % 64);
    }
    elo[j] = std::exp(lo);
    ehi[j] = std::exp(hi);
    if (tlo) (*tlo)[j] = lo;
    if (thi) (*thi)[j] = hi;
  }
}

// ---------------------------------------------------------------------------
// numpy's pairwise summation of an E-vector (DOUBLE_pairwise_sum, blocks of
// <= 128 with 8 accumulators, halving at multiples of 8) laid out over one
// wave for the exact local optimum (nemo_exact.hip): leaf block L (in order)
// owns 8 accumulator chains -- lanes 8 (L % 8) .. + 7 of register slot L / 8
// -- each chain its elements start + k + 8 m, its block's n % 8 trailing
// elements one per lane of the same group, and the recursion's additions run
// as one level per height, the node's value at its first leaf's lane.
// ---------------------------------------------------------------------------
struct PairwisePlan {
  int E = 0, nleaf = 0, ns = 0, nh = 0, maxrem = 0;
  // [ns][64] per (slot, lane): chain start element (-1: none), its element
  // count, the group's trailing element of this lane (-1: none), the group's
  // trailing count; [nh][64]: the lane whose value to add at that height (-1)
  std::vector<int32_t> start, cnt, rem, nrem, partner;
};

// the plan of elements [off, off + n) (numpy's recursion on that range; the
// plan's element indices are absolute)
inline bool build_pairwise_plan_range(long off, long n, PairwisePlan& pl);
inline bool build_pairwise_plan(int E, PairwisePlan& pl) { return build_pairwise_plan_range(0, E, pl); }

inline bool build_pairwise_plan_range(long off, long E, PairwisePlan& pl) {
  struct Leaf { long s, n; };
  std::vector<Leaf> leaves;
  struct Op { int h, lane, partner; };
  std::vector<Op> ops;
  // returns (first leaf, height)
  std::function<std::pair<int, int>(long, long)> rec = [&](long s, long n) -> std::pair<int, int> {
    if (n <= 128) {
      leaves.push_back({s, n});
      return {(int)leaves.size() - 1, 0};
    }
    long n2 = n / 2;
    n2 -= n2 % 8;
    const auto l = rec(s, n2);
    const auto r = rec(s + n2, n - n2);
    const int h = 1 + std::max(l.second, r.second);
    ops.push_back({h, l.first, r.first});
    return {l.first, h};
  };
  if (E < 1) return false;
  const int root_h = rec(off, E).second;
  pl = PairwisePlan{};
  pl.E = (int)(off + E);
  pl.nleaf = (int)leaves.size();
  if (pl.nleaf > 64) return false;  // one leaf result per lane for the tree
  pl.ns = (8 * pl.nleaf + 63) / 64;
  pl.nh = root_h;
  pl.start.assign((size_t)pl.ns * 64, -1);
  pl.cnt.assign((size_t)pl.ns * 64, 0);
  pl.rem.assign((size_t)pl.ns * 64, -1);
  pl.nrem.assign((size_t)pl.ns * 64, 0);
  pl.partner.assign((size_t)std::max(pl.nh, 1) * 64, -1);
  for (int L = 0; L < pl.nleaf; ++L) {
    const long s = leaves[L].s, n = leaves[L].n;
    const int u = L / 8, base = 8 * (L % 8);
    const long full = n >= 8 ? n - n % 8 : 0;   // n < 8 (E < 8): no chains, sum from 0.0
    const int nr = (int)(n - full);
    if (nr > 7) return false;
    pl.maxrem = std::max(pl.maxrem, nr);
    for (int k = 0; k < 8; ++k) {
      const size_t q = (size_t)u * 64 + base + k;
      if (full) {
        pl.start[q] = (int32_t)(s + k);
        pl.cnt[q] = (int32_t)(full / 8);
      }
      pl.rem[q] = k < nr ? (int32_t)(s + full + k) : -1;
      pl.nrem[q] = nr;
    }
  }
  for (const Op& o : ops) pl.partner[(size_t)(o.h - 1) * 64 + o.lane] = o.partner;
  return true;
}

// np.sum of more than 8192 terms: numpy's reduction runs its inner loop on
// buffer-sized chunks (np.getbufsize() = 8192 by default), each summed
// pairwise and added to the running result in order -- sum = ((pw(c0) +
// pw(c1)) + pw(c2)) + ..., measured against numpy 2.2 (tools/mp_probe.py,
// DESIGN.md 3.5e).  Each chunk of <= 8192 terms fits one wave plan (<= 64
// leaf blocks), so E takes ceil(E / 8192) plans with absolute element
// indices.  One part when E <= 8192.
constexpr long kNumpyBufsize = 8192;
inline bool build_pairwise_parts(int E, std::vector<PairwisePlan>& parts, int max_parts = 64) {
  parts.clear();
  if (E < 1) return false;
  const long np = (E + kNumpyBufsize - 1) / kNumpyBufsize;
  if (np > max_parts) return false;
  parts.assign((size_t)np, PairwisePlan{});
  for (long p = 0; p < np; ++p) {
    const long off = p * kNumpyBufsize, n = std::min<long>(kNumpyBufsize, E - off);
    if (!build_pairwise_plan_range(off, n, parts[(size_t)p])) {
      parts.clear();
      return false;
    }
  }
  return true;
}

// the parts' device rows, each padded to nsp slots: per part [start | cnt |
// rem | nrem] x [nsp][64] then partner [8][64] (-1: none); meta [part][2] =
// (tree height, largest trailing count)
inline int parts_slots(const std::vector<PairwisePlan>& parts) {
  int nsp = 0;
  for (const auto& p : parts) nsp = std::max(nsp, p.ns);
  return nsp;
}
inline void parts_device_rows(const std::vector<PairwisePlan>& parts, std::vector<int32_t>& dev,
                              std::vector<int32_t>& meta) {
  const int nsp = parts_slots(parts);
  dev.clear();
  meta.clear();
  for (const auto& p : parts) {
    auto pad = [&](const std::vector<int32_t>& v, int32_t fill) {
      for (int u = 0; u < nsp; ++u)
        for (int l = 0; l < 64; ++l) dev.push_back(u < p.ns ? v[(size_t)u * 64 + l] : fill);
    };
    pad(p.start, -1);
    pad(p.cnt, 0);
    pad(p.rem, -1);
    pad(p.nrem, 0);
    for (int h = 0; h < 8; ++h)
      for (int l = 0; l < 64; ++l) dev.push_back(h < p.nh ? p.partner[(size_t)h * 64 + l] : -1);
    meta.push_back(p.nh);
    meta.push_back(p.maxrem);
  }
}

// Where each element e sits in a plan-ordered row set ([ns][17][64] doubles:
// chain element m of slot u on lane l at (u * 17 + m) * 64 + l, the lane's
// trailing element at row 16): pos[e], every e < E exactly once.
inline void plan_positions(const PairwisePlan& pl, std::vector<int32_t>& pos) {
  pos.assign((size_t)pl.E, -1);
  for (int u = 0; u < pl.ns; ++u)
    for (int l = 0; l < 64; ++l) {
      const size_t q = (size_t)u * 64 + l;
      for (int m = 0; m < pl.cnt[q]; ++m) pos[(size_t)pl.start[q] + 8 * m] = (u * 17 + m) * 64 + l;
      if (pl.rem[q] >= 0) pos[(size_t)pl.rem[q]] = (u * 17 + 16) * 64 + l;
    }
}

// The D1 bit of parent row k at each lane's plan elements: bits[(k * ns + u)
// * 64 + l], bit m = element m of the lane's chain in slot u, bit 16 = its
// trailing element (0 where there is none)
inline void plan_lv_bits(const PairwisePlan& pl, int S, const uint64_t* d1, int nwords, std::vector<uint32_t>& bits) {
  bits.assign((size_t)S * pl.ns * 64, 0u);
  auto bit = [&](int k, long e) { return (uint32_t)((d1[(size_t)k * nwords + e / 64] >> (e % 64)) & 1ull); };
  for (int k = 0; k < S; ++k)
    for (int u = 0; u < pl.ns; ++u)
      for (int l = 0; l < 64; ++l) {
        const size_t q = (size_t)u * 64 + l;
        uint32_t w = 0;
        for (int m = 0; m < pl.cnt[q]; ++m) w |= bit(k, (long)pl.start[q] + 8 * m) << m;
        if (pl.rem[q] >= 0) w |= bit(k, pl.rem[q]) << 16;
        bits[((size_t)k * pl.ns + u) * 64 + l] = w;
      }
}

// plan_positions / plan_lv_bits over parts: part p's slot u is slot p nsp + u
inline void parts_positions(const std::vector<PairwisePlan>& parts, int E, std::vector<int32_t>& pos) {
  const int nsp = parts_slots(parts);
  pos.assign((size_t)E, -1);
  for (size_t p = 0; p < parts.size(); ++p) {
    const PairwisePlan& pl = parts[p];
    for (int u = 0; u < pl.ns; ++u)
      for (int l = 0; l < 64; ++l) {
        const size_t q = (size_t)u * 64 + l;
        const int gu = (int)p * nsp + u;
        for (int m = 0; m < pl.cnt[q]; ++m) pos[(size_t)pl.start[q] + 8 * m] = (gu * 17 + m) * 64 + l;
        if (pl.rem[q] >= 0) pos[(size_t)pl.rem[q]] = (gu * 17 + 16) * 64 + l;
      }
  }
}
inline void parts_lv_bits(const std::vector<PairwisePlan>& parts, int S, const uint64_t* d1, int nwords,
                          std::vector<uint32_t>& bits) {
  const int nsp = parts_slots(parts), ns = (int)parts.size() * nsp;
  bits.assign((size_t)S * ns * 64, 0u);
  for (size_t p = 0; p < parts.size(); ++p) {
    std::vector<uint32_t> b;
    plan_lv_bits(parts[p], S, d1, nwords, b);
    for (int k = 0; k < S; ++k)
      for (int u = 0; u < parts[p].ns; ++u)
        for (int l = 0; l < 64; ++l)
          bits[((size_t)k * ns + p * nsp + u) * 64 + l] = b[((size_t)k * parts[p].ns + u) * 64 + l];
  }
}

// the two addition chains of compute_scores (nem.py:25-34), in its order:
// chains[k] = 0 + A + ... (k times), chains[S + 1 + k] = B + A + ... (k times)
inline std::vector<double> knockdown_chains(int S, double A, double B) {
  std::vector<double> chains(2 * ((size_t)S + 1));
  chains[0] = 0.0;
  chains[(size_t)S + 1] = B;
  for (int k = 1; k <= S; ++k) {
    chains[k] = chains[k - 1] + A;
    chains[(size_t)S + 1 + k] = chains[(size_t)S + k] + A;
  }
  return chains;
}

// ---------------------------------------------------------------------------
// Worst-case |ll error| of the fixed-point score kernels
// ---------------------------------------------------------------------------
// The int8 kernels round every entry of the contraction once: Delta[i][j] of
// each permissible parent j, the free diagonal entry u1_i - u0_i and the row
// constant G_i (+ u0_i).  Those roundings are fixed per (child, parent) and
// repeat over the effects, so they add over effects instead of averaging out.
// At effect e the cell of child i carries one rounding per parent whose D1 bit
// is set at e, one for its own bit and one for G: at most
// min(colbits_e, k) + 1 terms, colbits_e = the number of rows with D1[.][e] = 1
// and k = S without a cap (k = cap + 1 with one: the parents and the child
// itself).  The column log-sum-exp is a convex combination of the rows, so its
// error is at most the largest cell error, and ll sums the columns:
//     |d ll| <= eps * sum_e (min(colbits_e, k) + 1) + E * series,
// eps = 2^-39 ln 2 for score_i8l_kernel (7 digit slices of x / ln 2 at
// 2^-38) and 2^(c - 49) for the 8-slice kernels, series = the relative error of
// each exp's assembly (score_i8l: degree-2 polynomial within 2.9e-13, plus the
// table entry and the product; the 8-slice kernels: degree 3, < 4e-17).
//
// colsum[k] = sum_e min(colbits_e, k), k = 0..S, from the staged D1 bits
// (d1 [S][nwords], bit e % 64 of word e / 64).
inline std::vector<double> fixed_point_colsums(int S, int E, const uint64_t* d1, int nwords) {
  std::vector<int> hist((size_t)S + 1, 0);  // effects with colbits_e == n
  for (int e = 0; e < E; ++e) {
    int n = 0;
    for (int j = 0; j < S; ++j) n += (int)((d1[(size_t)j * nwords + e / 64] >> (e % 64)) & 1ull);
    ++hist[n];
  }
  std::vector<double> colsum((size_t)S + 1, 0.0);
  for (int k = 0; k <= S; ++k) {
    double s = 0.0;
    for (int n = 0; n <= S; ++n) s += (double)hist[n] * (double)std::min(n, k);
    colsum[k] = s;
  }
  return colsum;
}

enum FixedPointKind { kFxLog2 = 0, kFxNatural = 1 };

// the bound above for a call with parent cap `cap` (0 = none; a cap >= S - 1
// is no cap); cexp = the model's int8 scale exponent (Ctx::i8_cexp)
inline double fixed_point_bound(int kind, int cexp, const std::vector<double>& colsum, int S, int E, int cap) {
  if (colsum.size() != (size_t)S + 1) return INFINITY;
  const int k = (cap > 0 && cap < S - 1) ? std::min(cap + 1, S) : S;
  const double terms = colsum[(size_t)k] + (double)E;
  if (kind == kFxLog2) {
    // half a unit of 2^-38 in y = x / ln 2, with 2^-10 of slack for the fp64
    // products that form the digits
    const double eps = std::ldexp(0.69314718055994530942, -39) * (1.0 + std::ldexp(1.0, -10));
    return eps * terms + 3.0e-13 * (double)E;
  }
  return std::ldexp(1.0, cexp - 49) * (1.0 + std::ldexp(1.0, -10)) * terms + 1.0e-16 * (double)E;
}

// ---------------------------------------------------------------------------
// InverseMethod.opt_b's pair loop as levels of independent pairs
// ---------------------------------------------------------------------------
// order_arr (utils.py:173-188) arranges a matrix by argsort(order) = pos:
// row/column a of M is node pos[a], so node i sits at index perm[i].
// InverseMethod.opt_b's loop (methods.py:125-127) visits, for i = 0..S-1,
// k = order[0 .. pos[i]-1].  Pair (i, k) moves M[a][b], a = perm[i],
// b = perm[k]; only a > b is inside the lower triangle solve_triangular
// reads.  Its objective reads B[a][b], i.e. the entries M[r][c] with
// b ~> c and r ~> a in the graph of lower-triangle pairs (~> : reachable,
// reflexive).  Levels: a pair goes after every earlier pair it reads and no
// earlier than any earlier pair that reads it (those must see its old
// value; a level reads before it commits).  One level = one launch.
// Entries: prob << 16 | i << 8 | k (S <= 256, nprob <= 32767).
struct InverseSchedule {
  std::vector<int32_t> pos;        // the orders the schedule was built for
  std::vector<int32_t> list;       // pair entries, level by level
  std::vector<int> level_off;      // level l = list[off[l] .. off[l+1])
  std::vector<int32_t> skip;       // permissible pairs outside the lower triangle
};

// true when `sch` already holds the schedule of these orders
inline bool build_inverse_schedule(InverseSchedule& sch, int S, int nprob, const int32_t* pos) {
  const size_t n = (size_t)nprob * S;
  if (sch.pos.size() == n && !sch.level_off.empty() && std::equal(pos, pos + n, sch.pos.begin()))
    return true;
  sch.pos.assign(pos, pos + n);
  std::vector<std::vector<int32_t>> levels;
  sch.skip.clear();
  const int W = (S + 63) / 64;
  for (int b = 0; b < nprob; ++b) {
    const int32_t* pb = pos + (size_t)b * S;
    std::vector<int> perm(S);
    for (int i = 0; i < S; ++i) perm[pb[i]] = i;
    // pairs in loop order
    std::vector<int> pa, pbb, pi;
    for (int i = 0; i < S; ++i)
      for (int p = 0; p < pb[i]; ++p) {
        const int k = perm[p];
        const int ra = perm[i], rb = perm[k];
        const int32_t ent = (b << 16) | (i << 8) | k;
        if (ra > rb) {
          pa.push_back(ra);
          pbb.push_back(rb);
          pi.push_back(ent);
        } else {
          sch.skip.push_back(ent);
        }
      }
    // reach[x] = bitset of y with y ~> x
    std::vector<uint64_t> reach((size_t)S * W, 0ull);
    std::vector<char> edge((size_t)S * S, 0);
    for (size_t q = 0; q < pa.size(); ++q) edge[(size_t)pa[q] * S + pbb[q]] = 1;
    for (int x = 0; x < S; ++x) {
      uint64_t* rx = &reach[(size_t)x * W];
      rx[x >> 6] |= 1ull << (x & 63);
      for (int d = 0; d < x; ++d)
        if (edge[(size_t)x * S + d])
          for (int w = 0; w < W; ++w) rx[w] |= reach[(size_t)d * W + w];
    }
    auto r = [&](int x, int y) { return (reach[(size_t)x * W + (y >> 6)] >> (y & 63)) & 1ull; };
    const size_t P = pa.size();
    std::vector<int> lev(P, 0);
    for (size_t p = 0; p < P; ++p) {
      const int a2 = pa[p], b2 = pbb[p];
      int l = 0;
      for (size_t q = 0; q < p; ++q) {
        const int a1 = pa[q], b1 = pbb[q];
        if (r(b1, b2) && r(a2, a1)) l = std::max(l, lev[q] + 1);  // p reads q
        if (r(b2, b1) && r(a1, a2)) l = std::max(l, lev[q]);      // q reads p
      }
      lev[p] = l;
      if ((int)levels.size() <= l) levels.resize(l + 1);
      levels[l].push_back(pi[p]);
    }
  }
  sch.list.clear();
  sch.level_off.assign(1, 0);
  for (auto& lv : levels) {
    sch.list.insert(sch.list.end(), lv.begin(), lv.end());
    sch.level_off.push_back((int)sch.list.size());
  }
  return false;
}

// ---------------------------------------------------------------------------
// The device's fixed-order sum of an evaluation's n partials (sum_partials in
// nemo_internal.h: lane l sums p[l], p[l + 64], ... in order, then six xor
// butterfly stages, lane 0's value) restated on the host, operation for
// operation: IEEE additions in the same order give the same bits.  The fused
// step's staged path copies eval #2's partials out with its other outputs and
// sums them here instead of in a finalize launch.
// ---------------------------------------------------------------------------
inline double sum_partials_host(const double* p, int n) {
  constexpr int kLanes = 64;
  double v[kLanes];
  for (int l = 0; l < kLanes; ++l) {
    double s = 0.0;
    for (int t = l; t < n; t += kLanes) s += p[t];
    v[l] = s;
  }
  for (int o = kLanes / 2; o >= 1; o >>= 1) {
    double w[kLanes];
    for (int l = 0; l < kLanes; ++l) w[l] = v[l] + v[l ^ o];
    for (int l = 0; l < kLanes; ++l) v[l] = w[l];
  }
  return v[0];
}

// ---------------------------------------------------------------------------
// Queue of asynchronous calls run in submission order on one library thread
// (nemo_optimal_weights_begin / _end)
// ---------------------------------------------------------------------------
// submit() hands a job to the worker (started on first use) and returns at
// once; collect() waits for the oldest job not yet collected and hands it
// back.  The destructor lets every job already submitted run to completion
// (their callers' output buffers are written even if never collected), then
// stops the worker; jobs not collected by then are freed.
//
// Two forms.  StepQueue(run): the worker runs each job to completion in turn.
// StepQueue(start, ready, finish, depth): a job is started (queued on the
// device; true = in flight, false = already complete, e.g. failed), and up to
// `depth` jobs are in flight at once; the oldest is finished (waited for,
// outputs handed back) when no further job can start, as soon as ready()
// reports its device work done -- so a job submitted while the device still
// runs the previous one is started before that one is waited for, and the
// device goes from one job to the next without waiting for the host.
template <class Job>
class StepQueue {
 public:
  using Runner = std::function<void(Job&)>;
  using Start = std::function<bool(Job&)>;
  using Ready = std::function<bool(Job&)>;
  using Finish = std::function<void(Job&)>;
  explicit StepQueue(Runner run)
      : start_([run](Job& j) {
          run(j);
          return false;
        }),
        depth_(1) {}
  StepQueue(Start start, Ready ready, Finish finish, int depth)
      : start_(std::move(start)), ready_(std::move(ready)), finish_(std::move(finish)),
        depth_(depth < 1 ? 1 : depth) {}
  StepQueue(const StepQueue&) = delete;
  StepQueue& operator=(const StepQueue&) = delete;
  ~StepQueue() { shutdown(); }

  // false (and *err set, nothing queued) if the job or the worker thread
  // could not be created; never throws
  bool submit(std::unique_ptr<Job> job, std::string* err) {
    try {
      std::lock_guard<std::mutex> g(mu_);
      if (stop_) {
        if (err) *err = "queue is shut down";
        return false;
      }
      jobs_.push_back(Entry{std::move(job), false});
      if (!worker_.joinable()) {
        try {
          worker_ = std::thread(&StepQueue::loop, this);
        } catch (...) {
          jobs_.pop_back();
          throw;
        }
      }
    } catch (const std::system_error& e) {
      if (err) *err = std::string("could not start the step thread: ") + e.what();
      return false;
    } catch (const std::bad_alloc&) {
      if (err) *err = "out of host memory queueing a step";
      return false;
    }
    cv_.notify_all();
    return true;
  }

  // the oldest job not yet collected, after it has run; nullptr if none
  std::unique_ptr<Job> collect() {
    std::unique_lock<std::mutex> lk(mu_);
    if (jobs_.empty()) return nullptr;
    cv_.wait(lk, [this] { return jobs_.front().done; });
    std::unique_ptr<Job> j = std::move(jobs_.front().job);
    jobs_.pop_front();
    --next_start_;
    return j;
  }

  // jobs submitted and not yet collected
  size_t pending() const {
    std::lock_guard<std::mutex> g(mu_);
    return jobs_.size();
  }

  // run every submitted job, then stop the worker (idempotent)
  void shutdown() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
    std::lock_guard<std::mutex> g(mu_);
    jobs_.clear();
    next_start_ = 0;
  }

 private:
  struct Entry {
    std::unique_ptr<Job> job;
    bool done;
  };
  static constexpr int kPollUs = 20;  // in-flight job's readiness poll while no new job is queued

  void mark_done(Job* j) {  // under mu_
    for (auto& e : jobs_)
      if (e.job.get() == j) {
        e.done = true;
        break;
      }
    cv_.notify_all();
  }

  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    std::deque<Job*> flying;  // started, not finished, oldest first
    for (;;) {
      // collect() only pops entries that are done, and none at or past
      // next_start_ is, so jobs_[next_start_] is the next job to start
      if (next_start_ < jobs_.size() && (int)flying.size() < depth_) {
        Job* j = jobs_[next_start_].job.get();
        ++next_start_;
        lk.unlock();
        const bool fly = start_(*j);
        lk.lock();
        if (fly) flying.push_back(j);
        else mark_done(j);
        continue;
      }
      if (!flying.empty()) {
        Job* j = flying.front();
        if ((int)flying.size() < depth_ && !stop_) {
          // a slot is free but nothing to start: finish the oldest once its
          // device work is done, and start a job that arrives meanwhile first
          lk.unlock();
          const bool rdy = ready_(*j);
          lk.lock();
          if (!rdy) {
            // (system_clock: pthread_cond_timedwait, which ThreadSanitizer
            // intercepts; a steady_clock wait maps to pthread_cond_clockwait)
            cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::microseconds(kPollUs),
                           [this] { return stop_ || next_start_ < jobs_.size(); });
            continue;
          }
        }
        flying.pop_front();
        lk.unlock();
        finish_(*j);
        lk.lock();
        mark_done(j);
        continue;
      }
      if (stop_ && next_start_ >= jobs_.size()) return;  // nothing queued or in flight
      cv_.wait(lk, [this] { return stop_ || next_start_ < jobs_.size(); });
    }
  }

  Start start_;
  Ready ready_;
  Finish finish_;
  int depth_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Entry> jobs_;  // submitted and not yet collected, oldest first
  size_t next_start_ = 0;   // jobs_[next_start_..] have not started
  bool stop_ = false;
  std::thread worker_;
};

}  // namespace host
}  // namespace nemo
