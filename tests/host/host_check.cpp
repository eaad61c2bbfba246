// host_check.cpp -- the C-ABI's host logic (nem-mcmc-optimization_amd/csrc/
// nemo_host.h) driven on the CPU, built by tests/test_host_sanitizers.py with
// g++ under -fsanitize=address,undefined and, separately, -fsanitize=thread.
// Prints "ok <checks>" and exits 0, or names the first failed check and
// exits 1.  No HIP: this is the part of libnemo.so that never touches a GPU.
#include "nemo_host.h"

#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <random>
#include <map>
#include <set>

using namespace nemo::host;

static int g_checks = 0;
#define CHECK(cond)                                                        \
  do {                                                                     \
    ++g_checks;                                                            \
    if (!(cond)) {                                                         \
      fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);   \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

// ---- argument checks -------------------------------------------------------
static void check_pos_rows() {
  std::vector<int32_t> pos = {0, 1, 2, 2, 0, 1, 1, 1, 0};
  CHECK(first_bad_pos_row(pos.data(), 2, 3) == -1);
  CHECK(first_bad_pos_row(pos.data(), 3, 3) == 2);
  std::vector<int32_t> neg = {0, -1};
  CHECK(first_bad_pos_row(neg.data(), 1, 2) == 0);
  std::vector<int32_t> big = {0, 2};
  CHECK(first_bad_pos_row(big.data(), 1, 2) == 0);
  CHECK(first_bad_pos_row(nullptr, 0, 5) == -1);
}

// ---- staging validation --------------------------------------------------------
// A table built the way nem.py builds it (off-diagonal row j = where(D[j] == 0,
// B, -A) for every child) is detected as factored with exactly the D1 bits and
// exp values the knockdown staging derives from D itself; any perturbation of
// one off-diagonal entry breaks the structure.
static void check_staging(std::mt19937_64& rng) {
  for (int trial = 0; trial < 30; ++trial) {
    const int S = 2 + (int)(rng() % 20), E = 1 + (int)(rng() % 200);
    const double A = -2.8904, B = -2.2513 - 0.01 * trial;
    std::vector<uint8_t> D((size_t)S * E);
    for (auto& d : D) d = (uint8_t)(rng() % 3 == 0);
    std::vector<double> T((size_t)S * S * E);
    for (int i = 0; i < S; ++i)
      for (int j = 0; j < S; ++j)
        for (int e = 0; e < E; ++e)
          T[((size_t)i * S + j) * E + e] =
              i == j ? 0.25 * (double)(rng() % 9) : (D[(size_t)j * E + e] ? -A : B);
    std::vector<uint64_t> d1a, d1b;
    std::vector<double> loa, hia, lob, hib;
    CHECK(detect_factored(S, E, T.data(), d1a, loa, hia));
    knockdown_factored(S, E, D.data(), A, B, d1b, lob, hib);
    CHECK(d1a == d1b && loa == lob);
    for (int j = 0; j < S; ++j) {
      bool any = false;
      for (int e = 0; e < E; ++e) any |= ((d1a[(size_t)j * ((E + 63) / 64) + e / 64] >> (e % 64)) & 1) != 0;
      if (any) CHECK(hia[j] == hib[j]);  // hi_j only matters where a bit is set
    }
    if (S > 2) {
      const int j = (int)(rng() % S), i = (j + 1 + (int)(rng() % (S - 1))) % S, e = (int)(rng() % E);
      std::vector<double> T2 = T;
      T2[((size_t)i * S + j) * E + e] += 1e-12;
      CHECK(!detect_factored(S, E, T2.data(), d1a, loa, hia));
    }
  }
  const std::vector<double> ch = knockdown_chains(3, 0.5, -1.0);
  CHECK(ch.size() == 8 && ch[0] == 0.0 && ch[3] == 1.5 && ch[4] == -1.0 && ch[7] == 0.5);
}

// ---- error bounds ------------------------------------------------------------
static void check_bounds(std::mt19937_64& rng) {
  for (int trial = 0; trial < 20; ++trial) {
    const int S = 2 + (int)(rng() % 70), E = 1 + (int)(rng() % 300);
    const int nwords = (E + 63) / 64;
    std::vector<uint64_t> d1((size_t)S * nwords);
    const uint64_t dens = rng() % 4;
    for (auto& w : d1) {
      w = rng();
      for (uint64_t k = 0; k < dens; ++k) w &= rng();
    }
    // bits past E are padding: the colsums must not read them
    for (int j = 0; j < S; ++j)
      if (E % 64) d1[(size_t)j * nwords + nwords - 1] &= (1ull << (E % 64)) - 1;
    const std::vector<double> cs = fixed_point_colsums(S, E, d1.data(), nwords);
    CHECK(cs.size() == (size_t)S + 1);
    for (int k = 0; k <= S; ++k) {
      double ref = 0.0;
      for (int e = 0; e < E; ++e) {
        int n = 0;
        for (int j = 0; j < S; ++j) n += (int)((d1[(size_t)j * nwords + e / 64] >> (e % 64)) & 1);
        ref += std::min(n, k);
      }
      CHECK(cs[(size_t)k] == ref);
    }
    // a cap never raises the bound; no cap equals cap >= S - 1
    const int cexp = (int)(rng() % 6);
    for (int kind : {kFxLog2, kFxNatural}) {
      const double b0 = fixed_point_bound(kind, cexp, cs, S, E, 0);
      CHECK(b0 > 0.0 && std::isfinite(b0));
      CHECK(fixed_point_bound(kind, cexp, cs, S, E, S - 1) == b0);
      double prev = 0.0;
      for (int cap = 1; cap < S - 1; ++cap) {
        const double b = fixed_point_bound(kind, cexp, cs, S, E, cap);
        CHECK(b <= b0 && b >= prev);
        prev = b;
      }
    }
    // the worst case the formula can reach: every row's bit set everywhere
    const double full = fixed_point_bound(kFxLog2, 0, std::vector<double>(cs.size(), 0.0), S, E, 0);
    CHECK(full > 0.0);
  }
  // a colsum vector of the wrong size is no bound at all
  CHECK(std::isinf(fixed_point_bound(kFxLog2, 0, std::vector<double>(3, 0.0), 5, 10, 0)));
}

// ---- InverseMethod level schedule ---------------------------------------------
// The reference's pair loop (methods.py:125-127) updates the pairs one at a
// time, each reading the entries its objective depends on (b ~> c and r ~> a
// in the graph of lower-triangle pairs).  The schedule runs a level's pairs
// together, all reading the state before the level.  Simulate both with an
// opaque update (a hash of everything read) and require the same final state.
static uint64_t mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  return h * 0xff51afd7ed558ccdull;
}

static void check_inverse_schedule(std::mt19937_64& rng) {
  for (int trial = 0; trial < 60; ++trial) {
    const int S = 2 + (int)(rng() % 24), nprob = 1 + (int)(rng() % 3);
    std::vector<int32_t> pos((size_t)nprob * S);
    for (int b = 0; b < nprob; ++b) {
      std::vector<int32_t> perm(S);
      for (int i = 0; i < S; ++i) perm[i] = i;
      std::shuffle(perm.begin(), perm.end(), rng);
      for (int i = 0; i < S; ++i) pos[(size_t)b * S + perm[i]] = i;
    }
    InverseSchedule sch;
    CHECK(!build_inverse_schedule(sch, S, nprob, pos.data()));
    CHECK(build_inverse_schedule(sch, S, nprob, pos.data()));  // cached
    std::set<int32_t> seen;
    for (int32_t e : sch.list) CHECK(seen.insert(e).second);
    for (int32_t e : sch.skip) CHECK(seen.insert(e).second);
    CHECK(sch.level_off.front() == 0 && sch.level_off.back() == (int)sch.list.size());
    for (size_t l = 0; l + 1 < sch.level_off.size(); ++l) CHECK(sch.level_off[l] < sch.level_off[l + 1]);
    for (int b = 0; b < nprob; ++b) {
      const int32_t* pb = pos.data() + (size_t)b * S;
      std::vector<int> perm(S);
      for (int i = 0; i < S; ++i) perm[pb[i]] = i;
      // the reference's loop order, lower-triangle pairs only
      std::vector<int32_t> loop;
      std::vector<char> edge((size_t)S * S, 0);
      size_t nperm = 0;
      for (int i = 0; i < S; ++i)
        for (int p = 0; p < pb[i]; ++p) {
          const int k = perm[p];
          const int32_t ent = (b << 16) | (i << 8) | k;
          ++nperm;
          CHECK(seen.count(ent));
          if (perm[i] > perm[k]) {
            loop.push_back(ent);
            edge[(size_t)perm[i] * S + perm[k]] = 1;
          }
        }
      // reachability by Floyd-Warshall (y ~> x: a chain of entries x -> .. -> y)
      std::vector<char> reach((size_t)S * S, 0);
      for (int x = 0; x < S; ++x) {
        reach[(size_t)x * S + x] = 1;
        for (int y = 0; y < S; ++y)
          if (edge[(size_t)x * S + y]) reach[(size_t)x * S + y] = 1;
      }
      for (int m = 0; m < S; ++m)
        for (int x = 0; x < S; ++x)
          if (reach[(size_t)x * S + m])
            for (int y = 0; y < S; ++y)
              if (reach[(size_t)m * S + y]) reach[(size_t)x * S + y] = 1;
      auto ab = [&](int32_t ent) {
        const int i = (ent >> 8) & 0xff, k = ent & 0xff;
        return std::make_pair(perm[i], perm[k]);
      };
      // reads(p) = entries (r, c) with b_p ~> c and r ~> a_p
      auto reads = [&](int32_t p, int32_t q) {
        const auto [ap, bp] = ab(p);
        const auto [aq, bq] = ab(q);
        return reach[(size_t)bq * S + bp] && reach[(size_t)ap * S + aq];
      };
      std::vector<uint64_t> seq((size_t)S * S), par;
      for (size_t k = 0; k < seq.size(); ++k) seq[k] = k * 0x1234567ull + 1;
      par = seq;
      std::vector<std::vector<size_t>> rd(loop.size());  // entries each pair reads
      std::map<int32_t, size_t> at;
      for (size_t p = 0; p < loop.size(); ++p) {
        at[loop[p]] = p;
        for (int32_t q : loop)
          if (reads(loop[p], q)) {
            const auto [aq, bq] = ab(q);
            rd[p].push_back((size_t)aq * S + bq);
          }
      }
      auto update = [&](const std::vector<uint64_t>& st, int32_t p) {
        uint64_t h = (uint64_t)p;
        for (size_t e : rd[at[p]]) h = mix(h, st[e]);
        return h;
      };
      for (int32_t p : loop) {
        const auto [a, bb] = ab(p);
        seq[(size_t)a * S + bb] = update(seq, p);
      }
      for (size_t l = 0; l + 1 < sch.level_off.size(); ++l) {
        std::vector<std::pair<size_t, uint64_t>> commit;
        for (int o = sch.level_off[l]; o < sch.level_off[l + 1]; ++o) {
          const int32_t p = sch.list[o];
          if ((p >> 16) != b) continue;
          const auto [a, bb] = ab(p);
          commit.push_back({(size_t)a * S + bb, update(par, p)});
        }
        for (auto& cv : commit) par[cv.first] = cv.second;
      }
      CHECK(seq == par);
      (void)nperm;
    }
    CHECK(seen.size() == sch.list.size() + sch.skip.size());
  }
}

// ---- the asynchronous step queue ---------------------------------------------
struct Job {
  int id;
  double* out;
  int rc = 0;
};

// the pipelined form (nemo_optimal_weights_begin): start() puts a job "on the
// device" (a deadline) unless it fails at once, ready() polls the deadline,
// finish() waits for it and writes the output.  At most `depth` jobs in
// flight, started in submission order, finished in the same order, each
// collected after its finish; shutdown still drains everything
struct PJob {
  int id;
  double* out;
  int rc = 0;
  std::chrono::steady_clock::time_point due{};
  bool started = false, finished = false;
};

static void check_pipelined_queue(std::mt19937_64& rng) {
  using clk = std::chrono::steady_clock;
  for (int depth : {1, 2, 3}) {
    std::atomic<int> in_flight{0}, max_flight{0}, last_started{-1}, last_finished{-1};
    std::atomic<bool> order_ok{true};
    std::mutex rmu;
    std::mt19937_64 jr(rng());
    auto start = [&](PJob& j) {
      if (j.id != last_started + 1) order_ok = false;
      last_started = j.id;
      j.started = true;
      if (j.id % 7 == 6) {  // fails at start: complete at once, never in flight
        j.rc = -3;
        *j.out = -3.0;
        return false;
      }
      unsigned us;
      {
        std::lock_guard<std::mutex> g(rmu);
        us = (unsigned)(jr() % 120);
      }
      j.due = clk::now() + std::chrono::microseconds(us);
      const int f = ++in_flight;
      int m = max_flight.load();
      while (f > m && !max_flight.compare_exchange_weak(m, f)) {
      }
      return true;
    };
    auto ready = [](PJob& j) { return clk::now() >= j.due; };
    auto finish = [&](PJob& j) {
      std::this_thread::sleep_until(j.due);
      if (j.id <= last_finished) order_ok = false;
      last_finished = j.id;
      *j.out = 10.0 * j.id;
      j.finished = true;
      --in_flight;
    };
    {
      StepQueue<PJob> q(start, ready, finish, depth);
      std::vector<double> out(300, -1.0);
      std::vector<std::unique_ptr<PJob>> back;
      int next = 0, got = 0;
      while (got < 300) {
        const int burst = 1 + (int)(rng() % 4);
        for (int k = 0; k < burst && next < 300; ++k, ++next)
          CHECK(q.submit(std::unique_ptr<PJob>(new PJob{next, &out[next]}), nullptr));
        if (rng() % 3 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 200));
        const int take = (int)(rng() % 3);
        for (int k = 0; k < take && got < next; ++k, ++got) {
          std::unique_ptr<PJob> j = q.collect();
          const bool failed = got % 7 == 6;
          CHECK(j && j->id == got && j->started && j->finished == !failed);
          CHECK(out[got] == (failed ? -3.0 : 10.0 * got) && j->rc == (failed ? -3 : 0));
        }
      }
      CHECK(q.collect() == nullptr && q.pending() == 0);
    }
    CHECK(order_ok.load() && max_flight.load() <= depth && in_flight.load() == 0);
    // shutdown with jobs queued and in flight: all of them finish
    {
      std::vector<double> out(40, -1.0);
      last_started = -1;
      last_finished = -1;
      StepQueue<PJob> q(start, ready, finish, depth);
      const int n = 1 + (int)(rng() % 40);
      for (int k = 0; k < n; ++k) CHECK(q.submit(std::unique_ptr<PJob>(new PJob{k, &out[k]}), nullptr));
      q.shutdown();
      for (int k = 0; k < n; ++k) CHECK(out[k] == (k % 7 == 6 ? -3.0 : 10.0 * k));
      CHECK(in_flight.load() == 0);
    }
  }
}

static void check_step_queue(std::mt19937_64& rng) {
  // collected in submission order, each after it ran
  {
    std::atomic<int> ran{0};
    StepQueue<Job> q([&](Job& j) {
      std::this_thread::sleep_for(std::chrono::microseconds(50 * (j.id % 3)));
      *j.out = 10.0 * j.id;
      j.rc = j.id % 5 == 4 ? -5 : 0;
      ++ran;
    });
    std::vector<double> out(200, -1.0);
    int next = 0, got = 0;
    while (got < 200) {
      const int burst = 1 + (int)(rng() % 4);
      for (int k = 0; k < burst && next < 200; ++k, ++next) {
        std::string err;
        CHECK(q.submit(std::unique_ptr<Job>(new Job{next, &out[next]}), &err));
      }
      const int take = (int)(rng() % 3);
      for (int k = 0; k < take && got < next; ++k, ++got) {
        std::unique_ptr<Job> j = q.collect();
        CHECK(j && j->id == got && out[got] == 10.0 * got && j->rc == (got % 5 == 4 ? -5 : 0));
      }
    }
    CHECK(q.collect() == nullptr);
    CHECK(q.pending() == 0 && ran == 200);
  }
  // shutdown with steps queued and not collected: every one still runs
  for (int trial = 0; trial < 20; ++trial) {
    std::vector<double> out(16, -1.0);
    {
      StepQueue<Job> q([](Job& j) {
        std::this_thread::sleep_for(std::chrono::microseconds(20));
        *j.out = j.id;
      });
      const int n = 1 + (int)(rng() % 16);
      for (int k = 0; k < n; ++k) CHECK(q.submit(std::unique_ptr<Job>(new Job{k, &out[k]}), nullptr));
      if (trial % 2) (void)q.collect();
      q.shutdown();
      for (int k = 0; k < n; ++k) CHECK(out[k] == k);
      std::string err;
      CHECK(!q.submit(std::unique_ptr<Job>(new Job{0, &out[0]}), &err) && !err.empty());
    }  // the destructor after shutdown: nothing left to join or free twice
  }
  // a queue destroyed without shutdown or any job
  { StepQueue<Job> q([](Job&) {}); }
  check_pipelined_queue(rng);
}

// ---- the device's fixed-order partial sum on the host ------------------------
// sum_partials_host restates sum_partials (nemo_internal.h): 64 strided lane
// sums, then xor butterflies with o = 32, 16, ..., 1, lane 0's value.  Checked
// against the same tree written backwards as a recursion: lane l's value
// after the stages down to o is its value and lane (l ^ o)'s after the stages
// down to 2o, added.  Values whose sums round, so another association shows.
static double after_stages(const double* lanes, int l, int o) {
  if (o == 64) return lanes[l];
  return after_stages(lanes, l, 2 * o) + after_stages(lanes, l ^ o, 2 * o);
}
static void check_sum_partials(std::mt19937_64& rng) {
  std::uniform_real_distribution<double> u(-1e3, 1e3);
  for (int n : {0, 1, 5, 63, 64, 65, 127, 200, 1000}) {
    std::vector<double> p(n);
    for (auto& x : p) x = u(rng) * (1.0 + 1e-9 * u(rng));
    double lanes[64];
    for (int l = 0; l < 64; ++l) {
      double s = 0.0;
      for (int t = l; t < n; t += 64) s += p[t];
      lanes[l] = s;
    }
    CHECK(sum_partials_host(p.data(), n) == after_stages(lanes, 0, 1));
  }
  const double small[3] = {1.0, 2.0, 3.0};
  CHECK(sum_partials_host(small, 3) == 6.0);
  CHECK(sum_partials_host(small, 0) == 0.0);
}

int main() {
  std::mt19937_64 rng(20261017);
  check_pos_rows();
  check_staging(rng);
  check_bounds(rng);
  check_inverse_schedule(rng);
  check_step_queue(rng);
  check_sum_partials(rng);
  printf("ok %d\n", g_checks);
  return 0;
}
