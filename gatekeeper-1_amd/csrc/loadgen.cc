// Open-loop admission load for the webhook benchmark (bench.py --config 5
// --coalesce-us): `clients` native threads issue single-review
// gk_query(violation) calls -- the reference webhook's one Review per request,
// pkg/webhook/policy.go:371-387 -- at `rate` requests/s in total, each call's
// rows copied out with gk_results_export as a caller would.  A client of the
// C ABI only (include/gkgpu.h), built as its own library (libgkload.so): the
// Python client threads it replaces serialized on the interpreter lock, so
// the measured tail was the load generator's, not the engine's.  A request's
// latency runs from its scheduled arrival to its rows and status in the
// caller's buffer (queueing behind a busy client or launch included).
#include <time.h>

#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gkgpu.h"

namespace {
double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}
void sleep_until(double t) {
  const double d = t - now_s();
  if (d <= 0) return;
  timespec ts;
  ts.tv_sec = (time_t)t;
  ts.tv_nsec = (long)((t - (double)ts.tv_sec) * 1e9);
  clock_nanosleep(CLOCK_MONOTONIC, TIMER_ABSTIME, &ts, nullptr);
}
}  // namespace

// lat_ms: n_requests latencies (request i = client i % clients, its k-th call
// i / clients); elapsed_s: first scheduled arrival to the last completion.
// Returns 0, or the first failing call's gk status.
extern "C" int gkload_open_loop(gk_engine* e, const char* path, const char* const* inputs, const size_t* lens,
                                size_t n_inputs, size_t n_requests, int clients, double rate, double* lat_ms,
                                double* elapsed_s) {
  if (!e || !inputs || !n_inputs || clients < 1 || rate <= 0 || !lat_ms) return GK_EINVAL;
  const double gap = clients / rate;  // each client's inter-arrival time
  std::atomic<int> err{0};
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  double t0 = 0;
  std::vector<double> done(clients, 0.0);
  std::vector<std::thread> th;
  th.reserve(clients);
  for (int c = 0; c < clients; ++c)
    th.emplace_back([&, c] {
      std::vector<char> buf(1 << 16);
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      const double base = t0 + c * gap / clients;
      for (size_t i = c, k = 0; i < n_requests; i += clients, ++k) {
        const double due = base + k * gap;
        sleep_until(due);
        const size_t j = i % n_inputs;
        gk_results* r = nullptr;
        int rc = gk_query(e, path, inputs[j], lens[j], &r);
        if (rc == GK_OK) {
          size_t need = 0;
          rc = gk_results_export(r, buf.data(), buf.size(), &need);
          if (rc != GK_OK && need > buf.size()) {
            buf.resize(need);
            rc = gk_results_export(r, buf.data(), buf.size(), &need);
          }
          uint32_t st = 0;
          if (rc == GK_OK) rc = gk_results_copy_status(r, &st, nullptr);
        }
        if (r) gk_results_free(r);
        if (rc != GK_OK) {
          int z = 0;
          err.compare_exchange_strong(z, rc);
        }
        const double t = now_s();
        lat_ms[i] = (t - due) * 1e3;
        done[c] = t;
      }
    });
  while (ready.load() < clients) std::this_thread::yield();
  t0 = now_s() + 0.05;
  go.store(true, std::memory_order_release);
  for (auto& t : th) t.join();
  double last = t0;
  for (double d : done) last = d > last ? d : last;
  if (elapsed_s) *elapsed_s = last - t0;
  return err.load();
}

// Closed-loop micro-batches (bench.py --config 5): `steps` gk_query_batch
// calls over the batches in turn (batch b = inputs[b * batch .. +batch)), each
// followed by gk_results_export of every row into one caller buffer and the
// per-review status words, as a native webhook replica reads them.  lat_ms:
// per call; rows / bytes (optional): totals over the calls.
extern "C" int gkload_batch_loop(gk_engine* e, const char* const* inputs, const size_t* lens, size_t n_batches,
                                 size_t batch, size_t steps, double* lat_ms, uint64_t* rows, uint64_t* bytes,
                                 uint64_t* flagged) {
  if (!e || !inputs || !lens || !n_batches || !batch || !lat_ms) return GK_EINVAL;
  std::vector<char> buf(1 << 20);
  std::vector<uint32_t> st(batch);
  uint64_t nrow = 0, nbytes = 0, nflag = 0;
  for (size_t s = 0; s < steps; ++s) {
    const size_t b = s % n_batches;
    const double t0 = now_s();
    gk_results* r = nullptr;
    int rc = gk_query_batch(e, inputs + b * batch, lens + b * batch, batch, &r);
    size_t need = 0;
    if (rc == GK_OK) {
      rc = gk_results_export(r, buf.data(), buf.size(), &need);
      if (rc != GK_OK && need > buf.size()) {
        buf.resize(need);
        rc = gk_results_export(r, buf.data(), buf.size(), &need);
      }
    }
    if (rc == GK_OK) rc = gk_results_copy_status(r, st.data(), nullptr);
    const double t1 = now_s();
    if (rc == GK_OK) {
      nrow += gk_results_count(r);
      for (uint32_t x : st) nflag += (x & 3) != 0;
    }
    if (r) gk_results_free(r);
    if (rc != GK_OK) return rc;
    lat_ms[s] = (t1 - t0) * 1e3;
    nbytes += need;
  }
  if (rows) *rows = nrow;
  if (bytes) *bytes = nbytes;
  if (flagged) *flagged = nflag;
  return GK_OK;
}
