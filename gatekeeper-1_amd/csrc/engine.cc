// gkgpu engine: drivers.Driver state, review flattening, constraint match
// compilation, device residency, kernel launch and result decoding.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <atomic>
#include <functional>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <thread>
#include <vector>

#include "../../include/gkgpu.h"
#include "common.h"
#include "compiler.h"
#include "flatten.h"
#include "jit.h"
#include "colplan.h"
#include "colstore.h"
#include "json.h"
#include "rego.h"
#include "regex.h"
#include "store.h"

namespace gk {
}
extern "C" int gk_launch_audit(const gk::DevArgs* args, hipStream_t stream);
extern "C" int gk_launch_compact(const gk::DevArgs* a, const gk::Viol* raw, const uint64_t* rfrec, uint32_t* tcnt,
                                 unsigned long long* toff, hipStream_t stream, uint64_t hint);
extern "C" int gk_launch_keys(const gk::DevArgs* args, hipStream_t stream);
extern "C" int gk_launch_format(const gk::DevArgs* args, hipStream_t stream, hipEvent_t* ev, uint64_t hint);
extern "C" int gk_launch_zero(void* const* ptrs, const uint64_t* bytes, uint32_t n, hipStream_t stream);
extern "C" size_t gk_devargs_size();
extern "C" int gk_launch_sample(const gk::Viol* out, uint64_t n, uint32_t* rflags, uint32_t nrev, const uint8_t* cerr,
                                uint32_t ncons, uint32_t nb, uint32_t limit, uint32_t* hist, uint32_t* cut,
                                unsigned long long* ftot, const char* bytes, gk::SampleRec* cand, uint32_t cap,
                                unsigned int* ncand, int select_only, hipStream_t stream);
extern "C" uint32_t gk_sample_fine(uint32_t nrev);
extern "C" int gk_launch_clock_probe(unsigned long long* out, uint32_t iters, hipStream_t stream);
extern "C" int gk_launch_filter(const gk::Viol* out, uint64_t n, uint32_t* rflags, const uint8_t* cerr,
                                gk::Viol* dst, unsigned long long* count, hipStream_t stream);

namespace gk {

static const char* TARGET = "admission.k8s.gatekeeper.sh";
static const char* CGROUP = "constraints.gatekeeper.sh";
static const char* EMPTY_NS_JSON = "{\"metadata\":{\"creationTimestamp\":null},\"spec\":{},\"status\":{}}";

using Clock = std::chrono::steady_clock;
static double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

// Integer A/B switch from the environment: unset -> def; a decimal in
// [0, max] -> that value; anything else is rejected loudly (stderr) and
// read as def, so a typo cannot silently select another mode.
static int env_mode(const char* name, int def, int max) {
  const char* v = getenv(name);
  if (!v || !*v) return def;
  char* end = nullptr;
  long x = strtol(v, &end, 10);
  if (*end || x < 0 || x > max) {
    fprintf(stderr, "gkgpu: ignoring %s=%s (expected an integer in [0, %d])\n", name, v, max);
    return def;
  }
  return (int)x;
}


// ------------------------------------------------------------------ device buffers
// Large host-to-device copies (a staged batch's node arena, ~1 GB per 1M Pods)
// go through two pinned 64 MB bounce buffers: host threads copy chunk k+1 into
// one while the DMA engine reads chunk k from the other.  A pageable
// hipMemcpy of the same bytes runs at a fraction of the link rate.
// GKGPU_PINNED_UPLOAD=0 keeps the plain hipMemcpy (A/B).
// the pinned bounce buffers, their stream and events: set up once per process
// (gk_engine_prepare does it ahead of the first staging: page-locking 128 MB
// is not part of a sweep)
struct Bounce {
  static constexpr size_t CH = 64ull << 20;
  std::mutex mu;
  char* pin[2] = {nullptr, nullptr};
  hipStream_t st = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  bool pending[2] = {false, false};  // a copy out of pin[b] may still be in flight
  int ok = -1;
  bool init_locked() {
    if (ok < 0)
      ok = env_mode("GKGPU_PINNED_UPLOAD", 1, 1) != 0 && hipHostMalloc((void**)&pin[0], CH, hipHostMallocDefault) == hipSuccess &&
           hipHostMalloc((void**)&pin[1], CH, hipHostMallocDefault) == hipSuccess &&
           hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
           hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) == hipSuccess;
    return ok > 0;
  }
};
static Bounce& bounce() {
  static Bounce* b = new Bounce();
  return *b;
}
static void upload_bounce_init() {
  Bounce& B = bounce();
  std::lock_guard<std::mutex> g(B.mu);
  B.init_locked();
}
static bool upload_bounce(void* dst, const char* src, size_t n) {
  Bounce& B = bounce();
  constexpr size_t CH = Bounce::CH;
  char** pin = B.pin;
  hipStream_t& st = B.st;
  hipEvent_t* ev = B.ev;
  bool* pending = B.pending;
  std::lock_guard<std::mutex> g(B.mu);
  if (!B.init_locked()) return hipMemcpy(dst, src, n, hipMemcpyHostToDevice) == hipSuccess;
  const int T = std::max(1, std::min(16, default_threads()));
  const bool trace = getenv("GKGPU_FLATTEN_TRACE") != nullptr;
  // GKGPU_BOUNCE_CHUNK (tests): a smaller chunk, to exercise many chunks
  const char* bc = getenv("GKGPU_BOUNCE_CHUNK");
  const size_t chunk = bc && atoll(bc) > 0 ? std::min<size_t>(CH, (size_t)atoll(bc)) : CH;
  double ms_copy = 0, ms_wait = 0;
  auto t_all = std::chrono::steady_clock::now();
  for (size_t off = 0, k = 0; off < n; off += chunk, ++k) {
    const size_t len = std::min(chunk, n - off);
    const int b = (int)(k & 1);
    auto tw = std::chrono::steady_clock::now();
    // the DMA of the chunk that last used this buffer (this call's, or a
    // failed earlier call's) must have drained it before it is refilled
    if (pending[b]) {
      if (hipEventSynchronize(ev[b]) != hipSuccess) { hipStreamSynchronize(st); return false; }
      pending[b] = false;
    }
    auto tc = std::chrono::steady_clock::now();
    ms_wait += std::chrono::duration<double, std::milli>(tc - tw).count();
    char* dstp = pin[b];
    const char* srcp = src + off;
    parallel_run(T, [&](int t) {
      const size_t lo = len * t / T, hi = len * (t + 1) / T;
      memcpy(dstp + lo, srcp + lo, hi - lo);
    });
    ms_copy += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc).count();
    if (hipMemcpyAsync((char*)dst + off, dstp, len, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipEventRecord(ev[b], st) != hipSuccess) {
      // earlier chunks may still be reading the pinned buffers: drain them
      hipStreamSynchronize(st);
      pending[0] = pending[1] = false;
      return false;
    }
    pending[b] = true;
  }
  const bool ok_sync = hipStreamSynchronize(st) == hipSuccess;
  if (ok_sync) pending[0] = pending[1] = false;
  if (trace)
    fprintf(stderr, "upload: %.1f MB in %.1f ms (host copies %.1f ms, DMA waits %.1f ms, %d threads)\n", n / 1e6,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_all).count(), ms_copy, ms_wait, T);
  return ok_sync;
}

struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  size_t used = 0;  // bytes uploaded (append-only arrays upload the tail)
  // Shared append-only tables (strings, pool, numbers) are read by kernels of
  // concurrent evaluations while another evaluation appends to them: a grown
  // table keeps its predecessor alive here (freed with the engine), so a
  // pointer an in-flight launch holds stays valid.
  std::vector<void*>* graveyard = nullptr;
  bool reserve(size_t n) {
    if (n <= cap) return true;
    size_t nc = std::max(n, cap * 2);
    nc = std::max<size_t>(nc, 4096);
    void* q = nullptr;
    if (hipMalloc(&q, nc) != hipSuccess) return false;
    // a device-to-device hipMemcpy does not wait for the copy on the host, and
    // the evaluation contexts' streams are non-blocking (no implicit order with
    // the null stream): finish it before any launch can read the new buffer
    if (p && used &&
        (hipMemcpy(q, p, used, hipMemcpyDeviceToDevice) != hipSuccess || hipStreamSynchronize(nullptr) != hipSuccess)) {
      hipFree(q);
      return false;
    }
    if (p) {
      if (graveyard) graveyard->push_back(p);
      else hipFree(p);
    }
    p = q;
    cap = nc;
    return true;
  }
  bool upload(const void* src, size_t n, bool append_only) {
    if (!reserve(n)) return false;
    size_t from = append_only ? std::min(used, n) : 0;
    // GKGPU_BOUNCE_MIN (tests): the smallest copy that takes the bounce path
    const char* bm = getenv("GKGPU_BOUNCE_MIN");
    const size_t bounce_min = bm ? (size_t)atoll(bm) : (16u << 20);
    if (n > from && n - from >= bounce_min) {
      if (!upload_bounce((char*)p + from, (const char*)src + from, n - from)) return false;
    } else if (n > from && hipMemcpy((char*)p + from, (const char*)src + from, n - from, hipMemcpyHostToDevice) != hipSuccess)
      return false;
    used = n;
    return true;
  }
  void free_() { if (p) hipFree(p); p = nullptr; cap = used = 0; }
};

// ------------------------------------------------------------------ engine state
struct TemplateEnt {
  std::string kind;
  bool supported = false;  // the whole template runs on the GPU
  bool guard = false;      // outside the subset; prog is its guard program
  std::string reason;
  std::string detail;      // gk_template_backend text
  std::string joins;       // gk_template_joins text
  int prog = -1;
};

struct ConstraintEnt {
  std::string kind, name;
  std::string json;        // the PutData document (kept to re-place it when the permanent region is compacted)
  uint32_t root = NO_ID;   // node of the whole constraint (permanent region)
  uint32_t nnodes = 0;     // nodes of its document
  MatchSpec spec{};
  std::string ea;          // enforcementAction as returned in results
  bool ea_error = false;   // non-string enforcementAction: Query fails
  bool kind_ok = true;
};

// a decoded row: message and details JSON are views into the evaluation's
// downloaded output bytes (gk_results::rbytes, shared with the per-caller
// results a coalesced launch is split into)
struct ResultRow {
  uint32_t review, constraint, seq, rule;
  std::string_view msg, details;
};

// Pinned host blocks for decoded result bytes: the readback copies the
// message bytes straight into a block the results then own (their rows view
// it), and freeing the results returns it here.  Process-wide and never torn
// down (a block may be released after its engine is gone; HIP may already be
// unloading at exit).
struct PinPool {
  std::mutex mu;
  std::vector<std::pair<size_t, char*>> free_;  // (capacity, block)
  size_t bytes = 0;                              // pinned bytes kept in free_
  // kept blocks: at most kKeepBytes in all, none above kKeepBlock (a burst of
  // large decodes must not leave gigabytes of host memory pinned)
  static constexpr size_t kKeepBytes = 256ull << 20, kKeepBlock = 96ull << 20;
};
static PinPool& pin_pool() {
  static PinPool* p = new PinPool();
  return *p;
}
// a block of at least n bytes, owned by the returned handle; nullptr on failure
static std::shared_ptr<const void> pinned_block(size_t n, char** out) {
  PinPool& pp = pin_pool();
  char* blk = nullptr;
  size_t cap = 0;
  {
    std::lock_guard<std::mutex> g(pp.mu);
    size_t best = pp.free_.size();
    for (size_t i = 0; i < pp.free_.size(); ++i)
      if (pp.free_[i].first >= n && pp.free_[i].first <= 4 * n + (1 << 16) &&
          (best == pp.free_.size() || pp.free_[i].first < pp.free_[best].first))
        best = i;
    if (best < pp.free_.size()) {
      cap = pp.free_[best].first;
      blk = pp.free_[best].second;
      pp.bytes -= cap;
      pp.free_.erase(pp.free_.begin() + best);
    }
  }
  if (!blk) {
    cap = std::max<size_t>(n + (n >> 2), 1 << 16);
    if (hipHostMalloc((void**)&blk, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
  }
  *out = blk;
  return std::shared_ptr<const void>(blk, [cap](const void* q) {
    PinPool& pp = pin_pool();
    std::lock_guard<std::mutex> g(pp.mu);
    if (pp.free_.size() < 16 && cap <= PinPool::kKeepBlock && pp.bytes + cap <= PinPool::kKeepBytes) {
      pp.free_.emplace_back(cap, (char*)q);
      pp.bytes += cap;
    } else {
      (void)hipHostFree((void*)q);
    }
  });
}

// One evaluation's device state: its stream, its launch events and every
// buffer a call writes (review columns and documents of a query, output
// tuples and bytes, flags, totals, sampling).  Concurrent evaluations
// (drivers.Driver.Query under local.go's read lock) each hold one; a pool
// keeps them for reuse.  The engine's permanent tables (constraint match
// words, bytecode, templates' kernels, the permanent node region, strings)
// are shared and read-only while evaluations run.
struct EvalCtx {
  std::mutex busy;  // held by the evaluation using it (and by a raw-output copy of its results)
  hipStream_t stream = nullptr;
  std::vector<hipEvent_t> events;
  DBuf d_mstr, d_mtop;  // memo-string arena + its cursor (V_GSTR)
  DBuf d_nodes, d_revs, d_out, d_bytes, d_counters, d_rflags, d_totals, d_rreason, d_prof, d_pchist, d_clist, d_gmemo,
      d_frec, d_hist, d_cut, d_ftot, d_cand, d_ncand, d_cerr, d_ebytes, d_lens, d_part;
  // the predicate kernels' chunked tuples and argument words before
  // compaction (devrt.h slot_reserve, kernels.hip gk_compact_*), tile counts
  DBuf d_out_raw, d_frec_raw, d_ctcnt, d_ctoff;
  // side streams for concurrent template launches (GKGPU_CONCURRENT), each
  // with its own cross-lane memo table (memo sites are per program)
  static constexpr int kSide = 3;
  hipStream_t side[kSide] = {nullptr, nullptr, nullptr};
  DBuf d_gmemo_side[kSide];
  std::vector<hipEvent_t> lev;  // per launch: start, end (timing) + the join event
  size_t out_cap = 1 << 20, bytes_cap = 64u << 20, ebytes_cap = 16u << 20, cand_cap = 1 << 14;
  uint64_t eval_epoch = 0;   // bumps on every evaluation (output buffers reused)
  uint64_t last_tuples = 0;  // the last evaluation's tuple count (sizes the passes' grids)
  uint64_t perm_gen = 0;     // engine generation whose permanent nodes d_nodes holds below perm_nodes
  uint32_t perm_nodes = 0;
  void* perm_buf = nullptr;  // the d_nodes buffer that copy went to
  NodeArena arena;           // host documents of the current query (node id perm_nodes + k)
  // pinned host staging for the readback: several device-to-host copies are
  // queued back to back and waited for once (a pageable copy syncs each time)
  unsigned int last_ncand = 0;  // sample candidates of the context's last audit (gk_batch_eval_audit)
  char* h_pin = nullptr;
  size_t h_pin_cap = 0;
  char* pin(size_t n) {
    if (n <= h_pin_cap) return h_pin;
    if (h_pin) hipHostFree(h_pin);
    h_pin = nullptr;
    h_pin_cap = 0;
    const size_t cap = std::max<size_t>(n + (n >> 1), 1 << 16);
    if (hipHostMalloc((void**)&h_pin, cap, hipHostMallocDefault) != hipSuccess) { h_pin = nullptr; return nullptr; }
    h_pin_cap = cap;
    return h_pin;
  }
  void release_all() {
    if (h_pin) hipHostFree(h_pin);
    h_pin = nullptr;
    h_pin_cap = 0;
    for (DBuf* b : {&d_nodes, &d_revs, &d_out, &d_bytes, &d_counters, &d_rflags, &d_totals, &d_rreason, &d_prof, &d_pchist,
                    &d_clist, &d_gmemo, &d_mstr, &d_mtop, &d_frec, &d_hist, &d_cut, &d_ftot, &d_cand, &d_ncand, &d_cerr, &d_ebytes, &d_lens,
                    &d_part, &d_out_raw, &d_frec_raw, &d_ctcnt, &d_ctoff})
      b->free_();
    for (hipEvent_t x : events) hipEventDestroy(x);
    events.clear();
    for (hipEvent_t x : lev) hipEventDestroy(x);
    lev.clear();
    for (int k = 0; k < kSide; ++k) {
      d_gmemo_side[k].free_();
      if (side[k]) hipStreamDestroy(side[k]);
      side[k] = nullptr;
    }
    if (stream) hipStreamDestroy(stream);
    stream = nullptr;
  }
};

}  // namespace gk

struct gk_results {
  std::vector<gk::ResultRow> rows;
  std::shared_ptr<const void> rbytes;  // the bytes rows view (a std::string or a pinned block)
  std::vector<uint32_t> status, reason;  // empty when no review was flagged (all zero)
  uint32_t nrev = 0;
  std::vector<uint64_t> totals;
  std::vector<std::string> ckind, cname, cea;
  std::vector<uint8_t> cea_error;          // per constraint: non-string enforcementAction (Query error)
  uint64_t excluded = 0;                   // reviews skipped by the process excluder
  double ms[5] = {0, 0, 0, 0, 0};
  uint64_t dev_tuples = 0, dev_bytes = 0;  // tuples / message bytes the kernels wrote
  gk::EvalCtx* ctx = nullptr;              // the evaluation context holding the device output
  uint64_t epoch = 0;                      // ... while its eval_epoch equals this
  uint64_t gen = 0;                        // engine generation (state of modules / data) evaluated
  std::vector<uint64_t> prof;              // GKGPU_PROFILE=1: per constraint VM step stats
  struct Sample { uint32_t review, constraint; uint16_t seq, rule; uint32_t msg_len; std::string msg; };
  std::vector<Sample> samples;             // gk_batch_eval_audit: first `limit` per constraint, in order
  uint64_t failed_lanes = 0;               // (review, constraint) lanes flagged error / fallback on the device
  bool audited = false;
  struct Launch { std::string kernel; double ms; uint32_t nconstraints; uint64_t tuples, bytes; };
  std::vector<Launch> launches;            // kernels of the last attempt, in launch order
};

struct gk_batch {
  gk_engine* eng = nullptr;
  uint64_t node_count = 0, str_bytes = 0;  // algorithmic input bytes of the staged documents
  bool str_bytes_done = false;
  uint64_t gen = 0;
  uint32_t nrev = 0;
  uint32_t node_begin = 0, node_end = 0;    // node ids of the batch's documents
  uint64_t excluded = 0;                    // reviews skipped by the process excluder
  double ms_parse = 0, ms_flatten = 0, ms_upload = 0;
  std::vector<gk::ReviewCol> cols;
  std::vector<gk::ResourceIds> resources;   // HandleViolation identity per batch index
  gk::NodeArena arena;                      // host copy of the documents (node id node_begin + k)
  gk::DBuf d_revs;
  gk::DBuf d_nodes;  // the batch's own device node array: permanent region + its documents
  uint64_t dev_bytes = 0;
  bool device_layout = false;  // d_nodes / d_revs hold the device-built path layout (node ids differ from arena's)
  // column form (colstore.h): d_nodes holds the permanent region + cv.nodes,
  // d_revs cv.cols, and the programs read the documents from the columns
  bool columnar = false;
  std::string col_why;         // why the node form was kept
  gk::ColStore cv;
  gk::DBuf d_cv_words, d_cv_bytes, d_cv_slots, d_cv_hash, d_cv_views, d_cv_tabs;
};

// Webhook micro-batch coalescer: concurrent single-review
// gk_query calls -- the webhook's one Client.Review per admission request
// (pkg/webhook/policy.go:371-387) -- are gathered into one launch of up to
// `max_batch` reviews or whatever arrived within `window_us` of the first.
// The first caller to find no batch collecting leads it: it waits for the
// window (or a full batch), takes the queue, evaluates it as one
// gk_query_batch and hands every caller its own results; callers that arrive
// while it evaluates queue up for the next leader.
struct CoalesceReq {
  const char* input = nullptr;
  size_t len = 0;
  gk_results* out = nullptr;
  int rc = GK_OK;
  std::string err;
  bool done = false;
};
struct Coalescer {
  std::mutex mu;
  std::condition_variable arrive;    // the collecting leader: a request arrived
  std::condition_variable finished;  // followers: results handed out / a new leader is needed
  std::vector<CoalesceReq*> queue;
  bool collecting = false;
  uint32_t inflight = 0;             // coalesced launches being evaluated
  uint32_t window_us = 0;            // 0: off (every gk_query launches alone)
  uint32_t max_batch = 256;
  uint64_t batches = 0, requests = 0;
};
// Under load a leader keeps collecting past its window while kMaxInflight
// launches are still being evaluated (the batch grows instead of a second
// small launch queueing behind them), for at most kWindowCap windows.
constexpr uint32_t kMaxInflight = 2;
constexpr uint32_t kWindowCap = 16;

struct gk_engine {
  // drivers.Driver's locking (local.go:62-68, 117, 303-304): evaluations
  // (Query and the batch calls) share `rw`; mutations (Put/Delete of modules
  // and data, excluder changes) take it exclusively, so an evaluation sees one
  // engine state from start to end.  `turn` makes a waiting mutation block new
  // readers (no writer starvation under a stream of queries).  `smu` guards
  // the string / number tables, which evaluations append to while they
  // flatten their documents.
  std::shared_mutex rw;
  std::mutex turn;
  std::mutex smu;
  std::mutex pool_mu;
  std::vector<std::unique_ptr<gk::EvalCtx>> ctxs;  // evaluation contexts (pool)
  Coalescer co;
  std::vector<void*> graveyard;                     // superseded shared device tables
  uint64_t prepared_gen = 0;  // generation the compiled state and device tables were prepared for
  bool prepared_dev = false;
  int device = 0;
  bool dev_ok = false;
  std::mutex dbg_mu;
  std::vector<uint32_t> pchist;  // last launch's per-pc execution counts (GKGPU_PROFILE=2)
  int profile = 0;  // GKGPU_PROFILE=1: VM step statistics per launch; 2: + per-pc histogram
  gk::Store st;
  uint32_t base_nodes = 0;  // the store's fixed nodes
  // modules
  std::map<std::string, std::string> modules;  // name -> source
  gk::ModuleSet mods;
  gk::CodeBank bank;
  std::vector<gk::Program> progs;
  uint64_t module_nodes = 0;  // permanent nodes the compiled templates' constants occupy
  // per-template kernels (jit.cc), parallel to progs
  struct Jit {
    std::string name, src, code, log;
    int state = 0;  // 0 not compiled, 1 code ready, -1 compile failed
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
  };
  std::vector<Jit> jits;
  bool jit_enabled = true;  // opts {"jit": false} / GKGPU_JIT=0 force the bytecode VM kernel
  bool host_only = false;    // opts {"host_only": true}: stage on the host only (CPU baseline / tests); no evaluation
  std::map<std::string, gk::TemplateEnt> templates;  // by constraint kind
  // the referenced-path plan of every program a constraint runs (colplan.h),
  // for the column form of staged batches; per engine generation
  std::mutex plan_mu;
  uint64_t plan_gen = ~0ull;
  gk::PathPlan plan;
  bool modules_dirty = true;
  // data
  std::map<std::pair<std::string, std::string>, gk::ConstraintEnt> constraints;
  std::vector<gk::ConstraintEnt*> corder;
  std::vector<uint32_t> mwords;
  bool constraints_dirty = true;
  std::map<std::string, std::string> inventory;  // external path -> json
  // hooks.audit: the synced inventory as a staged batch of make_review
  // documents, device-resident until the engine state changes (gen)
  std::mutex cache_mu;
  std::shared_ptr<gk_batch> cache_batch;
  uint64_t cache_builds = 0;
  std::map<std::string, std::pair<uint32_t, uint32_t>> ns_nodes;  // namespace name -> (node, node count)
  gk::NsCache ns_cache;                           // namespace name -> node (permanent)
  std::map<std::string, std::string> other_data;
  // process excluder (pkg/controller/config/process/excluder.go): process -> namespaces
  std::map<std::string, std::set<std::string>> excluded;
  uint32_t perm_nodes = 0;                        // nodes of the permanent region
  // data.inventory (templates' cross-resource joins): one permanent object
  // node whose members sync_inventory points at the current inventory tree
  uint32_t inv_node = gk::NO_ID;
  uint32_t inv_lo = 0, inv_hi = 0;  // node range of the current inventory tree
  bool inv_dirty = true;        // /external/ data changed since the tree was built
  bool uses_inventory = false;  // some compiled template reads data.inventory
  uint64_t gen = 1;                               // bumps on any mutation
  // regex
  std::map<uint32_t, std::pair<uint32_t, uint32_t>> dfa_index;  // pattern sid -> (word offset, status)
  std::vector<uint32_t> dfa_words;
  std::vector<uint32_t> dfa_keys, dfa_meta;
  // LDS stage (devrt.h stage_wave): byte-class-compressed DFAs (pattern sid ->
  // [word offset in dfa_c, bytes, nst | ncls << 16, start | sens << 16]; empty:
  // does not compress) and the per-constraint stage records
  std::map<uint32_t, std::vector<uint32_t>> cdfa_index;
  std::vector<uint32_t> dfa_c, stage;
  // device mirrors of the permanent tables (written under the exclusive lock,
  // except the append-only string / number tables: under smu, graveyard kept)
  uint32_t nfmtr = 0, nfmtb = 0;  // resolved format table (sync_tables; 0: not built)
  gk::DBuf d_nodes, d_strs, d_pool, d_sflags, d_nums, d_code, d_K, d_fmt, d_fmtr, d_fmtb, d_cons, d_mwords, d_progoff, d_dfa_keys,
      d_dfa_meta, d_dfa_words, d_stage, d_dfa_c;
  // gk_debug_host_args: host copies of the per-call tables (diagnostics / CPU baseline)
  std::vector<gk::MatchSpec> dbg_cons;
  std::vector<uint32_t> dbg_progoff, dbg_mwords, dbg_dfa_keys, dbg_dfa_meta, dbg_dfa_words, dbg_fmt;
  std::vector<gk::Node> dbg_nodes;
  std::vector<uint64_t> dbg_jleaf, dbg_jsite;
  std::vector<gk::StrEnt> dbg_strs;
  std::vector<uint8_t> dbg_sflags;
  std::vector<gk::NumEnt> dbg_nums;
  std::string dbg_pool;
  uint32_t dev_nodes_ok = 0;       // leading permanent nodes whose d_nodes copy matches the host arena
  size_t out_cap0 = 1 << 20;       // initial tuple capacity of a new context (opts max_violations)
  // inventory join indexes (build_joins; under the exclusive lock)
  std::vector<uint32_t> jdir;
  std::vector<uint64_t> jhash, jleaf;
  std::vector<uint32_t> jord;
  std::vector<uint64_t> jsite;      // plan_joins: 8 words per (constraint, site) key pass
  gk::DBuf d_jdir, d_jhash, d_jord, d_jleaf, d_jkeys;
  bool joins_built = false;         // the device indexes match the current state
  uint64_t join_indexes = 0, join_entries = 0, join_unindexed = 0, join_leaves = 0;
  double join_ms = 0;
};

namespace gk {

// The device string / number tables as one evaluation uses them: the current
// pointers, snapshotted under smu right after the evaluation's own strings
// were uploaded (grown tables keep their predecessors: DBuf::graveyard).
struct TablePtrs {
  const StrEnt* strs = nullptr;
  const uint8_t* pool = nullptr;
  const uint8_t* sflags = nullptr;
  const NumEnt* nums = nullptr;
};

}  // namespace gk

// Drops the transient node region (review documents of the last call).  The
// device mirror stays valid below the cut, so the next upload is incremental.
static void reset_transient(gk_engine* e) {
  e->st.nodes().resize(e->perm_nodes);
  e->dev_nodes_ok = std::min<uint32_t>(e->dev_nodes_ok, e->perm_nodes);
}

namespace gk {

// ------------------------------------------------------------------ path helpers
static inline int hexval(char c) { return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10; }
static std::vector<std::string> split_path(const std::string& p) {
  std::vector<std::string> out;
  out.reserve(8);
  size_t i = 0;
  while (i < p.size()) {
    while (i < p.size() && p[i] == '/') ++i;
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    if (j > i) {
      // storage.ParsePathEscaped: url.PathUnescape each segment
      out.emplace_back();
      std::string& u = out.back();
      u.reserve(j - i);
      for (size_t k = i; k < j; ++k) {
        if (p[k] == '%' && k + 2 < j && isxdigit((unsigned char)p[k + 1]) && isxdigit((unsigned char)p[k + 2])) {
          u.push_back((char)(hexval(p[k + 1]) * 16 + hexval(p[k + 2])));
          k += 2;
        } else u.push_back(p[k]);
      }
    }
    i = j;
  }
  return out;
}

// `templates["t"]["K"]` / `hooks["t"].library` -> path segments
static std::vector<std::string> pkg_path(const std::string& name) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i < name.size()) {
    if (name[i] == '.') { ++i; continue; }
    if (name[i] == '[') {
      size_t q = name.find('"', i);
      size_t q2 = name.find('"', q + 1);
      out.push_back(name.substr(q + 1, q2 - q - 1));
      i = name.find(']', q2) + 1;
      continue;
    }
    size_t j = i;
    while (j < name.size() && name[j] != '.' && name[j] != '[') ++j;
    out.push_back(name.substr(i, j - i));
    i = j;
  }
  return out;
}

}  // namespace gk

using namespace gk;

// gk_last_error: the message of this thread's last failed call (concurrent
// callers do not see each other's errors)
static thread_local std::string tl_err;
static int fail(gk_engine*, int code, const std::string& m) {
  tl_err = m;
  return code;
}

// ------------------------------------------------------------------ modules
static void rebuild_modules(gk_engine* e) {
  if (!e->modules_dirty) return;
  e->mods.clear();
  e->bank.clear();
  e->progs.clear();
  for (auto& j : e->jits) if (j.mod) hipModuleUnload(j.mod);
  e->jits.clear();
  e->templates.clear();
  // drop the transient region before appending new permanent constant nodes
  reset_transient(e);
  if (e->inv_node == NO_ID) {
    Node n{};
    n.type = NT_OBJ;
    e->inv_node = e->st.add_node(n);  // {} until sync_inventory builds the tree
    e->perm_nodes = (uint32_t)e->st.nodes().size();
  }
  e->bank.inventory_node = e->inv_node;
  e->uses_inventory = false;
  const size_t n_before = e->st.nodes().size();
  std::vector<std::shared_ptr<rego::Module>> parsed;
  for (auto& kv : e->modules) {
    auto m = rego::parse_module(kv.second);
    // the frameworks hooks + target library are served natively
    if (!m->pkg.empty() && m->pkg[0] == "hooks") continue;
    // GKGPU_REGO_SETS: set-algebra rewrites (rego.cc), a mask of the two
    // patterns, both on by default (profiles/r04/r04x_ab.txt: config 4
    // 1,582 -> 1,656 M evals/s against the comprehension form alone, whose
    // per-(container, probe) list made K8sRequiredProbes 1.86 -> 2.49 ms)
    if (const int sets = env_mode("GKGPU_REGO_SETS", 3, 3)) {
      const int n = rego::optimize_sets(*m, sets);
      if (getenv("GKGPU_SETS_TRACE")) fprintf(stderr, "optimize_sets %s: %d rewrites\n", kv.first.c_str(), n);
    }
    e->mods.add(m);
    parsed.push_back(m);
  }
  for (auto& m : parsed) {
    if (m->pkg.size() != 3 || m->pkg[0] != "templates" || m->pkg[1] != TARGET) continue;
    const std::string& kind = m->pkg[2];
    if (e->templates.count(kind)) continue;
    TemplateEnt te;
    te.kind = kind;
    try {
      Program p;
      try {
        p = compile_template(e->st, e->mods, m->pkg, e->bank);
        if (p.nregs > 192) throw Unsupported("register file too large");
      } catch (const Unsupported& ex) {
        // outside the subset: the guard program evaluates the match and every
        // body prefix before the first unsupported expression on the device;
        // only reviews that reach it go to the CPU (compile_template_guard)
        te.reason = ex.what();
        size_t code0 = e->bank.code.size();
        p = compile_template_guard(e->st, e->mods, m->pkg, e->bank);
        if (p.nregs > 192) {
          e->bank.code.resize(code0);
          throw;
        }
        te.guard = true;
      }
      // structural validation of the bytecode before it can reach the device:
      // the template program, then each join site's key program
      auto validate = [&](uint32_t off, uint32_t len, uint32_t nregs, bool key) {
        for (uint32_t k = 0; k < len; ++k) {
          const Ins& in = e->bank.code[off + k];
          auto reg_ok = [&](uint16_t r) { return r < nregs || r == 0xffff; };
          if (in.op >= OP_COUNT_) throw std::runtime_error("internal: bad opcode");
          const bool no_regs = in.op == OP_END || in.op == OP_JMP || in.op == OP_FAIL_FALLBACK || in.op == OP_ORD;
          if (!no_regs && (!reg_ok(in.a) || !reg_ok(in.b) || (in.op != OP_EMIT && !reg_ok(in.c))))
            throw std::runtime_error("internal: register out of range");
          if (in.op == OP_ITER_INIT && in.a + 1u >= nregs) throw std::runtime_error("internal: iterator registers");
          if (in.op == OP_CALL && in.b + (uint32_t)in.c > nregs) throw std::runtime_error("internal: call args");
          bool jmp = in.op == OP_JMP || in.op == OP_JUNDEF || in.op == OP_JFALSE || in.op == OP_JTRUE ||
                     in.op == OP_ITER_NEXT || in.op == OP_MEMO_GET || in.op == OP_JPROBE || in.op == OP_JNEXT;
          if ((in.op == OP_JPROBE && in.a + 1u >= nregs) || (in.op == OP_JVAR && in.b + 1u >= nregs))
            throw std::runtime_error("internal: join iterator registers");
          if (in.op == OP_JPROBE && (key || (in.y >> 8) >= p.joins.size())) throw std::runtime_error("internal: join site");
          if (!key && in.op == OP_KEYOUT)
            throw std::runtime_error("internal: key output in a template program");
          if (key && (in.op == OP_EMIT || in.op == OP_JNEXT || in.op == OP_JVAR))
            throw std::runtime_error("internal: emission in a join key program");
          if ((in.op == OP_MEMO_GET || in.op == OP_MEMO_PUT) && in.y >= MEMO_SLOTS) throw std::runtime_error("internal: memo slot");
          if (jmp && (in.x < off || in.x >= off + len)) throw std::runtime_error("internal: jump target");
          if ((in.op == OP_LOADK || in.op == OP_GETK) && in.x >= e->bank.consts.size()) throw std::runtime_error("internal: constant index");
          if (in.op == OP_SPRINTF && in.x >= e->bank.fmt.size()) throw std::runtime_error("internal: format index");
          if (in.op == OP_TABLE && (in.x >= e->bank.consts.size() || in.x + 1 + 2 * e->bank.consts[in.x] > e->bank.consts.size()))
            throw std::runtime_error("internal: table bounds");
        }
      };
      validate(p.code_off, p.code_len, p.nregs, false);
      for (auto& js : p.joins) validate(js.key_off, js.key_len, js.key_nregs, true);
      te.prog = (int)e->progs.size();
      te.supported = !te.guard;
      e->uses_inventory |= p.uses_inventory;
      e->progs.push_back(p);
      gk_engine::Jit j;
      j.name = jit_name(p, e->bank, e->st);
      j.src = jit_source(p, e->bank, e->st, j.name);
      e->jits.push_back(std::move(j));
    } catch (const std::exception& ex) {
      te.supported = false;
      te.guard = false;
      te.prog = -1;
      if (te.reason.empty()) te.reason = ex.what();
    }
    e->templates[kind] = te;
  }
  e->perm_nodes = (uint32_t)e->st.nodes().size();
  e->module_nodes = e->st.nodes().size() - n_before;
  e->modules_dirty = false;
  e->constraints_dirty = true;
  e->gen++;
}

// ------------------------------------------------------------------ constraint match compile
// Encodes a label selector (target_template_source.go:185-230) into match words.
static void encode_selector(Store& st, uint32_t sel, std::vector<uint32_t>& w) {
  size_t head = w.size();
  w.push_back(0);  // flags: 1 never, 2 error
  uint32_t flags = 0;
  // matchLabels := get_default(selector, "matchLabels", {})
  uint32_t ml = st.nodes().size() && sel != NO_ID && ntype(st, sel) == NT_OBJ ? gdef(st, sel, "matchLabels") : NO_ID;
  std::vector<std::pair<uint32_t, uint32_t>> pairs;
  uint8_t mt = ntype(st, ml);
  if (ml != NO_ID) {
    if (mt == NT_OBJ) {
      const Node n = st.nodes()[ml];
      for (uint32_t i = 0; i < n.n; ++i) {
        const Node& c = st.nodes()[n.first + i];
        pairs.push_back({c.key, c.type == NT_STR ? c.val : NO_ID});
      }
    } else if (mt == NT_ARR) {
      if (st.nodes()[ml].n > 0) flags |= 1;
    } else if (mt == NT_STR) {
      if (st.str(st.nodes()[ml].val).size() > 0) flags |= 1;
    } else {
      flags |= 2;  // count(number/bool)
    }
  }
  w.push_back((uint32_t)pairs.size());
  for (auto& p : pairs) { w.push_back(p.first); w.push_back(p.second); }
  // matchExpressions := get_default(selector, "matchExpressions", [])
  uint32_t me = ntype(st, sel) == NT_OBJ ? gdef(st, sel, "matchExpressions") : NO_ID;
  size_t nex_pos = w.size();
  w.push_back(0);
  uint32_t nex = 0;
  uint8_t met = ntype(st, me);
  if (met == NT_ARR || met == NT_OBJ) {
    const Node n = st.nodes()[me];
    for (uint32_t i = 0; i < n.n; ++i) {
      uint32_t ex = n.first + i;
      if (ntype(st, ex) != NT_OBJ) continue;  // me["operator"] undefined
      uint32_t opn = nget(st, ex, "operator"), keyn = nget(st, ex, "key");
      if (opn == NO_ID || keyn == NO_ID) continue;
      uint32_t op = SO_OTHER, ops;
      if (nstr(st, opn, &ops)) {
        if (ops == st.s_In) op = SO_IN;
        else if (ops == st.s_NotIn) op = SO_NOTIN;
        else if (ops == st.s_Exists) op = SO_EXISTS;
        else if (ops == st.s_DoesNotExist) op = SO_DOESNOTEXIST;
      }
      uint32_t key = NO_ID;
      nstr(st, keyn, &key);
      uint32_t vals = gdef(st, ex, "values");
      uint32_t vflags = 0;
      std::vector<uint32_t> vs;
      uint8_t vt = ntype(st, vals);
      if (vals == NO_ID) {
        // [] : count 0
      } else if (vt == NT_ARR || vt == NT_OBJ) {
        const Node vn = st.nodes()[vals];
        if (vn.n > 0) vflags |= 1;
        for (uint32_t j = 0; j < vn.n; ++j) {
          uint32_t s;
          if (nstr(st, vn.first + j, &s)) vs.push_back(s);
        }
      } else if (vt == NT_STR) {
        if (st.str(st.nodes()[vals].val).size() > 0) vflags |= 1;
      } else {
        vflags |= 2;
      }
      w.push_back(op);
      w.push_back(key);
      w.push_back(vflags);
      w.push_back((uint32_t)vs.size());
      for (auto s : vs) w.push_back(s);
      ++nex;
    }
  }
  w[nex_pos] = nex;
  w[head] = flags;
}

static void compile_constraint(gk_engine* e, ConstraintEnt& c) {
  Store& st = e->st;
  MatchSpec m{};
  m.prog = NO_ID;
  m.params = NO_ID;
  auto& W = e->mwords;
  uint32_t root = c.root;
  // spec := get_default(constraint, "spec", {}); match := get_default(spec, "match", {})
  uint32_t spec = gdef(st, root, "spec");
  uint32_t match = ntype(st, spec) == NT_OBJ ? gdef(st, spec, "match") : NO_ID;
  if (ntype(st, match) != NT_OBJ) match = NO_ID;
  // kinds
  m.kinds_off = (uint32_t)W.size();
  uint32_t kinds = match == NO_ID ? NO_ID : gdef(st, match, "kinds");
  if (kinds == NO_ID) {
    W.push_back(1);
    W.push_back(1); W.push_back(0xfffffffeu);
    W.push_back(1); W.push_back(0xfffffffeu);
  } else {
    uint8_t kt = ntype(st, kinds);
    std::vector<uint32_t> sel;
    uint32_t nsel = 0;
    if (kt == NT_ARR || kt == NT_OBJ) {
      const Node kn = st.nodes()[kinds];
      for (uint32_t i = 0; i < kn.n; ++i) {
        uint32_t ks = kn.first + i;
        std::vector<uint32_t> gs, ks2;
        for (int which = 0; which < 2; ++which) {
          uint32_t lst = ntype(st, ks) == NT_OBJ ? nget(st, ks, which == 0 ? "apiGroups" : "kinds") : NO_ID;
          uint8_t lt = ntype(st, lst);
          if (lt == NT_ARR || lt == NT_OBJ) {
            const Node ln = st.nodes()[lst];
            for (uint32_t j = 0; j < ln.n; ++j) {
              uint32_t s;
              if (nstr(st, ln.first + j, &s)) (which == 0 ? gs : ks2).push_back(s == st.s_star ? 0xfffffffeu : s);
            }
          }
        }
        sel.push_back((uint32_t)gs.size());
        sel.insert(sel.end(), gs.begin(), gs.end());
        sel.push_back((uint32_t)ks2.size());
        sel.insert(sel.end(), ks2.begin(), ks2.end());
        ++nsel;
      }
    }
    W.push_back(nsel);
    W.insert(W.end(), sel.begin(), sel.end());
  }
  auto enc_list = [&](const char* f, uint32_t flag, uint32_t* off) {
    *off = (uint32_t)W.size();
    uint32_t n = match == NO_ID ? NO_ID : nget(st, match, f);
    if (n == NO_ID) { W.push_back(0); return; }
    m.flags |= flag;
    std::vector<uint32_t> ids;
    uint8_t t = ntype(st, n);
    if (t == NT_ARR || t == NT_OBJ) {
      const Node ln = st.nodes()[n];
      for (uint32_t j = 0; j < ln.n; ++j) { uint32_t s; if (nstr(st, ln.first + j, &s)) ids.push_back(s); }
    }
    W.push_back((uint32_t)ids.size());
    W.insert(W.end(), ids.begin(), ids.end());
  };
  enc_list("namespaces", MF_HAS_NAMESPACES, &m.ns_off);
  enc_list("excludedNamespaces", MF_HAS_EXCLUDED, &m.exns_off);
  // namespaceSelector
  m.nssel_off = (uint32_t)W.size();
  if (match != NO_ID && nget(st, match, "namespaceSelector") != NO_ID) {
    m.flags |= MF_HAS_NSSEL;
    encode_selector(st, gdef(st, match, "namespaceSelector"), W);
  } else {
    encode_selector(st, NO_ID, W);
  }
  // scope
  uint32_t scope = match == NO_ID ? NO_ID : nget(st, match, "scope");
  if (scope != NO_ID) {
    m.flags |= MF_SCOPE_PRESENT;
    uint32_t s;
    if (nstr(st, scope, &s)) {
      std::string_view sv = st.str(s);
      if (sv == "*") m.flags |= MF_SCOPE_ANY;
      else if (sv == "Namespaced") m.flags |= MF_SCOPE_NS;
      else if (sv == "Cluster") m.flags |= MF_SCOPE_CLUSTER;
    }
  }
  m.labelsel_off = (uint32_t)W.size();
  encode_selector(st, match == NO_ID ? NO_ID : gdef(st, match, "labelSelector"), W);
  // hooks-level get_default (regolib/src.go:77-85): defined values (incl. null) win
  uint32_t hspec = nget(st, root, "spec");
  uint32_t params = ntype(st, hspec) == NT_OBJ ? nget(st, hspec, "parameters") : NO_ID;
  m.params = params;
  uint32_t ea = ntype(st, hspec) == NT_OBJ ? nget(st, hspec, "enforcementAction") : NO_ID;
  c.ea_error = false;
  if (ea == NO_ID) c.ea = "deny";
  else if (ntype(st, ea) == NT_STR) c.ea = std::string(st.str(st.nodes()[ea].val));
  else if (ntype(st, ea) == NT_NULL) c.ea = "";
  else { c.ea = ""; c.ea_error = true; }
  auto it = e->templates.find(c.kind);
  if (it != e->templates.end()) {
    // whole-template or guard program; without either, every matched review
    // goes to CPU OPA (devrt.h audit_body)
    if (it->second.prog >= 0) m.prog = (uint32_t)it->second.prog;
    else m.flags |= MF_FALLBACK;
  }
  c.spec = m;
}

// data.inventory = data.external[target], or {} without one (regolib
// src.go:66-72).  The synced objects (gk_put_data on /external/<target>/...)
// are assembled into one JSON tree by path segment, parsed into the permanent
// node region, and the engine's inventory node is pointed at its members, so
// compiled templates (a constant V_NODE of that node) see the current tree.
// Rebuilt lazily, only when a compiled template reads data.inventory.  The
// new tree replaces the previous one in place when that was the last thing in
// the permanent region; otherwise the old tree's nodes are garbage until the
// region is compacted (maybe_compact).
static void sync_inventory(gk_engine* e) {
  if (!e->uses_inventory || !e->inv_dirty || e->inv_node == NO_ID) return;
  const bool tr = getenv("GKGPU_PREPARE_TRACE") != nullptr;
  auto tp = Clock::now();
  auto step = [&](const char* what) {
    if (tr) fprintf(stderr, "inventory: %s %.1f ms\n", what, ms_since(tp));
    tp = Clock::now();
  };
  // the synced objects under /external/<target>/, their paths split (URL
  // unescaped) and ordered segment by segment -- the tree's member order
  std::vector<std::pair<const std::string*, const std::string*>> kvs;
  kvs.reserve(e->inventory.size());
  for (auto& kv : e->inventory) kvs.push_back({&kv.first, &kv.second});
  std::vector<std::vector<std::string>> segs(kvs.size());
  const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)default_threads(), kvs.size() / 4096));
  parallel_run(T, [&](int t) {
    for (size_t i = kvs.size() * t / T; i < kvs.size() * (t + 1) / T; ++i) segs[i] = split_path(*kvs[i].first);
  });
  std::vector<uint32_t> ents;
  ents.reserve(kvs.size());
  for (uint32_t i = 0; i < kvs.size(); ++i) {
    const auto& p = segs[i];
    if (p.size() < 3 || p[0] != "external" || p[1] != TARGET) continue;
    ents.push_back(i);
  }
  // (segments 0 and 1 are equal for every entry: order by the rest)
  step("split");
  auto seg_less = [&](uint32_t a, uint32_t b) {
    return std::lexicographical_compare(segs[a].begin() + 2, segs[a].end(), segs[b].begin() + 2, segs[b].end());
  };
  // the map's raw-path order is usually the segment order already (it is not
  // when an escape or a segment that prefixes another reorders them): check
  // in parallel, sort only if needed
  std::atomic<bool> sorted{true};
  if (ents.size() > 1) {
    const int TS = (int)std::max<size_t>(1, std::min<size_t>((size_t)default_threads(), ents.size() / 4096));
    parallel_run(TS, [&](int t) {
      const size_t m = ents.size() - 1;
      for (size_t i = m * t / TS; i < m * (t + 1) / TS && sorted.load(std::memory_order_relaxed); ++i)
        if (seg_less(ents[i + 1], ents[i])) sorted = false;
    });
  }
  if (!sorted) std::stable_sort(ents.begin(), ents.end(), seg_less);
  step("sort");
  const size_t n = ents.size();
  reset_transient(e);
  if (e->inv_hi > e->inv_lo && e->inv_hi == e->perm_nodes) {
    // the previous tree is the region's tail: reuse its space
    e->st.nodes().resize(e->inv_lo);
    e->perm_nodes = e->inv_lo;
  }
  e->inv_lo = (uint32_t)e->st.nodes().size();
  // every object parsed on the host threads into the permanent region
  // (flatten_docs), then the tree of path segments above them
  std::vector<std::string_view> docs(n);
  for (size_t i = 0; i < n; ++i) docs[i] = *kvs[ents[i]].second;
  NodeArena dst;
  std::vector<uint32_t> roots;
  std::string err;
  if (!flatten_docs(e->st, e->smu, docs, e->inv_lo, dst, roots, err)) throw std::runtime_error("inventory tree: " + err);
  step("flatten");
  {
    NodeArena& N = e->st.nodes();
    const size_t at = N.size();
    N.resize(at + dst.size());
    if (dst.size()) memcpy(N.data() + at, dst.data(), dst.size() * sizeof(Node));
  }
  // entries [lo, hi) share their first `depth` segments; a leaf at a segment
  // shadows deeper paths under it (one value per path); an object of more than
  // 0xffff members keeps the first 0xffff (flags bit 0), as parsed documents do
  std::function<Node(size_t, size_t, size_t)> tree = [&](size_t lo, size_t hi, size_t depth) -> Node {
    std::vector<std::pair<size_t, size_t>> groups;
    for (size_t i = lo; i < hi;) {
      const std::string& seg = segs[ents[i]][depth];
      size_t j = i;
      while (j < hi && segs[ents[j]][depth] == seg) ++j;
      groups.push_back({i, j});
      i = j;
    }
    Node o{};
    o.type = NT_OBJ;
    size_t cnt = groups.size();
    if (cnt > 0xffff) { o.flags |= 1; cnt = 0xffff; }
    const uint32_t first = (uint32_t)e->st.nodes().size();
    e->st.nodes().resize(first + cnt);
    for (size_t g = 0; g < cnt; ++g) {
      const size_t i = groups[g].first;
      const std::string& seg = segs[ents[i]][depth];
      Node c = segs[ents[i]].size() == depth + 1 ? e->st.nodes()[roots[i]] : tree(i, groups[g].second, depth + 1);
      c.key = e->st.intern(seg);
      e->st.nodes()[first + g] = c;
    }
    o.first = cnt ? first : 0;
    o.n = (uint16_t)cnt;
    return o;
  };
  const Node t = tree(0, n, 2);
  step("tree");
  e->inv_hi = (uint32_t)e->st.nodes().size();
  Node& slot = e->st.nodes()[e->inv_node];
  slot.type = t.type;
  slot.first = t.first;
  slot.n = t.n;
  slot.flags = t.flags;
  e->perm_nodes = (uint32_t)e->st.nodes().size();
  e->dev_nodes_ok = std::min<uint32_t>(e->dev_nodes_ok, std::min(e->inv_node, e->inv_lo));
  e->inv_dirty = false;
}

// Compaction of the permanent node region (under the exclusive lock): replaced
// or deleted constraints, namespaces and inventory trees leave their nodes
// behind (node ids are never reused while anything may refer to them).  When
// that garbage outgrows the live documents, the region is rebuilt from the
// kept JSON texts: constraints, cached namespaces, then the modules'
// constants and the inventory tree (rebuild_modules / sync_inventory).
static void maybe_compact(gk_engine* e, bool force = false) {
  uint64_t live = e->base_nodes + e->module_nodes + (e->inv_hi - e->inv_lo);
  for (auto& kv : e->constraints) live += kv.second.nnodes;
  for (auto& kv : e->ns_nodes) live += kv.second.second;
  const uint64_t garbage = e->perm_nodes > live ? e->perm_nodes - live : 0;
  // GKGPU_COMPACT_MIN (tests): compact as soon as the garbage exceeds this
  // many nodes (default: max(2^20, live nodes))
  const char* cm = getenv("GKGPU_COMPACT_MIN");
  const uint64_t limit = cm && *cm ? (uint64_t)atoll(cm) : std::max<uint64_t>(1u << 20, live);
  if (!force && garbage <= limit) return;
  e->st.nodes().resize(e->base_nodes);
  e->perm_nodes = e->base_nodes;
  e->dev_nodes_ok = 0;
  e->inv_node = NO_ID;
  e->inv_lo = e->inv_hi = 0;
  e->inv_dirty = true;
  e->modules_dirty = true;
  e->constraints_dirty = true;
  JDoc d;
  for (auto& kv : e->constraints) {
    ConstraintEnt& c = kv.second;
    JsonReader rd(c.json.data(), c.json.size(), &d);
    const int root = rd.parse();
    const size_t n0 = e->st.nodes().size();
    c.root = root >= 0 ? e->st.add_doc(d, root) : NO_ID;
    c.nnodes = (uint32_t)(e->st.nodes().size() - n0);
  }
  for (auto& kv : e->ns_nodes) {
    auto it = e->inventory.end();
    for (auto jt = e->inventory.begin(); jt != e->inventory.end(); ++jt) {
      auto q = split_path(jt->first);
      if (q.size() == 6 && q[2] == "cluster" && q[3] == "v1" && q[4] == "Namespace" && q[5] == kv.first) { it = jt; }
    }
    if (it == e->inventory.end()) continue;
    JsonReader rd(it->second.data(), it->second.size(), &d);
    const int root = rd.parse();
    const size_t n0 = e->st.nodes().size();
    const uint32_t node = root >= 0 ? e->st.add_doc(d, root) : NO_ID;
    kv.second = {node, (uint32_t)(e->st.nodes().size() - n0)};
    e->ns_cache[kv.first] = node;
  }
  e->perm_nodes = (uint32_t)e->st.nodes().size();
  e->gen++;
}

static void rebuild_constraints(gk_engine* e) {
  rebuild_modules(e);
  sync_inventory(e);
  if (!e->constraints_dirty) return;
  e->mwords.clear();
  e->corder.clear();
  for (auto& kv : e->constraints) {
    compile_constraint(e, kv.second);
    e->corder.push_back(&kv.second);
  }
  e->constraints_dirty = false;
}

// ------------------------------------------------------------------ regex tables
static void rebuild_regex(gk_engine* e) {
  // literal patterns of templates + every string in constraint parameters when a
  // template calls re_match with a computed pattern
  bool any_regex = false;
  std::vector<uint32_t> pats;
  for (auto& p : e->progs) {
    if (p.uses_regex) any_regex = true;
    pats.insert(pats.end(), p.regex_literals.begin(), p.regex_literals.end());
  }
  if (!any_regex) return;
  for (auto* c : e->corder) {
    uint32_t pr = c->spec.params;
    if (pr == NO_ID) continue;
    std::vector<uint32_t> stack{pr};
    while (!stack.empty()) {
      uint32_t n = stack.back();
      stack.pop_back();
      const Node nd = e->st.nodes()[n];
      if (nd.type == NT_STR) pats.push_back(nd.val);
      if (nd.type == NT_ARR || nd.type == NT_OBJ) for (uint32_t i = 0; i < nd.n; ++i) stack.push_back(nd.first + i);
    }
  }
  bool changed = false;
  for (uint32_t sid : pats) {
    if (e->dfa_index.count(sid)) continue;
    std::vector<uint32_t> words;
    int status = compile_regex_dfa(std::string(e->st.str(sid)), words);
    uint32_t off = (uint32_t)e->dfa_words.size();
    if (status == RX_OK) e->dfa_words.insert(e->dfa_words.end(), words.begin(), words.end());
    e->dfa_index[sid] = {off, (uint32_t)status};
    changed = true;
  }
  if (changed) {
    e->dfa_keys.clear();
    e->dfa_meta.clear();
    for (auto& kv : e->dfa_index) {
      e->dfa_keys.push_back(kv.first);
      e->dfa_meta.push_back(kv.second.first | (kv.second.second << 30));
    }
  }
}

// ------------------------------------------------------------------ LDS stage plan
// Per constraint (devrt.h stage_wave): the node window holding its whole
// parameters subtree, and the compressed DFAs of the regex patterns among its
// parameter strings (what re_match with a parameter pattern reads).
static void rebuild_stage(gk_engine* e) {
  e->stage.clear();
  const bool any_regex = !e->dfa_index.empty();
  for (auto* c : e->corder) {
    MatchSpec& m = c->spec;
    m.plo = 0;
    m.pn = 0;
    m.stage_off = NO_ID;
    if (m.params == NO_ID) continue;
    uint32_t lo = m.params, hi = m.params;
    std::vector<uint32_t> strs, stack{m.params};
    while (!stack.empty()) {
      const uint32_t n = stack.back();
      stack.pop_back();
      lo = std::min(lo, n);
      hi = std::max(hi, n);
      const Node nd = e->st.nodes()[n];
      if (nd.type == NT_STR) strs.push_back(nd.val);
      if (nd.type == NT_ARR || nd.type == NT_OBJ)
        for (uint32_t i = 0; i < nd.n; ++i) stack.push_back(nd.first + i);
    }
    m.plo = lo;
    m.pn = hi - lo + 1;
    if (!any_regex) continue;
    std::vector<uint32_t> rec;
    uint32_t bytes = 0;
    std::set<uint32_t> seen;
    for (uint32_t sid : strs) {
      if (!seen.insert(sid).second) continue;
      auto it = e->dfa_index.find(sid);
      if (it == e->dfa_index.end() || it->second.second != RX_OK) continue;
      auto ct = e->cdfa_index.find(sid);
      if (ct == e->cdfa_index.end()) {
        const size_t off = it->second.first, nst0 = e->dfa_words[off];
        const size_t len = std::min(e->dfa_words.size() - off, 3 + nst0 * 129);
        std::vector<uint32_t> dw(e->dfa_words.begin() + off, e->dfa_words.begin() + off + len);
        std::vector<uint8_t> t;
        uint32_t nst = 0, ncls = 0, start = 0, sens = 0;
        std::vector<uint32_t> ent;
        if (compress_regex_dfa(dw, 1024, t, nst, ncls, start, sens)) {
          ent = {(uint32_t)e->dfa_c.size(), (uint32_t)t.size(), nst | (ncls << 16), start | (sens << 16)};
          t.resize((t.size() + 3) & ~(size_t)3, 0);
          for (size_t k = 0; k < t.size(); k += 4) {
            uint32_t w;
            memcpy(&w, t.data() + k, 4);
            e->dfa_c.push_back(w);
          }
        }
        ct = e->cdfa_index.emplace(sid, ent).first;
      }
      if (ct->second.empty()) continue;
      const uint32_t nb = (ct->second[1] + 3) & ~3u;
      if (bytes + nb > 1024 || rec.size() / 5 >= 4) continue;  // devrt.h LDS_DFA_BYTES / LDS_DFA_MAX
      bytes += nb;
      rec.push_back(sid);
      rec.insert(rec.end(), ct->second.begin(), ct->second.end());
    }
    if (rec.empty()) continue;
    m.stage_off = (uint32_t)e->stage.size();
    e->stage.push_back((uint32_t)(rec.size() / 5));
    e->stage.insert(e->stage.end(), rec.begin(), rec.end());
  }
}

// ------------------------------------------------------------------ device sync + launch
static bool ensure_device(gk_engine* e) {
  if (e->dev_ok) return true;
  if (e->host_only) return false;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= e->device) return false;
  if (hipSetDevice(e->device) != hipSuccess) return false;
  e->dev_ok = true;
  return true;
}

template <class T>
static bool up(DBuf& b, const std::vector<T>& v, bool append_only) {
  return b.upload(v.data(), v.size() * sizeof(T), append_only);
}

// The string / number tables' new tails to the device (append-only), and the
// pointers an evaluation launches with.  Under smu: evaluations intern while
// they flatten.
static bool sync_strings(gk_engine* e, TablePtrs* out) {
  std::lock_guard<std::mutex> g(e->smu);
  if (hipSetDevice(e->device) != hipSuccess) return false;
  Store& st = e->st;
  const auto t0 = Clock::now();
  const size_t s0 = e->d_strs.used, p0 = e->d_pool.used;
  bool ok = up(e->d_strs, st.strings(), true);
  const double ms_strs = ms_since(t0);
  // +16: the device reads string bytes a dword at a time (devrt.h puts_) and may
  // touch up to 3 bytes past the last string
  ok = ok && e->d_pool.reserve(st.pool().size() + 16);
  const double ms_pres = ms_since(t0);
  ok = ok && e->d_pool.upload(st.pool().data(), st.pool().size(), true);
  const double ms_pool = ms_since(t0);
  ok = ok && up(e->d_sflags, st.str_flags(), true);
  ok = ok && up(e->d_nums, st.numbers(), true);
  if (getenv("GKGPU_FLATTEN_TRACE"))
    fprintf(stderr, "sync strings: entries %.1f ms (%zu -> %zu B), pool reserve %.1f ms, pool %.1f ms (%zu -> %zu B), flags+numbers %.1f ms\n",
            ms_strs, s0, e->d_strs.used, ms_pres - ms_strs, ms_pool - ms_pres, p0, e->d_pool.used, ms_since(t0) - ms_pool);
  if (out) {
    out->strs = (const StrEnt*)e->d_strs.p;
    out->pool = (const uint8_t*)e->d_pool.p;
    out->sflags = (const uint8_t*)e->d_sflags.p;
    out->nums = (const NumEnt*)e->d_nums.p;
  }
  return ok;
}

// The permanent tables to the device (under the exclusive lock: no evaluation
// in flight): the permanent node region's new tail, bytecode, constants,
// formats, constraints' match words, regex DFAs.
static bool sync_tables(gk_engine* e) {
  Store& st = e->st;
  bool ok = true;
  const size_t n = st.nodes().size();
  ok &= e->d_nodes.reserve(std::max<size_t>(n, 1) * sizeof(Node));
  if (ok && n > e->dev_nodes_ok)
    ok &= hipMemcpy((char*)e->d_nodes.p + (size_t)e->dev_nodes_ok * sizeof(Node), st.nodes().data() + e->dev_nodes_ok,
                    (n - e->dev_nodes_ok) * sizeof(Node), hipMemcpyHostToDevice) == hipSuccess;
  if (ok) { e->dev_nodes_ok = (uint32_t)n; e->d_nodes.used = n * sizeof(Node); }
  ok &= sync_strings(e, nullptr);
  ok &= up(e->d_code, e->bank.code, false);
  ok &= up(e->d_K, e->bank.consts, false);
  std::vector<uint32_t> fmt = e->bank.fmt;
  if (fmt.empty()) fmt.push_back(0);
  ok &= up(e->d_fmt, fmt, false);
  {
    // the format table with literal segments resolved to (0 | len << 8,
    // offset in the literal bytes): the size / format passes keep it in LDS
    // and print literals without the string table and pool (DevArgs.fmtr)
    std::vector<uint32_t> fr(fmt.size(), 0);
    std::string fb;
    bool okr = true;
    for (size_t off = 0; okr && off + 2 <= e->bank.fmt.size();) {
      const uint32_t nseg = e->bank.fmt[off];
      if (off + 2 + 2 * (size_t)nseg > e->bank.fmt.size()) { okr = false; break; }
      fr[off] = nseg;
      fr[off + 1] = e->bank.fmt[off + 1];
      for (uint32_t sg = 0; sg < nseg; ++sg) {
        const uint32_t kind = e->bank.fmt[off + 2 + 2 * sg], a = e->bank.fmt[off + 3 + 2 * sg];
        if (kind == 0) {
          const std::string_view lit = e->st.str(a);
          if (lit.size() >= (1u << 24)) { okr = false; break; }
          fr[off + 2 + 2 * sg] = (uint32_t)lit.size() << 8;
          fr[off + 3 + 2 * sg] = (uint32_t)fb.size();
          fb.append(lit.data(), lit.size());
        } else {
          fr[off + 2 + 2 * sg] = kind;
          fr[off + 3 + 2 * sg] = a;
        }
      }
      off += 2 + 2 * (size_t)nseg;
    }
    e->nfmtr = 0;
    e->nfmtb = 0;
    if (okr && !e->bank.fmt.empty()) {
      std::vector<uint32_t> fbw((fb.size() + 3) / 4 + 1, 0);
      memcpy(fbw.data(), fb.data(), fb.size());
      ok &= up(e->d_fmtr, fr, false) && up(e->d_fmtb, fbw, false);
      e->nfmtr = (uint32_t)fr.size();
      e->nfmtb = (uint32_t)fb.size();
    }
  }
  std::vector<MatchSpec> cons;
  for (auto* c : e->corder) cons.push_back(c->spec);
  if (cons.empty()) cons.push_back(MatchSpec{});
  ok &= up(e->d_cons, cons, false);
  std::vector<uint32_t> mw = e->mwords;
  if (mw.empty()) mw.push_back(0);
  ok &= up(e->d_mwords, mw, false);
  std::vector<uint32_t> po;
  for (auto& p : e->progs) po.push_back(p.code_off);
  if (po.empty()) po.push_back(0);
  ok &= up(e->d_progoff, po, false);
  std::vector<uint32_t> dk = e->dfa_keys, dm = e->dfa_meta, dw = e->dfa_words;
  if (dk.empty()) { dk.push_back(NO_ID); dm.push_back(2u << 30); }
  if (dw.empty()) dw.push_back(0);
  ok &= up(e->d_dfa_keys, dk, false);
  ok &= up(e->d_dfa_meta, dm, false);
  ok &= up(e->d_dfa_words, dw, false);
  std::vector<uint32_t> sg = e->stage, dc = e->dfa_c;
  if (sg.empty()) sg.push_back(0);
  if (dc.empty()) dc.push_back(0);
  ok &= up(e->d_stage, sg, false);
  ok &= up(e->d_dfa_c, dc, false);
  return ok;
}

// ------------------------------------------------------------------ inventory join indexes
// The value a lane sees for node `idx` (devrt.h nodeval), on the host.
static uint64_t host_nodeval(const Store& st, uint32_t idx) {
  const Node& n = st.nodes()[idx];
  switch (n.type) {
    case NT_NULL: return tag_val(V_NULL, 0);
    case NT_FALSE: return tag_val(V_BOOL, 0);
    case NT_TRUE: return tag_val(V_BOOL, 1);
    case NT_NUM: return tag_val(V_NUM, n.val);
    case NT_STR: return tag_val(V_STR, n.val);
    case NT_ARR: case NT_OBJ: return tag_val(V_NODE, idx);
  }
  return tag_val(V_UNDEF, 0);
}

// The solutions of `data.inventory<path>` in the order the device's
// iteration (op_iter_next / vget over the node store) produces them: rows of
// [leaf value, key at each variable selector].
static void enum_leaves(const Store& st, uint64_t v, const std::vector<JoinSite::Sel>& path, size_t q,
                        std::vector<uint64_t>& keys, std::vector<uint64_t>& rows, bool* arr_var) {
  if (q == path.size()) {
    rows.push_back(v);
    rows.insert(rows.end(), keys.begin(), keys.end());
    return;
  }
  if ((v >> 60) != V_NODE) return;  // a scalar has no members
  const uint32_t idx = (uint32_t)(v & 0x0fffffffffffffffull);
  const Node n = st.nodes()[idx];
  if (path[q].var) {
    if (n.type != NT_OBJ && n.n) *arr_var = true;  // a path variable bound to an index, not a string
    for (uint32_t c = 0; c < n.n; ++c) {
      const uint32_t ci = n.first + c;
      keys.push_back(n.type == NT_OBJ ? tag_val(V_STR, st.nodes()[ci].key) : tag_val(V_INT, c));
      enum_leaves(st, host_nodeval(st, ci), path, q + 1, keys, rows, arr_var);
      keys.pop_back();
    }
    return;
  }
  if (n.type != NT_OBJ) return;  // a string key selects nothing in an array
  for (uint32_t c = 0; c < n.n; ++c)
    if (st.nodes()[n.first + c].key == path[q].sid) {
      enum_leaves(st, host_nodeval(st, n.first + c), path, q + 1, keys, rows, arr_var);
      return;
    }
}

// Per (constraint, join site): the site's leaves are enumerated once per
// template, the key pass (kernels.hip gk_key_kernel) computes every leaf's key
// bucket on the device under the constraint's parameters, and the (hash, leaf
// row) pairs are sorted by hash, leaves in iteration order within a hash.  A
// key pass with a failed lane leaves the site unindexed (jdir ready = 0): its
// lanes take the plain scan, which reports that failure where the reference
// would.  Rebuilt whenever the engine is prepared (any mutation), under the
// exclusive lock, after sync_tables.
// The join plan of the current state (host data work, every prepare): the
// leaf rows of every (template, site) and one key-pass record per
// (constraint, site): [constraint, site, key program pc, row stride, first row
// word, leaves, parameters value, flags].  flags 1: a path variable iterates
// an array somewhere in the tree -- the planner assumed path variables are
// object keys (strings: compiler.cc err_free_call), so the site scans.
static void plan_joins(gk_engine* e) {
  e->jleaf.clear();
  e->jsite.clear();
  bool any = false;
  for (auto& p : e->progs) any = any || !p.joins.empty();
  if (!any || e->inv_node == NO_ID) return;
  Store& st = e->st;
  std::map<std::pair<uint32_t, uint32_t>, std::pair<uint64_t, uint32_t>> rows;  // -> (row0, leaves)
  std::map<std::pair<uint32_t, uint32_t>, bool> arr;
  for (uint32_t pi = 0; pi < e->progs.size(); ++pi)
    for (uint32_t s = 0; s < e->progs[pi].joins.size(); ++s) {
      const JoinSite& js = e->progs[pi].joins[s];
      const uint64_t row0 = e->jleaf.size();
      std::vector<uint64_t> keys;
      bool arr_var = false;
      enum_leaves(st, tag_val(V_NODE, e->inv_node), js.path, 0, keys, e->jleaf, &arr_var);
      rows[{pi, s}] = {row0, (uint32_t)((e->jleaf.size() - row0) / (1 + js.nvars))};
      arr[{pi, s}] = arr_var;
    }
  for (uint32_t ci = 0; ci < e->corder.size(); ++ci) {
    const MatchSpec& m = e->corder[ci]->spec;
    if (m.prog == NO_ID || (m.flags & MF_FALLBACK) || m.prog >= e->progs.size()) continue;
    const Program& p = e->progs[m.prog];
    for (uint32_t s = 0; s < p.joins.size() && s < JMAX_SITES; ++s) {
      const auto rw = rows[{m.prog, s}];
      const uint64_t params = m.params == NO_ID ? tag_val(V_NODE, 0) : host_nodeval(st, m.params);
      e->jsite.insert(e->jsite.end(),
                      {ci, s, p.joins[s].key_off, 1u + p.joins[s].nvars, rw.first, rw.second, params, arr[{m.prog, s}] ? 1u : 0u});
    }
  }
}

static bool build_joins(gk_engine* e) {
  const auto t0 = std::chrono::steady_clock::now();
  const size_t ncons = std::max<size_t>(e->corder.size(), 1);
  e->jdir.assign(ncons * JMAX_SITES * 4, 0);
  e->jhash.clear();
  e->jord.clear();
  e->join_indexes = e->join_entries = e->join_unindexed = e->join_leaves = 0;
  const bool any = !e->jsite.empty();
  bool ok = true;
  if (any) {
    std::vector<uint64_t> jl = e->jleaf;
    if (jl.empty()) jl.push_back(0);
    ok = ok && up(e->d_jleaf, jl, false);
    TablePtrs tp;
    ok = ok && sync_strings(e, &tp);
    std::vector<uint64_t> keys;
    for (size_t q = 0; ok && q < e->jsite.size(); q += 8) {
      const uint64_t* sr = &e->jsite[q];
      const uint32_t ci = (uint32_t)sr[0], s = (uint32_t)sr[1];
      const std::pair<uint64_t, uint32_t> rw{sr[4], (uint32_t)sr[5]};
      {
        uint32_t* dir = &e->jdir[((size_t)ci * JMAX_SITES + s) * 4];
        dir[0] = (uint32_t)e->jhash.size();
        dir[1] = 0;
        dir[2] = 0;
        const uint32_t stride = (uint32_t)sr[3];
        if (sr[7] & 1) { ++e->join_unindexed; continue; }
        keys.assign((size_t)rw.second * JKEYS_MAX, KH_NONE);
        if (rw.second) {
          ok = ok && e->d_jkeys.reserve((size_t)rw.second * JKEYS_MAX * 8);
          if (!ok) break;
          DevArgs a{};
          a.nodes = (const Node*)e->d_nodes.p;
          a.strs = tp.strs;
          a.pool = tp.pool;
          a.sflags = tp.sflags;
          a.nums = tp.nums;
          a.code = (const Ins*)e->d_code.p;
          a.K = (const uint64_t*)e->d_K.p;
          a.fmt = (const uint32_t*)e->d_fmt.p;
          a.cons = (const MatchSpec*)e->d_cons.p;
          a.mwords = (const uint32_t*)e->d_mwords.p;
          a.prog_off = (const uint32_t*)e->d_progoff.p;
          a.dfa_keys = (const uint32_t*)e->d_dfa_keys.p;
          a.dfa_meta = (const uint32_t*)e->d_dfa_meta.p;
          a.dfa_words = (const uint32_t*)e->d_dfa_words.p;
          a.stage = (const uint32_t*)e->d_stage.p;
          a.dfa_c = (const uint32_t*)e->d_dfa_c.p;
          a.ndfa = (uint32_t)std::max<size_t>(e->dfa_keys.size(), 1);
          a.ncode = (uint32_t)e->bank.code.size();
          a.ncons = (uint32_t)e->corder.size();
          a.nrev = rw.second;
          a.jleaf = (const uint64_t*)e->d_jleaf.p;
          a.jkeys = (uint64_t*)e->d_jkeys.p;
          a.jparams = sr[6];
          a.jpc = (uint32_t)sr[2];
          a.jstride = stride;
          a.jrow0 = rw.first;
          ok = gk_launch_keys(&a, nullptr) == 0 && hipStreamSynchronize(nullptr) == hipSuccess &&
               hipMemcpy(keys.data(), e->d_jkeys.p, keys.size() * 8, hipMemcpyDeviceToHost) == hipSuccess;
          if (!ok) break;
        }
        e->join_leaves += rw.second;
        bool failed = false;
        std::vector<std::pair<uint64_t, uint32_t>> ent;
        for (uint32_t i = 0; i < rw.second && !failed; ++i) {
          const uint64_t* k = &keys[(size_t)i * JKEYS_MAX];
          if (k[0] == KH_FAIL) { failed = true; break; }
          // a leaf once per distinct hash of its key values (the probe's body
          // iterates them itself)
          for (uint32_t j = 0; j < JKEYS_MAX && k[j] != KH_NONE; ++j) {
            bool dup = false;
            for (uint32_t h = 0; h < j; ++h) dup = dup || k[h] == k[j];
            if (!dup) ent.push_back({k[j], (uint32_t)(rw.first + (uint64_t)i * stride)});
          }
        }
        if (failed) { ++e->join_unindexed; continue; }
        std::stable_sort(ent.begin(), ent.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
        for (auto& en : ent) { e->jhash.push_back(en.first); e->jord.push_back(en.second); }
        dir[1] = (uint32_t)ent.size();
        dir[2] = 1;
        ++e->join_indexes;
        e->join_entries += ent.size();
      }
    }
  }
  std::vector<uint64_t> jh = e->jhash;
  std::vector<uint32_t> jo = e->jord;
  if (jh.empty()) jh.push_back(0);
  if (jo.empty()) jo.push_back(0);
  if (e->jleaf.empty()) { std::vector<uint64_t> z{0}; ok = ok && up(e->d_jleaf, z, false); }
  ok = ok && up(e->d_jdir, e->jdir, false) && up(e->d_jhash, jh, false) && up(e->d_jord, jo, false);
  e->joins_built = ok && any;
  e->join_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (getenv("GKGPU_JOIN_TRACE"))
    fprintf(stderr, "joins: %llu indexes, %llu entries, %llu unindexed, %llu leaves, %.2f ms\n",
            (unsigned long long)e->join_indexes, (unsigned long long)e->join_entries,
            (unsigned long long)e->join_unindexed, (unsigned long long)e->join_leaves, e->join_ms);
  return ok;
}

// The join index pointers a launch passes (null: every site scans).
static void set_join_args(const gk_engine* e, DevArgs& a) {
  if (!e->joins_built) return;
  a.jdir = (const uint32_t*)e->d_jdir.p;
  a.jhash = (const uint64_t*)e->d_jhash.p;
  a.jord = (const uint32_t*)e->d_jord.p;
  a.jleaf = (const uint64_t*)e->d_jleaf.p;
}

// Compiles (hipRTC, in parallel) every template kernel not yet built; with a
// device, loads the code objects.  A template whose kernel fails to compile
// stays on the bytecode VM kernel (same semantics, slower).
static void ensure_jit(gk_engine* e, bool load) {
  if (!e->jit_enabled) return;
  std::vector<std::thread> th;
  for (auto& j : e->jits) {
    if (j.state != 0) continue;
    th.emplace_back([&j] { j.state = jit_compile(j.src, j.code, j.log) ? 1 : -1; });
  }
  for (auto& t : th) t.join();
  if (!load) return;
  std::vector<gk_engine::Jit*> all;
  for (auto& j : e->jits) all.push_back(&j);
  for (auto* jp : all) {
    auto& j = *jp;
    if (j.state != 1 || j.fn) continue;
    if (hipModuleLoadData(&j.mod, j.code.data()) != hipSuccess ||
        hipModuleGetFunction(&j.fn, j.mod, j.name.c_str()) != hipSuccess) {
      if (j.mod) hipModuleUnload(j.mod);
      j.mod = nullptr;
      j.fn = nullptr;
      j.state = -1;
      j.log = "module load failed";
    }
  }
}

// ------------------------------------------------------------------ locking
// Brings the compiled state (templates, constraints' match words, inventory
// tree, regex DFAs) and the device tables up to date with the last mutation.
// Called with the exclusive lock held.
static int prepare_locked(gk_engine* e, bool device) {
  // GKGPU_PREPARE_TRACE: the time of each step on stderr
  const bool tr = getenv("GKGPU_PREPARE_TRACE") != nullptr;
  auto tp = Clock::now();
  auto step = [&](const char* what) {
    if (tr) fprintf(stderr, "prepare: %s %.1f ms\n", what, ms_since(tp));
    tp = Clock::now();
  };
  try {
    maybe_compact(e);
    step("compact");
    rebuild_constraints(e);
    step("constraints");
    rebuild_regex(e);
    step("regex");
    rebuild_stage(e);
    step("stage");
    plan_joins(e);
    step("plan joins");
  } catch (const std::exception& ex) {
    return fail(e, GK_EPARSE, ex.what());
  }
  if (device && ensure_device(e)) {
    ensure_jit(e, true);
    step("jit");
    if (!sync_tables(e)) return fail(e, GK_EDEVICE, "device upload failed");
    step("tables");
    // without indexes every join site scans (same results): a failed build
    // (device memory, a key-pass launch) costs time, not correctness
    if (!build_joins(e)) {
      e->joins_built = false;
      fprintf(stderr, "gkgpu: inventory join indexes not built (%s); join sites scan\n",
              hipGetErrorString(hipGetLastError()));
    }
    step("joins");
  }
  e->prepared_gen = e->gen;
  // the device side was brought up to date, or there is no device to use
  // (the evaluation then fails with GK_EDEVICE)
  e->prepared_dev = device;
  return GK_OK;
}

static bool prepared(const gk_engine* e, bool device) {
  return e->prepared_gen == e->gen && (!device || e->prepared_dev);
}

// An evaluation's hold on the engine: the shared lock, taken once the engine
// is prepared for this state (a stale engine is prepared under the exclusive
// lock first, then the shared lock is taken again).
struct ReadLock {
  std::shared_lock<std::shared_mutex> lk;
};
// the shared lock without preparing (reads of the mutation-side state)
static void read_lock_raw(gk_engine* e, ReadLock& r) {
  { std::lock_guard<std::mutex> t(e->turn); }
  r.lk = std::shared_lock<std::shared_mutex>(e->rw);
}
static int read_lock(gk_engine* e, ReadLock& r, bool device) {
  for (;;) {
    { std::lock_guard<std::mutex> t(e->turn); }
    r.lk = std::shared_lock<std::shared_mutex>(e->rw);
    if (prepared(e, device)) return GK_OK;
    r.lk.unlock();
    std::lock_guard<std::mutex> t(e->turn);
    std::unique_lock<std::shared_mutex> w(e->rw);
    if (!prepared(e, device)) {
      int rc = prepare_locked(e, device);
      if (rc != GK_OK) return rc;
    }
  }
}

// A mutation's hold: new readers queue behind it on `turn`
struct WriteLock {
  std::lock_guard<std::mutex> t;
  std::unique_lock<std::shared_mutex> w;
  explicit WriteLock(gk_engine* e) : t(e->turn), w(e->rw) {}
};

// An evaluation context from the pool (a new one when all are busy)
struct CtxLease {
  gk_engine* e;
  EvalCtx* x = nullptr;
  std::unique_lock<std::mutex> hold;
  explicit CtxLease(gk_engine* eng) : e(eng) {
    std::lock_guard<std::mutex> g(e->pool_mu);
    for (auto& c : e->ctxs) {
      std::unique_lock<std::mutex> h(c->busy, std::try_to_lock);
      if (h.owns_lock()) { x = c.get(); hold = std::move(h); return; }
    }
    e->ctxs.push_back(std::make_unique<EvalCtx>());
    x = e->ctxs.back().get();
    x->out_cap = e->out_cap0;
    if (const char* tc = getenv("GKGPU_TEST_CAPS")) {
      // tests: initial tuple, staged-byte and output-byte capacities (overflow paths)
      unsigned long long t = 0, eb = 0, b = 0;
      if (sscanf(tc, "%llu,%llu,%llu", &t, &eb, &b) == 3 && t && eb && b) {
        x->out_cap = t;
        x->ebytes_cap = eb;
        x->bytes_cap = b;
      }
    }
    hold = std::unique_lock<std::mutex>(x->busy);
  }
};

// device-to-host copy on the context's stream (concurrent evaluations do not
// serialize on the null stream)
static bool d2h(EvalCtx* x, void* dst, const void* src, size_t n) {
  if (!n) return true;
  return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, x->stream) == hipSuccess &&
         hipStreamSynchronize(x->stream) == hipSuccess;
}

static bool ctx_device(gk_engine* e, EvalCtx* x) {
  if (hipSetDevice(e->device) != hipSuccess) return false;
  if (!x->stream && hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess) return false;
  return true;
}

// The device node array of a query: the engine's permanent region (copied on
// the device, once per engine state) followed by the call's documents.
static bool ctx_nodes(gk_engine* e, EvalCtx* x, const NodeArena& arena) {
  const size_t perm = e->perm_nodes;
  if (!x->d_nodes.reserve((perm + arena.size() + 1) * sizeof(Node))) return false;
  // a grown buffer starts empty (DBuf::reserve keeps only uploaded bytes): the
  // permanent region is copied again into it
  if (x->perm_gen != e->prepared_gen || x->perm_nodes != perm || x->perm_buf != x->d_nodes.p) {
    if (perm && hipMemcpyAsync(x->d_nodes.p, e->d_nodes.p, perm * sizeof(Node), hipMemcpyDeviceToDevice, x->stream) != hipSuccess)
      return false;
    x->perm_gen = e->prepared_gen;
    x->perm_nodes = (uint32_t)perm;
    x->perm_buf = x->d_nodes.p;
  }
  if (arena.size() &&
      hipMemcpyAsync((char*)x->d_nodes.p + perm * sizeof(Node), arena.data(), arena.size() * sizeof(Node),
                     hipMemcpyHostToDevice, x->stream) != hipSuccess)
    return false;
  return hipStreamSynchronize(x->stream) == hipSuccess;
}

// Runs the launch plan over `cols` on the evaluation context `x` (its stream
// and output buffers): `revbuf` holds the columns on the device (uploaded here
// when it is the context's own buffer), `nodes` the documents, `tp` the string
// tables as of this call.  Shared lock held.
static int launch_and_collect(gk_engine* e, EvalCtx* x, const TablePtrs& tp, const std::vector<ReviewCol>& cols,
                              DBuf* revbuf, bool decode, gk_results* res, const void* nodes, uint64_t n_excluded = 0,
                              uint32_t nperm = NO_ID, bool audit = false, const gk_batch* colb = nullptr) {
  if (nperm == NO_ID) nperm = e->perm_nodes;  // a query's documents follow the engine's permanent region
  uint32_t nrev = (uint32_t)cols.size();
  uint32_t ncons = (uint32_t)e->corder.size();
  res->nrev = nrev;
  res->gen = e->gen;
  res->excluded = n_excluded;
  res->totals.assign(ncons, 0);
  for (auto* c : e->corder) {
    res->ckind.push_back(c->kind);
    res->cname.push_back(c->name);
    res->cea.push_back(c->ea);
    res->cea_error.push_back(c->ea_error);
  }
  if (nrev == 0) return GK_OK;
  // reviews the process excluder skipped (manager.go:362-365) carry GK_REVIEW_EXCLUDED
  auto mark_excluded = [&]() {
    if (!n_excluded) return;
    if (res->status.empty()) { res->status.assign(nrev, 0); res->reason.assign(nrev, 0); }
    for (uint32_t r = 0; r < nrev; ++r)
      if (cols[r].flags & RC_EXCLUDED) res->status[cols[r].orig == NO_ID ? r : cols[r].orig] |= GK_REVIEW_EXCLUDED;
  };
  // reviews flagged for fallback on the host never reach the device when there are no constraints
  if (ncons == 0) {
    res->status.assign(nrev, 0);
    res->reason.assign(nrev, 0);
    for (uint32_t r = 0; r < nrev; ++r)
      if (cols[r].flags & RC_FALLBACK) res->status[cols[r].orig == NO_ID ? r : cols[r].orig] = GK_REVIEW_FALLBACK;
    mark_excluded();
    return GK_OK;
  }
  if (!e->dev_ok || !ctx_device(e, x)) return fail(e, GK_EDEVICE, "no HIP device available");
  res->ctx = x;
  auto t0 = Clock::now();
  if (revbuf == &x->d_revs || !revbuf->p || revbuf->used != cols.size() * sizeof(ReviewCol)) {
    if (!up(*revbuf, cols, false)) return fail(e, GK_EDEVICE, "device upload failed");
  }
  // output buffers: tuples + their deferred-argument words (frec, structure of
  // arrays), bytes staged at emission (ebytes), per-tuple byte counts and tile
  // sums of the size pass, final message bytes (+16: dword reads past the end)
  auto reserve_out = [&]() {
    return x->d_out.reserve(x->out_cap * sizeof(Viol)) && x->d_frec.reserve(x->out_cap * FMT_MAXARGS * 8) &&
           x->d_out_raw.reserve(x->out_cap * sizeof(Viol)) && x->d_frec_raw.reserve(x->out_cap * FMT_MAXARGS * 8) &&
           x->d_ctcnt.reserve((x->out_cap / 256 + 2) * 4) && x->d_ctoff.reserve((x->out_cap / 256 + 2) * 8) &&
           x->d_lens.reserve(x->out_cap * 4) && x->d_part.reserve((x->out_cap / FTILE + 2) * 8) &&
           x->d_ebytes.reserve(x->ebytes_cap + 16) && x->d_bytes.reserve(x->bytes_cap + 16);
  };
  bool ok = x->d_rflags.reserve(nrev * 4) && x->d_rreason.reserve(nrev * 4) && x->d_totals.reserve(ncons * 8) &&
            x->d_counters.reserve(64 + 16 * (e->progs.size() + 1)) && reserve_out();
  if (!ok) return fail(e, GK_EDEVICE, "device allocation failed");
  // launch plan: constraints grouped by template kernel (jit.cc); the bytecode
  // VM kernel takes every constraint whose template has no kernel / program
  ensure_jit(e, true);
  struct Step { hipFunction_t fn; std::string name; uint32_t off, n; };
  std::vector<Step> plan;
  std::vector<uint32_t> clist_host;  // constraint indices in launch order
  {
    std::vector<std::vector<uint32_t>> groups(e->progs.size() + 1);
    for (uint32_t c = 0; c < ncons; ++c) {
      uint32_t p = e->corder[c]->spec.prog;
      bool jit = p != NO_ID && p < e->jits.size() && e->jits[p].fn;
      groups[jit ? p : e->progs.size()].push_back(c);
    }
    std::vector<uint32_t>& clist = clist_host;
    for (size_t g = 0; g < groups.size(); ++g) {
      if (groups[g].empty()) continue;
      bool vm = g == e->progs.size();
      plan.push_back({vm ? nullptr : e->jits[g].fn, vm ? std::string("audit_kernel") : e->jits[g].name,
                      (uint32_t)clist.size(), (uint32_t)groups[g].size()});
      clist.insert(clist.end(), groups[g].begin(), groups[g].end());
    }
    if (!up(x->d_clist, clist, false)) return fail(e, GK_EDEVICE, "device upload failed");
  }
  res->ms[1] = ms_since(t0);
  for (int attempt = 0; attempt < 4; ++attempt) {
    // per-call state (flags, reasons, totals, counters, memo-string cursor, memo
    // tables) is zeroed by one gk_zero dispatch below, once the streams are known
    bool prof = e->profile && x->d_prof.reserve(ncons * 32);
    if (prof) hipMemsetAsync(x->d_prof.p, 0, ncons * 32, x->stream);
    DevArgs a{};
    a.prof = prof ? (unsigned long long*)x->d_prof.p : nullptr;
    uint32_t ncode = (uint32_t)e->bank.code.size();
    bool hist = e->profile >= 2 && x->d_pchist.reserve(ncode * 4);
    if (hist) hipMemsetAsync(x->d_pchist.p, 0, ncode * 4, x->stream);
    a.pchist = hist ? (unsigned int*)x->d_pchist.p : nullptr;
    a.nodes = (const Node*)nodes;
    // memo keys on permanent nodes (devrt.h gm_key); GKGPU_MEMO_NODES=0: scalars only (A/B)
    a.nperm = env_mode("GKGPU_MEMO_NODES", 1, 1) ? nperm : 0;
    // memo-string arena (devrt.h gm_value_slow): one per evaluation, read by
    // the format pass after every template launch (GKGPU_MEMO_STRINGS=0: off, A/B)
    if (env_mode("GKGPU_GMEMO", 1, 1) != 0 && env_mode("GKGPU_MEMO_STRINGS", 1, 1) != 0 &&
        x->d_mstr.reserve(MSTR_BYTES) && x->d_mtop.reserve(8)) {
      a.mstr = (char*)x->d_mstr.p;
      a.mstr_top = (unsigned long long*)x->d_mtop.p;
      a.mstr_cap = MSTR_BYTES;
    }
    a.strs = tp.strs;
    a.pool = tp.pool;
    a.sflags = tp.sflags;
    a.nums = tp.nums;
    a.code = (const Ins*)e->d_code.p;
    a.K = (const uint64_t*)e->d_K.p;
    a.fmt = (const uint32_t*)e->d_fmt.p;
    if (e->nfmtr && env_mode("GKGPU_FMT_RESOLVED", 1, 1)) {  // A/B switch (default on)
      a.fmtr = (const uint32_t*)e->d_fmtr.p;
      a.fmtb = (const char*)e->d_fmtb.p;
      a.nfmt = e->nfmtr;
      a.nfmtb = e->nfmtb;
    }
    a.cons = (const MatchSpec*)e->d_cons.p;
    a.mwords = (const uint32_t*)e->d_mwords.p;
    a.prog_off = (const uint32_t*)e->d_progoff.p;
    a.revs = (const ReviewCol*)revbuf->p;
    a.dfa_keys = (const uint32_t*)e->d_dfa_keys.p;
    a.dfa_meta = (const uint32_t*)e->d_dfa_meta.p;
    a.dfa_words = (const uint32_t*)e->d_dfa_words.p;
    a.stage = (const uint32_t*)e->d_stage.p;
    a.dfa_c = (const uint32_t*)e->d_dfa_c.p;
    a.ndfa = (uint32_t)std::max<size_t>(e->dfa_keys.size(), 1);
    a.ncode = (uint32_t)e->bank.code.size();
    a.ncons = ncons;
    a.nrev = nrev;
    a.ntiles = (nrev + 63) / 64;
    a.out = (Viol*)x->d_out.p;
    a.out_cap = x->out_cap;
    a.counters = (unsigned long long*)x->d_counters.p;
    a.bytes = (char*)x->d_bytes.p;
    a.bytes_cap = x->bytes_cap;
    a.rflags = (uint32_t*)x->d_rflags.p;
    a.totals = (unsigned long long*)x->d_totals.p;
    a.rreason = (uint32_t*)x->d_rreason.p;
    a.frec = (uint64_t*)x->d_frec.p;
    a.ebytes = (char*)x->d_ebytes.p;
    a.ebytes_cap = x->ebytes_cap;
    a.lens = (uint32_t*)x->d_lens.p;
    a.part = (unsigned long long*)x->d_part.p;
    if (colb && colb->columnar) {  // the batch's documents in column form (colstore.h)
      a.cv_words = (const uint32_t*)colb->d_cv_words.p;
      a.cv_bytes = (const uint8_t*)colb->d_cv_bytes.p;
      a.cv_slots = (const CvSlot*)colb->d_cv_slots.p;
      a.cv_hash = (const CvHash*)colb->d_cv_hash.p;
      a.cv_views = (const uint32_t*)colb->d_cv_views.p;
      a.cv_tabs = (const uint32_t*)colb->d_cv_tabs.p;
      a.cv_hmask = (uint32_t)colb->cv.hash.size() - 1;
      a.cv_on = 1;
    }
    set_join_args(e, a);
    while (x->events.size() < plan.size() + 5) {
      hipEvent_t ev1;
      if (hipEventCreate(&ev1) != hipSuccess) return fail(e, GK_EDEVICE, "event creation failed");
      x->events.push_back(ev1);
    }
    const std::vector<hipEvent_t>& ev = x->events;
    hipEventRecord(ev[0], x->stream);
    // GKGPU_CONCURRENT: the template launches go round-robin to the context's
    // stream and up to three side streams, each with its own memo table, and
    // run side by side; the compaction waits for all of them.  Per-launch
    // timing uses per-launch events.  Default (2): micro-batches only (up to
    // 65,536 reviews: latency-bound launches); a sweep's launches each fill
    // the GPU and measured no faster side by side (profiles/r04/r04s_ab.txt).
    int nstream = 1;
    const int conc = env_mode("GKGPU_CONCURRENT", 2, 2);
    if (plan.size() > 1 && (conc == 1 || (conc == 2 && nrev <= 65536))) {
      nstream = (int)std::min<size_t>(plan.size(), 1 + EvalCtx::kSide);
      for (int k = 0; k + 1 < nstream; ++k)
        if (!x->side[k] && hipStreamCreateWithFlags(&x->side[k], hipStreamNonBlocking) != hipSuccess) { nstream = k + 1; break; }
    }
    while (x->lev.size() < 2 * plan.size() + 1) {
      hipEvent_t ev1;
      if (hipEventCreate(&ev1) != hipSuccess) return fail(e, GK_EDEVICE, "event creation failed");
      x->lev.push_back(ev1);
    }
    const hipEvent_t ev_go = x->lev[2 * plan.size()];
    {
      // one dispatch zeroes the call's state and every used stream's memo table
      // (launches sharing a table salt their memo hashes: DevArgs gm_salt)
      const bool gm_on = env_mode("GKGPU_GMEMO", 1, 1) != 0;  // A/B switch
      void* zp[12];
      uint64_t zb[12];
      uint32_t zn = 0;
      auto zero = [&](void* p, uint64_t b) { if (p && b) { zp[zn] = p; zb[zn] = b; ++zn; } };
      zero(x->d_rflags.p, (uint64_t)nrev * 4);
      zero(x->d_rreason.p, (uint64_t)nrev * 4);
      zero(x->d_totals.p, (uint64_t)ncons * 8);
      zero(x->d_counters.p, 64 + 16 * (uint64_t)plan.size());
      if (a.mstr_top) zero(x->d_mtop.p, 8);
      bool any_fn = false;
      for (auto& pl : plan) any_fn = any_fn || pl.fn;
      for (int si = 0; si < nstream && gm_on && any_fn; ++si) {
        DBuf& gm = si == 0 ? x->d_gmemo : x->d_gmemo_side[si - 1];
        if (gm.reserve((size_t)GMEMO_ENTRIES * 32)) zero(gm.p, (uint64_t)GMEMO_ENTRIES * 32);
      }
      if (gk_launch_zero(zp, zb, zn, x->stream) != 0) return fail(e, GK_EDEVICE, "launch failed");
    }
    if (nstream > 1) {
      hipEventRecord(ev_go, x->stream);
      for (int k = 0; k + 1 < nstream; ++k) hipStreamWaitEvent(x->side[k], ev_go, 0);
    }
    std::vector<DevArgs> argv(plan.size(), a);  // live until the stream sync below
    for (size_t i = 0; i < plan.size(); ++i) {
      const int si = nstream > 1 ? (int)(i % (size_t)nstream) : 0;
      hipStream_t st = si == 0 ? x->stream : x->side[si - 1];
      DBuf& gmemo = si == 0 ? x->d_gmemo : x->d_gmemo_side[si - 1];
      argv[i].clist = (const uint32_t*)x->d_clist.p + plan[i].off;
      argv[i].nclist = plan[i].n;
      // chunked tuple slots go to the raw arrays; gk_compact packs them below
      argv[i].out = (Viol*)x->d_out_raw.p;
      argv[i].frec = (uint64_t*)x->d_frec_raw.p;
      const DevArgs& a = argv[i];
      int lr;
      hipEventRecord(x->lev[2 * i], st);
      if (plan[i].fn) {
        // template kernel: a cleared cross-lane memo table (devrt.h gm_get)
        const bool gm_on = env_mode("GKGPU_GMEMO", 1, 1) != 0;  // A/B switch
        if (gm_on && gmemo.reserve((size_t)GMEMO_ENTRIES * 32)) {  // (zeroed above)
          argv[i].gmemo = (uint64_t*)gmemo.p;
          argv[i].gmemo_mask = GMEMO_ENTRIES - 1;
          argv[i].gm_salt = (uint64_t)(i + 1) * 0xd6e8feb86659fd93ull;
        }
        uint64_t threads = (uint64_t)a.ntiles * a.nclist * 64;
        uint32_t blocks = (uint32_t)((threads + 255) / 256);
        // the arguments travel in the dispatch's kernarg segment (devrt.h gk_args)
        void* params[] = {(void*)&argv[i]};
        lr = (int)hipModuleLaunchKernel(plan[i].fn, blocks, 1, 1, 256, 1, 1, 0, st, params, nullptr);
      } else {
        lr = gk_launch_audit(&a, st);
      }
      hipEventRecord(x->lev[2 * i + 1], st);
      // cumulative (tuples, bytes) after this launch -> per-launch output counts
      // (tuples: counters[6], the waves' used slots; counters[0] counts holes
      // too); concurrent launches: from the constraint totals instead (below)
      if (nstream == 1) {
        hipMemcpyAsync((char*)x->d_counters.p + 64 + 16 * i, (char*)x->d_counters.p + 48, 8, hipMemcpyDeviceToDevice, st);
        hipMemcpyAsync((char*)x->d_counters.p + 72 + 16 * i, (char*)x->d_counters.p + 8, 8, hipMemcpyDeviceToDevice, st);
      }
      if (lr != 0) {
        return fail(e, GK_EDEVICE, "kernel launch failed (" + plan[i].name + "): " + hipGetErrorString((hipError_t)lr));
      }
    }
    for (int k = 0; k + 1 < nstream; ++k) {  // join the side streams
      hipEventRecord(x->lev[2 * plan.size()], x->side[k]);
      hipStreamWaitEvent(x->stream, x->lev[2 * plan.size()], 0);
    }
    hipEventRecord(ev[plan.size()], x->stream);
    // the tuples of every launch above packed, then the size, spine and format passes
    // pass grids sized for ~2x this context's last output (GKGPU_PASS_HINT=0: for the capacity)
    const uint64_t pass_hint = env_mode("GKGPU_PASS_HINT", 1, 1) ? std::max<uint64_t>(2 * x->last_tuples, 65536) : 0;
    int flr = gk_launch_compact(&a, (const Viol*)x->d_out_raw.p, (const uint64_t*)x->d_frec_raw.p,
                                (uint32_t*)x->d_ctcnt.p, (unsigned long long*)x->d_ctoff.p, x->stream, pass_hint);
    if (flr != 0) return fail(e, GK_EDEVICE, std::string("kernel launch failed (compact): ") + hipGetErrorString((hipError_t)flr));
    hipEventRecord(ev[plan.size() + 1], x->stream);
    flr = gk_launch_format(&a, x->stream, &x->events[plan.size() + 2], pass_hint);
    if (flr != 0) return fail(e, GK_EDEVICE, std::string("kernel launch failed (format): ") + hipGetErrorString((hipError_t)flr));
    // one wait for the kernels and the small readbacks: counters, per-launch
    // counter snapshots, totals, and the per-review flags and reasons, queued
    // into the context's pinned buffer
    const size_t o_snap = 32, o_tot = o_snap + 16 * plan.size(), o_fl = o_tot + 8 * (size_t)ncons,
                 o_rs = o_fl + 4 * (size_t)nrev, o_end = o_rs + 4 * (size_t)nrev;
    char* hp = x->pin(o_end);
    if (!hp) return fail(e, GK_EDEVICE, "pinned host allocation failed");
    bool qok = hipMemcpyAsync(hp, x->d_counters.p, 32, hipMemcpyDeviceToHost, x->stream) == hipSuccess &&
               hipMemcpyAsync(hp + o_snap, (char*)x->d_counters.p + 64, 16 * plan.size(), hipMemcpyDeviceToHost,
                              x->stream) == hipSuccess &&
               hipMemcpyAsync(hp + o_tot, x->d_totals.p, 8 * (size_t)ncons, hipMemcpyDeviceToHost, x->stream) == hipSuccess;
    // a large batch (an audit sweep) reads the per-review words only when
    // something was flagged (below); a micro-batch reads them right away
    const bool early_flags = nrev <= 65536;
    if (early_flags)
      qok = qok &&
            hipMemcpyAsync(hp + o_fl, x->d_rflags.p, 4 * (size_t)nrev, hipMemcpyDeviceToHost, x->stream) == hipSuccess &&
            hipMemcpyAsync(hp + o_rs, x->d_rreason.p, 4 * (size_t)nrev, hipMemcpyDeviceToHost, x->stream) == hipSuccess;
    if (!qok || hipStreamSynchronize(x->stream) != hipSuccess) return fail(e, GK_EDEVICE, "kernel execution failed");
    // [0] tuples, [1] staged bytes, [2] lanes that flagged their review (error/fallback), [3] output bytes
    uint64_t counters[4];
    memcpy(counters, hp, 32);
    if (getenv("GKGPU_LAUNCH_TRACE"))
      fprintf(stderr, "launch: attempt %d, %zu launches, slots %llu (cap %zu), staged bytes %llu (cap %zu)\n", attempt,
              plan.size(), (unsigned long long)counters[0], x->out_cap, (unsigned long long)counters[1], x->ebytes_cap);
    if (counters[0] > x->out_cap || counters[1] > x->ebytes_cap) {
      x->out_cap = std::max<size_t>(x->out_cap * 2, counters[0] + 1024);
      x->ebytes_cap = std::max<size_t>(x->ebytes_cap * 2, (size_t)counters[1] + 65536);
      if (!reserve_out()) return fail(e, GK_EDEVICE, "device allocation failed");
      continue;
    }
    if (counters[3] > x->bytes_cap) {
      // the tuples are complete; only the output bytes did not fit: grow them
      // and run the passes again
      x->bytes_cap = std::max<size_t>(x->bytes_cap * 2, (size_t)counters[3] + 65536);
      if (!reserve_out()) return fail(e, GK_EDEVICE, "device allocation failed");
      a.bytes = (char*)x->d_bytes.p;
      a.bytes_cap = x->bytes_cap;
      flr = gk_launch_format(&a, x->stream, &x->events[plan.size() + 2], pass_hint);
      if (flr != 0 || hipStreamSynchronize(x->stream) != hipSuccess) return fail(e, GK_EDEVICE, "format pass failed");
      d2h(x, counters, x->d_counters.p, 32);
    }
    res->launches.clear();
    std::vector<uint64_t> snap(2 * plan.size());
    memcpy(snap.data(), hp + o_snap, 16 * plan.size());
    std::vector<uint64_t> ctot(ncons);
    memcpy(ctot.data(), hp + o_tot, ncons * 8);
    {
      float all = 0;
      hipEventElapsedTime(&all, ev[0], ev[plan.size()]);
      res->ms[2] += all;  // predicate launches: wall time (they may overlap)
    }
    for (size_t i = 0; i < plan.size(); ++i) {
      float kms = 0;
      hipEventElapsedTime(&kms, x->lev[2 * i], x->lev[2 * i + 1]);
      uint64_t tup = 0, byt = 0;
      if (nstream == 1) {
        const uint64_t t0 = i ? snap[2 * i - 2] : 0, b0 = i ? snap[2 * i - 1] : 0;
        tup = snap[2 * i] - t0;
        byt = snap[2 * i + 1] - b0;
      } else {  // the launch's constraints' clean emissions (bytes: not split per launch)
        for (uint32_t k = 0; k < plan[i].n; ++k) tup += ctot[clist_host[plan[i].off + k]];
      }
      res->launches.push_back({plan[i].name, (double)kms, plan[i].n, tup, byt});
    }
    {
      float k_cmp = 0, k_size = 0, k_spine = 0, k_fmt = 0;
      hipEventElapsedTime(&k_cmp, ev[plan.size()], ev[plan.size() + 1]);
      hipEventElapsedTime(&k_size, ev[plan.size() + 1], ev[plan.size() + 2]);
      hipEventElapsedTime(&k_spine, ev[plan.size() + 2], ev[plan.size() + 3]);
      hipEventElapsedTime(&k_fmt, ev[plan.size() + 3], ev[plan.size() + 4]);
      res->ms[2] += k_cmp + k_size + k_spine + k_fmt;
      res->launches.push_back({"gk_compact", (double)k_cmp, 0, counters[0], 0});
      res->launches.push_back({"gk_size_kernel", (double)k_size, 0, 0, 0});
      res->launches.push_back({"gk_scan_spine", (double)k_spine, 0, 0, 0});
      res->launches.push_back({"gk_format_kernel", (double)k_fmt, 0, 0, counters[3]});
    }
    auto t1 = Clock::now();
    res->dev_tuples = counters[0];
    x->last_tuples = counters[0];
    res->dev_bytes = counters[3];
    res->failed_lanes = counters[2];
    res->epoch = ++x->eval_epoch;
    std::vector<uint64_t> tot(ncons);
    memcpy(tot.data(), hp + o_tot, ncons * 8);
    for (uint32_t c = 0; c < ncons; ++c) res->totals[c] = tot[c];
    bool ea_err = false;
    for (auto* c : e->corder) ea_err |= c->ea_error;
    if (!decode && !ea_err && counters[2] == 0 && !hist && !prof) {
      // nothing flagged: per-review status stays implicit (all zero), so the
      // audit step downloads a few counters instead of 8 bytes per review
      res->ms[3] = ms_since(t1);
      mark_excluded();
      return GK_OK;
    }
    res->status.assign(nrev, 0);
    res->reason.assign(nrev, 0);
    if (early_flags) {
      memcpy(res->status.data(), hp + o_fl, nrev * 4);
      memcpy(res->reason.data(), hp + o_rs, nrev * 4);
    } else {
      d2h(x, res->status.data(), x->d_rflags.p, nrev * 4);
      d2h(x, res->reason.data(), x->d_rreason.p, nrev * 4);
    }
    if (hist) {
      std::lock_guard<std::mutex> g(e->dbg_mu);
      e->pchist.assign(ncode, 0);
      d2h(x, e->pchist.data(), x->d_pchist.p, ncode * 4);
    }
    if (prof) {
      res->prof.assign(ncons * 4, 0);
      d2h(x, res->prof.data(), x->d_prof.p, ncons * 32);
    }
    bool flagged = false;
    for (uint32_t r = 0; r < nrev && !flagged; ++r) flagged = res->status[r] & (GK_REVIEW_ERROR | GK_REVIEW_FALLBACK);
    if (!decode && !flagged && !ea_err) { res->ms[3] = ms_since(t1); mark_excluded(); return GK_OK; }
    if (audit && !ea_err) {
      // the audit sampling passes recount the totals on the device without the
      // flagged reviews (gk_sample_*): no tuple download (14M tuples = 450 MB
      // at config 4) just to recount them here
      for (auto& s : res->status) s &= (GK_REVIEW_ERROR | GK_REVIEW_FALLBACK);
      res->ms[3] = ms_since(t1);
      mark_excluded();
      return GK_OK;
    }
    std::vector<Viol> vs(counters[0]);
    std::shared_ptr<const void> rb;  // the message bytes the rows view
    const char* bp = nullptr;
    {
      // tuples into the context's pinned buffer and (decoding) message bytes
      // into a pinned block the results keep: two copies, one wait, no host
      // copy of the bytes (a large output goes through pageable copies)
      const size_t tb = counters[0] * sizeof(Viol), bb = decode ? counters[3] : 0;
      char* hq = tb <= ((size_t)64 << 20) ? x->pin(tb) : nullptr;
      char* hb = nullptr;
      if (hq && bb && bb <= ((size_t)64 << 20)) rb = pinned_block(bb, &hb);
      if (hq && (!bb || hb)) {
        bool cok = true;
        if (tb) cok = hipMemcpyAsync(hq, x->d_out.p, tb, hipMemcpyDeviceToHost, x->stream) == hipSuccess;
        if (bb && cok) cok = hipMemcpyAsync(hb, x->d_bytes.p, bb, hipMemcpyDeviceToHost, x->stream) == hipSuccess;
        if (!cok || ((tb || bb) && hipStreamSynchronize(x->stream) != hipSuccess))
          return fail(e, GK_EDEVICE, "result download failed");
        if (tb) memcpy(vs.data(), hq, tb);
        bp = hb;
      } else {
        rb.reset();
        if (tb) d2h(x, vs.data(), x->d_out.p, tb);
        if (decode) {
          auto bytes = std::make_shared<std::string>(bb, '\0');
          if (bb) d2h(x, &(*bytes)[0], x->d_bytes.p, bb);
          bp = bytes->data();
          rb = bytes;
        }
      }
    }
    res->ms[3] = ms_since(t1);
    auto t2 = Clock::now();
    // constraint errors: non-string enforcementAction fails the whole Query
    for (auto& v : vs) {
      if (e->corder[v.constraint]->ea_error) res->status[v.review] |= GK_REVIEW_ERROR;
    }
    // totals count only reviews the engine answered (flagged ones go to CPU OPA)
    std::fill(res->totals.begin(), res->totals.end(), 0);
    for (auto& v : vs)
      if (!(res->status[v.review] & (GK_REVIEW_ERROR | GK_REVIEW_FALLBACK))) res->totals[v.constraint]++;
    if (!decode) {
      for (auto& s : res->status) s &= (GK_REVIEW_ERROR | GK_REVIEW_FALLBACK);
      mark_excluded();
      res->ms[4] = ms_since(t2);
      return GK_OK;
    }
    // deterministic order: review, autoreject first, constraint order, emission
    // order -- a counting pass by review, then each review's few rows sorted
    auto within = [](const Viol& x, const Viol& y) {
      bool ax = x.rule == RULE_AUTOREJECT, ay = y.rule == RULE_AUTOREJECT;
      if (ax != ay) return ax;
      if (x.constraint != y.constraint) return x.constraint < y.constraint;
      return x.seq < y.seq;
    };
    {
      const size_t nr = res->status.size();
      bool in_range = true;
      for (auto& v : vs) in_range = in_range && v.review < nr;
      if (in_range && nr && vs.size() > 64) {
        std::vector<uint32_t> at(nr + 1, 0);
        for (auto& v : vs) at[v.review + 1]++;
        for (size_t r = 0; r < nr; ++r) at[r + 1] += at[r];
        std::vector<Viol> sorted(vs.size());
        std::vector<uint32_t> put(at.begin(), at.end() - 1);
        for (auto& v : vs) sorted[put[v.review]++] = v;
        for (size_t r = 0; r < nr; ++r)
          if (at[r + 1] - at[r] > 1) std::sort(sorted.begin() + at[r], sorted.begin() + at[r + 1], within);
        vs.swap(sorted);
      } else {
        std::sort(vs.begin(), vs.end(), [&](const Viol& x, const Viol& y) {
          if (x.review != y.review) return x.review < y.review;
          return within(x, y);
        });
      }
    }
    res->rbytes = rb;
    if (!bp) bp = "";
    res->rows.reserve(vs.size());
    for (auto& v : vs) {
      if (res->status[v.review] & (GK_REVIEW_ERROR | GK_REVIEW_FALLBACK)) continue;
      ResultRow row;
      row.review = v.review;
      row.constraint = v.constraint;
      row.seq = v.seq;
      row.rule = v.rule;
      row.msg = std::string_view(bp + v.msg_off, v.msg_len);
      row.details = std::string_view(bp + v.msg_off + v.msg_len, v.det_len);
      res->rows.push_back(row);
    }
    for (auto& s : res->status) s &= (GK_REVIEW_ERROR | GK_REVIEW_FALLBACK);
    mark_excluded();
    res->ms[4] = ms_since(t2);
    return GK_OK;
  }
  return fail(e, GK_EDEVICE, "output buffer overflow");
}

// ------------------------------------------------------------------ C ABI
extern "C" {

int gk_device_available(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}

int gk_engine_create(const char* opts_json, gk_engine** out) {
  if (!out) return GK_EINVAL;
  if (gk_devargs_size() != sizeof(DevArgs)) return GK_EINVAL;
  auto* e = new gk_engine();
  if (opts_json && *opts_json) {
    JDoc d;
    JsonReader rd(opts_json, strlen(opts_json), &d);
    int r = rd.parse();
    if (r >= 0) {
      int dv = d.get(r, "device");
      if (dv >= 0 && d.nodes[dv].type == NT_NUM) e->device = atoi(d.str(d.nodes[dv]));
      int jv = d.get(r, "jit");
      if (jv >= 0 && d.nodes[jv].type == NT_FALSE) e->jit_enabled = false;
      int hv = d.get(r, "host_only");
      if (hv >= 0 && d.nodes[hv].type == NT_TRUE) e->host_only = true;
      int cv = d.get(r, "coalesce_us");
      if (cv >= 0 && d.nodes[cv].type == NT_NUM) e->co.window_us = (uint32_t)std::min(1000000ll, std::max(0ll, atoll(d.str(d.nodes[cv]))));
      int cm = d.get(r, "coalesce_max");
      if (cm >= 0 && d.nodes[cm].type == NT_NUM) e->co.max_batch = (uint32_t)std::min(65536ll, std::max(1ll, atoll(d.str(d.nodes[cm]))));
      int mv = d.get(r, "max_violations");
      if (mv >= 0 && d.nodes[mv].type == NT_NUM) e->out_cap0 = std::max<size_t>(64, (size_t)atoll(d.str(d.nodes[mv])));
    }
  }
  {
    const char* pe = getenv("GKGPU_PROFILE");
    e->profile = pe ? atoi(pe) : 0;
    const char* je = getenv("GKGPU_JIT");
    if (je && *je == '0') e->jit_enabled = false;
  }
  e->perm_nodes = (uint32_t)e->st.nodes().size();
  e->base_nodes = e->perm_nodes;
  e->d_strs.graveyard = e->d_pool.graveyard = e->d_sflags.graveyard = e->d_nums.graveyard = &e->graveyard;
  *out = e;
  return GK_OK;
}

void gk_engine_destroy(gk_engine* e) {
  if (!e) return;
  e->cache_batch.reset();
  for (auto& x : e->ctxs) x->release_all();
  for (DBuf* b : {&e->d_nodes, &e->d_strs, &e->d_pool, &e->d_sflags, &e->d_nums, &e->d_code, &e->d_K, &e->d_fmt,
                  &e->d_fmtr, &e->d_fmtb, &e->d_cons, &e->d_mwords, &e->d_progoff, &e->d_dfa_keys, &e->d_dfa_meta, &e->d_dfa_words,
                  &e->d_stage, &e->d_dfa_c})
    b->free_();
  for (void* p : e->graveyard) hipFree(p);
  for (auto& j : e->jits) if (j.mod) hipModuleUnload(j.mod);
  delete e;
}

const char* gk_last_error(gk_engine* e) { return e ? tl_err.c_str() : "null engine"; }

int gk_init(gk_engine* e) {
  if (!e) return GK_EINVAL;
  return GK_OK;
}

int gk_put_module(gk_engine* e, const char* name, const char* src, size_t len) {
  if (!e || !name || !src) return GK_EINVAL;
  WriteLock g(e);
  std::string s(src, len);
  try {
    rego::parse_module(s);
  } catch (const std::exception& ex) {
    return fail(e, GK_EPARSE, ex.what());
  }
  e->modules[name] = s;
  e->modules_dirty = true;
  e->gen++;
  return GK_OK;
}

static int delete_modules_locked(gk_engine* e, const std::string& prefix) {
  std::string p = "__modset_" + prefix + "_idx_";
  int n = 0;
  for (auto it = e->modules.begin(); it != e->modules.end();) {
    if (it->first.compare(0, p.size(), p) == 0) { it = e->modules.erase(it); ++n; }
    else ++it;
  }
  if (n) { e->modules_dirty = true; e->gen++; }
  return n;
}

int gk_put_modules(gk_engine* e, const char* prefix, const char* const* srcs, const size_t* lens, size_t n) {
  if (!e || !prefix) return GK_EINVAL;
  WriteLock g(e);
  std::vector<std::string> ss;
  for (size_t i = 0; i < n; ++i) {
    std::string s(srcs[i], lens ? lens[i] : strlen(srcs[i]));
    try {
      rego::parse_module(s);
    } catch (const std::exception& ex) {
      return fail(e, GK_EPARSE, ex.what());
    }
    ss.push_back(s);
  }
  delete_modules_locked(e, prefix);
  for (size_t i = 0; i < ss.size(); ++i)
    e->modules["__modset_" + std::string(prefix) + "_idx_" + std::to_string(i)] = ss[i];
  e->modules_dirty = true;
  e->gen++;
  return GK_OK;
}

int gk_delete_module(gk_engine* e, const char* name, int* deleted) {
  if (!e || !name) return GK_EINVAL;
  WriteLock g(e);
  int d = (int)e->modules.erase(name);
  if (d) { e->modules_dirty = true; e->gen++; }
  if (deleted) *deleted = d;
  return GK_OK;
}

int gk_delete_modules(gk_engine* e, const char* prefix, int* count) {
  if (!e || !prefix) return GK_EINVAL;
  WriteLock g(e);
  int n = delete_modules_locked(e, prefix);
  if (count) *count = n;
  return GK_OK;
}

int gk_put_data(gk_engine* e, const char* path, const char* json, size_t len) {
  if (!e || !path || !json) return GK_EINVAL;
  WriteLock g(e);
  auto p = split_path(path);
  JDoc d;
  JsonReader rd(json, len, &d);
  int root = rd.parse();
  if (root < 0) return fail(e, GK_EINVAL, "invalid JSON: " + d.err);
  e->gen++;
  if (p.size() == 6 && p[0] == "constraints" && p[1] == TARGET && p[2] == "cluster" && p[3] == CGROUP) {
    rebuild_modules(e);
    reset_transient(e);
    ConstraintEnt c;
    c.kind = p[4];
    c.name = p[5];
    c.json.assign(json, len);
    const size_t n0 = e->st.nodes().size();
    c.root = e->st.add_doc(d, root);
    c.nnodes = (uint32_t)(e->st.nodes().size() - n0);
    e->perm_nodes = (uint32_t)e->st.nodes().size();
    e->constraints[{c.kind, c.name}] = c;
    e->constraints_dirty = true;
    return GK_OK;
  }
  if (p.size() >= 2 && p[0] == "external" && p[1] == TARGET) {
    std::string key(path);
    e->inventory[key] = std::string(json, len);
    e->inv_dirty = true;
    if (p.size() == 6 && p[2] == "cluster" && p[3] == "v1" && p[4] == "Namespace") {
      rebuild_modules(e);
      reset_transient(e);
      const size_t n0 = e->st.nodes().size();
      const uint32_t node = e->st.add_doc(d, root);
      e->ns_cache[p[5]] = node;
      e->ns_nodes[p[5]] = {node, (uint32_t)(e->st.nodes().size() - n0)};
      e->perm_nodes = (uint32_t)e->st.nodes().size();
    }
    return GK_OK;
  }
  e->other_data[path] = std::string(json, len);
  return GK_OK;
}

int gk_delete_data(gk_engine* e, const char* path, int* deleted) {
  if (!e || !path) return GK_EINVAL;
  WriteLock g(e);
  auto p = split_path(path);
  int d = 0;
  e->gen++;
  auto prefix_match = [&](const std::vector<std::string>& q) {
    if (q.size() < p.size()) return false;
    for (size_t i = 0; i < p.size(); ++i) if (q[i] != p[i]) return false;
    return true;
  };
  for (auto it = e->constraints.begin(); it != e->constraints.end();) {
    std::vector<std::string> q{"constraints", TARGET, "cluster", CGROUP, it->first.first, it->first.second};
    if (prefix_match(q)) { it = e->constraints.erase(it); d = 1; e->constraints_dirty = true; }
    else ++it;
  }
  for (auto it = e->inventory.begin(); it != e->inventory.end();) {
    if (prefix_match(split_path(it->first))) { it = e->inventory.erase(it); d = 1; e->inv_dirty = true; }
    else ++it;
  }
  for (auto it = e->ns_cache.begin(); it != e->ns_cache.end();) {
    std::vector<std::string> q{"external", TARGET, "cluster", "v1", "Namespace", it->first};
    if (prefix_match(q)) { e->ns_nodes.erase(it->first); it = e->ns_cache.erase(it); d = 1; }
    else ++it;
  }
  for (auto it = e->other_data.begin(); it != e->other_data.end();) {
    if (prefix_match(split_path(it->first))) { it = e->other_data.erase(it); d = 1; }
    else ++it;
  }
  if (p.empty()) {
    e->constraints.clear();
    e->inventory.clear();
    e->ns_cache.clear();
    e->ns_nodes.clear();
    e->other_data.clear();
    d = 1;
    e->inv_dirty = true;
  }
  if (deleted) *deleted = d;
  return GK_OK;
}

// n independent Query(violation, input) calls (drivers/local/local.go:302-359)
// evaluated in one launch.  Shared lock: concurrent callers each flatten
// their documents into their own evaluation context and run on its stream.
static int eval_inputs(gk_engine* e, const std::vector<std::pair<const char*, size_t>>& inputs, gk_results** out) {
  ReadLock rl;
  int rc = read_lock(e, rl, true);
  if (rc != GK_OK) return rc;
  if (!e->dev_ok) return fail(e, GK_EDEVICE, "no HIP device available");
  CtxLease lease(e);
  EvalCtx* x = lease.x;
  auto res = std::make_unique<gk_results>();
  auto t0 = Clock::now();
  std::vector<ReviewCol> cols;
  std::string err;
  if (!flatten_reviews(e->st, e->smu, e->ns_cache, inputs, e->perm_nodes, x->arena, cols, err))
    return fail(e, GK_EINVAL, err);
  res->ms[0] = ms_since(t0);
  TablePtrs tp;
  if (!ctx_device(e, x) || !sync_strings(e, &tp) || !ctx_nodes(e, x, x->arena))
    return fail(e, GK_EDEVICE, "device upload failed");
  rc = launch_and_collect(e, x, tp, cols, &x->d_revs, true, res.get(), x->d_nodes.p);
  if (rc != GK_OK) return rc;
  *out = res.release();
  return GK_OK;
}

// One caller's share of a coalesced launch: its rows (review index 0), status
// and totals; the constraint table and timings of the launch.  The raw device
// output stays with the launch (not exported per caller).
static gk_results* split_results(const gk_results& all, uint32_t k) {
  auto* r = new gk_results();
  r->nrev = 1;
  r->rbytes = all.rbytes;
  r->totals.assign(all.totals.size(), 0);
  // rows are sorted by review (launch_and_collect): this caller's run
  auto lo = std::lower_bound(all.rows.begin(), all.rows.end(), k,
                             [](const ResultRow& row, uint32_t kk) { return row.review < kk; });
  for (auto it = lo; it != all.rows.end() && it->review == k; ++it) {
    r->rows.push_back(*it);
    r->rows.back().review = 0;
    if (it->constraint < r->totals.size()) ++r->totals[it->constraint];
  }
  if (!all.status.empty()) {
    r->status.push_back(all.status[k]);
    r->reason.push_back(all.reason.empty() ? 0 : all.reason[k]);
  }
  r->ckind = all.ckind;
  r->cname = all.cname;
  r->cea = all.cea;
  r->cea_error = all.cea_error;
  for (int i = 0; i < 5; ++i) r->ms[i] = all.ms[i];
  r->gen = all.gen;
  r->launches = all.launches;
  return r;
}

static int coalesced_query(gk_engine* e, const char* input, size_t len, gk_results** out) {
  Coalescer& c = e->co;
  CoalesceReq me;
  me.input = input;
  me.len = len;
  std::unique_lock<std::mutex> lk(c.mu);
  c.queue.push_back(&me);
  if (c.collecting) c.arrive.notify_one();
  while (!me.done) {
    const bool queued = std::find(c.queue.begin(), c.queue.end(), &me) != c.queue.end();
    if (!queued || c.collecting) {
      c.finished.wait(lk);
      continue;
    }
    // lead the next micro-batch: collect for the window (or until full);
    // past it, keep collecting while kMaxInflight launches are evaluating
    c.collecting = true;
    const auto t0 = Clock::now();
    const auto deadline = t0 + std::chrono::microseconds(c.window_us);
    const auto cap = t0 + std::chrono::microseconds((uint64_t)c.window_us * kWindowCap);
    for (;;) {
      if (c.queue.size() >= c.max_batch) break;
      const bool busy = c.inflight >= kMaxInflight;
      if (c.arrive.wait_until(lk, busy ? cap : deadline) == std::cv_status::timeout) {
        if (!busy || Clock::now() >= cap) break;
      } else if (!busy && Clock::now() >= deadline) {
        break;
      }
    }
    const size_t take = std::min<size_t>(c.queue.size(), c.max_batch);
    std::vector<CoalesceReq*> batch(c.queue.begin(), c.queue.begin() + take);
    c.queue.erase(c.queue.begin(), c.queue.begin() + take);
    c.collecting = false;
    ++c.inflight;
    ++c.batches;
    c.requests += batch.size();
    c.finished.notify_all();  // requests left in the queue elect the next leader
    lk.unlock();
    // A failed launch (an input that is not JSON, a device or arena failure)
    // must not fail unrelated callers: the batch is bisected and each half
    // evaluated again, so every caller gets the result an uncoalesced
    // gk_query would have given it, at O(bad * log(batch)) extra launches
    // instead of one launch per request.
    std::function<void(size_t, size_t)> serve = [&](size_t lo, size_t hi) {
      std::vector<std::pair<const char*, size_t>> in;
      in.reserve(hi - lo);
      for (size_t k = lo; k < hi; ++k) in.push_back({batch[k]->input, batch[k]->len});
      gk_results* all = nullptr;
      const int rc = eval_inputs(e, in, &all);
      std::unique_ptr<gk_results> hold(all);
      if (rc == GK_OK) {
        for (size_t k = lo; k < hi; ++k) { batch[k]->rc = GK_OK; batch[k]->out = split_results(*all, (uint32_t)(k - lo)); }
        return;
      }
      if (hi - lo == 1) {
        batch[lo]->rc = rc;
        batch[lo]->err = tl_err;
        return;
      }
      const size_t mid = lo + (hi - lo) / 2;
      serve(lo, mid);
      serve(mid, hi);
    };
    serve(0, batch.size());
    lk.lock();
    for (auto* q : batch) q->done = true;
    --c.inflight;
    c.arrive.notify_all();  // a leader waiting on the in-flight launches
    c.finished.notify_all();
  }
  lk.unlock();
  if (me.rc != GK_OK) return fail(e, me.rc, me.err);
  *out = me.out;
  return GK_OK;
}

int gk_audit_cache_stats(gk_engine* e, uint64_t* builds, uint64_t* reviews) {
  if (!e) return GK_EINVAL;
  std::lock_guard<std::mutex> g(e->cache_mu);
  if (builds) *builds = e->cache_builds;
  if (reviews) *reviews = e->cache_batch ? e->cache_batch->nrev : 0;
  return GK_OK;
}

int gk_coalesce_stats(gk_engine* e, uint64_t* batches, uint64_t* requests) {
  if (!e) return GK_EINVAL;
  std::lock_guard<std::mutex> g(e->co.mu);
  if (batches) *batches = e->co.batches;
  if (requests) *requests = e->co.requests;
  return GK_OK;
}

// hooks.audit (Client.Audit, client.go:805-833): every synced object of the
// inventory reviewed against every constraint in one query
// (target_template_source.go:46-89 matching_reviews_and_constraints).  The
// inventory is kept as a staged batch -- make_review / add_field documents in
// the path-grouped layout, device-resident -- built on the first audit after a
// change of the engine state (a mutation bumps gen) and evaluated as it is by
// every later one: repeated audits do no per-object JSON work.  Reviews are
// numbered in inventory path order (the row's review index).
// The from-cache page of the synced inventory (shared lock held): objects in
// inventory path order, each with its path's fields; paths that name no
// review (a group/version with two slashes, another depth) are skipped.
struct CachePage {
  std::vector<std::vector<std::string>> segs;
  std::vector<Page::CacheKey> keys;
  std::vector<uint64_t> offs;
  std::string objs;
  Page pg;
};
static void build_cache_page(gk_engine* e, CachePage& c) {
  std::vector<const std::string*> js;
  c.segs.reserve(e->inventory.size());
  for (auto& kv : e->inventory) {
    auto q = split_path(kv.first);
    bool ok = q.size() >= 2 && q[0] == "external" && q[1] == TARGET &&
              ((q.size() == 7 && q[2] == "namespace") || (q.size() == 6 && q[2] == "cluster"));
    if (ok) {
      // make_group_version: "g/v" -> (g, v), "v" -> ("", v); more slashes: no review
      const std::string& gv = q[q.size() - 3];
      const size_t sl = gv.find('/');
      ok = sl == std::string::npos || gv.find('/', sl + 1) == std::string::npos;
    }
    if (!ok) continue;
    c.segs.push_back(std::move(q));
    js.push_back(&kv.second);
  }
  const size_t n = c.segs.size();
  c.keys.resize(n);
  c.offs.assign(n + 1, 0);
  for (size_t i = 0; i < n; ++i) c.offs[i + 1] = c.offs[i] + js[i]->size();
  c.objs.assign(c.offs[n], '\0');
  const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)default_threads(), n / 4096));
  parallel_run(T, [&](int t) {
    for (size_t i = n * t / T; i < n * (t + 1) / T; ++i) {
      if (!js[i]->empty()) memcpy(&c.objs[c.offs[i]], js[i]->data(), js[i]->size());
      const auto& q = c.segs[i];
      const bool nsd = q.size() == 7;
      const std::string& gv = q[q.size() - 3];
      const size_t sl = gv.find('/');
      Page::CacheKey& k = c.keys[i];
      k.namespaced = nsd;
      k.ns = nsd ? std::string_view(q[3]) : std::string_view();
      k.group = sl == std::string::npos ? std::string_view() : std::string_view(gv).substr(0, sl);
      k.version = sl == std::string::npos ? std::string_view(gv) : std::string_view(gv).substr(sl + 1);
      k.kind = q[q.size() - 2];
      k.name = q[q.size() - 1];
    }
  });
  c.pg = Page{c.objs.data(), c.offs.data(), n, nullptr, nullptr, 0, nullptr};
  c.pg.cache = c.keys.data();
}

static int stage_page_locked(gk_engine* e, const Page& page, gk_batch** out);
// the staged batch of the current engine state's inventory (built on first
// use after a mutation; shared lock held by the caller)
static int cache_batch_locked(gk_engine* e, std::shared_ptr<gk_batch>* out) {
  std::lock_guard<std::mutex> g(e->cache_mu);
  if (!e->cache_batch || e->cache_batch->gen != e->gen) {
    e->cache_batch.reset();
    CachePage cp;
    build_cache_page(e, cp);
    gk_batch* nb = nullptr;
    const int rc = stage_page_locked(e, cp.pg, &nb);
    if (rc != GK_OK) return rc;
    e->cache_batch = std::shared_ptr<gk_batch>(nb, gk_batch_free);
    ++e->cache_builds;
  }
  *out = e->cache_batch;
  return GK_OK;
}
static int audit_from_cache(gk_engine* e, gk_results** out) {
  ReadLock rl;
  int rc = read_lock(e, rl, !e->host_only);
  if (rc != GK_OK) return rc;
  std::shared_ptr<gk_batch> b;
  rc = cache_batch_locked(e, &b);
  if (rc != GK_OK) return rc;
  if (!e->dev_ok || !b->d_nodes.p) return fail(e, GK_EDEVICE, "no HIP device available");
  CtxLease lease(e);
  TablePtrs tp;
  if (!ctx_device(e, lease.x) || !sync_strings(e, &tp)) return fail(e, GK_EDEVICE, "device upload failed");
  auto res = std::make_unique<gk_results>();
  rc = launch_and_collect(e, lease.x, tp, b->cols, &b->d_revs, true, res.get(), b->d_nodes.p, 0, b->node_begin, false,
                          b.get());
  if (rc != GK_OK) return rc;
  *out = res.release();
  return GK_OK;
}

int gk_query(gk_engine* e, const char* path, const char* input_json, size_t len, gk_results** out) {
  if (!e || !path || !out) return GK_EINVAL;
  std::string p(path);
  std::string viol = std::string("hooks[\"") + TARGET + "\"].violation";
  std::string aud = std::string("hooks[\"") + TARGET + "\"].audit";
  if (p == viol) {
    if (e->co.window_us) return coalesced_query(e, input_json ? input_json : "null", input_json ? len : 4, out);
    std::vector<std::pair<const char*, size_t>> in;
    in.push_back({input_json ? input_json : "null", input_json ? len : 4});
    return eval_inputs(e, in, out);
  }
  if (p == aud) return audit_from_cache(e, out);
  return fail(e, GK_EQUERY, "unsupported query path: " + p);
}

int gk_query_batch(gk_engine* e, const char* const* inputs, const size_t* lens, size_t n, gk_results** out) {
  if (!e || !out) return GK_EINVAL;
  std::vector<std::pair<const char*, size_t>> in;
  for (size_t i = 0; i < n; ++i) in.push_back({inputs[i], lens ? lens[i] : strlen(inputs[i])});
  return eval_inputs(e, in, out);
}

// Divergence- and match-aware evaluation order of a page's reviews
// (perm[k] = batch index of the k-th evaluated review).
// Divergence-aware order: a wavefront evaluates 64 consecutive reviews, and
// its lanes run as long as the largest document (e.g. the Pod with the most
// containers).  Evaluating reviews in order of document size (node count)
// puts similar documents in one wave; each column records the review's
// index in the caller's batch, which every output carries (devrt.h
// audit_body), so results are unchanged.
//
// Ahead of size, two match-affinity keys keep reviews that a constraint's
// match stage rejects together, so those wavefronts exit after the match
// instead of idling beside a few matching lanes: one bit per constraint
// with a namespaces / excludedNamespaces list (membership of the review's
// namespace), then the kind id.  Keys only reorder work; matching itself is
// unchanged.
// GKGPU_MATCH_ORDER (A/B switch): 0 = size keys only, 1 = signature first,
// 2 (default) = kind, array elements, signature, nodes
static void review_order(gk_engine* e, const std::vector<ReviewCol>& cols, const std::vector<uint32_t>& weight,
                         size_t lo, size_t hi, std::vector<uint32_t>& perm) {
  const size_t n = hi - lo;
  const int mode = env_mode("GKGPU_MATCH_ORDER", 2, 2);
  const bool match_order = mode != 0;
  std::vector<uint32_t> sig(n, 0);  // indexed by batch index - lo
  if (match_order && !e->constraints_dirty) {
    const auto& W = e->mwords;
    auto in_list = [&](uint32_t off, uint32_t id) {
      if (off >= W.size()) return false;
      uint32_t n = W[off];
      for (uint32_t j = 0; j < n && off + 1 + j < W.size(); ++j) if (W[off + 1 + j] == id) return true;
      return false;
    };
    // one signature per distinct namespace-name id (reviews share a few
    // thousand namespaces), then a lookup per review
    std::unordered_map<uint32_t, uint32_t> by_ns;
    for (size_t i = lo; i < hi; ++i) {
      uint32_t id = cols[i].nsname;
      auto it = by_ns.find(id);
      if (it == by_ns.end()) {
        uint32_t s = 0, bit = 0;
        for (auto* c : e->corder) {
          if (bit >= 16) break;
          const MatchSpec& m = c->spec;
          if (!(m.flags & (MF_HAS_NAMESPACES | MF_HAS_EXCLUDED))) continue;
          bool in = ((m.flags & MF_HAS_NAMESPACES) && in_list(m.ns_off, id)) ||
                    ((m.flags & MF_HAS_EXCLUDED) && in_list(m.exns_off, id));
          if (in) s |= 1u << bit;
          ++bit;
        }
        it = by_ns.emplace(id, s).first;
      }
      sig[i - lo] = it->second;
    }
  }
  perm.resize(n);
  for (size_t i = 0; i < n; ++i) perm[i] = (uint32_t)(lo + i);
  // the keys packed into one 60-bit integer per review (kind ids ranked, so
  // their order is kept), then a stable LSD radix sort: the same permutation
  // as the comparison sort below, which stays for more than 4096 kinds
  std::vector<uint32_t> kind_ids;
  kind_ids.reserve(64);
  {
    std::unordered_set<uint32_t> seen;
    for (size_t i = lo; i < hi; ++i)
      if (seen.insert(cols[i].kind).second) kind_ids.push_back(cols[i].kind);
    std::sort(kind_ids.begin(), kind_ids.end());
  }
  // within a kind, the largest documents first: their wavefronts run longest,
  // and launched last they would leave a tail (r03ah: ContainerLimits -0.5 %,
  // RequiredProbes -1.7 % on config 2; GKGPU_ORDER_DESC=0 is the A/B switch)
  const bool desc = env_mode("GKGPU_ORDER_DESC", 1, 1) != 0;
  if (kind_ids.size() <= 4096) {
    std::unordered_map<uint32_t, uint64_t> krank;
    for (size_t k = 0; k < kind_ids.size(); ++k) krank[kind_ids[k]] = k;
    std::vector<uint64_t> key(n);
    uint32_t last_kind = NO_ID;
    uint64_t last_rank = 0;
    for (size_t i = lo; i < hi; ++i) {
      if (cols[i].kind != last_kind) { last_kind = cols[i].kind; last_rank = krank[last_kind]; }
      const uint64_t w = desc ? (uint64_t)(0xffffffffu - weight[i]) : weight[i], sg = sig[i - lo] & 0xffffu;
      if (mode == 2) key[i - lo] = (last_rank << 48) | ((w >> 20) << 36) | (sg << 20) | (w & 0xfffffu);
      else key[i - lo] = (sg << 44) | ((match_order ? last_rank : 0) << 32) | w;
    }
    std::vector<uint32_t> tmp(perm.size());
    std::vector<uint32_t> cnt(256);
    for (int sh = 0; sh < 64; sh += 8) {
      std::fill(cnt.begin(), cnt.end(), 0);
      for (uint32_t x : perm) ++cnt[(key[x - lo] >> sh) & 0xff];
      if (*std::max_element(cnt.begin(), cnt.end()) == perm.size()) continue;  // one bucket: order kept
      uint32_t run = 0;
      for (auto& c : cnt) { uint32_t v = c; c = run; run += v; }
      for (uint32_t x : perm) tmp[cnt[(key[x - lo] >> sh) & 0xff]++] = x;
      perm.swap(tmp);
    }
  } else std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) {
    if (mode == 2) {  // kind, array elements, namespace-list bits, nodes
      if (cols[a].kind != cols[b].kind) return cols[a].kind < cols[b].kind;
      if ((weight[a] >> 20) != (weight[b] >> 20)) return (weight[a] >> 20) < (weight[b] >> 20);
      if (sig[a - lo] != sig[b - lo]) return sig[a - lo] < sig[b - lo];
      return weight[a] < weight[b];
    }
    if (sig[a - lo] != sig[b - lo]) return sig[a - lo] < sig[b - lo];
    if (match_order && cols[a].kind != cols[b].kind) return cols[a].kind < cols[b].kind;
    return weight[a] < weight[b];
  });
}

// Flattens one page of audit objects (flatten.cc, parallel host threads) and,
// for staged batches, chooses the evaluation order.  `out` receives the
// columns (in evaluation order; each carries its batch index in `orig` when
// reordered), the HandleViolation resource identity per batch index and the
// number of reviews the process excluder skipped.
static int flatten_page_into(gk_engine* e, const Page& page, bool order_by_size, NodeArena& arena,
                             std::vector<ReviewCol>& cols, std::vector<ResourceIds>* resources, uint64_t* excluded,
                             double* ms_parse = nullptr, uint32_t* paths = nullptr, DevLayout* dl = nullptr) {
  FlatResult fr;
  std::string err;
  auto exit_ = e->excluded.find("audit");
  // (Client.Audit from the cache applies no excluder: manager.go:195-197)
  const std::set<std::string>* ex = exit_ == e->excluded.end() || page.cache ? nullptr : &exit_->second;
  // GKGPU_PATH_LAYOUT (A/B switch, default on): staged batches' documents in
  // the path-grouped layout (flatten.h), ordered with the reviews
  const bool path_layout = order_by_size && env_mode("GKGPU_PATH_LAYOUT", 1, 1) != 0;
  std::vector<uint32_t> perm;
  const OrderFn ord = [&](const FlatResult& f, size_t lo, size_t hi, std::vector<uint32_t>& p) {
    review_order(e, f.cols, f.weight, lo, hi, p);
  };
  if (!flatten_page(e->st, e->smu, e->ns_cache, ex, page, default_threads(), e->perm_nodes, arena, fr, err,
                    path_layout ? &ord : nullptr, path_layout ? &perm : nullptr, path_layout ? dl : nullptr))
    return fail(e, GK_EINVAL, err);
  if (dl && !path_layout) dl->nroots = NO_ID;  // no device layout: the host arena is uploaded as it is
  if (ms_parse) *ms_parse = fr.ms_parse;
  if (paths) *paths = fr.paths;
  if (resources) resources->swap(fr.resources);
  if (excluded) *excluded = fr.excluded;
  cols.swap(fr.cols);
  const bool trace = getenv("GKGPU_FLATTEN_TRACE") != nullptr;
  auto t_ord = Clock::now();
  if (order_by_size) {
    if (!path_layout) review_order(e, cols, fr.weight, 0, cols.size(), perm);
    std::vector<ReviewCol> sorted(cols.size());
    const size_t n = perm.size();
    const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)default_threads(), n / 65536));
    parallel_run(T, [&](int t) {
      for (size_t i = n * t / T; i < n * (t + 1) / T; ++i) { sorted[i] = cols[perm[i]]; sorted[i].orig = perm[i]; }
    });
    cols.swap(sorted);
    if (trace) fprintf(stderr, "flatten: review order %.1f ms\n", ms_since(t_ord));
  }
  return GK_OK;
}

// The char** form of a page: namespaces given per object are de-duplicated by
// text into the page's namespace table (the audit loop's nsCache).
struct PageBuf {
  Page page;
  std::vector<uint64_t> obj_offs, ns_offs;
  std::string objs, nss;
  std::vector<uint32_t> obj_ns;
};

static void page_from_arrays(const char* const* objs, const size_t* obj_lens, const char* const* ns_json,
                             const size_t* ns_lens, size_t n, PageBuf& pb) {
  pb.obj_offs.resize(n + 1);
  size_t tot = 0;
  for (size_t i = 0; i < n; ++i) tot += obj_lens ? obj_lens[i] : strlen(objs[i]);
  pb.objs.resize(tot);
  uint64_t off = 0;
  std::unordered_map<std::string_view, uint32_t> ns_idx;
  pb.obj_ns.assign(n, NO_ID);
  std::vector<std::string_view> ns_list;
  for (size_t i = 0; i < n; ++i) {
    size_t l = obj_lens ? obj_lens[i] : strlen(objs[i]);
    pb.obj_offs[i] = off;
    if (l) memcpy(&pb.objs[off], objs[i], l);
    off += l;
    const char* ns = (ns_json && ns_json[i]) ? ns_json[i] : nullptr;
    size_t nl = ns ? (ns_lens ? ns_lens[i] : strlen(ns)) : 0;
    if (!ns || nl == 0) continue;
    std::string_view key(ns, nl);
    auto it = ns_idx.find(key);
    if (it == ns_idx.end()) {
      it = ns_idx.emplace(key, (uint32_t)ns_list.size()).first;
      ns_list.push_back(key);
    }
    pb.obj_ns[i] = it->second;
  }
  pb.obj_offs[n] = off;
  pb.ns_offs.resize(ns_list.size() + 1);
  uint64_t no = 0;
  for (size_t k = 0; k < ns_list.size(); ++k) { pb.ns_offs[k] = no; no += ns_list[k].size(); }
  pb.ns_offs[ns_list.size()] = no;
  pb.nss.resize(no);
  for (size_t k = 0; k < ns_list.size(); ++k)
    if (!ns_list[k].empty()) memcpy(&pb.nss[pb.ns_offs[k]], ns_list[k].data(), ns_list[k].size());
  pb.page.objs = pb.objs.data();
  pb.page.obj_offs = pb.obj_offs.data();
  pb.page.n = n;
  pb.page.nss = pb.nss.data();
  pb.page.ns_offs = pb.ns_offs.data();
  pb.page.n_ns = ns_list.size();
  pb.page.obj_ns = pb.obj_ns.data();
}

static int review_page(gk_engine* e, const Page& page, gk_results** out) {
  ReadLock rl;
  int rc = read_lock(e, rl, true);
  if (rc != GK_OK) return rc;
  if (!e->dev_ok) return fail(e, GK_EDEVICE, "no HIP device available");
  CtxLease lease(e);
  EvalCtx* x = lease.x;
  auto res = std::make_unique<gk_results>();
  auto t0 = Clock::now();
  std::vector<ReviewCol> cols;
  uint64_t excluded = 0;
  rc = flatten_page_into(e, page, false, x->arena, cols, nullptr, &excluded);
  if (rc != GK_OK) return rc;
  res->ms[0] = ms_since(t0);
  TablePtrs tp;
  if (!ctx_device(e, x) || !sync_strings(e, &tp) || !ctx_nodes(e, x, x->arena))
    return fail(e, GK_EDEVICE, "device upload failed");
  rc = launch_and_collect(e, x, tp, cols, &x->d_revs, true, res.get(), x->d_nodes.p, excluded);
  if (rc != GK_OK) return rc;
  *out = res.release();
  return GK_OK;
}

int gk_review_objects(gk_engine* e, const char* const* objs, const size_t* obj_lens, const char* const* ns_json,
                      const size_t* ns_lens, size_t n, gk_results** out) {
  if (!e || !out || (n && !objs)) return GK_EINVAL;
  PageBuf pb;
  page_from_arrays(objs, obj_lens, ns_json, ns_lens, n, pb);
  return review_page(e, pb.page, out);
}

int gk_review_page(gk_engine* e, const char* objs, const uint64_t* obj_offs, size_t n, const char* nss,
                   const uint64_t* ns_offs, size_t n_ns, const uint32_t* obj_ns, gk_results** out) {
  if (!e || !out || (n && (!objs || !obj_offs)) || (n_ns && (!nss || !ns_offs))) return GK_EINVAL;
  Page pg{objs, obj_offs, n, nss, ns_offs, n_ns, obj_ns};
  return review_page(e, pg, out);
}

// A staged batch's device node array: the engine's permanent region (copied on
// the device) followed by the batch's documents (large ones through the
// pinned bounce buffers, engine.cc upload_bounce).
static bool batch_upload(gk_engine* e, gk_batch* b) {
  const size_t perm = b->node_begin, docs = b->arena.size();
  if (!b->d_nodes.reserve((perm + docs + 1) * sizeof(Node))) return false;
  if (perm && (hipMemcpy(b->d_nodes.p, e->d_nodes.p, perm * sizeof(Node), hipMemcpyDeviceToDevice) != hipSuccess ||
               hipStreamSynchronize(nullptr) != hipSuccess))  // (see DBuf::reserve)
    return false;
  const size_t bytes = docs * sizeof(Node);
  char* dst = (char*)b->d_nodes.p + perm * sizeof(Node);
  const char* bm = getenv("GKGPU_BOUNCE_MIN");  // tests: the smallest copy that takes the bounce path
  const size_t bounce_min = bm ? (size_t)atoll(bm) : (16u << 20);
  if (bytes >= bounce_min) {
    if (!upload_bounce(dst, (const char*)b->arena.data(), bytes)) return false;
  } else if (bytes && hipMemcpy(dst, b->arena.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
    return false;
  }
  b->d_nodes.used = (perm + docs) * sizeof(Node);
  return true;
}

extern "C" int gk_device_layout(const Node* D, uint64_t nD, uint32_t base, const uint32_t* beg, const uint32_t* evalpos,
                                const uint32_t* root_d, const uint32_t* slot, uint32_t nrev, uint32_t nroots, Node* N,
                                ReviewCol* cols, uint32_t ncols, uint64_t* n_out, hipStream_t s);

// batch_upload for the device layout: the permanent region as batch_upload
// does, the per-document arena D into a scratch buffer, then layout.hip
// permutes it into the batch's node array and rewrites the uploaded review
// columns' node ids.  The host arena keeps D (the CPU checker reads it).
static bool batch_upload_layout(gk_engine* e, gk_batch* b, const DevLayout& dl) {
  const size_t perm = b->node_begin, docs = b->arena.size();
  const uint32_t nrev = (uint32_t)dl.beg.size();
  if (!docs || !nrev || b->cols.size() != nrev || dl.evalpos.size() != nrev || dl.root_d.size() != nrev ||
      dl.slot.size() != nrev)
    return batch_upload(e, b);
  const auto t0 = Clock::now();
  if (!b->d_nodes.reserve((perm + docs + 1) * sizeof(Node))) return false;
  if (perm && (hipMemcpy(b->d_nodes.p, e->d_nodes.p, perm * sizeof(Node), hipMemcpyDeviceToDevice) != hipSuccess ||
               hipStreamSynchronize(nullptr) != hipSuccess))
    return false;
  const double ms_nodes = ms_since(t0);
  DBuf dD, dbeg, deval, droot, dslot;
  bool ok = dD.reserve(docs * sizeof(Node)) && dbeg.reserve(nrev * 4) && deval.reserve(nrev * 4) &&
            droot.reserve(nrev * 4) && dslot.reserve(nrev * 4);
  const double ms_scratch = ms_since(t0);
  const size_t bytes = docs * sizeof(Node);
  const char* bm = getenv("GKGPU_BOUNCE_MIN");
  const size_t bounce_min = bm ? (size_t)atoll(bm) : (16u << 20);
  if (ok) ok = bytes >= bounce_min ? upload_bounce(dD.p, (const char*)b->arena.data(), bytes)
                                   : hipMemcpy(dD.p, b->arena.data(), bytes, hipMemcpyHostToDevice) == hipSuccess;
  const double ms_up = ms_since(t0);
  ok = ok && hipMemcpy(dbeg.p, dl.beg.data(), nrev * 4, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(deval.p, dl.evalpos.data(), nrev * 4, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(droot.p, dl.root_d.data(), nrev * 4, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(dslot.p, dl.slot.data(), nrev * 4, hipMemcpyHostToDevice) == hipSuccess;
  const double ms_small = ms_since(t0);
  hipStream_t st = nullptr;
  uint64_t nout = 0;
  if (ok) ok = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
  if (ok)
    ok = gk_device_layout((const Node*)dD.p, docs, b->node_begin, (const uint32_t*)dbeg.p, (const uint32_t*)deval.p,
                          (const uint32_t*)droot.p, (const uint32_t*)dslot.p, nrev, dl.nroots,
                          (Node*)b->d_nodes.p + perm, (ReviewCol*)b->d_revs.p, nrev, &nout, st) == 0;
  if (st) hipStreamDestroy(st);
  const double ms_layout = ms_since(t0);
  for (DBuf* x : {&dD, &dbeg, &deval, &droot, &dslot}) x->free_();
  if (getenv("GKGPU_FLATTEN_TRACE"))
    fprintf(stderr, "upload layout: node buffer %.1f ms, scratch %.1f ms, upload %.1f ms, tables %.1f ms, layout %.1f ms, free %.1f ms\n",
            ms_nodes, ms_scratch - ms_nodes, ms_up - ms_scratch, ms_small - ms_up, ms_layout - ms_small, ms_since(t0) - ms_layout);
  if (!ok) return false;
  b->d_nodes.used = (perm + docs) * sizeof(Node);
  b->device_layout = true;
  return true;
}

// The merged referenced-path plan of the programs the constraints run
// (colplan.h), cached per engine generation.  Shared lock held.
static gk::PathPlan batch_plan(gk_engine* e) {
  std::lock_guard<std::mutex> g(e->plan_mu);
  if (e->plan_gen != e->gen) {
    gk::PathPlan P;
    P.nodes.emplace_back();
    std::set<uint32_t> progs;
    for (auto* c : e->corder)
      if (c->spec.prog != NO_ID && c->spec.prog < e->progs.size()) progs.insert(c->spec.prog);
    for (uint32_t p : progs) P.merge(gk::plan_paths(e->progs[p], e->bank));
    e->plan = std::move(P);
    e->plan_gen = e->gen;
  }
  return e->plan;
}

// GKGPU_COLUMNS (A/B switch, default on): staged batches in column form (colstore.h)
static bool columns_on() { return env_mode("GKGPU_COLUMNS", 1, 1) != 0; }

// The column form's device arrays: the permanent region and the kept
// subtrees as the batch's node array, the review columns, the path columns.
static bool batch_upload_columns(gk_engine* e, gk_batch* b) {
  const auto t0 = Clock::now();
  const ColStore& cv = b->cv;
  const size_t perm = b->node_begin, kept = cv.nodes.size();
  if (!b->d_nodes.reserve((perm + kept + 1) * sizeof(Node))) return false;
  if (perm && (hipMemcpy(b->d_nodes.p, e->d_nodes.p, perm * sizeof(Node), hipMemcpyDeviceToDevice) != hipSuccess ||
               hipStreamSynchronize(nullptr) != hipSuccess))  // (see DBuf::reserve)
    return false;
  if (kept && hipMemcpy((char*)b->d_nodes.p + perm * sizeof(Node), cv.nodes.data(), kept * sizeof(Node),
                        hipMemcpyHostToDevice) != hipSuccess)
    return false;
  b->d_nodes.used = (perm + kept) * sizeof(Node);
  const double ms_nodes = ms_since(t0);
  bool ok = b->d_revs.upload(cv.cols.data(), cv.cols.size() * sizeof(ReviewCol), false);
  const double ms_cols = ms_since(t0);
  ok = ok && b->d_cv_words.upload(cv.words.data(), cv.words.size() * 4, false) &&
       b->d_cv_bytes.upload(cv.bytes.data(), cv.bytes.size(), false);
  const double ms_words = ms_since(t0);
  ok = ok && up(b->d_cv_slots, cv.slots, false) && up(b->d_cv_hash, cv.hash, false) && up(b->d_cv_views, cv.views, false) &&
       up(b->d_cv_tabs, cv.tabs, false);
  if (getenv("GKGPU_FLATTEN_TRACE"))
    fprintf(stderr, "upload columns: nodes %.1f ms, review columns %.1f ms, path columns %.1f ms, tables %.1f ms\n", ms_nodes,
            ms_cols - ms_nodes, ms_words - ms_cols, ms_since(t0) - ms_words);
  return ok;
}

static int stage_page(gk_engine* e, const Page& page, gk_batch** out) {
  ReadLock rl;
  int rc = read_lock(e, rl, !e->host_only);
  if (rc != GK_OK) return rc;
  return stage_page_locked(e, page, out);
}

// stage_page under the caller's shared lock
static int stage_page_locked(gk_engine* e, const Page& page, gk_batch** out) {
  int rc = GK_OK;
  auto t0 = Clock::now();
  auto b = std::make_unique<gk_batch>();
  b->eng = e;
  b->node_begin = e->perm_nodes;
  const bool size_order = env_mode("GKGPU_SIZE_ORDER", 1, 1) != 0;  // A/B switch (default on)
  // GKGPU_DEVICE_LAYOUT (A/B switch, default on): the path-grouped layout is
  // built on the device (layout.hip) from the per-document arena
  DevLayout dl;
  // (the column form starts from the per-document arena too: no placement)
  const bool dev_layout =
      (columns_on() || (!e->host_only && e->dev_ok)) && env_mode("GKGPU_DEVICE_LAYOUT", 1, 1) != 0;
  rc = flatten_page_into(e, page, size_order, b->arena, b->cols, &b->resources, &b->excluded, &b->ms_parse, nullptr,
                         dev_layout ? &dl : nullptr);
  if (rc != GK_OK) return rc;
  b->ms_flatten = ms_since(t0);
  b->node_end = b->node_begin + (uint32_t)b->arena.size();
  b->nrev = (uint32_t)page.n;
  b->gen = e->gen;
  b->node_count = b->node_end - b->node_begin;
  auto t1 = Clock::now();
  if (columns_on()) {
    const gk::PathPlan plan = batch_plan(e);
    b->columnar = gk::build_columns(plan, e->st.nodes().data(), b->node_begin, b->arena.data(), b->arena.size(), b->cols,
                                    e->st, e->smu, b->cv, b->col_why);
    if (getenv("GKGPU_FLATTEN_TRACE"))
      fprintf(stderr, "columns: %s %.1f ms, %llu bytes%s%s\n", b->columnar ? "built" : "not used", ms_since(t1),
              (unsigned long long)b->cv.total_bytes(), b->columnar ? "" : ": ", b->col_why.c_str());
  }
  b->ms_flatten = ms_since(t0);  // (the column build included)
  t1 = Clock::now();              // the upload phase starts here
  if (e->host_only) {  // documents stay in the host arena only (gk_debug_host_args)
    *out = b.release();
    return GK_OK;
  }
  if (!e->dev_ok) return fail(e, GK_EDEVICE, "no HIP device available");
  const bool trace = getenv("GKGPU_FLATTEN_TRACE") != nullptr;
  bool up_ok = sync_strings(e, nullptr);
  const double ms_tables = ms_since(t1);
  double ms_cols = ms_tables;
  if (b->columnar) {
    up_ok = up_ok && batch_upload_columns(e, b.get());
  } else {
    up_ok = up_ok && up(b->d_revs, b->cols, false);
    ms_cols = ms_since(t1);
    if (dev_layout && dl.nroots != NO_ID) up_ok = up_ok && batch_upload_layout(e, b.get(), dl);
    else up_ok = up_ok && batch_upload(e, b.get());
  }
  if (trace)
    fprintf(stderr, "stage upload: strings %.1f ms, columns %.1f ms, nodes %.1f ms\n", ms_tables, ms_cols - ms_tables,
            ms_since(t1) - ms_cols);
  if (!up_ok) {
    b->d_revs.free_();
    b->d_nodes.free_();
    return fail(e, GK_EDEVICE, "upload failed");
  }
  b->ms_upload = ms_since(t1);
  b->dev_bytes = b->columnar ? b->cv.total_bytes()
                             : (uint64_t)(b->node_end - b->node_begin) * sizeof(Node) + b->cols.size() * sizeof(ReviewCol);
  release_parts_async();
  *out = b.release();
  return GK_OK;
}

int gk_batch_stage_objects(gk_engine* e, const char* const* objs, const size_t* obj_lens, const char* const* ns_json,
                           const size_t* ns_lens, size_t n, gk_batch** out) {
  if (!e || !out || (n && !objs)) return GK_EINVAL;
  PageBuf pb;
  page_from_arrays(objs, obj_lens, ns_json, ns_lens, n, pb);
  return stage_page(e, pb.page, out);
}

int gk_batch_stage_page(gk_engine* e, const char* objs, const uint64_t* obj_offs, size_t n, const char* nss,
                        const uint64_t* ns_offs, size_t n_ns, const uint32_t* obj_ns, gk_batch** out) {
  if (!e || !out || (n && (!objs || !obj_offs)) || (n_ns && (!nss || !ns_offs))) return GK_EINVAL;
  Page pg{objs, obj_offs, n, nss, ns_offs, n_ns, obj_ns};
  return stage_page(e, pg, out);
}

int gk_batch_timing(const gk_batch* b, double* ms3) {
  if (!b || !ms3) return GK_EINVAL;
  ms3[0] = b->ms_parse;
  ms3[1] = b->ms_flatten;
  ms3[2] = b->ms_upload;
  return GK_OK;
}

uint64_t gk_batch_excluded(const gk_batch* b) { return b ? b->excluded : 0; }

int gk_batch_resource(gk_engine* e, const gk_batch* b, size_t review, gk_resource* out) {
  if (!e || !b || !out || review >= b->resources.size()) return GK_EINVAL;
  std::lock_guard<std::mutex> g(e->smu);  // string table (appended to by concurrent evaluations)
  const ResourceIds& r = b->resources[review];
  auto put = [&](char* dst, uint32_t sid) {
    std::string_view v = e->st.str(sid);
    size_t n = std::min<size_t>(v.size(), GK_RESOURCE_FIELD - 1);
    memcpy(dst, v.data(), n);
    dst[n] = 0;
    return v.size() < GK_RESOURCE_FIELD;
  };
  int cut = !put(out->api_version, r.api_version);
  cut += !put(out->kind, r.kind);
  cut += !put(out->name, r.name);
  cut += !put(out->namespace_, r.ns);
  bool ok = cut == 0;
  return ok ? GK_OK : GK_ERANGE;
}

int gk_batch_eval(gk_engine* e, gk_batch* b, int decode, gk_results** out) {
  if (!e || !b || !out) return GK_EINVAL;
  ReadLock rl;
  int rc = read_lock(e, rl, true);
  if (rc != GK_OK) return rc;
  if (b->gen != e->gen) return fail(e, GK_EINVAL, "engine state changed since the batch was staged");
  if (!e->dev_ok || !b->d_nodes.p) return fail(e, GK_EDEVICE, "no HIP device available");
  CtxLease lease(e);
  TablePtrs tp;
  if (!ctx_device(e, lease.x) || !sync_strings(e, &tp)) return fail(e, GK_EDEVICE, "device upload failed");
  auto res = std::make_unique<gk_results>();
  rc = launch_and_collect(e, lease.x, tp, b->cols, &b->d_revs, decode != 0, res.get(), b->d_nodes.p, b->excluded,
                          b->node_begin, false, b);
  if (rc != GK_OK) return rc;
  *out = res.release();
  return GK_OK;
}

// The audit status of one sweep over a staged batch (pkg/audit/manager.go:462-508):
// exact per-constraint totals over the reviews the engine answered, and the
// first `limit` results per constraint in evaluation order (batch index,
// autoreject first, emission order), selected on the device (kernels.hip
// gk_sample_*) so only O(constraints x limit) records reach the host.
static int batch_eval_audit_locked(gk_engine* e, gk_batch* b, uint32_t limit, gk_results** out);
int gk_batch_eval_audit(gk_engine* e, gk_batch* b, uint32_t limit, gk_results** out) {
  if (!e || !b || !out) return GK_EINVAL;
  ReadLock rl;
  int rc = read_lock(e, rl, true);
  if (rc != GK_OK) return rc;
  return batch_eval_audit_locked(e, b, limit, out);
}

int gk_audit_cache_sample(gk_engine* e, uint32_t limit, gk_results** out) {
  if (!e || !out) return GK_EINVAL;
  if (e->host_only) return fail(e, GK_EDEVICE, "host-only engine");
  ReadLock rl;
  int rc = read_lock(e, rl, true);
  if (rc != GK_OK) return rc;
  std::shared_ptr<gk_batch> b;
  rc = cache_batch_locked(e, &b);
  if (rc != GK_OK) return rc;
  return batch_eval_audit_locked(e, b.get(), limit, out);
}

static int batch_eval_audit_locked(gk_engine* e, gk_batch* b, uint32_t limit, gk_results** out) {
  int rc = GK_OK;
  if (b->gen != e->gen) return fail(e, GK_EINVAL, "engine state changed since the batch was staged");
  if (!e->dev_ok || !b->d_nodes.p) return fail(e, GK_EDEVICE, "no HIP device available");
  CtxLease lease(e);
  EvalCtx* x = lease.x;
  TablePtrs tp;
  if (!ctx_device(e, x) || !sync_strings(e, &tp)) return fail(e, GK_EDEVICE, "device upload failed");
  auto resp = std::make_unique<gk_results>();
  gk_results* res = resp.get();
  rc = launch_and_collect(e, x, tp, b->cols, &b->d_revs, false, res, b->d_nodes.p, b->excluded, b->node_begin, true, b);
  if (rc != GK_OK) return rc;
  res->audited = true;
  const uint32_t ncons = (uint32_t)e->corder.size(), nrev = b->nrev;
  if (ncons == 0 || nrev == 0) { *out = resp.release(); return GK_OK; }
  if (res->dev_tuples == 0) {
    std::fill(res->totals.begin(), res->totals.end(), 0);
    *out = resp.release();
    return GK_OK;
  }
  const uint32_t nb = gk_sample_fine(nrev);
  bool any_err = false;
  std::vector<uint8_t> cerr(ncons, 0);
  for (uint32_t c = 0; c < ncons; ++c) { cerr[c] = e->corder[c]->ea_error; any_err |= cerr[c] != 0; }
  bool ok = x->d_hist.reserve((size_t)ncons * (nb + 256) * 4) && x->d_cut.reserve(ncons * 8) && x->d_ftot.reserve(ncons * 8) &&
            x->d_ncand.reserve(16) && x->d_cand.reserve(x->cand_cap * sizeof(SampleRec)) &&
            (!any_err || up(x->d_cerr, cerr, false));
  if (!ok) return fail(e, GK_EDEVICE, "device allocation failed");
  auto t0 = Clock::now();
  hipEvent_t ev0 = x->events[0], ev1 = x->events[1];
  hipEventRecord(ev0, x->stream);
  unsigned int ncand = 0;
  // one wait per pass: the candidate count, the totals and the first K
  // candidates (K from the last audit's count) come back in one batch of
  // async copies into the context's pinned buffer
  const size_t o_tot = 16, o_cand = o_tot + (size_t)ncons * 8;
  size_t kcand = 0;
  char* hp = nullptr;
  for (int pass = 0; pass < 3; ++pass) {
    // no lane failed and no enforcementAction error: every review counts, and
    // the sampling passes skip the per-tuple review-flag reads
    uint32_t* rf = (any_err || res->failed_lanes) ? (uint32_t*)x->d_rflags.p : nullptr;
    int lr = gk_launch_sample((const Viol*)x->d_out.p, res->dev_tuples, rf, nrev,
                              any_err ? (const uint8_t*)x->d_cerr.p : nullptr, ncons, nb, std::max<uint32_t>(limit, 1),
                              (uint32_t*)x->d_hist.p, (uint32_t*)x->d_cut.p, (unsigned long long*)x->d_ftot.p,
                              (const char*)x->d_bytes.p, (SampleRec*)x->d_cand.p, (uint32_t)x->cand_cap,
                              (unsigned int*)x->d_ncand.p, pass > 0, x->stream);
    if (lr != 0) return fail(e, GK_EDEVICE, std::string("sample launch failed: ") + hipGetErrorString((hipError_t)lr));
    if (pass == 0) hipEventRecord(ev1, x->stream);
    kcand = std::min<size_t>(x->cand_cap, std::max<size_t>(2 * (size_t)x->last_ncand, 256));
    hp = x->pin(o_cand + kcand * sizeof(SampleRec));
    if (!hp) return fail(e, GK_EDEVICE, "pinned host allocation failed");
    if (hipMemcpyAsync(hp, x->d_ncand.p, 4, hipMemcpyDeviceToHost, x->stream) != hipSuccess ||
        hipMemcpyAsync(hp + o_tot, x->d_ftot.p, (size_t)ncons * 8, hipMemcpyDeviceToHost, x->stream) != hipSuccess ||
        hipMemcpyAsync(hp + o_cand, x->d_cand.p, kcand * sizeof(SampleRec), hipMemcpyDeviceToHost, x->stream) !=
            hipSuccess ||
        hipStreamSynchronize(x->stream) != hipSuccess)
      return fail(e, GK_EDEVICE, "sample pass failed");
    memcpy(&ncand, hp, 4);
    if (ncand <= x->cand_cap) break;
    x->cand_cap = std::max<size_t>(x->cand_cap * 2, (size_t)ncand + 1024);
    if (!x->d_cand.reserve(x->cand_cap * sizeof(SampleRec))) return fail(e, GK_EDEVICE, "device allocation failed");
  }
  float kms = 0;
  hipEventElapsedTime(&kms, ev0, ev1);
  res->launches.push_back({"gk_sample", (double)kms, ncons, 0, 0});
  if (ncand > x->cand_cap) return fail(e, GK_EDEVICE, "sample candidates past capacity");
  x->last_ncand = ncand;
  std::vector<uint64_t> ftot(ncons);
  std::vector<SampleRec> cand(ncand);
  memcpy(ftot.data(), hp + o_tot, (size_t)ncons * 8);
  if (ncand <= kcand) memcpy(cand.data(), hp + o_cand, (size_t)ncand * sizeof(SampleRec));
  else if (!d2h(x, cand.data(), x->d_cand.p, (size_t)ncand * sizeof(SampleRec)))  // more than the last audit's
    return fail(e, GK_EDEVICE, "sample copy failed");
  for (uint32_t c = 0; c < ncons; ++c) res->totals[c] = ftot[c];
  std::sort(cand.begin(), cand.end(), [](const SampleRec& x, const SampleRec& y) {
    if (x.constraint != y.constraint) return x.constraint < y.constraint;
    if (x.review != y.review) return x.review < y.review;
    bool ax = x.rule == RULE_AUTOREJECT, ay = y.rule == RULE_AUTOREJECT;
    if (ax != ay) return ax;
    return x.seq < y.seq;
  });
  uint32_t cur = NO_ID, taken = 0;
  for (const SampleRec& r : cand) {
    if (r.constraint != cur) { cur = r.constraint; taken = 0; }
    if (taken >= limit) continue;
    ++taken;
    gk_results::Sample sm;
    sm.review = r.review;
    sm.constraint = r.constraint;
    sm.seq = r.seq;
    sm.rule = r.rule;
    sm.msg_len = r.msg_len;
    sm.msg.assign((const char*)r.msg, std::min<uint32_t>(r.msg_len, SAMPLE_MSG));
    res->samples.push_back(std::move(sm));
  }
  res->ms[4] += ms_since(t0);
  *out = resp.release();
  return GK_OK;
}

size_t gk_results_sample_count(const gk_results* r) { return r ? r->samples.size() : 0; }

int gk_results_sample_get(const gk_results* r, size_t i, gk_sample_view* out) {
  if (!r || !out || i >= r->samples.size()) return GK_EINVAL;
  const auto& s = r->samples[i];
  out->review = s.review;
  out->constraint = s.constraint;
  out->seq = s.seq;
  out->rule = s.rule;
  out->msg_len = s.msg_len;
  out->msg = s.msg.data();
  out->msg_stored = s.msg.size();
  out->enforcement_action = r->cea[s.constraint].c_str();
  return GK_OK;
}

int gk_results_samples_export(const gk_results* r, void* buf, size_t cap, size_t* needed) {
  if (!r) return GK_EINVAL;
  size_t n = 0;
  for (const auto& smp : r->samples) n += 20 + smp.msg.size();
  if (needed) *needed = n;
  if (!buf || cap < n) return buf ? GK_EINVAL : GK_OK;
  char* p = (char*)buf;
  for (const auto& smp : r->samples) {
    const uint32_t a[2] = {smp.review, smp.constraint};
    const uint16_t b[2] = {smp.seq, smp.rule};
    const uint32_t c[2] = {smp.msg_len, (uint32_t)smp.msg.size()};
    memcpy(p, a, 8);
    memcpy(p + 8, b, 4);
    memcpy(p + 12, c, 8);
    p += 20;
    if (!smp.msg.empty()) memcpy(p, smp.msg.data(), smp.msg.size());
    p += smp.msg.size();
  }
  return GK_OK;
}

const char* gk_results_constraint_action(const gk_results* r, size_t c) {
  return r && c < r->cea.size() ? r->cea[c].c_str() : nullptr;
}

void gk_batch_free(gk_batch* b) {
  if (!b) return;
  b->d_revs.free_();
  b->d_nodes.free_();
  for (DBuf* d : {&b->d_cv_words, &b->d_cv_bytes, &b->d_cv_slots, &b->d_cv_hash, &b->d_cv_views, &b->d_cv_tabs}) d->free_();
  delete b;
}

uint64_t gk_batch_device_bytes(const gk_batch* b) { return b ? b->dev_bytes : 0; }

int gk_batch_stats(const gk_batch* cb, uint64_t* reviews, uint64_t* nodes, uint64_t* str_bytes, uint64_t* col_bytes) {
  if (!cb) return GK_EINVAL;
  gk_batch* b = const_cast<gk_batch*>(cb);
  if (str_bytes && !b->str_bytes_done && b->eng) {
    // one pass over every staged document node and each distinct string value
    // it references (computed on first request: not part of staging)
    std::lock_guard<std::mutex> g(b->eng->smu);
    const Store& st = b->eng->st;
    std::vector<uint8_t> seen(st.nstrings(), 0);
    for (const Node& nd : b->arena)
      if (nd.type == NT_STR && nd.val < seen.size() && !seen[nd.val]) { seen[nd.val] = 1; b->str_bytes += st.strings()[nd.val].len; }
    b->str_bytes_done = true;
  }
  if (reviews) *reviews = b->nrev;
  if (nodes) *nodes = b->node_count;
  if (str_bytes) *str_bytes = b->str_bytes;
  if (col_bytes) *col_bytes = (uint64_t)b->cols.size() * sizeof(ReviewCol);
  return GK_OK;
}

int gk_results_flag_counts(const gk_results* r, uint64_t* errors, uint64_t* fallbacks) {
  if (!r) return GK_EINVAL;
  uint64_t ne = 0, nf = 0;
  for (uint32_t s : r->status) { ne += (s & GK_REVIEW_ERROR) != 0; nf += (s & GK_REVIEW_FALLBACK) != 0; }  // empty: none
  if (errors) *errors = ne;
  if (fallbacks) *fallbacks = nf;
  return GK_OK;
}

int gk_results_copy_status(const gk_results* r, uint32_t* status, uint32_t* reason) {
  if (!r) return GK_EINVAL;
  if (status) {
    if (r->status.empty()) memset(status, 0, (size_t)r->nrev * 4);
    else memcpy(status, r->status.data(), r->status.size() * 4);
  }
  if (reason) {
    if (r->reason.empty()) memset(reason, 0, (size_t)r->nrev * 4);
    else memcpy(reason, r->reason.data(), r->reason.size() * 4);
  }
  return GK_OK;
}

// diagnostics (GKGPU_PROFILE=1): per constraint [sum VM steps, max lane steps,
// lanes that ran a program, sum over waves of the wave's max lane steps]
extern "C" size_t gk_results_vm_profile(const gk_results* r, uint64_t* out, size_t n) {
  if (!r) return 0;
  if (out) for (size_t i = 0; i < n && i < r->prof.size(); ++i) out[i] = r->prof[i];
  return r->prof.size();
}

size_t gk_results_launches(const gk_results* r) { return r ? r->launches.size() : 0; }

int gk_results_launch(const gk_results* r, size_t i, const char** kernel, double* ms, uint32_t* nconstraints,
                      uint64_t* tuples, uint64_t* bytes) {
  if (!r || i >= r->launches.size()) return GK_EINVAL;
  if (kernel) *kernel = r->launches[i].kernel.c_str();
  if (ms) *ms = r->launches[i].ms;
  if (nconstraints) *nconstraints = r->launches[i].nconstraints;
  if (tuples) *tuples = r->launches[i].tuples;
  if (bytes) *bytes = r->launches[i].bytes;
  return GK_OK;
}

// Staging's device-side first use, ahead of the first staging: the device
// layout's kernels (and rocPRIM's) are loaded by a two-node layout, and the
// stream-ordered pool its temporaries come from keeps freed memory instead of
// returning it after every staging.
static void device_layout_warmup() {
  static std::once_flag once;
  std::call_once(once, [] {
    hipMemPool_t pool = nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess && pool) {
      uint64_t keep = UINT64_MAX;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
    Node h[2] = {};
    h[0].type = NT_OBJ;
    h[0].n = 1;
    h[0].first = 1;
    h[0].val = 1;
    h[1].type = NT_STR;
    const uint32_t one[4] = {0, 0, 0, 0};  // beg, evalpos, root_d, slot of the one review
    ReviewCol hc{};
    hc.root = 0;
    hc.labels = hc.old_labels = hc.ns_labels = NO_ID;
    DBuf dD, dN, dv, dc;
    hipStream_t st = nullptr;
    uint64_t nout = 0;
    if (dD.reserve(sizeof h) && dN.reserve(sizeof h) && dv.reserve(sizeof one) && dc.reserve(sizeof hc) &&
        hipMemcpy(dD.p, h, sizeof h, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(dv.p, one, sizeof one, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(dc.p, &hc, sizeof hc, hipMemcpyHostToDevice) == hipSuccess &&
        hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess) {
      const uint32_t* v = (const uint32_t*)dv.p;
      (void)gk_device_layout((const Node*)dD.p, 2, 0, v, v + 1, v + 2, v + 3, 1, 1, (Node*)dN.p, (ReviewCol*)dc.p, 1,
                             &nout, st);
    }
    if (st) hipStreamDestroy(st);
    for (DBuf* x : {&dD, &dN, &dv, &dc}) x->free_();
  });
}

int gk_engine_prepare(gk_engine* e, int device) {
  if (!e) return GK_EINVAL;
  ReadLock rl;
  const int rc = read_lock(e, rl, device != 0 && !e->host_only);
  if (rc == GK_OK && device != 0 && !e->host_only && e->dev_ok) {
    // staging's process-wide resources: the pinned upload buffers and the
    // host worker pool
    upload_bounce_init();
    parallel_run(default_threads(), [](int) {});
    if (env_mode("GKGPU_DEVICE_LAYOUT", 1, 1) != 0) device_layout_warmup();
  }
  return rc;
}

int gk_template_backend(gk_engine* e, const char* kind, int* backend, const char** detail) {
  if (!e || !kind) return GK_EINVAL;
  WriteLock g(e);  // compiles on demand
  try {
    rebuild_modules(e);
  } catch (const std::exception& ex) {
    return fail(e, GK_EPARSE, ex.what());
  }
  auto it = e->templates.find(kind);
  if (it == e->templates.end()) return GK_ENOTFOUND;
  int b = 0;
  const char* d = it->second.reason.c_str();
  if (it->second.supported) {
    ensure_jit(e, false);
    auto& j = e->jits[it->second.prog];
    b = j.state == 1 ? 2 : 1;
    d = j.state == 1 ? j.name.c_str() : (e->jit_enabled ? j.log.c_str() : "jit disabled");
  } else if (it->second.guard) {
    b = 3;  // guard program on the GPU, CPU OPA for the reviews that reach an unsupported expression
    ensure_jit(e, false);
    auto& j = e->jits[it->second.prog];
    it->second.detail = it->second.reason + (j.state == 1 ? " [guard kernel " + j.name + "]" : " [guard: bytecode VM]");
    d = it->second.detail.c_str();
  }
  if (backend) *backend = b;
  if (detail) *detail = d;
  return GK_OK;
}

int gk_results_copy_device_output(gk_engine* e, const gk_results* r, void* tuples_dst, void* bytes_dst,
                                  uint64_t* n_tuples) {
  if (!e || !r) return GK_EINVAL;
  EvalCtx* x = r->ctx;
  if (!x || r->epoch == 0) return fail(e, GK_EINVAL, "the results hold no device output");
  ReadLock rl;
  int rc = read_lock(e, rl, true);
  if (rc != GK_OK) return rc;
  std::lock_guard<std::mutex> hold(x->busy);  // the context may not start another evaluation meanwhile
  if (r->epoch != x->eval_epoch || r->gen != e->gen)
    return fail(e, GK_EINVAL, "device output was overwritten by a later evaluation on this engine");
  uint64_t kept = 0;
  if (tuples_dst && r->dev_tuples) {
    // only the tuples of reviews the engine answered (rows of
    // reviews flagged error / fallback, or of a constraint whose
    // enforcementAction is invalid, belong to the CPU re-run, not to this output)
    const uint32_t ncons = (uint32_t)e->corder.size();
    bool any_err = false;
    std::vector<uint8_t> cerr(ncons, 0);
    for (uint32_t c = 0; c < ncons; ++c) { cerr[c] = e->corder[c]->ea_error; any_err |= cerr[c] != 0; }
    if (!x->d_ncand.reserve(16) || (any_err && !up(x->d_cerr, cerr, false)))
      return fail(e, GK_EDEVICE, "device allocation failed");
    int lr = gk_launch_filter((const Viol*)x->d_out.p, r->dev_tuples, (uint32_t*)x->d_rflags.p,
                              any_err ? (const uint8_t*)x->d_cerr.p : nullptr, (Viol*)tuples_dst,
                              (unsigned long long*)x->d_ncand.p, x->stream);
    if (lr != 0) return fail(e, GK_EDEVICE, std::string("device copy failed (filter launch): ") + hipGetErrorString((hipError_t)lr));
    hipError_t ce = hipMemcpyAsync(&kept, x->d_ncand.p, 8, hipMemcpyDeviceToHost, x->stream);
    if (ce == hipSuccess) ce = hipStreamSynchronize(x->stream);
    if (ce != hipSuccess) return fail(e, GK_EDEVICE, std::string("device copy failed (filter): ") + hipGetErrorString(ce));
  }
  if (bytes_dst && r->dev_bytes) {
    hipError_t ce = hipMemcpyAsync(bytes_dst, x->d_bytes.p, r->dev_bytes, hipMemcpyDeviceToDevice, x->stream);
    if (ce == hipSuccess) ce = hipStreamSynchronize(x->stream);
    if (ce != hipSuccess) return fail(e, GK_EDEVICE, std::string("device copy failed (bytes): ") + hipGetErrorString(ce));
  }
  if (n_tuples) *n_tuples = kept;
  return GK_OK;
}

int gk_results_device_counts(const gk_results* r, uint64_t* tuples, uint64_t* bytes) {
  if (!r) return GK_EINVAL;
  if (tuples) *tuples = r->dev_tuples;
  if (bytes) *bytes = r->dev_bytes;
  return GK_OK;
}

int gk_excluder_add(gk_engine* e, const char* const* processes, size_t np, const char* const* namespaces, size_t nn) {
  if (!e || (np && !processes) || (nn && !namespaces)) return GK_EINVAL;
  WriteLock g(e);
  static const char* all[] = {"audit", "webhook", "sync"};  // excluder.go allProcesses
  for (size_t i = 0; i < nn; ++i)
    for (size_t j = 0; j < np; ++j) {
      if (!namespaces[i] || !processes[j]) return GK_EINVAL;
      if (!strcmp(processes[j], "*")) for (const char* p : all) e->excluded[p].insert(namespaces[i]);
      else e->excluded[processes[j]].insert(namespaces[i]);
    }
  e->gen++;  // staged batches applied the previous exclusions
  return GK_OK;
}

int gk_excluder_clear(gk_engine* e) {
  if (!e) return GK_EINVAL;
  WriteLock g(e);
  e->excluded.clear();
  e->gen++;
  return GK_OK;
}

int gk_excluder_is_excluded(gk_engine* e, const char* process, const char* ns) {
  if (!e || !process || !ns) return 0;
  ReadLock rl;
  read_lock_raw(e, rl);
  auto it = e->excluded.find(process);
  return it != e->excluded.end() && it->second.count(ns) ? 1 : 0;
}

uint64_t gk_results_excluded(const gk_results* r) { return r ? r->excluded : 0; }

int gk_dump(gk_engine* e, char** out) {
  if (!e || !out) return GK_EINVAL;
  ReadLock rl;
  read_lock_raw(e, rl);
  std::string s = "{\"modules\":[";
  bool first = true;
  for (auto& kv : e->modules) {
    if (!first) s += ",";
    first = false;
    s += "\"";
    for (char c : kv.first) { if (c == '"' || c == '\\') s.push_back('\\'); s.push_back(c); }
    s += "\"";
  }
  s += "],\"constraints\":" + std::to_string(e->constraints.size()) + ",\"templates\":{";
  first = true;
  for (auto& kv : e->templates) {
    if (!first) s += ",";
    first = false;
    s += "\"" + kv.first + "\":" + (kv.second.supported ? "\"gpu\"" : "\"fallback\"");
  }
  s += "}}";
  *out = strdup(s.c_str());
  return GK_OK;
}

void gk_free_string(char* s) { free(s); }

size_t gk_results_count(const gk_results* r) { return r ? r->rows.size() : 0; }

int gk_results_get(const gk_results* r, size_t i, gk_result_view* out) {
  if (!r || !out || i >= r->rows.size()) return GK_EINVAL;
  const ResultRow& row = r->rows[i];
  out->review = row.review;
  out->constraint = row.constraint;
  out->constraint_kind = r->ckind[row.constraint].c_str();
  out->constraint_name = r->cname[row.constraint].c_str();
  out->msg = row.msg.data();
  out->msg_len = row.msg.size();
  out->details_json = row.details.data();
  out->details_len = row.details.size();
  out->enforcement_action = r->cea[row.constraint].c_str();
  return GK_OK;
}

int gk_results_export(const gk_results* r, void* buf, size_t cap, size_t* needed) {
  if (!r) return GK_EINVAL;
  size_t n = 0;
  for (const ResultRow& row : r->rows) n += 16 + row.msg.size() + row.details.size();
  if (needed) *needed = n;
  if (!buf || cap < n) return buf ? GK_EINVAL : GK_OK;
  char* p = (char*)buf;
  for (const ResultRow& row : r->rows) {
    const uint32_t h[4] = {row.review, row.constraint, (uint32_t)row.msg.size(), (uint32_t)row.details.size()};
    memcpy(p, h, 16);
    p += 16;
    if (!row.msg.empty()) memcpy(p, row.msg.data(), row.msg.size());
    p += row.msg.size();
    if (!row.details.empty()) memcpy(p, row.details.data(), row.details.size());
    p += row.details.size();
  }
  return GK_OK;
}

size_t gk_results_reviews(const gk_results* r) { return r ? std::max<size_t>(r->nrev, r->status.size()) : 0; }
uint32_t gk_results_review_status(const gk_results* r, size_t i) { return r && i < r->status.size() ? r->status[i] : 0; }
uint32_t gk_results_review_reason(const gk_results* r, size_t i) { return r && i < r->reason.size() ? r->reason[i] : 0; }
size_t gk_results_constraints(const gk_results* r) { return r ? r->totals.size() : 0; }
uint64_t gk_results_constraint_total(const gk_results* r, size_t c) { return r && c < r->totals.size() ? r->totals[c] : 0; }
int gk_results_timing(const gk_results* r, double* ms5) {
  if (!r || !ms5) return GK_EINVAL;
  for (int i = 0; i < 5; ++i) ms5[i] = r->ms[i];
  return GK_OK;
}
void gk_results_free(gk_results* r) { delete r; }
uint64_t gk_results_generation(const gk_results* r) { return r ? r->gen : 0; }

int gk_template_status(gk_engine* e, const char* kind, const char** reason) {
  if (!e || !kind) return -1;
  WriteLock g(e);  // compiles on demand
  try {
    rebuild_modules(e);
  } catch (const std::exception& ex) {
    fail(e, GK_EPARSE, ex.what());
    return -1;
  }
  auto it = e->templates.find(kind);
  if (it == e->templates.end()) return -1;
  if (reason) *reason = it->second.reason.c_str();
  return it->second.supported ? 1 : 0;
}

int gk_template_joins(gk_engine* e, const char* kind, const char** sites) {
  if (!e || !kind) return GK_EINVAL;
  WriteLock g(e);  // compiles on demand
  try {
    rebuild_modules(e);
  } catch (const std::exception& ex) {
    return fail(e, GK_EPARSE, ex.what());
  }
  auto it = e->templates.find(kind);
  if (it == e->templates.end()) return GK_ENOTFOUND;
  it->second.joins.clear();
  int n = 0;
  if (it->second.prog >= 0)
    for (auto& js : e->progs[it->second.prog].joins) {
      it->second.joins += (n ? ";" : "") + js.desc;
      ++n;
    }
  if (sites) *sites = it->second.joins.c_str();
  return n;
}

// diagnostics: the referenced-path plan of a template's program (colplan.h);
// *out is malloc'd (gk_free_string)
extern "C" int gk_debug_template_paths(gk_engine* e, const char* kind, char** out) {
  if (!e || !kind || !out) return GK_EINVAL;
  WriteLock g(e);
  try {
    rebuild_modules(e);
  } catch (const std::exception& ex) {
    return fail(e, GK_EPARSE, ex.what());
  }
  auto it = e->templates.find(kind);
  if (it == e->templates.end() || it->second.prog < 0) return GK_ENOTFOUND;
  const std::string d = gk::plan_paths(e->progs[it->second.prog], e->bank).describe(e->st);
  *out = strdup(d.c_str());
  return GK_OK;
}

int gk_join_stats(gk_engine* e, uint64_t* indexes, uint64_t* entries, uint64_t* unindexed, uint64_t* leaves,
                  double* build_ms) {
  if (!e) return GK_EINVAL;
  ReadLock rl;
  int rc = read_lock(e, rl, true);
  if (rc != GK_OK) return rc;
  if (indexes) *indexes = e->join_indexes;
  if (entries) *entries = e->join_entries;
  if (unindexed) *unindexed = e->join_unindexed;
  if (leaves) *leaves = e->join_leaves;
  if (build_ms) *build_ms = e->join_ms;
  return GK_OK;
}

size_t gk_constraint_count(gk_engine* e) {
  if (!e) return 0;
  ReadLock rl;
  if (read_lock(e, rl, false) != GK_OK) return 0;
  return e->corder.size();
}

int gk_constraint_info(gk_engine* e, size_t i, const char** kind, const char** name) {
  if (!e) return GK_EINVAL;
  ReadLock rl;
  int rc = read_lock(e, rl, false);
  if (rc != GK_OK) return rc;
  if (i >= e->corder.size()) return GK_EINVAL;
  if (kind) *kind = e->corder[i]->kind.c_str();
  if (name) *name = e->corder[i]->name.c_str();
  return GK_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ diagnostics
extern "C" int gk_debug_store_sizes(gk_engine* e, uint64_t* nodes, uint64_t* strings) {
  if (!e) return GK_EINVAL;
  ReadLock rl;
  int rc = read_lock(e, rl, false);  // permanent region as the next evaluation sees it
  if (rc != GK_OK) return rc;
  std::lock_guard<std::mutex> g(e->smu);
  if (nodes) *nodes = e->st.nodes().size();
  if (strings) *strings = e->st.nstrings();
  return GK_OK;
}

// A staged batch of Query inputs ({"review": ...} documents, as gk_query_batch
// takes them): lets tests evaluate arbitrary review documents through
// gk_batch_eval, and through the CPU baseline on a host-only engine.
// a fresh staged batch of the from-cache reviews (hooks.audit's documents;
// tests run the CPU checker over it)
extern "C" int gk_debug_stage_cache(gk_engine* e, gk_batch** out) {
  if (!e || !out) return GK_EINVAL;
  ReadLock rl;
  int rc = read_lock(e, rl, !e->host_only);
  if (rc != GK_OK) return rc;
  CachePage cp;
  build_cache_page(e, cp);
  return stage_page_locked(e, cp.pg, out);
}

extern "C" int gk_debug_stage_inputs(gk_engine* e, const char* const* inputs, const size_t* lens, size_t n,
                                     gk_batch** out) {
  if (!e || !out || (n && !inputs)) return GK_EINVAL;
  ReadLock rl;
  int rc = read_lock(e, rl, !e->host_only);
  if (rc != GK_OK) return rc;
  std::vector<std::pair<const char*, size_t>> in;
  for (size_t i = 0; i < n; ++i) in.push_back({inputs[i], lens ? lens[i] : strlen(inputs[i])});
  auto b = std::make_unique<gk_batch>();
  b->eng = e;
  b->node_begin = e->perm_nodes;
  std::string err;
  if (!flatten_reviews(e->st, e->smu, e->ns_cache, in, e->perm_nodes, b->arena, b->cols, err))
    return fail(e, GK_EINVAL, err);
  b->node_end = b->node_begin + (uint32_t)b->arena.size();
  b->nrev = (uint32_t)n;
  b->gen = e->gen;
  b->resources.assign(n, ResourceIds{e->st.s_empty, e->st.s_empty, e->st.s_empty, e->st.s_empty});
  b->node_count = b->node_end - b->node_begin;
  if (e->host_only) { *out = b.release(); return GK_OK; }
  if (!e->dev_ok || !sync_strings(e, nullptr) || !up(b->d_revs, b->cols, false) || !batch_upload(e, b.get())) {
    b->d_revs.free_();
    b->d_nodes.free_();
    return fail(e, GK_EDEVICE, "upload failed");
  }
  *out = b.release();
  return GK_OK;
}

// The launch arguments of a staged batch with HOST pointers: the host arena
// holds the same documents as the batch's device nodes while the batch is the
// last one staged and the engine is unchanged.  Used only by the CPU baseline
// (oracle/cpuvm.cc), which runs the same bytecode on host threads; `out` must
// be a gk::DevArgs (checked by size).
// The shader clock (MHz) a spinning wavefront sees on the engine's device:
// s_memtime ticks over s_memrealtime's 100 MHz reference (kernels.hip
// gk_clock_probe).  Diagnostics for box-to-box variance of kernel times.
extern "C" int gk_debug_clock_mhz(gk_engine* e, double* mhz) {
  if (!e || !mhz) return GK_EINVAL;
  ReadLock rl;
  int rc = read_lock(e, rl, true);
  if (rc != GK_OK) return rc;
  if (!e->dev_ok) return fail(e, GK_EDEVICE, "no HIP device available");
  CtxLease lease(e);
  if (!ctx_device(e, lease.x)) return fail(e, GK_EDEVICE, "no HIP device available");
  hipStream_t stream = lease.x->stream;
  unsigned long long* d = nullptr;
  unsigned long long h[3] = {0, 0, 0};
  if (hipMalloc(&d, sizeof h) != hipSuccess) return fail(e, GK_EDEVICE, "device allocation failed");
  int lr = gk_launch_clock_probe(d, 1u << 22, stream);
  bool ok = lr == 0 && hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, stream) == hipSuccess &&
            hipStreamSynchronize(stream) == hipSuccess;
  hipFree(d);
  if (!ok || h[1] == 0) return fail(e, GK_EDEVICE, "clock probe failed");
  *mhz = 100.0 * (double)h[0] / (double)h[1];
  return GK_OK;
}

// The key-pass records of the join plan as of the last gk_debug_host_args
// (8 words per (constraint, site): engine.cc plan_joins); for the CPU checker.
extern "C" int gk_debug_join_plan(gk_engine* e, const uint64_t** sites, uint64_t* nsites) {
  if (!e || !sites || !nsites) return GK_EINVAL;
  std::lock_guard<std::mutex> dg(e->dbg_mu);
  *sites = e->dbg_jsite.empty() ? nullptr : e->dbg_jsite.data();
  *nsites = e->dbg_jsite.size() / 8;
  return GK_OK;
}

extern "C" int gk_debug_host_args(gk_engine* e, const gk_batch* b, void* out, size_t out_size) {
  if (!e || !b || !out || out_size != sizeof(DevArgs)) return GK_EINVAL;
  ReadLock rl;
  int rc = read_lock(e, rl, false);
  if (rc != GK_OK) return rc;
  if (b->gen != e->gen || b->node_begin != e->perm_nodes)
    return fail(e, GK_EINVAL, "engine state changed since the batch was staged");
  std::lock_guard<std::mutex> dg(e->dbg_mu);
  // host copies: the permanent region followed by the batch's documents, and
  // the string / number tables as of now (concurrent evaluations append to them)
  e->dbg_nodes.assign(e->st.nodes().begin(), e->st.nodes().begin() + e->perm_nodes);
  e->dbg_nodes.insert(e->dbg_nodes.end(), b->arena.begin(), b->arena.end());
  {
    std::lock_guard<std::mutex> g(e->smu);
    e->dbg_strs = e->st.strings();
    e->dbg_sflags = e->st.str_flags();
    e->dbg_nums = e->st.numbers();
    e->dbg_pool = e->st.pool();
  }
  e->dbg_cons.clear();
  for (auto* c : e->corder) e->dbg_cons.push_back(c->spec);
  if (e->dbg_cons.empty()) e->dbg_cons.push_back(MatchSpec{});
  e->dbg_progoff.clear();
  for (auto& p : e->progs) e->dbg_progoff.push_back(p.code_off);
  if (e->dbg_progoff.empty()) e->dbg_progoff.push_back(0);
  e->dbg_mwords = e->mwords;
  if (e->dbg_mwords.empty()) e->dbg_mwords.push_back(0);
  e->dbg_fmt = e->bank.fmt;
  if (e->dbg_fmt.empty()) e->dbg_fmt.push_back(0);
  e->dbg_dfa_keys = e->dfa_keys;
  e->dbg_dfa_meta = e->dfa_meta;
  e->dbg_dfa_words = e->dfa_words;
  if (e->dbg_dfa_keys.empty()) { e->dbg_dfa_keys.push_back(NO_ID); e->dbg_dfa_meta.push_back(2u << 30); }
  if (e->dbg_dfa_words.empty()) e->dbg_dfa_words.push_back(0);
  e->dbg_pool.append(16, '\0');  // dword reads past the last string (devrt.h puts_)
  e->dbg_jleaf = e->jleaf;
  e->dbg_jsite = e->jsite;
  DevArgs a{};
  // the join plan's leaf rows (the CPU checker builds its own indexes from
  // them: oracle/cpuvm.cc gkcpu_build_joins; without, every site scans)
  a.jleaf = e->dbg_jleaf.empty() ? nullptr : e->dbg_jleaf.data();
  a.nodes = e->dbg_nodes.data();
  a.strs = e->dbg_strs.data();
  a.pool = (const uint8_t*)e->dbg_pool.data();
  a.sflags = e->dbg_sflags.data();
  a.nums = e->dbg_nums.data();
  a.code = e->bank.code.data();
  a.K = e->bank.consts.data();
  a.fmt = e->dbg_fmt.data();
  a.cons = e->dbg_cons.data();
  a.mwords = e->dbg_mwords.data();
  a.prog_off = e->dbg_progoff.data();
  a.revs = b->cols.data();
  a.dfa_keys = e->dbg_dfa_keys.data();
  a.dfa_meta = e->dbg_dfa_meta.data();
  a.dfa_words = e->dbg_dfa_words.data();
  a.ndfa = (uint32_t)e->dbg_dfa_keys.size();
  a.ncode = (uint32_t)e->bank.code.size();
  a.ncons = (uint32_t)e->corder.size();
  a.nrev = (uint32_t)b->cols.size();
  a.ntiles = (a.nrev + 63) / 64;
  memcpy(out, &a, sizeof a);
  return GK_OK;
}

// gk_debug_host_args over the batch's column form (colstore.h): the
// permanent region followed by the kept subtrees, the review columns with
// their ids, and the host path columns -- the CPU checker then evaluates
// exactly what the device reads.  GK_EINVAL when the batch is in node form.
extern "C" int gk_debug_host_args_columns(gk_engine* e, const gk_batch* b, void* out, size_t out_size) {
  if (!e || !b || !b->columnar) return GK_EINVAL;
  int rc = gk_debug_host_args(e, b, out, out_size);
  if (rc != GK_OK) return rc;
  std::lock_guard<std::mutex> dg(e->dbg_mu);
  e->dbg_nodes.resize(e->perm_nodes);
  e->dbg_nodes.insert(e->dbg_nodes.end(), b->cv.nodes.begin(), b->cv.nodes.end());
  DevArgs a;
  memcpy(&a, out, sizeof a);
  a.nodes = e->dbg_nodes.data();
  a.revs = b->cv.cols.data();
  a.cv_words = b->cv.words.data();
  a.cv_bytes = b->cv.bytes.data();
  a.cv_slots = b->cv.slots.data();
  a.cv_hash = b->cv.hash.data();
  a.cv_views = b->cv.views.data();
  a.cv_tabs = b->cv.tabs.data();
  a.cv_hmask = (uint32_t)b->cv.hash.size() - 1;
  a.cv_on = 1;
  memcpy(out, &a, sizeof a);
  return GK_OK;
}

// the batch's storage form: 1 columns (*schema: the path schema, *why: ""),
// 0 nodes (*why: the reason the columns were not used)
extern "C" int gk_batch_columns(const gk_batch* b, const char** schema, const char** why, uint64_t* bytes) {
  if (!b) return GK_EINVAL;
  if (schema) *schema = b->cv.schema.c_str();
  if (why) *why = b->col_why.c_str();
  if (bytes) *bytes = b->cv.total_bytes();
  return b->columnar ? 1 : 0;
}

// Content hash over a staged batch's review columns (in order), the documents
// and label objects they reference in `all` (node ids as the columns give
// them) and the resource ids: equal for every layout of the same batch.
// Caller holds e->smu.
static uint64_t columns_hash(gk_engine* e, const Node* all, const std::vector<ReviewCol>& cols,
                             const std::vector<ResourceIds>& resources) {
  uint64_t h = 0;
  for (size_t i = 0; i < cols.size(); ++i) {
    const ReviewCol& c = cols[i];
    auto sh = [&](uint32_t sid) -> uint64_t {
      if (sid == NO_ID) return 7;
      std::string_view v = e->st.str(sid);
      return fnv1a(v.data(), v.size());
    };
    uint64_t x = doc_hash(e->st, all, c.root) * 31 + sh(c.group);
    x = x * 31 + sh(c.kind);
    x = x * 31 + sh(c.ns);
    x = x * 31 + sh(c.nsname);
    x = x * 31 + doc_hash(e->st, all, c.labels);
    x = x * 31 + doc_hash(e->st, all, c.old_labels);
    x = x * 31 + doc_hash(e->st, all, c.ns_labels);
    x = x * 31 + c.flags;
    const ResourceIds& r = resources[i];
    x = x * 31 + sh(r.api_version);
    x = x * 31 + sh(r.kind);
    x = x * 31 + sh(r.name);
    x = x * 31 + sh(r.ns);
    h = (h ^ x) * 1099511628211ull + i;
  }
  return h;
}

// The staged batch as the kernels see it: the device node array and review
// columns downloaded and hashed as gk_debug_flatten_page hashes the host
// forms (GPU tests of the device-built layout, layout.hip).
extern "C" int gk_debug_batch_hash(gk_engine* e, const gk_batch* b, uint64_t* hash) {
  if (!e || !b || !hash) return GK_EINVAL;
  ReadLock rl;
  int rc = read_lock(e, rl, false);
  if (rc != GK_OK) return rc;
  if (!b->d_nodes.p || !b->d_revs.p) return fail(e, GK_EINVAL, "batch has no device copy");
  const size_t nn = b->node_end;
  std::vector<Node> all(nn);
  std::vector<ReviewCol> cols(b->cols.size());
  if (hipMemcpy(all.data(), b->d_nodes.p, nn * sizeof(Node), hipMemcpyDeviceToHost) != hipSuccess ||
      (cols.size() && hipMemcpy(cols.data(), b->d_revs.p, cols.size() * sizeof(ReviewCol), hipMemcpyDeviceToHost) != hipSuccess))
    return fail(e, GK_EDEVICE, "device download failed");
  // columns back to batch order (the resource ids' and gk_debug_flatten_page's)
  std::vector<ReviewCol> bcols(cols.size());
  if (b->resources.size() != cols.size()) return fail(e, GK_EINVAL, "column without resource ids");
  for (size_t i = 0; i < cols.size(); ++i) {
    const uint32_t o = b->cols[i].orig == NO_ID ? (uint32_t)i : b->cols[i].orig;
    if (o >= cols.size()) return fail(e, GK_EINVAL, "column order out of range");
    bcols[o] = cols[i];
    bcols[o].orig = NO_ID;
  }
  std::lock_guard<std::mutex> sg(e->smu);
  *hash = columns_hash(e, all.data(), bcols, b->resources);
  return GK_OK;
}

// Flattens a page on `threads` host threads without a device (diagnostics and
// CPU tests): *hash = content hash over every review's columns and document,
// ms2 = [parse + build, total flatten].  The documents are dropped afterwards.
extern "C" int gk_debug_flatten_page(gk_engine* e, const char* objs, const uint64_t* obj_offs, size_t n,
                                     const char* nss, const uint64_t* ns_offs, size_t n_ns, const uint32_t* obj_ns,
                                     int threads, uint64_t* hash, uint64_t* nodes, double* ms2) {
  if (!e) return GK_EINVAL;
  ReadLock rl;
  int rc = read_lock(e, rl, false);
  if (rc != GK_OK) return rc;
  Page pg{objs, obj_offs, n, nss, ns_offs, n_ns, obj_ns};
  FlatResult fr;
  std::string err;
  NodeArena arena;
  auto t0 = Clock::now();
  auto exit_ = e->excluded.find("audit");
  const std::set<std::string>* ex = exit_ == e->excluded.end() ? nullptr : &exit_->second;
  // threads < 0: the staged-batch form (path-grouped layout in evaluation order) on -threads threads
  std::vector<uint32_t> perm;
  const OrderFn ord = [&](const FlatResult& f, size_t lo, size_t hi, std::vector<uint32_t>& p) {
    review_order(e, f.cols, f.weight, lo, hi, p);
  };
  const int nt = threads > 0 ? threads : threads < 0 ? -threads : default_threads();
  // GKGPU_DEBUG_DEVICE_FORM (with threads < 0): the per-document arena the
  // device layout pass (layout.hip) starts from
  DevLayout dl;
  const bool dform = threads < 0 && getenv("GKGPU_DEBUG_DEVICE_FORM");
  if (!flatten_page(e->st, e->smu, e->ns_cache, ex, pg, nt, e->perm_nodes, arena, fr, err, threads < 0 ? &ord : nullptr,
                    threads < 0 ? &perm : nullptr, dform ? &dl : nullptr))
    return fail(e, GK_EINVAL, err);
  if (dform && (dl.beg.size() != fr.cols.size() || dl.nroots > fr.cols.size()))
    return fail(e, GK_EINVAL, "device layout inputs do not match the columns");
  double tot = ms_since(t0);
  std::vector<Node> all(e->st.nodes().begin(), e->st.nodes().begin() + e->perm_nodes);
  all.insert(all.end(), arena.begin(), arena.end());
  std::lock_guard<std::mutex> sg(e->smu);
  const uint64_t h = columns_hash(e, all.data(), fr.cols, fr.resources);
  if (hash) *hash = h;
  if (nodes) *nodes = fr.node_count;
  if (ms2) { ms2[0] = fr.ms_parse; ms2[1] = tot; }
  return GK_OK;
}

extern "C" int gk_debug_disasm(gk_engine* e, const char* kind, char** out) {
  if (!e || !kind || !out) return GK_EINVAL;
  ReadLock rl;
  int rc = read_lock(e, rl, false);
  if (rc != GK_OK) return rc;
  std::lock_guard<std::mutex> dg(e->dbg_mu);
  auto it = e->templates.find(kind);
  if (it == e->templates.end() || it->second.prog < 0) return GK_ENOTFOUND;
  const Program& p = e->progs[it->second.prog];
  static const char* names[] = {"END", "JMP", "JUNDEF", "JFALSE", "JTRUE", "LOADK", "LOADREV", "LOADPARAM", "MOV",
                                "GET", "GETK", "ITER_INIT", "ITER_NEXT", "CMP", "ARITH", "LIST_NEW", "LIST_ADD",
                                "OBJ_PUT", "YIELD", "CALL", "SPRINTF", "EMIT", "LEN_EQ", "FAIL_FALLBACK", "TABLE",
                                "MEMO_GET", "MEMO_PUT", "ORD", "JPROBE", "JNEXT", "JVAR", "KEYOUT"};
  static_assert(sizeof(names) / sizeof(names[0]) == OP_COUNT_, "opcode names");
  std::string s = "nregs=" + std::to_string(p.nregs) + " len=" + std::to_string(p.code_len) + "\n";
  for (uint32_t i = 0; i < p.code_len; ++i) {
    const Ins& in = e->bank.code[p.code_off + i];
    char buf[160];
    uint32_t pc = p.code_off + i;
    snprintf(buf, sizeof buf, "%10u %5u %-10s a=%u b=%u c=%u x=%u y=%u", pc < e->pchist.size() ? e->pchist[pc] : 0u, pc,
             in.op < OP_COUNT_ ? names[in.op] : "?", in.a, in.b, in.c, in.x, in.y);
    s += buf;
    if ((in.op == OP_LOADK || in.op == OP_GETK) && in.x < e->bank.consts.size()) {
      uint64_t k = e->bank.consts[in.x];
      uint32_t tag = (uint32_t)(k >> 60);
      if (tag == V_STR) s += "  ; \"" + std::string(e->st.str((uint32_t)(k & 0xffffffffu))) + "\"";
      else { char kb[48]; snprintf(kb, sizeof kb, "  ; tag=%u pay=%llu", tag, (unsigned long long)(k & 0x0fffffffffffffffull)); s += kb; }
    }
    s += "\n";
  }
  *out = strdup(s.c_str());
  return GK_OK;
}
