// Parallel host flattener (see flatten.h).
//
// Phase 1 (parallel): each thread parses a contiguous range of the page's
// objects and builds their review documents in a thread-local Store (its own
// string / number interning, its own node arena; the well-known strings have
// the same ids in every Store because every Store interns them first).
// Phase 2 (serial, small): every thread's distinct strings and numbers are
// interned into the engine's Store, giving per-thread id maps.
// Phase 3 (parallel): each thread copies its nodes into the engine arena at its
// offset, rewriting string / number ids and child indices, and relocates its
// review columns.
#include "flatten.h"

#include <algorithm>
#include <sched.h>
#include <cstdlib>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <immintrin.h>
#include <map>
#include <functional>
#include <memory>
#include <thread>
#include <mutex>
#include <unordered_map>

namespace gk {

static const char* EMPTY_NS_JSON = "{\"metadata\":{\"creationTimestamp\":null},\"spec\":{},\"status\":{}}";
static constexpr uint32_t kFixedNodes = 4;  // every Store starts with nodes {} null false true
// path-grouped layout (flatten.h): local marker of a Namespace document's
// nodes, whose runs every review of the namespace shares
static constexpr uint8_t kShared = 0x80;

int default_threads() {
  const char* v = getenv("GKGPU_THREADS");
  if (v && *v) {
    int n = atoi(v);
    if (n >= 1 && n <= 256) return n;
  }
  // the host cores this process is leased: its CPU affinity set, capped by a
  // cgroup CPU quota (the GPU box grants a 16-CPU share of a 256-CPU host:
  // cpu.max "1600000 100000", affinity 0-255)
  static const int leased = [] {
    int n = 0;
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = CPU_COUNT(&cs);
    if (n <= 0) n = (int)std::max(1u, std::thread::hardware_concurrency());
    long long q = 0, per = 0;
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char a[32] = {0};
      if (fscanf(f, "%31s %lld", a, &per) == 2 && strcmp(a, "max") != 0) q = atoll(a);
      fclose(f);
    } else if (FILE* f2 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
      if (fscanf(f2, "%lld", &q) != 1) q = 0;
      fclose(f2);
      if (FILE* f3 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
        if (fscanf(f3, "%lld", &per) != 1) per = 0;
        fclose(f3);
      }
    }
    if (q > 0 && per > 0) n = std::min<int>(n, (int)std::max<long long>(1, (q + per - 1) / per));
    return std::max(1, std::min(n, 256));
  }();
  return leased;
}

// ------------------------------------------------------------------ worker pool
namespace {
struct PoolJob {
  const std::function<void(int)>* f;
  int n;
  std::atomic<int> next{1};  // next unclaimed index (the caller runs 0)
  std::atomic<int> left;
  std::mutex mu;
  std::condition_variable cv;
};
// Jobs, not indices, are queued: a thread claims the next index of the job
// at the queue's front with one atomic.  The caller of run() helps only with
// its OWN job's indices -- never another caller's task, so a caller holding a
// lock across parallel_run (merge_parts' smu, the upload's Bounce::mu) cannot
// be stalled by someone else's long part, nor re-enter a lock it holds.
struct WorkPool {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::shared_ptr<PoolJob>> q;  // jobs with indices left to claim
  std::atomic<int> pending{0};  // q.size(), readable without the lock
  int workers = 0;
  static void finish(PoolJob& j) {
    if (j.left.fetch_sub(1) == 1) {
      std::lock_guard<std::mutex> g(j.mu);
      j.cv.notify_all();
    }
  }
  void retire(const std::shared_ptr<PoolJob>& job) {  // every index claimed: off the queue
    std::lock_guard<std::mutex> g(mu);
    for (auto it = q.begin(); it != q.end(); ++it)
      if (*it == job) { q.erase(it); pending.fetch_sub(1, std::memory_order_relaxed); break; }
  }
  void worker() {
    for (;;) {
      // spin a little before sleeping: a micro-batch's phases (parse, intern,
      // relocate) and the next request come back to back, and waking a
      // sleeping thread takes longer than a 256-request part's parse
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(200);
      for (int k = 0; pending.load(std::memory_order_relaxed) == 0; ++k) {
        _mm_pause();
        if ((k & 63) == 63 && std::chrono::steady_clock::now() >= until) break;
      }
      std::shared_ptr<PoolJob> job;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !q.empty(); });
        job = q.front();
      }
      const int i = job->next.fetch_add(1);
      if (i >= job->n) { retire(job); continue; }
      (*job->f)(i);
      finish(*job);
    }
  }
  void run(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    if (n == 1) { f(0); return; }
    auto job = std::make_shared<PoolJob>();
    job->f = &f;
    job->n = n;
    job->left = n;
    {
      std::lock_guard<std::mutex> g(mu);
      const int want = std::max(1, default_threads() - 1);
      while (workers < want) {
        std::thread([this] { worker(); }).detach();
        ++workers;
      }
      q.push_back(job);
      pending.fetch_add(1, std::memory_order_relaxed);
    }
    cv.notify_all();
    f(0);
    finish(*job);
    for (int i; (i = job->next.fetch_add(1)) < n;) {  // help with this job only
      f(i);
      finish(*job);
    }
    retire(job);
    std::unique_lock<std::mutex> lk(job->mu);
    job->cv.wait(lk, [&] { return job->left.load() == 0; });
  }
};
WorkPool& pool() {
  static WorkPool* p = new WorkPool();  // never destroyed: detached workers outlive static destructors
  return *p;
}
}  // namespace

void parallel_run(int n, const std::function<void(int)>& f) { pool().run(n, f); }

ReviewCol review_columns(const Store& st, const Store& gst, const NsCache& ns_cache, uint32_t root,
                         bool* ns_labels_global) {
  ReviewCol rc{};
  *ns_labels_global = false;
  rc.root = root;
  rc.orig = NO_ID;
  rc.group = rc.kind = rc.ns = rc.nsname = NO_ID;
  rc.labels = rc.old_labels = rc.ns_labels = NO_ID;
  if (root == NO_ID) return rc;  // input.review undefined: nothing matches
  if (ntype(st, root) != NT_OBJ) { rc.flags |= RC_FALLBACK; return rc; }
  rc.flags |= RC_REVIEW_DEF;
  uint32_t kind = nget(st, root, st.s_kind);
  if (kind != NO_ID) {
    if (ntype(st, kind) != NT_OBJ) { rc.flags |= RC_FALLBACK; return rc; }
    rc.flags |= RC_KIND_OK;
    uint32_t g = nget(st, kind, st.s_group), k = nget(st, kind, st.s_kind);
    if (g != NO_ID && ntype(st, g) != NT_STR) { rc.flags |= RC_FALLBACK; return rc; }
    if (k != NO_ID && ntype(st, k) != NT_STR) { rc.flags |= RC_FALLBACK; return rc; }
    if (g != NO_ID) rc.group = st.nodes()[g].val;
    if (k != NO_ID) rc.kind = st.nodes()[k].val;
    if (rc.group == st.s_empty && rc.kind == st.s_Namespace) rc.flags |= RC_IS_NS;
  }
  uint32_t ns = nget(st, root, st.s_namespace);
  if (ns != NO_ID) {
    if (ntype(st, ns) != NT_STR) { rc.flags |= RC_FALLBACK; return rc; }
    rc.flags |= RC_HAS_NS;
    rc.ns = st.nodes()[ns].val;
    if (rc.ns == st.s_empty) rc.flags |= RC_NS_EMPTY;
  } else {
    rc.flags |= RC_NS_EMPTY;
  }
  uint32_t obj = nget(st, root, st.s_object);
  uint32_t old = nget(st, root, st.s_oldObject);
  if (rc.flags & RC_IS_NS) {
    uint32_t nm = NO_ID;
    uint32_t md = ntype(st, obj) == NT_OBJ ? nget(st, obj, st.s_metadata) : NO_ID;
    if (ntype(st, md) == NT_OBJ) nm = nget(st, md, st.s_name);
    if (nm != NO_ID) {
      if (ntype(st, nm) != NT_STR) { rc.flags |= RC_FALLBACK; return rc; }
      rc.nsname = st.nodes()[nm].val;
      rc.flags |= RC_NAME_OK;
    }
  } else {
    rc.nsname = rc.ns;
  }
  // object / oldObject emptiness: get_default(review, "object", {}) == {}
  auto empty = [&](uint32_t n) { return n == NO_ID || ntype(st, n) == NT_NULL || is_empty_obj(st, n); };
  auto labels_of = [&](uint32_t o, uint32_t* out) -> bool {
    uint32_t md = ntype(st, o) == NT_OBJ ? gdef(st, o, "metadata") : NO_ID;
    if (md != NO_ID && ntype(st, md) != NT_OBJ) { *out = NO_ID; return ntype(st, o) == NT_OBJ ? false : true; }
    uint32_t lb = md == NO_ID ? NO_ID : gdef(st, md, "labels");
    if (lb == NO_ID) { *out = NO_ID; return true; }
    if (ntype(st, lb) != NT_OBJ) return false;
    const Node ln = st.nodes()[lb];
    for (uint32_t i = 0; i < ln.n; ++i) if (st.nodes()[ln.first + i].type != NT_STR) return false;
    *out = lb;
    return true;
  };
  bool oe = empty(obj), le = empty(old);
  if (!oe && ntype(st, obj) != NT_OBJ) { rc.flags |= RC_FALLBACK; return rc; }
  if (!le && ntype(st, old) != NT_OBJ) { rc.flags |= RC_FALLBACK; return rc; }
  if (!oe) { if (!labels_of(obj, &rc.labels)) { rc.flags |= RC_FALLBACK; return rc; } rc.flags |= RC_LABELS_OBJ; }
  if (!le) { if (!labels_of(old, &rc.old_labels)) { rc.flags |= RC_FALLBACK; return rc; } rc.flags |= RC_LABELS_OLD; }
  // namespace object for namespaceSelector: _unstable.namespace, else the cache
  uint32_t un = nget(st, root, st.s_unstable);
  uint32_t unns = ntype(st, un) == NT_OBJ ? nget(st, un, st.s_namespace) : NO_ID;
  if (un != NO_ID && ntype(st, un) != NT_OBJ) { rc.flags |= RC_FALLBACK; return rc; }
  auto ns_labels = [&](const Store& s, uint32_t nsobj) -> bool {
    uint32_t md = gdef(s, nsobj, "metadata");
    if (md != NO_ID && ntype(s, md) != NT_OBJ) return false;
    uint32_t lb = md == NO_ID ? NO_ID : gdef(s, md, "labels");
    if (lb != NO_ID) {
      if (ntype(s, lb) != NT_OBJ) return false;
      const Node ln = s.nodes()[lb];
      for (uint32_t i = 0; i < ln.n; ++i) if (s.nodes()[ln.first + i].type != NT_STR) return false;
    }
    rc.ns_labels = lb;
    return true;
  };
  if (unns != NO_ID) {
    if (ntype(st, unns) != NT_OBJ) { rc.flags |= RC_FALLBACK; return rc; }
    rc.flags |= RC_UNSTABLE_NS;
    if (!ns_labels(st, unns)) { rc.flags |= RC_FALLBACK; return rc; }
  } else if (rc.flags & RC_HAS_NS) {
    auto it = ns_cache.find(std::string(st.str(rc.ns)));
    if (it != ns_cache.end()) {
      uint32_t nsn = it->second;
      if (ntype(gst, nsn) == NT_FALSE) {
        // falsy cached value: not "cached" for autoreject, no get_ns solution
      } else {
        if (ntype(gst, nsn) != NT_OBJ) { rc.flags |= RC_FALLBACK; return rc; }
        rc.flags |= RC_NS_CACHED;
        if (!ns_labels(gst, nsn)) { rc.flags |= RC_FALLBACK; return rc; }
        *ns_labels_global = rc.ns_labels != NO_ID;
      }
    }
  }
  return rc;
}

namespace {

struct NsDoc {
  uint32_t root = NO_ID;   // placed root node of the Namespace document
  std::string name;        // metadata.name ("" when absent)
  uint32_t sid = NO_ID;    // its string id
};

// string id of member `key` of the object record `o`, if it is a string
inline uint32_t member_str(const Store& st, const Node& o, uint32_t key) {
  if (o.type != NT_OBJ) return NO_ID;
  const Node* c = st.nodes().data() + o.first;
  for (uint32_t i = 0; i < o.n; ++i)
    if (c[i].key == key) return c[i].type == NT_STR ? c[i].val : NO_ID;
  return NO_ID;
}
inline const Node* member(const Store& st, const Node& o, uint32_t key) {
  if (o.type != NT_OBJ) return nullptr;
  const Node* c = st.nodes().data() + o.first;
  for (uint32_t i = 0; i < o.n; ++i)
    if (c[i].key == key) return &c[i];
  return nullptr;
}

struct Keys {
  uint32_t apiVersion;
  explicit Keys(Store& st) : apiVersion(st.intern("apiVersion")) {}
};

// Review(AugmentedUnstructured{obj, ns}) envelope (pkg/target/target.go:129-163,
// admission/v1beta1 AdmissionRequest json field order):
//   uid kind resource [name] [namespace] operation userInfo object oldObject options _unstable
// `obj` is the object's parsed root record (Store::parse_doc).
uint32_t build_object_review(Store& st, const Keys& K, const Node& obj, const NsDoc& ns, ResourceIds* res) {
  uint32_t s_apiv = member_str(st, obj, K.apiVersion);
  uint32_t s_kind = member_str(st, obj, st.s_kind);
  uint32_t s_name = NO_ID, s_objns = NO_ID;
  if (const Node* md = member(st, obj, st.s_metadata)) {
    s_name = member_str(st, *md, st.s_name);
    s_objns = member_str(st, *md, st.s_namespace);
  }
  if (s_apiv == NO_ID) s_apiv = st.s_empty;
  if (s_kind == NO_ID) s_kind = st.s_empty;
  if (s_name == NO_ID) s_name = st.s_empty;
  if (s_objns == NO_ID) s_objns = st.s_empty;
  // schema.ParseGroupVersion: "v" -> ("", v), "g/v" -> (g, v); more slashes
  // fail to parse, and unstructured.GroupVersionKind() then returns an EMPTY
  // GVK (unstructured.go:425-432): the review's kind.kind is "" as well
  uint32_t s_group = st.s_empty, s_version = st.s_empty;
  {
    std::string apiv(st.str(s_apiv));
    size_t slash = apiv.find('/');
    if (slash == std::string::npos) s_version = s_apiv;
    else if (apiv.find('/', slash + 1) == std::string::npos) {
      s_group = st.intern(apiv.data(), slash);
      s_version = st.intern(apiv.data() + slash + 1, apiv.size() - slash - 1);
    } else {
      s_kind = st.s_empty;
    }
  }
  const bool has_name = s_name != st.s_empty, has_ns = !ns.name.empty();
  uint32_t nch = 9 + (has_name ? 1 : 0) + (has_ns ? 1 : 0);
  // the envelope: root, its children, kind{3}, resource{3}, _unstable{1}
  uint32_t root = (uint32_t)st.nodes().size();
  st.nodes().resize(root + 1 + nch + 3 + 3 + 1);
  Node* N = st.nodes().data();
  uint32_t first = root + 1, kf = first + nch, rf = kf + 3, uf = rf + 3;
  auto obj_node = [&](uint32_t key, uint32_t f, uint32_t n) { Node x{}; x.key = key; x.type = NT_OBJ; x.first = f; x.n = (uint16_t)n; return x; };
  auto str_node = [&](uint32_t key, uint32_t sid) { Node x{}; x.key = key; x.type = NT_STR; x.val = sid; return x; };
  auto lit_node = [&](uint32_t key, uint8_t t) { Node x{}; x.key = key; x.type = t; return x; };
  N[root] = obj_node(0, first, nch);
  uint32_t i = first;
  N[i++] = str_node(st.s_uid, st.s_empty);
  N[i++] = obj_node(st.s_kind, kf, 3);
  N[i++] = obj_node(st.s_resource, rf, 3);
  if (has_name) N[i++] = str_node(st.s_name, s_name);
  if (has_ns) N[i++] = str_node(st.s_namespace, ns.sid);
  N[i++] = str_node(st.s_operation, st.s_empty);
  N[i++] = obj_node(st.s_userInfo, 0, 0);
  Node o = obj;
  o.key = st.s_object;
  N[i++] = o;
  N[i++] = lit_node(st.s_oldObject, NT_NULL);
  N[i++] = lit_node(st.s_options, NT_NULL);
  N[i++] = obj_node(st.s_unstable, uf, 1);
  N[kf] = str_node(st.s_group, s_group);
  N[kf + 1] = str_node(st.s_version, s_version);
  N[kf + 2] = str_node(st.s_kind, s_kind);
  N[rf] = str_node(st.s_group, st.s_empty);
  N[rf + 1] = str_node(st.s_version, st.s_empty);
  N[rf + 2] = str_node(st.s_resource, st.s_empty);
  // _unstable: {"namespace": <ns>} (the page's shared Namespace document)
  Node nsn = N[ns.root];
  nsn.key = st.s_namespace;
  nsn.flags &= (uint8_t)~kShared;  // the review's own node; its members are the shared run
  N[uf] = nsn;
  // HandleViolation: apiVersion = group/version (version alone when group is "")
  res->api_version = s_group == st.s_empty ? s_version : s_apiv;
  res->kind = s_kind;
  res->name = s_name;
  res->ns = s_objns;
  return root;
}

// hooks.audit's review of a synced object (target_template_source.go:46-89):
//   make_review: {"kind": {"group", "version", "kind"}, "name": name, "object": obj}
//   add_field(r, "namespace", ns) for namespaced objects: the keys of r whose
//   values are truthy plus "namespace", each value get_default(r, k, ns) -- so
//   a null object becomes the namespace string, and the members keep that order
// `obj` is the object's parsed root record.
uint32_t build_cache_review(Store& st, const Keys& K, const Node& obj, const Page::CacheKey& ck, ResourceIds* res) {
  const uint32_t s_group = st.intern(ck.group.data(), ck.group.size());
  const uint32_t s_version = st.intern(ck.version.data(), ck.version.size());
  const uint32_t s_kind = st.intern(ck.kind.data(), ck.kind.size());
  const uint32_t s_name = st.intern(ck.name.data(), ck.name.size());
  const uint32_t s_ns = ck.namespaced ? st.intern(ck.ns.data(), ck.ns.size()) : st.s_empty;
  // add_field drops a falsy member: an object that is JSON `false`
  const bool has_obj = !(ck.namespaced && obj.type == NT_FALSE);
  const uint32_t nch = 2 + (has_obj ? 1 : 0) + (ck.namespaced ? 1 : 0);
  const uint32_t root = (uint32_t)st.nodes().size();
  st.nodes().resize(root + 1 + nch + 3);
  Node* N = st.nodes().data();
  const uint32_t first = root + 1, kf = first + nch;
  auto obj_node = [&](uint32_t key, uint32_t f, uint32_t n) { Node x{}; x.key = key; x.type = NT_OBJ; x.first = f; x.n = (uint16_t)n; return x; };
  auto str_node = [&](uint32_t key, uint32_t sid) { Node x{}; x.key = key; x.type = NT_STR; x.val = sid; return x; };
  N[root] = obj_node(0, first, nch);
  uint32_t i = first;
  N[i++] = obj_node(st.s_kind, kf, 3);
  N[i++] = str_node(st.s_name, s_name);
  if (has_obj) {
    if (ck.namespaced && obj.type == NT_NULL) {
      N[i++] = str_node(st.s_object, s_ns);  // get_default(r, "object", namespace)
    } else {
      Node o = obj;
      o.key = st.s_object;
      N[i++] = o;
    }
  }
  if (ck.namespaced) N[i++] = str_node(st.s_namespace, s_ns);
  N[kf] = str_node(st.s_group, s_group);
  N[kf + 1] = str_node(st.s_version, s_version);
  N[kf + 2] = str_node(st.s_kind, s_kind);
  // HandleViolation (target.go:193-244): apiVersion from review.kind, the
  // object's own metadata name / namespace
  uint32_t s_oname = NO_ID, s_ons = NO_ID;
  if (const Node* md = member(st, obj, st.s_metadata)) {
    s_oname = member_str(st, *md, st.s_name);
    s_ons = member_str(st, *md, st.s_namespace);
  }
  if (s_group == st.s_empty) res->api_version = s_version;
  else {
    std::string av = std::string(ck.group) + "/" + std::string(ck.version);
    res->api_version = st.intern(av.data(), av.size());
  }
  res->kind = s_kind;
  res->name = s_oname == NO_ID ? st.s_empty : s_oname;
  res->ns = s_ons == NO_ID ? st.s_empty : s_ons;
  (void)K;
  return root;
}

// ------------------------------------------------------------------ path-grouped layout (flatten.h)
constexpr uint32_t kElem = 0xfffffffeu;   // path key of array elements
constexpr uint32_t kMaxPaths = 1u << 16;  // per part; further distinct paths share their parent's region

// A part's document paths: path 0 is the review root; path(child) =
// (path(parent), member key id | kElem), key ids local to the part.  A path
// names the region that holds the member runs of its instances.
struct PathTab {
  std::unordered_map<uint64_t, uint32_t> m;
  std::vector<std::pair<uint32_t, uint32_t>> def;  // (parent, key)
  static constexpr uint32_t C = 4096;
  std::vector<uint64_t> ck;                         // direct-mapped cache of m
  std::vector<uint32_t> cv;
  PathTab() : def{{NO_ID, NO_ID}}, ck(C, ~0ull), cv(C, 0) {}
  uint32_t child(uint32_t parent, uint32_t key) {
    const uint64_t k = ((uint64_t)parent << 32) | key;
    const uint32_t h = (uint32_t)((k * 0x9e3779b97f4a7c15ull) >> 52) & (C - 1);
    if (ck[h] == k) return cv[h];
    uint32_t id;
    auto it = m.find(k);
    if (it != m.end()) id = it->second;
    else if (def.size() >= kMaxPaths) return parent;  // full: the table never changes again
    else {
      id = (uint32_t)def.size();
      m.emplace(k, id);
      def.push_back({parent, key});
    }
    ck[h] = k;
    cv[h] = id;
    return id;
  }
};

struct Part {
  Store st;
  size_t lo = 0, hi = 0;
  std::vector<ReviewCol> cols;
  std::vector<uint8_t> nsglob;       // per review: rc.ns_labels is a global node
  std::vector<uint32_t> weight;
  std::vector<ResourceIds> res;
  std::vector<uint32_t> ns_roots;    // placed Namespace documents (their runs are shared by reviews)
  // staged layout: the part's document paths and the nodes each path's
  // region receives from the part, counted while each document is hot
  bool count_paths = false;
  PathTab paths;
  std::vector<uint64_t> pcount;
  uint64_t excluded = 0;
  std::string err;
  // phase 2 maps (local id -> global id)
  std::vector<uint32_t> smap, nmap;
  uint64_t node_off = 0;             // global index of this part's node kFixedNodes
  std::vector<uint32_t> rbeg;        // per review: its first local node (device layout)
  bool dirty = false;                // returned to the pool unreset (ready_part)
};

// Flattener parts are pooled: a new Part allocates its store's tables and
// arenas, and for a webhook micro-batch (256 AdmissionReviews on 16 parts) the
// page faults and mmap calls of those allocations serialized the parts on the
// process's memory map (0.8 ms of setup, parsing that did not scale with
// threads).  Parts come back reset, allocations kept; a batch's parts return
// to the pool only if small (a 1M-Pod page's parts hold ~1 GB).
void reset_part(Part& p) {
  p.st.reset();
  p.lo = p.hi = 0;
  p.cols.clear();
  p.nsglob.clear();
  p.weight.clear();
  p.res.clear();
  p.ns_roots.clear();
  p.count_paths = false;
  p.paths = PathTab();
  p.pcount.clear();
  p.excluded = 0;
  p.err.clear();
  p.smap.clear();
  p.nmap.clear();
  p.node_off = 0;
  p.rbeg.clear();
}
size_t part_bytes(const Part& p) {
  return p.st.bytes() + p.smap.capacity() * 4 + p.nmap.capacity() * 4 + p.cols.capacity() * sizeof(ReviewCol);
}
struct PartPool {
  std::mutex mu;
  std::map<int, std::vector<std::vector<Part>>> free;
  std::vector<std::vector<Part>> grave;  // large parts awaiting release
};
PartPool& part_pool() {
  static PartPool* p = new PartPool();
  return *p;
}
}  // namespace
void release_parts_async() {
  std::vector<std::vector<Part>> w;
  {
    PartPool& pp = part_pool();
    std::lock_guard<std::mutex> g(pp.mu);
    w.swap(pp.grave);
  }
  if (!w.empty()) std::thread([w = std::move(w)]() mutable { w.clear(); }).detach();
}
namespace {
std::vector<Part> take_parts(int T) {
  release_parts_async();  // an earlier caller's, if it did not
  {
    PartPool& pp = part_pool();
    std::lock_guard<std::mutex> g(pp.mu);
    auto it = pp.free.find(T);
    if (it != pp.free.end() && !it->second.empty()) {
      std::vector<Part> v = std::move(it->second.back());
      it->second.pop_back();
      return v;
    }
  }
  return std::vector<Part>(T);
}
// A pooled part is reset by the worker that next uses it (ready_part, first
// thing in each parallel task): resetting on return cleared 16 parts' tables
// and string caches (~160 KB each) serially on the caller's thread (~0.2 ms of
// a micro-batch).
void ready_part(Part& p) {
  if (!p.dirty) return;
  reset_part(p);
  p.dirty = false;
}
void give_parts(std::vector<Part>& v) {
  size_t bytes = 0;
  for (auto& p : v) bytes += part_bytes(p);
  if (v.empty()) return;
  if (bytes > (64u << 20)) {
    // a page's parts (~1.5 GB for 1M Pods): released off the caller's path
    // (unmapping them took ~50 ms of a staging), after its upload
    // (release_parts_async: unmapping while the upload pins pages stalled both)
    PartPool& pp = part_pool();
    std::lock_guard<std::mutex> g(pp.mu);
    pp.grave.push_back(std::move(v));
    v.clear();
    return;
  }
  for (auto& p : v) p.dirty = true;
  PartPool& pp = part_pool();
  std::lock_guard<std::mutex> g(pp.mu);
  auto& l = pp.free[(int)v.size()];
  if (l.size() < 8) l.push_back(std::move(v));
}

void run_part(Part& p, const Store& gst, const NsCache& ns_cache, const std::set<std::string>* ex, const Page& pg) {
  Store& st = p.st;
  const Keys K(st);
  std::vector<NsDoc> ns_docs(pg.n_ns);
  NsDoc empty_ns;
  const size_t n = p.hi - p.lo;
  p.cols.reserve(n);
  p.nsglob.reserve(n);
  p.weight.reserve(n);
  p.res.reserve(n);
  // about one node per 9 bytes of JSON for these documents, plus the envelopes
  st.nodes().reserve((pg.obj_offs[p.hi] - pg.obj_offs[p.lo]) / 8 + n * 20 + 1024);
  std::string err;
  auto ns_doc = [&](uint32_t k) -> NsDoc* {
    NsDoc* d = k == NO_ID || k >= pg.n_ns ? &empty_ns : &ns_docs[k];
    if (d->root != NO_ID) return d;
    const char* s = EMPTY_NS_JSON;
    size_t len = strlen(EMPTY_NS_JSON);
    if (d != &empty_ns) { s = pg.nss + pg.ns_offs[k]; len = pg.ns_offs[k + 1] - pg.ns_offs[k]; }
    Node r;
    if (!st.parse_doc(s, len, &r, &err)) { p.err = "invalid namespace JSON at " + std::to_string(k) + ": " + err; return nullptr; }
    if (const Node* md = member(st, r, st.s_metadata)) {
      uint32_t nm = member_str(st, *md, st.s_name);
      if (nm != NO_ID) { d->name = std::string(st.str(nm)); d->sid = nm; }
    }
    d->root = st.add_node(r);
    p.ns_roots.push_back(d->root);
    if (p.count_paths) {  // every review of the namespace shares these runs
      std::vector<uint32_t> q{d->root};
      for (size_t h = 0; h < q.size(); ++h) {
        Node& x = st.nodes()[q[h]];
        x.flags |= kShared;
        if (x.type == NT_OBJ || x.type == NT_ARR)
          for (uint32_t c = 0; c < x.n; ++c) q.push_back(x.first + c);
      }
    }
    return d;
  };
  // staged layout: the nodes each document path's region receives from a
  // review, counted right after the review is built (its nodes are in cache)
  std::vector<uint64_t> stack;
  auto count_paths = [&](uint32_t root) {
    const Node* ln = st.nodes().data();
    stack.clear();
    stack.push_back(root);
    while (!stack.empty()) {
      const uint64_t e = stack.back();
      stack.pop_back();
      const uint32_t path = (uint32_t)(e >> 32);
      const Node& x = ln[(uint32_t)e];
      if ((x.type != NT_OBJ && x.type != NT_ARR) || x.n == 0 || (ln[x.first].flags & kShared)) continue;
      if (path >= p.pcount.size()) p.pcount.resize(path + 64, 0);
      p.pcount[path] += x.n;
      const bool obj = x.type == NT_OBJ;
      for (uint32_t c = 0; c < x.n; ++c) {
        Node& y = st.nodes()[x.first + c];
        if ((y.type == NT_OBJ || y.type == NT_ARR) && y.n) {
          // the child's path, kept in its (unused) value field for the layout
          // pass (Remap clears it)
          y.val = p.paths.child(path, obj ? y.key : kElem);
          stack.push_back((uint64_t)(x.first + c) | ((uint64_t)y.val << 32));
        }
      }
    }
  };
  for (size_t i = p.lo; i < p.hi; ++i) {
    size_t n0 = st.nodes().size();
    p.rbeg.push_back((uint32_t)n0);
    Node obj;
    if (!st.parse_doc(pg.objs + pg.obj_offs[i], pg.obj_offs[i + 1] - pg.obj_offs[i], &obj, &err)) {
      p.err = "invalid object JSON at " + std::to_string(i) + ": " + err;
      return;
    }
    if (pg.cache) {
      ResourceIds rid{};
      const uint32_t root = build_cache_review(st, K, obj, pg.cache[i], &rid);
      bool glob = false;
      p.cols.push_back(review_columns(st, gst, ns_cache, root, &glob));
      p.cols.back().flags |= RC_AUDIT;
      p.nsglob.push_back(glob);
      p.res.push_back(rid);
      if (p.count_paths) count_paths(root);
      uint32_t elems = 0;
      const Node* nv = st.nodes().data();
      const size_t n1 = st.nodes().size();
      for (size_t k = n0; k < n1; ++k)
        if (nv[k].type == NT_ARR) elems += nv[k].n;
      p.weight.push_back((std::min<uint32_t>(elems, 0xfff) << 20) | std::min<uint32_t>((uint32_t)(n1 - n0), 0xfffff));
      continue;
    }
    if (ex && !ex->empty()) {
      uint32_t ons = NO_ID;
      if (const Node* md = member(st, obj, st.s_metadata)) ons = member_str(st, *md, st.s_namespace);
      if (ex->count(ons == NO_ID ? std::string() : std::string(st.str(ons)))) {
        st.nodes().resize(n0);  // drop the object's nodes
        ReviewCol rc{};
        rc.root = NO_ID;
        rc.group = rc.kind = rc.ns = rc.nsname = rc.labels = rc.old_labels = rc.ns_labels = NO_ID;
        rc.orig = NO_ID;
        rc.flags = RC_EXCLUDED;  // no RC_REVIEW_DEF: the match stage skips it
        p.cols.push_back(rc);
        p.nsglob.push_back(0);
        p.weight.push_back(0);
        p.res.push_back(ResourceIds{st.s_empty, st.s_empty, st.s_empty, st.s_empty});
        ++p.excluded;
        continue;
      }
    }
    NsDoc* ns = ns_doc(pg.obj_ns ? pg.obj_ns[i] : NO_ID);
    if (!ns) return;
    ResourceIds rid{};
    uint32_t root = build_object_review(st, K, obj, *ns, &rid);
    bool glob = false;
    p.cols.push_back(review_columns(st, gst, ns_cache, root, &glob));
    p.nsglob.push_back(glob);
    p.res.push_back(rid);
    if (p.count_paths) count_paths(root);
    // size key: array elements (what templates iterate: containers, ports,
    // volumes ...) first, then document nodes
    uint32_t elems = 0;
    const Node* nv = st.nodes().data();
    const size_t n1 = st.nodes().size();
    for (size_t k = n0; k < n1; ++k)
      if (nv[k].type == NT_ARR) elems += nv[k].n;
    uint32_t nn = (uint32_t)(n1 - n0);
    p.weight.push_back((std::min<uint32_t>(elems, 0xfff) << 20) | std::min<uint32_t>(nn, 0xfffff));
  }
}

struct Remap {
  const std::vector<uint32_t>& smap;
  const std::vector<uint32_t>& nmap;
  // a local node's scalar fields in global ids (key: by its parent's type)
  Node operator()(Node y, bool obj_member) const {
    if (obj_member) y.key = smap[y.key];
    if (y.type == NT_STR) y.val = smap[y.val];
    else if (y.type == NT_NUM) y.val = nmap[y.val];
    else if (y.type == NT_OBJ || y.type == NT_ARR) y.val = 0;  // the layout's path id (count_paths)
    y.flags &= (uint8_t)~kShared;
    return y;
  }
};

// Phase 3 of a staged page in the path-grouped layout (flatten.h).  Phase 2
// (string / number interning) is done, and every part counted the nodes each
// of its paths' regions receives (run_part).  Parts are ordered and placed
// independently (the evaluation order is part-major: each part's reviews in
// their own order, so a wavefront straddles two parts at most at the
// boundaries), which keeps every pass over a part's arena on its own thread:
//   1. columns with global string ids, then each part's evaluation order;
//   2. the Namespace documents, placed once after the review roots;
//   3. the parts' paths -> global paths; region g holds part 0's nodes at g,
//      then part 1's, ...;
//   4. per part, its reviews' nodes in its evaluation order at its cursors.
static bool layout_parts(std::vector<Part>& parts, uint32_t base, NodeArena& dst, FlatResult& out, size_t n,
                         std::string& err, const OrderFn& order, std::vector<uint32_t>& perm,
                         std::chrono::steady_clock::time_point t1) {
  using Clock = std::chrono::steady_clock;
  auto ms = [](Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  const int T = (int)parts.size();
  auto pfor = [&](const std::function<void(int)>& f) { parallel_run(T, f); };
  // 1.
  out.cols.resize(n);
  out.weight.resize(n);
  out.resources.resize(n);
  pfor([&](int t) {
    Part& p = parts[t];
    auto str = [&](uint32_t s) { return s == NO_ID ? NO_ID : p.smap[s]; };
    for (size_t i = 0; i < p.cols.size(); ++i) {
      ReviewCol rc = p.cols[i];
      rc.group = str(rc.group);
      rc.kind = str(rc.kind);
      rc.ns = str(rc.ns);
      rc.nsname = str(rc.nsname);
      out.cols[p.lo + i] = rc;
      out.weight[p.lo + i] = p.weight[i];
      const ResourceIds& r = p.res[i];
      out.resources[p.lo + i] = ResourceIds{str(r.api_version), str(r.kind), str(r.name), str(r.ns)};
    }
  });
  auto t2 = Clock::now();
  std::vector<std::vector<uint32_t>> porder(T);
  std::vector<uint64_t> nlive_of(T, 0);
  pfor([&](int t) {
    Part& p = parts[t];
    order(out, p.lo, p.hi, porder[t]);
    for (uint32_t i : porder[t]) nlive_of[t] += out.cols[i].root != NO_ID;
  });
  perm.clear();
  perm.reserve(n);
  for (int t = 0; t < T; ++t) {
    if (porder[t].size() != parts[t].hi - parts[t].lo) { err = "review order: bad permutation"; return false; }
    perm.insert(perm.end(), porder[t].begin(), porder[t].end());
  }
  std::vector<uint64_t> root_at(T, 0);  // the part's first root position
  uint64_t nlive = 0;
  for (int t = 0; t < T; ++t) { root_at[t] = nlive; nlive += nlive_of[t]; }
  auto t3 = Clock::now();
  // 2.
  std::vector<std::unordered_map<uint32_t, uint32_t>> nsmap(T);
  uint64_t at_ns = nlive;
  std::vector<std::pair<uint32_t, uint64_t>> q;  // (local id, position)
  std::vector<Node> nsnodes;
  for (int t = 0; t < T; ++t) {
    Part& p = parts[t];
    const Node* ln = p.st.nodes().data();
    const Remap rm{p.smap, p.nmap};
    for (uint32_t r : p.ns_roots) {
      q.clear();
      q.push_back({r, at_ns});
      nsmap[t][r] = (uint32_t)(base + at_ns);
      nsnodes.push_back(rm(ln[r], false));
      ++at_ns;
      for (size_t h = 0; h < q.size(); ++h) {
        const auto [l, at] = q[h];
        const Node& x = ln[l];
        if ((x.type != NT_OBJ && x.type != NT_ARR) || x.n == 0) continue;
        nsnodes[at - nlive].first = (uint32_t)(base + at_ns);
        for (uint32_t c = 0; c < x.n; ++c) {
          const uint32_t lc = x.first + c;
          nsmap[t][lc] = (uint32_t)(base + at_ns);
          nsnodes.push_back(rm(ln[lc], x.type == NT_OBJ));
          q.push_back({lc, at_ns});
          ++at_ns;
        }
      }
    }
  }
  // 3. global paths (a part's paths are numbered parent first)
  std::unordered_map<uint64_t, uint32_t> gm;
  std::vector<std::vector<uint32_t>> g_of(T);
  uint32_t G = 1;
  for (int t = 0; t < T; ++t) {
    const PathTab& pt = parts[t].paths;
    g_of[t].assign(pt.def.size(), 0);
    for (uint32_t l = 1; l < pt.def.size(); ++l) {
      const uint32_t key = pt.def[l].second == kElem ? kElem : parts[t].smap[pt.def[l].second];
      const uint64_t k = ((uint64_t)g_of[t][pt.def[l].first] << 32) | key;
      auto it = gm.find(k);
      if (it == gm.end()) it = gm.emplace(k, G++).first;
      g_of[t][l] = it->second;
    }
  }
  std::vector<std::vector<uint64_t>> pg(G, std::vector<uint64_t>(T, 0));  // nodes of part t at path g
  for (int t = 0; t < T; ++t) {
    const Part& p = parts[t];
    for (uint32_t l = 0; l < p.pcount.size(); ++l)
      if (p.pcount[l]) pg[g_of[t][l]][t] += p.pcount[l];
  }
  uint64_t total = at_ns;
  for (uint32_t g = 0; g < G; ++g)
    for (int t = 0; t < T; ++t) {
      const uint64_t v = pg[g][t];
      pg[g][t] = base + total;  // part t's first node in region g
      total += v;
    }
  if ((uint64_t)base + total >= NO_ID) { err = "node arena exceeds 2^32 nodes"; return false; }
  auto t4 = Clock::now();
  dst.resize(total);
  Node* dn = dst.data();
  if (!nsnodes.empty()) memcpy(dn + nlive, nsnodes.data(), nsnodes.size() * sizeof(Node));
  // 4.
  std::vector<std::string> perr(T);
  auto place_part = [&](int t) {
    Part& p = parts[t];
    const Node* ln = p.st.nodes().data();
    const Remap rm{p.smap, p.nmap};
    std::vector<uint64_t> cur(p.paths.def.size(), 0), stack;
    for (uint32_t l = 0; l < cur.size(); ++l) cur[l] = pg[g_of[t][l]][t];
    uint64_t k = root_at[t];
    for (uint32_t i : porder[t]) {
      const size_t j = i - p.lo;
      const ReviewCol& lc = p.cols[j];
      if (lc.root == NO_ID) continue;
      const uint32_t nroot = (uint32_t)(base + k);
      dn[k] = rm(ln[lc.root], false);
      dn[k].key = 0;
      ++k;
      uint32_t lb = NO_ID, old = NO_ID;
      // depth first; stack entries: local id | path << 32, then the new id
      stack.clear();
      stack.push_back(lc.root);
      stack.push_back(nroot);
      while (!stack.empty()) {
        const uint32_t nid = (uint32_t)stack.back();
        stack.pop_back();
        const uint64_t e = stack.back();
        stack.pop_back();
        const uint32_t path = (uint32_t)(e >> 32);
        const Node& x = ln[(uint32_t)e];
        if ((x.type != NT_OBJ && x.type != NT_ARR) || x.n == 0) continue;
        if (ln[x.first].flags & kShared) {  // a Namespace document's members: placed once, shared
          auto it = nsmap[t].find(x.first);
          if (it == nsmap[t].end()) { perr[t] = "path layout: unplaced shared run"; return; }
          dn[nid - base].first = it->second;
          continue;
        }
        const bool obj = x.type == NT_OBJ;
        const uint64_t start = cur[path];
        cur[path] += x.n;
        dn[nid - base].first = (uint32_t)start;
        Node* out_run = dn + (start - base);
        for (uint32_t c = 0; c < x.n; ++c) {
          const uint32_t l = x.first + c;
          const Node& y = ln[l];
          out_run[c] = rm(y, obj);
          if (l == lc.labels) lb = (uint32_t)(start + c);
          if (l == lc.old_labels) old = (uint32_t)(start + c);
          if ((y.type == NT_OBJ || y.type == NT_ARR) && y.n) {
            stack.push_back((uint64_t)l | ((uint64_t)y.val << 32));  // its path (count_paths)
            stack.push_back(start + c);
          }
        }
      }
      ReviewCol& rc = out.cols[i];
      rc.root = nroot;
      rc.labels = lc.labels == NO_ID ? NO_ID : lb;
      rc.old_labels = lc.old_labels == NO_ID ? NO_ID : old;
      if ((lc.labels != NO_ID && lb == NO_ID) || (lc.old_labels != NO_ID && old == NO_ID)) {
        perr[t] = "path layout: a label node was not placed";
        return;
      }
      if (!p.nsglob[j] && lc.ns_labels != NO_ID) {
        auto it = nsmap[t].find(lc.ns_labels);
        if (it == nsmap[t].end()) { perr[t] = "path layout: namespace labels outside the Namespace document"; return; }
        rc.ns_labels = it->second;
      }
    }
    // every cursor advanced by exactly the count run_part made
    for (uint32_t l = 0; l < cur.size(); ++l)
      if (cur[l] - pg[g_of[t][l]][t] != (l < p.pcount.size() ? p.pcount[l] : 0)) {
        perr[t] = "path layout: region count mismatch";
        return;
      }
  };
  if (getenv("GKGPU_PLACE_TWICE")) {  // diagnostics: the placement once more into touched memory
    auto ta = Clock::now();
    pfor(place_part);
    fprintf(stderr, "flatten: place (first touch) %.1f ms\n", ms(ta, Clock::now()));
  }
  pfor(place_part);
  for (auto& e : perr)
    if (!e.empty()) { err = e; return false; }
  out.excluded = 0;
  for (auto& p : parts) out.excluded += p.excluded;
  out.node_count = total;
  out.paths = G;
  auto t5 = Clock::now();
  out.ms_layout = ms(t3, t5);
  out.ms_merge = ms(t1, t5);
  if (getenv("GKGPU_FLATTEN_TRACE"))
    fprintf(stderr, "flatten: intern+columns %.1f ms, order %.1f ms, path layout: regions %.1f + place %.1f ms (%u paths, %llu nodes)\n",
            ms(t1, t2), ms(t2, t3), ms(t3, t4), ms(t4, t5), G, (unsigned long long)total);
  return true;
}

}  // namespace

// Phase 3 for the device layout (flatten.h DevLayout, layout.hip): the parts'
// nodes relocated into one per-document arena D (as without a layout), every
// container's `val` its global document path (kSharedPath for the shared
// Namespace runs), plus what the device pass needs per review: where its
// document starts in D, its evaluation position and its root's slot.
static bool relocate_for_device(std::vector<Part>& parts, uint32_t base, NodeArena& dst, FlatResult& out, size_t n,
                                std::string& err, const OrderFn& order, std::vector<uint32_t>& perm, DevLayout& dl) {
  using Clock = std::chrono::steady_clock;
  auto ms_between = [](Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  const auto t0 = Clock::now();
  const int T = (int)parts.size();
  auto pfor = [&](const std::function<void(int)>& f) { parallel_run(T, f); };
  // columns with global string ids (node ids below), each part's evaluation order
  out.cols.resize(n);
  out.weight.resize(n);
  out.resources.resize(n);
  pfor([&](int t) {
    Part& p = parts[t];
    auto str = [&](uint32_t s) { return s == NO_ID ? NO_ID : p.smap[s]; };
    for (size_t i = 0; i < p.cols.size(); ++i) {
      ReviewCol rc = p.cols[i];
      rc.group = str(rc.group);
      rc.kind = str(rc.kind);
      rc.ns = str(rc.ns);
      rc.nsname = str(rc.nsname);
      out.cols[p.lo + i] = rc;
      out.weight[p.lo + i] = p.weight[i];
      const ResourceIds& r = p.res[i];
      out.resources[p.lo + i] = ResourceIds{str(r.api_version), str(r.kind), str(r.name), str(r.ns)};
    }
  });
  const auto t_cols = Clock::now();
  std::vector<std::vector<uint32_t>> porder(T);
  pfor([&](int t) { order(out, parts[t].lo, parts[t].hi, porder[t]); });
  perm.clear();
  perm.reserve(n);
  for (int t = 0; t < T; ++t) {
    if (porder[t].size() != parts[t].hi - parts[t].lo) { err = "review order: bad permutation"; return false; }
    perm.insert(perm.end(), porder[t].begin(), porder[t].end());
  }
  // global paths (a part's paths are numbered parent first)
  std::unordered_map<uint64_t, uint32_t> gm;
  std::vector<std::vector<uint32_t>> g_of(T);
  uint32_t G = 1;
  for (int t = 0; t < T; ++t) {
    const PathTab& pt = parts[t].paths;
    g_of[t].assign(pt.def.size(), 0);
    for (uint32_t l = 1; l < pt.def.size(); ++l) {
      const uint32_t key = pt.def[l].second == kElem ? kElem : parts[t].smap[pt.def[l].second];
      const uint64_t k = ((uint64_t)g_of[t][pt.def[l].first] << 32) | key;
      auto it = gm.find(k);
      if (it == gm.end()) it = gm.emplace(k, G++).first;
      g_of[t][l] = it->second;
    }
  }
  uint64_t total = 0;
  for (auto& p : parts) {
    p.node_off = total;
    total += p.st.nodes().size() - kFixedNodes;
  }
  if ((uint64_t)base + total >= NO_ID) { err = "node arena exceeds 2^32 nodes"; return false; }
  const auto t_ord = Clock::now();
  dst.resize(total);
  dl.beg.assign(n, 0);
  Node* dn = dst.data();
  pfor([&](int t) {
    Part& p = parts[t];
    const auto& ln = p.st.nodes();
    const uint32_t goff = base + (uint32_t)p.node_off - kFixedNodes;
    Node* d = dn + p.node_off - kFixedNodes;
    auto node = [&](uint32_t x) { return x == NO_ID ? NO_ID : (x < kFixedNodes ? x : x + goff); };
    const std::vector<uint32_t>& gp = g_of[t];
    for (size_t k = kFixedNodes; k < ln.size(); ++k) {
      Node x = ln[k];
      if (x.type == NT_STR) x.val = p.smap[x.val];
      else if (x.type == NT_NUM) x.val = p.nmap[x.val];
      else if (x.type == NT_ARR || x.type == NT_OBJ) {
        if (x.flags & kShared) x.val = DevLayout::kSharedPath;
        else x.val = x.n && x.val < gp.size() ? gp[x.val] : 0;
        if (x.n) x.first += goff;
      }
      d[k] = x;  // kShared stays: the device pass reads and clears it
    }
    for (size_t k = kFixedNodes; k < ln.size(); ++k) {
      const Node& x = ln[k];
      if (x.type != NT_OBJ) continue;
      for (uint32_t c = 0; c < x.n; ++c) d[x.first + c].key = p.smap[ln[x.first + c].key];
    }
    for (size_t i = 0; i < p.cols.size(); ++i) {
      ReviewCol& rc = out.cols[p.lo + i];
      rc.root = node(p.cols[i].root);
      rc.labels = node(p.cols[i].labels);
      rc.old_labels = node(p.cols[i].old_labels);
      if (!p.nsglob[i]) rc.ns_labels = node(p.cols[i].ns_labels);
      dl.beg[p.lo + i] = (uint32_t)(p.node_off + (i < p.rbeg.size() ? p.rbeg[i] : ln.size()) - kFixedNodes);
    }
  });
  const auto t_rel = Clock::now();
  dl.evalpos.assign(n, 0);
  dl.slot.assign(n, NO_ID);
  dl.root_d.assign(n, NO_ID);
  // evaluation positions and root slots (live roots numbered in evaluation
  // order): a count per chunk of perm, a prefix, then the chunks in parallel
  {
    const size_t np = perm.size();
    const int C = (int)std::max<size_t>(1, std::min<size_t>((size_t)T * 4, np / 16384));
    std::vector<uint32_t> live_in(C + 1, 0);
    parallel_run(C, [&](int c) {
      uint32_t m = 0;
      for (size_t k = np * c / C; k < np * (c + 1) / C; ++k) m += out.cols[perm[k]].root != NO_ID;
      live_in[c + 1] = m;
    });
    for (int c = 0; c < C; ++c) live_in[c + 1] += live_in[c];
    parallel_run(C, [&](int c) {
      uint32_t live = live_in[c];
      for (size_t k = np * c / C; k < np * (c + 1) / C; ++k) {
        const uint32_t b = perm[k];
        dl.evalpos[b] = (uint32_t)k;
        dl.root_d[b] = out.cols[b].root;
        if (out.cols[b].root != NO_ID) dl.slot[b] = live++;
      }
    });
    dl.nroots = live_in[C];
  }
  out.excluded = 0;
  for (auto& p : parts) out.excluded += p.excluded;
  out.node_count = total;
  out.paths = G;
  if (getenv("GKGPU_FLATTEN_TRACE"))
    fprintf(stderr, "flatten: device form: columns %.1f ms, order %.1f ms, relocate %.1f ms, layout inputs %.1f ms\n",
            ms_between(t0, t_cols), ms_between(t_cols, t_ord), ms_between(t_ord, t_rel), ms_between(t_rel, Clock::now()));
  return true;
}

// Phases 2 and 3 of every flattening: the parts' strings and numbers are
// interned into the engine store (under `smu`: concurrent evaluations intern
// into the one table), then each part's nodes are copied into `dst` -- node id
// base + k lives at dst[k] -- with string / number ids and child indices
// rewritten, and its columns relocated.
static bool merge_parts(Store& gst, std::mutex& smu, std::vector<Part>& parts, uint32_t base, NodeArena& dst,
                        FlatResult& out, size_t n, std::string& err, const OrderFn* order = nullptr,
                        std::vector<uint32_t>* perm = nullptr, DevLayout* dl = nullptr) {
  using Clock = std::chrono::steady_clock;
  auto t1 = Clock::now();
  const int T = (int)parts.size();
  static const uint32_t nwell = Store().nstrings();  // well-known ids shared by every Store
  size_t extra = 0;
  for (auto& p : parts) extra += p.st.nstrings() - nwell;
  {
    std::lock_guard<std::mutex> g(smu);
    std::vector<const Store*> src;
    for (auto& p : parts) src.push_back(&p.st);
    std::vector<std::vector<uint32_t>> maps;
    // (a micro-batch's few thousand strings: parallel lookups, serial inserts)
    gst.intern_parts(src, nwell, maps, T);
    for (size_t k = 0; k < parts.size(); ++k) parts[k].smap.swap(maps[k]);
    for (auto& p : parts) {
      const Store& ls = p.st;
      const auto& nums = ls.numbers();
      p.nmap.resize(nums.size());
      for (uint32_t k = 0; k < nums.size(); ++k) {
        std::string_view v = ls.str(nums[k].text);
        p.nmap[k] = gst.number(v.data(), v.size());
      }
    }
  }
  auto t15 = Clock::now();
  if (getenv("GKGPU_FLATTEN_TRACE"))
    fprintf(stderr, "flatten: intern %.1f ms (%zu strings)\n", std::chrono::duration<double, std::milli>(t15 - t1).count(),
            extra);
  if (order && dl) return relocate_for_device(parts, base, dst, out, n, err, *order, *perm, *dl);
  if (order) return layout_parts(parts, base, dst, out, n, err, *order, *perm, t1);
  uint64_t total = 0;
  for (auto& p : parts) {
    p.node_off = total;  // position in dst
    total += p.st.nodes().size() - kFixedNodes;
  }
  if ((uint64_t)base + total >= NO_ID) { err = "node arena exceeds 2^32 nodes"; return false; }
  dst.resize(total);
  out.cols.resize(n);
  out.weight.resize(n);
  out.resources.resize(n);
  {
    Node* dn = dst.data();
    auto relocate = [&](Part& p) {
      const auto& ln = p.st.nodes();
      // local node k >= kFixedNodes -> global base + node_off + k - kFixedNodes;
      // the fixed nodes ({} null false true) are global 0..3 in every store
      const uint32_t goff = base + (uint32_t)p.node_off - kFixedNodes;
      Node* d = dn + p.node_off - kFixedNodes;  // d[k] = dst slot of local node k
      auto node = [&](uint32_t x) { return x == NO_ID ? NO_ID : (x < kFixedNodes ? x : x + goff); };
      auto str = [&](uint32_t s) { return s == NO_ID ? NO_ID : p.smap[s]; };
      for (size_t k = kFixedNodes; k < ln.size(); ++k) {
        Node x = ln[k];
        if (x.type == NT_STR) x.val = p.smap[x.val];
        else if (x.type == NT_NUM) x.val = p.nmap[x.val];
        else if ((x.type == NT_ARR || x.type == NT_OBJ) && x.n) x.first += goff;
        d[k] = x;
      }
      // object member keys: rewrite in the copied arena (a child is copied
      // before or after its parent; keys are only meaningful under objects)
      for (size_t k = kFixedNodes; k < ln.size(); ++k) {
        const Node& x = ln[k];
        if (x.type != NT_OBJ) continue;
        for (uint32_t c = 0; c < x.n; ++c) d[x.first + c].key = p.smap[ln[x.first + c].key];
      }
      for (size_t i = 0; i < p.cols.size(); ++i) {
        ReviewCol rc = p.cols[i];
        rc.root = node(rc.root);
        rc.group = str(rc.group);
        rc.kind = str(rc.kind);
        rc.ns = str(rc.ns);
        rc.nsname = str(rc.nsname);
        rc.labels = node(rc.labels);
        rc.old_labels = node(rc.old_labels);
        if (!p.nsglob[i]) rc.ns_labels = node(rc.ns_labels);
        out.cols[p.lo + i] = rc;
        out.weight[p.lo + i] = p.weight[i];
        const ResourceIds& r = p.res[i];
        out.resources[p.lo + i] = ResourceIds{str(r.api_version), str(r.kind), str(r.name), str(r.ns)};
      }
    };
    parallel_run(T, [&](int t) { relocate(parts[t]); });
  }
  if (getenv("GKGPU_FLATTEN_TRACE"))
    fprintf(stderr, "flatten: relocate %.1f ms\n", std::chrono::duration<double, std::milli>(Clock::now() - t15).count());
  out.excluded = 0;
  for (auto& p : parts) out.excluded += p.excluded;
  out.node_count = total;
  out.ms_merge = std::chrono::duration<double, std::milli>(Clock::now() - t1).count();
  return true;
}

bool flatten_page(Store& gst, std::mutex& smu, const NsCache& ns_cache, const std::set<std::string>* excluded,
                  const Page& pg, int threads, uint32_t base, NodeArena& dst, FlatResult& out, std::string& err,
                  const OrderFn* order, std::vector<uint32_t>* perm, DevLayout* dl) {
  using Clock = std::chrono::steady_clock;
  auto t0 = Clock::now();
  const size_t n = pg.n;
  int T = std::max(1, threads);
  // at least ~2k objects per thread: below that the merge costs more than it saves
  T = (int)std::min<size_t>((size_t)T, std::max<size_t>(1, n / 2048));
  std::vector<Part> parts = take_parts(T);
  struct Give { std::vector<Part>& v; ~Give() { give_parts(v); } } give{parts};
  parallel_run(T, [&](int t) {
    Part& p = parts[t];
    ready_part(p);
    p.lo = n * t / T;
    p.hi = n * (t + 1) / T;
    p.count_paths = order != nullptr;
    run_part(p, gst, ns_cache, excluded, pg);
  });
  for (auto& p : parts)
    if (!p.err.empty()) { err = p.err; return false; }
  out.ms_parse = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
  if (getenv("GKGPU_FLATTEN_TRACE")) fprintf(stderr, "flatten: parse %.1f ms\n", out.ms_parse);
  if (order && !perm) { err = "flatten_page: order without perm"; return false; }
  return merge_parts(gst, smu, parts, base, dst, out, n, err, order, perm, dl);
}

bool flatten_docs(Store& gst, std::mutex& smu, const std::vector<std::string_view>& docs, uint32_t base, NodeArena& dst,
                  std::vector<uint32_t>& roots, std::string& err) {
  const size_t n = docs.size();
  const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)default_threads(), n / 2048));
  std::vector<Part> parts = take_parts(T);
  struct Give { std::vector<Part>& v; ~Give() { give_parts(v); } } give{parts};
  parallel_run(T, [&](int t) {
    Part& p = parts[t];
    ready_part(p);
    p.lo = n * t / T;
    p.hi = n * (t + 1) / T;
    std::string perr;
    for (size_t i = p.lo; i < p.hi; ++i) {
      Node r;
      if (!p.st.parse_doc(docs[i].data(), docs[i].size(), &r, &perr)) {
        p.err = "invalid JSON at " + std::to_string(i) + ": " + perr;
        return;
      }
      p.rbeg.push_back(p.st.add_node(r));  // (the part-local id of the placed root)
    }
  });
  for (auto& p : parts)
    if (!p.err.empty()) { err = p.err; return false; }
  FlatResult out;
  if (!merge_parts(gst, smu, parts, base, dst, out, 0, err)) return false;
  roots.resize(n);
  for (auto& p : parts)
    for (size_t i = p.lo; i < p.hi; ++i) roots[i] = base + (uint32_t)p.node_off + p.rbeg[i - p.lo] - kFixedNodes;
  return true;
}

bool flatten_reviews(Store& gst, std::mutex& smu, const NsCache& ns_cache,
                     const std::vector<std::pair<const char*, size_t>>& inputs, uint32_t base, NodeArena& dst,
                     std::vector<ReviewCol>& cols, std::string& err) {
  // parts of >= 16 inputs on the worker pool (a webhook micro-batch of 256
  // AdmissionReviews: 16 parts); the first input that is not JSON fails the call
  const size_t n = inputs.size();
  const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)default_threads(), n / 16));
  using Clock = std::chrono::steady_clock;
  const auto t0 = Clock::now();
  std::vector<Part> parts = take_parts(T);
  struct Give { std::vector<Part>& v; ~Give() { give_parts(v); } } give{parts};
  const auto t1 = Clock::now();
  std::vector<double> pt0(T), pt1(T);
  parallel_run(T, [&](int t) {
    Part& p = parts[t];
    pt0[t] = std::chrono::duration<double, std::milli>(Clock::now() - t1).count();
    ready_part(p);
    p.lo = n * t / T;
    p.hi = n * (t + 1) / T;
    struct Stamp { double& x; Clock::time_point b; ~Stamp() { x = std::chrono::duration<double, std::milli>(Clock::now() - b).count(); } } stamp{pt1[t], t1};
    std::string perr;
    for (size_t i = p.lo; i < p.hi; ++i) {
      // the input document straight into the part's arena; input.review is
      // its "review" member (encoding/json: the last of duplicate keys)
      Node top;
      if (!p.st.parse_doc(inputs[i].first, inputs[i].second, &top, &perr)) {
        p.err = "invalid input JSON: " + perr;
        return;
      }
      const Node* rvn = member(p.st, top, p.st.s_review);
      const uint32_t rn = rvn ? (uint32_t)(rvn - p.st.nodes().data()) : NO_ID;
      bool glob = false;
      p.cols.push_back(review_columns(p.st, gst, ns_cache, rn, &glob));
      p.nsglob.push_back(glob);
      p.weight.push_back(0);
      p.res.push_back(ResourceIds{p.st.s_empty, p.st.s_empty, p.st.s_empty, p.st.s_empty});
    }
  });
  for (auto& p : parts)
    if (!p.err.empty()) { err = p.err; return false; }
  const auto t2 = Clock::now();
  FlatResult out;
  if (!merge_parts(gst, smu, parts, base, dst, out, n, err)) return false;
  cols.swap(out.cols);
  if (getenv("GKGPU_FLATTEN_TRACE") && atoi(getenv("GKGPU_FLATTEN_TRACE")) > 1)
    for (int t = 0; t < T; ++t) fprintf(stderr, "  part %d: %.3f .. %.3f ms\n", t, pt0[t], pt1[t]);
  if (getenv("GKGPU_FLATTEN_TRACE"))
    fprintf(stderr, "flatten_reviews: %d parts: setup %.3f ms, parse %.3f ms, merge %.3f ms\n", T,
            std::chrono::duration<double, std::milli>(t1 - t0).count(), std::chrono::duration<double, std::milli>(t2 - t1).count(),
            std::chrono::duration<double, std::milli>(Clock::now() - t2).count());
  return true;
}

}  // namespace gk

namespace gk {

// Content hash of a document (type, keys, string / number text, structure),
// independent of node and string ids: compares flattenings across thread counts.
uint64_t doc_hash(const Store& st, const Node* nodes, uint32_t node) {
  if (node == NO_ID) return 0x9e3779b97f4a7c15ull;
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](uint64_t x) { h ^= x + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2); };
  auto mixs = [&](uint32_t sid) { std::string_view v = st.str(sid); mix(fnv1a(v.data(), v.size())); };
  std::vector<std::pair<uint32_t, bool>> stack{{node, false}};
  while (!stack.empty()) {
    auto [k, obj_child] = stack.back();
    stack.pop_back();
    const Node& x = nodes[k];
    mix(x.type);
    if (obj_child) mixs(x.key);
    if (x.type == NT_STR) mixs(x.val);
    else if (x.type == NT_NUM) mixs(st.numbers()[x.val].text);
    else if (x.type == NT_ARR || x.type == NT_OBJ) {
      mix(x.n);
      for (uint32_t c = x.n; c-- > 0;) stack.push_back({x.first + c, x.type == NT_OBJ});
    }
  }
  return h;
}

}  // namespace gk
