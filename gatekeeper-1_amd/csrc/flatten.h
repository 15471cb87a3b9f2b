// Host flattener: Kubernetes objects (JSON text) -> review documents in the
// interned node arena + per-review match columns, on many host threads.
//
// Replaces the per-object JSON round trips of the reference audit loop
// (pkg/target/target.go:129-163 json.Marshal into AdmissionRequest.Object,
// drivers/local/local.go:331 MarshalIndent, rego.go:1478-1496 RoundTrip +
// InterfaceToValue) with one parse per object into a layout the kernels read.
#pragma once
#include <stdint.h>

#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <string_view>
#include <vector>

#include "common.h"
#include "json.h"
#include "store.h"

namespace gk {

// ------------------------------------------------------------------ node helpers (host)
inline uint32_t nget(const Store& st, uint32_t node, uint32_t key) {
  if (node == NO_ID) return NO_ID;
  const Node& n = st.nodes()[node];
  if (n.type != NT_OBJ) return NO_ID;
  for (uint32_t i = 0; i < n.n; ++i) if (st.nodes()[n.first + i].key == key) return n.first + i;
  return NO_ID;
}
inline uint32_t nget(const Store& st, uint32_t node, const char* key) {
  uint32_t k = st.find(key, strlen(key));
  return k == NO_ID ? NO_ID : nget(st, node, k);
}
inline uint8_t ntype(const Store& st, uint32_t n) { return n == NO_ID ? NT_NONE : st.nodes()[n].type; }
inline bool nstr(const Store& st, uint32_t n, uint32_t* sid) {
  if (n == NO_ID || st.nodes()[n].type != NT_STR) return false;
  *sid = st.nodes()[n].val;
  return true;
}
inline bool is_empty_obj(const Store& st, uint32_t n) { return n != NO_ID && st.nodes()[n].type == NT_OBJ && st.nodes()[n].n == 0; }
// get_default (target_template_source.go:110-125): missing / null -> default (NO_ID == {})
inline uint32_t gdef(const Store& st, uint32_t obj, const char* key) {
  uint32_t v = nget(st, obj, key);
  if (v == NO_ID || st.nodes()[v].type == NT_NULL) return NO_ID;
  return v;
}

// The synced Namespace cache data.external[target].cluster.v1.Namespace
// (node ids in the engine's global store).
using NsCache = std::map<std::string, uint32_t>;

// Match columns of a review document rooted at `root` in `st`
// (target_template_source.go:131-386 inputs).  Cached namespaces are nodes of
// `gst` (the engine's store); *ns_labels_global reports that rc.ns_labels
// refers to one of them rather than to a node of `st`.
ReviewCol review_columns(const Store& st, const Store& gst, const NsCache& ns_cache, uint32_t root,
                         bool* ns_labels_global);

// One page of audit objects: concatenated JSON texts and, per object, the
// index of its Namespace object (nsCache.Get, pkg/audit/manager.go:96-115;
// NO_ID = cluster-scoped, reviewed with an empty corev1.Namespace{}).
struct Page {
  const char* objs = nullptr;
  const uint64_t* obj_offs = nullptr;  // n + 1 offsets
  size_t n = 0;
  const char* nss = nullptr;
  const uint64_t* ns_offs = nullptr;   // n_ns + 1 offsets
  size_t n_ns = 0;
  const uint32_t* obj_ns = nullptr;    // per object: namespace index or NO_ID
  // From-cache reviews (hooks.audit over the synced inventory,
  // target_template_source.go:46-89): per object, the fields of its inventory
  // path; each review is then make_review / add_field's document instead of
  // the audit envelope, and no namespace is excluded or attached.
  struct CacheKey {
    std::string_view group, version, kind, name, ns;
    bool namespaced;
  };
  const CacheKey* cache = nullptr;
};

// HandleViolation's Resource identity of a review (pkg/target/target.go:193-244):
// apiVersion from review.kind {group, version}, kind = review.kind.kind, and
// the object's metadata name / namespace (unstructured GetName/GetNamespace).
struct ResourceIds {
  uint32_t api_version, kind, name, ns;  // global string ids
};

struct FlatResult {
  std::vector<ReviewCol> cols;        // batch order (orig = NO_ID)
  std::vector<uint32_t> weight;       // size key per review: array elements << 20 | nodes
  std::vector<ResourceIds> resources; // per review (batch order)
  uint64_t excluded = 0;              // reviews skipped by the process excluder
  uint64_t node_count = 0;
  uint32_t paths = 0;                 // path-grouped layout: document paths (regions) laid out
  double ms_parse = 0, ms_merge = 0, ms_layout = 0;
};

// Evaluation order of the reviews [lo, hi) of a flattened page, computed from
// its columns (string ids global, node ids not yet final) and size keys:
// perm[k] = the batch index of the review of the range evaluated k-th.  Given
// to flatten_page, it selects the path-grouped node layout below.
using OrderFn = std::function<void(const FlatResult&, size_t lo, size_t hi, std::vector<uint32_t>& perm)>;

// Flattens a page on `threads` host threads.  The review documents go to `dst`
// (node id base + k at dst[k]; ids below base are the engine store's
// permanent nodes); their strings and numbers are interned into `st` under
// `smu`.  Objects whose metadata.namespace is in `excluded_ns`
// (Excluder.IsNamespaceExcluded(Audit, ns), manager.go:362-365) get a column
// flagged RC_EXCLUDED and no document.  Returns false with `err` on malformed
// JSON.
//
// Without `order`, each document's nodes are contiguous (BFS per document, in
// batch order).  With `order` (staged batches), the nodes are laid out
// **path-grouped** in evaluation order (`perm`: part-major, each host
// thread's range of the page in the order `order` gives it):
//   [review roots, in evaluation order]
//   [Namespace documents (shared by the reviews of a namespace)]
//   [one region per document path P (root.object.spec.containers[*] ...):
//    the member runs of every instance of P, in evaluation order]
// An object's (array's) members stay one contiguous run in document order, so
// every consumer of the node store reads it unchanged; what changes is that
// the wavefront's 64 consecutive reviews find their nodes at one path next to
// each other (a column of node runs per path) instead of in 64 documents.
// With `order` and `dl` (staged batches on a device), the path-grouped layout
// is built on the device instead (layout.hip gk_device_layout): `dst` is the
// per-document arena D -- every container's `val` its global document path --
// and `dl` what the device pass needs per review.
struct DevLayout {
  static constexpr uint32_t kSharedPath = 0xffffffffu;  // a shared Namespace run
  std::vector<uint32_t> beg;      // per batch index: the D index of its document's first node
  std::vector<uint32_t> evalpos;  // per batch index: its evaluation position
  std::vector<uint32_t> root_d;   // per batch index: its root's id in D (NO_ID: excluded)
  std::vector<uint32_t> slot;     // per batch index: its root's index in the layout (NO_ID: excluded)
  uint32_t nroots = 0;            // live reviews
};
// large flattener parts kept since their flattening are released on a
// background thread (callers that upload: after the upload)
void release_parts_async();

bool flatten_page(Store& st, std::mutex& smu, const NsCache& ns_cache, const std::set<std::string>* excluded_ns,
                  const Page& page, int threads, uint32_t base, NodeArena& dst, FlatResult& out, std::string& err,
                  const OrderFn* order = nullptr, std::vector<uint32_t>* perm = nullptr, DevLayout* dl = nullptr);

// Query inputs ({"review": ...} documents, Driver.Query's input) into `dst`
// likewise, with their match columns.
bool flatten_reviews(Store& st, std::mutex& smu, const NsCache& ns_cache,
                     const std::vector<std::pair<const char*, size_t>>& inputs, uint32_t base, NodeArena& dst,
                     std::vector<ReviewCol>& cols, std::string& err);

// Parses standalone JSON documents (the inventory's synced objects) on the
// host threads into `dst` (node id base + k at dst[k], strings interned into
// `st` under `smu`); roots[i] = the placed root node id of docs[i].  False +
// err on malformed JSON (the index of the first bad document).
bool flatten_docs(Store& st, std::mutex& smu, const std::vector<std::string_view>& docs, uint32_t base, NodeArena& dst,
                  std::vector<uint32_t>& roots, std::string& err);

int default_threads();

// Runs f(0) .. f(n-1) in parallel on the engine's persistent host workers
// (created once, sized to default_threads()) and the calling thread; returns
// when all are done.  Concurrent callers share the workers.  A webhook
// micro-batch is too small to pay for starting threads per call.
void parallel_run(int n, const std::function<void(int)>& f);

// id-independent content hash of the document rooted at `node` (`nodes`: the
// node array its ids index; strings and numbers of `st`)
uint64_t doc_hash(const Store& st, const Node* nodes, uint32_t node);

}  // namespace gk
