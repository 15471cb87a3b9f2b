// Host-side interned document store: strings, numbers and the node arena that
// is mirrored into HBM.  Append-only between resets, so device copies are
// refreshed by uploading the tail.
#pragma once
#include <sys/mman.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <cstdlib>
#include <new>
#include <string_view>
#include <utility>
#include <vector>

#include "common.h"
#include "json.h"

namespace gk {

// Growable node array without element initialisation (every node is written
// before it is read); large arenas grow by realloc, which remaps pages instead
// of copying them.
class NodeArena {
 public:
  NodeArena() = default;
  NodeArena(const NodeArena&) = delete;
  NodeArena& operator=(const NodeArena&) = delete;
  NodeArena(NodeArena&& o) noexcept : p_(o.p_), n_(o.n_), cap_(o.cap_) { o.p_ = nullptr; o.n_ = o.cap_ = 0; }
  ~NodeArena() { free(p_); }
  size_t size() const { return n_; }
  size_t capacity() const { return cap_; }
  Node* data() { return p_; }
  const Node* data() const { return p_; }
  Node& operator[](size_t i) { return p_[i]; }
  const Node& operator[](size_t i) const { return p_[i]; }
  Node* begin() { return p_; }
  Node* end() { return p_ + n_; }
  const Node* begin() const { return p_; }
  const Node* end() const { return p_ + n_; }
  Node& back() { return p_[n_ - 1]; }
  void reserve(size_t n) { if (n > cap_) grow(n); }
  void resize(size_t n) { if (n > cap_) grow(n); n_ = n; }  // new nodes are uninitialised
  void push_back(const Node& x) { if (n_ == cap_) grow(n_ + 1); p_[n_++] = x; }
 private:
  void grow(size_t need) {
    size_t nc = cap_ ? cap_ * 2 : 1024;
    if (nc < need) nc = need;
    const size_t bytes = nc * sizeof(Node);
    Node* q;
    if (bytes >= (32u << 20)) {
      // large arenas (a staged page's documents, ~1 GB per 1M Pods): 2 MB
      // aligned and marked for transparent huge pages, so their first touch
      // by the flattener threads takes ~500 page faults per GB instead of
      // ~260K (the faults of a fresh arena serialize on the process's
      // memory map)
      void* m = nullptr;
      if (posix_memalign(&m, 2u << 20, bytes) != 0 || !m) throw std::bad_alloc();
      madvise(m, bytes, MADV_HUGEPAGE);
      q = (Node*)m;
      if (n_) memcpy(q, p_, n_ * sizeof(Node));
      free(p_);
    } else {
      q = (Node*)realloc(p_, bytes);
      if (!q) throw std::bad_alloc();
    }
    p_ = q;
    cap_ = nc;
  }
  Node* p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
};

// exact decimal text -> 64-bit-mantissa binary float, round-half-even
// (math/big Float.SetString at prec 64; topdown/builtins/builtins.go:161-172)
bool decimal_to_bf64(const char* s, size_t n, uint64_t* mant, int32_t* exp, bool* neg);
// Go strconv.ParseInt(s, 10, 64)
bool parse_int64(const char* s, size_t n, int64_t* out);
// Go fmt %v text of a number argument (topdown/strings.go:355-367)
std::string go_number_print(const char* s, size_t n);

class Store {
 public:
  Store();
  // back to the state of a new Store (the well-known strings, the four fixed
  // nodes), keeping the allocations: pooled flattener parts reuse their stores
  void reset();

  // -- strings
  uint32_t intern(const char* p, size_t n);
  uint32_t intern(const std::string& s) { return intern(s.data(), s.size()); }
  uint32_t intern(std::string_view s) { return intern(s.data(), s.size()); }
  uint32_t intern(const char* s) { return intern(s, strlen(s)); }
  std::string_view str(uint32_t id) const { return std::string_view(pool_.data() + strs_[id].off, strs_[id].len); }
  uint32_t nstrings() const { return (uint32_t)strs_.size(); }
  const std::vector<StrEnt>& strings() const { return strs_; }
  const std::string& pool() const { return pool_; }
  const std::vector<uint8_t>& str_flags() const { return sflags_; }
  uint32_t find(const char* p, size_t n) const;  // NO_ID if absent
  // make room for `n` more strings without rehashing while they are interned
  void reserve_strings(size_t n);
  // intern strings [first, nstrings) of every store in `src` on `threads`
  // threads; maps[p][s] = this store's id of src[p]'s string s (s < first: s)
  void intern_parts(const std::vector<const Store*>& src, uint32_t first, std::vector<std::vector<uint32_t>>& maps,
                    int threads);

  // -- numbers (interned by text)
  uint32_t number(const char* p, size_t n);
  const std::vector<NumEnt>& numbers() const { return nums_; }

  // -- nodes
  NodeArena& nodes() { return nodes_; }
  const NodeArena& nodes() const { return nodes_; }
  // Append the document rooted at j (BFS layout, contiguous children); returns root index.
  uint32_t add_doc(const JDoc& d, int j);
  // Parse JSON text straight into the arena (no intermediate DOM): a children
  // block is appended when its object / array closes, so every block is
  // contiguous.  The root comes back as a node record (not placed): the caller
  // stores it where the document hangs (e.g. review.object).  false + err on
  // malformed JSON.  Duplicate object keys keep the last value
  // (encoding/json into map[string]interface{}).
  bool parse_doc(const char* p, size_t n, Node* root, std::string* err);
  // Append a scalar / empty object node.
  uint32_t add_node(const Node& n);
  // Start a new object node with `n` children reserved; returns index of first child.
  uint32_t reserve(uint32_t n);

  size_t bytes() const { return pool_.size() + strs_.size() * sizeof(StrEnt) + nodes_.size() * sizeof(Node) + nums_.size() * sizeof(NumEnt); }

  // well-known string ids
  uint32_t s_empty, s_review, s_parameters, s_kind, s_group, s_version, s_name, s_namespace, s_object,
      s_oldObject, s_metadata, s_labels, s_unstable, s_msg, s_details, s_uid, s_resource, s_operation,
      s_userInfo, s_options, s_deny, s_creationTimestamp, s_spec, s_status, s_star, s_In, s_NotIn, s_Exists,
      s_DoesNotExist, s_Namespace, s_apiGroups, s_kinds, s_true, s_false, s_null;

 private:
  std::string pool_;
  std::vector<StrEnt> strs_;
  std::vector<uint8_t> sflags_;
  std::vector<uint64_t> table_;  // open addressing: hash tag << 32 | (string id + 1); 0 = empty
  std::vector<NumEnt> nums_;
  std::vector<uint32_t> num_table_;
  NodeArena nodes_;
  struct BfsEnt { int jn; uint32_t an, key; };
  std::vector<BfsEnt> bfs_;  // add_doc work queue (reused)
  std::vector<Node> pend_;   // parse_doc: children of the open objects / arrays
  std::string scratch_;      // parse_doc: unescaped string bytes
  // direct-mapped cache of short strings (<= 32 bytes: the bytes themselves are
  // the tag, so a hit touches one 40-byte entry instead of the table, the
  // string entry and the pool -- object keys and repeated values)
  struct ShortEnt { uint64_t w[4]; uint32_t len, id; };
  static constexpr size_t kShortCache = 4096;
  std::vector<ShortEnt> short_;
  uint32_t intern_slow(const char* p, size_t n, uint64_t hv);
  friend class DocParser;
  void init();
  void grow();
  void rehash(size_t sz);
  void grow_num();
};

inline uint64_t fnv1a(const char* p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) { h ^= (unsigned char)p[i]; h *= 1099511628211ull; }
  return h;
}

// string hash of the intern tables: 8 bytes per step (strings here are mostly
// short keys, names and images)
inline uint64_t str_hash(const char* p, size_t n) {
  auto mix = [](uint64_t a, uint64_t b) {
    __uint128_t m = (__uint128_t)(a ^ 0xa0761d6478bd642full) * (b ^ 0xe7037ed1a0b428dbull);
    return (uint64_t)m ^ (uint64_t)(m >> 64);
  };
  uint64_t h = 0x2d358dccaa6c78a5ull ^ n;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    h = mix(h, w);
  }
  if (i < n) {
    uint64_t w = 0;
    memcpy(&w, p + i, n - i);
    h = mix(h, w ^ 0x8ebc6af09c88c6e3ull);
  }
  return mix(h, 0x589965cc75374cc3ull);
}

}  // namespace gk
