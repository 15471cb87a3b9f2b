// Host-side interned document store: strings, numbers and the node arena that
// is mirrored into HBM.  Append-only between resets, so device copies are
// refreshed by uploading the tail.
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>
#include <string_view>
#include <vector>

#include "common.h"
#include "json.h"

namespace gk {

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

  // -- strings
  uint32_t intern(const char* p, size_t n);
  uint32_t intern(const std::string& s) { return intern(s.data(), s.size()); }
  std::string_view str(uint32_t id) const { return std::string_view(pool_.data() + strs_[id].off, strs_[id].len); }
  uint32_t nstrings() const { return (uint32_t)strs_.size(); }
  const std::vector<StrEnt>& strings() const { return strs_; }
  const std::string& pool() const { return pool_; }
  const std::vector<uint8_t>& str_flags() const { return sflags_; }
  uint32_t find(const char* p, size_t n) const;  // NO_ID if absent

  // -- numbers (interned by text)
  uint32_t number(const char* p, size_t n);
  const std::vector<NumEnt>& numbers() const { return nums_; }

  // -- nodes
  std::vector<Node>& nodes() { return nodes_; }
  const std::vector<Node>& nodes() const { return nodes_; }
  // Append the document rooted at j (BFS layout, contiguous children); returns root index.
  uint32_t add_doc(const JDoc& d, int j);
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
  std::vector<uint32_t> table_;  // open addressing: string id + 1 (0 = empty)
  std::vector<NumEnt> nums_;
  std::vector<uint32_t> num_table_;
  std::vector<Node> nodes_;
  void grow();
  void grow_num();
};

inline uint64_t fnv1a(const char* p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) { h ^= (unsigned char)p[i]; h *= 1099511628211ull; }
  return h;
}

}  // namespace gk
