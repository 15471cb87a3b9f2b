// Referenced-path plan of a compiled template (north_star "columnar,
// path-interned ... arrays in HBM"; SURVEY.md 8(d) algorithmic bytes).
//
// The reference hands each review to OPA as a whole JSON document
// (pkg/target/target.go:145 json.Marshal(obj.Object), drivers/local/local.go:331
// json.MarshalIndent(input)).  A compiled template reads only a few paths of
// it.  plan_paths runs a forward data-flow analysis over the template's
// bytecode and returns the trie of document paths below `input.review` the
// program may read, with how each is used:
//   * navigated (a constant-key lookup: `.spec.containers`),
//   * looked up with a computed key (`ctr[probe]`, a parameter-derived key),
//   * iterated (`containers[_]`),
//   * counted, or
//   * used whole (compared, printed, passed to a builtin that reads
//     composites, added to a heap collection).
// The staging (colstore.cc) turns the trie into the batch's column schema:
// paths only navigated become 4-byte value columns of their table's rows
// (arrays become child tables with CSR ranges); a path used whole whose value
// is composite keeps its subtree as document nodes.  Paths no program reads
// are not uploaded at all.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "compiler.h"
#include "store.h"

namespace gk {

enum : uint8_t { PU_DYN = 1, PU_ITER = 2, PU_LEN = 4, PU_WHOLE = 8, PU_IDX = 16 };
constexpr uint32_t PK_ANY = 0xffffffffu;  // step: any member / element

struct PathNode {
  uint32_t parent = 0;
  uint32_t key = PK_ANY;  // string id of the member key, or PK_ANY
  uint8_t uses = 0;       // PU_* on the value at this path
  std::map<uint32_t, uint32_t> kids;  // key -> node
};

struct PathPlan {
  std::vector<PathNode> nodes;  // [0] = the review document (input.review)
  bool ok = true;               // false: columns cannot serve the program (why)
  std::string why;
  uint32_t child(uint32_t at, uint32_t key);
  void merge(const PathPlan& o);  // union (the batch's plan over every template)
  std::string describe(const Store& st) const;
};

PathPlan plan_paths(const Program& p, const CodeBank& bank);

}  // namespace gk
