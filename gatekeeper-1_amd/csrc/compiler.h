// ConstraintTemplate Rego -> predicate bytecode (host).
//
// Each template's `violation` rules compile into one loop-nest program that
// the GPU VM runs per (review, constraint) pair: generators (`x[_]`, unbound
// selector variables, partial-set rule references) become ITER loops,
// functions / complete rules / comprehensions / `not` are inlined as
// solution-collecting sub-blocks with OPA's semantics (functions yield once,
// conflicting values are an error, `false` from a statement call is
// undefined; eval.go:1405-1497), and every solution of a `violation` body
// EMITs (msg, details).  Anything outside the supported subset throws
// Unsupported and the template is served by the CPU OPA fallback.
#pragma once
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"
#include "rego.h"
#include "store.h"

namespace gk {

struct Unsupported : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// An inventory join site (compiler.cc join_site): `X := data.inventory<path>`
// whose body later requires `A == key(X)` with A bound before the iteration.
// The engine enumerates the path's leaves in iteration order, runs `key` (a
// program of the body literals that derive the key from the leaf; input.review
// is the leaf) on the device per leaf, and keeps (key hash, leaf) sorted per
// constraint: OP_JPROBE iterates only the leaves in A's bucket.
struct JoinSite {
  struct Sel {
    bool var = false;   // an unbound variable (iterated); else a constant string key
    uint32_t sid = 0;   // the key's string id
  };
  std::vector<Sel> path;  // selectors after `data.inventory`
  uint32_t nvars = 0;     // variable selectors (leaf row: leaf value, then their keys)
  uint32_t key_off = 0, key_len = 0, key_nregs = 0;  // the key program in the code bank
  std::string desc;       // diagnostics
};

struct Program {
  uint32_t code_off = 0;   // offset into the global code array
  uint32_t code_len = 0;
  uint32_t nregs = 0;
  bool uses_regex = false;
  bool uses_inventory = false;  // reads data.inventory (the engine keeps its tree current)
  std::vector<uint32_t> regex_literals;  // string ids of literal patterns
  std::vector<std::string> rules;
  // guard programs (compile_template_guard): expressions outside the subset
  // compiled to OP_FAIL_FALLBACK, and the first one's reason
  uint32_t fallback_sites = 0;
  std::string fallback_reason;
  std::vector<JoinSite> joins;  // inventory join sites (site index = OP_JPROBE y >> 8)
};

// All modules known to the driver, indexed by package path.
struct ModuleSet {
  std::map<std::vector<std::string>, std::vector<std::shared_ptr<rego::Module>>> by_pkg;
  void clear() { by_pkg.clear(); }
  void add(const std::shared_ptr<rego::Module>& m) { by_pkg[m->pkg].push_back(m); }
  // rules named `name` in package `pkg` (all modules of the package)
  std::vector<std::shared_ptr<rego::Rule>> rules(const std::vector<std::string>& pkg, const std::string& name) const;
  bool has_pkg(const std::vector<std::string>& pkg) const { return by_pkg.count(pkg) > 0; }
};

// Global code / constant tables shared by all programs (uploaded to HBM).
struct CodeBank {
  std::vector<Ins> code;
  std::vector<uint64_t> consts;    // K table (tagged values)
  std::vector<uint32_t> fmt;       // sprintf format words
  // the engine's data.inventory node (an object node whose members the engine
  // points at the current inventory tree; NO_ID: joins are unsupported)
  uint32_t inventory_node = 0xffffffffu;
  void clear() { code.clear(); consts.clear(); fmt.clear(); }
};

// Compile the template entry package `pkg` (must define `violation`).
Program compile_template(Store& st, const ModuleSet& mods, const std::vector<std::string>& pkg, CodeBank& bank);

// The same template with every body expression outside the subset compiled to
// OP_FAIL_FALLBACK (reason FB_TEMPLATE) where OPA would evaluate it: the
// expressions before it run on the device as a guard, so only the (review,
// constraint) pairs that reach an unsupported expression go to the CPU.
// Throws Unsupported only for constructs outside any rule body.
Program compile_template_guard(Store& st, const ModuleSet& mods, const std::vector<std::string>& pkg, CodeBank& bank);

// Tagged-value helpers shared with the engine.
inline uint64_t tag_val(uint32_t tag, uint64_t payload) { return ((uint64_t)tag << 60) | (payload & 0x0fffffffffffffffull); }

}  // namespace gk
