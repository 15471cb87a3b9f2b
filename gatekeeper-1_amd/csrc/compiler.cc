// Rego -> loop-nest bytecode compiler (continuation-passing codegen).
//
// compile_term(t, fail, k): emits code that computes every value of term t;
// for each value it runs continuation k(reg, fail') where fail' is the label
// to jump to for the next value (backtracking).  Generators (unbound ref
// selectors, partial-set references) open ITER loops whose NEXT label is the
// continuation's failure label; when a loop is exhausted control goes to the
// enclosing failure label.  Solution-collecting constructs (function calls,
// complete rules, comprehensions, negation) compile their inner body with a
// fresh "done" label and continue after it.
#include "compiler.h"
#include "regex.h"

#include <functional>
#include <map>
#include <set>

namespace gk {
using namespace rego;

std::vector<std::shared_ptr<Rule>> ModuleSet::rules(const std::vector<std::string>& pkg, const std::string& name) const {
  std::vector<std::shared_ptr<Rule>> out;
  auto it = by_pkg.find(pkg);
  if (it == by_pkg.end()) return out;
  for (auto& m : it->second)
    for (auto& r : m->rules)
      if (r->name == name) out.push_back(r);
  return out;
}

namespace {

constexpr uint16_t NOREG = 0xffff;

struct Env {
  std::map<std::string, int> vars;
  // lazy arrays (Comp::lazy_def): a local bound to array comprehensions (in
  // order) that is never materialized; its element iterations run them
  struct LazyPart {
    TermP compr;
    std::vector<std::string> locals;  // names its body binds (unbound at the definition)
  };
  std::map<std::string, std::vector<LazyPart>> lazy;
  // parameter-derived locals (`label := input.parameters.label`): the value as a
  // term over input.parameters, so a join's key program can recompute it
  std::map<std::string, TermP> pdef;
  Env* parent = nullptr;
  const TermP* pdef_lookup(const std::string& v) const {
    for (const Env* e = this; e; e = e->parent) {
      if (e->vars.count(v)) {
        auto it = e->pdef.find(v);
        return it == e->pdef.end() ? nullptr : &it->second;
      }
    }
    return nullptr;
  }
  const Module* mod = nullptr;
  int lookup(const std::string& v) const {
    for (const Env* e = this; e; e = e->parent) {
      auto it = e->vars.find(v);
      if (it != e->vars.end()) return it->second;
    }
    return -1;
  }
  const std::vector<LazyPart>* lazy_lookup(const std::string& v) const {
    for (const Env* e = this; e; e = e->parent) {
      if (e->vars.count(v)) return nullptr;
      auto it = e->lazy.find(v);
      if (it != e->lazy.end()) return &it->second;
    }
    return nullptr;
  }
};

using K = std::function<void(int reg, int fail)>;
using KE = std::function<void(int fail)>;

const std::map<std::string, uint32_t> kBuiltins = {
    {"count", BI_COUNT}, {"any", BI_ANY}, {"all", BI_ALL}, {"startswith", BI_STARTSWITH},
    {"endswith", BI_ENDSWITH}, {"contains", BI_CONTAINS}, {"re_match", BI_RE_MATCH}, {"regex.match", BI_RE_MATCH},
    {"to_number", BI_TO_NUMBER}, {"replace", BI_REPLACE}, {"substring", BI_SUBSTRING},
    {"is_number", BI_IS_NUMBER}, {"is_string", BI_IS_STRING}, {"is_boolean", BI_IS_BOOLEAN},
    {"is_array", BI_IS_ARRAY}, {"is_object", BI_IS_OBJECT}, {"is_set", BI_IS_SET}, {"is_null", BI_IS_NULL},
    {"lower", BI_LOWER}, {"upper", BI_UPPER}, {"trim", BI_TRIM}, {"split", BI_SPLIT}, {"concat", BI_CONCAT},
    {"indexof", BI_INDEXOF}, {"trim_prefix", BI_TRIM_PREFIX}, {"trim_suffix", BI_TRIM_SUFFIX},
    {"sort", BI_SORT}, {"array.concat", BI_ARRAY_CONCAT},
};
const std::map<uint32_t, int> kArity = {
    {BI_COUNT, 1}, {BI_ANY, 1}, {BI_ALL, 1}, {BI_STARTSWITH, 2}, {BI_ENDSWITH, 2}, {BI_CONTAINS, 2},
    {BI_RE_MATCH, 2}, {BI_TO_NUMBER, 1}, {BI_REPLACE, 3}, {BI_SUBSTRING, 3}, {BI_IS_NUMBER, 1},
    {BI_IS_STRING, 1}, {BI_IS_BOOLEAN, 1}, {BI_IS_ARRAY, 1}, {BI_IS_OBJECT, 1}, {BI_IS_SET, 1},
    {BI_IS_NULL, 1}, {BI_LOWER, 1}, {BI_UPPER, 1}, {BI_TRIM, 2}, {BI_SPLIT, 2}, {BI_CONCAT, 2},
    {BI_INDEXOF, 2}, {BI_TRIM_PREFIX, 2}, {BI_TRIM_SUFFIX, 2}, {BI_SORT, 1}, {BI_ARRAY_CONCAT, 2},
};
const std::map<std::string, uint32_t> kCmp = {{"equal", CMP_EQ}, {"neq", CMP_NE}, {"lt", CMP_LT},
                                              {"lte", CMP_LE}, {"gt", CMP_GT}, {"gte", CMP_GE}};
const std::map<std::string, uint32_t> kArith = {{"plus", AR_PLUS}, {"minus", AR_MINUS}, {"mul", AR_MUL},
                                                {"div", AR_DIV}, {"rem", AR_REM}, {"or", AR_OR}, {"and", AR_AND}};

class Comp {
 public:
  Comp(Store& st, const ModuleSet& mods, CodeBank& bank, bool guard) : st_(st), mods_(mods), bank_(bank), guard_(guard) {}

  Program run(const std::vector<std::string>& pkg) {
    auto rules = mods_.rules(pkg, "violation");
    if (rules.empty()) throw Unsupported("template has no violation rule");
    const bool fuse_on = !getenv("GKGPU_FUSE") || atoi(getenv("GKGPU_FUSE")) != 0;  // A/B switch, default on
    for (size_t ri = 0; ri < rules.size();) {
      const auto& r = rules[ri];
      // violation bodies sharing their first expression: one fused group
      // (the OP_ORD keys keep topdown's rule-by-rule emission order)
      size_t rj = ri + 1;
      if (fuse_on && !guard_ && r->kind == Rule::PSET && !r->is_else)
        while (rj < rules.size() && rules[rj]->kind == Rule::PSET && fusable(r, rules[rj], {}, {}, {})) ++rj;
      if (rj - ri >= 2) {
        int save = reg_top_;
        for (size_t j = ri; j < rj; ++j) prog_.rules.push_back(rules[j]->name);
        int Lg = label();
        Env env;
        env.mod = r->mod;
        fuse_ok_ = false;  // groups do not nest
        fused_bodies(rules, ri, rj, {}, &env, nullptr, Lg,
                     [&](size_t j, Env* e2, int f) { emit_violation(rules[j], e2, (int)j, f); });
        place(Lg);
        emit(OP_ORD, 0, 0, 0, 0, 0x80000000u | (uint32_t)(rj - ri));
        reg_top_ = save;
        ri = rj;
        continue;
      }
      const int idx = (int)ri;
      prog_.rules.push_back(r->name);
      const size_t code0 = code_.size(), labels0 = labels_.size();
      int save = reg_top_;
      try {
        if (r->kind != Rule::PSET) throw Unsupported("violation must be a partial set rule");
        int Lr = label();
        Env env;
        env.mod = r->mod;
        const auto& body = cbody(r, {});
        fuse_ok_ = fuse_on;
        body_k(body, 0, &env, Lr, [&, idx](int f) { emit_violation(r, &env, idx, f); });
        fuse_ok_ = false;
        place(Lr);
      } catch (const Unsupported& ex) {
        fuse_ok_ = false;
        // guard mode: a rule whose body cannot be compiled at all sends every
        // review that reaches it (every matched review) to the CPU
        if (!guard_) throw;
        code_.resize(code0);
        labels_.resize(labels0);
        loop_base_.clear();
        loop_var_lo_.clear();
        if (prog_.fallback_reason.empty()) prog_.fallback_reason = ex.what();
        ++prog_.fallback_sites;
        emit(OP_FAIL_FALLBACK, 0, 0, 0, 0, FB_TEMPLATE);
      }
      reg_top_ = save;
      ++ri;
    }
    emit(OP_END);
    return finish();
  }

 private:
  Store& st_;
  const ModuleSet& mods_;
  CodeBank& bank_;
  const bool guard_;
  std::vector<Ins> code_;
  std::vector<int> labels_;
  std::map<uint64_t, uint32_t> kidx_;
  int reg_top_ = 0, max_reg_ = 0;
  const Term* stmt_key_ = nullptr;  // last selector of the statement-level ref being compiled
  // Complete rules are evaluated once per lane: a lane's input (one review x one
  // constraint's parameters) is fixed and `with` is outside the subset, so the
  // value cannot change.  Each cached rule owns a (value, evaluated) register
  // pair numbered from kVReg while compiling; finish() renumbers them above the
  // scratch registers and clears the flags at program entry.
  static constexpr int kVReg = 10000;
  static constexpr size_t kMaxCachedRules = 16;
  std::map<const Rule*, std::pair<int, int>> crule_;
  int inline_depth_ = 0;
  std::map<std::pair<const void*, bool>, int> memo_;  // memo slot per (function, statement form)
  // Lane constants (registers numbered from kLReg while compiling, renumbered
  // by finish()): the input roots, loaded at entry, and constant-key paths
  // below them read inside loops, set to false at entry and looked up at
  // their first use.
  static constexpr int kLReg = 11000, kMaxLaneRegs = 16;
  int lreg_n_ = 0, rev_reg_ = -1, par_reg_ = -1;
  std::map<std::pair<int, std::vector<uint64_t>>, int> lpath_;  // (root, keys) -> value register
  bool lane_const(int r) const { return r >= kLReg && r < kLReg + lreg_n_; }
  static bool lane_paths_on() {
    static const bool on = !getenv("GKGPU_LANE_PATHS") || atoi(getenv("GKGPU_LANE_PATHS")) != 0;  // A/B
    return on;
  }
  int input_root(bool review) {
    int& r = review ? rev_reg_ : par_reg_;
    if (r < 0) r = kLReg + lreg_n_++;
    return r;
  }
  std::vector<int> loop_base_;  // register base of each enclosing ITER loop (innermost last)
  Program prog_;

  // Loops the value written to `dst` escapes: depths (lo, hi] (1-based), packed
  // into an instruction's y field as lo | hi << 8.  A register allocated before
  // loop j started lives outside loop j, so a heap value stored into it must
  // survive loop j's per-iteration heap reset.
  uint32_t escape_range(int dst) {
    int dd = 0;
    for (int b : loop_base_) if (b <= dst) ++dd;
    int cd = (int)loop_base_.size();
    if (dd >= cd) return 0;
    return (uint32_t)(dd + 1) | ((uint32_t)cd << 8);
  }
  void open_loop(int it, int coll) {
    if (loop_base_.size() >= 15) throw Unsupported("loop nesting too deep");
    emit(OP_ITER_INIT, (uint16_t)it, (uint16_t)coll, 0, 0, (uint32_t)loop_base_.size() + 1);
    loop_base_.push_back(reg_top_);
    loop_var_lo_.push_back(it + 2);  // the key / value registers (allocated right after the iterator's)
  }
  void close_loop() { loop_base_.pop_back(); loop_var_lo_.pop_back(); }
  std::vector<int> loop_var_lo_;  // per open loop: its lowest register written per iteration
  int depth() const { return (int)loop_base_.size(); }
  std::map<std::pair<const Rule*, std::string>, std::vector<ExprP>> cbody_cache_;

  // ---------------------------------------------------------------- emit
  int label() { labels_.push_back(-1); return (int)labels_.size() - 1; }
  void place(int l) { labels_[l] = (int)code_.size(); }
  void emit(uint16_t op, uint16_t a = 0, uint16_t b = 0, uint16_t c = 0, uint32_t x = 0, uint32_t y = 0) {
    code_.push_back(Ins{op, a, b, c, x, y});
  }
  void emit_jmp(uint16_t op, int a, int lbl) { emit(op, (uint16_t)a, 0, 0, (uint32_t)lbl, 0); }
  int alloc(int n = 1) {
    int r = reg_top_;
    reg_top_ += n;
    if (reg_top_ > max_reg_) max_reg_ = reg_top_;
    if (reg_top_ > 4000) throw Unsupported("register pressure");
    return r;
  }
  uint32_t kconst(uint64_t v) {
    auto it = kidx_.find(v);
    if (it != kidx_.end()) return it->second;
    uint32_t i = (uint32_t)bank_.consts.size();
    bank_.consts.push_back(v);
    kidx_[v] = i;
    return i;
  }
  int loadk(uint64_t v) {
    int r = alloc();
    emit(OP_LOADK, (uint16_t)r, 0, 0, kconst(v));
    return r;
  }

  Program finish() {
    if (!crule_.empty() || lreg_n_) {
      const int base = max_reg_, lbase = base + 2 * (int)crule_.size();
      auto map = [&](int r) {
        if (r >= kLReg) return lbase + (r - kLReg);
        if (r >= kVReg) return base + (r - kVReg);
        return r;
      };
      auto remap = [&](uint16_t& r) { if (r != NOREG) r = (uint16_t)map(r); };
      for (auto& in : code_) { remap(in.a); remap(in.b); remap(in.c); }
      std::vector<Ins> pro;
      uint32_t kf = kconst(tag_val(V_BOOL, 0));
      for (auto& cr : crule_) pro.push_back(Ins{OP_LOADK, (uint16_t)map(cr.second.second), 0, 0, kf, 0});
      // lane constants: the review and parameters roots, and the "looked up"
      // flags of the cached paths below them
      if (rev_reg_ >= 0) pro.push_back(Ins{OP_LOADREV, (uint16_t)map(rev_reg_), 0, 0, 0, 0});
      if (par_reg_ >= 0) pro.push_back(Ins{OP_LOADPARAM, (uint16_t)map(par_reg_), 0, 0, 0, 0});
      for (auto& lp : lpath_) pro.push_back(Ins{OP_LOADK, (uint16_t)map(lp.second), 0, 0, kf, 0});
      code_.insert(code_.begin(), pro.begin(), pro.end());
      for (auto& l : labels_) if (l >= 0) l += (int)pro.size();
      max_reg_ = lbase + lreg_n_;
    }
    prog_.code_off = (uint32_t)bank_.code.size();
    prog_.code_len = (uint32_t)code_.size();
    for (auto& in : code_) {
      switch (in.op) {
        case OP_JMP: case OP_JUNDEF: case OP_JFALSE: case OP_JTRUE: case OP_ITER_NEXT: case OP_MEMO_GET:
        case OP_JPROBE: case OP_JNEXT:
          if (labels_[in.x] < 0) throw std::runtime_error("unplaced label");
          in.x = prog_.code_off + (uint32_t)labels_[in.x];
          break;
        default: break;
      }
      bank_.code.push_back(in);
    }
    prog_.nregs = (uint32_t)max_reg_;
    return prog_;
  }

  // ---------------------------------------------------------------- values
  // A literal whose text is a canonical integer below 2^46 in magnitude ("0",
  // "1000", "-3"; not "1.0", "01", "-0", "1e3") loads as an exact V_INT: it
  // prints, compares and serialises exactly like its V_NUM form, and the
  // device's inline int/int compare and arithmetic paths apply to it.
  static bool canonical_small_int(const std::string& s, int64_t* v) {
    size_t i = 0;
    bool neg = false;
    if (i < s.size() && s[i] == '-') { neg = true; ++i; }
    if (i >= s.size() || s.size() - i > 14) return false;
    if (s[i] == '0' && (s.size() - i > 1 || neg)) return false;
    int64_t x = 0;
    for (; i < s.size(); ++i) {
      if (s[i] < '0' || s[i] > '9') return false;
      x = x * 10 + (s[i] - '0');
    }
    if (x >= (1ll << 46)) return false;
    *v = neg ? -x : x;
    return true;
  }

  uint64_t scalar_val(const TermP& t) {
    switch (t->stype) {
      case S_NULL: return tag_val(V_NULL, 0);
      case S_FALSE: return tag_val(V_BOOL, 0);
      case S_TRUE: return tag_val(V_BOOL, 1);
      case S_NUM: {
        int64_t iv;
        if (canonical_small_int(t->s, &iv)) return tag_val(V_INT, (uint64_t)iv & 0x0000ffffffffffffull);
        return tag_val(V_NUM, st_.number(t->s.data(), t->s.size()));
      }
      case S_STR: return tag_val(V_STR, st_.intern(t->s));
    }
    throw Unsupported("bad scalar");
  }
  bool is_const(const TermP& t) {
    if (t->k == T_SCALAR) return true;
    if (t->k == T_ARRAY) { for (auto& x : t->items) if (!is_const(x)) return false; return true; }
    if (t->k == T_OBJECT) {
      for (size_t i = 0; i < t->items.size(); i += 2) {
        if (t->items[i]->k != T_SCALAR || t->items[i]->stype != S_STR) return false;
        if (!is_const(t->items[i + 1])) return false;
      }
      return true;
    }
    return false;
  }
  // fill node `idx` from constant term t
  void fill_const(uint32_t idx, const TermP& t, uint32_t key) {
    Node n{};
    n.key = key;
    if (t->k == T_SCALAR) {
      switch (t->stype) {
        case S_NULL: n.type = NT_NULL; break;
        case S_FALSE: n.type = NT_FALSE; break;
        case S_TRUE: n.type = NT_TRUE; break;
        case S_NUM: n.type = NT_NUM; n.val = st_.number(t->s.data(), t->s.size()); break;
        case S_STR: n.type = NT_STR; n.val = st_.intern(t->s); break;
      }
      st_.nodes()[idx] = n;
      return;
    }
    bool obj = t->k == T_OBJECT;
    uint32_t cnt = obj ? (uint32_t)t->items.size() / 2 : (uint32_t)t->items.size();
    n.type = obj ? NT_OBJ : NT_ARR;
    n.n = (uint16_t)cnt;
    n.first = st_.reserve(cnt);
    st_.nodes()[idx] = n;
    for (uint32_t i = 0; i < cnt; ++i) {
      if (obj) fill_const(n.first + i, t->items[2 * i + 1], st_.intern(t->items[2 * i]->s));
      else fill_const(n.first + i, t->items[i], i);
    }
  }
  uint64_t const_value(const TermP& t) {
    if (t->k == T_SCALAR) return scalar_val(t);
    if (t->k == T_OBJECT && t->items.empty()) return tag_val(V_NODE, 0);
    uint32_t idx = st_.reserve(1);
    fill_const(idx, t, 0);
    return tag_val(V_NODE, idx);
  }

  // ---------------------------------------------------------------- scope
  bool is_global(const Env* env, const std::string& v) {
    if (v == "input" || v == "data") return true;
    if (env->mod) {
      if (!mods_.rules(env->mod->pkg, v).empty()) return true;
      for (auto& im : env->mod->imports) if (im.second == v) return true;
    }
    return false;
  }
  bool unbound(const Env* env, const TermP& t) {
    return t->k == T_VAR && env->lookup(t->s) < 0 && !is_global(env, t->s);
  }
  bool ground(const Env* env, const TermP& t) {
    std::vector<std::string> vs;
    term_vars(t, vs);
    for (auto& v : vs) if (env->lookup(v) < 0 && !is_global(env, v)) return false;
    return true;
  }

  const std::vector<ExprP>& cbody(const std::shared_ptr<Rule>& r, const std::vector<std::string>& safe) {
    std::string key;
    for (auto& s : safe) key += s + ",";
    auto ck = std::make_pair((const Rule*)r.get(), key);
    auto it = cbody_cache_.find(ck);
    if (it != cbody_cache_.end()) return it->second;
    Env tmp;
    tmp.mod = r->mod;
    std::vector<std::string> sf = safe;
    for (auto& a : r->args) term_vars(a, sf);
    auto b = compile_body(r->body, sf, [&](const std::string& v) { return is_global(&tmp, v); });
    return cbody_cache_[ck] = b;
  }

  // ---------------------------------------------------------------- bodies
  void body_k(const std::vector<ExprP>& body, size_t i, Env* env, int fail, const KE& succ) {
    if (i < body.size() && lazy_def(body, i, env)) { body_k(body, i + 1, env, fail, succ); return; }
    if (guard_) { guarded_body_k(body, i, env, fail, succ); return; }
    if (i == body.size()) { succ(fail); return; }
    if (join_site(body, i, env, fail, succ)) return;
    if (lazy_inline(body, i, env, fail, succ)) return;
    expr(body[i], env, fail, [&, i, env](int f) { body_k(body, i + 1, env, f, succ); });
  }

  // Guard mode (compile_template_guard): a body expression outside the subset
  // compiles to OP_FAIL_FALLBACK at the point OPA would evaluate it.  Bodies
  // are conjunctions evaluated in order (after OPA's safety reordering, which
  // cbody applies), so the expressions before it act as a device-evaluated
  // guard: a (review, constraint) whose evaluation never reaches the
  // unsupported expression has exactly the results of the compiled prefix
  // (usually none, e.g. `input.review.kind.kind == "Service"` for a Pod), and
  // one that reaches it is routed whole to the CPU.  The innermost enclosing
  // body catches; the code, labels, registers, loops and bindings emitted for
  // the failed expression are rolled back first.
  void guarded_body_k(const std::vector<ExprP>& body, size_t i, Env* env, int fail, const KE& succ) {
    const size_t code0 = code_.size(), labels0 = labels_.size(), loops0 = loop_base_.size();
    const int reg0 = reg_top_, depth0 = inline_depth_;
    const Term* key0 = stmt_key_;
    const std::map<std::string, int> vars0 = env->vars;
    try {
      if (i == body.size()) succ(fail);
      else expr(body[i], env, fail, [&, i, env](int f) { body_k(body, i + 1, env, f, succ); });
    } catch (const Unsupported& ex) {
      if (code_.size() < code0 || labels_.size() < labels0) throw;  // cannot roll back (nested guard already did)
      code_.resize(code0);
      labels_.resize(labels0);
      loop_base_.resize(loops0);
      loop_var_lo_.resize(loops0);
      reg_top_ = reg0;
      inline_depth_ = depth0;
      stmt_key_ = key0;
      env->vars = vars0;
      if (prog_.fallback_reason.empty()) prog_.fallback_reason = ex.what();
      ++prog_.fallback_sites;
      emit(OP_FAIL_FALLBACK, 0, 0, 0, 0, FB_TEMPLATE);
    }
  }

  // ---------------------------------------------------------------- lazy arrays
  // An array comprehension bound to a local that the rest of the body only
  // iterates -- `x[_]`, directly or through array.concat / aliases -- is not
  // materialized: each iteration runs the comprehension's body as a generator
  // (in order, so elements come in array order, duplicates kept).  This is
  // how demo/basic's K8sUniqueLabel scans data.inventory
  // (k8suniquelabel_template.yaml:49-52: cluster_objs / ns_objs /
  // array.concat / all_objs[_]) without holding the whole inventory in the
  // lane heap.  The comprehension is pure, so evaluating it at its use (with
  // the definition's bindings, which stay bound) gives the same elements.
  static bool is_wild(const TermP& t) { return t && t->k == T_VAR && t->s.rfind("$_", 0) == 0; }
  static bool is_var(const TermP& t, const std::string& x) { return t && t->k == T_VAR && t->s == x; }
  static bool concat_call(const ExprP& e) {
    if (e->kind != Expr::TERM || e->negated || !e->withs.empty()) return false;
    const TermP& t = e->terms[0];
    return t->k == T_CALL && t->op == std::vector<std::string>{"array", "concat"} && t->items.size() == 3 &&
           t->items[0]->k == T_VAR && t->items[1]->k == T_VAR && t->items[2]->k == T_VAR;
  }
  static bool alias_expr(const ExprP& e, std::string* dst, std::string* src) {
    if ((e->kind != Expr::ASSIGN && e->kind != Expr::UNIFY) || e->negated || !e->withs.empty() || e->terms.size() != 2)
      return false;
    if (e->terms[0]->k != T_VAR || e->terms[1]->k != T_VAR) return false;
    *dst = e->terms[0]->s;
    *src = e->terms[1]->s;
    return true;
  }
  // every occurrence of x inside t is `x[<wildcard>]...`
  static bool lazy_term_ok(const TermP& t, const std::string& x) {
    if (!t) return true;
    switch (t->k) {
      case T_SCALAR: return true;
      case T_VAR: return t->s != x;
      case T_REF:
        if (is_var(t->head, x)) {
          if (t->items.empty() || !is_wild(t->items[0])) return false;
        } else if (!lazy_term_ok(t->head, x)) {
          return false;
        }
        for (auto& i : t->items) if (!lazy_term_ok(i, x)) return false;
        return true;
      case T_ARRCOMPR: case T_SETCOMPR: case T_OBJCOMPR:
        if (!lazy_term_ok(t->key, x) || !lazy_term_ok(t->value, x)) return false;
        for (auto& e : t->body) if (!lazy_expr_ok(e, x)) return false;
        return true;
      default:
        for (auto& i : t->items) if (!lazy_term_ok(i, x)) return false;
        return true;
    }
  }
  static bool lazy_expr_ok(const ExprP& e, const std::string& x) {
    for (auto& t : e->terms) if (!lazy_term_ok(t, x)) return false;
    for (auto& w : e->withs) if (!lazy_term_ok(w.target, x) || !lazy_term_ok(w.value, x)) return false;
    return true;
  }
  // x (defined by body[i]) may stay lazy: every later use iterates it, or
  // feeds an array.concat / alias whose result may stay lazy
  bool lazy_ok(const std::vector<ExprP>& body, size_t i, const std::string& x, int depth = 0) {
    if (depth > 8) return false;
    bool used = false;
    for (size_t j = i + 1; j < body.size(); ++j) {
      const ExprP& e = body[j];
      std::string dst, src;
      if (concat_call(e) && (is_var(e->terms[0]->items[0], x) || is_var(e->terms[0]->items[1], x))) {
        if (is_var(e->terms[0]->items[2], x) || !lazy_ok(body, j, e->terms[0]->items[2]->s, depth + 1)) return false;
        used = true;
        continue;
      }
      if (alias_expr(e, &dst, &src) && src == x) {
        if (dst == x || !lazy_ok(body, j, dst, depth + 1)) return false;
        used = true;
        continue;
      }
      if (!lazy_expr_ok(e, x)) return false;
      used = used || !lazy_term_ok_unused(e, x);
    }
    return used;
  }
  static bool lazy_term_ok_unused(const ExprP& e, const std::string& x) {
    // true when x does not occur in e at all (also inside comprehension bodies)
    struct F {
      static bool occ(const TermP& t, const std::string& x) {
        if (!t) return false;
        if (t->k == T_VAR) return t->s == x;
        if (occ(t->head, x) || occ(t->key, x) || occ(t->value, x)) return true;
        for (auto& i : t->items) if (occ(i, x)) return true;
        for (auto& b : t->body)
          for (auto& u : b->terms) if (occ(u, x)) return true;
        return false;
      }
    };
    for (auto& t : e->terms) if (F::occ(t, x)) return false;
    return true;
  }
  bool lazy_def(const std::vector<ExprP>& body, size_t i, Env* env) {
    if (!lazy_on()) return false;
    const ExprP& e = body[i];
    std::string dst, src;
    if ((e->kind == Expr::ASSIGN || e->kind == Expr::UNIFY) && !e->negated && e->withs.empty() && e->terms.size() == 2 &&
        e->terms[0]->k == T_VAR && e->terms[1]->k == T_ARRCOMPR && unbound(env, e->terms[0])) {
      const std::string& x = e->terms[0]->s;
      if (!lazy_ok(body, i, x)) return false;
      Env::LazyPart part{e->terms[1], {}};
      compr_locals(e->terms[1], env, part.locals);
      env->lazy[x] = {part};
      return true;
    }
    if (concat_call(e)) {
      const TermP& c = e->terms[0];
      const auto* a = env->lazy_lookup(c->items[0]->s);
      const auto* b = env->lazy_lookup(c->items[1]->s);
      if (!a || !b || !unbound(env, c->items[2]) || !lazy_ok(body, i, c->items[2]->s)) return false;
      std::vector<Env::LazyPart> l = *a;
      l.insert(l.end(), b->begin(), b->end());
      env->lazy[c->items[2]->s] = l;
      return true;
    }
    if (alias_expr(e, &dst, &src)) {
      const auto* a = env->lazy_lookup(src);
      if (!a || env->lookup(dst) >= 0 || !lazy_ok(body, i, dst)) return false;
      env->lazy[dst] = *a;
      return true;
    }
    return false;
  }
  static bool lazy_on() {
    const char* v = getenv("GKGPU_LAZY_ARRAYS");  // A/B switch, default on
    return !v || atoi(v) != 0;
  }
  // names a comprehension's body binds itself (not bound in env)
  void compr_locals(const TermP& t, Env* env, std::vector<std::string>& out) {
    std::function<void(const TermP&)> rec = [&](const TermP& u) {
      if (!u) return;
      if (u->k == T_VAR) {
        if (u->s != "input" && u->s != "data" && env->lookup(u->s) < 0 && !is_global(env, u->s)) out.push_back(u->s);
        return;
      }
      rec(u->head);
      rec(u->key);
      rec(u->value);
      for (auto& i : u->items) rec(i);
      for (auto& b : u->body)
        for (auto& v : b->terms) rec(v);
    };
    for (auto& b : t->body)
      for (auto& v : b->terms) rec(v);
    rec(t->key);
  }
  // `x[_]...` over a lazy array: each comprehension's solutions in turn
  void lazy_iter(const std::vector<Env::LazyPart>& list, const TermP& ref, Env* env, int fail, const K& k) {
    const auto& path = ref->items;
    NoFuse nf(this);  // array order is observable
    for (auto& part : list)
      for (auto& v : part.locals)
        if (env->lookup(v) >= 0) throw Unsupported("lazy array: comprehension local " + v + " bound at its use");
    for (size_t c = 0; c < list.size(); ++c) {
      const TermP& C = list[c].compr;
      const bool last = c + 1 == list.size();
      const int Lnext = last ? fail : label();
      Env inner;
      inner.parent = env;
      inner.mod = env->mod;
      body_k(C->body, 0, &inner, Lnext, [&](int f) {
        term(C->key, &inner, f, [&](int vr, int f2) {
          const int idx = loadk(tag_val(V_INT, 0));  // the index wildcard is never read
          bind(env, path[0]->s, idx);
          walk(vr, path, 1, env, f2, k);
          unbind(env, path[0]->s);
          emit_jmp(OP_JMP, 0, f2);
        });
      });
      if (last) emit_jmp(OP_JMP, 0, fail);
      else place(Lnext);
    }
  }

  // ---------------------------------------------------------------- inventory joins
  // The cross-resource templates (k8suniqueserviceselector_template.yaml:40-44,
  // k8suniquelabel_template.yaml:49-52) iterate every synced object and keep
  // the ones whose key equals the review's:
  //     other := data.inventory.namespace[ns][_][_][name]      (body[i])
  //     ... other_selector := flatten_selector(other) ...      (the key slice)
  //     input_selector == other_selector                       (body[j])
  // A scan is O(inventory) per review.  join_site compiles such an iteration
  // as a probe of a hash index -- the engine's key pass (kernels.hip
  // gk_key_kernel) runs the key slice once per leaf and keeps (key hash, leaf)
  // sorted per constraint -- so each review visits only the leaves in its
  // key's bucket, in iteration order.  Every body literal after body[i] still
  // runs for those leaves (the equality included: a hash collision finds
  // nothing), and the plain scan is compiled beside the probe for lanes without
  // an index (none built, a key pass that failed, a composite probe value).
  // The probe skips the literals between body[i] and body[j] for leaves outside
  // the bucket, so join_site requires those to be error-free (err_free_expr):
  // skipping an undefined literal changes nothing, skipping an error would.
  static bool joins_on() {
    const char* v = getenv("GKGPU_JOINS");  // A/B switch, default on
    return !v || atoi(v) != 0;
  }
  const std::vector<std::string>* str_vars_ = nullptr;  // err_free_call: variables known to hold strings
  struct JoinPlan {
    std::string x;                       // the leaf variable
    std::vector<JoinSite::Sel> path;
    std::vector<std::string> pvars;      // names of the variable selectors (in order)
    TermP a;                             // the probe side (a variable bound before body[i], or a constant)
    TermP key;                           // the key side (a term over x and slice outputs)
    std::vector<ExprP> slice;            // literals of (i, j) that derive the key
    std::vector<std::string> params;     // parameter-derived locals the key reads
  };

  // value of a parameter-derived term as a term over input.parameters
  TermP param_def(const Env* env, const TermP& t) {
    if (t->k == T_SCALAR) return t;
    if (t->k == T_VAR) {
      if (is_global(env, t->s)) return nullptr;
      const TermP* d = env->pdef_lookup(t->s);
      return d ? *d : nullptr;
    }
    if (t->k == T_REF && t->head && t->head->k == T_VAR && t->head->s == "input" && env->lookup("input") < 0 &&
        !t->items.empty() && t->items[0]->k == T_SCALAR && t->items[0]->s == "parameters") {
      auto c = std::make_shared<Term>(*t);
      for (auto& it : c->items) {
        if (it->k == T_SCALAR) continue;
        TermP d = it->k == T_VAR ? param_def(env, it) : nullptr;
        if (!d || d->k != T_SCALAR) return nullptr;
        it = d;
      }
      return c;
    }
    return nullptr;
  }

  static void occ_vars(const TermP& t, std::set<std::string>& out) {
    if (!t) return;
    if (t->k == T_VAR) { out.insert(t->s); return; }
    occ_vars(t->head, out);
    occ_vars(t->key, out);
    occ_vars(t->value, out);
    for (auto& i : t->items) occ_vars(i, out);
    for (auto& b : t->body)
      for (auto& u : b->terms) occ_vars(u, out);
  }
  static std::set<std::string> expr_vars(const ExprP& e) {
    std::set<std::string> s;
    for (auto& t : e->terms) occ_vars(t, s);
    return s;
  }
  // variables a literal binds (given the ones bound before it), or false when
  // it is not a single-valued definition (a generator, a negation, a test)
  bool defines(const ExprP& e, const std::set<std::string>& bound, const Env* env, std::string* out) {
    if (e->negated || !e->withs.empty()) return false;
    auto iter_free = [&](const TermP& t) {
      // no ref selector is an unbound variable (which would iterate)
      std::function<bool(const TermP&)> ok = [&](const TermP& u) -> bool {
        if (!u) return true;
        if (u->k == T_ARRCOMPR || u->k == T_SETCOMPR || u->k == T_OBJCOMPR) return true;  // collected, not iterated
        if (u->k == T_REF)
          for (auto& s : u->items)
            if (s->k == T_VAR && !bound.count(s->s) && env->lookup(s->s) < 0 && !is_global(env, s->s) &&
                s->s.rfind("$_", 0) != 0)
              return false;
        if (!ok(u->head)) return false;
        for (auto& s : u->items) if (!ok(s)) return false;
        return true;
      };
      return ok(t);
    };
    if ((e->kind == Expr::ASSIGN || e->kind == Expr::UNIFY) && e->terms.size() == 2 && e->terms[0]->k == T_VAR &&
        !bound.count(e->terms[0]->s) && env->lookup(e->terms[0]->s) < 0 && !is_global(env, e->terms[0]->s)) {
      if (!iter_free(e->terms[1])) return false;
      *out = e->terms[0]->s;
      return true;
    }
    if (e->kind == Expr::TERM && e->terms[0]->k == T_CALL && !e->terms[0]->items.empty()) {
      const TermP& o = e->terms[0]->items.back();
      if (o->k != T_VAR || o->s.rfind("$l", 0) != 0 || bound.count(o->s)) return false;
      for (size_t q = 0; q + 1 < e->terms[0]->items.size(); ++q) if (!iter_free(e->terms[0]->items[q])) return false;
      *out = o->s;
      return true;
    }
    return false;
  }

  // user functions a call resolves to (module-local name or data.<pkg>.<name>)
  std::vector<std::shared_ptr<Rule>> fn_rules(const Module* mod, const std::vector<std::string>& op) {
    if (op.size() == 1 && mod) return mods_.rules(mod->pkg, op[0]);
    if (op.size() >= 2 && op[0] == "data") {
      std::vector<std::string> pkg(op.begin() + 1, op.end() - 1);
      return mods_.rules(pkg, op.back());
    }
    return {};
  }
  // the term never reads `input` (also through the functions it calls)
  bool input_free(const TermP& t, const Module* mod, int depth) {
    if (!t) return true;
    if (t->k == T_VAR) return t->s != "input";
    if (t->k == T_CALL) {
      auto rules = fn_rules(mod, t->op);
      if (!rules.empty()) {
        if (depth > 6) return false;
        for (auto& r : rules) {
          for (auto& e : cbody(r, {}))
            for (auto& u : e->terms) if (!input_free(u, r->mod, depth + 1)) return false;
          if (!input_free(r->value, r->mod, depth + 1)) return false;
        }
      }
    }
    if (!input_free(t->head, mod, depth) || !input_free(t->key, mod, depth) || !input_free(t->value, mod, depth))
      return false;
    for (auto& i : t->items) if (!input_free(i, mod, depth)) return false;
    for (auto& b : t->body)
      for (auto& u : b->terms) if (!input_free(u, mod, depth)) return false;
    return true;
  }

  // ---- error-freedom (conservative): the literal cannot raise an evaluation
  // error (only succeed or be undefined).  Comparisons and lookups never err;
  // sprintf over an array literal does not; a user function does not when its
  // bodies do not and no two of them can yield different values (a single
  // body, one constant value, or bodies that test one path against the same
  // constant with == and != -- make_apiversion's shape).
  // value kinds the analysis can prove, for builtins that err on others: 1 a
  // collection (count), 2 a set (set difference).  Locals resolve through
  // their definitions in ctx_body_; a complete rule through its one body.
  const std::vector<ExprP>* ctx_body_ = nullptr;
  const std::vector<TermP>* ctx_args_ = nullptr;  // the function's arguments (fn_err_free)
  static bool expr_mentions(const ExprP& e, const std::string& v) {
    std::vector<std::string> vs;
    for (auto& u : e->terms) term_vars(u, vs);
    return std::find(vs.begin(), vs.end(), v) != vs.end();
  }
  int coll_kind(const TermP& t, const Module* mod, int depth) {
    if (!t || depth > 8) return 0;
    switch (t->k) {
      case T_SETCOMPR: case T_SET: return 2;
      case T_ARRCOMPR: case T_ARRAY: case T_OBJCOMPR: case T_OBJECT: return 1;
      case T_VAR: {
        // an argument is whatever the caller passes (and shadows a rule name)
        if (ctx_args_) {
          std::vector<std::string> vs;
          for (auto& a : *ctx_args_) term_vars(a, vs);
          if (std::find(vs.begin(), vs.end(), t->s) != vs.end()) return 0;
        }
        // the variable's definition: `v := term`, or `v = term` / the output
        // of a set difference when nothing before it mentions v (otherwise the
        // unification is a test on a value bound elsewhere)
        if (ctx_body_)
          for (auto& e : *ctx_body_) {
            if (!e->negated) {
              if (e->kind == Expr::ASSIGN && e->terms.size() == 2 && e->terms[0]->k == T_VAR && e->terms[0]->s == t->s)
                return coll_kind(e->terms[1], mod, depth + 1);
              if (e->kind == Expr::UNIFY && e->terms.size() == 2 && e->terms[0]->k == T_VAR && e->terms[0]->s == t->s)
                return coll_kind(e->terms[1], mod, depth + 1);
              if (e->kind == Expr::TERM && e->terms[0]->k == T_CALL && e->terms[0]->items.size() == 3 &&
                  e->terms[0]->items[2]->k == T_VAR && e->terms[0]->items[2]->s == t->s &&
                  e->terms[0]->op == std::vector<std::string>{"minus"})
                return coll_kind(e->terms[0]->items[0], mod, depth + 1) == 2 &&
                               coll_kind(e->terms[0]->items[1], mod, depth + 1) == 2
                           ? 2
                           : 0;
            }
            if (expr_mentions(e, t->s)) return 0;  // bound (or used) before any definition
          }
        if (mod) {
          auto rs = mods_.rules(mod->pkg, t->s);
          if (rs.size() == 1 && rs[0]->kind == Rule::COMPLETE && !rs[0]->is_default && !rs[0]->is_else) {
            const auto* save = ctx_body_;
            const auto* save_a = ctx_args_;
            ctx_body_ = &cbody(rs[0], {});
            ctx_args_ = nullptr;
            const int k = coll_kind(rs[0]->value, rs[0]->mod, depth + 1);
            ctx_body_ = save;
            ctx_args_ = save_a;
            return k;
          }
        }
        return 0;
      }
      default: return 0;
    }
  }
  // a rule referenced as a value cannot err: error-free bodies, and a complete
  // rule cannot conflict (one body, or one constant value)
  bool rule_err_free(const std::vector<std::shared_ptr<Rule>>& rules, int depth) {
    if (depth > 6) return false;
    bool same_const = true;
    for (auto& r : rules) {
      if (r->is_else || (r->kind != Rule::COMPLETE && r->kind != Rule::PSET)) return false;
      const auto* save = ctx_body_;
      const auto* save_a = ctx_args_;
      ctx_body_ = &cbody(r, {});
      ctx_args_ = nullptr;
      bool ok = true;
      for (auto& e : *ctx_body_) ok = ok && err_free_expr(e, r->mod, depth + 1);
      ok = ok && err_free_term(r->kind == Rule::PSET ? r->key : r->value, r->mod, depth + 1);
      ctx_body_ = save;
      ctx_args_ = save_a;
      if (!ok) return false;
      same_const = same_const && r->value && is_const(r->value) && same_term(r->value, rules[0]->value);
    }
    return rules[0]->kind == Rule::PSET || rules.size() == 1 || same_const;
  }
  bool err_free_term(const TermP& t, const Module* mod, int depth) {
    if (!t) return true;
    switch (t->k) {
      case T_SCALAR: return true;
      case T_VAR: {
        if (mod && t->s != "input" && t->s != "data") {
          auto rs = mods_.rules(mod->pkg, t->s);
          if (!rs.empty()) return rule_err_free(rs, depth);
        }
        return true;
      }
      case T_SETCOMPR: case T_ARRCOMPR: {
        if (!err_free_term(t->key, mod, depth)) return false;
        for (auto& e : t->body) if (!err_free_expr(e, mod, depth)) return false;
        return true;
      }
      case T_REF:
        if (!t->head || t->head->k != T_VAR) return false;
        if (mod && t->head->s != "input" && t->head->s != "data" && !mods_.rules(mod->pkg, t->head->s).empty()) return false;
        if (t->head->s == "data" && (t->items.empty() || t->items[0]->k != T_SCALAR || t->items[0]->s != "inventory")) return false;
        for (auto& i : t->items) if (!err_free_term(i, mod, depth)) return false;
        return true;
      case T_ARRAY: case T_SET:
        for (auto& i : t->items) if (!err_free_term(i, mod, depth)) return false;
        return true;
      case T_OBJECT:
        for (size_t q = 0; q < t->items.size(); q += 2)
          if (t->items[q]->k != T_SCALAR || !err_free_term(t->items[q + 1], mod, depth)) return false;
        return true;
      case T_CALL: return err_free_call(t, mod, depth);
      default: return false;
    }
  }
  bool err_free_call(const TermP& t, const Module* mod, int depth) {
    static const std::set<std::string> cmp = {"equal", "neq", "lt", "lte", "gt", "gte"};
    size_t nargs = t->items.size();
    if (!t->items.empty() && t->items.back()->k == T_VAR && t->items.back()->s.rfind("$l", 0) == 0) --nargs;
    for (size_t q = 0; q < nargs; ++q) if (!err_free_term(t->items[q], mod, depth)) return false;
    if (t->op.size() == 1 && cmp.count(t->op[0])) return true;
    if (t->op == std::vector<std::string>{"count"}) return nargs == 1 && coll_kind(t->items[0], mod, 0) >= 1;
    if (t->op == std::vector<std::string>{"minus"})
      return nargs == 2 && coll_kind(t->items[0], mod, 0) == 2 && coll_kind(t->items[1], mod, 0) == 2;
    if (t->op == std::vector<std::string>{"sprintf"})
      return nargs == 2 && t->items[0]->k == T_SCALAR && t->items[0]->stype == S_STR && t->items[1]->k == T_ARRAY;
    if (t->op == std::vector<std::string>{"re_match"} || t->op == std::vector<std::string>{"regex", "match"}) {
      // a valid literal pattern over a string: no error (regex.go:89-102
      // errs on a bad pattern or a non-string operand)
      if (nargs != 2 || t->items[0]->k != T_SCALAR || t->items[0]->stype != S_STR) return false;
      std::vector<uint32_t> dfa;
      if (compile_regex_dfa(t->items[0]->s, dfa) != RX_OK) return false;
      const TermP& a = t->items[1];
      if (a->k == T_SCALAR) return a->stype == S_STR;
      return a->k == T_VAR && str_vars_ && std::find(str_vars_->begin(), str_vars_->end(), a->s) != str_vars_->end();
    }
    auto rules = fn_rules(mod, t->op);
    if (rules.empty() || depth > 6) return false;
    return fn_err_free(rules, depth + 1);
  }
  bool err_free_expr(const ExprP& e, const Module* mod, int depth) {
    if (!e->withs.empty()) return false;
    if (e->kind == Expr::SOME) return true;
    for (auto& t : e->terms) if (!err_free_term(t, mod, depth)) return false;
    return true;
  }
  bool fn_err_free(const std::vector<std::shared_ptr<Rule>>& rules, int depth) {
    for (auto& r : rules) {
      if (r->kind != Rule::FUNC || r->is_else || r->is_default) return false;
      const auto* save = ctx_body_;
      const auto* save_a = ctx_args_;
      ctx_body_ = &cbody(r, {});
      ctx_args_ = &r->args;
      bool ok = true;
      for (auto& e : *ctx_body_) ok = ok && err_free_expr(e, r->mod, depth);
      ok = ok && err_free_term(r->value, r->mod, depth);
      ctx_body_ = save;
      ctx_args_ = save_a;
      if (!ok) return false;
    }
    if (rules.size() == 1) return true;
    bool same_const = true;
    for (auto& r : rules) same_const = same_const && r->value && is_const(r->value) && same_term(r->value, rules[0]->value);
    if (same_const) return true;
    for (size_t p = 0; p < rules.size(); ++p)
      for (size_t q = p + 1; q < rules.size(); ++q)
        if (!exclusive(rules[p], rules[q])) return false;
    return true;
  }
  // canonical text of a body-local term: function arguments by position,
  // single-assignment locals by their definition, constant-key refs
  bool canon(const TermP& t, const std::shared_ptr<Rule>& r, const std::vector<ExprP>& body, int depth, std::string* out) {
    if (depth > 8) return false;
    if (t->k == T_SCALAR) { *out = std::to_string(t->stype) + ":" + t->s; return true; }
    if (t->k == T_VAR) {
      for (size_t a = 0; a < r->args.size(); ++a)
        if (r->args[a]->k == T_VAR && r->args[a]->s == t->s) { *out = "$arg" + std::to_string(a); return true; }
      for (auto& e : body)
        if ((e->kind == Expr::ASSIGN || e->kind == Expr::UNIFY) && !e->negated && e->terms.size() == 2 &&
            e->terms[0]->k == T_VAR && e->terms[0]->s == t->s)
          return canon(e->terms[1], r, body, depth + 1, out);
      return false;
    }
    if (t->k == T_REF && t->head && t->head->k == T_VAR) {
      std::string h;
      if (!canon(t->head, r, body, depth + 1, &h)) return false;
      for (auto& i : t->items) {
        if (i->k != T_SCALAR) return false;
        h += "[" + std::to_string(i->stype) + ":" + i->s + "]";
      }
      *out = h;
      return true;
    }
    return false;
  }
  bool exclusive(const std::shared_ptr<Rule>& r1, const std::shared_ptr<Rule>& r2) {
    struct Test { std::string path, c; bool eq; };
    auto tests = [&](const std::shared_ptr<Rule>& r) {
      std::vector<Test> out;
      const auto& body = cbody(r, {});
      for (auto& e : body) {
        if (e->negated || e->kind != Expr::TERM || e->terms[0]->k != T_CALL) continue;
        const TermP& c = e->terms[0];
        if (c->op.size() != 1 || (c->op[0] != "equal" && c->op[0] != "neq") || c->items.size() != 2) continue;
        const TermP *p = &c->items[0], *k = &c->items[1];
        if ((*p)->k == T_SCALAR) std::swap(p, k);
        if ((*k)->k != T_SCALAR) continue;
        std::string ps;
        if (!canon(*p, r, body, 0, &ps)) continue;
        out.push_back({ps, std::to_string((*k)->stype) + ":" + (*k)->s, c->op[0] == "equal"});
      }
      return out;
    };
    for (auto& a : tests(r1))
      for (auto& b : tests(r2))
        if (a.path == b.path && a.c == b.c && a.eq != b.eq) return true;
    return false;
  }

  bool plan_join(const std::vector<ExprP>& body, size_t i, Env* env, JoinPlan& P) {
    const ExprP& e = body[i];
    if ((e->kind != Expr::ASSIGN && e->kind != Expr::UNIFY) || e->negated || !e->withs.empty() || e->terms.size() != 2)
      return false;
    const TermP& xv = e->terms[0];
    const TermP& ref = e->terms[1];
    if (xv->k != T_VAR || !unbound(env, xv) || env->lazy_lookup(xv->s)) return false;
    if (ref->k != T_REF || !ref->head || ref->head->k != T_VAR || ref->head->s != "data" || env->lookup("data") >= 0)
      return false;
    if (ref->items.empty() || ref->items[0]->k != T_SCALAR || ref->items[0]->s != "inventory") return false;
    if (bank_.inventory_node == 0xffffffffu) return false;
    P = JoinPlan{};
    P.x = xv->s;
    std::set<std::string> bound;  // bound by body[i..j)
    bound.insert(P.x);
    for (size_t q = 1; q < ref->items.size(); ++q) {
      const TermP& s = ref->items[q];
      JoinSite::Sel sel;
      if (s->k == T_SCALAR && s->stype == S_STR) {
        sel.sid = st_.intern(s->s);
      } else if (s->k == T_VAR && unbound(env, s) && !bound.count(s->s)) {
        sel.var = true;
        P.pvars.push_back(s->s);
        bound.insert(s->s);
      } else {
        return false;
      }
      P.path.push_back(sel);
    }
    if (P.pvars.empty()) return false;
    std::vector<std::set<std::string>> defs(body.size());
    for (size_t j = i + 1; j < body.size(); ++j) {
      const ExprP& ej = body[j];
      // the key equality: `A == K` / `A = K` with A bound before body[i]
      TermP l, r;
      if (!ej->negated && ej->withs.empty()) {
        if (ej->kind == Expr::TERM && ej->terms[0]->k == T_CALL && ej->terms[0]->op == std::vector<std::string>{"equal"} &&
            ej->terms[0]->items.size() == 2) {
          l = ej->terms[0]->items[0];
          r = ej->terms[0]->items[1];
        } else if (ej->kind == Expr::UNIFY && ej->terms.size() == 2) {
          l = ej->terms[0];
          r = ej->terms[1];
        }
      }
      auto outer = [&](const TermP& t) {
        return (t->k == T_VAR && !bound.count(t->s) && env->lookup(t->s) >= 0) || (t->k == T_SCALAR);
      };
      auto over_x = [&](const TermP& t) {
        std::set<std::string> vs;
        occ_vars(t, vs);
        bool dep = false;  // reads the leaf (directly or through a local derived from it)
        for (auto& v : vs) {
          if (bound.count(v)) { dep = true; continue; }
          if (is_global(env, v)) continue;
          if (env->lookup(v) >= 0 && env->pdef_lookup(v)) continue;
          if (v.rfind("$_", 0) == 0 && env->lookup(v) < 0) continue;  // a wildcard: several key values
          return false;
        }
        return dep;
      };
      if (l && r) {
        if (outer(r) && !outer(l)) std::swap(l, r);
        if (outer(l) && !outer(r) && over_x(r)) {
          P.a = l;
          P.key = r;
          // the key slice: definitions the key depends on, back to body[i]
          std::set<std::string> need;
          occ_vars(P.key, need);
          std::vector<bool> in_slice(j, false);
          for (size_t m = j; m-- > i + 1;) {
            std::string d;
            bool hit = false;
            for (auto& v : defs[m]) if (need.count(v)) hit = true;
            if (!hit) continue;
            std::set<std::string> pre;  // bound before body[m]
            pre.insert(P.x);
            for (auto& v : P.pvars) pre.insert(v);
            for (size_t q = i + 1; q < m; ++q) pre.insert(defs[q].begin(), defs[q].end());
            if (!defines(body[m], pre, env, &d)) return false;
            in_slice[m] = true;
            for (auto& v : expr_vars(body[m])) need.insert(v);
          }
          str_vars_ = &P.pvars;  // object keys: strings (engine.cc plan_joins checks the tree)
          for (size_t m = i + 1; m < j; ++m) {
            if (in_slice[m]) { P.slice.push_back(body[m]); continue; }
            if (!err_free_expr(body[m], env->mod, 0)) { str_vars_ = nullptr; return false; }  // skipped outside the bucket
          }
          str_vars_ = nullptr;
          // what the slice and key read besides the leaf: their own outputs,
          // globals (functions) and parameter-derived locals; never input or
          // the path variables (the key pass binds the leaf only)
          std::set<std::string> own;
          for (size_t m = i + 1; m < j; ++m) if (in_slice[m]) own.insert(defs[m].begin(), defs[m].end());
          for (auto& v : need) {
            if (v == P.x || own.count(v) || v.rfind("$_", 0) == 0) continue;
            if (is_global(env, v)) return false;  // input, data, rule references
            if (std::find(P.pvars.begin(), P.pvars.end(), v) != P.pvars.end()) return false;
            if (env->lookup(v) >= 0 && env->pdef_lookup(v)) { P.params.push_back(v); continue; }
            return false;
          }
          for (auto& s : P.slice)
            for (auto& t : s->terms) if (!input_free(t, env->mod, 0)) return false;
          if (!input_free(P.key, env->mod, 0)) return false;
          return true;
        }
      }
      // not the equality: what it binds (for later literals)
      std::string d;
      std::set<std::string> pre = bound;
      if (defines(ej, pre, env, &d)) { defs[j].insert(d); bound.insert(d); continue; }
      // any other literal must be a test over bound values (a generator or a
      // binding this planner does not follow ends the search)
      std::set<std::string> vs = expr_vars(ej);
      if (!ej->negated)
        for (auto& v : vs)
          if (!bound.count(v) && env->lookup(v) < 0 && !is_global(env, v)) return false;
    }
    return false;
  }

  // the key program of a join: input.review is the leaf; the slice, then the key
  JoinSite compile_key(const JoinPlan& P, const Env* env) {
    Comp sub(st_, mods_, bank_, false);
    Env kenv;
    kenv.mod = env->mod;
    sub.bind(&kenv, P.x, sub.input_root(true));
    const int Lend = sub.label();
    // the parameter-derived locals (each undefined parameter: no key), then
    // the slice and the key
    std::function<void(size_t, int)> params = [&](size_t q, int f) {
      if (q == P.params.size()) {
        sub.body_k(P.slice, 0, &kenv, f, [&](int f2) {
          // every value of the key (a generator in it yields several), then the next
          sub.term(P.key, &kenv, f2, [&](int r, int f3) {
            sub.emit(OP_KEYOUT, (uint16_t)r);
            sub.emit_jmp(OP_JMP, 0, f3);
          });
        });
        return;
      }
      const TermP* d = env->pdef_lookup(P.params[q]);
      if (!d) throw Unsupported("join key parameter");
      sub.term(*d, &kenv, f, [&, q](int r, int f2) {
        sub.bind(&kenv, P.params[q], r);
        params(q + 1, f2);
      });
    };
    params(0, Lend);
    sub.place(Lend);
    sub.emit(OP_END);
    Program kp = sub.finish();
    JoinSite js;
    js.path = P.path;
    js.nvars = (uint32_t)P.pvars.size();
    js.key_off = kp.code_off;
    js.key_len = kp.code_len;
    js.key_nregs = kp.nregs;
    if (js.key_nregs > 192) throw Unsupported("join key program registers");
    js.desc = "data.inventory";
    for (size_t q = 0; q < P.path.size(); ++q) js.desc += P.path[q].var ? "[_]" : "." + std::string(st_.str(P.path[q].sid));
    return js;
  }

  bool join_site(const std::vector<ExprP>& body, size_t i, Env* env, int fail, const KE& succ) {
    if (!joins_on() || guard_ || prog_.joins.size() >= JMAX_SITES) return false;
    JoinPlan P;
    if (!plan_join(body, i, env, P)) return false;
    JoinSite js;
    try {
      js = compile_key(P, env);
    } catch (const Unsupported&) {
      return false;  // the scan remains
    }
    const uint32_t site = (uint32_t)prog_.joins.size();
    prog_.joins.push_back(js);
    NoFuse nf(this);
    const int save = reg_top_;
    int av;
    if (P.a->k == T_SCALAR) av = loadk(scalar_val(P.a));
    else av = env->lookup(P.a->s);
    if (loop_base_.size() >= 15) throw Unsupported("loop nesting too deep");
    const int it = alloc(2);
    const int leaf = alloc();
    const int vb = alloc((int)P.pvars.size());
    const int Lscan = label();
    emit(OP_JPROBE, (uint16_t)it, (uint16_t)av, 0, (uint32_t)Lscan, ((uint32_t)loop_base_.size() + 1) | (site << 8));
    loop_base_.push_back(reg_top_);
    loop_var_lo_.push_back(it + 2);
    const int Ln = label();
    place(Ln);
    emit(OP_JNEXT, (uint16_t)it, (uint16_t)leaf, 0, (uint32_t)fail, (uint32_t)depth());
    for (size_t q = 0; q < P.pvars.size(); ++q) emit(OP_JVAR, (uint16_t)(vb + q), (uint16_t)it, 0, 0, (uint32_t)q);
    bind(env, P.x, leaf);
    for (size_t q = 0; q < P.pvars.size(); ++q) bind(env, P.pvars[q], vb + (int)q);
    body_k(body, i + 1, env, Ln, succ);
    for (auto& v : P.pvars) unbind(env, v);
    unbind(env, P.x);
    emit_jmp(OP_JMP, 0, Ln);
    close_loop();
    // no index for this lane: the iteration as written
    place(Lscan);
    reg_top_ = save;
    expr(body[i], env, fail, [&, i, env](int f) { body_k(body, i + 1, env, f, succ); });
    return true;
  }

  // `v = L[_]` over a lazy array L (lazy_def): each comprehension's body,
  // then `v = <its element>`, then the rest of this body, compiled in line --
  // the same solutions in the same order as lazy_iter, but a join inside a
  // comprehension (unique-label's `o = data.inventory.namespace[_][_][_][_]`)
  // now sees the key equality that follows the element's use.  Only when a
  // part has a join site.
  bool lazy_inline(const std::vector<ExprP>& body, size_t i, Env* env, int fail, const KE& succ) {
    if (!joins_on() || guard_) return false;
    const ExprP& e = body[i];
    if ((e->kind != Expr::ASSIGN && e->kind != Expr::UNIFY) || e->negated || !e->withs.empty() || e->terms.size() != 2)
      return false;
    const TermP& v = e->terms[0];
    const TermP& r = e->terms[1];
    if (v->k != T_VAR || !unbound(env, v) || r->k != T_REF || !r->head || r->head->k != T_VAR || r->items.size() != 1 ||
        !is_wild(r->items[0]))
      return false;
    const auto* lz = env->lazy_lookup(r->head->s);
    if (!lz) return false;
    std::vector<std::vector<ExprP>> bodies;
    bool any = false;
    for (auto& part : *lz) {
      for (auto& l : part.locals) if (env->lookup(l) >= 0) return false;
      std::vector<ExprP> b = part.compr->body;
      auto el = std::make_shared<Expr>();
      el->kind = Expr::UNIFY;
      el->terms = {v, part.compr->key};
      b.push_back(el);
      b.insert(b.end(), body.begin() + i + 1, body.end());
      for (size_t q = 0; q < part.compr->body.size() && !any; ++q) {
        JoinPlan P;
        any = plan_join(b, q, env, P);
      }
      bodies.push_back(std::move(b));
    }
    if (!any) return false;
    NoFuse nf(this);  // array order is observable
    for (size_t c = 0; c < bodies.size(); ++c) {
      const bool last = c + 1 == bodies.size();
      const int Lnext = last ? fail : label();
      body_k(bodies[c], 0, env, Lnext, succ);
      if (last) emit_jmp(OP_JMP, 0, fail);
      else place(Lnext);
    }
    return true;
  }

  void expr(const ExprP& e, Env* env, int fail, const KE& k) {
    if (!e->withs.empty()) throw Unsupported("with modifier in template");
    if (e->kind == Expr::SOME) { k(fail); return; }
    if (e->negated) {
      int save = reg_top_;
      int flag = loadk(tag_val(V_BOOL, 0));
      int Ld = label();
      Env inner;
      inner.parent = env;
      inner.mod = env->mod;
      int t = loadk(tag_val(V_BOOL, 1));
      expr_pos(e, &inner, Ld, [&](int f) { emit(OP_MOV, (uint16_t)flag, (uint16_t)t); emit_jmp(OP_JMP, 0, f); });
      place(Ld);
      emit_jmp(OP_JTRUE, flag, fail);
      k(fail);
      reg_top_ = save;
      return;
    }
    expr_pos(e, env, fail, k);
  }

  void expr_pos(const ExprP& e, Env* env, int fail, const KE& k) {
    if (e->kind == Expr::TERM) {
      const TermP& t = e->terms[0];
      if (t->k == T_CALL) {
        call(t, env, fail, true, [&](int r, int f) { emit_jmp(OP_JFALSE, r, f); k(f); });
      } else {
        // a statement-level ref: only its definedness/truthiness is observed
        // (rule_ref may then unify an object-pattern key member by member)
        stmt_key_ = (t->k == T_REF && !t->items.empty()) ? t->items.back().get() : nullptr;
        term(t, env, fail, [&](int r, int f) { emit_jmp(OP_JFALSE, r, f); k(f); });
        stmt_key_ = nullptr;
      }
      return;
    }
    unify(e->terms[0], e->terms[1], env, fail, k);
  }

  // ---------------------------------------------------------------- unify
  void bind(Env* env, const std::string& v, int r) { env->vars[v] = r; }
  void unbind(Env* env, const std::string& v) { env->vars.erase(v); env->pdef.erase(v); }

  bool pattern_has_unbound(const Env* env, const TermP& t) {
    std::vector<std::string> vs;
    term_vars(t, vs);
    for (auto& v : vs) if (env->lookup(v) < 0 && !is_global(env, v)) return true;
    return false;
  }

  void unify(const TermP& a, const TermP& b, Env* env, int fail, const KE& k) {
    if (unbound(env, a)) {
      term(b, env, fail, [&](int r, int f) {
        if (env->lookup(a->s) >= 0) {  // bound by a generator inside b
          int t = alloc();
          emit(OP_CMP, (uint16_t)t, (uint16_t)env->lookup(a->s), (uint16_t)r, 0, CMP_EQ);
          emit_jmp(OP_JFALSE, t, f);
          k(f);
          return;
        }
        bind(env, a->s, r);
        if (TermP d = param_def(env, b)) env->pdef[a->s] = d;
        k(f);
        unbind(env, a->s);
      });
      return;
    }
    if (unbound(env, b)) { unify(b, a, env, fail, k); return; }
    if ((a->k == T_ARRAY || a->k == T_OBJECT) && pattern_has_unbound(env, a)) {
      term(b, env, fail, [&](int r, int f) { unify_value(a, r, env, f, k); });
      return;
    }
    if ((b->k == T_ARRAY || b->k == T_OBJECT) && pattern_has_unbound(env, b)) {
      term(a, env, fail, [&](int r, int f) { unify_value(b, r, env, f, k); });
      return;
    }
    term(a, env, fail, [&](int ra, int f) {
      term(b, env, f, [&](int rb, int f2) {
        int t = alloc();
        emit(OP_CMP, (uint16_t)t, (uint16_t)ra, (uint16_t)rb, 0, CMP_EQ);
        emit_jmp(OP_JFALSE, t, f2);
        k(f2);
      });
    });
  }

  // unify a pattern term with the value in register r
  void unify_value(const TermP& p, int r, Env* env, int fail, const KE& k) {
    if (unbound(env, p)) {
      bind(env, p->s, r);
      k(fail);
      unbind(env, p->s);
      return;
    }
    if (p->k == T_ARRAY && pattern_has_unbound(env, p)) {
      int t = alloc();
      emit(OP_LEN_EQ, (uint16_t)t, (uint16_t)r, 0, 0, (uint32_t)p->items.size() | (LK_ARR << 24));
      emit_jmp(OP_JFALSE, t, fail);
      unify_items(p, r, 0, env, fail, k, false);
      return;
    }
    if (p->k == T_OBJECT && pattern_has_unbound(env, p)) {
      for (size_t i = 0; i < p->items.size(); i += 2)
        if (p->items[i]->k != T_SCALAR) throw Unsupported("object pattern with non-constant key");
      int t = alloc();
      emit(OP_LEN_EQ, (uint16_t)t, (uint16_t)r, 0, 0, (uint32_t)(p->items.size() / 2) | (LK_OBJ << 24));
      emit_jmp(OP_JFALSE, t, fail);
      unify_items(p, r, 0, env, fail, k, true);
      return;
    }
    term(p, env, fail, [&](int rp, int f) {
      int t = alloc();
      emit(OP_CMP, (uint16_t)t, (uint16_t)rp, (uint16_t)r, 0, CMP_EQ);
      emit_jmp(OP_JFALSE, t, f);
      k(f);
    });
  }
  void unify_items(const TermP& p, int r, size_t i, Env* env, int fail, const KE& k, bool obj) {
    size_t n = obj ? p->items.size() / 2 : p->items.size();
    if (i == n) { k(fail); return; }
    int v = alloc();
    uint64_t key = obj ? scalar_val(p->items[2 * i]) : tag_val(V_INT, i);
    emit(OP_GETK, (uint16_t)v, (uint16_t)r, 0, kconst(key));
    emit_jmp(OP_JUNDEF, v, fail);
    const TermP& sub = obj ? p->items[2 * i + 1] : p->items[i];
    unify_value(sub, v, env, fail, [&, i](int f) { unify_items(p, r, i + 1, env, f, k, obj); });
  }

  // ---------------------------------------------------------------- terms
  void term(const TermP& t, Env* env, int fail, const K& k) {
    switch (t->k) {
      case T_SCALAR: { int r = loadk(scalar_val(t)); k(r, fail); return; }
      case T_VAR: {
        int r = env->lookup(t->s);
        if (r >= 0) { k(r, fail); return; }
        auto tmp = std::make_shared<Term>();
        tmp->k = T_REF;
        tmp->head = t;
        ref(tmp, env, fail, k);
        return;
      }
      case T_REF: ref(t, env, fail, k); return;
      case T_CALL: call(t, env, fail, false, k); return;
      case T_ARRAY: case T_OBJECT:
        if (is_const(t)) { int r = loadk(const_value(t)); k(r, fail); return; }
        // fallthrough
      case T_SET: build_list(t, env, fail, k); return;
      case T_ARRCOMPR: case T_SETCOMPR: case T_OBJCOMPR: compr(t, env, fail, k); return;
    }
  }

  void build_list(const TermP& t, Env* env, int fail, const K& k) {
    uint32_t kind = t->k == T_SET ? LK_SET : t->k == T_ARRAY ? LK_ARR : LK_OBJ;
    items_k(t->items, 0, {}, env, fail, [&, kind](const std::vector<int>& regs, int f) {
      int l = alloc();
      emit(OP_LIST_NEW, (uint16_t)l, 0, 0, 0, kind);
      if (kind == LK_OBJ) {
        for (size_t i = 0; i < regs.size(); i += 2) emit(OP_OBJ_PUT, (uint16_t)l, (uint16_t)regs[i], (uint16_t)regs[i + 1], 0, escape_range(l));
      } else {
        for (int r : regs) emit(OP_LIST_ADD, (uint16_t)l, (uint16_t)r, 0, 0, escape_range(l));
      }
      k(l, f);
    });
  }

  using KV = std::function<void(const std::vector<int>&, int)>;
  void items_k(const std::vector<TermP>& items, size_t i, std::vector<int> acc, Env* env, int fail, const KV& k) {
    if (i == items.size()) { k(acc, fail); return; }
    term(items[i], env, fail, [&, i, acc](int r, int f) {
      auto a2 = acc;
      a2.push_back(r);
      items_k(items, i + 1, a2, env, f, k);
    });
  }

  void compr(const TermP& t, Env* env, int fail, const K& k) {
    NoFuse nf(this);  // array order is observable
    int save = reg_top_;
    uint32_t kind = t->k == T_SETCOMPR ? LK_SET : t->k == T_ARRCOMPR ? LK_ARR : LK_OBJ;
    int out = alloc();
    emit(OP_LIST_NEW, (uint16_t)out, 0, 0, 0, kind);
    int Ld = label();
    Env inner;
    inner.parent = env;
    inner.mod = env->mod;
    body_k(t->body, 0, &inner, Ld, [&](int f) {
      if (kind == LK_OBJ) {
        term(t->key, &inner, f, [&](int kr, int f2) {
          term(t->value, &inner, f2, [&](int vr, int f3) {
            emit(OP_OBJ_PUT, (uint16_t)out, (uint16_t)kr, (uint16_t)vr, 0, escape_range(out));
            emit_jmp(OP_JMP, 0, f3);
          });
        });
      } else {
        term(t->key, &inner, f, [&](int vr, int f2) {
          emit(OP_LIST_ADD, (uint16_t)out, (uint16_t)vr, 0, 0, escape_range(out));
          emit_jmp(OP_JMP, 0, f2);
        });
      }
    });
    place(Ld);
    k(out, fail);
    reg_top_ = save;
  }

  // ---------------------------------------------------------------- refs
  void ref(const TermP& t, Env* env, int fail, const K& k) {
    const TermP& head = t->head;
    const auto& path = t->items;
    if (head->k == T_CALL) {
      call(head, env, fail, false, [&](int r, int f) { walk(r, path, 0, env, f, k); });
      return;
    }
    if (head->k != T_VAR) throw Unsupported("ref head");
    int r = env->lookup(head->s);
    if (r >= 0) { walk(r, path, 0, env, fail, k); return; }
    if (const auto* lz = env->lazy_lookup(head->s)) {
      if (path.empty() || !is_wild(path[0])) throw Unsupported("lazy array use");
      lazy_iter(*lz, t, env, fail, k);
      return;
    }
    if (head->s == "input") {
      if (path.empty()) throw Unsupported("whole input document");
      const TermP& p0 = path[0];
      if (p0->k != T_SCALAR || p0->stype != S_STR) throw Unsupported("dynamic input key");
      std::vector<TermP> rest(path.begin() + 1, path.end());
      if (p0->s != "review" && p0->s != "parameters") { emit_jmp(OP_JMP, 0, fail); return; }  // input.<other> is undefined
      // the lane's input roots are loaded once, at program entry
      walk(input_root(p0->s == "review"), rest, 0, env, fail, k);
      return;
    }
    if (head->s == "data") { data_ref(path, env, fail, k); return; }
    if (env->mod) {
      auto rules = mods_.rules(env->mod->pkg, head->s);
      if (!rules.empty()) { rule_ref(rules, path, 0, env, fail, k); return; }
      for (auto& im : env->mod->imports) {
        if (im.second == head->s) {
          if (im.first.empty() || im.first[0] != "data") throw Unsupported("import of non-data document");
          std::vector<TermP> p2;
          for (size_t i = 1; i < im.first.size(); ++i) p2.push_back(mk_scalar(S_STR, im.first[i]));
          p2.insert(p2.end(), path.begin(), path.end());
          data_ref(p2, env, fail, k);
          return;
        }
      }
    }
    throw Unsupported("unsafe variable " + head->s);
  }

  void data_ref(const std::vector<TermP>& path, Env* env, int fail, const K& k) {
    std::vector<std::string> pkg;
    for (size_t i = 0; i < path.size(); ++i) {
      if (path[i]->k != T_SCALAR || path[i]->stype != S_STR) break;
      if (mods_.has_pkg(pkg)) {
        auto rules = mods_.rules(pkg, path[i]->s);
        if (!rules.empty()) { rule_ref(rules, path, i + 1, env, fail, k); return; }
      }
      pkg.push_back(path[i]->s);
    }
    if (!path.empty() && path[0]->k == T_SCALAR && path[0]->s == "inventory") {
      // data.inventory: regolib src.go:30-31,66-72 evaluates every template
      // `with data.inventory as data.external[target]` (or {} when absent);
      // the engine keeps that tree in the permanent node region behind one
      // node whose index is a constant here (engine.cc sync_inventory)
      if (bank_.inventory_node == 0xffffffffu) throw Unsupported("data.inventory (cross-resource join)");
      prog_.uses_inventory = true;
      int r = loadk(tag_val(V_NODE, bank_.inventory_node));
      walk(r, path, 1, env, fail, k);
      return;
    }
    throw Unsupported("reference to base data");
  }

  void walk(int r, const std::vector<TermP>& path, size_t i, Env* env, int fail, const K& k) {
    if (i == path.size()) { k(r, fail); return; }
    const TermP& sel = path[i];
    if (unbound(env, sel)) {
      int it = alloc(2);
      int kr = alloc(), vr = alloc();
      open_loop(it, r);
      int Ln = label();
      place(Ln);
      emit(OP_ITER_NEXT, (uint16_t)it, (uint16_t)kr, (uint16_t)vr, (uint32_t)fail, (uint32_t)depth());
      bind(env, sel->s, kr);
      walk(vr, path, i + 1, env, Ln, k);
      unbind(env, sel->s);
      emit_jmp(OP_JMP, 0, Ln);
      close_loop();
      return;
    }
    if (sel->k == T_SCALAR) {
      const uint64_t key = scalar_val(sel);
      if (lane_const(r) && lane_paths_on() && depth() > 0) {
        // inside a loop, a constant-key path below the lane's input (input.
        // review.kind.kind, input.parameters.cpu) is the same every iteration:
        // looked up at its first use, then read from one register (initially
        // false: a genuinely false value is just looked up again)
        size_t j = i;
        std::vector<uint64_t> keys;
        while (j < path.size() && path[j]->k == T_SCALAR) keys.push_back(scalar_val(path[j++]));
        auto lp = lpath_.find({r, keys});
        if (lp == lpath_.end() && lreg_n_ < kMaxLaneRegs) lp = lpath_.emplace(std::make_pair(r, keys), kLReg + lreg_n_++).first;
        if (lp != lpath_.end()) {
          const int v = lp->second;
          int Lhave = label(), Lcomp = label();
          emit_jmp(OP_JFALSE, v, Lcomp);
          emit_jmp(OP_JMP, 0, Lhave);
          place(Lcomp);
          int cur = r;
          for (uint64_t kk : keys) {
            int t = alloc();
            emit(OP_GETK, (uint16_t)t, (uint16_t)cur, 0, kconst(kk));  // vget of undefined is undefined
            cur = t;
          }
          emit(OP_MOV, (uint16_t)v, (uint16_t)cur);
          place(Lhave);
          emit_jmp(OP_JUNDEF, v, fail);
          walk(v, path, j, env, fail, k);
          return;
        }
      }
      auto pc = path_cache_.find({r, key});
      if (pc != path_cache_.end()) {  // looked up once per solution of a fused group's generator
        emit_jmp(OP_JUNDEF, pc->second, fail);
        walk(pc->second, path, i + 1, env, fail, k);
        return;
      }
      int v = alloc();
      emit(OP_GETK, (uint16_t)v, (uint16_t)r, 0, kconst(key));
      emit_jmp(OP_JUNDEF, v, fail);
      walk(v, path, i + 1, env, fail, k);
      return;
    }
    if ((sel->k == T_ARRAY || sel->k == T_OBJECT) && pattern_has_unbound(env, sel)) {
      // pattern selector: iterate members and unify
      int it = alloc(2);
      int kr = alloc(), vr = alloc();
      open_loop(it, r);
      int Ln = label();
      place(Ln);
      emit(OP_ITER_NEXT, (uint16_t)it, (uint16_t)kr, (uint16_t)vr, (uint32_t)fail, (uint32_t)depth());
      unify_value(sel, kr, env, Ln, [&](int f) { walk(vr, path, i + 1, env, f, k); });
      emit_jmp(OP_JMP, 0, Ln);
      close_loop();
      return;
    }
    term(sel, env, fail, [&, r, i](int kr, int f) {
      int v = alloc();
      emit(OP_GET, (uint16_t)v, (uint16_t)r, (uint16_t)kr);
      emit_jmp(OP_JUNDEF, v, f);
      walk(v, path, i + 1, env, f, k);
    });
  }

  // ---------------------------------------------------------------- rules
  void rule_ref(const std::vector<std::shared_ptr<Rule>>& rules, const std::vector<TermP>& path, size_t i, Env* env,
                int fail, const K& k) {
    auto kind = rules[0]->kind;
    if (kind == Rule::FUNC) throw Unsupported("function referenced without call");
    if (kind == Rule::COMPLETE) {
      complete_value(rules, fail, [&](int r, int f) { walk(r, path, i, env, f, k); });
      return;
    }
    if (kind == Rule::POBJ) throw Unsupported("partial object rule");
    // partial set
    bool stmt = i + 1 == path.size() && path[i].get() == stmt_key_;
    stmt_key_ = nullptr;
    if (i == path.size()) { full_set(rules, fail, k); return; }
    const TermP& key = path[i];
    // rule-head variables prebound from ground parts of the caller's key
    auto prebinds = [&](const std::shared_ptr<Rule>& r) {
      std::vector<std::pair<std::string, TermP>> pre_terms;
      if (r->key->k == T_VAR && ground(env, key)) pre_terms.push_back({r->key->s, key});
      if (r->key->k == T_OBJECT && key->k == T_OBJECT) {
        for (size_t a = 0; a < key->items.size(); a += 2) {
          if (key->items[a]->k != T_SCALAR) continue;
          for (size_t b = 0; b < r->key->items.size(); b += 2) {
            const TermP& hk = r->key->items[b];
            if (hk->k == T_SCALAR && hk->stype == key->items[a]->stype && hk->s == key->items[a]->s &&
                r->key->items[b + 1]->k == T_VAR && ground(env, key->items[a + 1]))
              pre_terms.push_back({r->key->items[b + 1]->s, key->items[a + 1]});
          }
        }
      }
      return pre_terms;
    };
    auto safe_of = [](const std::vector<std::pair<std::string, TermP>>& pts) {
      std::vector<std::string> safe;
      for (auto& pt : pts) safe.push_back(pt.first);
      return safe;
    };
    // the rule's key unified with the caller's key, then the caller's continuation
    auto head_k = [&](const std::shared_ptr<Rule>& r, Env* renv, int f2) {
      if (stmt && same_object_keys(key, r->key)) {
        // `s[{"msg": msg, "field": "x"}]` as a statement against a rule head
        // `s[{"msg": m, "field": f}]`: object unification is member-wise
        // unification over equal key sets, so the head object is never built
        unify_members(key, r->key, 0, env, renv, f2, [&](int f4) { int tr = loadk(tag_val(V_BOOL, 1)); k(tr, f4); });
        return;
      }
      term(r->key, renv, f2, [&](int kv, int f3) {
        unify_value(key, kv, env, f3, [&](int f4) { walk(kv, path, i + 1, env, f4, k); });
      });
    };
    for (size_t ri = 0; ri < rules.size();) {
      const auto& r = rules[ri];
      if (r->is_else) throw Unsupported("else");
      auto pre_terms = prebinds(r);
      const auto safe = safe_of(pre_terms);
      size_t rj = ri + 1;
      if (fuse_ok_ && !guard_)
        while (rj < rules.size() && fusable(rules[ri], rules[rj], pre_terms, prebinds(rules[rj]), safe)) ++rj;
      if (rj - ri >= 2) {
        rule_group(rules, ri, rj, pre_terms, safe, env, head_k);
        ri = rj;
        continue;
      }
      int save = reg_top_;
      int Lr = label();
      Env renv;
      renv.mod = r->mod;
      prebind(pre_terms, 0, env, &renv, Lr, [&](int f) {
        const auto& body = cbody(r, safe);
        body_k(body, 0, &renv, f, [&](int f2) { head_k(r, &renv, f2); });
      });
      place(Lr);
      reg_top_ = save;
      ++ri;
    }
    emit_jmp(OP_JMP, 0, fail);
  }

  // ---------------------------------------------------------------- rule groups
  // Consecutive bodies of one partial set whose first expression is the same
  // (the ContainerLimits shape: eight bodies each starting with
  // `container := input.review.object.spec[field][_]`) are fused: that
  // expression is evaluated once and, for each of its solutions, the rest of
  // every body in turn -- one pass over the containers instead of eight.
  // Rego bodies have no side effects, so the group yields the same solutions;
  // only their order changes (solution-major instead of body-major), and OP_ORD
  // keys let flush_wave number the emissions in the reference's body-major
  // order (devrt.h op_ord).  Errors and fallbacks abort the lane either way.
  // Fusion is confined to contexts whose solutions only reach emissions (not
  // comprehensions, function or complete-rule values, sets) and does not nest.
  bool fuse_ok_ = false;
  struct NoFuse {
    Comp* c;
    bool saved;
    explicit NoFuse(Comp* cc) : c(cc), saved(cc->fuse_ok_) { c->fuse_ok_ = false; }
    ~NoFuse() { c->fuse_ok_ = saved; }
  };

  static bool same_term(const TermP& a, const TermP& b) {
    if (a == b) return true;
    if (!a || !b) return false;
    // wildcards (`_`, renamed $_N by the parser) are each used once: any two match
    const bool wild = a->k == T_VAR && b->k == T_VAR && a->s.rfind("$_", 0) == 0 && b->s.rfind("$_", 0) == 0;
    if (a->k != b->k || a->stype != b->stype || (a->s != b->s && !wild) || a->op != b->op) return false;
    if (!same_term(a->head, b->head) || !same_term(a->key, b->key) || !same_term(a->value, b->value)) return false;
    if (a->items.size() != b->items.size() || a->body.size() != b->body.size()) return false;
    for (size_t x = 0; x < a->items.size(); ++x) if (!same_term(a->items[x], b->items[x])) return false;
    for (size_t x = 0; x < a->body.size(); ++x) if (!same_expr(a->body[x], b->body[x])) return false;
    return true;
  }
  static bool same_expr(const ExprP& a, const ExprP& b) {
    if (a->kind != b->kind || a->negated != b->negated || !a->withs.empty() || !b->withs.empty()) return false;
    if (a->terms.size() != b->terms.size()) return false;
    for (size_t x = 0; x < a->terms.size(); ++x) if (!same_term(a->terms[x], b->terms[x])) return false;
    return true;
  }

  bool fusable(const std::shared_ptr<Rule>& a, const std::shared_ptr<Rule>& b,
               const std::vector<std::pair<std::string, TermP>>& pa,
               const std::vector<std::pair<std::string, TermP>>& pb, const std::vector<std::string>& safe) {
    if (b->is_else || a->mod != b->mod || pa.size() != pb.size()) return false;
    for (size_t x = 0; x < pa.size(); ++x)
      if (pa[x].first != pb[x].first || pa[x].second.get() != pb[x].second.get()) return false;
    const auto& ba = cbody(a, safe);
    const auto& bb = cbody(b, safe);
    if (ba.size() < 2 || bb.size() < 2) return false;
    return ba[0]->kind != Expr::SOME && same_expr(ba[0], bb[0]);
  }

  // Shared lookups of a fused group: constant-key paths below the generator's
  // variable (`container.resources.limits`, `container.name`) that two or more
  // of the group's bodies read are looked up once per solution, in the group's
  // prologue, and walk() reads them from registers (keyed by (base register,
  // key), so a shadowing variable never hits).  A lookup is total and pure
  // (vget of a missing member or of a scalar is undefined), so evaluating it
  // ahead of the bodies changes nothing but the count of lookups.
  std::map<std::pair<int, uint64_t>, int> path_cache_;

  void collect_paths(const TermP& t, const std::string& var, std::vector<std::vector<TermP>>& out) {
    if (!t) return;
    if (t->k == T_REF && t->head && t->head->k == T_VAR && t->head->s == var) {
      std::vector<TermP> keys;
      for (auto& it : t->items) {
        if (it->k != T_SCALAR) break;
        keys.push_back(it);
      }
      if (!keys.empty()) out.push_back(keys);
    }
    collect_paths(t->head, var, out);
    collect_paths(t->key, var, out);
    collect_paths(t->value, var, out);
    for (auto& it : t->items) collect_paths(it, var, out);
    for (auto& e : t->body)
      for (auto& x : e->terms) collect_paths(x, var, out);
  }

  // prologue of a fused group: the shared paths under each variable the
  // generator bound (registers allocated here stay live for the bodies)
  void group_prologue(const std::vector<std::shared_ptr<Rule>>& rules, size_t lo, size_t hi,
                      const std::vector<std::string>& safe, const Env& renv, const Env* outer) {
    if (getenv("GKGPU_FUSE_CSE") && atoi(getenv("GKGPU_FUSE_CSE")) == 0) return;  // A/B switch, default on
    for (auto& vr : renv.vars) {
      if (outer && outer->lookup(vr.first) == vr.second) continue;  // bound before the generator
      std::map<std::vector<std::string>, std::set<size_t>> users;
      std::map<std::vector<std::string>, std::vector<TermP>> terms;
      for (size_t j = lo; j < hi; ++j) {
        const auto& body = cbody(rules[j], safe);
        std::vector<std::vector<TermP>> refs;
        for (size_t x = 1; x < body.size(); ++x)
          for (auto& t : body[x]->terms) collect_paths(t, vr.first, refs);
        for (auto& keys : refs)
          for (size_t n = 1; n <= keys.size(); ++n) {
            std::vector<std::string> sig;
            for (size_t q = 0; q < n; ++q) sig.push_back(std::to_string(keys[q]->stype) + ":" + keys[q]->s);
            users[sig].insert(j);
            terms[sig] = std::vector<TermP>(keys.begin(), keys.begin() + n);
          }
      }
      std::map<std::vector<std::string>, int> reg_of;  // ordered: a prefix precedes its extensions
      for (auto& u : users) {
        if (u.second.size() < 2 || reg_of.size() >= 12) continue;
        const auto& keys = terms[u.first];
        int base = vr.second;
        if (keys.size() > 1) {
          auto pit = reg_of.find(std::vector<std::string>(u.first.begin(), u.first.end() - 1));
          if (pit == reg_of.end()) continue;
          base = pit->second;
        }
        const uint64_t key = scalar_val(keys.back());
        int v = alloc();
        emit(OP_GETK, (uint16_t)v, (uint16_t)base, 0, kconst(key));
        reg_of[u.first] = v;
        path_cache_[{base, key}] = v;
      }
    }
  }

  using HeadK = std::function<void(const std::shared_ptr<Rule>&, Env*, int)>;
  void rule_group(const std::vector<std::shared_ptr<Rule>>& rules, size_t lo, size_t hi,
                  const std::vector<std::pair<std::string, TermP>>& pre_terms, const std::vector<std::string>& safe,
                  Env* env, const HeadK& head_k) {
    NoFuse nf(this);
    int save = reg_top_;
    int Lg = label();
    Env renv;
    renv.mod = rules[lo]->mod;
    prebind(pre_terms, 0, env, &renv, Lg, [&](int f) {
      fused_bodies(rules, lo, hi, safe, &renv, env, f, [&](size_t j, Env* e2, int f2) { head_k(rules[j], e2, f2); });
    });
    place(Lg);
    emit(OP_ORD, 0, 0, 0, 0, 0x80000000u | (uint32_t)(hi - lo));
    reg_top_ = save;
  }

  // the shared first expression of rules [lo, hi), then per solution the rest
  // of each body in turn (OP_ORD key j - lo), each ending in tail(j, env, fail)
  void fused_bodies(const std::vector<std::shared_ptr<Rule>>& rules, size_t lo, size_t hi,
                    const std::vector<std::string>& safe, Env* renv, const Env* outer, int fail,
                    const std::function<void(size_t, Env*, int)>& tail) {
    const auto& first = cbody(rules[lo], safe);
    expr(first[0], renv, fail, [&](int fnext) {
      auto saved_cache = path_cache_;
      group_prologue(rules, lo, hi, safe, *renv, outer);
      const int save2 = reg_top_;
      for (size_t j = lo; j < hi; ++j) {
        const auto& r = rules[j];
        const auto& body = cbody(r, safe);
        int Ln = label();
        emit(OP_ORD, 0, 0, 0, 0, (uint32_t)(j - lo));
        Env e2;
        e2.mod = r->mod;
        e2.parent = renv->parent;
        e2.vars = renv->vars;
        body_k(body, 1, &e2, Ln, [&, j](int f2) { tail(j, &e2, f2); });
        place(Ln);
        reg_top_ = save2;
      }
      path_cache_ = saved_cache;
      emit_jmp(OP_JMP, 0, fnext);
    });
  }

  // both object literals with scalar keys, the same key set, no duplicates
  static bool same_object_keys(const TermP& a, const TermP& b) {
    if (a->k != T_OBJECT || b->k != T_OBJECT || a->items.size() != b->items.size()) return false;
    for (size_t x = 0; x < a->items.size(); x += 2) {
      const TermP& ka = a->items[x];
      if (ka->k != T_SCALAR) return false;
      int found = 0;
      for (size_t y = 0; y < b->items.size(); y += 2) {
        const TermP& kb = b->items[y];
        if (kb->k != T_SCALAR) return false;
        if (kb->stype == ka->stype && kb->s == ka->s) ++found;
      }
      if (found != 1) return false;
      for (size_t z = x + 2; z < a->items.size(); z += 2)
        if (a->items[z]->k == T_SCALAR && a->items[z]->stype == ka->stype && a->items[z]->s == ka->s) return false;
    }
    return true;
  }

  void unify_members(const TermP& pat, const TermP& head, size_t x, Env* env, Env* renv, int fail, const KE& k) {
    if (x == pat->items.size()) { k(fail); return; }
    const TermP& ka = pat->items[x];
    size_t y = 0;
    while (!(head->items[y]->stype == ka->stype && head->items[y]->s == ka->s)) y += 2;
    term(head->items[y + 1], renv, fail, [&, x](int hv, int f) {
      unify_value(pat->items[x + 1], hv, env, f, [&, x](int f2) { unify_members(pat, head, x + 2, env, renv, f2, k); });
    });
  }

  void prebind(const std::vector<std::pair<std::string, TermP>>& pts, size_t i, Env* caller, Env* renv, int fail,
               const KE& k) {
    if (i == pts.size()) { k(fail); return; }
    term(pts[i].second, caller, fail, [&, i](int r, int f) {
      bind(renv, pts[i].first, r);
      prebind(pts, i + 1, caller, renv, f, k);
    });
  }

  void full_set(const std::vector<std::shared_ptr<Rule>>& rules, int fail, const K& k) {
    NoFuse nf(this);
    int save = reg_top_;
    int out = alloc();
    emit(OP_LIST_NEW, (uint16_t)out, 0, 0, 0, LK_SET);
    for (auto& r : rules) {
      int Lr = label();
      Env renv;
      renv.mod = r->mod;
      body_k(cbody(r, {}), 0, &renv, Lr, [&](int f) {
        term(r->key, &renv, f, [&](int kv, int f2) { emit(OP_LIST_ADD, (uint16_t)out, (uint16_t)kv, 0, 0, escape_range(out)); emit_jmp(OP_JMP, 0, f2); });
      });
      place(Lr);
    }
    k(out, fail);
    reg_top_ = save;
  }

  void complete_value(const std::vector<std::shared_ptr<Rule>>& rules, int fail, const K& k) {
    NoFuse nf(this);
    auto it = crule_.find(rules[0].get());
    if (it == crule_.end() && crule_.size() < kMaxCachedRules) {
      int n = (int)crule_.size();
      it = crule_.emplace(rules[0].get(), std::make_pair(kVReg + 2 * n, kVReg + 2 * n + 1)).first;
    }
    if (it == crule_.end()) { complete_eval(rules, fail, k); return; }
    int val = it->second.first, done = it->second.second;
    int Lhave = label();
    emit_jmp(OP_JTRUE, done, Lhave);
    {
      int save = reg_top_;
      // the value outlives every enclosing loop's iteration heap: pin them all
      uint32_t rng = depth() ? (1u | ((uint32_t)depth() << 8)) : 0u;
      int u = loadk(tag_val(V_UNDEF, 0));
      emit(OP_MOV, (uint16_t)val, (uint16_t)u);
      complete_into(rules, val, rng);
      int t = loadk(tag_val(V_BOOL, 1));
      emit(OP_MOV, (uint16_t)done, (uint16_t)t);
      reg_top_ = save;
    }
    place(Lhave);
    emit_jmp(OP_JUNDEF, val, fail);
    k(val, fail);
  }

  // all bodies of a complete rule yield into `out` (conflicting values are an
  // error; a constant default applies when none is defined)
  void complete_into(const std::vector<std::shared_ptr<Rule>>& rules, int out, uint32_t rng) {
    TermP def;
    for (auto& r : rules) {
      if (r->is_else) throw Unsupported("else");
      if (r->is_default) { def = r->value; continue; }
      int Lr = label();
      Env renv;
      renv.mod = r->mod;
      body_k(cbody(r, {}), 0, &renv, Lr, [&](int f) {
        term(r->value, &renv, f, [&](int v, int f2) { emit(OP_YIELD, (uint16_t)out, (uint16_t)v, 0, 0, rng); emit_jmp(OP_JMP, 0, f2); });
      });
      place(Lr);
    }
    if (def) {
      if (!is_const(def)) throw Unsupported("non-constant default");
      int Lh = label();
      int dv = loadk(const_value(def));
      int Lskip = label();
      emit_jmp(OP_JUNDEF, out, Lh);
      emit_jmp(OP_JMP, 0, Lskip);
      place(Lh);
      emit(OP_MOV, (uint16_t)out, (uint16_t)dv);
      place(Lskip);
    }
  }

  void complete_eval(const std::vector<std::shared_ptr<Rule>>& rules, int fail, const K& k) {
    NoFuse nf(this);
    int save = reg_top_;
    int out = loadk(tag_val(V_UNDEF, 0));
    TermP def;
    for (auto& r : rules) {
      if (r->is_else) throw Unsupported("else");
      if (r->is_default) { def = r->value; continue; }
      int Lr = label();
      Env renv;
      renv.mod = r->mod;
      body_k(cbody(r, {}), 0, &renv, Lr, [&](int f) {
        term(r->value, &renv, f, [&](int v, int f2) { emit(OP_YIELD, (uint16_t)out, (uint16_t)v, 0, 0, escape_range(out)); emit_jmp(OP_JMP, 0, f2); });
      });
      place(Lr);
    }
    if (def) {
      if (!is_const(def)) throw Unsupported("non-constant default");
      int Lh = label();
      int dv = loadk(const_value(def));
      int Lskip = label();
      emit_jmp(OP_JUNDEF, out, Lh);
      emit_jmp(OP_JMP, 0, Lskip);
      place(Lh);
      emit(OP_MOV, (uint16_t)out, (uint16_t)dv);
      place(Lskip);
    }
    emit_jmp(OP_JUNDEF, out, fail);
    k(out, fail);
    reg_top_ = save;
  }

  // ---------------------------------------------------------------- calls
  std::vector<std::shared_ptr<Rule>> resolve_func(const std::vector<std::string>& op, const Env* env) {
    if (op.size() == 1 && env->mod) {
      auto r = mods_.rules(env->mod->pkg, op[0]);
      if (!r.empty()) return r;
      for (auto& im : env->mod->imports)
        if (im.second == op[0] && !im.first.empty() && im.first[0] == "data") {
          std::vector<std::string> pkg(im.first.begin() + 1, im.first.end() - 1);
          return mods_.rules(pkg, im.first.back());
        }
      return {};
    }
    std::vector<std::string> full;
    if (op[0] == "data") full.assign(op.begin() + 1, op.end());
    else if (env->mod) {
      for (auto& im : env->mod->imports)
        if (im.second == op[0] && !im.first.empty() && im.first[0] == "data") {
          full.assign(im.first.begin() + 1, im.first.end());
          full.insert(full.end(), op.begin() + 1, op.end());
        }
    }
    if (full.empty()) return {};
    std::vector<std::string> pkg(full.begin(), full.end() - 1);
    return mods_.rules(pkg, full.back());
  }

  void call(const TermP& t, Env* env, int fail, bool stmt, const K& k) {
    NoFuse nf(this);  // function values (and builtin arguments) are not emissions
    std::string name;
    for (size_t i = 0; i < t->op.size(); ++i) name += (i ? "." : "") + t->op[i];
    auto rules = resolve_func(t->op, env);
    if (!rules.empty()) {
      if (rules[0]->kind != Rule::FUNC) throw Unsupported("call of non-function rule " + name);
      size_t nargs = rules[0]->args.size();
      bool has_out = t->items.size() == nargs + 1;
      if (!has_out && t->items.size() != nargs) throw Unsupported("arity mismatch " + name);
      std::vector<TermP> args(t->items.begin(), t->items.begin() + nargs);
      int tab = table_func(rules, stmt && !has_out);
      items_k(args, 0, {}, env, fail, [&, has_out, tab](const std::vector<int>& regs, int f) {
        int out;
        if (tab >= 0) {
          out = alloc();
          emit(OP_TABLE, (uint16_t)out, (uint16_t)regs[0], 0, (uint32_t)tab);
        } else {
          out = loadk(tag_val(V_UNDEF, 0));
          // A call whose argument is computed inside the innermost loop (the
          // loop's element, a path below it) meets new arguments every
          // iteration; an impure function's lane memo would only cost
          // registers there.  Pure functions keep theirs: the cross-lane memo
          // serves other lanes.
          bool varying = false;
          if (!loop_var_lo_.empty())
            for (int r : regs) varying |= r >= loop_var_lo_.back() && r < kVReg;
          bool skip = varying && !pure_func(rules);
          // the set rewrites' helpers (rego.cc optimize_sets) take a document
          // collection as an argument: a memo key nobody else meets
          skip = skip || name.rfind("__gk_", 0) == 0;
          int slot = nargs >= 1 && nargs <= 2 && !skip ? memo_slot(rules, stmt && !has_out) : -1;
          int Lhit = label();
          uint16_t k1 = nargs == 2 ? (uint16_t)regs[1] : NOREG;
          if (slot >= 0) emit(OP_MEMO_GET, (uint16_t)out, (uint16_t)regs[0], k1, (uint32_t)Lhit, (uint32_t)slot);
          if (++inline_depth_ > 64) throw Unsupported("recursion / inline depth");
          // every body yields one constant and none can err: the first
          // solution is the value (OPA would go on through the other bodies
          // and solutions only to find the same value; GKGPU_FN_EARLY=1, A/B)
          const int Ldone = early_exit_ok(rules) ? label() : -1;
          for (auto& r : rules) inline_func(r, regs, out, stmt && !has_out, Ldone);
          if (Ldone >= 0) place(Ldone);
          --inline_depth_;
          if (slot >= 0) emit(OP_MEMO_PUT, (uint16_t)out, (uint16_t)regs[0], k1, pure_func(rules) ? 1u : 0u, (uint32_t)slot);
          place(Lhit);
        }
        emit_jmp(OP_JUNDEF, out, f);
        if (has_out) {
          unify_value(t->items.back(), out, env, f, [&](int f2) { int tr = loadk(tag_val(V_BOOL, 1)); k(tr, f2); });
        } else {
          k(out, f);
        }
      });
      return;
    }
    std::string op = name;
    auto ci = kCmp.find(op);
    auto ai = kArith.find(op);
    if (ci != kCmp.end() || ai != kArith.end()) {
      bool has_out = t->items.size() == 3;
      if (t->items.size() != 2 && !has_out) throw Unsupported("operator arity");
      std::vector<TermP> args(t->items.begin(), t->items.begin() + 2);
      items_k(args, 0, {}, env, fail, [&, has_out](const std::vector<int>& regs, int f) {
        int d = alloc();
        if (ci != kCmp.end()) emit(OP_CMP, (uint16_t)d, (uint16_t)regs[0], (uint16_t)regs[1], 0, ci->second);
        else emit(OP_ARITH, (uint16_t)d, (uint16_t)regs[0], (uint16_t)regs[1], 0, ai->second);
        finish_call(t, d, has_out, env, f, k);
      });
      return;
    }
    if (op == "sprintf") {
      bool has_out = t->items.size() == 3;
      const TermP& fmt = t->items[0];
      if (fmt->k != T_SCALAR || fmt->stype != S_STR) throw Unsupported("sprintf with non-constant format");
      uint32_t fidx = parse_format(fmt->s);
      term(t->items[1], env, fail, [&, has_out, fidx](int ar, int f) {
        int d = alloc();
        emit(OP_SPRINTF, (uint16_t)d, (uint16_t)ar, 0, fidx);
        finish_call(t, d, has_out, env, f, k);
      });
      return;
    }
    auto bi = kBuiltins.find(op);
    if (bi == kBuiltins.end()) throw Unsupported("builtin " + op);
    int arity = kArity.at(bi->second);
    bool has_out = (int)t->items.size() == arity + 1;
    if ((int)t->items.size() != arity && !has_out) throw Unsupported("builtin arity " + op);
    if (bi->second == BI_RE_MATCH) {
      prog_.uses_regex = true;
      if (t->items[0]->k == T_SCALAR && t->items[0]->stype == S_STR) prog_.regex_literals.push_back(st_.intern(t->items[0]->s));
    }
    std::vector<TermP> args(t->items.begin(), t->items.begin() + arity);
    uint32_t id = bi->second;
    items_k(args, 0, {}, env, fail, [&, has_out, id, arity](const std::vector<int>& regs, int f) {
      int base = alloc(arity);
      for (int i = 0; i < arity; ++i) emit(OP_MOV, (uint16_t)(base + i), (uint16_t)regs[i]);
      int d = alloc();
      emit(OP_CALL, (uint16_t)d, (uint16_t)base, (uint16_t)arity, 0, id);
      finish_call(t, d, has_out, env, f, k);
    });
  }

  void finish_call(const TermP& t, int d, bool has_out, Env* env, int f, const K& k) {
    if (has_out) {
      unify_value(t->items.back(), d, env, f, [&](int f2) { int tr = loadk(tag_val(V_BOOL, 1)); k(tr, f2); });
    } else {
      k(d, f);
    }
  }

  // A function is pure when nothing under it refers to input, data, a rule of
  // the package or an import: its value is then a function of its arguments
  // alone, the same in every lane, so template kernels share it across lanes
  // (devrt.h gm_get / gm_put; flagged by x = 1 on its OP_MEMO_PUT).
  std::map<const Rule*, int> pure_;  // 1 pure, 2 impure, 3 being checked
  bool pure_func(const std::vector<std::shared_ptr<Rule>>& rules) {
    for (auto& r : rules) {
      auto it = pure_.find(r.get());
      if (it != pure_.end()) {
        if (it->second != 1) return false;
        continue;
      }
      pure_[r.get()] = 3;
      Env env;
      env.mod = r->mod;
      bool ok = r->kind == Rule::FUNC && !r->is_else;
      for (auto& a : r->args) ok = ok && pure_term(a, &env);
      ok = ok && pure_term(r->value, &env) && pure_body(r->body, &env);
      pure_[r.get()] = ok ? 1 : 2;
      if (!ok) return false;
    }
    return true;
  }
  bool pure_body(const std::vector<ExprP>& body, Env* env) {
    for (auto& e : body) {
      if (!e->withs.empty()) return false;
      for (auto& t : e->terms) if (!pure_term(t, env)) return false;
    }
    return true;
  }
  bool pure_term(const TermP& t, Env* env) {
    if (!t) return true;
    switch (t->k) {
      case T_SCALAR: return true;
      case T_VAR: return !is_global(env, t->s);
      case T_CALL: {
        if (t->op.empty()) return false;
        auto fr = resolve_func(t->op, env);
        if (!fr.empty()) {
          if (!pure_func(fr)) return false;
        } else if (t->op[0] == "input" || t->op[0] == "data" || is_global(env, t->op[0])) {
          return false;
        }
        for (auto& a : t->items) if (!pure_term(a, env)) return false;
        return true;
      }
      default: break;
    }
    if (!pure_term(t->head, env) || !pure_term(t->key, env) || !pure_term(t->value, env)) return false;
    for (auto& a : t->items) if (!pure_term(a, env)) return false;
    return pure_body(t->body, env);
  }

  // One memo slot per (function, statement-form) per template; see devrt.h
  // memo_stable for which values are cached.  -1 once the slots run out.
  int memo_slot(const std::vector<std::shared_ptr<Rule>>& rules, bool stmt) {
    auto key = std::make_pair((const void*)rules[0].get(), stmt);
    auto it = memo_.find(key);
    if (it != memo_.end()) return it->second;
    if (memo_.size() >= MEMO_SLOTS) return -1;
    int s = (int)memo_.size();
    memo_[key] = s;
    return s;
  }

  // A one-argument function whose every definition is `f("key") = scalar { true }`
  // is a constant table: the argument unifies with at most one distinct key, so
  // evaluating all bodies (topdown evalFunc) reduces to one lookup.  Duplicate
  // keys must carry the same value text (else the general path reports the
  // conflict at run time).  As a statement (`f(x)` without output) a `false`
  // value makes the call undefined, so such entries are left out.  Returns the
  // table's offset in the constant bank, or -1.
  int table_func(const std::vector<std::shared_ptr<Rule>>& rules, bool stmt) {
    std::vector<std::pair<uint64_t, uint64_t>> ents;
    std::map<std::string, std::string> seen;
    for (auto& r : rules) {
      if (r->kind != Rule::FUNC || r->is_else || r->is_default || r->args.size() != 1) return -1;
      const TermP& a = r->args[0];
      if (a->k != T_SCALAR || a->stype != S_STR) return -1;
      if (!r->value || r->value->k != T_SCALAR) return -1;
      for (auto& e : r->body) {
        if (e->kind != Expr::TERM || e->negated || !e->withs.empty() || e->terms.size() != 1) return -1;
        if (e->terms[0]->k != T_SCALAR || e->terms[0]->stype != S_TRUE) return -1;
      }
      std::string vt = std::to_string(r->value->stype) + ":" + r->value->s;
      auto it = seen.find(a->s);
      if (it != seen.end()) {
        if (it->second != vt) return -1;
        continue;
      }
      seen[a->s] = vt;
      if (stmt && r->value->stype == S_FALSE) continue;
      ents.push_back({scalar_val(a), scalar_val(r->value)});
    }
    if (rules.empty()) return -1;
    uint32_t off = (uint32_t)bank_.consts.size();
    bank_.consts.push_back(ents.size());
    for (auto& e : ents) { bank_.consts.push_back(e.first); bank_.consts.push_back(e.second); }
    return (int)off;
  }

  bool early_exit_ok(const std::vector<std::shared_ptr<Rule>>& rules) {
    // default on (GKGPU_FN_EARLY=0: off, A/B): profiles/r05/r05a_early_ab.txt,
    // K8sRequiredProbes 1.85 -> 1.67 ms (config 2), 5.10 -> 4.58 ms (config 4)
    static const bool on = !getenv("GKGPU_FN_EARLY") || atoi(getenv("GKGPU_FN_EARLY")) != 0;
    if (!on || rules.empty()) return false;
    for (auto& r : rules)
      if (!r->value || !is_const(r->value) || !same_term(r->value, rules[0]->value)) {
        if (getenv("GKGPU_FN_TRACE")) fprintf(stderr, "fn %s: value not one constant\n", rules[0]->name.c_str());
        return false;
      }
    const bool ok = fn_err_free(rules, 0);
    if (getenv("GKGPU_FN_TRACE")) fprintf(stderr, "fn %s: early exit %s\n", rules[0]->name.c_str(), ok ? "yes" : "no");
    return ok;
  }

  void inline_func(const std::shared_ptr<Rule>& r, const std::vector<int>& args, int out, bool stmt, int done = -1) {
    if (r->is_else) throw Unsupported("else in function");
    int save = reg_top_;
    int Lend = label();
    Env fenv;
    fenv.mod = r->mod;
    args_k(r, args, 0, &fenv, Lend, [&](int f) {
      body_k(cbody(r, {}), 0, &fenv, f, [&](int f2) {
        term(r->value, &fenv, f2, [&](int v, int f3) {
          if (stmt) emit_jmp(OP_JFALSE, v, f3);
          emit(OP_YIELD, (uint16_t)out, (uint16_t)v, 0, 0, escape_range(out));
          emit_jmp(OP_JMP, 0, done >= 0 ? done : f3);
        });
      });
    });
    place(Lend);
    reg_top_ = save;
  }

  void args_k(const std::shared_ptr<Rule>& r, const std::vector<int>& args, size_t i, Env* fenv, int fail, const KE& k) {
    if (i == args.size()) { k(fail); return; }
    const TermP& p = r->args[i];
    if (p->k == T_VAR && fenv->lookup(p->s) < 0) {
      bind(fenv, p->s, args[i]);
      args_k(r, args, i + 1, fenv, fail, k);
      return;
    }
    unify_value(p, args[i], fenv, fail, [&, i](int f) { args_k(r, args, i + 1, fenv, f, k); });
  }

  // ---------------------------------------------------------------- sprintf
  // format words: [nseg, (kind, a)...]; kind 0 literal (a = string id), 1 = %v/%s/%d arg (a = arg idx | verb<<16),
  // 2 = extra-args marker (Go %!(EXTRA ...)) handled at run time, 3 = missing arg (a = verb)
  uint32_t parse_format(const std::string& f) {
    std::vector<uint32_t> w;
    std::string lit;
    uint32_t argi = 0;
    auto flush = [&]() {
      if (!lit.empty()) { w.push_back(0); w.push_back(st_.intern(lit)); lit.clear(); }
    };
    for (size_t i = 0; i < f.size(); ++i) {
      if (f[i] != '%') { lit.push_back(f[i]); continue; }
      if (i + 1 >= f.size()) throw Unsupported("sprintf: trailing %");
      char v = f[++i];
      if (v == '%') { lit.push_back('%'); continue; }
      if (v != 'v' && v != 's' && v != 'd') throw Unsupported(std::string("sprintf verb %") + v);
      flush();
      w.push_back(1);
      w.push_back(argi++ | ((uint32_t)v << 16));
    }
    flush();
    uint32_t off = (uint32_t)bank_.fmt.size();
    bank_.fmt.push_back((uint32_t)w.size() / 2);
    bank_.fmt.push_back(argi);  // expected arg count
    bank_.fmt.insert(bank_.fmt.end(), w.begin(), w.end());
    return off;
  }

  // ---------------------------------------------------------------- emit
  void emit_violation(const std::shared_ptr<Rule>& r, Env* env, int idx, int f) {
    const TermP& key = r->key;
    if (key->k == T_OBJECT) {
      TermP msg, det;
      bool ok = true;
      for (size_t i = 0; i < key->items.size(); i += 2) {
        if (key->items[i]->k != T_SCALAR) { ok = false; break; }
        if (key->items[i]->stype == S_STR && key->items[i]->s == "msg") msg = key->items[i + 1];
        if (key->items[i]->stype == S_STR && key->items[i]->s == "details") det = key->items[i + 1];
      }
      if (ok) {
        if (!msg) { emit_jmp(OP_JMP, 0, f); return; }
        term(msg, env, f, [&](int mr, int f2) {
          if (det) {
            term(det, env, f2, [&](int dr, int f3) {
              emit(OP_EMIT, (uint16_t)mr, (uint16_t)dr, (uint16_t)depth(), 0, (uint32_t)idx);
              emit_jmp(OP_JMP, 0, f3);
            });
          } else {
            emit(OP_EMIT, (uint16_t)mr, NOREG, (uint16_t)depth(), 0, (uint32_t)idx);
            emit_jmp(OP_JMP, 0, f2);
          }
        });
        return;
      }
    }
    term(key, env, f, [&](int kv, int f2) {
      int m = alloc(), d = alloc();
      emit(OP_GETK, (uint16_t)m, (uint16_t)kv, 0, kconst(tag_val(V_STR, st_.s_msg)));
      emit_jmp(OP_JUNDEF, m, f2);
      emit(OP_GETK, (uint16_t)d, (uint16_t)kv, 0, kconst(tag_val(V_STR, st_.s_details)));
      emit(OP_EMIT, (uint16_t)m, (uint16_t)d, (uint16_t)depth(), 0, (uint32_t)idx);
      emit_jmp(OP_JMP, 0, f2);
    });
  }
};

}  // namespace

static Program compile_impl(Store& st, const ModuleSet& mods, const std::vector<std::string>& pkg, CodeBank& bank,
                            bool guard) {
  // a failed template leaves no code behind in the shared bank
  size_t code0 = bank.code.size(), k0 = bank.consts.size(), f0 = bank.fmt.size();
  try {
    Comp c(st, mods, bank, guard);
    return c.run(pkg);
  } catch (...) {
    bank.code.resize(code0);
    bank.consts.resize(k0);
    bank.fmt.resize(f0);
    throw;
  }
}

Program compile_template(Store& st, const ModuleSet& mods, const std::vector<std::string>& pkg, CodeBank& bank) {
  return compile_impl(st, mods, pkg, bank, false);
}

Program compile_template_guard(Store& st, const ModuleSet& mods, const std::vector<std::string>& pkg, CodeBank& bank) {
  return compile_impl(st, mods, pkg, bank, true);
}

}  // namespace gk
