// Rego subset lexer/parser and OPA compiler rewrites (host side).
//
// Grammar precedence follows OPA's: relation < `|` < `&` < `+ -` < `* / %`.
// Rewrites mirror vendor/github.com/open-policy-agent/opa/ast/compile.go:
//   * RewriteExprTerms (expandExpr/expandExprTerm, compile.go:2967-3104):
//     nested calls are hoisted into `f(args..., $lN)` expressions;
//   * CheckSafetyRuleBodies (reorderBodyForSafety): expressions are moved after
//     the ones that bind their inputs;
//   * RewriteDynamicTerms (compile.go:2828-2960): call-argument refs and
//     ref-valued selectors rooted at global documents are hoisted into
//     `$lN = ref` before the expression (observable inside `not`; pinned by
//     pkg/target/regolib/autoreject_test.rego:test_with_undefined_ns vs
//     util_test.rego:test_has_field_no_field).
#include "rego.h"

#include <algorithm>
#include <set>
#include <stdexcept>

namespace gk {
namespace rego {

TermP mk_scalar(int stype, const std::string& s) {
  auto t = std::make_shared<Term>();
  t->k = T_SCALAR;
  t->stype = stype;
  t->s = s;
  return t;
}
TermP mk_var(const std::string& name) {
  auto t = std::make_shared<Term>();
  t->k = T_VAR;
  t->s = name;
  return t;
}
TermP mk_call(const std::vector<std::string>& op, const std::vector<TermP>& args) {
  auto t = std::make_shared<Term>();
  t->k = T_CALL;
  t->op = op;
  t->items = args;
  return t;
}
static TermP mk(TermKind k) {
  auto t = std::make_shared<Term>();
  t->k = k;
  return t;
}

// ------------------------------------------------------------------ lexer
namespace {
enum TokKind { K_EOF, K_NL, K_IDENT, K_STR, K_NUM, K_OP };
struct Tok {
  TokKind k;
  std::string text;  // identifier / op / number text / unquoted string
  int line;
};

bool is_ident_start(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_'; }
bool is_ident(char c) { return is_ident_start(c) || (c >= '0' && c <= '9'); }

void put_utf8(std::string& b, uint32_t cp) {
  if (cp < 0x80) b.push_back((char)cp);
  else if (cp < 0x800) { b.push_back((char)(0xC0 | (cp >> 6))); b.push_back((char)(0x80 | (cp & 0x3F))); }
  else if (cp < 0x10000) { b.push_back((char)(0xE0 | (cp >> 12))); b.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); b.push_back((char)(0x80 | (cp & 0x3F))); }
  else { b.push_back((char)(0xF0 | (cp >> 18))); b.push_back((char)(0x80 | ((cp >> 12) & 0x3F))); b.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); b.push_back((char)(0x80 | (cp & 0x3F))); }
}

std::vector<Tok> lex(const std::string& src) {
  std::vector<Tok> out;
  size_t i = 0, n = src.size();
  int line = 1;
  while (i < n) {
    char c = src[i];
    if (c == ' ' || c == '\t' || c == '\r') { ++i; continue; }
    if (c == '#') { while (i < n && src[i] != '\n') ++i; continue; }
    if (c == '\n') { out.push_back({K_NL, "\n", line}); ++line; ++i; continue; }
    if (c == '`') {
      size_t j = src.find('`', i + 1);
      if (j == std::string::npos) throw std::runtime_error("unterminated raw string");
      out.push_back({K_STR, src.substr(i + 1, j - i - 1), line});
      for (size_t k = i; k < j; ++k) if (src[k] == '\n') ++line;
      i = j + 1;
      continue;
    }
    if (c == '"') {
      std::string s;
      ++i;
      while (i < n && src[i] != '"') {
        if (src[i] == '\n') throw std::runtime_error("newline in string");
        if (src[i] == '\\') {
          ++i;
          if (i >= n) break;
          char e = src[i++];
          switch (e) {
            case '"': s.push_back('"'); break;
            case '\\': s.push_back('\\'); break;
            case '/': s.push_back('/'); break;
            case 'b': s.push_back('\b'); break;
            case 'f': s.push_back('\f'); break;
            case 'n': s.push_back('\n'); break;
            case 'r': s.push_back('\r'); break;
            case 't': s.push_back('\t'); break;
            case 'u': {
              if (i + 4 > n) throw std::runtime_error("bad \\u escape");
              uint32_t cp = (uint32_t)std::stoul(src.substr(i, 4), nullptr, 16);
              i += 4;
              put_utf8(s, cp);
              break;
            }
            default: throw std::runtime_error("bad escape");
          }
        } else s.push_back(src[i++]);
      }
      if (i >= n) throw std::runtime_error("unterminated string");
      ++i;
      out.push_back({K_STR, s, line});
      continue;
    }
    if (c >= '0' && c <= '9') {
      size_t j = i;
      if (src[j] == '0') ++j; else while (j < n && isdigit((unsigned char)src[j])) ++j;
      if (j < n && src[j] == '.' && j + 1 < n && isdigit((unsigned char)src[j + 1])) { ++j; while (j < n && isdigit((unsigned char)src[j])) ++j; }
      if (j < n && (src[j] == 'e' || src[j] == 'E')) {
        size_t k = j + 1;
        if (k < n && (src[k] == '+' || src[k] == '-')) ++k;
        if (k < n && isdigit((unsigned char)src[k])) { j = k; while (j < n && isdigit((unsigned char)src[j])) ++j; }
      }
      out.push_back({K_NUM, src.substr(i, j - i), line});
      i = j;
      continue;
    }
    if (is_ident_start(c)) {
      size_t j = i;
      while (j < n && is_ident(src[j])) ++j;
      out.push_back({K_IDENT, src.substr(i, j - i), line});
      i = j;
      continue;
    }
    static const char* two[] = {":=", "==", "!=", "<=", ">="};
    bool done = false;
    for (auto t : two) if (src.compare(i, 2, t) == 0) { out.push_back({K_OP, t, line}); i += 2; done = true; break; }
    if (done) continue;
    if (std::string("{}[]().,;:=<>+-*/%|&").find(c) != std::string::npos) { out.push_back({K_OP, std::string(1, c), line}); ++i; continue; }
    throw std::runtime_error(std::string("unexpected character '") + c + "'");
  }
  out.push_back({K_EOF, "", line});
  return out;
}

const char* infix_name(const std::string& o) {
  if (o == "==") return "equal";
  if (o == "!=") return "neq";
  if (o == "<") return "lt";
  if (o == "<=") return "lte";
  if (o == ">") return "gt";
  if (o == ">=") return "gte";
  if (o == "|") return "or";
  if (o == "&") return "and";
  if (o == "+") return "plus";
  if (o == "-") return "minus";
  if (o == "*") return "mul";
  if (o == "/") return "div";
  if (o == "%") return "rem";
  return nullptr;
}

const std::vector<std::vector<std::string>> LEVELS = {{"==", "!=", "<", "<=", ">", ">="}, {"|"}, {"&"}, {"+", "-"}, {"*", "/", "%"}};

class Parser {
 public:
  explicit Parser(const std::string& src) : t_(lex(src)) { nl_.push_back(false); }

  std::shared_ptr<Module> module() {
    auto m = std::make_shared<Module>();
    expect("package");
    m->pkg = ref_path();
    while (peek().k != K_EOF) {
      if (at("import")) {
        next();
        auto p = ref_path();
        std::string alias = p.back();
        if (at("as")) { next(); alias = next().text; }
        m->imports.push_back({p, alias});
        continue;
      }
      for (auto& r : rule()) { r->mod = m.get(); m->rules.push_back(r); }
    }
    return m;
  }

 private:
  std::vector<Tok> t_;
  size_t i_ = 0;
  int wild_ = 0;
  std::vector<bool> nl_;

  const Tok& peek(int k = 0) {
    size_t j = i_;
    int cnt = 0;
    while (true) {
      if (t_[j].k == K_NL && !nl_.back()) { ++j; continue; }
      if (cnt == k || t_[j].k == K_EOF) return t_[j];
      ++cnt;
      ++j;
    }
  }
  Tok next() {
    while (t_[i_].k == K_NL && !nl_.back()) ++i_;
    return t_[i_++];
  }
  void skip_nl() { while (t_[i_].k == K_NL) ++i_; }
  bool at(const char* s) {
    const Tok& t = peek();
    return (t.k == K_OP || t.k == K_IDENT) && t.text == s;
  }
  void expect(const char* s) {
    Tok t = next();
    if (t.text != s) throw std::runtime_error("line " + std::to_string(t.line) + ": expected '" + s + "' got '" + t.text + "'");
  }
  TermP fresh_wild() { return mk_var("$_" + std::to_string(++wild_)); }

  std::vector<std::string> ref_path() {
    Tok t = next();
    if (t.k != K_IDENT) throw std::runtime_error("expected identifier");
    std::vector<std::string> p{t.text};
    while (true) {
      const Tok& n = t_[i_];
      if (n.k == K_OP && n.text == ".") { ++i_; p.push_back(next().text); }
      else if (n.k == K_OP && n.text == "[") { ++i_; p.push_back(next().text); expect("]"); }
      else break;
    }
    return p;
  }

  std::vector<std::shared_ptr<Rule>> rule() {
    bool def = false;
    if (at("default")) { next(); def = true; }
    Tok name = next();
    if (name.k != K_IDENT) throw std::runtime_error("line " + std::to_string(name.line) + ": expected rule name");
    auto r = std::make_shared<Rule>();
    r->name = name.text;
    r->is_default = def;
    if (at("(")) {
      next();
      while (!at(")")) { r->args.push_back(term()); if (at(",")) next(); }
      expect(")");
      r->kind = Rule::FUNC;
    } else if (at("[")) {
      next();
      r->key = term();
      expect("]");
      r->kind = Rule::PSET;
    }
    if (at("=") || at(":=")) {
      next();
      r->value = term();
      if (r->kind == Rule::PSET) r->kind = Rule::POBJ;
    }
    std::vector<std::shared_ptr<Rule>> out;
    if (!def && at("{")) r->body = braced_body();
    out.push_back(r);
    while (at("else")) {
      next();
      auto e = std::make_shared<Rule>();
      e->name = r->name; e->kind = r->kind; e->key = r->key; e->args = r->args; e->is_else = true;
      if (at("=") || at(":=")) { next(); e->value = term(); } else e->value = mk_scalar(S_TRUE, "true");
      if (at("{")) e->body = braced_body();
      out.push_back(e);
    }
    if ((r->kind == Rule::COMPLETE || r->kind == Rule::FUNC) && !r->value) r->value = mk_scalar(S_TRUE, "true");
    return out;
  }

  std::vector<ExprP> braced_body() {
    expect("{");
    nl_.push_back(true);
    auto b = body_until("}");
    expect("}");
    nl_.pop_back();
    return b;
  }

  bool with_follows() {
    size_t j = i_;
    while (t_[j].k == K_NL) ++j;
    return t_[j].k == K_IDENT && t_[j].text == "with";
  }

  std::vector<ExprP> body_until(const char* closer) {
    std::vector<ExprP> b;
    while (true) {
      skip_nl();
      const Tok& t = t_[i_];
      if (t.k == K_OP && t.text == closer) break;
      if (t.k == K_OP && t.text == ";") { ++i_; continue; }
      b.push_back(expr());
      const Tok& u = t_[i_];
      if (u.k == K_NL || (u.k == K_OP && (u.text == ";" || u.text == closer))) continue;
      throw std::runtime_error("line " + std::to_string(u.line) + ": unexpected '" + u.text + "'");
    }
    return b;
  }

  ExprP expr() {
    auto e = std::make_shared<Expr>();
    e->line = peek().line;
    if (at("some")) {
      next();
      e->kind = Expr::SOME;
      e->terms.push_back(term());
      while (at(",")) { next(); e->terms.push_back(term()); }
      return e;
    }
    if (at("not")) { next(); e->negated = true; }
    TermP lhs = term();
    if (at(":=")) { next(); e->kind = Expr::ASSIGN; e->terms = {lhs, term()}; }
    else if (at("=")) { next(); e->kind = Expr::UNIFY; e->terms = {lhs, term()}; }
    else { e->kind = Expr::TERM; e->terms = {lhs}; }
    while (with_follows()) {
      skip_nl();
      next();
      With w;
      w.target = term();
      expect("as");
      w.value = term();
      e->withs.push_back(w);
    }
    return e;
  }

  TermP term(size_t level = 0, bool no_bar = false) {
    if (level == LEVELS.size()) return unary();
    if (no_bar && LEVELS[level].size() == 1 && LEVELS[level][0] == "|") return term(level + 1, no_bar);
    TermP lhs = term(level + 1, no_bar);
    while (true) {
      const Tok& t = peek();
      if (t.k == K_OP && std::find(LEVELS[level].begin(), LEVELS[level].end(), t.text) != LEVELS[level].end()) {
        std::string o = next().text;
        while (t_[i_].k == K_NL) ++i_;
        TermP rhs = term(level + 1, no_bar);
        lhs = mk_call({infix_name(o)}, {lhs, rhs});
      } else break;
    }
    return lhs;
  }

  TermP unary() {
    const Tok& t = peek();
    if (t.k == K_OP && t.text == "-") {
      const Tok& n = peek(1);
      if (n.k == K_NUM) { next(); Tok num = next(); return mk_scalar(S_NUM, "-" + num.text); }
      next();
      TermP operand = unary();
      return mk_call({"minus"}, {mk_scalar(S_NUM, "0"), operand});
    }
    return postfix();
  }

  TermP postfix() {
    TermP head = primary();
    std::vector<TermP> path;
    while (true) {
      const Tok& t = peek();
      if (t.k == K_OP && t.text == ".") {
        next();
        Tok f = next();
        path.push_back(mk_scalar(S_STR, f.text));
      } else if (t.k == K_OP && t.text == "[") {
        next();
        nl_.push_back(false);
        TermP sel = term();
        expect("]");
        nl_.pop_back();
        path.push_back(sel);
      } else if (t.k == K_OP && t.text == "(" && head->k == T_VAR) {
        std::vector<std::string> names{head->s};
        for (auto& p : path) {
          if (p->k != T_SCALAR || p->stype != S_STR) throw std::runtime_error("dynamic call target");
          names.push_back(p->s);
        }
        next();
        nl_.push_back(false);
        std::vector<TermP> args;
        while (!at(")")) { args.push_back(term()); if (at(",")) next(); }
        expect(")");
        nl_.pop_back();
        head = mk_call(names, args);
        path.clear();
      } else break;
    }
    if (path.empty()) return head;
    auto r = mk(T_REF);
    r->head = head;
    r->items = path;
    return r;
  }

  TermP primary() {
    Tok t = next();
    if (t.k == K_NUM) return mk_scalar(S_NUM, t.text);
    if (t.k == K_STR) return mk_scalar(S_STR, t.text);
    if (t.k == K_IDENT) {
      if (t.text == "true") return mk_scalar(S_TRUE, "true");
      if (t.text == "false") return mk_scalar(S_FALSE, "false");
      if (t.text == "null") return mk_scalar(S_NULL, "null");
      if (t.text == "_") return fresh_wild();
      return mk_var(t.text);
    }
    if (t.k == K_OP && t.text == "(") {
      nl_.push_back(false);
      TermP in = term();
      expect(")");
      nl_.pop_back();
      return in;
    }
    if (t.k == K_OP && t.text == "[") return array_or_compr();
    if (t.k == K_OP && t.text == "{") return brace();
    throw std::runtime_error("line " + std::to_string(t.line) + ": unexpected token '" + t.text + "'");
  }

  TermP array_or_compr() {
    nl_.push_back(false);
    if (at("]")) { next(); nl_.pop_back(); return mk(T_ARRAY); }
    TermP first = term(0, true);
    if (at("|")) {
      next();
      nl_.back() = true;
      auto body = body_until("]");
      expect("]");
      nl_.pop_back();
      auto c = mk(T_ARRCOMPR);
      c->key = first;
      c->body = body;
      return c;
    }
    auto a = mk(T_ARRAY);
    a->items.push_back(first);
    while (at(",")) { next(); if (at("]")) break; a->items.push_back(term()); }
    expect("]");
    nl_.pop_back();
    return a;
  }

  TermP brace() {
    nl_.push_back(false);
    if (at("}")) { next(); nl_.pop_back(); return mk(T_OBJECT); }
    TermP first = term(0, true);
    if (at(":")) {
      next();
      TermP val = term(0, true);
      if (at("|")) {
        next();
        nl_.back() = true;
        auto body = body_until("}");
        expect("}");
        nl_.pop_back();
        auto c = mk(T_OBJCOMPR);
        c->key = first;
        c->value = val;
        c->body = body;
        return c;
      }
      auto o = mk(T_OBJECT);
      o->items = {first, val};
      while (at(",")) {
        next();
        if (at("}")) break;
        TermP k = term();
        expect(":");
        TermP v = term();
        o->items.push_back(k);
        o->items.push_back(v);
      }
      expect("}");
      nl_.pop_back();
      return o;
    }
    if (at("|")) {
      next();
      nl_.back() = true;
      auto body = body_until("}");
      expect("}");
      nl_.pop_back();
      auto c = mk(T_SETCOMPR);
      c->key = first;
      c->body = body;
      return c;
    }
    auto s = mk(T_SET);
    s->items.push_back(first);
    while (at(",")) { next(); if (at("}")) break; s->items.push_back(term()); }
    expect("}");
    nl_.pop_back();
    return s;
  }
};
}  // namespace

std::shared_ptr<Module> parse_module(const std::string& src) {
  Parser p(src);
  return p.module();
}

// ------------------------------------------------------------------ set algebra
// count(A - {k | T[k]}) == count(A)  <=>  no member a of A has T[a] truthy:
// the comprehension collects exactly the keys k whose T[k] is defined and not
// false (a scalar or missing T gives the empty set, and so does a lookup), and
// |A - B| = |A| - |A & B|.  The rewrite never builds the two sets (heap lists
// per lane in the template kernels: k8srequiredprobes' probe_field_empty,
// demo/agilebank/templates/k8srequiredprobes_template.yaml:36-40).  A must be
// a set, and defined: it is restricted to a rule of the module whose value is
// a set comprehension (always defined).
static bool is_var(const TermP& t, const std::string& name = "") {
  return t && t->k == T_VAR && (name.empty() || t->s == name);
}
static bool is_call(const TermP& t, const char* op, size_t nargs) {
  return t && t->k == T_CALL && t->op.size() == 1 && t->op[0] == op && t->items.size() == nargs;
}
static bool mentions(const TermP& t, const std::string& v);
static bool mentions_body(const std::vector<ExprP>& body, const std::string& v) {
  for (auto& e : body) {
    for (auto& t : e->terms) if (mentions(t, v)) return true;
    for (auto& w : e->withs) if (mentions(w.target, v) || mentions(w.value, v)) return true;
  }
  return false;
}
static bool mentions(const TermP& t, const std::string& v) {
  if (!t) return false;
  if (t->k == T_VAR && t->s == v) return true;
  if (mentions(t->head, v) || mentions(t->key, v) || mentions(t->value, v)) return true;
  for (auto& x : t->items) if (mentions(x, v)) return true;
  return mentions_body(t->body, v);
}
static bool set_rule(const Module& m, const std::string& name) {
  int n = 0;
  bool ok = true;
  for (auto& r : m.rules) {
    if (r->name != name) continue;
    ++n;
    if (r->kind != Rule::COMPLETE || r->is_default || r->is_else || !r->args.empty()) { ok = false; continue; }
    if (r->value && r->value->k == T_SETCOMPR && r->body.empty()) continue;
    ok = ok && r->body.size() == 1 && r->body[0]->kind == Expr::ASSIGN && !r->body[0]->negated &&
         r->body[0]->withs.empty() && r->body[0]->terms.size() == 2 && is_var(r->body[0]->terms[0]) &&
         r->body[0]->terms[1]->k == T_SETCOMPR && is_var(r->value, r->body[0]->terms[0]->s);
  }
  return n == 1 && ok;
}
// the variables of t outside any comprehension it holds (a comprehension's
// own variables are local to it)
static void outer_vars(const TermP& t, std::set<std::string>& out) {
  if (!t) return;
  if (t->k == T_VAR) { out.insert(t->s); return; }
  if (t->k == T_ARRCOMPR || t->k == T_SETCOMPR || t->k == T_OBJCOMPR) return;
  outer_vars(t->head, out);
  for (auto& x : t->items) outer_vars(x, out);
}
// T (the comprehension's collection, lifted out of it by a rewrite) may only
// name variables bound before body position i -- a rule argument, a variable
// of an earlier expression, `input` / `data` or a rule of the module.  A
// variable local to the comprehension (a wildcard, an unbound name) would
// otherwise be hoisted into the enclosing body and change what it means.
static bool closed_before(const Module& m, const Rule& r, const std::vector<ExprP>& b, size_t i, const TermP& T,
                          const std::string& k) {
  std::set<std::string> need;
  outer_vars(T, need);
  if (mentions(T, k)) return false;
  std::set<std::string> bound = {"input", "data"};
  for (auto& a : r.args) outer_vars(a, bound);
  for (size_t q = 0; q < i && q < b.size(); ++q)
    for (auto& t : b[q]->terms) outer_vars(t, bound);
  for (auto& x : m.rules) bound.insert(x->name);
  for (auto& v : need)
    if (v.rfind("$", 0) == 0 || !bound.count(v)) return false;
  // T's selectors: constants or variables (a ref selector would be hoisted
  // out of the comprehension by RewriteDynamicTerms)
  if (T->k == T_REF)
    for (auto& x : T->items)
      if (x->k != T_SCALAR && x->k != T_VAR) return false;
  return true;
}

int optimize_sets(Module& m, int mask) {
  int done = 0;
  for (size_t ri = 0; ri < m.rules.size() && (mask & 1); ++ri) {
    Rule& r = *m.rules[ri];
    auto& b = r.body;
    for (size_t i = 0; i + 2 < b.size() + 0 && i < b.size(); ++i) {
      // E1: v1 := {k | T[k]}
      const ExprP e1 = b[i];
      if (e1->kind != Expr::ASSIGN || e1->negated || !e1->withs.empty() || e1->terms.size() != 2 || !is_var(e1->terms[0]))
        continue;
      const TermP c = e1->terms[1];
      if (c->k != T_SETCOMPR || !is_var(c->key) || c->body.size() != 1) continue;
      const ExprP cb = c->body[0];
      if (cb->kind != Expr::TERM || cb->negated || !cb->withs.empty() || cb->terms.size() != 1) continue;
      const TermP ref = cb->terms[0];
      const std::string k = c->key->s, v1 = e1->terms[0]->s;
      if (ref->k != T_REF || ref->items.empty() || !is_var(ref->items.back(), k) || mentions(ref->head, k)) continue;
      bool kin = false;
      for (size_t q = 0; q + 1 < ref->items.size(); ++q) kin = kin || mentions(ref->items[q], k);
      if (kin) continue;
      // E2: v2 := A - v1, E3: count(v2) == count(A) (either side), later in the body
      for (size_t j = i + 1; j < b.size(); ++j) {
        const ExprP e2 = b[j];
        if (e2->kind != Expr::ASSIGN || e2->negated || !e2->withs.empty() || e2->terms.size() != 2 || !is_var(e2->terms[0]))
          continue;
        const TermP mi = e2->terms[1];
        if (!is_call(mi, "minus", 2) || !is_var(mi->items[1], v1) || !is_var(mi->items[0])) continue;
        const std::string A = mi->items[0]->s, v2 = e2->terms[0]->s;
        for (size_t l = j + 1; l < b.size(); ++l) {
          const ExprP e3 = b[l];
          if (e3->kind != Expr::TERM || e3->negated || !e3->withs.empty() || e3->terms.size() != 1) continue;
          const TermP eq = e3->terms[0];
          if (!is_call(eq, "equal", 2) || !is_call(eq->items[0], "count", 1) || !is_call(eq->items[1], "count", 1)) continue;
          const TermP x0 = eq->items[0]->items[0], x1 = eq->items[1]->items[0];
          if (!((is_var(x0, v2) && is_var(x1, A)) || (is_var(x0, A) && is_var(x1, v2)))) continue;
          // v1 and v2 used nowhere else; A is the module's set rule, not shadowed
          std::vector<ExprP> rest;
          for (size_t q = 0; q < b.size(); ++q)
            if (q != i && q != j && q != l) rest.push_back(b[q]);
          bool shadow = false;
          for (auto& a : r.args) shadow = shadow || mentions(a, A);
          for (auto& q : b)
            if ((q->kind == Expr::ASSIGN || q->kind == Expr::SOME) && !q->terms.empty() && mentions(q->terms[0], A)) shadow = true;
          if (mentions_body(rest, v1) || mentions_body(rest, v2) || mentions(r.value, v1) || mentions(r.value, v2) ||
              mentions(r.key, v1) || mentions(r.key, v2) || shadow || !set_rule(m, A))
            continue;
          TermP T;
          if (ref->items.size() == 1) T = ref->head;
          else {
            T = mk(T_REF);
            T->head = ref->head;
            T->items.assign(ref->items.begin(), ref->items.end() - 1);
          }
          if (!closed_before(m, r, b, i, T, k)) continue;
          auto ne = std::make_shared<Expr>();
          ne->kind = Expr::TERM;
          ne->negated = true;
          ne->line = e3->line;
          ne->terms = {mk_call({"__gk_anyin"}, {mk_var(A), T})};
          std::vector<ExprP> nb;
          for (size_t q = 0; q < b.size(); ++q) {
            if (q == i || q == j) continue;
            nb.push_back(q == l ? ne : b[q]);
          }
          b.swap(nb);
          ++done;
          goto next_rule;
        }
      }
    }
  next_rule:;
  }
  const bool anyin = done > 0;
  // Second pattern: v1 := {k | T[k]}; v2 := A - v1 (v1 used nowhere else, A a
  // set: a comprehension assigned earlier in the body or a set rule) becomes
  // v2 := {e | e := A[i]; not T[e]} -- the members of A whose T[a] is
  // undefined or false, the set A - {k | T[k]} without building the second
  // set (k8srequiredlabels' `missing := required - provided`,
  // demo/agilebank/templates/k8srequiredlabels_template.yaml:41-43).
  int fresh = 0;
  for (size_t ri = 0; ri < m.rules.size() && (mask & 2); ++ri) {
    Rule& r = *m.rules[ri];
    auto& b = r.body;
    for (size_t i = 0; i < b.size(); ++i) {
      const ExprP e1 = b[i];
      if (e1->kind != Expr::ASSIGN || e1->negated || !e1->withs.empty() || e1->terms.size() != 2 || !is_var(e1->terms[0]))
        continue;
      const TermP c = e1->terms[1];
      if (c->k != T_SETCOMPR || !is_var(c->key) || c->body.size() != 1) continue;
      const ExprP cb = c->body[0];
      if (cb->kind != Expr::TERM || cb->negated || !cb->withs.empty() || cb->terms.size() != 1) continue;
      const TermP ref = cb->terms[0];
      const std::string k = c->key->s, v1 = e1->terms[0]->s;
      if (ref->k != T_REF || ref->items.empty() || !is_var(ref->items.back(), k) || mentions(ref->head, k)) continue;
      bool kin = false;
      for (size_t q = 0; q + 1 < ref->items.size(); ++q) kin = kin || mentions(ref->items[q], k);
      if (kin) continue;
      bool hit = false;
      for (size_t j = i + 1; j < b.size() && !hit; ++j) {
        const ExprP e2 = b[j];
        if (e2->kind != Expr::ASSIGN || e2->negated || !e2->withs.empty() || e2->terms.size() != 2 || !is_var(e2->terms[0]))
          continue;
        const TermP mi = e2->terms[1];
        if (!is_call(mi, "minus", 2) || !is_var(mi->items[1], v1) || !is_var(mi->items[0])) continue;
        const std::string A = mi->items[0]->s;
        // A: assigned a set comprehension earlier in this body (and nowhere
        // else), or the module's set rule (not shadowed)
        int assigned = 0;
        bool local_set = false;
        for (size_t q = 0; q < b.size(); ++q) {
          const ExprP& x = b[q];
          if ((x->kind == Expr::ASSIGN || x->kind == Expr::UNIFY || x->kind == Expr::SOME) && !x->terms.empty() &&
              mentions(x->terms[0], A)) {
            ++assigned;
            local_set = q < j && x->kind == Expr::ASSIGN && !x->negated && x->terms.size() == 2 && is_var(x->terms[0], A) &&
                        x->terms[1]->k == T_SETCOMPR;
          }
        }
        bool arg = false;
        for (auto& a : r.args) arg = arg || mentions(a, A);
        const bool set_ok = arg ? false : assigned == 1 ? local_set : assigned == 0 ? set_rule(m, A) : false;
        std::vector<ExprP> rest;
        for (size_t q = 0; q < b.size(); ++q)
          if (q != i && q != j) rest.push_back(b[q]);
        if (!set_ok || mentions_body(rest, v1) || mentions(r.value, v1) || mentions(r.key, v1)) continue;
        TermP T;
        if (ref->items.size() == 1) T = ref->head;
        else {
          T = mk(T_REF);
          T->head = ref->head;
          T->items.assign(ref->items.begin(), ref->items.end() - 1);
        }
        if (!closed_before(m, r, b, i, T, k)) continue;
        const std::string e = "__gk_e" + std::to_string(fresh), ix = "__gk_i" + std::to_string(fresh);
        ++fresh;
        auto it = mk(T_REF);
        it->head = mk_var(A);
        it->items = {mk_var(ix)};
        auto x1 = std::make_shared<Expr>();
        x1->kind = Expr::ASSIGN;
        x1->terms = {mk_var(e), it};
        auto lk = mk(T_REF);
        lk->head = T;
        lk->items = {mk_var(e)};
        if (T->k == T_REF) {  // T[e] as one ref: T's path then e
          lk->head = T->head;
          lk->items = T->items;
          lk->items.push_back(mk_var(e));
        }
        auto x2 = std::make_shared<Expr>();
        x2->kind = Expr::TERM;
        x2->negated = true;
        x2->terms = {lk};
        auto sc = mk(T_SETCOMPR);
        sc->key = mk_var(e);
        sc->body = {x1, x2};
        auto ne = std::make_shared<Expr>(*e2);
        ne->terms = {e2->terms[0], sc};
        std::vector<ExprP> nb;
        for (size_t q = 0; q < b.size(); ++q) {
          if (q == i) continue;
          nb.push_back(q == j ? ne : b[q]);
        }
        b.swap(nb);
        ++done;
        hit = true;
      }
      if (hit) i = (size_t)-1;  // rescan this body from the start (indices moved)
    }
  }
  if (anyin) {
    bool have = false;
    for (auto& r : m.rules) have = have || r->name == "__gk_anyin";
    if (!have) {
      // __gk_anyin(s, x) = true { y := s[w]; x[y] }
      auto f = std::make_shared<Rule>();
      f->kind = Rule::FUNC;
      f->name = "__gk_anyin";
      f->args = {mk_var("__gk_s"), mk_var("__gk_x")};
      f->value = mk_scalar(S_TRUE, "true");
      f->mod = &m;
      auto it = mk(T_REF);
      it->head = mk_var("__gk_s");
      it->items = {mk_var("__gk_w")};
      auto a1 = std::make_shared<Expr>();
      a1->kind = Expr::ASSIGN;
      a1->terms = {mk_var("__gk_y"), it};
      auto lk = mk(T_REF);
      lk->head = mk_var("__gk_x");
      lk->items = {mk_var("__gk_y")};
      auto a2 = std::make_shared<Expr>();
      a2->kind = Expr::TERM;
      a2->terms = {lk};
      f->body = {a1, a2};
      m.rules.push_back(f);
    }
  }
  return done;
}

// ------------------------------------------------------------------ vars
static void all_vars(const TermP& t, std::vector<std::string>& out);
static void iter_vars(const TermP& t, std::vector<std::string>& out);

static void compr_free_vars(const TermP& t, std::vector<std::string>& out) {
  std::vector<std::string> used, bound;
  for (auto& e : t->body) {
    for (auto& x : e->terms) all_vars(x, used);
    if (e->kind == Expr::ASSIGN || e->kind == Expr::UNIFY) {
      all_vars(e->terms[0], bound);
      if (e->kind == Expr::UNIFY) all_vars(e->terms[1], bound);
    }
    for (auto& x : e->terms) iter_vars(x, bound);
    // call output args bind too
    if (e->kind == Expr::TERM && e->terms[0]->k == T_CALL && !e->terms[0]->items.empty())
      all_vars(e->terms[0]->items.back(), bound);
  }
  if (t->key) all_vars(t->key, used);
  if (t->value) all_vars(t->value, used);
  std::set<std::string> b(bound.begin(), bound.end());
  for (auto& v : used) if (!b.count(v) && v.rfind("$_", 0) != 0) out.push_back(v);
}

static void all_vars(const TermP& t, std::vector<std::string>& out) {
  if (!t) return;
  switch (t->k) {
    case T_VAR: out.push_back(t->s); break;
    case T_REF: all_vars(t->head, out); for (auto& p : t->items) all_vars(p, out); break;
    case T_CALL: case T_ARRAY: case T_SET: case T_OBJECT: for (auto& p : t->items) all_vars(p, out); break;
    case T_ARRCOMPR: case T_SETCOMPR: case T_OBJCOMPR: compr_free_vars(t, out); break;
    default: break;
  }
}

static void iter_vars(const TermP& t, std::vector<std::string>& out) {
  if (!t) return;
  switch (t->k) {
    case T_REF:
      iter_vars(t->head, out);
      for (auto& p : t->items) { if (p->k == T_VAR) out.push_back(p->s); else iter_vars(p, out); }
      break;
    case T_CALL: case T_ARRAY: case T_SET: case T_OBJECT: for (auto& p : t->items) iter_vars(p, out); break;
    default: break;
  }
}

void term_vars(const TermP& t, std::vector<std::string>& out) { all_vars(t, out); }

// ------------------------------------------------------------------ rewrites
namespace {
struct Rewriter {
  std::function<bool(const std::string&)> is_global;
  int gen = 0;
  TermP fresh() { return mk_var("$l" + std::to_string(++gen)); }

  // ---- RewriteExprTerms
  std::vector<ExprP> expand_body(const std::vector<ExprP>& body) {
    std::vector<ExprP> out;
    for (auto& e : body) expand_expr(e, out);
    return out;
  }
  void expand_expr(const ExprP& e, std::vector<ExprP>& out) {
    if (e->kind == Expr::SOME) { out.push_back(e); return; }
    std::vector<ExprP> support;
    auto ne = std::make_shared<Expr>(*e);
    if (e->kind == Expr::TERM) {
      const TermP& t = e->terms[0];
      if (t->k == T_CALL) {
        auto c = std::make_shared<Term>(*t);
        for (auto& a : c->items) a = expand_term(a, support);
        ne->terms = {c};
      } else {
        ne->terms = {t->k == T_REF ? expand_ref(t, support) : expand_term(t, support)};
      }
    } else {
      ne->terms.clear();
      for (auto& t : e->terms) ne->terms.push_back(expand_term(t, support));
    }
    for (auto& s : support) { s->withs = e->withs; out.push_back(s); }
    out.push_back(ne);
  }
  TermP expand_term(const TermP& t, std::vector<ExprP>& support) {
    switch (t->k) {
      case T_CALL: {
        auto c = std::make_shared<Term>(*t);
        for (auto& a : c->items) a = expand_term(a, support);
        TermP v = fresh();
        c->items.push_back(v);
        auto se = std::make_shared<Expr>();
        se->kind = Expr::TERM;
        se->terms = {c};
        support.push_back(se);
        return v;
      }
      case T_REF: return expand_ref(t, support);
      case T_ARRAY: case T_SET: case T_OBJECT: {
        auto c = std::make_shared<Term>(*t);
        for (auto& a : c->items) a = expand_term(a, support);
        return c;
      }
      case T_ARRCOMPR: case T_SETCOMPR: case T_OBJCOMPR: {
        auto c = std::make_shared<Term>(*t);
        std::vector<ExprP> inner;
        if (c->key) c->key = expand_term(c->key, inner);
        if (c->value) c->value = expand_term(c->value, inner);
        std::vector<ExprP> b = c->body;
        b.insert(b.end(), inner.begin(), inner.end());
        c->body = expand_body(b);
        return c;
      }
      default: return t;
    }
  }
  TermP expand_ref(const TermP& t, std::vector<ExprP>& support) {
    auto r = std::make_shared<Term>(*t);
    for (auto& p : r->items) p = expand_term(p, support);
    if (r->head->k == T_CALL) r->head = expand_term(r->head, support);
    return r;
  }

  // ---- safety reordering
  std::set<std::string> vs(const TermP& t) {
    std::vector<std::string> v;
    all_vars(t, v);
    std::set<std::string> o;
    for (auto& x : v) if (!is_global(x)) o.insert(x);
    return o;
  }
  std::set<std::string> its(const TermP& t) {
    std::vector<std::string> v;
    iter_vars(t, v);
    std::set<std::string> o;
    for (auto& x : v) if (!is_global(x)) o.insert(x);
    return o;
  }
  static std::set<std::string> minus(const std::set<std::string>& a, const std::set<std::string>& b) {
    std::set<std::string> o;
    for (auto& x : a) if (!b.count(x)) o.insert(x);
    return o;
  }
  static bool subset(const std::set<std::string>& a, const std::set<std::string>& b) {
    for (auto& x : a) if (!b.count(x)) return false;
    return true;
  }
  // returns (needs, outputs)
  std::pair<std::set<std::string>, std::set<std::string>> needs_outputs(const ExprP& e, const std::set<std::string>& safe) {
    std::set<std::string> wv;
    for (auto& w : e->withs) { auto x = vs(w.value); wv.insert(x.begin(), x.end()); }
    if (e->kind == Expr::SOME) return {{}, {}};
    if (e->negated) {
      std::set<std::string> nd;
      for (auto& t : e->terms) { auto a = minus(vs(t), its(t)); nd.insert(a.begin(), a.end()); }
      std::set<std::string> o;
      for (auto& x : nd) if (x.rfind("$_", 0) != 0) o.insert(x);
      o.insert(wv.begin(), wv.end());
      return {o, {}};
    }
    if (e->kind == Expr::TERM) {
      const TermP& t = e->terms[0];
      auto it = minus(its(t), safe);
      std::set<std::string> outs = it;
      std::set<std::string> needs = minus(vs(t), it);
      // call output argument (after RewriteExprTerms)
      if (t->k == T_CALL && !t->items.empty() && t->items.back()->k == T_VAR && t->op.size() >= 1 && call_has_output(t)) {
        const std::string& ov = t->items.back()->s;
        if (!safe.count(ov)) { needs.erase(ov); outs.insert(ov); }
      }
      needs.insert(wv.begin(), wv.end());
      return {needs, outs};
    }
    const TermP& l = e->terms[0];
    const TermP& r = e->terms[1];
    auto rn = minus(vs(r), its(r));
    if (subset(rn, safe)) {
      auto o = vs(l);
      auto ri = its(r);
      o.insert(ri.begin(), ri.end());
      rn.insert(wv.begin(), wv.end());
      return {rn, o};
    }
    if (e->kind == Expr::UNIFY) {
      auto ln = minus(vs(l), its(l));
      if (subset(ln, safe)) {
        auto o = vs(r);
        auto li = its(l);
        o.insert(li.begin(), li.end());
        ln.insert(wv.begin(), wv.end());
        return {ln, o};
      }
    }
    rn.insert(wv.begin(), wv.end());
    return {rn, {}};
  }
  std::function<bool(const TermP&)> call_has_output;

  std::vector<ExprP> reorder(const std::vector<ExprP>& body, std::set<std::string> safe) {
    std::vector<ExprP> rem = body, out;
    while (!rem.empty()) {
      bool placed = false;
      for (size_t i = 0; i < rem.size(); ++i) {
        auto no = needs_outputs(rem[i], safe);
        if (subset(no.first, safe)) {
          out.push_back(reorder_nested(rem[i], safe));
          safe.insert(no.second.begin(), no.second.end());
          rem.erase(rem.begin() + i);
          placed = true;
          break;
        }
      }
      if (!placed) {
        for (auto& e : rem) out.push_back(e);
        break;
      }
    }
    return out;
  }
  ExprP reorder_nested(const ExprP& e, const std::set<std::string>& safe) {
    auto ne = std::make_shared<Expr>(*e);
    for (auto& t : ne->terms) t = reorder_term(t, safe);
    return ne;
  }
  TermP reorder_term(const TermP& t, const std::set<std::string>& safe) {
    if (!t) return t;
    switch (t->k) {
      case T_ARRCOMPR: case T_SETCOMPR: case T_OBJCOMPR: {
        auto c = std::make_shared<Term>(*t);
        c->body = reorder(c->body, safe);
        return c;
      }
      case T_REF: {
        auto c = std::make_shared<Term>(*t);
        c->head = reorder_term(c->head, safe);
        for (auto& p : c->items) p = reorder_term(p, safe);
        return c;
      }
      case T_CALL: case T_ARRAY: case T_SET: case T_OBJECT: {
        auto c = std::make_shared<Term>(*t);
        for (auto& p : c->items) p = reorder_term(p, safe);
        return c;
      }
      default: return t;
    }
  }

  // ---- RewriteDynamicTerms
  bool is_ref(const TermP& t) {
    if (t->k == T_VAR) return is_global(t->s);
    if (t->k == T_REF) return t->head->k == T_VAR && is_global(t->head->s);
    return false;
  }
  std::vector<ExprP> dynamics(const std::vector<ExprP>& body) {
    std::vector<ExprP> out;
    for (auto& e : body) {
      if (e->kind == Expr::SOME) { out.push_back(e); continue; }
      std::vector<ExprP> res;
      auto ne = std::make_shared<Expr>(*e);
      if (e->kind == Expr::ASSIGN || e->kind == Expr::UNIFY) {
        ne->terms = {dyn_in_term(e, e->terms[0], res), dyn_in_term(e, e->terms[1], res)};
      } else if (e->terms[0]->k == T_CALL) {
        auto c = std::make_shared<Term>(*e->terms[0]);
        // optimize_sets' `not __gk_anyin(A, T)` stands for count(A - {k | T[k]})
        // == count(A), where an undefined T is the empty set: T stays in the
        // call (undefined there -> the call is undefined -> `not` holds)
        // instead of being hoisted before the expression, where an undefined
        // T would fail the body
        const bool anyin = c->op.size() == 1 && c->op[0] == "__gk_anyin";
        for (size_t ai = 0; ai < c->items.size(); ++ai)
          if (!(anyin && ai == 1)) c->items[ai] = dyn_one(e, c->items[ai], res);
        ne->terms = {c};
      } else {
        ne->terms = {dyn_in_term(e, e->terms[0], res)};
      }
      out.insert(out.end(), res.begin(), res.end());
      out.push_back(ne);
    }
    return out;
  }
  TermP dyn_in_term(const ExprP& orig, const TermP& t, std::vector<ExprP>& res) {
    switch (t->k) {
      case T_REF: {
        auto c = std::make_shared<Term>(*t);
        for (auto& p : c->items) p = dyn_one(orig, p, res);
        return c;
      }
      case T_ARRCOMPR: case T_SETCOMPR: case T_OBJCOMPR: {
        auto c = std::make_shared<Term>(*t);
        c->body = dynamics(c->body);
        return c;
      }
      case T_VAR: if (is_global(t->s)) return t; return dyn_one(orig, t, res);
      default: return dyn_one(orig, t, res);
    }
  }
  TermP dyn_one(const ExprP& orig, const TermP& t, std::vector<ExprP>& res) {
    if (is_ref(t)) {
      TermP x = t;
      if (t->k == T_REF) {
        auto c = std::make_shared<Term>(*t);
        for (auto& p : c->items) p = dyn_one(orig, p, res);
        x = c;
      }
      TermP v = fresh();
      auto ge = std::make_shared<Expr>();
      ge->kind = Expr::UNIFY;
      ge->terms = {v, x};
      ge->withs = orig->withs;
      res.push_back(ge);
      return v;
    }
    switch (t->k) {
      case T_ARRAY: case T_SET: case T_OBJECT: {
        auto c = std::make_shared<Term>(*t);
        for (auto& p : c->items) p = dyn_one(orig, p, res);
        return c;
      }
      case T_ARRCOMPR: case T_SETCOMPR: case T_OBJCOMPR: {
        TermP c = dyn_in_term(orig, t, res);
        TermP v = fresh();
        auto ge = std::make_shared<Expr>();
        ge->kind = Expr::UNIFY;
        ge->terms = {v, c};
        ge->withs = orig->withs;
        res.push_back(ge);
        return v;
      }
      default: return t;
    }
  }
};
}  // namespace

std::vector<ExprP> compile_body(const std::vector<ExprP>& body, const std::vector<std::string>& safe,
                                const std::function<bool(const std::string&)>& is_global) {
  static int gen_base = 0;
  Rewriter rw;
  rw.is_global = is_global;
  rw.gen = gen_base;
  rw.call_has_output = [](const TermP& t) { return t->items.back()->s.rfind("$l", 0) == 0; };
  auto b = rw.expand_body(body);
  b = rw.reorder(b, std::set<std::string>(safe.begin(), safe.end()));
  b = rw.dynamics(b);
  gen_base = rw.gen + 1;
  return b;
}

}  // namespace rego
}  // namespace gk
