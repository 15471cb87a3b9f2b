// Rego subset front end (host): lexer, parser, and the OPA compiler rewrites
// that change evaluation semantics (RewriteExprTerms, safety reordering,
// RewriteDynamicTerms — vendor/github.com/open-policy-agent/opa/ast/compile.go).
#pragma once
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace gk {
namespace rego {

struct Term;
struct Expr;
using TermP = std::shared_ptr<Term>;
using ExprP = std::shared_ptr<Expr>;

enum TermKind { T_SCALAR, T_VAR, T_REF, T_ARRAY, T_OBJECT, T_SET, T_ARRCOMPR, T_SETCOMPR, T_OBJCOMPR, T_CALL };
enum ScalarType { S_NULL = 1, S_FALSE = 2, S_TRUE = 3, S_NUM = 4, S_STR = 5 };

struct Term {
  TermKind k;
  int stype = 0;                 // scalar type
  std::string s;                 // scalar text / var name
  TermP head;                    // ref head (var or call)
  std::vector<TermP> items;      // ref path, array/set items, call args, object pairs (k0,v0,k1,v1..)
  std::vector<std::string> op;   // call target path
  TermP key, value;              // comprehension head
  std::vector<ExprP> body;       // comprehension body
};

struct With { TermP target, value; };

struct Expr {
  enum Kind { TERM, ASSIGN, UNIFY, SOME } kind = TERM;
  bool negated = false;
  std::vector<TermP> terms;
  std::vector<With> withs;
  int line = 0;
};

struct Module;
struct Rule {
  enum Kind { COMPLETE, PSET, POBJ, FUNC } kind = COMPLETE;
  std::string name;
  TermP key, value;
  std::vector<TermP> args;
  std::vector<ExprP> body;
  bool is_default = false, is_else = false;
  Module* mod = nullptr;
  // compiled body (after rewrites), cached per rule
  std::vector<ExprP> cbody;
  bool compiled = false;
};

struct Module {
  std::vector<std::string> pkg;
  std::vector<std::pair<std::vector<std::string>, std::string>> imports;  // (path, alias)
  std::vector<std::shared_ptr<Rule>> rules;
};

// Parse a module; throws std::runtime_error on syntax errors.
std::shared_ptr<Module> parse_module(const std::string& src);

// Term constructors
TermP mk_scalar(int stype, const std::string& s);
TermP mk_var(const std::string& name);
TermP mk_call(const std::vector<std::string>& op, const std::vector<TermP>& args);

// Apply OPA's body rewrites to a rule body.  `is_global(name)` tells whether a
// variable name resolves to a root document / rule (input, data, rules of the
// package, import aliases); `safe` are variables bound on entry (function args).
std::vector<ExprP> compile_body(const std::vector<ExprP>& body, const std::vector<std::string>& safe,
                                const std::function<bool(const std::string&)>& is_global);

// variables of a term (excluding comprehension-local ones)
void term_vars(const TermP& t, std::vector<std::string>& out);

// Set-algebra rewrite of a module's rule bodies (rego.cc optimize_sets):
//   v1 := {k | T[k]}; v2 := A - v1; count(v2) == count(A)
// with A a rule of the module whose value is a set comprehension, and v1, v2
// used nowhere else, becomes `not __gk_anyin(A, T)`, the function
// `__gk_anyin(s, x) = true { y := s[_]; x[y] }` added to the module (mask
// bit 1); `v1 := {k | T[k]}; v2 := A - v1` becomes a comprehension over A
// with a negated lookup (mask bit 2).  Returns the number of bodies rewritten.
int optimize_sets(Module& m, int mask = 3);

}  // namespace rego
}  // namespace gk
