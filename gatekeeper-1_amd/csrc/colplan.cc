// Referenced-path plan of a compiled template (colplan.h).
#include "colplan.h"

#include <algorithm>
#include <set>
#include <sstream>

namespace gk {

void bc_regs(const Ins& in, std::vector<uint32_t>& rd, std::vector<uint32_t>& wr);  // jit.cc
void bc_succ(const Ins& in, uint32_t pc, std::vector<uint32_t>& out);               // jit.cc

namespace {
constexpr uint32_t kMaxDepth = 12;  // deeper paths (a lookup loop walking a chain) are used whole
using PSet = std::set<uint32_t>;
using State = std::map<uint16_t, PSet>;

uint32_t depth_of(const PathPlan& P, uint32_t n) {
  uint32_t d = 0;
  while (n) { n = P.nodes[n].parent; ++d; }
  return d;
}
}  // namespace

uint32_t PathPlan::child(uint32_t at, uint32_t key) {
  auto it = nodes[at].kids.find(key);
  if (it != nodes[at].kids.end()) return it->second;
  PathNode n;
  n.parent = at;
  n.key = key;
  nodes.push_back(n);
  const uint32_t id = (uint32_t)nodes.size() - 1;
  nodes[at].kids[key] = id;
  return id;
}

void PathPlan::merge(const PathPlan& o) {
  if (!o.ok) { ok = false; if (why.empty()) why = o.why; }
  if (nodes.empty()) nodes.emplace_back();
  // walk o's trie alongside ours
  std::vector<std::pair<uint32_t, uint32_t>> st{{0, 0}};
  while (!st.empty()) {
    auto [a, b] = st.back();
    st.pop_back();
    nodes[a].uses |= o.nodes[b].uses;
    for (const auto& kv : o.nodes[b].kids) {
      const uint32_t c = child(a, kv.first);
      st.push_back({c, kv.second});
    }
  }
}

std::string PathPlan::describe(const Store& st) const {
  std::ostringstream o;
  std::vector<std::pair<uint32_t, std::string>> todo{{0, "review"}};
  while (!todo.empty()) {
    auto [n, name] = todo.back();
    todo.pop_back();
    const PathNode& x = nodes[n];
    std::string u;
    if (x.uses & PU_DYN) u += " dyn";
    if (x.uses & PU_ITER) u += " iter";
    if (x.uses & PU_LEN) u += " len";
    if (x.uses & PU_WHOLE) u += " whole";
    if (x.uses & PU_IDX) u += " idx";
    o << name << (u.empty() ? "" : " [" + u.substr(1) + "]") << "\n";
    for (auto it = x.kids.rbegin(); it != x.kids.rend(); ++it)
      todo.push_back({it->second, name + (it->first == PK_ANY ? std::string("[*]") : "." + std::string(st.str(it->first)))});
  }
  if (!ok) o << "NOT COLUMNAR: " << why << "\n";
  return o.str();
}

// Forward may-analysis over the program's CFG: on entry to each instruction,
// for each register, the document paths (trie nodes) its value may be.  Uses
// mark the trie; memo slots carry the paths their stored values may be.
PathPlan plan_paths(const Program& p, const CodeBank& bank) {
  PathPlan P;
  P.nodes.emplace_back();
  const uint32_t b0 = p.code_off, n = p.code_len;
  std::map<uint32_t, PSet> slot_paths;
  std::vector<uint32_t> rd, wr, succ;
  auto mark = [&](const State& s, uint32_t r, uint8_t u) {
    if (r == 0xffff) return;
    auto it = s.find((uint16_t)r);
    if (it == s.end()) return;
    for (uint32_t q : it->second) P.nodes[q].uses |= u;
  };
  auto paths = [&](const State& s, uint32_t r) -> PSet {
    auto it = s.find((uint16_t)r);
    return it == s.end() ? PSet{} : it->second;
  };
  auto set = [&](State& s, uint32_t r, PSet v) {
    if (r == 0xffff) return;
    if (v.empty()) s.erase((uint16_t)r);
    else s[(uint16_t)r] = std::move(v);
  };
  auto step = [&](const PSet& from, uint32_t key) {
    PSet out;
    for (uint32_t q : from) {
      if (depth_of(P, q) >= kMaxDepth) { P.nodes[q].uses |= PU_WHOLE; continue; }
      out.insert(P.child(q, key));
    }
    return out;
  };
  for (int round = 0; round < 8; ++round) {
    std::vector<State> in(n);
    std::vector<char> reached(n, 0);
    std::vector<uint32_t> work;
    if (n) { reached[0] = 1; work.push_back(0); }
    bool slots_changed = false;
    auto flow = [&](uint32_t to, const State& s) {
      if (to < b0 || to >= b0 + n) return;
      const uint32_t k = to - b0;
      if (!reached[k]) { reached[k] = 1; in[k] = s; work.push_back(k); return; }
      bool grew = false;
      for (const auto& kv : s) {
        PSet& d = in[k][kv.first];
        for (uint32_t q : kv.second) grew |= d.insert(q).second;
      }
      if (grew) work.push_back(k);
    };
    while (!work.empty()) {
      const uint32_t k = work.back();
      work.pop_back();
      const Ins& in_ = bank.code[b0 + k];
      State s = in[k];
      switch (in_.op) {
        case OP_LOADREV: set(s, in_.a, PSet{0}); break;
        case OP_MOV: set(s, in_.a, paths(s, in_.b)); break;
        case OP_GETK: {
          const uint64_t K = in_.x < bank.consts.size() ? bank.consts[in_.x] : 0;
          const PSet from = paths(s, in_.b);
          const uint32_t t = (uint32_t)(K >> 60);
          if (t == V_STR) set(s, in_.a, step(from, (uint32_t)(K & 0xffffffffu)));
          else if (t == V_NUM || t == V_INT) { mark(s, in_.b, PU_IDX); set(s, in_.a, step(from, PK_ANY)); }
          else { mark(s, in_.b, PU_WHOLE); set(s, in_.a, PSet{}); }
          break;
        }
        case OP_GET: {
          mark(s, in_.b, PU_DYN);
          mark(s, in_.c, PU_WHOLE);  // a document value used as a key
          set(s, in_.a, step(paths(s, in_.b), PK_ANY));
          break;
        }
        case OP_ITER_INIT: {
          mark(s, in_.b, PU_ITER);
          set(s, in_.a, paths(s, in_.b));
          set(s, in_.a + 1u, PSet{});
          break;
        }
        case OP_ITER_NEXT: {
          const PSet el = step(paths(s, in_.a), PK_ANY);
          set(s, in_.a + 1u, PSet{});
          set(s, in_.b, PSet{});
          set(s, in_.c, el);
          break;
        }
        case OP_CALL: {
          const uint32_t id = in_.y;
          for (uint32_t i = 0; i < in_.c; ++i) {
            const uint32_t r = in_.b + i;
            if (id == BI_COUNT) mark(s, r, PU_LEN);
            else if (id == BI_IS_NUMBER || id == BI_IS_STRING || id == BI_IS_BOOLEAN || id == BI_IS_NULL ||
                     id == BI_IS_ARRAY || id == BI_IS_OBJECT || id == BI_IS_SET)
              ;  // type tests (tclass of a column value is exact)
            else if (id == BI_STARTSWITH || id == BI_ENDSWITH || id == BI_CONTAINS || id == BI_RE_MATCH ||
                     id == BI_TO_NUMBER || id == BI_REPLACE || id == BI_SUBSTRING || id == BI_LOWER ||
                     id == BI_UPPER || id == BI_TRIM || id == BI_TRIM_PREFIX || id == BI_TRIM_SUFFIX ||
                     id == BI_SPLIT || id == BI_INDEXOF || (id == BI_CONCAT && i == 0))
              mark(s, r, PU_WHOLE);  // scalars; a composite operand is an error either way
            else
              mark(s, r, PU_WHOLE);
          }
          set(s, in_.a, PSet{});
          break;
        }
        case OP_LEN_EQ: mark(s, in_.b, PU_LEN); set(s, in_.a, PSet{}); break;
        case OP_YIELD: {
          PSet u = paths(s, in_.a);
          for (uint32_t q : paths(s, in_.b)) u.insert(q);
          set(s, in_.a, u);
          break;
        }
        case OP_MEMO_GET: {
          PSet u = paths(s, in_.a);
          auto it = slot_paths.find(in_.y);
          if (it != slot_paths.end()) u.insert(it->second.begin(), it->second.end());
          set(s, in_.a, u);
          break;
        }
        case OP_MEMO_PUT: {
          PSet& d = slot_paths[in_.y];
          for (uint32_t q : paths(s, in_.a)) slots_changed |= d.insert(q).second;
          break;
        }
        case OP_JUNDEF: case OP_JFALSE: case OP_JTRUE: case OP_JMP: case OP_END: case OP_ORD:
        case OP_FAIL_FALLBACK:
          break;
        default: {
          // every other operand is used whole (compared, printed, collected, hashed)
          bc_regs(in_, rd, wr);
          for (uint32_t r : rd) mark(s, r, PU_WHOLE);
          for (uint32_t w : wr) set(s, w, PSet{});
          break;
        }
      }
      bc_succ(in_, b0 + k, succ);
      for (uint32_t t : succ) flow(t, s);
    }
    if (!slots_changed) break;
  }
  const uint8_t root = P.nodes[0].uses;
  if (root & (PU_WHOLE | PU_ITER | PU_LEN)) {
    P.ok = false;
    P.why = "the review document is used whole";
  }
  return P;
}

}  // namespace gk
