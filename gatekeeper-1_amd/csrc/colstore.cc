// Columnar staged batches (colstore.h).
//
// Four passes over the batch's documents, the first three parallel over
// chunks of reviews (evaluation order):
//   A. discover the schema: which paths of the plan occur, with which kinds
//      of value (scalar / object / array), and, under a computed-key lookup,
//      every member key the batch has there;
//   B. decide each path's storage: columns, or document nodes where a program
//      reads the value whole; number the object views and element tables;
//   C. count each chunk's element rows per table (CSR offsets), then fill the
//      value words;
//   D. copy the subtrees kept as nodes (and the label objects the match stage
//      scans) into the batch's compact node array.
#include "colstore.h"

#include <algorithm>
#include <atomic>
#include <mutex>
#include <sstream>
#include <unordered_map>

#include "flatten.h"

namespace gk {
namespace {

constexpr uint8_t S_SCALAR = 1, S_OBJ = 2, S_ARR = 4, S_BIG = 8;  // S_BIG: an object with the fallback flag
constexpr uint32_t kChunk = 2048;
constexpr uint32_t kMaxDynKeys = 32;  // a computed-key object with more distinct keys stays nodes

struct SNode {
  std::vector<uint32_t> plan;                       // plan-trie nodes reading this path
  std::vector<std::pair<uint32_t, uint32_t>> kids;  // member key -> snode (objects)
  uint32_t elem = NO_ID;                            // element snode (arrays)
  uint32_t maxlen = 0;
  uint8_t seen = 0;
  uint8_t uses = 0;   // OR of the plan nodes' uses
  bool dyn = false;   // some plan looks members up by a computed key: every key descends
  bool keyed = false; // the planned constant keys have their snodes
  // decided in pass B
  bool node = false;
  uint32_t table = 0, view = NO_ID, tab = NO_ID, slot = NO_ID;
};

struct Schema {
  const PathPlan* P = nullptr;
  std::vector<SNode> n;
  std::vector<uint32_t> const_keys(uint32_t s) const {
    std::vector<uint32_t> k;
    for (uint32_t p : n[s].plan)
      for (const auto& kv : P->nodes[p].kids)
        if (kv.first != PK_ANY) k.push_back(kv.first);
    std::sort(k.begin(), k.end());
    k.erase(std::unique(k.begin(), k.end()), k.end());
    return k;
  }
  uint32_t kid(uint32_t s, uint32_t key) const {
    for (const auto& kv : n[s].kids) if (kv.first == key) return kv.second;
    return NO_ID;
  }
  uint32_t make(const std::vector<uint32_t>& plan) {
    SNode x;
    x.plan = plan;
    for (uint32_t p : plan) {
      x.uses |= P->nodes[p].uses;
      x.dyn |= (P->nodes[p].uses & PU_DYN) != 0;
    }
    n.push_back(std::move(x));
    return (uint32_t)n.size() - 1;
  }
  // the member `key` of object path s (created on first use)
  uint32_t member(uint32_t s, uint32_t key) {
    uint32_t k = kid(s, key);
    if (k != NO_ID) return k;
    std::vector<uint32_t> pl;
    for (uint32_t p : n[s].plan) {
      const auto& kids = P->nodes[p].kids;
      auto it = kids.find(key);
      if (it != kids.end()) pl.push_back(it->second);
      if (P->nodes[p].uses & PU_DYN) {
        auto a = kids.find(PK_ANY);
        if (a != kids.end()) pl.push_back(a->second);
      }
    }
    std::sort(pl.begin(), pl.end());
    pl.erase(std::unique(pl.begin(), pl.end()), pl.end());
    k = make(pl);
    n[s].kids.push_back({key, k});
    return k;
  }
  uint32_t element(uint32_t s) {
    if (n[s].elem != NO_ID) return n[s].elem;
    std::vector<uint32_t> pl;
    for (uint32_t p : n[s].plan) {
      auto a = P->nodes[p].kids.find(PK_ANY);
      if (a != P->nodes[p].kids.end()) pl.push_back(a->second);
    }
    std::sort(pl.begin(), pl.end());
    pl.erase(std::unique(pl.begin(), pl.end()), pl.end());
    const uint32_t e = make(pl);
    n[s].elem = e;
    return e;
  }
};

struct Docs {
  const Node* perm;
  uint32_t nb;
  const Node* arena;
  const Node& operator()(uint32_t id) const { return id >= nb ? arena[id - nb] : perm[id]; }
};

// pass A: one document path instance
void discover(Schema& S, const Docs& D, uint32_t s, uint32_t id) {
  const Node& x = D(id);
  if (x.type == NT_OBJ) {
    S.n[s].seen |= S_OBJ;
    if (x.flags & 1) S.n[s].seen |= S_BIG;
    S.n[s].maxlen = std::max<uint32_t>(S.n[s].maxlen, x.n);
    // an object read whole / iterated / counted stays nodes: nothing below matters
    if (s != 0 && (S.n[s].uses & (PU_WHOLE | PU_ITER | PU_LEN | PU_IDX))) return;
    if (S.n[s].dyn && S.n[s].kids.size() > kMaxDynKeys) { S.n[s].seen |= S_BIG; return; }
    if (!S.n[s].keyed) {  // planned keys get slots even where absent
      for (uint32_t k : S.const_keys(s)) S.member(s, k);
      S.n[s].keyed = true;
    }
    for (uint32_t i = 0; i < x.n; ++i) {
      const uint32_t c = x.first + i;
      const uint32_t key = D(c).key;
      uint32_t k = S.kid(s, key);
      if (k == NO_ID) {
        if (!S.n[s].dyn) continue;  // a member no program reads
        k = S.member(s, key);
      }
      discover(S, D, k, c);
    }
  } else if (x.type == NT_ARR) {
    S.n[s].seen |= S_ARR;
    S.n[s].maxlen = std::max<uint32_t>(S.n[s].maxlen, x.n);
    if (S.n[s].uses & PU_WHOLE) return;
    const uint32_t e = S.element(s);
    for (uint32_t i = 0; i < x.n; ++i) discover(S, D, e, x.first + i);
  } else {
    S.n[s].seen |= S_SCALAR;
  }
}

// merges thread schema b's subtree at bs into a's at as
void merge_schema(Schema& A, uint32_t as, const Schema& B, uint32_t bs) {
  A.n[as].seen |= B.n[bs].seen;
  A.n[as].maxlen = std::max(A.n[as].maxlen, B.n[bs].maxlen);
  for (const auto& kv : B.n[bs].kids) merge_schema(A, A.member(as, kv.first), B, kv.second);
  if (B.n[bs].elem != NO_ID) merge_schema(A, A.element(as), B, B.n[bs].elem);
}

bool scalar_word(const Node& x, uint32_t& w) {
  switch (x.type) {
    case NT_NULL: w = CW_LIT << CW_SHIFT; return true;
    case NT_FALSE: w = (CW_LIT << CW_SHIFT) | 1u; return true;
    case NT_TRUE: w = (CW_LIT << CW_SHIFT) | 2u; return true;
    case NT_NUM: if (x.val > CW_PAY) return false; w = (CW_NUM << CW_SHIFT) | x.val; return true;
    case NT_STR: if (x.val > CW_PAY) return false; w = (CW_STR << CW_SHIFT) | x.val; return true;
  }
  return false;
}

}  // namespace

bool build_columns(const PathPlan& plan, const Node* perm, uint32_t node_begin, const Node* arena, size_t n_arena,
                   const std::vector<ReviewCol>& cols, const Store& st, std::mutex& smu, ColStore& out,
                   std::string& why) {
  (void)n_arena;
  if (!plan.ok) { why = plan.why; return false; }
  const Docs D{perm, node_begin, arena};
  const uint32_t nrev = (uint32_t)cols.size();
  const uint32_t nchunk = (nrev + kChunk - 1) / kChunk;
  const int T = std::max(1, std::min<int>(default_threads(), (int)nchunk));
  // ---- A
  std::vector<Schema> local(T);
  for (auto& s : local) { s.P = &plan; s.make({0}); }
  std::atomic<uint32_t> next{0};
  parallel_run(T, [&](int t) {
    Schema& S = local[t];
    for (;;) {
      const uint32_t c = next.fetch_add(1);
      if (c >= nchunk) break;
      for (uint32_t r = c * kChunk; r < std::min(nrev, (c + 1) * kChunk); ++r)
        if (cols[r].root != NO_ID) discover(S, D, 0, cols[r].root);
    }
  });
  Schema S;
  S.P = &plan;
  S.make({0});
  for (auto& l : local) merge_schema(S, 0, l, 0);
  local.clear();
  // ---- B: storage, views, tables (a breadth-first walk below the root)
  std::vector<uint32_t> views_of, tabs_of;  // snode of each view / table
  {
    std::vector<uint32_t> q{0};
    S.n[0].view = 0;
    views_of.push_back(0);
    tabs_of.push_back(NO_ID);  // table 0: the reviews
    for (size_t qi = 0; qi < q.size(); ++qi) {
      const uint32_t s = q[qi];
      SNode& x = S.n[s];
      const bool composite = x.seen & (S_OBJ | S_ARR);
      if (s != 0 && composite) {
        const bool obj = x.seen & S_OBJ, arr = x.seen & S_ARR;
        x.node = (x.uses & PU_WHOLE) || (x.seen & S_BIG) || (obj && (x.uses & (PU_ITER | PU_LEN | PU_IDX))) ||
                 (obj && x.dyn && x.kids.size() > kMaxDynKeys) || (arr && x.maxlen > 0xffff);
      }
      if (x.node) continue;
      if ((x.seen & S_OBJ) && s != 0) {
        x.view = (uint32_t)views_of.size();
        views_of.push_back(s);
      }
      if (x.seen & S_ARR) {
        x.tab = (uint32_t)tabs_of.size();
        tabs_of.push_back(x.elem);
        if (x.elem != NO_ID) S.n[x.elem].table = x.tab;
      }
      if (x.view != NO_ID)
        for (const auto& kv : x.kids) {
          S.n[kv.second].table = x.table;
          q.push_back(kv.second);
        }
      if (x.tab != NO_ID && x.elem != NO_ID) q.push_back(x.elem);
    }
    if (views_of.size() > 4096 || tabs_of.size() > 4096) { why = "too many object views / element tables"; return false; }
  }
  // ---- C1: element rows per chunk and table
  const uint32_t ntab = (uint32_t)tabs_of.size();
  std::vector<uint64_t> counts((size_t)nchunk * ntab, 0);
  std::function<void(uint32_t, uint32_t, uint64_t*)> count = [&](uint32_t s, uint32_t id, uint64_t* cnt) {
    const SNode& x = S.n[s];
    if (x.node) return;
    const Node& d = D(id);
    if (d.type == NT_OBJ && x.view != NO_ID) {
      for (const auto& kv : x.kids) {
        for (uint32_t i = 0; i < d.n; ++i)
          if (D(d.first + i).key == kv.first) { count(kv.second, d.first + i, cnt); break; }
      }
    } else if (d.type == NT_ARR && x.tab != NO_ID) {
      cnt[x.tab] += d.n;
      if (x.elem != NO_ID)
        for (uint32_t i = 0; i < d.n; ++i) count(x.elem, d.first + i, cnt);
    }
  };
  next = 0;
  parallel_run(T, [&](int) {
    for (;;) {
      const uint32_t c = next.fetch_add(1);
      if (c >= nchunk) break;
      uint64_t* cnt = &counts[(size_t)c * ntab];
      for (uint32_t r = c * kChunk; r < std::min(nrev, (c + 1) * kChunk); ++r)
        if (cols[r].root != NO_ID) count(0, cols[r].root, cnt);
    }
  });
  std::vector<uint64_t> rows(ntab, 0);  // table sizes; counts become each chunk's first row
  rows[0] = nrev;
  for (uint32_t t = 1; t < ntab; ++t) {
    uint64_t acc = 0;
    for (uint32_t c = 0; c < nchunk; ++c) {
      const uint64_t k = counts[(size_t)c * ntab + t];
      counts[(size_t)c * ntab + t] = acc;
      acc += k;
    }
    rows[t] = acc;
    if (acc > CW_PAY) { why = "element table too large"; return false; }
  }
  // slots and their columns
  out = ColStore{};
  out.node_begin = node_begin;
  uint64_t words = 0;
  {
    std::vector<uint32_t> q{0};
    for (size_t qi = 0; qi < q.size(); ++qi) {
      const SNode& x = S.n[q[qi]];
      if (!x.node) {  // (a path kept as nodes has its value column, nothing below)
        if (x.view != NO_ID) for (const auto& kv : x.kids) q.push_back(kv.second);
        if (x.tab != NO_ID && x.elem != NO_ID) q.push_back(x.elem);
      }
      if (q[qi] == 0) continue;
      SNode& y = S.n[q[qi]];
      CvSlot sl{};
      sl.col = (uint32_t)words;
      words += rows[y.table];
      sl.lencol = NO_ID;
      if (y.tab != NO_ID && !y.node) {
        sl.lencol = (uint32_t)words;
        words += rows[y.table];
      }
      sl.view = (uint16_t)(y.view == NO_ID ? 0 : y.view);
      sl.tab = (uint16_t)(y.tab == NO_ID ? 0 : y.tab);
      y.slot = (uint32_t)out.slots.size();
      out.slots.push_back(sl);
      if (words > 0xffffffffull) { why = "columns exceed 4G words"; return false; }
    }
  }
  out.words.assign(words, 0);
  out.rows = 0;
  for (uint64_t r : rows) out.rows += r;
  // ---- C2: fill
  struct NodeRef { uint64_t at; uint32_t src; };
  std::vector<std::vector<NodeRef>> refs(T);
  std::atomic<bool> bad{false};
  std::function<void(uint32_t, uint32_t, uint64_t, uint64_t*, std::vector<NodeRef>&)> fill =
      [&](uint32_t s, uint32_t id, uint64_t row, uint64_t* cur, std::vector<NodeRef>& nr) {
        const SNode& x = S.n[s];
        const Node& d = D(id);
        uint32_t w = 0;
        const uint64_t at = (uint64_t)out.slots[x.slot].col + row;
        if (d.type != NT_OBJ && d.type != NT_ARR) {
          if (!scalar_word(d, w)) { bad = true; return; }
          out.words[at] = w;
          return;
        }
        if (x.node) {
          nr.push_back({at, id});
          return;
        }
        if (d.type == NT_OBJ) {
          out.words[at] = CW_OBJ << CW_SHIFT;
          for (const auto& kv : x.kids)
            for (uint32_t i = 0; i < d.n; ++i)
              if (D(d.first + i).key == kv.first) { fill(kv.second, d.first + i, row, cur, nr); break; }
          return;
        }
        const uint64_t first = cur[x.tab];
        cur[x.tab] += d.n;
        out.words[at] = (CW_ARR << CW_SHIFT) | (uint32_t)first;
        out.words[(uint64_t)out.slots[x.slot].lencol + row] = d.n;
        if (x.elem != NO_ID)
          for (uint32_t i = 0; i < d.n; ++i) fill(x.elem, d.first + i, first + i, cur, nr);
      };
  next = 0;
  parallel_run(T, [&](int t) {
    std::vector<uint64_t> cur(ntab);
    for (;;) {
      const uint32_t c = next.fetch_add(1);
      if (c >= nchunk) break;
      for (uint32_t k = 1; k < ntab; ++k) cur[k] = counts[(size_t)c * ntab + k];
      for (uint32_t r = c * kChunk; r < std::min(nrev, (c + 1) * kChunk); ++r) {
        if (cols[r].root == NO_ID) continue;
        const Node& d = D(cols[r].root);
        if (d.type != NT_OBJ) { bad = true; continue; }
        for (const auto& kv : S.n[0].kids)
          for (uint32_t i = 0; i < d.n; ++i)
            if (D(d.first + i).key == kv.first) { fill(kv.second, d.first + i, r, cur.data(), refs[t]); break; }
      }
    }
  });
  if (bad) { why = "a value id does not fit a column word"; return false; }
  // ---- D: subtrees kept as nodes (shared ones once)
  std::unordered_map<uint32_t, uint32_t> copied;
  auto copy = [&](uint32_t src) -> uint32_t {
    if (src < node_begin) return src;  // the permanent region is uploaded as it is
    auto it = copied.find(src);
    if (it != copied.end()) return it->second;
    const uint32_t dst = node_begin + (uint32_t)out.nodes.size();
    out.nodes.push_back(D(src));
    // breadth-first: each composite's children as one contiguous run
    std::vector<std::pair<uint32_t, uint32_t>> q{{src, dst}};
    for (size_t qi = 0; qi < q.size(); ++qi) {
      const Node sn = D(q[qi].first);
      if (sn.type != NT_OBJ && sn.type != NT_ARR) continue;
      const uint32_t run = node_begin + (uint32_t)out.nodes.size();
      out.nodes[q[qi].second - node_begin].first = run;
      for (uint32_t i = 0; i < sn.n; ++i) {
        out.nodes.push_back(D(sn.first + i));
        q.push_back({sn.first + i, run + i});
      }
    }
    copied[src] = dst;
    return dst;
  };
  for (auto& v : refs)
    for (const NodeRef& r : v) {
      const uint32_t d = copy(r.src);
      out.words[r.at] = (CW_NODE << CW_SHIFT) | d;
    }
  out.cols = cols;
  for (ReviewCol& rc : out.cols) {
    rc.root = NO_ID;
    if (rc.labels != NO_ID) rc.labels = copy(rc.labels);
    if (rc.old_labels != NO_ID) rc.old_labels = copy(rc.old_labels);
    if (rc.ns_labels != NO_ID) rc.ns_labels = copy(rc.ns_labels);
  }
  if ((uint64_t)node_begin + out.nodes.size() > CW_PAY) { why = "kept nodes exceed the column word"; return false; }
  // object views, element tables, the (view, key) hash
  out.views.assign(views_of.size(), 0);
  for (size_t v = 0; v < views_of.size(); ++v) out.views[v] = S.n[views_of[v]].dyn ? CV_COMPLETE : 0;
  out.tabs.assign(ntab, NO_ID);
  for (uint32_t t = 1; t < ntab; ++t) if (tabs_of[t] != NO_ID) out.tabs[t] = S.n[tabs_of[t]].slot;
  size_t entries = 0;
  for (uint32_t v : views_of) entries += S.n[v].kids.size();
  size_t hs = 16;
  while (hs < 2 * entries + 1) hs <<= 1;
  out.hash.assign(hs, CvHash{NO_ID, 0, 0, 0});
  for (size_t v = 0; v < views_of.size(); ++v)
    for (const auto& kv : S.n[views_of[v]].kids) {
      const uint32_t slot = S.n[kv.second].slot;
      if (slot == NO_ID) continue;
      uint32_t i = cv_hash_of((uint32_t)v, kv.first) & (uint32_t)(hs - 1);
      while (out.hash[i].view != NO_ID) i = (i + 1) & (uint32_t)(hs - 1);
      out.hash[i] = CvHash{(uint32_t)v, kv.first, slot, 0};
    }
  // description (diagnostics): path, storage
  {
    std::lock_guard<std::mutex> g(smu);  // (the string table grows under concurrent flattens)
    std::ostringstream o;
    std::vector<std::pair<uint32_t, std::string>> todo{{0, "review"}};
    while (!todo.empty()) {
      auto [s, name] = todo.back();
      todo.pop_back();
      const SNode& x = S.n[s];
      o << name << ":" << (x.node ? " nodes" : "") << (x.view != NO_ID ? " view" + std::to_string(x.view) : "")
        << (x.tab != NO_ID ? " table" + std::to_string(x.tab) : "") << ((x.seen & S_SCALAR) ? " scalars" : "")
        << (x.dyn ? " complete" : "") << "\n";
      if (x.node) continue;
      if (x.elem != NO_ID && x.tab != NO_ID) todo.push_back({x.elem, name + "[*]"});
      if (x.view != NO_ID)
        for (auto it = x.kids.rbegin(); it != x.kids.rend(); ++it)
          todo.push_back({it->second, name + "." + std::string(st.str(it->first))});
    }
    out.schema = o.str();
  }
  return true;
}

}  // namespace gk
