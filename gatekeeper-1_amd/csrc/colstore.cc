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
#include <cstring>
#include <atomic>
#include <mutex>
#include <sstream>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <unordered_map>

#include "flatten.h"

namespace gk {
namespace {

// S_BIG: an object with the fallback flag; S_PAY: a string or number (a payload)
constexpr uint8_t S_SCALAR = 1, S_OBJ = 2, S_ARR = 4, S_BIG = 8, S_PAY = 16;
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

// per-chunk element counts of a thread's local schema (pass A): the arrays'
// lengths summed per local snode
struct ChunkCount {
  std::vector<uint64_t> n;          // per local snode
  std::vector<uint32_t> touched;
  void add(uint32_t s, uint64_t k) {
    if (s >= n.size()) n.resize(s + 64, 0);
    if (!n[s]) touched.push_back(s);
    n[s] += k;
  }
};

struct Docs {
  const Node* perm;
  uint32_t nb;
  size_t na;
  const Node* arena;
  const Node& operator()(uint32_t id) const { return id >= nb ? arena[id - nb] : perm[id]; }
  // the passes visit reviews in evaluation order, so consecutive documents
  // lie far apart in the arena: each walk is a chain of dependent misses.  A
  // document's nodes are one block around its root; fetching the block of a
  // review a few positions ahead overlaps those misses.
  void prefetch(uint32_t root) const {
    if (root == NO_ID || root < nb) return;
    const size_t a = root - nb;
    const size_t lo = a >= kPfBefore ? a - kPfBefore : 0, hi = std::min(na, a + kPfAfter);
    for (size_t i = lo; i < hi; i += 4) __builtin_prefetch(arena + i, 0, 0);
  }
  static constexpr size_t kPfBefore = 80, kPfAfter = 2;  // (a root follows its members: the parser places a run at its close)
};
constexpr uint32_t kAhead = 6;

// pass A: one document path instance
void discover(Schema& S, const Docs& D, uint32_t s, uint32_t id, ChunkCount& cc) {
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
      discover(S, D, k, c, cc);
    }
  } else if (x.type == NT_ARR) {
    S.n[s].seen |= S_ARR;
    S.n[s].maxlen = std::max<uint32_t>(S.n[s].maxlen, x.n);
    if (S.n[s].uses & PU_WHOLE) return;
    cc.add(s, x.n);
    const uint32_t e = S.element(s);
    for (uint32_t i = 0; i < x.n; ++i) discover(S, D, e, x.first + i, cc);
  } else {
    S.n[s].seen |= (x.type == NT_STR || x.type == NT_NUM) ? (S_SCALAR | S_PAY) : S_SCALAR;
  }
}

// merges thread schema b's subtree at bs into a's at as; map[b snode] = a snode
void merge_schema(Schema& A, uint32_t as, const Schema& B, uint32_t bs, std::vector<uint32_t>& map) {
  map[bs] = as;
  A.n[as].seen |= B.n[bs].seen;
  A.n[as].maxlen = std::max(A.n[as].maxlen, B.n[bs].maxlen);
  for (const auto& kv : B.n[bs].kids) merge_schema(A, A.member(as, kv.first), B, kv.second, map);
  if (B.n[bs].elem != NO_ID) merge_schema(A, A.element(as), B, B.n[bs].elem, map);
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
  if (!plan.ok) { why = plan.why; return false; }
  using Clock = std::chrono::steady_clock;
  const auto t0 = Clock::now();
  auto ms = [&]() { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); };
  const bool trace = getenv("GKGPU_FLATTEN_TRACE") != nullptr;
  const Docs D{perm, node_begin, n_arena, arena};
  const uint32_t nrev = (uint32_t)cols.size();
  const uint32_t nchunk = (nrev + kChunk - 1) / kChunk;
  const int T = std::max(1, std::min<int>(default_threads(), (int)nchunk));
  // ---- A
  std::vector<Schema> local(T);
  for (auto& s : local) { s.P = &plan; s.make({0}); }
  std::atomic<uint32_t> next{0};
  // per chunk: (thread, [(local snode, elements)])
  std::vector<std::pair<int, std::vector<std::pair<uint32_t, uint64_t>>>> ccount(nchunk);
  parallel_run(T, [&](int t) {
    Schema& S = local[t];
    ChunkCount cc;
    for (;;) {
      const uint32_t c = next.fetch_add(1);
      if (c >= nchunk) break;
      const uint32_t r1 = std::min(nrev, (c + 1) * kChunk);
      for (uint32_t r = c * kChunk; r < r1; ++r) {
        if (r + kAhead < r1) D.prefetch(cols[r + kAhead].root);
        if (cols[r].root != NO_ID) discover(S, D, 0, cols[r].root, cc);
      }
      ccount[c].first = t;
      for (uint32_t s : cc.touched) { ccount[c].second.push_back({s, cc.n[s]}); cc.n[s] = 0; }
      cc.touched.clear();
    }
  });
  Schema S;
  S.P = &plan;
  S.make({0});
  std::vector<std::vector<uint32_t>> lmap(T);
  for (int t = 0; t < T; ++t) {
    lmap[t].assign(local[t].n.size(), NO_ID);
    merge_schema(S, 0, local[t], 0, lmap[t]);
  }
  local.clear();
  if (trace) fprintf(stderr, "columns: A discover %.1f ms\n", ms());
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
  if (trace) fprintf(stderr, "columns: B decide %.1f ms\n", ms());
  // ---- C1: element rows per chunk and table (counted in pass A)
  const uint32_t ntab = (uint32_t)tabs_of.size();
  std::vector<uint64_t> counts((size_t)nchunk * ntab, 0);
  for (uint32_t c = 0; c < nchunk; ++c)
    for (const auto& sc : ccount[c].second) {
      const uint32_t g = lmap[ccount[c].first][sc.first];
      if (g == NO_ID || S.n[g].node || S.n[g].tab == NO_ID) continue;
      counts[(size_t)c * ntab + S.n[g].tab] += sc.second;
    }
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
  if (trace) fprintf(stderr, "columns: C1 count %.1f ms\n", ms());
  // slots and their columns
  out.slots.clear();
  out.hash.clear();
  out.views.clear();
  out.tabs.clear();
  out.nodes.resize(0);
  out.node_begin = node_begin;
  uint64_t words = 0, bytes = 0;
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
      if (!(y.seen & (S_ARR | S_PAY)) && !(y.node && (y.seen & S_OBJ))) {
        sl.flags = CVS_BYTES;  // tags only: objects, literals, undefined
        sl.col = (uint32_t)bytes;
        bytes += rows[y.table];
      } else {
        sl.col = (uint32_t)words;
        words += rows[y.table];
      }
      sl.lencol = NO_ID;
      if (y.tab != NO_ID && !y.node) {
        sl.lencol = (uint32_t)words;
        words += rows[y.table];
      }
      sl.view = (uint16_t)(y.view == NO_ID ? 0 : y.view);
      sl.tab = (uint16_t)(y.tab == NO_ID ? 0 : y.tab);
      y.slot = (uint32_t)out.slots.size();
      out.slots.push_back(sl);
      if (words > 0xffffffffull || bytes > 0xffffffffull) { why = "columns exceed 4G words"; return false; }
    }
  }
  out.words.resize(words);  // (each chunk zeroes its own rows of every column below)
  out.bytes.resize(bytes);
  out.rows = 0;
  for (uint64_t r : rows) out.rows += r;
  if (trace) fprintf(stderr, "columns: alloc %.1f ms (%llu words)\n", ms(), (unsigned long long)words);
  // the label objects of the Namespace documents (shared by the reviews of a
  // namespace): copied once, first
  std::unordered_map<uint32_t, uint32_t> shared;
  auto copy_into = [&](std::vector<Node>& dst, uint32_t src, uint32_t id0) -> uint32_t {
    // breadth-first: each composite's children as one contiguous run; ids
    // are id0 + position in dst
    const uint32_t root = id0 + (uint32_t)dst.size();
    const Node top = D(src);
    dst.push_back(top);
    if (top.type != NT_OBJ && top.type != NT_ARR) return root;
    {  // the common case (a label object): scalar members only, no queue
      bool flat = true;
      for (uint32_t i = 0; i < top.n && flat; ++i) flat = D(top.first + i).type != NT_OBJ && D(top.first + i).type != NT_ARR;
      if (flat) {
        dst.back().first = id0 + (uint32_t)dst.size();
        for (uint32_t i = 0; i < top.n; ++i) dst.push_back(D(top.first + i));
        return root;
      }
    }
    thread_local std::vector<std::pair<uint32_t, uint32_t>> q;
    q.clear();
    q.push_back({src, root});
    for (size_t qi = 0; qi < q.size(); ++qi) {
      const Node sn = D(q[qi].first);
      if (sn.type != NT_OBJ && sn.type != NT_ARR) continue;
      const uint32_t run = id0 + (uint32_t)dst.size();
      dst[q[qi].second - id0].first = run;
      for (uint32_t i = 0; i < sn.n; ++i) {
        dst.push_back(D(sn.first + i));
        q.push_back({sn.first + i, run + i});
      }
    }
    return root;
  };
  std::vector<Node> shared_nodes;
  for (const ReviewCol& rc : cols)
    if (rc.ns_labels != NO_ID && rc.ns_labels >= node_begin && !shared.count(rc.ns_labels))
      shared[rc.ns_labels] = copy_into(shared_nodes, rc.ns_labels, node_begin);
  const uint32_t nshared = (uint32_t)shared_nodes.size();
  // a bit per document node: is it one of `shared` (most references are not:
  // the test spares a hash lookup per reference)
  std::vector<uint64_t> shared_bit((n_arena + 64) / 64, 0);
  for (const auto& kv : shared) {
    const size_t a = kv.first - node_begin;
    shared_bit[a >> 6] |= 1ull << (a & 63);
  }
  auto is_shared = [&](uint32_t src) {
    const size_t a = src - node_begin;
    return (shared_bit[a >> 6] >> (a & 63)) & 1;
  };
  // ---- C2: fill the words; per chunk, the subtrees kept as nodes go to the
  // chunk's own node list (ids relocated once the chunks' sizes are known)
  struct Chunk {
    std::vector<Node> nodes;                           // .first: local index
    std::vector<std::pair<uint64_t, uint32_t>> words;  // (word position, local node)
    std::vector<std::pair<uint64_t, uint32_t>> cols;   // (review * 3 + label field, local node)
  };
  std::vector<Chunk> chunks(nchunk);
  out.cols.resize(nrev);
  // per slot: its table, for the chunks' zeroing
  std::vector<std::pair<uint32_t, uint32_t>> slot_tab;  // (slot, table)
  for (uint32_t s2 = 1; s2 < S.n.size(); ++s2)
    if (S.n[s2].slot != NO_ID) slot_tab.push_back({S.n[s2].slot, S.n[s2].table});
  std::atomic<bool> bad{false};
  struct Filler {
    const Schema& S;
    const Docs& D;
    ColStore& out;
    std::atomic<bool>& bad;
    uint64_t* cur;
    std::vector<std::pair<uint32_t, uint64_t>> refs;  // (source node, word position) of the review
    // the view's member columns of object d: one pass over its members, the
    // first member of a key wins (as every reader's scan does)
    void members(const SNode& x, const Node& d, uint64_t row) {
      const size_t nk = x.kids.size();
      if (nk > 64) {
        for (const auto& kv : x.kids)
          for (uint32_t i = 0; i < d.n; ++i)
            if (D(d.first + i).key == kv.first) { fill(kv.second, d.first + i, row); break; }
        return;
      }
      uint64_t done = 0;
      for (uint32_t i = 0; i < d.n; ++i) {
        const uint32_t key = D(d.first + i).key;
        for (size_t j = 0; j < nk; ++j)
          if (x.kids[j].first == key) {
            if (!(done >> j & 1)) { done |= 1ull << j; fill(x.kids[j].second, d.first + i, row); }
            break;
          }
      }
    }
    void put(const SNode& x, uint64_t at, uint32_t w) {
      if (out.slots[x.slot].flags & CVS_BYTES) out.bytes[at] = cv_word_byte(w);
      else out.words[at] = w;
    }
    void fill(uint32_t s, uint32_t id, uint64_t row) {
      const SNode& x = S.n[s];
      const Node& d = D(id);
      const uint64_t at = (uint64_t)out.slots[x.slot].col + row;
      if (d.type != NT_OBJ && d.type != NT_ARR) {
        uint32_t w = 0;
        if (!scalar_word(d, w)) { bad = true; return; }
        put(x, at, w);
        return;
      }
      if (x.node) { refs.push_back({id, at}); return; }
      if (d.type == NT_OBJ) {
        put(x, at, CW_OBJ << CW_SHIFT);
        members(x, d, row);
        return;
      }
      const uint64_t first = cur[x.tab];
      cur[x.tab] += d.n;
      out.words[at] = (CW_ARR << CW_SHIFT) | (uint32_t)first;
      out.words[(uint64_t)out.slots[x.slot].lencol + row] = d.n;
      if (x.elem != NO_ID)
        for (uint32_t i = 0; i < d.n; ++i) fill(x.elem, d.first + i, first + i);
    }
  };
  next = 0;
  parallel_run(T, [&](int) {
    std::vector<uint64_t> cur(ntab);
    Filler F{S, D, out, bad, cur.data(), {}};
    std::vector<std::pair<uint32_t, uint32_t>> mine;  // (source, local) copied for this review
    for (;;) {
      const uint32_t c = next.fetch_add(1);
      if (c >= nchunk) break;
      Chunk& ch = chunks[c];
      for (uint32_t k = 1; k < ntab; ++k) cur[k] = counts[(size_t)c * ntab + k];
      // this chunk's rows of every column start undefined (CW_ABSENT)
      for (const auto& st2 : slot_tab) {
        const uint32_t t = st2.second;
        const uint64_t lo = t == 0 ? (uint64_t)c * kChunk : counts[(size_t)c * ntab + t];
        const uint64_t hi = t == 0 ? std::min<uint64_t>(nrev, (uint64_t)(c + 1) * kChunk)
                                   : (c + 1 < nchunk ? counts[(size_t)(c + 1) * ntab + t] : rows[t]);
        if (hi <= lo) continue;
        const CvSlot& sl = out.slots[st2.first];
        if (sl.flags & CVS_BYTES) memset(out.bytes.data() + sl.col + lo, 0, hi - lo);
        else memset(out.words.data() + sl.col + lo, 0, (hi - lo) * 4);
        if (sl.lencol != NO_ID) memset(out.words.data() + sl.lencol + lo, 0, (hi - lo) * 4);
      }
      const uint32_t r1 = std::min(nrev, (c + 1) * kChunk);
      for (uint32_t r = c * kChunk; r < r1; ++r) {
        if (r + kAhead < r1) D.prefetch(cols[r + kAhead].root);
        ReviewCol rc = cols[r];
        F.refs.clear();
        mine.clear();
        if (rc.root != NO_ID) {
          const Node& d = D(rc.root);
          if (d.type != NT_OBJ) { bad = true; continue; }
          F.members(S.n[0], d, r);
        }
        auto local = [&](uint32_t src) {  // the review's copy of src (once per review)
          for (const auto& m : mine) if (m.first == src) return m.second;
          const uint32_t l = copy_into(ch.nodes, src, 0);
          mine.push_back({src, l});
          return l;
        };
        for (const auto& rf : F.refs) {
          if (rf.first < node_begin) { out.words[rf.second] = (CW_NODE << CW_SHIFT) | rf.first; continue; }
          if (is_shared(rf.first)) out.words[rf.second] = (CW_NODE << CW_SHIFT) | shared.at(rf.first);
          else ch.words.push_back({rf.second, local(rf.first)});
        }
        uint32_t* lf[3] = {&rc.labels, &rc.old_labels, &rc.ns_labels};
        for (int f = 0; f < 3; ++f) {
          const uint32_t src = *lf[f];
          if (src == NO_ID || src < node_begin) continue;
          if (is_shared(src)) { *lf[f] = shared.at(src); continue; }
          ch.cols.push_back({(uint64_t)r * 3 + f, local(src)});
        }
        rc.root = NO_ID;
        out.cols[r] = rc;
      }
    }
  });
  if (bad) { why = "a value id does not fit a column word"; return false; }
  if (trace) fprintf(stderr, "columns: C2 fill %.1f ms\n", ms());
  // ---- D: the kept subtrees in one array: the shared ones, then chunk by chunk
  std::vector<uint64_t> base(nchunk + 1, nshared);
  for (uint32_t c = 0; c < nchunk; ++c) base[c + 1] = base[c] + chunks[c].nodes.size();
  if ((uint64_t)node_begin + base[nchunk] > CW_PAY) { why = "kept nodes exceed the column word"; return false; }
  out.nodes.resize(base[nchunk]);
  std::copy(shared_nodes.begin(), shared_nodes.end(), out.nodes.begin());
  next = 0;
  parallel_run(T, [&](int) {
    for (;;) {
      const uint32_t c = next.fetch_add(1);
      if (c >= nchunk) break;
      Chunk& ch = chunks[c];
      const uint32_t g = node_begin + (uint32_t)base[c];  // global id of local 0
      Node* dst = out.nodes.data() + base[c];
      for (size_t i = 0; i < ch.nodes.size(); ++i) {
        Node nd = ch.nodes[i];
        if (nd.type == NT_OBJ || nd.type == NT_ARR) nd.first += g;
        dst[i] = nd;
      }
      for (const auto& w : ch.words) out.words[w.first] = (CW_NODE << CW_SHIFT) | (g + w.second);
      for (const auto& f : ch.cols) {
        ReviewCol& rc = out.cols[f.first / 3];
        (f.first % 3 == 0 ? rc.labels : f.first % 3 == 1 ? rc.old_labels : rc.ns_labels) = g + f.second;
      }
      std::vector<Node>().swap(ch.nodes);
    }
  });
  if (trace) fprintf(stderr, "columns: D nodes %.1f ms (%zu kept)\n", ms(), out.nodes.size());
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
        << (x.slot != NO_ID && (out.slots[x.slot].flags & CVS_BYTES) ? " bytes" : "")
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
