// Go RE2 subset -> byte DFA (host).  Semantics of re_match
// (vendor/github.com/open-policy-agent/opa/topdown/regex.go:21-34): Go
// regexp.Compile + unanchored MatchString over the UTF-8 text.
//   * `^` / `\A` = beginning of text, `$` / `\z` = end of text (no (?m));
//   * `.` = any character except '\n' (any with (?s)); classes \d \w \s ASCII;
//   * `\s` = [\t\n\f\r ] (Go's Perl class: no \v, regexp/syntax perl_groups.go);
//   * (?i) is Go's simple case folding (regexp/syntax appendFoldedClass): the
//     ASCII letters pair up, and a set holding k/K also matches U+212A (KELVIN
//     SIGN) and one holding s/S U+017F (LATIN SMALL LETTER LONG S) -- the only
//     non-ASCII members of ASCII letters' fold orbits -- as their UTF-8 byte
//     sequences; lazy quantifiers behave like greedy for a match/no-match answer.
// Constructs whose behaviour depends on UTF-8 decoding (`.`, negated classes,
// \D \W \S) mark the DFA "utf8-sensitive": the kernel serves texts with bytes
// >= 0x80 through the CPU fallback.  \b, Unicode classes, (?m), (?U) and
// backtracking-only syntax are RX_UNSUPPORTED; syntax Go rejects is RX_INVALID.
#include "regex.h"

#include <algorithm>
#include <bitset>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>

namespace gk {
namespace {

struct RxErr {
  int status;
};

using CSet = std::bitset<256>;

struct Ast {
  enum T { LIT, CAT, ALT, STAR, PLUS, QUEST, REP, BOL, EOL, EMPTY } t;
  CSet set;
  std::vector<std::shared_ptr<Ast>> kids;
  int mn = 0, mx = 0;  // REP: mx = -1 unbounded
};
using AstP = std::shared_ptr<Ast>;

AstP mk(Ast::T t) { auto a = std::make_shared<Ast>(); a->t = t; return a; }

struct Parser {
  std::string p;
  size_t i = 0;
  bool icase = false, dotall = false;
  bool utf8_sensitive = false;

  [[noreturn]] void invalid() { throw RxErr{RX_INVALID}; }
  [[noreturn]] void unsupported() { throw RxErr{RX_UNSUPPORTED}; }

  AstP parse() {
    AstP a = alt();
    if (i != p.size()) {
      if (p[i] == ')') invalid();  // unexpected )
      invalid();
    }
    return a;
  }
  AstP alt() {
    std::vector<AstP> br{cat()};
    while (i < p.size() && p[i] == '|') { ++i; br.push_back(cat()); }
    if (br.size() == 1) return br[0];
    auto a = mk(Ast::ALT);
    a->kids = br;
    return a;
  }
  AstP cat() {
    auto a = mk(Ast::CAT);
    while (i < p.size() && p[i] != '|' && p[i] != ')') {
      AstP at = atom();
      if (!at) continue;
      at = quant(at);
      a->kids.push_back(at);
    }
    if (a->kids.empty()) return mk(Ast::EMPTY);
    if (a->kids.size() == 1) return a->kids[0];
    return a;
  }
  static bool isdig(char c) { return c >= '0' && c <= '9'; }
  AstP quant(AstP a) {
    bool repeated = false;
    while (i < p.size()) {
      char c = p[i];
      AstP q;
      if (c == '*' || c == '+' || c == '?') {
        if (repeated) invalid();  // invalid nested repetition operator
        q = mk(c == '*' ? Ast::STAR : c == '+' ? Ast::PLUS : Ast::QUEST);
        ++i;
      } else if (c == '{') {
        size_t j = i + 1;
        int mn = 0, mx = 0;
        if (j >= p.size() || !isdig(p[j])) break;  // literal '{'
        size_t s = j;
        while (j < p.size() && isdig(p[j])) ++j;
        mn = std::stoi(p.substr(s, std::min<size_t>(j - s, 6)));
        if (j < p.size() && p[j] == ',') {
          ++j;
          if (j < p.size() && isdig(p[j])) {
            size_t s2 = j;
            while (j < p.size() && isdig(p[j])) ++j;
            mx = std::stoi(p.substr(s2, std::min<size_t>(j - s2, 6)));
          } else mx = -1;
        } else mx = mn;
        if (j >= p.size() || p[j] != '}') break;  // literal
        if (repeated) invalid();
        if (mn > 1000 || mx > 1000 || (mx >= 0 && mx < mn)) invalid();
        q = mk(Ast::REP);
        q->mn = mn;
        q->mx = mx;
        i = j + 1;
      } else break;
      if (i < p.size() && p[i] == '?') ++i;  // lazy: same match/no-match answer
      if (a->t == Ast::BOL || a->t == Ast::EOL || a->t == Ast::EMPTY) {
        // Go accepts e.g. `^*`; keep semantics: repetition of an empty-width op
      }
      q->kids.push_back(a);
      a = q;
      repeated = true;
    }
    return a;
  }
  CSet fold(CSet s) {
    if (!icase) return s;
    for (int c = 'a'; c <= 'z'; ++c) {
      if (s[c] || s[c - 32]) { s[c] = true; s[c - 32] = true; }
    }
    return s;
  }
  // a (folded) byte set as a node: under (?i) a set with k or s also matches
  // the UTF-8 of U+212A (E2 84 AA) / U+017F (C5 BF), Go's fold orbits of those
  // letters (unicode.SimpleFold); negated sets stay single bytes (they are
  // utf8-sensitive, so non-ASCII subjects take the CPU fallback)
  AstP lit(const CSet& s) {
    auto a = mk(Ast::LIT);
    a->set = s;
    if (!icase || !(s['k'] || s['s'])) return a;
    auto alt = mk(Ast::ALT);
    alt->kids.push_back(a);
    auto seq = [&](std::initializer_list<int> bytes) {
      auto c = mk(Ast::CAT);
      for (int b : bytes) {
        auto l = mk(Ast::LIT);
        l->set[b] = true;
        c->kids.push_back(l);
      }
      alt->kids.push_back(c);
    };
    if (s['k']) seq({0xE2, 0x84, 0xAA});
    if (s['s']) seq({0xC5, 0xBF});
    return alt;
  }
  static CSet cls_digit() { CSet s; for (int c = '0'; c <= '9'; ++c) s[c] = true; return s; }
  static CSet cls_word() {
    CSet s = cls_digit();
    for (int c = 'a'; c <= 'z'; ++c) s[c] = s[c - 32] = true;
    s['_'] = true;
    return s;
  }
  static CSet cls_space() { CSet s; for (char c : std::string("\t\n\f\r ")) s[(unsigned char)c] = true; return s; }
  static CSet ascii_neg(const CSet& s) {
    CSet r;
    for (int c = 0; c < 128; ++c) r[c] = !s[c];
    return r;
  }
  // parse an escape after '\'; returns true and fills set for class escapes,
  // or a single byte in *ch
  bool escape(CSet* set, int* ch) {
    if (i >= p.size()) invalid();
    char c = p[i++];
    switch (c) {
      case 'd': *set = cls_digit(); return true;
      case 'w': *set = cls_word(); return true;
      case 's': *set = cls_space(); return true;
      case 'D': *set = ascii_neg(cls_digit()); utf8_sensitive = true; return true;
      case 'W': *set = ascii_neg(cls_word()); utf8_sensitive = true; return true;
      case 'S': *set = ascii_neg(cls_space()); utf8_sensitive = true; return true;
      case 'n': *ch = '\n'; return false;
      case 't': *ch = '\t'; return false;
      case 'r': *ch = '\r'; return false;
      case 'f': *ch = '\f'; return false;
      case 'v': *ch = '\v'; return false;
      case 'a': *ch = '\a'; return false;
      case 'x': {
        if (i < p.size() && p[i] == '{') unsupported();
        if (i + 2 > p.size()) invalid();
        int v = 0;
        for (int k = 0; k < 2; ++k) {
          char h = p[i++];
          int d = isdig(h) ? h - '0' : (h >= 'a' && h <= 'f') ? h - 'a' + 10 : (h >= 'A' && h <= 'F') ? h - 'A' + 10 : -1;
          if (d < 0) invalid();
          v = v * 16 + d;
        }
        if (v >= 0x80) unsupported();
        *ch = v;
        return false;
      }
      case 'p': case 'P': case 'Q': case 'E': case 'b': case 'B': case 'C': unsupported();
      default:
        if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || isdig(c)) {
          if (c == '0') unsupported();  // octal
          invalid();
        }
        if ((unsigned char)c >= 0x80) invalid();
        *ch = (unsigned char)c;
        return false;
    }
  }
  AstP atom() {
    char c = p[i];
    if (c == '(') {
      ++i;
      if (i < p.size() && p[i] == '?') {
        ++i;
        if (i < p.size() && p[i] == 'P') {
          ++i;
          if (i >= p.size() || p[i] != '<') invalid();
          size_t e = p.find('>', i);
          if (e == std::string::npos) invalid();
          i = e + 1;
        } else {
          // flags: (?flags) or (?flags:re)
          bool neg = false;
          bool saw = false;
          bool ni = icase, ns = dotall;
          while (i < p.size() && p[i] != ')' && p[i] != ':') {
            char f = p[i++];
            saw = true;
            if (f == '-') { if (neg) invalid(); neg = true; continue; }
            if (f == 'i') ni = !neg;
            else if (f == 's') ns = !neg;
            else if (f == 'm' || f == 'U') unsupported();
            else invalid();
          }
          if (i >= p.size()) invalid();
          if (!saw && p[i] == ')') invalid();
          if (p[i] == ')') {
            ++i;
            icase = ni;
            dotall = ns;
            return nullptr;
          }
          ++i;  // ':'
          bool oi = icase, os = dotall;
          icase = ni;
          dotall = ns;
          AstP a = alt();
          icase = oi;
          dotall = os;
          if (i >= p.size() || p[i] != ')') invalid();
          ++i;
          return a;
        }
      }
      bool oi = icase, os = dotall;
      AstP a = alt();
      icase = oi;
      dotall = os;
      if (i >= p.size() || p[i] != ')') invalid();
      ++i;
      return a;
    }
    if (c == '*' || c == '+' || c == '?') invalid();  // missing argument to repetition operator
    if (c == '{') {
      // `{` not starting a valid repeat is a literal
      size_t save = i;
      ++i;
      auto a = mk(Ast::LIT);
      a->set['{'] = true;
      (void)save;
      return a;
    }
    if (c == '^') { ++i; return mk(Ast::BOL); }
    if (c == '$') { ++i; return mk(Ast::EOL); }
    if (c == '.') {
      ++i;
      auto a = mk(Ast::LIT);
      for (int b = 0; b < 128; ++b) a->set[b] = true;
      if (!dotall) a->set['\n'] = false;
      utf8_sensitive = true;
      return a;
    }
    if (c == '[') return cls();
    if (c == '\\') {
      ++i;
      if (i < p.size() && p[i] == 'A') { ++i; return mk(Ast::BOL); }
      if (i < p.size() && p[i] == 'z') { ++i; return mk(Ast::EOL); }
      CSet s;
      int ch = -1;
      if (!escape(&s, &ch)) s[ch] = true;
      return lit(fold(s));
    }
    // literal (UTF-8 multi-byte sequences are literal byte strings)
    unsigned char u = (unsigned char)c;
    if (u >= 0x80) {
      if (icase) unsupported();
      size_t len = (u >= 0xF0) ? 4 : (u >= 0xE0) ? 3 : (u >= 0xC0) ? 2 : 1;
      auto a = mk(Ast::CAT);
      for (size_t k = 0; k < len && i < p.size(); ++k) {
        auto l = mk(Ast::LIT);
        l->set[(unsigned char)p[i++]] = true;
        a->kids.push_back(l);
      }
      return a;
    }
    ++i;
    CSet one;
    one[u] = true;
    return lit(fold(one));
  }
  AstP cls() {
    ++i;  // '['
    bool neg = false;
    if (i < p.size() && p[i] == '^') { neg = true; ++i; }
    CSet s;
    bool first = true;
    while (true) {
      if (i >= p.size()) invalid();  // missing closing ]
      char c = p[i];
      if (c == ']' && !first) { ++i; break; }
      first = false;
      if (c == '[' && i + 1 < p.size() && p[i + 1] == ':') unsupported();
      int lo;
      if (c == '\\') {
        ++i;
        CSet es;
        int ch = -1;
        if (escape(&es, &ch)) { s |= es; continue; }
        lo = ch;
      } else {
        if ((unsigned char)c >= 0x80) unsupported();
        lo = (unsigned char)c;
        ++i;
      }
      if (i + 1 < p.size() && p[i] == '-' && p[i + 1] != ']') {
        ++i;
        int hi;
        if (p[i] == '\\') {
          ++i;
          CSet es;
          int ch = -1;
          if (escape(&es, &ch)) invalid();
          hi = ch;
        } else {
          if ((unsigned char)p[i] >= 0x80) unsupported();
          hi = (unsigned char)p[i++];
        }
        if (hi < lo) invalid();
        for (int b = lo; b <= hi; ++b) s[b] = true;
      } else {
        s[lo] = true;
      }
    }
    s = fold(s);
    if (!neg) return lit(s);
    auto a = mk(Ast::LIT);
    a->set = ascii_neg(s);
    utf8_sensitive = true;  // also matches any non-ASCII character
    return a;
  }
};

// ------------------------------------------------------------------ NFA
struct NState {
  enum T { CHAR, SPLIT, JMP, BOL, EOL, MATCH } t;
  CSet set;
  int out = -1, out2 = -1;
};

struct Nfa {
  std::vector<NState> s;
  int add(NState::T t) {
    if (s.size() > 20000) throw RxErr{RX_UNSUPPORTED};
    NState n;
    n.t = t;
    s.push_back(n);
    return (int)s.size() - 1;
  }
  struct Frag { int start; std::vector<int*> outs_idx; std::vector<std::pair<int, int>> outs; };
  // fragment: start state + list of (state, which-out) dangling edges
  void patch(std::vector<std::pair<int, int>>& outs, int to) {
    for (auto& o : outs) (o.second == 0 ? s[o.first].out : s[o.first].out2) = to;
  }
  std::pair<int, std::vector<std::pair<int, int>>> build(const AstP& a) {
    switch (a->t) {
      case Ast::LIT: { int x = add(NState::CHAR); s[x].set = a->set; return {x, {{x, 0}}}; }
      case Ast::BOL: { int x = add(NState::BOL); return {x, {{x, 0}}}; }
      case Ast::EOL: { int x = add(NState::EOL); return {x, {{x, 0}}}; }
      case Ast::EMPTY: { int x = add(NState::JMP); return {x, {{x, 0}}}; }
      case Ast::CAT: {
        auto f = build(a->kids[0]);
        for (size_t k = 1; k < a->kids.size(); ++k) {
          auto g = build(a->kids[k]);
          patch(f.second, g.first);
          f.second = g.second;
        }
        return f;
      }
      case Ast::ALT: {
        auto f = build(a->kids[0]);
        for (size_t k = 1; k < a->kids.size(); ++k) {
          auto g = build(a->kids[k]);
          int sp = add(NState::SPLIT);
          s[sp].out = f.first;
          s[sp].out2 = g.first;
          f.first = sp;
          f.second.insert(f.second.end(), g.second.begin(), g.second.end());
        }
        return f;
      }
      case Ast::STAR: {
        auto f = build(a->kids[0]);
        int sp = add(NState::SPLIT);
        s[sp].out = f.first;
        patch(f.second, sp);
        return {sp, {{sp, 1}}};
      }
      case Ast::PLUS: {
        auto f = build(a->kids[0]);
        int sp = add(NState::SPLIT);
        s[sp].out = f.first;
        patch(f.second, sp);
        return {f.first, {{sp, 1}}};
      }
      case Ast::QUEST: {
        auto f = build(a->kids[0]);
        int sp = add(NState::SPLIT);
        s[sp].out = f.first;
        f.second.push_back({sp, 1});
        return {sp, f.second};
      }
      case Ast::REP: {
        // x{n,m} = x^n (x?)^(m-n); x{n,} = x^n x*
        auto cat = mk(Ast::CAT);
        for (int k = 0; k < a->mn; ++k) cat->kids.push_back(a->kids[0]);
        if (a->mx < 0) {
          auto st = mk(Ast::STAR);
          st->kids.push_back(a->kids[0]);
          cat->kids.push_back(st);
        } else {
          for (int k = a->mn; k < a->mx; ++k) {
            auto q = mk(Ast::QUEST);
            q->kids.push_back(a->kids[0]);
            cat->kids.push_back(q);
          }
        }
        if (cat->kids.empty()) return build(mk(Ast::EMPTY));
        return build(cat);
      }
    }
    throw RxErr{RX_UNSUPPORTED};
  }
};

void closure(const Nfa& n, std::vector<int> seeds, bool bol, bool eol, std::set<int>& out) {
  std::vector<int> st = seeds;
  std::set<int> seen;
  while (!st.empty()) {
    int x = st.back();
    st.pop_back();
    if (x < 0 || seen.count(x)) continue;
    seen.insert(x);
    const NState& s = n.s[x];
    switch (s.t) {
      case NState::SPLIT: st.push_back(s.out); st.push_back(s.out2); break;
      case NState::JMP: st.push_back(s.out); break;
      case NState::BOL: if (bol) st.push_back(s.out); break;
      case NState::EOL: out.insert(x); if (eol) st.push_back(s.out); break;
      default: out.insert(x); break;
    }
  }
}

}  // namespace

int compile_regex_dfa(const std::string& pattern, std::vector<uint32_t>& out) {
  try {
    Parser ps;
    ps.p = pattern;
    AstP ast = ps.parse();
    Nfa nfa;
    auto f = nfa.build(ast);
    int m = nfa.add(NState::MATCH);
    nfa.patch(f.second, m);
    int start = f.first;
    bool anchored = false;
    // unanchored search: restart at every position unless the pattern
    // can only match at the beginning (leading ^ on every branch)
    {
      std::set<int> c0;
      closure(nfa, {start}, false, false, c0);
      std::set<int> c1;
      closure(nfa, {start}, true, false, c1);
      anchored = c0.empty() && !c1.empty() ? false : false;  // always restart; BOL states simply fail later
    }
    (void)anchored;
    std::map<std::vector<int>, int> ids;
    std::vector<std::vector<int>> states;
    std::vector<bool> is_start;
    auto intern = [&](const std::set<int>& s, bool st0) {
      std::vector<int> v(s.begin(), s.end());
      if (st0) v.push_back(-1);  // the start state (position 0) is distinct
      auto it = ids.find(v);
      if (it != ids.end()) return it->second;
      int id = (int)states.size();
      ids[v] = id;
      states.push_back(v);
      is_start.push_back(st0);
      if (states.size() > 4000) throw RxErr{RX_UNSUPPORTED};
      return id;
    };
    std::set<int> s0;
    closure(nfa, {start}, true, false, s0);
    intern(s0, true);
    std::vector<std::vector<int>> trans;
    std::vector<uint32_t> acc;
    for (size_t k = 0; k < states.size(); ++k) {
      std::vector<int> cur;
      for (int x : states[k]) if (x >= 0) cur.push_back(x);
      bool st0 = is_start[k];
      uint32_t a = 0;
      for (int x : cur) if (nfa.s[x].t == NState::MATCH) a |= 1;
      {
        std::vector<int> seeds;
        for (int x : cur) if (nfa.s[x].t == NState::EOL) seeds.push_back(nfa.s[x].out);
        std::set<int> e;
        closure(nfa, seeds, st0, true, e);
        for (int x : e) if (nfa.s[x].t == NState::MATCH) a |= 2;
      }
      acc.push_back(a);
      std::vector<int> row(256, -1);
      for (int c = 0; c < 256; ++c) {
        std::vector<int> seeds;
        for (int x : cur) if (nfa.s[x].t == NState::CHAR && nfa.s[x].set[c]) seeds.push_back(nfa.s[x].out);
        seeds.push_back(start);  // unanchored restart (BOL edges fail past position 0)
        std::set<int> nx;
        closure(nfa, seeds, false, false, nx);
        row[c] = nx.empty() ? -1 : intern(nx, false);
      }
      trans.push_back(row);
    }
    uint32_t nst = (uint32_t)states.size();
    out.push_back(nst);
    out.push_back(0);
    out.push_back(ps.utf8_sensitive ? 1u : 0u);
    for (uint32_t k = 0; k < nst; ++k) {
      out.push_back(acc[k]);
      for (int c = 0; c < 256; c += 2) {
        uint32_t lo = trans[k][c] < 0 ? 0xffffu : (uint32_t)trans[k][c];
        uint32_t hi = trans[k][c + 1] < 0 ? 0xffffu : (uint32_t)trans[k][c + 1];
        out.push_back(lo | (hi << 16));
      }
    }
    return RX_OK;
  } catch (const RxErr& e) {
    return e.status;
  } catch (...) {
    return RX_UNSUPPORTED;
  }
}

int run_regex_dfa(const uint32_t* d, const std::string& text) {
  uint32_t nst = d[0], s = d[1], sens = d[2];
  const uint32_t* st = d + 3;
  for (unsigned char c : text) {
    if (c >= 0x80 && sens) return -2;
    const uint32_t* row = st + s * 129;
    if (row[0] & 1) return 1;
    uint32_t w = row[1 + (c >> 1)];
    s = (c & 1) ? (w >> 16) : (w & 0xffff);
    if (s >= nst) return 0;
  }
  return (st[s * 129] & 3) ? 1 : 0;
}

}  // namespace gk

extern "C" int gk_regex_test(const char* pattern, const char* text, size_t len) {
  std::vector<uint32_t> w;
  int st = gk::compile_regex_dfa(pattern, w);
  if (st == gk::RX_INVALID) return -1;
  if (st != gk::RX_OK) return -2;
  return gk::run_regex_dfa(w.data(), std::string(text, len));
}

namespace gk {

// Byte-class compression of a DFA in compile_regex_dfa's layout, for the LDS
// copy a wavefront stages (devrt.h re_run_lds): two bytes share a class when
// every state sends them to the same state, so a row needs one entry per class
// instead of 256.  Layout: [0, 256) class of each byte, then nst x ncls u8
// transitions (255 = dead), then nst u8 accept flags (bit0 match already
// found, bit1 accepting at end of text).  false when there are more than 254
// states or the table exceeds max_bytes.
bool compress_regex_dfa(const std::vector<uint32_t>& d, size_t max_bytes, std::vector<uint8_t>& out, uint32_t& nst,
                        uint32_t& ncls, uint32_t& start, uint32_t& sens) {
  if (d.size() < 3) return false;
  nst = d[0];
  start = d[1];
  sens = d[2];
  if (nst == 0 || nst > 254 || d.size() < 3 + (size_t)nst * 129) return false;
  const uint32_t* st = d.data() + 3;
  auto target = [&](uint32_t s, uint32_t c) -> uint32_t {
    uint32_t w = st[s * 129 + 1 + (c >> 1)];
    uint32_t t = (c & 1) ? (w >> 16) : (w & 0xffff);
    return t >= nst ? 255u : t;
  };
  std::vector<uint8_t> cls(256);
  std::vector<uint32_t> rep;  // a representative byte per class
  for (uint32_t c = 0; c < 256; ++c) {
    uint32_t k = 0;
    for (; k < rep.size(); ++k) {
      bool same = true;
      for (uint32_t s = 0; s < nst && same; ++s) same = target(s, c) == target(s, rep[k]);
      if (same) break;
    }
    if (k == rep.size()) rep.push_back(c);
    cls[c] = (uint8_t)k;
  }
  ncls = (uint32_t)rep.size();
  const size_t bytes = 256 + (size_t)nst * ncls + nst;
  if (bytes > max_bytes) return false;
  out.assign(bytes, 0);
  for (uint32_t c = 0; c < 256; ++c) out[c] = cls[c];
  for (uint32_t s = 0; s < nst; ++s) {
    for (uint32_t k = 0; k < ncls; ++k) out[256 + s * ncls + k] = (uint8_t)target(s, rep[k]);
    out[256 + (size_t)nst * ncls + s] = (uint8_t)(st[s * 129] & 3);
  }
  return true;
}

// host-side matcher over the compressed form (tests): the semantics of
// run_regex_dfa / devrt.h re_run
int run_regex_cdfa(const std::vector<uint8_t>& t, uint32_t nst, uint32_t ncls, uint32_t start, uint32_t sens,
                   const std::string& text) {
  uint32_t s = start;
  for (unsigned char c : text) {
    if (c >= 0x80 && sens) return -2;
    if (t[256 + (size_t)nst * ncls + s] & 1) return 1;
    s = t[256 + (size_t)s * ncls + t[c]];
    if (s >= nst) return 0;
  }
  return (t[256 + (size_t)nst * ncls + s] & 3) ? 1 : 0;
}

}  // namespace gk

// the byte-class-compressed form of the same DFA (tests: must agree with
// gk_regex_test on every input); -3 when the DFA does not compress
extern "C" int gk_regex_ctest(const char* pattern, const char* text, size_t len) {
  std::vector<uint32_t> w;
  int st = gk::compile_regex_dfa(pattern, w);
  if (st == gk::RX_INVALID) return -1;
  if (st != gk::RX_OK) return -2;
  std::vector<uint8_t> t;
  uint32_t nst, ncls, start, sens;
  if (!gk::compress_regex_dfa(w, 1 << 20, t, nst, ncls, start, sens)) return -3;
  return gk::run_regex_cdfa(t, nst, ncls, start, sens, std::string(text, len));
}
