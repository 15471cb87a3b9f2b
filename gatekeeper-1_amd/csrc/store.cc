// Host-side interned store (strings, numbers, node arena) + exact number
// conversions matching Go's math/big / strconv behaviour.
#include "store.h"

#include <emmintrin.h>
#include "flatten.h"

#include <atomic>
#include <charconv>
#include <chrono>
#include <cstdio>
#include <functional>
#include <stdexcept>
#include <thread>
#include <cmath>
#include <cstdlib>
#include <deque>

namespace gk {

// ------------------------------------------------------------------ bignum
namespace {
struct Big {
  std::vector<uint32_t> w;  // little endian
  void trim() { while (!w.empty() && w.back() == 0) w.pop_back(); }
  bool zero() const { return w.empty(); }
  int bitlen() const {
    if (w.empty()) return 0;
    return (int)(w.size() - 1) * 32 + (32 - __builtin_clz(w.back()));
  }
  void mul_small(uint32_t m) {
    uint64_t c = 0;
    for (auto& x : w) { uint64_t v = (uint64_t)x * m + c; x = (uint32_t)v; c = v >> 32; }
    if (c) w.push_back((uint32_t)c);
  }
  void add_small(uint32_t a) {
    uint64_t c = a;
    for (auto& x : w) { if (!c) break; uint64_t v = (uint64_t)x + c; x = (uint32_t)v; c = v >> 32; }
    if (c) w.push_back((uint32_t)c);
  }
  void shl(int s) {
    if (zero() || s == 0) return;
    int ws = s / 32, bs = s % 32;
    std::vector<uint32_t> r(w.size() + ws + 1, 0);
    for (size_t i = 0; i < w.size(); ++i) {
      uint64_t v = (uint64_t)w[i] << bs;
      r[i + ws] |= (uint32_t)v;
      r[i + ws + 1] |= (uint32_t)(v >> 32);
    }
    w.swap(r);
    trim();
  }
  bool bit(int i) const { return (size_t)(i / 32) < w.size() && ((w[i / 32] >> (i % 32)) & 1); }
  static int cmp(const Big& a, const Big& b) {
    if (a.w.size() != b.w.size()) return a.w.size() < b.w.size() ? -1 : 1;
    for (size_t i = a.w.size(); i-- > 0;) if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
    return 0;
  }
  void sub(const Big& b) {  // *this >= b
    int64_t br = 0;
    for (size_t i = 0; i < w.size(); ++i) {
      int64_t v = (int64_t)w[i] - (i < b.w.size() ? b.w[i] : 0) - br;
      br = v < 0;
      w[i] = (uint32_t)(v + (br ? (1ll << 32) : 0));
    }
    trim();
  }
  // quotient bits (q) and remainder (r) of a / b, via shift-subtract
  static void divmod(const Big& a, const Big& b, Big& q, Big& r) {
    q.w.assign(a.w.size() + 1, 0);
    r.w.clear();
    for (int i = a.bitlen() - 1; i >= 0; --i) {
      r.shl(1);
      if (a.bit(i)) { if (r.w.empty()) r.w.push_back(1); else r.w[0] |= 1; }
      if (cmp(r, b) >= 0) { r.sub(b); q.w[i / 32] |= 1u << (i % 32); }
    }
    q.trim();
  }
  uint64_t low64() const { return (w.size() > 0 ? w[0] : 0) | ((uint64_t)(w.size() > 1 ? w[1] : 0) << 32); }
};
}  // namespace

bool decimal_to_bf64(const char* s, size_t n, uint64_t* mant, int32_t* exp, bool* neg) {
  size_t i = 0;
  *neg = false;
  if (i < n && (s[i] == '-' || s[i] == '+')) { *neg = s[i] == '-'; ++i; }
  Big d;
  int ndig = 0, frac = 0;
  bool seen_dot = false, any = false;
  for (; i < n; ++i) {
    char c = s[i];
    if (c >= '0' && c <= '9') {
      any = true;
      if (!d.zero() || c != '0') { d.mul_small(10); d.add_small(c - '0'); if (d.w.empty() && c != '0') d.w.push_back(c - '0'); ++ndig; }
      if (seen_dot) ++frac;
    } else if (c == '.' && !seen_dot) {
      seen_dot = true;
    } else break;
  }
  if (!any) return false;
  long e10 = 0;
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    ++i;
    bool en = false;
    if (i < n && (s[i] == '+' || s[i] == '-')) { en = s[i] == '-'; ++i; }
    if (i >= n) return false;
    long v = 0;
    for (; i < n; ++i) {
      if (s[i] < '0' || s[i] > '9') return false;
      v = v * 10 + (s[i] - '0');
      if (v > 100000) return false;
    }
    e10 = en ? -v : v;
  }
  if (i != n) return false;
  if (ndig > 800) return false;
  e10 -= frac;
  if (d.zero()) { *mant = 0; *exp = 0; return true; }
  if (e10 > 800 || e10 < -800) return false;
  if (e10 >= 0) {
    for (long k = 0; k < e10; ++k) d.mul_small(10);
    int L = d.bitlen();
    if (L <= 64) {
      uint64_t v = d.low64();
      *mant = v << (64 - L);
      *exp = L - 64;
      return true;
    }
    int sh = L - 64;
    // q = d >> sh, remainder bits
    Big q = d;
    // shift right by sh
    {
      int ws = sh / 32, bs = sh % 32;
      std::vector<uint32_t> r;
      for (size_t j = ws; j < q.w.size(); ++j) {
        uint64_t v = q.w[j] >> bs;
        if (bs && j + 1 < q.w.size()) v |= (uint64_t)q.w[j + 1] << (32 - bs);
        r.push_back((uint32_t)v);
      }
      q.w.swap(r);
      q.trim();
    }
    uint64_t m = q.low64();
    bool half = d.bit(sh - 1);
    bool rest = false;
    for (int b = 0; b < sh - 1 && !rest; ++b) rest = d.bit(b);
    bool up = half && (rest || (m & 1));
    int32_t e = sh;
    if (up) { ++m; if (m == 0) { m = 1ull << 63; ++e; } }
    *mant = m;
    *exp = e;
    return true;
  }
  // d / 10^k
  Big den;
  den.w.push_back(1);
  for (long k = 0; k < -e10; ++k) den.mul_small(10);
  int t = 64 + den.bitlen() - d.bitlen();
  for (int iter = 0; iter < 4; ++iter) {
    Big num = d;
    if (t > 0) num.shl(t);
    Big denx = den;
    if (t < 0) denx.shl(-t);
    Big q, r;
    Big::divmod(num, denx, q, r);
    int ql = q.bitlen();
    if (ql > 64) { --t; continue; }
    if (ql < 64) { ++t; continue; }
    uint64_t m = q.low64();
    // round half even: compare 2r with denx
    r.shl(1);
    int c = Big::cmp(r, denx);
    int32_t e = -t;
    if (c > 0 || (c == 0 && (m & 1))) { ++m; if (m == 0) { m = 1ull << 63; ++e; } }
    *mant = m;
    *exp = e;
    return true;
  }
  return false;
}

bool parse_int64(const char* s, size_t n, int64_t* out) {
  if (n == 0) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
  if (i >= n) return false;
  unsigned __int128 v = 0;
  for (; i < n; ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
    if (v > ((unsigned __int128)1 << 63)) return false;
  }
  if (!neg && v > (((unsigned __int128)1 << 63) - 1)) return false;
  *out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
  return true;
}

// Go strconv 'g' shortest formatting (%v of float64): %e when exp < -4 || exp >= 6
static std::string go_float_v(double f) {
  if (std::isinf(f)) return f > 0 ? "+Inf" : "-Inf";
  if (std::isnan(f)) return "NaN";
  if (f == 0) return std::signbit(f) ? "-0" : "0";
  char buf[64];
  auto res = std::to_chars(buf, buf + sizeof(buf), std::fabs(f), std::chars_format::scientific);
  std::string sci(buf, res.ptr);
  size_t epos = sci.find('e');
  std::string mant = sci.substr(0, epos);
  int ex = atoi(sci.c_str() + epos + 1);
  std::string digits;
  for (char c : mant) if (c != '.') digits.push_back(c);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  int dp = ex + 1;
  std::string out;
  if (ex < -4 || ex >= 6) {
    out = digits.substr(0, 1);
    if (digits.size() > 1) out += "." + digits.substr(1);
    out += "e";
    out += ex < 0 ? "-" : "+";
    int ae = ex < 0 ? -ex : ex;
    if (ae < 10) out += "0";
    out += std::to_string(ae);
  } else if (dp <= 0) {
    out = "0." + std::string(-dp, '0') + digits;
  } else if ((size_t)dp >= digits.size()) {
    out = digits + std::string(dp - digits.size(), '0');
  } else {
    out = digits.substr(0, dp) + "." + digits.substr(dp);
  }
  return (f < 0 ? "-" : "") + out;
}

std::string go_number_print(const char* s, size_t n) {
  int64_t v;
  if (parse_int64(s, n, &v)) return std::to_string(v);
  std::string t(s, n);
  char* end = nullptr;
  double f = strtod(t.c_str(), &end);
  if (end != t.c_str() + t.size()) return t;
  if (std::isinf(f)) return t;  // Float64() fails -> number text
  return go_float_v(f);
}

// ------------------------------------------------------------------ Store
Store::Store() {
  table_.assign(1 << 12, 0);
  num_table_.assign(1 << 10, 0);
  init();
}

void Store::reset() {
  pool_.clear();
  strs_.clear();
  sflags_.clear();
  if (table_.size() > (1u << 16)) table_.assign(1 << 12, 0);
  else std::fill(table_.begin(), table_.end(), 0);
  nums_.clear();
  if (num_table_.size() > (1u << 14)) num_table_.assign(1 << 10, 0);
  else std::fill(num_table_.begin(), num_table_.end(), 0);
  nodes_.resize(0);
  if (!short_.empty()) std::fill(short_.begin(), short_.end(), ShortEnt{{0, 0, 0, 0}, ~0u, 0});
  init();
}

void Store::init() {
  s_empty = intern("", 0);
  s_review = intern("review"); s_parameters = intern("parameters"); s_kind = intern("kind");
  s_group = intern("group"); s_version = intern("version"); s_name = intern("name");
  s_namespace = intern("namespace"); s_object = intern("object"); s_oldObject = intern("oldObject");
  s_metadata = intern("metadata"); s_labels = intern("labels"); s_unstable = intern("_unstable");
  s_msg = intern("msg"); s_details = intern("details"); s_uid = intern("uid"); s_resource = intern("resource");
  s_operation = intern("operation"); s_userInfo = intern("userInfo"); s_options = intern("options");
  s_deny = intern("deny"); s_creationTimestamp = intern("creationTimestamp"); s_spec = intern("spec");
  s_status = intern("status"); s_star = intern("*"); s_In = intern("In"); s_NotIn = intern("NotIn");
  s_Exists = intern("Exists"); s_DoesNotExist = intern("DoesNotExist"); s_Namespace = intern("Namespace");
  s_apiGroups = intern("apiGroups"); s_kinds = intern("kinds"); s_true = intern("true");
  s_false = intern("false"); s_null = intern("null");
  // node 0 is a permanent empty object ({}), node 1 null, node 2 false, node 3 true
  Node e{};
  e.type = NT_OBJ;
  nodes_.push_back(e);
  e.type = NT_NULL; nodes_.push_back(e);
  e.type = NT_FALSE; nodes_.push_back(e);
  e.type = NT_TRUE; nodes_.push_back(e);
}

// Intern table: open addressing, one 64-bit slot per entry = hash tag (high 32
// bits of the string hash) << 32 | (string id + 1); 0 = empty.  A probe only
// touches the string table and pool when the tags agree.
static inline uint64_t slot_of(uint64_t h, uint32_t id) { return (h & 0xffffffff00000000ull) | (uint64_t)(id + 1); }

void Store::rehash(size_t sz) {
  std::vector<uint64_t> t(sz, 0);
  size_t mask = sz - 1;
  for (uint32_t id = 0; id < strs_.size(); ++id) {
    uint64_t hv = str_hash(pool_.data() + strs_[id].off, strs_[id].len);
    size_t h = hv & mask;
    while (t[h]) h = (h + 1) & mask;
    t[h] = slot_of(hv, id);
  }
  table_.swap(t);
}

void Store::grow() { rehash(table_.size() * 2); }

void Store::reserve_strings(size_t n) {
  size_t want = (strs_.size() + n) * 2 + 1;
  if (want > table_.size()) {
    size_t sz = table_.size();
    while (sz < want) sz *= 2;
    rehash(sz);
  }
  strs_.reserve(strs_.size() + n);
  sflags_.reserve(sflags_.size() + n);
}

uint32_t Store::find(const char* p, size_t n) const {
  size_t mask = table_.size() - 1;
  uint64_t hv = str_hash(p, n);
  uint64_t tag = hv & 0xffffffff00000000ull;
  size_t h = hv & mask;
  while (uint64_t e = table_[h]) {
    if ((e & 0xffffffff00000000ull) == tag) {
      uint32_t id = (uint32_t)e - 1;
      const StrEnt& s = strs_[id];
      if (s.len == n && memcmp(pool_.data() + s.off, p, n) == 0) return id;
    }
    h = (h + 1) & mask;
  }
  return NO_ID;
}

static uint8_t str_flags_of(const char* p, size_t n) {
  uint8_t fl = SF_ASCII_PRINT;
  for (size_t i = 0; i < n; ++i) {
    unsigned char c = (unsigned char)p[i];
    if (c >= 0x80) { fl |= SF_NON_ASCII; fl &= ~SF_ASCII_PRINT; }
    else if (c < 0x20 || c == 0x7f) { fl &= ~SF_ASCII_PRINT; }
    else if (c == '"' || c == '\\') fl |= SF_NEEDS_ESC;
  }
  return fl;
}

uint32_t Store::intern(const char* p, size_t n) {
  if (n <= 32 && !short_.empty()) {  // (the cache is set up by parse_doc)
    // the string as four words (overlapping loads; with n they determine it)
    uint64_t w[4] = {0, 0, 0, 0};
    if (n > 16) { memcpy(&w[0], p, 8); memcpy(&w[1], p + 8, 8); memcpy(&w[2], p + n - 16, 8); memcpy(&w[3], p + n - 8, 8); }
    else if (n >= 8) { memcpy(&w[0], p, 8); memcpy(&w[1], p + n - 8, 8); }
    else if (n >= 4) {
      uint32_t lo, hi;
      memcpy(&lo, p, 4);
      memcpy(&hi, p + n - 4, 4);
      w[0] = lo | (uint64_t)hi << 32;
    } else if (n) {
      w[0] = (uint8_t)p[0] | (uint32_t)(uint8_t)p[n >> 1] << 8 | (uint32_t)(uint8_t)p[n - 1] << 16;
    }
    const uint64_t k = (w[0] * 0x9e3779b97f4a7c15ull) ^ (w[1] * 0xc2b2ae3d27d4eb4full) ^
                       ((w[2] ^ (w[3] << 1)) * 0x94d049bb133111ebull) ^ (n * 0x165667b19e3779f9ull);
    ShortEnt& e = short_[(k >> 40) & (kShortCache - 1)];
    if (e.len == n && e.w[0] == w[0] && e.w[1] == w[1] && e.w[2] == w[2] && e.w[3] == w[3]) return e.id;
    const uint32_t id = intern_slow(p, n, str_hash(p, n));
    e = ShortEnt{{w[0], w[1], w[2], w[3]}, (uint32_t)n, id};
    return id;
  }
  return intern_slow(p, n, str_hash(p, n));
}

uint32_t Store::intern_slow(const char* p, size_t n, uint64_t hv) {
  size_t mask = table_.size() - 1;
  uint64_t tag = hv & 0xffffffff00000000ull;
  size_t h = hv & mask;
  while (uint64_t e = table_[h]) {
    if ((e & 0xffffffff00000000ull) == tag) {
      uint32_t id = (uint32_t)e - 1;
      const StrEnt& s = strs_[id];
      if (s.len == n && memcmp(pool_.data() + s.off, p, n) == 0) return id;
    }
    h = (h + 1) & mask;
  }
  uint32_t id = (uint32_t)strs_.size();
  StrEnt se{(uint32_t)pool_.size(), (uint32_t)n};
  pool_.append(p, n);
  strs_.push_back(se);
  sflags_.push_back(str_flags_of(p, n));
  table_[h] = slot_of(hv, id);
  if (strs_.size() * 2 > table_.size()) grow();
  return id;
}

void Store::grow_num() {
  std::vector<uint32_t> t(num_table_.size() * 2, 0);
  size_t mask = t.size() - 1;
  for (uint32_t id = 0; id < nums_.size(); ++id) {
    size_t h = (size_t)nums_[id].text * 2654435761u & mask;
    while (t[h]) h = (h + 1) & mask;
    t[h] = id + 1;
  }
  num_table_.swap(t);
}

uint32_t Store::number(const char* p, size_t n) {
  uint32_t text = intern(p, n);
  size_t mask = num_table_.size() - 1;
  size_t h = (size_t)text * 2654435761u & mask;
  while (uint32_t e = num_table_[h]) {
    if (nums_[e - 1].text == text) return e - 1;
    h = (h + 1) & mask;
  }
  NumEnt ne{};
  ne.text = text;
  int64_t iv;
  if (parse_int64(p, n, &iv)) { ne.i = iv; ne.flags |= NF_INT64; }
  uint64_t m; int32_t e; bool neg;
  if (decimal_to_bf64(p, n, &m, &e, &neg)) { ne.mant = m; ne.exp = e; ne.neg = neg; ne.flags |= NF_BF_OK; }
  std::string pr = go_number_print(p, n);
  ne.print = intern(pr);
  ne.flags |= NF_PRINT_OK;
  uint32_t id = (uint32_t)nums_.size();
  nums_.push_back(ne);
  num_table_[h] = id + 1;
  if (nums_.size() * 2 > num_table_.size()) grow_num();
  return id;
}

uint32_t Store::add_node(const Node& n) {
  nodes_.push_back(n);
  return (uint32_t)nodes_.size() - 1;
}

uint32_t Store::reserve(uint32_t n) {
  uint32_t f = (uint32_t)nodes_.size();
  nodes_.resize(nodes_.size() + n);
  return f;
}

uint32_t Store::add_doc(const JDoc& d, int j) {
  uint32_t root = (uint32_t)nodes_.size();
  nodes_.push_back(Node{});
  std::vector<BfsEnt>& q = bfs_;
  q.clear();
  q.push_back(BfsEnt{j, root, 0});
  for (size_t qi = 0; qi < q.size(); ++qi) {
    const BfsEnt be = q[qi];
    const uint32_t an = be.an;
    const JNode& x = d.nodes[be.jn];
    Node& out = nodes_[an];
    out = Node{};
    out.key = be.key;
    out.type = x.type;
    switch (x.type) {
      case NT_STR: out.val = intern(d.buf.data() + x.s_off, x.s_len); break;
      case NT_NUM: out.val = number(d.buf.data() + x.s_off, x.s_len); break;
      case NT_ARR:
      case NT_OBJ: {
        uint32_t cnt = x.n;
        if (cnt > 0xffff) { nodes_[an].flags |= 1; cnt = 0xffff; }
        uint32_t first = (uint32_t)nodes_.size();
        nodes_.resize(nodes_.size() + cnt);
        Node& o2 = nodes_[an];
        o2.first = first;
        o2.n = (uint16_t)cnt;
        uint32_t i = 0;
        for (int c = x.first; c >= 0 && i < cnt; c = d.nodes[c].next, ++i)
          q.push_back(BfsEnt{c, first + i, x.type == NT_OBJ ? intern(d.buf.data() + d.nodes[c].k_off, d.nodes[c].k_len) : i});
        break;
      }
      default: break;
    }
  }
  return root;
}

}  // namespace gk

namespace gk {

// Single-pass JSON -> node arena (Store::parse_doc).  Grammar and string
// decoding follow JsonReader (json.h) exactly; only the output differs.
class DocParser {
 public:
  DocParser(Store& st, const char* p, size_t n, std::string* err) : st_(st), p_(p), e_(p + n), err_(err) {}

  bool run(Node* root) {
    st_.pend_.clear();
    ws();
    if (!value(root, 0)) return false;
    ws();
    if (p_ != e_) return fail("trailing data");
    return true;
  }

 private:
  Store& st_;
  const char* p_;
  const char* e_;
  std::string* err_;

  bool fail(const char* m) {
    if (err_ && err_->empty()) *err_ = m;
    return false;
  }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\t' || *p_ == '\r')) ++p_;
  }
  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  static void put_utf8(std::string& b, uint32_t cp) {
    if (cp < 0x80) b.push_back((char)cp);
    else if (cp < 0x800) { b.push_back((char)(0xC0 | (cp >> 6))); b.push_back((char)(0x80 | (cp & 0x3F))); }
    else if (cp < 0x10000) {
      b.push_back((char)(0xE0 | (cp >> 12))); b.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      b.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      b.push_back((char)(0xF0 | (cp >> 18))); b.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      b.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); b.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  // a JSON string, interned; false on error
  bool string(uint32_t* sid) {
    if (p_ >= e_ || *p_ != '"') return false;
    ++p_;
    const char* s = p_;
    // 16 bytes at a time to the first quote, backslash or control byte
    const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), c1f = _mm_set1_epi8(0x1f);
    while (e_ - p_ >= 16) {
      const __m128i v = _mm_loadu_si128((const __m128i*)p_);
      const __m128i hit = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, q), _mm_cmpeq_epi8(v, bs)),
                                       _mm_cmpeq_epi8(_mm_max_epu8(v, c1f), c1f));
      const unsigned m = (unsigned)_mm_movemask_epi8(hit);
      if (m) { p_ += __builtin_ctz(m); goto scanned; }
      p_ += 16;
    }
    while (p_ < e_ && *p_ != '"' && *p_ != '\\' && (unsigned char)*p_ >= 0x20) ++p_;
  scanned:
    if (p_ < e_ && *p_ == '"') {  // no escapes: intern straight from the input
      *sid = st_.intern(s, (size_t)(p_ - s));
      ++p_;
      return true;
    }
    std::string& b = st_.scratch_;
    b.assign(s, (size_t)(p_ - s));
    while (p_ < e_ && *p_ != '"') {
      unsigned char c = (unsigned char)*p_;
      if (c < 0x20) return false;
      if (c == '\\') {
        ++p_;
        if (p_ >= e_) return false;
        char esc = *p_++;
        switch (esc) {
          case '"': b.push_back('"'); break;
          case '\\': b.push_back('\\'); break;
          case '/': b.push_back('/'); break;
          case 'b': b.push_back('\b'); break;
          case 'f': b.push_back('\f'); break;
          case 'n': b.push_back('\n'); break;
          case 'r': b.push_back('\r'); break;
          case 't': b.push_back('\t'); break;
          case 'u': {
            if (e_ - p_ < 4) return false;
            uint32_t cp = 0;
            for (int i = 0; i < 4; ++i) { int h = hexv(p_[i]); if (h < 0) return false; cp = cp * 16 + h; }
            p_ += 4;
            if (cp >= 0xD800 && cp < 0xDC00) {
              if (e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
                uint32_t lo = 0;
                bool ok = true;
                for (int i = 0; i < 4; ++i) { int h = hexv(p_[2 + i]); if (h < 0) { ok = false; break; } lo = lo * 16 + h; }
                if (ok && lo >= 0xDC00 && lo < 0xE000) { p_ += 6; cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00); }
                else cp = 0xFFFD;
              } else cp = 0xFFFD;
            } else if (cp >= 0xDC00 && cp < 0xE000) cp = 0xFFFD;
            put_utf8(b, cp);
            break;
          }
          default: return false;
        }
      } else {
        b.push_back((char)c);
        ++p_;
      }
    }
    if (p_ >= e_) return false;
    ++p_;
    *sid = st_.intern(b.data(), b.size());
    return true;
  }
  // moves pend_[base..] into a fresh contiguous arena block
  uint32_t close_block(size_t base, uint32_t* n, uint8_t* flags) {
    std::vector<Node>& pd = st_.pend_;
    size_t cnt = pd.size() - base;
    if (cnt > 0xffff) { *flags |= 1; cnt = 0xffff; }
    uint32_t first = (uint32_t)st_.nodes_.size();
    st_.nodes_.resize(st_.nodes_.size() + cnt);
    if (cnt) memcpy(st_.nodes_.data() + first, pd.data() + base, cnt * sizeof(Node));
    pd.resize(base);
    *n = (uint32_t)cnt;
    return first;
  }
  // encoding/json into map[string]interface{}: the last value of a key wins
  // (the kept members stay in source order, as JsonReader::dedupe keeps them)
  void dedupe(size_t base) {
    std::vector<Node>& pd = st_.pend_;
    size_t n = pd.size() - base;
    if (n < 2) return;
    bool dup = false;
    for (size_t a = base; a < pd.size() && !dup; ++a)
      for (size_t b = a + 1; b < pd.size(); ++b)
        if (pd[a].key == pd[b].key) { dup = true; break; }
    if (!dup) return;
    size_t w = base;
    for (size_t a = base; a < pd.size(); ++a) {
      bool later = false;
      for (size_t b = a + 1; b < pd.size() && !later; ++b) later = pd[a].key == pd[b].key;
      if (!later) pd[w++] = pd[a];
    }
    pd.resize(w);
  }
  bool value(Node* out, int depth) {
    if (depth > 512) return fail("nesting too deep");
    if (p_ >= e_) return fail("unexpected end");
    *out = Node{};
    char c = *p_;
    if (c == '{') {
      ++p_;
      out->type = NT_OBJ;
      ws();
      size_t base = st_.pend_.size();
      if (p_ < e_ && *p_ == '}') { ++p_; return true; }
      while (true) {
        ws();
        uint32_t key;
        if (!string(&key)) return fail("bad object key");
        ws();
        if (p_ >= e_ || *p_ != ':') return fail("expected ':'");
        ++p_;
        ws();
        Node v;
        if (!value(&v, depth + 1)) return false;
        v.key = key;
        st_.pend_.push_back(v);
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == '}') { ++p_; break; }
        return fail("expected ',' or '}'");
      }
      dedupe(base);
      uint32_t n;
      out->first = close_block(base, &n, &out->flags);
      out->n = (uint16_t)n;
      return true;
    }
    if (c == '[') {
      ++p_;
      out->type = NT_ARR;
      ws();
      size_t base = st_.pend_.size();
      if (p_ < e_ && *p_ == ']') { ++p_; return true; }
      uint32_t i = 0;
      while (true) {
        ws();
        Node v;
        if (!value(&v, depth + 1)) return false;
        v.key = i++;
        st_.pend_.push_back(v);
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == ']') { ++p_; break; }
        return fail("expected ',' or ']'");
      }
      uint32_t n;
      out->first = close_block(base, &n, &out->flags);
      out->n = (uint16_t)n;
      return true;
    }
    if (c == '"') {
      out->type = NT_STR;
      if (!string(&out->val)) return fail("bad string");
      return true;
    }
    if (c == 't') { if (e_ - p_ >= 4 && memcmp(p_, "true", 4) == 0) { p_ += 4; out->type = NT_TRUE; return true; } return fail("bad literal"); }
    if (c == 'f') { if (e_ - p_ >= 5 && memcmp(p_, "false", 5) == 0) { p_ += 5; out->type = NT_FALSE; return true; } return fail("bad literal"); }
    if (c == 'n') { if (e_ - p_ >= 4 && memcmp(p_, "null", 4) == 0) { p_ += 4; out->type = NT_NULL; return true; } return fail("bad literal"); }
    if (c == '-' || (c >= '0' && c <= '9')) {
      const char* s = p_;
      if (*p_ == '-') ++p_;
      if (p_ >= e_) return fail("bad number");
      if (*p_ == '0') ++p_;
      else if (*p_ >= '1' && *p_ <= '9') { while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_; }
      else return fail("bad number");
      if (p_ < e_ && *p_ == '.') {
        ++p_;
        if (p_ >= e_ || !(*p_ >= '0' && *p_ <= '9')) return fail("bad number");
        while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
      }
      if (p_ < e_ && (*p_ == 'e' || *p_ == 'E')) {
        ++p_;
        if (p_ < e_ && (*p_ == '+' || *p_ == '-')) ++p_;
        if (p_ >= e_ || !(*p_ >= '0' && *p_ <= '9')) return fail("bad number");
        while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
      }
      out->type = NT_NUM;
      out->val = st_.number(s, (size_t)(p_ - s));
      return true;
    }
    return fail("unexpected character");
  }
};

bool Store::parse_doc(const char* p, size_t n, Node* root, std::string* err) {
  if (short_.empty()) short_.assign(kShortCache, ShortEnt{{0, 0, 0, 0}, ~0u, 0});
  DocParser d(*this, p, n, err);
  return d.run(root);
}

}  // namespace gk

namespace gk {

// Parallel merge of thread-local stores' strings (flatten.cc phase 2).
//  A (per part): strings already in this store map to their ids; the rest
//    become candidates, bucketed into 256 shards by the hash's top byte.
//  B (per shard): candidates are de-duplicated across parts (hash, then bytes).
//  C: shard id / byte ranges by prefix sum; the tables are resized once.
//  D (per shard): entries, bytes and flags are written in place, and each new
//    string is inserted into the open-addressing table with a CAS on its slot
//    (new strings are distinct, so a taken slot only means "probe on").
//  E (per part): candidates' map entries point at their shard's ids.
// Ids are assigned shard by shard, so they differ from serial interning's;
// nothing depends on id order (the engine compares strings by id for equality
// and by bytes for order).
void Store::intern_parts(const std::vector<const Store*>& src, uint32_t first,
                         std::vector<std::vector<uint32_t>>& maps, int threads) {
  const size_t P = src.size();
  constexpr uint32_t S = 256;
  struct Cand { uint64_t hv; uint32_t lid, gidx; };
  auto t0 = std::chrono::steady_clock::now();
  maps.assign(P, {});
  {
    // a micro-batch's few thousand strings: interned one by one (the sharded
    // phases' fixed cost -- 256 shards x parts of candidate lists -- is larger)
    size_t extra = 0;
    for (const Store* ls : src) extra += ls->nstrings() > first ? ls->nstrings() - first : 0;
    if (extra < 8192) {
      // the parts look their strings up in parallel (the table is only read;
      // the caller holds the store's lock), then the misses are interned in
      // part order -- a webhook micro-batch's strings are mostly known
      auto look = [&](size_t p) {
        const Store& ls = *src[p];
        auto& m = maps[p];
        m.resize(ls.nstrings());
        for (uint32_t k = 0; k < first && k < ls.nstrings(); ++k) m[k] = k;
        for (uint32_t k = first; k < ls.nstrings(); ++k) {
          std::string_view v = ls.str(k);
          m[k] = find(v.data(), v.size());
        }
      };
      if (threads > 1 && P > 1) parallel_run((int)P, [&](int p) { look((size_t)p); });
      else for (size_t p = 0; p < P; ++p) look(p);
      for (size_t p = 0; p < P; ++p) {
        const Store& ls = *src[p];
        auto& m = maps[p];
        for (uint32_t k = first; k < ls.nstrings(); ++k)
          if (m[k] == NO_ID) m[k] = intern(ls.str(k));
      }
      return;
    }
  }
  std::vector<std::vector<std::vector<Cand>>> cand(P, std::vector<std::vector<Cand>>(S));
  auto pfor = [&](size_t n, const std::function<void(size_t)>& f) {
    std::atomic<size_t> next{0};
    auto work = [&] { for (size_t i; (i = next.fetch_add(1)) < n;) f(i); };
    parallel_run(std::max(1, threads), [&](int) { work(); });
  };
  // A
  pfor(P, [&](size_t p) {
    const Store& ls = *src[p];
    auto& m = maps[p];
    m.resize(ls.nstrings());
    for (uint32_t s = 0; s < first && s < ls.nstrings(); ++s) m[s] = s;
    const size_t mask = table_.size() - 1;
    for (uint32_t s = first; s < ls.nstrings(); ++s) {
      std::string_view v = ls.str(s);
      const uint64_t hv = str_hash(v.data(), v.size()), tag = hv & 0xffffffff00000000ull;
      uint32_t id = NO_ID;
      for (size_t h = hv & mask; uint64_t e = table_[h]; h = (h + 1) & mask) {
        if ((e & 0xffffffff00000000ull) != tag) continue;
        const StrEnt& se = strs_[(uint32_t)e - 1];
        if (se.len == v.size() && memcmp(pool_.data() + se.off, v.data(), v.size()) == 0) { id = (uint32_t)e - 1; break; }
      }
      if (id != NO_ID) m[s] = id;
      else cand[p][hv >> 56].push_back(Cand{hv, s, 0});
    }
  });
  {
    size_t ncand = 0;  // an upper bound of the new strings: room without rehashing later
    for (auto& cp : cand)
      for (auto& v : cp) ncand += v.size();
    reserve_strings(ncand);
  }
  auto tA = std::chrono::steady_clock::now();
  // B
  struct Rep { uint64_t hv; uint32_t part, lid; };
  std::vector<std::vector<Rep>> reps(S);
  std::vector<uint64_t> shard_bytes(S, 0);
  pfor(S, [&](size_t sh) {
    size_t tot = 0;
    for (size_t p = 0; p < P; ++p) tot += cand[p][sh].size();
    if (!tot) return;
    size_t sz = 16;
    while (sz < tot * 2) sz *= 2;
    std::vector<uint32_t> tab(sz, 0);  // rep index + 1
    auto& R = reps[sh];
    R.reserve(tot);
    for (size_t p = 0; p < P; ++p) {
      for (Cand& c : cand[p][sh]) {
        std::string_view v = src[p]->str(c.lid);
        size_t h = (size_t)(c.hv * 0x9e3779b97f4a7c15ull >> 20) & (sz - 1);
        for (;; h = (h + 1) & (sz - 1)) {
          const uint32_t e = tab[h];
          if (!e) {
            tab[h] = (uint32_t)R.size() + 1;
            c.gidx = (uint32_t)R.size();
            R.push_back(Rep{c.hv, (uint32_t)p, c.lid});
            shard_bytes[sh] += v.size();
            break;
          }
          const Rep& r = R[e - 1];
          if (r.hv == c.hv && src[r.part]->str(r.lid) == v) { c.gidx = e - 1; break; }
        }
      }
    }
  });
  auto tB = std::chrono::steady_clock::now();
  // C
  std::vector<uint32_t> base_id(S);
  std::vector<uint64_t> base_off(S);
  uint32_t nid = (uint32_t)strs_.size();
  uint64_t off = pool_.size();
  for (uint32_t sh = 0; sh < S; ++sh) {
    base_id[sh] = nid;
    base_off[sh] = off;
    nid += (uint32_t)reps[sh].size();
    off += shard_bytes[sh];
  }
  if (off > 0xffffffffull) throw std::runtime_error("string pool exceeds 4 GiB");
  while ((size_t)nid * 2 > table_.size()) grow();  // (reserve_strings above already made room)
  strs_.resize(nid);
  sflags_.resize(nid);
  pool_.resize(off);
  auto tC = std::chrono::steady_clock::now();
  // D
  const size_t mask = table_.size() - 1;
  pfor(S, [&](size_t sh) {
    uint64_t o = base_off[sh];
    char* pool = &pool_[0];
    for (size_t k = 0; k < reps[sh].size(); ++k) {
      const Rep& r = reps[sh][k];
      std::string_view v = src[r.part]->str(r.lid);
      const uint32_t id = base_id[sh] + (uint32_t)k;
      if (!v.empty()) memcpy(pool + o, v.data(), v.size());
      strs_[id] = StrEnt{(uint32_t)o, (uint32_t)v.size()};
      sflags_[id] = str_flags_of(v.data(), v.size());
      o += v.size();
      const uint64_t slot = slot_of(r.hv, id);
      for (size_t h = r.hv & mask;; h = (h + 1) & mask) {
        uint64_t zero = 0;
        if (__atomic_compare_exchange_n(&table_[h], &zero, slot, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) break;
      }
    }
  });
  auto tD = std::chrono::steady_clock::now();
  // E
  pfor(P, [&](size_t p) {
    auto& m = maps[p];
    for (uint32_t sh = 0; sh < S; ++sh)
      for (const Cand& c : cand[p][sh]) m[c.lid] = base_id[sh] + c.gidx;
  });
  if (getenv("GKGPU_FLATTEN_TRACE")) {
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    fprintf(stderr, "intern_parts: A %.1f B %.1f C %.1f D %.1f E %.1f ms\n", ms(t0, tA), ms(tA, tB), ms(tB, tC), ms(tC, tD),
            ms(tD, std::chrono::steady_clock::now()));
  }
}

}  // namespace gk
