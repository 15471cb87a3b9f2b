// Minimal, allocation-light JSON reader producing a temporary DOM.
// Strings are unescaped into a scratch buffer; numbers keep their source text
// (OPA keeps json.Number text: util/json.go UseNumber, ast/term.go:53-110).
// Object members keep source order.
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

namespace gk {

struct JNode {
  uint8_t type;        // NodeType
  uint32_t s_off = 0;  // string value / number text (into JDoc::buf)
  uint32_t s_len = 0;
  uint32_t k_off = 0;  // member key (into JDoc::buf)
  uint32_t k_len = 0;
  int32_t first = -1;  // first child
  int32_t next = -1;   // next sibling
  uint32_t n = 0;      // child count
};

struct JDoc {
  std::vector<JNode> nodes;
  std::string buf;
  std::string err;

  const char* str(const JNode& n) const { return buf.data() + n.s_off; }
  const char* key(const JNode& n) const { return buf.data() + n.k_off; }
  // child of object `o` with key
  int get(int o, const char* k, size_t klen) const {
    if (o < 0 || nodes[o].type != 7) return -1;
    for (int c = nodes[o].first; c >= 0; c = nodes[c].next)
      if (nodes[c].k_len == klen && memcmp(buf.data() + nodes[c].k_off, k, klen) == 0) return c;
    return -1;
  }
  int get(int o, const char* k) const { return get(o, k, strlen(k)); }
  bool is_str(int n, const char* s) const {
    if (n < 0 || nodes[n].type != 5) return false;
    size_t l = strlen(s);
    return nodes[n].s_len == l && memcmp(buf.data() + nodes[n].s_off, s, l) == 0;
  }
  std::string sval(int n) const { return std::string(buf.data() + nodes[n].s_off, nodes[n].s_len); }
};

class JsonReader {
 public:
  JsonReader(const char* p, size_t n, JDoc* d) : p_(p), e_(p + n), d_(d) {}

  // returns root index or -1 (d->err set)
  int parse() {
    d_->nodes.clear();
    d_->buf.clear();
    d_->err.clear();
    ws();
    int r = value(0);
    if (r < 0) return -1;
    ws();
    if (p_ != e_) return fail("trailing data");
    return r;
  }

 private:
  const char* p_;
  const char* e_;
  JDoc* d_;

  int fail(const char* m) {
    if (d_->err.empty()) d_->err = m;
    return -1;
  }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\t' || *p_ == '\r')) ++p_;
  }
  int newnode(uint8_t t) {
    d_->nodes.push_back(JNode());
    d_->nodes.back().type = t;
    return (int)d_->nodes.size() - 1;
  }
  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  void put_utf8(uint32_t cp) {
    std::string& b = d_->buf;
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
  // parse a JSON string into d_->buf; returns false on error
  bool string(uint32_t* off, uint32_t* len) {
    if (p_ >= e_ || *p_ != '"') return false;
    ++p_;
    *off = (uint32_t)d_->buf.size();
    const char* s = p_;
    // fast path: no escapes
    while (p_ < e_ && *p_ != '"' && *p_ != '\\' && (unsigned char)*p_ >= 0x20) ++p_;
    d_->buf.append(s, p_ - s);
    while (p_ < e_ && *p_ != '"') {
      unsigned char c = (unsigned char)*p_;
      if (c < 0x20) return false;
      if (c == '\\') {
        ++p_;
        if (p_ >= e_) return false;
        char esc = *p_++;
        switch (esc) {
          case '"': d_->buf.push_back('"'); break;
          case '\\': d_->buf.push_back('\\'); break;
          case '/': d_->buf.push_back('/'); break;
          case 'b': d_->buf.push_back('\b'); break;
          case 'f': d_->buf.push_back('\f'); break;
          case 'n': d_->buf.push_back('\n'); break;
          case 'r': d_->buf.push_back('\r'); break;
          case 't': d_->buf.push_back('\t'); break;
          case 'u': {
            if (e_ - p_ < 4) return false;
            uint32_t cp = 0;
            for (int i = 0; i < 4; ++i) { int h = hexv(p_[i]); if (h < 0) return false; cp = cp * 16 + h; }
            p_ += 4;
            if (cp >= 0xD800 && cp < 0xDC00) {
              // surrogate pair
              if (e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
                uint32_t lo = 0; bool ok = true;
                for (int i = 0; i < 4; ++i) { int h = hexv(p_[2 + i]); if (h < 0) { ok = false; break; } lo = lo * 16 + h; }
                if (ok && lo >= 0xDC00 && lo < 0xE000) { p_ += 6; cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00); }
                else cp = 0xFFFD;
              } else cp = 0xFFFD;
            } else if (cp >= 0xDC00 && cp < 0xE000) cp = 0xFFFD;
            put_utf8(cp);
            break;
          }
          default: return false;
        }
      } else {
        d_->buf.push_back((char)c);
        ++p_;
      }
    }
    if (p_ >= e_) return false;
    ++p_;
    *len = (uint32_t)d_->buf.size() - *off;
    return true;
  }
  int value(int depth) {
    if (depth > 512) return fail("nesting too deep");
    if (p_ >= e_) return fail("unexpected end");
    char c = *p_;
    if (c == '{') {
      ++p_;
      int o = newnode(7);
      ws();
      int last = -1;
      uint32_t cnt = 0;
      if (p_ < e_ && *p_ == '}') { ++p_; return o; }
      while (true) {
        ws();
        uint32_t ko, kl;
        if (!string(&ko, &kl)) return fail("bad object key");
        ws();
        if (p_ >= e_ || *p_ != ':') return fail("expected ':'");
        ++p_;
        ws();
        int v = value(depth + 1);
        if (v < 0) return -1;
        d_->nodes[v].k_off = ko;
        d_->nodes[v].k_len = kl;
        if (last < 0) d_->nodes[o].first = v; else d_->nodes[last].next = v;
        last = v;
        ++cnt;
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == '}') { ++p_; break; }
        return fail("expected ',' or '}'");
      }
      // duplicate keys: encoding/json keeps the last value
      d_->nodes[o].n = cnt;
      dedupe(o);
      return o;
    }
    if (c == '[') {
      ++p_;
      int a = newnode(6);
      ws();
      int last = -1;
      uint32_t cnt = 0;
      if (p_ < e_ && *p_ == ']') { ++p_; return a; }
      while (true) {
        ws();
        int v = value(depth + 1);
        if (v < 0) return -1;
        if (last < 0) d_->nodes[a].first = v; else d_->nodes[last].next = v;
        last = v;
        ++cnt;
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == ']') { ++p_; break; }
        return fail("expected ',' or ']'");
      }
      d_->nodes[a].n = cnt;
      return a;
    }
    if (c == '"') {
      int s = newnode(5);
      uint32_t off, len;
      if (!string(&off, &len)) return fail("bad string");
      d_->nodes[s].s_off = off;
      d_->nodes[s].s_len = len;
      return s;
    }
    if (c == 't') { if (e_ - p_ >= 4 && memcmp(p_, "true", 4) == 0) { p_ += 4; return newnode(3); } return fail("bad literal"); }
    if (c == 'f') { if (e_ - p_ >= 5 && memcmp(p_, "false", 5) == 0) { p_ += 5; return newnode(2); } return fail("bad literal"); }
    if (c == 'n') { if (e_ - p_ >= 4 && memcmp(p_, "null", 4) == 0) { p_ += 4; return newnode(1); } return fail("bad literal"); }
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
      int nn = newnode(4);
      d_->nodes[nn].s_off = (uint32_t)d_->buf.size();
      d_->nodes[nn].s_len = (uint32_t)(p_ - s);
      d_->buf.append(s, p_ - s);
      return nn;
    }
    return fail("unexpected character");
  }
  void dedupe(int o) {
    // encoding/json into map[string]interface{}: a later duplicate key replaces
    // the earlier value (and Go maps have no order anyway)
    JNode* N = d_->nodes.data();
    const char* B = d_->buf.data();
    if (N[o].n < 2) return;
    auto same = [&](int a, int b) { return N[a].k_len == N[b].k_len && memcmp(B + N[a].k_off, B + N[b].k_off, N[a].k_len) == 0; };
    bool dup = false;
    for (int a = N[o].first; a >= 0 && !dup; a = N[a].next)
      for (int b = N[a].next; b >= 0; b = N[b].next)
        if (same(a, b)) { dup = true; break; }
    if (!dup) return;
    // keep each key's last occurrence, in source order
    int head = -1, tail = -1;
    uint32_t cnt = 0;
    for (int a = N[o].first; a >= 0;) {
      int next = N[a].next;
      bool later = false;
      for (int b = next; b >= 0 && !later; b = N[b].next) later = same(a, b);
      if (!later) {
        if (tail < 0) head = a; else N[tail].next = a;
        tail = a;
        ++cnt;
      }
      a = next;
    }
    N[tail].next = -1;
    N[o].first = head;
    N[o].n = cnt;
  }
};

}  // namespace gk
