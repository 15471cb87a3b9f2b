#include <algorithm>
// Template JIT (see jit.h).
#include "jit.h"

#include "regex.h"

#include <hip/hiprtc.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <sstream>
#include <sys/stat.h>
#include <unistd.h>

// device runtime sources, embedded at build time (Makefile: build/rtsrc.cc)
extern const char gk_rt_common_h[];
extern const char gk_rt_devrt_h[];

namespace gk {
namespace {

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) { h ^= c; h *= 1099511628211ull; }
  return h;
}

// -amdgpu-prealloc-sgpr-spill-vgprs: the VGPRs whose lanes hold spilled SGPRs
// are allocated up front and reserved for the whole function.  Without it this
// toolchain (ROCm 7.2) miscompiles large template kernels: round 5 saw lost
// rows and a faulting join kernel, round 6 a GPU memory fault in the unfused
// K8sContainerLimits kernel (tests/test_gpu_parity.py
// test_emission_order_is_topdown_order[jit-0], profiles/r06/r06h_fault.txt)
// after the option was turned off because round 5's reproducers ran clean.  In
// that kernel's ISA without the option the predicate's spill-lane VGPRs
// (v124-v126) are shuffled through AGPRs that also serve as ordinary spill
// slots (1,872 other writes of v125); with it they are written only by
// v_writelane and the epilogue reload (tools/isa_spill_lanes.py,
// profiles/r06/r06h_isa_spill_lanes.txt).  The option measured neutral
// (r06e_lanecap_prealloc_ab.txt).  GKGPU_JIT_PREALLOC=0 (diagnostic) drops it.
const char* kOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-w", "-mllvm", "-amdgpu-prealloc-sgpr-spill-vgprs"};
constexpr int kNOpts = 6;
std::vector<const char*> base_opts() {
  const char* e = getenv("GKGPU_JIT_PREALLOC");
  const bool pre = !(e && e[0] == '0');
  return std::vector<const char*>(kOpts, kOpts + (pre ? kNOpts : kNOpts - 2));
}

std::string hex16(uint64_t v) {
  char b[17];
  snprintf(b, sizeof b, "%016llx", (unsigned long long)v);
  return b;
}

// Registers an instruction reads as values that must be plain strings (a
// deferred sprintf is forced into the lane buffer first).  Not listed: MOV and
// YIELD (copy the deferred value; op_yield forces before a conflict check),
// EMIT's message (formatted into the output at flush), jumps (a V_FMT is
// neither undefined nor a boolean), MEMO_PUT (never caches a V_FMT) and
// MEMO_GET: a V_FMT argument is no memo key (gm_key), so the call is
// evaluated with the deferred value -- get_message(parameters, def_msg) in
// demo/agilebank's k8srequiredlabels returns def_msg still unprinted, and a
// constraint with a `message` parameter never prints it at all.
std::vector<uint32_t> fmt_reads(const Ins& in) {
  std::vector<uint32_t> rs;
  auto add = [&](uint32_t r) { if (r != 0xffff) rs.push_back(r); };
  switch (in.op) {
    case OP_GET: case OP_CMP: case OP_ARITH: add(in.b); add(in.c); break;
    case OP_GETK: case OP_ITER_INIT: case OP_SPRINTF: case OP_LEN_EQ: case OP_TABLE: case OP_EMIT: case OP_JPROBE:
      add(in.b);
      break;
    case OP_LIST_ADD: add(in.a); add(in.b); break;
    case OP_OBJ_PUT: add(in.a); add(in.b); add(in.c); break;
    case OP_CALL: for (uint32_t i = 0; i < in.c; ++i) add(in.b + i); break;
    default: break;
  }
  return rs;
}

bool lazy_fmt(const Ins& in) { return in.op == OP_SPRINTF && in.x < (1u << 24); }

// Which registers may hold a deferred sprintf (V_FMT) on entry to each
// instruction: forward data flow over the template's control-flow graph.  A
// register becomes "maybe V_FMT" where a lazy sprintf (or a copy of such a
// value) writes it, and stops being one at any other write or where it is forced.
struct FmtFlow {
  uint32_t nw = 1;
  std::vector<std::vector<uint64_t>> in;
  std::vector<char> reached;
  bool has(uint32_t k, uint32_t r) const { return r < 64 * nw && ((in[k][r >> 6] >> (r & 63)) & 1); }
};

FmtFlow fmt_flow(const Program& p, const CodeBank& bank) {
  const uint32_t b0 = p.code_off, n = p.code_len;
  FmtFlow F;
  F.nw = (p.nregs + 64) / 64;
  F.in.assign(n, std::vector<uint64_t>(F.nw, 0));
  F.reached.assign(n, 0);
  auto has = [&](const std::vector<uint64_t>& s, uint32_t r) { return r < 64 * F.nw && ((s[r >> 6] >> (r & 63)) & 1); };
  auto put = [&](std::vector<uint64_t>& s, uint32_t r, bool v) {
    if (r >= 64 * F.nw) return;
    if (v) s[r >> 6] |= 1ull << (r & 63);
    else s[r >> 6] &= ~(1ull << (r & 63));
  };
  std::vector<uint32_t> work;
  auto flow = [&](uint32_t to, const std::vector<uint64_t>& s) {
    if (to < b0 || to >= b0 + n) return;
    uint32_t k = to - b0;
    bool ch = !F.reached[k];
    F.reached[k] = 1;
    for (uint32_t w = 0; w < F.nw; ++w) {
      uint64_t nv = F.in[k][w] | s[w];
      if (nv != F.in[k][w]) { F.in[k][w] = nv; ch = true; }
    }
    if (ch) work.push_back(k);
  };
  if (n) { F.reached[0] = 1; work.push_back(0); }
  while (!work.empty()) {
    uint32_t k = work.back();
    work.pop_back();
    const Ins& in = bank.code[b0 + k];
    std::vector<uint64_t> s = F.in[k];
    for (uint32_t r : fmt_reads(in)) put(s, r, false);  // forced here
    uint32_t next = b0 + k + 1;
    switch (in.op) {
      case OP_END: case OP_FAIL_FALLBACK: continue;
      case OP_JMP: flow(in.x, s); continue;
      case OP_JUNDEF: case OP_JFALSE: case OP_JTRUE: flow(in.x, s); flow(next, s); continue;
      case OP_ITER_NEXT:
        flow(in.x, s);
        if (in.b != 0xffff) put(s, in.b, false);
        if (in.c != 0xffff) put(s, in.c, false);
        flow(next, s);
        continue;
      case OP_JPROBE:
        put(s, in.a, false);
        put(s, in.a + 1u, false);
        flow(in.x, s);
        flow(next, s);
        continue;
      case OP_JNEXT:
        flow(in.x, s);
        put(s, in.b, false);
        flow(next, s);
        continue;
      case OP_MEMO_GET: {
        std::vector<uint64_t> t = s;
        put(t, in.a, false);
        flow(in.x, t);
        flow(next, s);
        continue;
      }
      case OP_MOV: put(s, in.a, has(s, in.b)); break;
      case OP_YIELD: if (has(s, in.b)) put(s, in.a, true); break;
      case OP_ITER_INIT: put(s, in.a, false); put(s, in.a + 1u, false); break;
      case OP_EMIT: case OP_MEMO_PUT: case OP_ORD: break;
      default: put(s, in.a, lazy_fmt(in)); break;
    }
    flow(next, s);
  }
  return F;
}

// Available lookups: which registers already hold R[base][K[x]] on entry to
// each instruction, on every path (forward must-analysis over the template's
// control-flow graph).  Rego values are immutable and rule bodies have no side
// effects, so a lookup whose base and result registers are unchanged since
// can be replaced by a copy.  This reaches across inlined function calls:
// K8sContainerLimits' missing(container.resources.limits, "cpu") reads
// limits["cpu"], which the group prologue already looked up (compiler.cc
// group_prologue).  A fact dies when its base or result register is written
// (or forced from a deferred sprintf), and all facts die at OP_ITER_NEXT, where
// the lane heap of the previous iteration is reclaimed.
struct LookFlow {
  // kidx: a constant's index, or DYN | key register (a lookup with a computed
  // key, e.g. RequiredProbes' ctr[probe]); res: the register holding the
  // result, or NOREG when it is in the shadow local of the lookup at pc spc
  static constexpr uint32_t DYN = 0x80000000u;
  struct Fact { uint16_t base; uint32_t kidx; uint16_t res; uint32_t spc = 0; };
  struct State {
    bool top = true;                     // not reached yet (identity of the meet)
    std::vector<Fact> facts;             // sorted by (base, kidx)
    std::map<uint16_t, uint32_t> konst;  // register -> constant index (OP_LOADK)
  };
  std::vector<State> in;
  // register holding R[base][K[kidx]] on entry to instruction k, or -1
  int find(uint32_t k, uint16_t base, uint32_t kidx) const {
    if (k >= in.size() || in[k].top) return -1;
    for (const Fact& f : in[k].facts) if (f.base == base && f.kidx == kidx) return f.res;
    return -1;
  }
  // the pc whose shadow local holds R[base][R[key]] on entry to k, or -1
  int find_dyn(uint32_t k, uint16_t base, uint16_t key) const {
    if (k >= in.size() || in[k].top) return -1;
    for (const Fact& f : in[k].facts)
      if (f.base == base && f.kidx == (DYN | key) && f.res == 0xffff) return (int)f.spc;
    return -1;
  }
  int konst(uint32_t k, uint16_t r) const {
    if (k >= in.size() || in[k].top) return -1;
    auto it = in[k].konst.find(r);
    return it == in[k].konst.end() ? -1 : (int)it->second;
  }
};

// Emissions whose message is a deferred sprintf of an argument list built
// right before it (forward must-analysis): `L := [x0, .., xn-1]` (LIST_NEW of
// an array, n LIST_ADDs), `F := sprintf(fmt, L)` (lazy), then EMIT(F).  On
// entry to each instruction, the registers F known to hold such a value with
// the argument registers still unchanged.  The emission then takes the
// arguments from those registers (devrt.h op_emit_args) instead of reading
// the list back out of the lane heap -- K8sContainerLimits' eight bodies per
// container build their lists past the 16 LDS heap words, so the read-back
// went to the private segment.
void ins_regs(const Ins& in, std::vector<uint32_t>& rd, std::vector<uint32_t>& wr);
void ins_succ(const Ins& in, uint32_t pc, std::vector<uint32_t>& out);
struct EmitFlow {
  struct LFact { uint16_t list; uint16_t n; uint16_t args[FMT_MAXARGS]; uint32_t newpc = 0; uint32_t ys[FMT_MAXARGS] = {}; };
  // mu: on some paths F holds undefined instead (a function's result that
  // one path leaves unset); the emission then checks the tag first
  // site: the sprintf's pc; its argument registers are copied there into
  // shadow locals (es<site>_i), so later reuse of those registers is harmless
  struct FFact {
    uint16_t f, list, n;
    uint16_t args[FMT_MAXARGS];
    bool mu = false;
    uint32_t site = 0;
    uint32_t newpc = 0;              // the list's LIST_NEW
    uint32_t ys[FMT_MAXARGS] = {};   // its LIST_ADDs' y operands
  };
  struct State {
    bool top = true;
    std::vector<LFact> lists;
    std::vector<FFact> fmts;
    std::vector<uint16_t> undef;  // registers known to hold undefined (sorted)
  };
  std::vector<State> in;
  // r holds undefined on entry to instruction k, on every path
  bool undef_at(uint32_t k, uint16_t r) const {
    return k < in.size() && !in[k].top && std::binary_search(in[k].undef.begin(), in[k].undef.end(), r);
  }
  const FFact* find(uint32_t k, uint16_t f) const {
    if (k >= in.size() || in[k].top) return nullptr;
    for (const FFact& x : in[k].fmts) if (x.f == f) return &x;
    return nullptr;
  }
};
static bool emitflow_on() {
  const char* v = getenv("GKGPU_JIT_EMITARGS");  // A/B switch, default on
  return !v || atoi(v) != 0;
}
static bool same_lfact(const EmitFlow::LFact& a, const EmitFlow::LFact& b) {
  if (a.list != b.list || a.n != b.n || a.newpc != b.newpc) return false;
  for (uint16_t i = 0; i < a.n; ++i) if (a.args[i] != b.args[i]) return false;
  return true;
}
static bool same_ffact(const EmitFlow::FFact& a, const EmitFlow::FFact& b) {
  return a.f == b.f && a.site == b.site && a.n == b.n && a.mu == b.mu;
}
EmitFlow emit_flow(const Program& p, const CodeBank& bank, const FmtFlow& F) {
  const uint32_t b0 = p.code_off, n = p.code_len;
  EmitFlow EF;
  EF.in.assign(n, EmitFlow::State{});
  if (!emitflow_on()) return EF;
  using State = EmitFlow::State;
  auto mentions_l = [](const EmitFlow::LFact& x, uint32_t r) {
    if (x.list == r) return true;
    for (uint16_t i = 0; i < x.n; ++i) if (x.args[i] == r) return true;
    return false;
  };
  auto mentions_f = [](const EmitFlow::FFact& x, uint32_t r) { return x.f == r; };
  auto kill = [&](State& s, uint32_t r) {
    if (r == 0xffff) return;
    s.undef.erase(std::remove(s.undef.begin(), s.undef.end(), (uint16_t)r), s.undef.end());
    s.lists.erase(std::remove_if(s.lists.begin(), s.lists.end(), [&](const EmitFlow::LFact& x) { return mentions_l(x, r); }),
                  s.lists.end());
    s.fmts.erase(std::remove_if(s.fmts.begin(), s.fmts.end(), [&](const EmitFlow::FFact& x) { return mentions_f(x, r); }),
                 s.fmts.end());
  };
  std::vector<uint32_t> work;
  auto flow = [&](uint32_t to, const State& s) {
    if (to < b0 || to >= b0 + n) return;
    State& d = EF.in[to - b0];
    if (d.top) { d = s; d.top = false; work.push_back(to - b0); return; }
    std::vector<EmitFlow::LFact> nl;
    for (const auto& x : d.lists)
      for (const auto& y : s.lists) if (same_lfact(x, y)) { nl.push_back(x); break; }
    auto has_undef = [](const State& t, uint16_t r) { return std::binary_search(t.undef.begin(), t.undef.end(), r); };
    auto same_but_mu = [](EmitFlow::FFact a, EmitFlow::FFact b) { a.mu = b.mu = false; return same_ffact(a, b); };
    std::vector<EmitFlow::FFact> nf;
    for (const auto& x : d.fmts) {
      bool kept = false;
      for (const auto& y : s.fmts)
        if (same_but_mu(x, y)) { EmitFlow::FFact z = x; z.mu = x.mu || y.mu; nf.push_back(z); kept = true; break; }
      if (!kept && has_undef(s, x.f)) { EmitFlow::FFact z = x; z.mu = true; nf.push_back(z); }
    }
    for (const auto& y : s.fmts) {
      bool there = false;
      for (const auto& x : d.fmts) there = there || x.f == y.f;
      if (!there && has_undef(d, y.f)) { EmitFlow::FFact z = y; z.mu = true; nf.push_back(z); }
    }
    std::vector<uint16_t> nu;
    std::set_intersection(d.undef.begin(), d.undef.end(), s.undef.begin(), s.undef.end(), std::back_inserter(nu));
    bool fchanged = nf.size() != d.fmts.size();
    for (size_t i = 0; !fchanged && i < nf.size(); ++i) fchanged = !same_ffact(nf[i], d.fmts[i]);
    if (nl.size() != d.lists.size() || fchanged || nu.size() != d.undef.size()) {
      d.lists.swap(nl);
      d.fmts.swap(nf);
      d.undef.swap(nu);
      work.push_back(to - b0);
    }
  };
  if (n) { EF.in[0].top = false; work.push_back(0); }
  std::vector<uint32_t> rd, wr, succ;
  while (!work.empty()) {
    const uint32_t k = work.back();
    work.pop_back();
    const Ins& in = bank.code[b0 + k];
    State s = EF.in[k];
    for (uint32_t r : fmt_reads(in)) if (F.has(k, r)) kill(s, r);  // forced here: the register changes
    switch (in.op) {
      case OP_ITER_NEXT: case OP_JNEXT:
        // the previous iteration's heap is reclaimed: no fact crosses
        s.lists.clear();
        s.fmts.clear();
        ins_regs(in, rd, wr);
        for (uint32_t r : wr) kill(s, r);
        break;
      case OP_LIST_NEW: {
        kill(s, in.a);
        if (in.y == LK_ARR) {
          EmitFlow::LFact lf{};
          lf.list = in.a;
          lf.newpc = b0 + k;
          s.lists.push_back(lf);
        }
        break;
      }
      case OP_LOADK:
        kill(s, in.a);
        if (in.x < bank.consts.size() && bank.consts[in.x] == 0) {  // undefined
          s.undef.insert(std::lower_bound(s.undef.begin(), s.undef.end(), (uint16_t)in.a), (uint16_t)in.a);
        }
        break;
      case OP_LIST_ADD: {
        // the list grows: sprintf values over it no longer describe it
        s.fmts.erase(std::remove_if(s.fmts.begin(), s.fmts.end(),
                                    [&](const EmitFlow::FFact& x) { return x.f == in.a || x.list == in.a; }),
                     s.fmts.end());
        EmitFlow::LFact* lf = nullptr;
        for (auto& x : s.lists) if (x.list == in.a) lf = &x;
        bool ok = lf && in.b != 0xffff && in.b != in.a && lf->n < FMT_MAXARGS;
        if (ok) { lf->ys[lf->n] = in.y; lf->args[lf->n++] = in.b; }
        s.lists.erase(std::remove_if(s.lists.begin(), s.lists.end(),
                                     [&](const EmitFlow::LFact& x) { return (x.list == in.a && !ok) || (x.list != in.a && mentions_l(x, in.a)); }),
                      s.lists.end());
        break;
      }
      case OP_SPRINTF: {
        const EmitFlow::LFact* lf = nullptr;
        for (const auto& x : s.lists) if (x.list == in.b) lf = &x;
        EmitFlow::FFact ff{};
        const bool ok = lazy_fmt(in) && lf && in.a != in.b && in.x + 1 < bank.fmt.size() && lf->n == bank.fmt[in.x + 1];
        if (ok) {
          ff.f = in.a;
          ff.list = in.b;
          ff.n = lf->n;
          ff.site = b0 + k;
          ff.newpc = lf->newpc;
          for (uint16_t i = 0; i < lf->n; ++i) { ff.args[i] = lf->args[i]; ff.ys[i] = lf->ys[i]; }
        }
        kill(s, in.a);
        if (ok) s.fmts.push_back(ff);
        break;
      }
      case OP_MOV: case OP_YIELD: {
        // a copy (a yield assigns, or errs on a conflicting value): the
        // destination describes the same sprintf
        const EmitFlow::FFact* src = nullptr;
        for (const auto& x : s.fmts) if (x.f == in.b) src = &x;
        EmitFlow::FFact cp{};
        const bool ok = src && in.a != in.b && in.a != src->list;
        if (ok) cp = *src;
        kill(s, in.a);
        if (ok) {
          cp.f = in.a;
          s.fmts.push_back(cp);
        }
        break;
      }
      default:
        ins_regs(in, rd, wr);
        for (uint32_t r : rd)
          s.lists.erase(std::remove_if(s.lists.begin(), s.lists.end(), [&](const EmitFlow::LFact& x) { return x.list == r; }),
                        s.lists.end());
        for (uint32_t r : wr) kill(s, r);
        break;
    }
    ins_succ(in, b0 + k, succ);
    for (uint32_t t : succ) flow(t, s);
  }
  return EF;
}

// Document-derived registers (must-analysis): on entry to each instruction,
// the registers that hold, on every path, a value read out of the review or
// the parameters -- a document node or a scalar, never a lane-heap value --
// so a lookup on them stays valid when a loop reclaims its heap (look_flow).
FmtFlow doc_flow(const Program& p, const CodeBank& bank) {
  const uint32_t b0 = p.code_off, n = p.code_len;
  FmtFlow F;
  F.nw = (p.nregs + 64) / 64;
  F.in.assign(n, std::vector<uint64_t>(F.nw, ~0ull));  // unreached: TOP
  F.reached.assign(n, 0);
  auto has = [&](const std::vector<uint64_t>& s, uint32_t r) { return r < 64 * F.nw && ((s[r >> 6] >> (r & 63)) & 1); };
  auto put = [&](std::vector<uint64_t>& s, uint32_t r, bool v) {
    if (r >= 64 * F.nw) return;
    if (v) s[r >> 6] |= 1ull << (r & 63);
    else s[r >> 6] &= ~(1ull << (r & 63));
  };
  std::vector<uint32_t> work;
  auto flow = [&](uint32_t to, const std::vector<uint64_t>& s) {
    if (to < b0 || to >= b0 + n) return;
    uint32_t k = to - b0;
    bool ch = !F.reached[k];
    F.reached[k] = 1;
    for (uint32_t w = 0; w < F.nw; ++w) {
      uint64_t nv = F.in[k][w] & s[w];
      if (nv != F.in[k][w]) { F.in[k][w] = nv; ch = true; }
    }
    if (ch) work.push_back(k);
  };
  if (n) {
    F.reached[0] = 1;
    std::fill(F.in[0].begin(), F.in[0].end(), 0ull);  // entry: nothing is known
    work.push_back(0);
  }
  while (!work.empty()) {
    uint32_t k = work.back();
    work.pop_back();
    const Ins& in = bank.code[b0 + k];
    std::vector<uint64_t> s = F.in[k];
    const uint32_t next = b0 + k + 1;
    switch (in.op) {
      case OP_END: case OP_FAIL_FALLBACK: continue;
      case OP_JMP: flow(in.x, s); continue;
      case OP_JUNDEF: case OP_JFALSE: case OP_JTRUE: flow(in.x, s); flow(next, s); continue;
      case OP_ITER_NEXT: {
        flow(in.x, s);
        const bool dv = has(s, in.a);
        if (in.b != 0xffff) put(s, in.b, dv);  // an object's key (interned string) or an array index
        if (in.c != 0xffff) put(s, in.c, dv);
        flow(next, s);
        continue;
      }
      case OP_JPROBE:
        put(s, in.a, false);
        put(s, in.a + 1u, false);
        flow(in.x, s);
        flow(next, s);
        continue;
      case OP_JNEXT:
        flow(in.x, s);
        put(s, in.b, false);
        flow(next, s);
        continue;
      case OP_MEMO_GET: {
        std::vector<uint64_t> t = s;
        put(t, in.a, false);
        flow(in.x, t);
        flow(next, s);
        continue;
      }
      case OP_LOADREV: case OP_LOADPARAM: put(s, in.a, true); break;
      case OP_MOV: case OP_GET: case OP_GETK: put(s, in.a, has(s, in.b)); break;
      case OP_ITER_INIT: put(s, in.a, has(s, in.b)); put(s, in.a + 1u, false); break;
      case OP_EMIT: case OP_MEMO_PUT: case OP_ORD: break;
      default: put(s, in.a, false); break;
    }
    flow(next, s);
  }
  return F;
}

static bool dyn_cse_on() {
  const char* v = getenv("GKGPU_JIT_DYNCSE");  // A/B switch, default on
  return !v || atoi(v) != 0;
}

static bool lookflow_on() {
  const char* v = getenv("GKGPU_JIT_CSE");  // A/B switch, default on
  return !v || atoi(v) != 0;
}

LookFlow look_flow(const Program& p, const CodeBank& bank, const FmtFlow& F, const FmtFlow& DF) {
  const uint32_t b0 = p.code_off, n = p.code_len;
  LookFlow LF;
  LF.in.assign(n, LookFlow::State{});
  if (!lookflow_on()) return LF;
  using State = LookFlow::State;
  auto kill = [](State& s, uint32_t r) {
    if (r == 0xffff) return;
    s.facts.erase(std::remove_if(s.facts.begin(), s.facts.end(),
                                 [&](const LookFlow::Fact& f) {
                                   return f.base == r || f.res == r || f.kidx == (LookFlow::DYN | r);
                                 }),
                  s.facts.end());
    s.konst.erase((uint16_t)r);
  };
  auto keep_docs = [&](State& s, uint32_t k) {
    s.facts.erase(std::remove_if(s.facts.begin(), s.facts.end(),
                                 [&](const LookFlow::Fact& f) { return !(DF.reached[k] && DF.has(k, f.base)); }),
                  s.facts.end());
  };
  auto add = [](State& s, uint16_t base, uint32_t kidx, uint16_t res) {
    if (base == res) return;
    for (auto& f : s.facts)
      if (f.base == base && f.kidx == kidx) { f.res = res; return; }
    s.facts.push_back({base, kidx, res});
    std::sort(s.facts.begin(), s.facts.end(), [](const LookFlow::Fact& x, const LookFlow::Fact& y) {
      return x.base != y.base ? x.base < y.base : x.kidx < y.kidx;
    });
  };
  std::vector<uint32_t> work;
  auto flow = [&](uint32_t to, const State& s) {
    if (to < b0 || to >= b0 + n) return;
    State& d = LF.in[to - b0];
    if (d.top) { d = s; d.top = false; work.push_back(to - b0); return; }
    // meet: facts and constants present (identically) on both sides
    std::vector<LookFlow::Fact> nf;
    for (const auto& f : d.facts)
      for (const auto& g : s.facts)
        if (f.base == g.base && f.kidx == g.kidx && f.res == g.res && f.spc == g.spc) { nf.push_back(f); break; }
    std::map<uint16_t, uint32_t> nk;
    for (const auto& kv : d.konst) {
      auto it = s.konst.find(kv.first);
      if (it != s.konst.end() && it->second == kv.second) nk.insert(kv);
    }
    if (nf.size() != d.facts.size() || nk.size() != d.konst.size()) {
      d.facts.swap(nf);
      d.konst.swap(nk);
      work.push_back(to - b0);
    }
  };
  if (n) { LF.in[0].top = false; work.push_back(0); }
  while (!work.empty()) {
    uint32_t k = work.back();
    work.pop_back();
    const Ins& in = bank.code[b0 + k];
    State s = LF.in[k];
    for (uint32_t r : fmt_reads(in)) if (F.has(k, r)) kill(s, r);  // forced here
    const uint32_t next = b0 + k + 1;
    switch (in.op) {
      case OP_END: case OP_FAIL_FALLBACK: continue;
      case OP_JMP: flow(in.x, s); continue;
      case OP_JUNDEF: case OP_JFALSE: case OP_JTRUE: flow(in.x, s); flow(next, s); continue;
      case OP_ITER_NEXT: {
        // the previous iteration's heap is reclaimed: a fact survives only if
        // its base holds a document (or parameters) value on every path, so
        // that the looked-up value is no heap value either (doc_flow)
        keep_docs(s, k);
        flow(in.x, s);
        kill(s, in.b);
        kill(s, in.c);
        flow(next, s);
        continue;
      }
      case OP_JPROBE:
        kill(s, in.a);
        kill(s, in.a + 1u);
        flow(in.x, s);
        flow(next, s);
        continue;
      case OP_JNEXT:
        // like OP_ITER_NEXT: the previous iteration's heap is reclaimed here
        keep_docs(s, k);
        flow(in.x, s);
        kill(s, in.b);
        flow(next, s);
        continue;
      case OP_MEMO_GET: {
        State t = s;
        kill(t, in.a);
        flow(in.x, t);
        flow(next, s);
        continue;
      }
      case OP_LOADK: kill(s, in.a); s.konst[in.a] = in.x; break;
      case OP_MOV: {
        auto it = s.konst.find(in.b);
        const int kb = it == s.konst.end() ? -1 : (int)it->second;
        kill(s, in.a);
        if (kb >= 0) s.konst[in.a] = (uint32_t)kb;
        break;
      }
      case OP_GETK: kill(s, in.a); add(s, in.b, in.x, in.a); break;
      case OP_GET: {
        auto it = s.konst.find(in.c);
        const int kc = it == s.konst.end() ? -1 : (int)it->second;
        kill(s, in.a);
        if (kc >= 0 && in.a != in.c) add(s, in.b, (uint32_t)kc, in.a);
        else if (kc < 0 && in.a != in.b && in.a != in.c && dyn_cse_on() && DF.reached[k] && DF.has(k, in.b)) {
          // computed key: the result in this site's shadow local
          s.facts.erase(std::remove_if(s.facts.begin(), s.facts.end(),
                                       [&](const LookFlow::Fact& f) {
                                         return f.base == in.b && f.kidx == (LookFlow::DYN | in.c);
                                       }),
                        s.facts.end());
          s.facts.push_back({in.b, LookFlow::DYN | in.c, 0xffff, b0 + k});
          std::sort(s.facts.begin(), s.facts.end(), [](const LookFlow::Fact& x, const LookFlow::Fact& y) {
            return x.base != y.base ? x.base < y.base : x.kidx < y.kidx;
          });
        }
        break;
      }
      case OP_ITER_INIT: kill(s, in.a); kill(s, in.a + 1u); break;
      case OP_EMIT: case OP_MEMO_PUT: case OP_ORD: break;
      default: kill(s, in.a); break;
    }
    flow(next, s);
  }
  return LF;
}

// Parameter-derived registers (devrt.h GK_LDS_PARAMS): which registers may
// hold a node of the constraint's parameters subtree on entry to each
// instruction (forward may-analysis).  Lookups and iterations over such a
// register read the wave's LDS copy of the subtree (vget_p / op_iter_next_p);
// those fall back to the node store for a node outside the staged window, so
// the analysis only picks the cheaper path, it never decides a result.
FmtFlow param_flow(const Program& p, const CodeBank& bank) {
  const uint32_t b0 = p.code_off, n = p.code_len;
  FmtFlow F;
  F.nw = (p.nregs + 64) / 64;
  F.in.assign(n, std::vector<uint64_t>(F.nw, 0));
  F.reached.assign(n, 0);
  auto has = [&](const std::vector<uint64_t>& s, uint32_t r) { return r < 64 * F.nw && ((s[r >> 6] >> (r & 63)) & 1); };
  auto put = [&](std::vector<uint64_t>& s, uint32_t r, bool v) {
    if (r >= 64 * F.nw) return;
    if (v) s[r >> 6] |= 1ull << (r & 63);
    else s[r >> 6] &= ~(1ull << (r & 63));
  };
  std::vector<uint32_t> work;
  auto flow = [&](uint32_t to, const std::vector<uint64_t>& s) {
    if (to < b0 || to >= b0 + n) return;
    uint32_t k = to - b0;
    bool ch = !F.reached[k];
    F.reached[k] = 1;
    for (uint32_t w = 0; w < F.nw; ++w) {
      uint64_t nv = F.in[k][w] | s[w];
      if (nv != F.in[k][w]) { F.in[k][w] = nv; ch = true; }
    }
    if (ch) work.push_back(k);
  };
  if (n) { F.reached[0] = 1; work.push_back(0); }
  while (!work.empty()) {
    uint32_t k = work.back();
    work.pop_back();
    const Ins& in = bank.code[b0 + k];
    std::vector<uint64_t> s = F.in[k];
    const uint32_t next = b0 + k + 1;
    switch (in.op) {
      case OP_END: case OP_FAIL_FALLBACK: continue;
      case OP_JMP: flow(in.x, s); continue;
      case OP_JUNDEF: case OP_JFALSE: case OP_JTRUE: flow(in.x, s); flow(next, s); continue;
      case OP_ITER_NEXT: {
        flow(in.x, s);
        const bool pv = has(s, in.a);
        if (in.b != 0xffff) put(s, in.b, false);
        if (in.c != 0xffff) put(s, in.c, pv);
        flow(next, s);
        continue;
      }
      case OP_JPROBE:
        put(s, in.a, false);
        put(s, in.a + 1u, false);
        flow(in.x, s);
        flow(next, s);
        continue;
      case OP_JNEXT:
        flow(in.x, s);
        put(s, in.b, false);
        flow(next, s);
        continue;
      case OP_MEMO_GET: {
        std::vector<uint64_t> t = s;
        put(t, in.a, false);
        flow(in.x, t);
        flow(next, s);
        continue;
      }
      case OP_LOADPARAM: put(s, in.a, true); break;
      case OP_MOV: case OP_GET: case OP_GETK: put(s, in.a, has(s, in.b)); break;
      case OP_YIELD: if (has(s, in.b)) put(s, in.a, true); break;
      case OP_ITER_INIT: put(s, in.a, has(s, in.b)); put(s, in.a + 1u, false); break;
      case OP_EMIT: case OP_MEMO_PUT: case OP_ORD: break;
      default: put(s, in.a, false); break;
    }
    flow(next, s);
  }
  return F;
}

static bool lds_stage_on() {
  const char* v = getenv("GKGPU_LDS_STAGE");  // A/B switch, default on
  return !v || atoi(v) != 0;
}

// A literal re_match pattern's DFA (regex.cc layout; the semantics of re_run /
// run_regex_dfa) as code: a switch over states with byte ranges as compares,
// so matching loads only the subject's bytes.  "" when too large to inline.
std::string regex_fn(const std::string& fn, const std::vector<uint32_t>& d) {
  uint32_t nst = d[0], start = d[1], sens = d[2];
  const uint32_t* st = d.data() + 3;
  auto target = [&](uint32_t k, uint32_t c) -> uint32_t {
    uint32_t w = st[k * 129 + 1 + (c >> 1)];
    return (c & 1) ? (w >> 16) : (w & 0xffff);
  };
  if (nst > 64) return "";
  std::ostringstream o;
  size_t ranges = 0;
  o << "__device__ GK_HOT int " << fn << "(SView v) {\n  uint32_t s = " << start << "u;\n"
    << "  for (uint32_t i = 0; i < v.n; ++i) {\n    uint32_t c = (uint8_t)v.p[i];\n";
  if (sens) o << "    if (c >= 0x80u) return -2;\n";
  o << "    switch (s) {\n";
  for (uint32_t k = 0; k < nst; ++k) {
    o << "      case " << k << "u:";
    if (st[k * 129] & 1) { o << " return 1;\n"; continue; }
    for (uint32_t c = 0; c < 256;) {
      uint32_t t = target(k, c), e = c;
      while (e + 1 < 256 && target(k, e + 1) == t) ++e;
      if (t < nst) {
        ++ranges;
        if (c == e) o << " if (c == " << c << "u) { s = " << t << "u; break; }";
        else o << " if (c >= " << c << "u && c <= " << e << "u) { s = " << t << "u; break; }";
      }
      c = e + 1;
    }
    o << " return 0;\n";
  }
  o << "      default: return 0;\n    }\n  }\n";
  std::vector<uint32_t> acc;
  for (uint32_t k = 0; k < nst; ++k) if (st[k * 129] & 3) acc.push_back(k);
  if (acc.empty()) {
    o << "  return 0;\n";
  } else {
    o << "  switch (s) {";
    for (uint32_t k : acc) o << " case " << k << "u:";
    o << " return 1; default: return 0; }\n";
  }
  o << "}\n";
  if (ranges > 1024) return "";
  return o.str();
}

// OP_TABLE over string keys only (mem_multiple-style suffix tables) inlined:
// the argument's bytes are compared with each key as immediates (a non-string
// argument equals no key).  "" when the table is not of that shape.
std::string table_inline(const CodeBank& bank, const Store& st, uint32_t off, const std::string& dst,
                         const std::string& arg, const std::function<std::string(uint64_t)>& lit) {
  const uint64_t* T = bank.consts.data() + off;
  uint32_t n = (uint32_t)T[0];
  size_t maxlen = 0;
  std::vector<std::string> keys;
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t kv = T[1 + 2 * i];
    if ((kv >> 60) != V_STR) return "";
    uint64_t sid = kv & 0x0fffffffffffffffull;
    if (sid >= st.nstrings()) return "";
    keys.emplace_back(st.str((uint32_t)sid));
    maxlen = std::max(maxlen, keys.back().size());
  }
  if (n == 0 || n > 64 || maxlen > 8) return "";
  std::ostringstream o;
  o << "{ uint64_t t_ = 0x0000000000000000ull; if (is_strv(" << arg << ")) { SView s_ = sview(L, " << arg << ");";
  for (size_t j = 0; j < maxlen; ++j) o << " uint32_t c" << j << "_ = s_.n > " << j << "u ? (uint8_t)s_.p[" << j << "] : 0u;";
  for (uint32_t i = 0; i < n; ++i) {
    o << (i ? " else if (" : " if (") << "s_.n == " << keys[i].size() << "u";
    for (size_t j = 0; j < keys[i].size(); ++j) o << " && c" << j << "_ == " << (unsigned)(uint8_t)keys[i][j] << "u";
    o << ") t_ = " << lit(T[2 + 2 * i]) << ";";
  }
  o << " } " << dst << " = t_; }";
  return o.str();
}

// Registers an instruction reads and writes (the VM's semantics,
// kernels.hip run_program); MEMO_GET's write is the hit path's.
void ins_regs(const Ins& in, std::vector<uint32_t>& rd, std::vector<uint32_t>& wr) {
  rd.clear();
  wr.clear();
  auto R = [&](uint32_t r) { if (r != 0xffff) rd.push_back(r); };
  auto W = [&](uint32_t r) { if (r != 0xffff) wr.push_back(r); };
  switch (in.op) {
    case OP_JUNDEF: case OP_JFALSE: case OP_JTRUE: case OP_KEYOUT: R(in.a); break;
    case OP_LOADK: case OP_LOADREV: case OP_LOADPARAM: case OP_LIST_NEW: W(in.a); break;
    case OP_MOV: case OP_GETK: case OP_SPRINTF: case OP_TABLE: case OP_LEN_EQ: R(in.b); W(in.a); break;
    case OP_GET: case OP_CMP: case OP_ARITH: R(in.b); R(in.c); W(in.a); break;
    case OP_ITER_INIT: R(in.b); W(in.a); W(in.a + 1u); break;
    case OP_ITER_NEXT: R(in.a); R(in.a + 1u); W(in.a + 1u); W(in.b); W(in.c); break;
    case OP_LIST_ADD: case OP_YIELD: R(in.a); R(in.b); W(in.a); break;
    case OP_OBJ_PUT: R(in.a); R(in.b); R(in.c); W(in.a); break;
    case OP_CALL: for (uint32_t i = 0; i < in.c; ++i) R(in.b + i); W(in.a); break;
    case OP_EMIT: R(in.a); R(in.b); break;
    case OP_MEMO_GET: R(in.b); R(in.c); W(in.a); break;
    case OP_MEMO_PUT: R(in.a); R(in.b); R(in.c); break;
    case OP_JPROBE: R(in.b); W(in.a); W(in.a + 1u); break;
    case OP_JNEXT: R(in.a); R(in.a + 1u); W(in.a + 1u); W(in.b); break;
    case OP_JVAR: R(in.b); R(in.b + 1u); W(in.a); break;
    default: break;
  }
}

// successors of the instruction at pc (absolute), for data flow
void ins_succ(const Ins& in, uint32_t pc, std::vector<uint32_t>& out) {
  out.clear();
  switch (in.op) {
    case OP_END: case OP_FAIL_FALLBACK: return;
    case OP_JMP: out.push_back(in.x); return;
    case OP_JUNDEF: case OP_JFALSE: case OP_JTRUE: case OP_ITER_NEXT: case OP_MEMO_GET: case OP_JPROBE: case OP_JNEXT:
      out.push_back(in.x);
      out.push_back(pc + 1);
      return;
    default: out.push_back(pc + 1); return;
  }
}

bool jump_op(uint16_t op) {
  return op == OP_JMP || op == OP_JUNDEF || op == OP_JFALSE || op == OP_JTRUE || op == OP_ITER_NEXT ||
         op == OP_MEMO_GET || op == OP_JPROBE || op == OP_JNEXT;
}

struct Gen {
  std::string pre;   // helper functions (literal regex DFAs)
  std::string body;  // body of the predicate function
  bool param_reads = false;  // lookups / iterations over parameter nodes (vget_p, op_iter_next_p)
  bool param_regex = false;  // re_match with a computed (parameter) pattern (re_run -> re_run_lds)
  uint32_t param_iter_depth = 0;  // deepest loop level of an iteration over a parameter collection
};

// Body of the predicate function: one statement per bytecode instruction.
// Unlike the VM, the generated code does not test L.fail after every helper
// call (a scratch load per call): the first failure recorded in the lane wins
// either way, helpers return well-formed values (undefined) once it is set,
// and a failed lane's staged tuples are discarded by flush_wave — so running
// on to the end yields the same lane outcome at no cost to passing lanes.
Gen generate(const Program& p, const CodeBank& bank, const Store& st) {
  const uint32_t b0 = p.code_off, b1 = p.code_off + p.code_len;
  std::set<uint32_t> labels, memo, memo2, gslots;
  std::map<uint32_t, int> memo_sites;
  for (uint32_t pc = b0; pc < b1; ++pc) {
    const Ins& in = bank.code[pc];
    switch (in.op) {
      case OP_JMP: case OP_JUNDEF: case OP_JFALSE: case OP_JTRUE: case OP_ITER_NEXT: case OP_MEMO_GET:
      case OP_JPROBE: case OP_JNEXT:
        labels.insert(in.x);
        break;
      default: break;
    }
    if (in.op == OP_MEMO_GET || in.op == OP_MEMO_PUT) memo.insert(in.y);
    if (in.op == OP_MEMO_GET && ++memo_sites[in.y] == 2) memo2.insert(in.y);
    if (in.op == OP_MEMO_PUT && in.x == 1) gslots.insert(in.y);  // pure function: cross-lane memo
  }
  // Register pressure: a memo slot's register entries (key, key, value, flag;
  // two entries for slots with several call sites) stay live across the whole
  // predicate.  Slots of pure functions also have the cross-lane memo (gm_get),
  // which answers them from L2 without the registers: measured on config 2 (1M
  // Pods, tools/gpu_r02h.sh) K8sContainerLimits 6.34 -> 5.02 ms without the
  // register entries, 5.45 ms with one entry per slot.
  std::set<uint32_t> lslots = memo;  // slots with register entries
  for (uint32_t m : gslots) { lslots.erase(m); memo2.erase(m); }
  FmtFlow F = fmt_flow(p, bank);
  FmtFlow DF = doc_flow(p, bank);
  LookFlow LK = look_flow(p, bank, F, DF);
  EmitFlow EFL = emit_flow(p, bank, F);
  // sprintf sites whose arguments a fused emission reads: their shadow locals
  std::map<uint32_t, std::vector<uint16_t>> esites;  // site pc -> argument registers there
  std::map<uint32_t, EmitFlow::FFact> efacts;  // site pc -> its fact (list, LIST_NEW pc, add operands)
  for (uint32_t pc = b0; pc < b1; ++pc) {
    const Ins& in = bank.code[pc];
    if (in.op != OP_EMIT || in.b == in.a) continue;
    if (const EmitFlow::FFact* ff = EFL.find(pc - b0, in.a))
      if (ff->n > 0) { esites[ff->site] = std::vector<uint16_t>(ff->args, ff->args + ff->n); efacts[ff->site] = *ff; }
  }
  // Sites whose list exists only for the emission (GKGPU_JIT_EMITDCE, default
  // on): every read of a value that may be a deferred sprintf is a copy, a
  // definedness test or a fused emission; the list is built in straight-line
  // code right before the sprintf and dead after it.  Then the list is not
  // built at all -- the sprintf value carries its format only -- and the
  // emission's slow path (arguments that are not plain scalars) builds it
  // from the shadow copies (devrt.h op_emit_args_build).
  std::set<uint32_t> dce_sites, dce_pcs;
  // fused emissions whose details register is the one-member object literal
  // built by the two instructions right before the emission: emit pc -> its
  // OBJ_PUT pc (devrt.h op_emit_args_kvd; the LIST_NEW goes into dce_pcs)
  std::map<uint32_t, uint32_t> kv_sites;
  {
    const char* dv = getenv("GKGPU_JIT_EMITDCE");
    bool prog_ok = (!dv || atoi(dv) != 0) && !efacts.empty();
    std::vector<uint32_t> rd, wr;
    for (uint32_t pc = b0; prog_ok && pc < b1; ++pc) {
      const Ins& in = bank.code[pc];
      const uint32_t k = pc - b0;
      if (!F.reached[k]) continue;
      for (uint32_t r : fmt_reads(in)) if (F.has(k, r)) prog_ok = false;
      ins_regs(in, rd, wr);
      for (uint32_t r : rd) {
        if (!F.has(k, r)) continue;
        const bool fused = in.op == OP_EMIT && in.b != in.a && r == in.a && EFL.find(k, in.a) && EFL.find(k, in.a)->n > 0;
        // (a yield only into an output known to be undefined: op_yield forces
        // a V_FMT to compare it with a defined one)
        const bool copy = in.op == OP_MOV || (in.op == OP_YIELD && r == in.b && r != in.a && EFL.undef_at(k, in.a));
        if (!(copy || in.op == OP_JUNDEF || in.op == OP_JFALSE || in.op == OP_JTRUE || fused))
          prog_ok = false;
      }
    }
    // liveness (backward may-analysis) for "the list is dead after the sprintf"
    const uint32_t nw = (p.nregs + 64) / 64;
    std::vector<std::vector<uint64_t>> live(prog_ok ? p.code_len : 0, std::vector<uint64_t>(nw, 0));
    std::vector<uint32_t> sc;
    for (bool changed = prog_ok; changed;) {
      changed = false;
      for (uint32_t k = p.code_len; k-- > 0;) {
        const uint32_t pc = b0 + k;
        std::vector<uint64_t> out(nw, 0);
        ins_succ(bank.code[pc], pc, sc);
        for (uint32_t t : sc)
          if (t >= b0 && t < b1) for (uint32_t w = 0; w < nw; ++w) out[w] |= live[t - b0][w];
        ins_regs(bank.code[pc], rd, wr);
        for (uint32_t r : wr) if (r < 64 * nw) out[r >> 6] &= ~(1ull << (r & 63));
        for (uint32_t r : rd) if (r < 64 * nw) out[r >> 6] |= 1ull << (r & 63);
        if (out != live[k]) { live[k] = out; changed = true; }
      }
    }
    for (const auto& ef : efacts) {
      if (!prog_ok) break;
      const EmitFlow::FFact& ff = ef.second;
      const uint32_t S = ff.site, N = ff.newpc, Lr = ff.list;
      bool ok = N >= b0 && N < S && S + 1 < b1 && Lr < 64 * nw;
      // dead after the sprintf
      if (ok) ok = !((live[S + 1 - b0][Lr >> 6] >> (Lr & 63)) & 1);
      // straight-line: no jump into (N, S], no jump out of [N, S)
      std::vector<uint32_t> adds;
      for (uint32_t pc = N; ok && pc <= S; ++pc) {
        if (pc > N && labels.count(pc)) ok = false;
        const Ins& in = bank.code[pc];
        if (pc < S && jump_op(in.op)) ok = false;
        if (pc > N && pc < S && in.op == OP_LIST_ADD && in.a == Lr) adds.push_back(pc);
        if (pc > N && pc < S && in.op == OP_LIST_NEW && in.a == Lr) ok = false;
        // nothing between the LIST_NEW and the sprintf may read the list but
        // its own LIST_ADDs (a copy of it, or the list added into another
        // container, would hold what the unbuilt list's register held)
        if (pc > N && pc < S && ok) {
          ins_regs(in, rd, wr);
          const bool own_add = in.op == OP_LIST_ADD && in.a == Lr && in.b != Lr;
          for (uint32_t r : rd) if (r == Lr && !own_add) ok = false;
        }
      }
      if (ok && adds.size() != ff.n) ok = false;
      // escape ranges packed 10 bits each (devrt.h esc_unpack), six arguments at most
      for (uint16_t i = 0; ok && i < ff.n; ++i) ok = (ff.ys[i] & 0xffu) < 32 && (ff.ys[i] >> 8) < 32;
      if (ff.n > 6) ok = false;
      if (!ok) continue;
      dce_sites.insert(S);
      dce_pcs.insert(N);
      for (uint32_t a : adds) dce_pcs.insert(a);
    }
    const char* kvv = getenv("GKGPU_JIT_KVDCE");  // A/B switch, default on
    const bool kv_on = !kvv || atoi(kvv) != 0;
    for (uint32_t E = b0 + 2; prog_ok && kv_on && E + 1 < b1; ++E) {
      const Ins& em = bank.code[E];
      if (em.op != OP_EMIT || em.b == 0xffff || em.b == em.a) continue;
      const EmitFlow::FFact* ff = EFL.find(E - b0, em.a);
      if (!ff || ff->n == 0 || ff->mu || ff->n + 2 > 6) continue;
      const Ins& put = bank.code[E - 1];
      const Ins& nw0 = bank.code[E - 2];
      const uint32_t Dr = em.b;
      if (put.op != OP_OBJ_PUT || put.a != Dr || put.b == Dr || put.c == Dr || nw0.op != OP_LIST_NEW || nw0.a != Dr ||
          nw0.y != LK_OBJ || labels.count(E - 1) || labels.count(E) || Dr >= 64 * nw)
        continue;
      if ((live[E + 1 - b0][Dr >> 6] >> (Dr & 63)) & 1) continue;  // the object is read after the emission
      kv_sites[E] = E - 1;
      dce_pcs.insert(E - 2);
    }
  }
  // computed-key lookups whose result a later lookup reuses: their shadow locals
  std::set<uint32_t> shadowed;
  for (uint32_t pc = b0; pc < b1; ++pc) {
    const Ins& in = bank.code[pc];
    if (in.op != OP_GET || LK.konst(pc - b0, in.c) >= 0) continue;
    const int spc = LK.find_dyn(pc - b0, in.b, in.c);
    if (spc >= 0 && (uint32_t)spc != pc) shadowed.insert((uint32_t)spc);
  }
  FmtFlow PF = param_flow(p, bank);
  const bool pstage = lds_stage_on();
  Gen g;
  // literal re_match patterns compiled to code
  std::vector<std::pair<uint64_t, std::string>> relits;  // (pattern value, function)
  {
    std::ostringstream pre;
    std::set<uint32_t> seen;
    for (uint32_t sid : p.regex_literals) {
      if (!seen.insert(sid).second) continue;
      std::vector<uint32_t> d;
      if (compile_regex_dfa(std::string(st.str(sid)), d) != RX_OK) continue;
      std::string fn = "re_lit_" + std::to_string(relits.size());
      std::string code = regex_fn(fn, d);
      if (code.empty()) continue;
      pre << code;
      relits.push_back({((uint64_t)V_STR << 60) | sid, fn});
    }
    g.pre = pre.str();
  }
  std::ostringstream o;
  auto R = [](uint32_t r) { return "r" + std::to_string(r); };
  // no initializers: the compiler writes every register before reading it (the
  // VM kernel relies on the same), and zero-initialising would make all of them
  // live from entry — register pressure, hence occupancy
  o << "  uint64_t ";
  for (uint32_t r = 0; r < p.nregs; ++r) o << (r ? ", " : "") << R(r);
  if (!p.nregs) o << "unused_";
  o << ";\n";
  // The shadow and memo locals below start at 0: they are read only behind
  // their valid flags, but a read of an uninitialised local is undefined
  // behaviour, which the optimiser may exploit across the whole predicate
  const std::string Z = " = 0";
  for (uint32_t pc : shadowed) o << "  uint64_t dk" << pc << Z << ";\n";
  for (const auto& es : esites)
    for (size_t i = 0; i < es.second.size(); ++i) o << "  uint64_t es" << es.first << "_" << i << Z << ";\n";
  // memo slots are locals too: (key0, key1, value, valid)
  for (uint32_t m : lslots) {
    o << "  uint64_t mk0_" << m << " = 0, mk1_" << m << " = 0, mv_" << m << " = 0; bool mok_" << m << " = false;\n";
    if (memo2.count(m))
      o << "  uint64_t mkb0_" << m << " = 0, mkb1_" << m << " = 0, mvb_" << m << " = 0; bool mokb_" << m << " = false;\n";
  }
  // Param-keyed register memo (GKGPU_JIT_PMEMO, default on): a pure call whose
  // arguments are derived from the constraint's parameters (jit.cc
  // param_flow) -- canonify_cpu(input.parameters.cpu) in K8sContainerLimits,
  // evaluated once per container -- keeps its last (arguments, value) in
  // registers at that call site, so only the lane's first call probes the
  // cross-lane memo.  The key is compared, so a varying parameter (an
  // iteration over a parameter list) only misses.
  std::set<uint32_t> psite;            // MEMO_GET pcs with a register entry
  std::map<uint32_t, uint32_t> put_site;  // their MEMO_PUT pc -> MEMO_GET pc
  {
    const char* pm = getenv("GKGPU_JIT_PMEMO");
    if (!pm || atoi(pm) != 0)
      for (uint32_t pc = b0; pc < b1; ++pc) {
        const Ins& in = bank.code[pc];
        const uint32_t k = pc - b0;
        if (in.op != OP_MEMO_GET || !gslots.count(in.y) || lslots.count(in.y) || !PF.reached[k]) continue;
        if (!PF.has(k, in.b) || (in.c != 0xffff && !PF.has(k, in.c))) continue;
        if (in.x < 1 || in.x > b1 || bank.code[in.x - 1].op != OP_MEMO_PUT || bank.code[in.x - 1].y != in.y) continue;
        psite.insert(pc);
        put_site[in.x - 1] = pc;
      }
  }
  const char* UND = "0x0000000000000000ull";
  std::function<std::string(uint64_t)> lit = [](uint64_t v) {
    char kb[40];
    snprintf(kb, sizeof kb, "0x%016llxull", (unsigned long long)v);
    return std::string(kb);
  };
  auto emit = [&](uint32_t pc, std::ostringstream& o, const std::string& RET) {
    const Ins& in = bank.code[pc];
    const uint32_t k = pc - b0;
    if (labels.count(pc)) o << "L" << pc << ":;\n";
    std::string a = R(in.a), b = R(in.b), c = R(in.c), x = "L" + std::to_string(in.x);
    std::string y = std::to_string(in.y) + "u";
    if (F.reached[k])
      for (uint32_t r : fmt_reads(in))
        if (F.has(k, r)) o << "  if (vtag(" << R(r) << ") == V_FMT) " << R(r) << " = force_fmt(L, " << R(r) << ");\n";
    o << "  ";
    switch (in.op) {
      case OP_END: o << RET; break;
      case OP_JMP: o << "goto " << x << ";"; break;
      case OP_JUNDEF: o << "if (vtag(" << a << ") == V_UNDEF) goto " << x << ";"; break;
      case OP_JFALSE: o << "if (" << a << " == " << lit(((uint64_t)V_BOOL << 60) | 0) << ") goto " << x << ";"; break;
      case OP_JTRUE: o << "if (" << a << " == " << lit(((uint64_t)V_BOOL << 60) | 1) << ") goto " << x << ";"; break;
      case OP_LOADK: o << a << " = " << lit(bank.consts[in.x]) << ";"; break;
      case OP_LOADREV: o << a << " = review;"; break;
      case OP_LOADPARAM: o << a << " = params;"; break;
      case OP_MOV: o << a << " = " << b << ";"; break;
      case OP_GET: {
        const int kc = LK.konst(k, in.c);
        const int have = kc >= 0 ? LK.find(k, in.b, (uint32_t)kc) : -1;
        const int dyn = kc < 0 ? LK.find_dyn(k, in.b, in.c) : -1;
        if (have == (int)in.a) o << "/* " << a << " holds " << b << "[" << c << "] */";
        else if (have >= 0) o << a << " = " << R((uint32_t)have) << ";  // = vget(L, " << b << ", " << c << ")";
        else if (dyn >= 0 && (uint32_t)dyn != pc) o << a << " = dk" << dyn << ";  // = vget(L, " << b << ", " << c << ")";
        else if (pstage && PF.has(k, in.b)) { o << a << " = vget_p(L, " << b << ", " << c << ", plo, pn);"; g.param_reads = true; }
        else o << a << " = vget(L, " << b << ", " << c << ");";
        if (shadowed.count(pc)) o << " dk" << pc << " = " << a << ";";
        break;
      }
      case OP_GETK: {
        const int have = LK.find(k, in.b, in.x);
        if (have == (int)in.a) o << "/* " << a << " holds " << b << "[K" << in.x << "] */";
        else if (have >= 0) o << a << " = " << R((uint32_t)have) << ";  // = vget(L, " << b << ", K" << in.x << ")";
        else if (pstage && PF.has(k, in.b)) {
          o << a << " = vget_p(L, " << b << ", " << lit(bank.consts[in.x]) << ", plo, pn);";
          g.param_reads = true;
        } else o << a << " = vget(L, " << b << ", " << lit(bank.consts[in.x]) << ");";
        break;
      }
      case OP_ITER_INIT: o << "op_iter_init(L, " << a << ", " << R(in.a + 1) << ", " << b << ", " << y << ");"; break;
      case OP_ITER_NEXT:
        if (pstage && PF.has(k, in.a)) {
          o << "{ uint64_t k_ = " << UND << ", v_ = " << UND << "; if (!op_iter_next_p(L, " << a << ", " << R(in.a + 1)
            << ", " << y << ", k_, v_, plo, pn)) goto " << x << ";";
          g.param_reads = true;
          g.param_iter_depth = std::max<uint32_t>(g.param_iter_depth, in.y);
        } else {
          o << "{ uint64_t k_ = " << UND << ", v_ = " << UND << "; if (!op_iter_next(L, " << a << ", " << R(in.a + 1)
            << ", " << y << ", k_, v_)) goto " << x << ";";
        }
        if (in.b != 0xffff) o << " " << b << " = k_;";
        if (in.c != 0xffff) o << " " << c << " = v_;";
        o << " }";
        break;
      case OP_CMP: o << "if (!op_cmp(L, " << y << ", " << b << ", " << c << ", " << a << ")) " << RET; break;
      case OP_ARITH: o << a << " = arith(L, " << y << ", " << b << ", " << c << ");"; break;
      case OP_LIST_NEW:
        if (dce_pcs.count(pc)) o << "/* " << a << ": the argument list of a fused emission */";
        else o << a << " = list_new(L, " << y << ", 4);";
        break;
      case OP_LIST_ADD:
        if (dce_pcs.count(pc)) o << "/* " << a << " += " << b << " */";
        else o << "if (!op_list_add(L, " << a << ", " << b << ", " << y << ")) " << RET;
        break;
      case OP_OBJ_PUT:
        if (kv_sites.count(pc + 1) && kv_sites.at(pc + 1) == pc) o << "/* " << a << "[" << b << "] = " << c << " (the emission's details) */";
        else o << "if (!op_obj_put(L, " << a << ", " << b << ", " << c << ", " << y << ")) " << RET;
        break;
      case OP_YIELD:
        if (EFL.undef_at(k, in.a) && in.a != in.b)  // into an output known to be undefined: a copy (no conflict check)
          o << a << " = " << b << ";" << (in.y ? " if (heap_val(" + a + ")) pin_escape(L, " + y + ");" : std::string());
        else
          o << "if (!op_yield(L, " << a << ", " << b << ", " << y << ")) " << RET;
        break;
      case OP_CALL: {
        // builtins are called directly with register operands (no argument
        // array, no dispatch on the builtin id)
        std::string A0 = R(in.b), A1 = R(in.b + 1), A2 = R(in.b + 2);
        switch (in.y) {
          case BI_COUNT: o << a << " = bi_count(L, " << A0 << ");"; break;
          case BI_ANY: case BI_ALL: o << a << " = bi_anyall(L, " << in.y << "u, " << A0 << ");"; break;
          case BI_STARTSWITH: case BI_ENDSWITH: case BI_CONTAINS:
            o << a << " = bi_strpred(L, " << in.y << "u, " << A0 << ", " << A1 << ");";
            break;
          case BI_RE_MATCH: {
            // re_match is pure: with interned pattern and subject (the usual
            // case: a constraint parameter against a document value) the
            // cross-lane memo answers repeats of the pair from L2 instead of
            // stepping the DFA over the subject's bytes again (gm_put keeps
            // only successful booleans).  GKGPU_RE_MEMO=0: A/B switch.
            // Not for a literal pattern (an inlined DFA, typically inside a
            // pure function the memo already answers: K8sContainerLimits'
            // canonify_cpu ran 4.48 -> 4.73 ms with it).
            const char* rm = getenv("GKGPU_RE_MEMO");
            const bool memo_re = (!rm || atoi(rm) != 0) && LK.konst(k, in.b) < 0;
            if (LK.konst(k, in.b) < 0) g.param_regex = true;
            const std::string site = std::to_string(0x10000u + k) + "u";
            o << "{ uint64_t p_ = " << A0 << ", s_ = " << A1 << "; if (!is_strv(p_) || !is_strv(s_)) { lane_error(L); "
              << a << " = " << UND << "; }";
            if (memo_re) o << " else if (gm_get(" << site << ", p_, s_, " << a << ")) {}";
            o << " else {";
            for (size_t i = 0; i < relits.size(); ++i)
              o << (i ? " else if (p_ == " : " if (p_ == ") << lit(relits[i].first) << ") " << a << " = re_result(L, "
                << relits[i].second << "(sview(L, s_)));";
            o << (relits.empty() ? " " : " else ") << a << " = re_result(L, re_run(L, p_, s_));";
            if (memo_re) o << " gm_put(L, " << site << ", p_, s_, " << a << ");";
            o << " } }";
            break;
          }
          case BI_TO_NUMBER: o << a << " = bi_to_number(L, " << A0 << ");"; break;
          case BI_REPLACE: o << a << " = bi_replace(L, " << A0 << ", " << A1 << ", " << A2 << ");"; break;
          case BI_SUBSTRING: o << a << " = bi_substring(L, " << A0 << ", " << A1 << ", " << A2 << ");"; break;
          case BI_IS_NUMBER: o << a << " = mkv(V_BOOL, is_numv(" << A0 << "));"; break;
          case BI_IS_STRING: o << a << " = mkv(V_BOOL, is_strv(" << A0 << "));"; break;
          default: {
            uint32_t n = in.c ? in.c : 1;
            o << "{ uint64_t av_[" << n << "] = {";
            for (uint32_t i = 0; i < in.c; ++i) o << (i ? ", " : "") << R(in.b + i);
            if (!in.c) o << "0";
            o << "}; " << a << " = call_builtin(L, " << y << ", av_); }";
            break;
          }
        }
        break;
      }
      case OP_SPRINTF: {
        // (a fused emission's shadow copies of the arguments, before the write)
        auto es = esites.find(pc);
        if (es != esites.end())
          for (size_t i = 0; i < es->second.size(); ++i) o << "es" << pc << "_" << i << " = " << R(es->second[i]) << "; ";
        if (dce_sites.count(pc))  // the format alone: the fused emission has the arguments
          o << a << " = mkv(V_FMT, (uint64_t)" << in.x << "u << 32);";
        else if (lazy_fmt(in) && in.x + 1 < bank.fmt.size())  // argument count as an immediate (no table load)
          o << a << " = lazy_sprintf_n(L, " << in.x << "u, " << b << ", " << bank.fmt[in.x + 1] << "u);";
        else
          o << a << " = " << (lazy_fmt(in) ? "lazy_sprintf" : "do_sprintf") << "(L, " << in.x << "u, " << b << ");";
        break;
      }
      case OP_LEN_EQ: o << a << " = op_len_eq(L, " << b << ", " << y << ");"; break;
      case OP_EMIT: {
        // (with details: a register the fast path reads for a one-member object, devrt.h det_fast)
        const EmitFlow::FFact* ff = in.b != in.a ? EFL.find(k, in.a) : nullptr;
        const std::string D = in.b == 0xffff ? std::string(UND) : b;
        if (ff && ff->n > 0) {
          // (mu: the argument registers are read only where the message is the sprintf)
          if (ff->mu) o << "if (vtag(" << a << ") == V_FMT) ";
          o << "{ const uint64_t ea_[" << ff->n << "] = {";
          for (uint16_t i = 0; i < ff->n; ++i) o << (i ? ", " : "") << "es" << ff->site << "_" << i;
          uint64_t yp = 0;
          for (uint16_t i = 0; dce_sites.count(ff->site) && i < ff->n; ++i)
            yp |= (uint64_t)((ff->ys[i] & 0x1fu) | (((ff->ys[i] >> 8) & 0x1fu) << 5)) << (10 * i);
          if (kv_sites.count(pc)) {
            const Ins& put = bank.code[kv_sites.at(pc)];
            o << "}; if (!op_emit_args_kvd<" << (dce_sites.count(ff->site) ? "true" : "false") << ">(L, " << a << ", "
              << R(put.b) << ", " << R(put.c) << ", " << put.y << "u, " << in.c << "u, " << y << ", ea_, " << yp << "ull)) "
              << RET << " }";
          } else if (dce_sites.count(ff->site)) {
            o << "}; if (!op_emit_args_build(L, " << a << ", " << D << ", " << in.c << "u, " << y << ", ea_, " << yp
              << "ull)) " << RET << " }";
          } else {
            o << "}; if (!op_emit_args(L, " << a << ", " << D << ", " << in.c << "u, " << y << ", ea_)) " << RET << " }";
          }
          if (ff->mu)
            o << " else if (!op_emit(L, " << a << ", " << D << ", " << in.c << "u, " << y << ")) " << RET;
        } else {
          o << "if (!op_emit(L, " << a << ", " << (in.b == 0xffff ? std::string(UND) : b) << ", " << in.c << "u, " << y
            << ")) " << RET;
        }
        break;
      }
      case OP_MEMO_GET: {
        // two entries per slot (most recent first): call sites of one function
        // with alternating arguments (canonify_mem(x) vs canonify_mem(max)) hit
        std::string m = std::to_string(in.y), k1 = in.c == 0xffff ? std::string("0ull") : c;
        if (lslots.count(in.y))
          o << "if (mok_" << m << " && mk0_" << m << " == " << b << " && mk1_" << m << " == " << k1 << ") { " << a
            << " = mv_" << m << "; goto " << x << "; }";
        if (memo2.count(in.y))
          o << " if (mokb_" << m << " && mkb0_" << m << " == " << b << " && mkb1_" << m << " == " << k1 << ") { " << a
            << " = mvb_" << m << "; goto " << x << "; }";
        if (psite.count(pc)) {
          const std::string ps = std::to_string(pc);
          o << " if (psok_" << ps << " && psk0_" << ps << " == " << b << " && psk1_" << ps << " == " << k1 << ") { " << a
            << " = psv_" << ps << "; goto " << x << "; }";
          if (gslots.count(in.y))
            o << " if (gm_get(" << m << "u, " << b << ", " << k1 << ", " << a << ")) { psk0_" << ps << " = " << b
              << "; psk1_" << ps << " = " << k1 << "; psv_" << ps << " = " << a << "; psok_" << ps << " = true; goto " << x
              << "; }";
        } else if (gslots.count(in.y)) {
          o << " if (gm_get(" << m << "u, " << b << ", " << k1 << ", " << a << ")) goto " << x << ";";
        }
        break;
      }
      case OP_MEMO_PUT: {
        std::string m = std::to_string(in.y), k1 = in.c == 0xffff ? std::string("0ull") : c;
        if (lslots.count(in.y)) {
          o << "if (memo_stable(" << b << ") && memo_stable(" << k1 << ") && memo_stable(" << a << ")) { ";
          if (memo2.count(in.y))
            o << "mkb0_" << m << " = mk0_" << m << "; mkb1_" << m << " = mk1_" << m << "; mvb_" << m << " = mv_" << m
              << "; mokb_" << m << " = mok_" << m << "; ";
          o << "mk0_" << m << " = " << b << "; mk1_" << m << " = " << k1 << "; mv_" << m << " = " << a << "; mok_" << m
            << " = true; }";
        }
        if (gslots.count(in.y)) o << " gm_put(L, " << m << "u, " << b << ", " << k1 << ", " << a << ");";
        auto pg = put_site.find(pc);
        if (pg != put_site.end()) {
          const std::string ps = std::to_string(pg->second);
          o << " if (memo_stable(" << a << ")) { psk0_" << ps << " = " << b << "; psk1_" << ps << " = " << k1 << "; psv_"
            << ps << " = " << a << "; psok_" << ps << " = true; }";
        }
        break;
      }
      case OP_TABLE: {
        std::string t = table_inline(bank, st, in.x, a, b, lit);
        if (t.empty()) o << a << " = op_table(L, gk_args.K + " << in.x << "u, " << b << ");";
        else o << t;
        break;
      }
      case OP_FAIL_FALLBACK: o << "lane_fallback(L, " << y << "); " << RET; break;
      case OP_ORD: o << "op_ord(L, " << y << ");"; break;
      case OP_JPROBE:
        o << "if (!op_jprobe(L, " << a << ", " << R(in.a + 1) << ", " << b << ", " << y << ")) goto " << x << ";";
        break;
      case OP_JNEXT:
        o << "{ uint64_t v_ = " << UND << "; if (!op_jnext(L, " << a << ", " << R(in.a + 1) << ", " << y << ", v_)) goto "
          << x << "; " << b << " = v_; }";
        break;
      case OP_JVAR: o << a << " = op_jvar(" << b << ", " << R(in.b + 1) << ", " << y << ");"; break;
      default: o << "lane_fallback(L, FB_UNSUPPORTED); " << RET; break;
    }
    o << "\n";
  };

  // Outlined pure-function bodies (GKGPU_JIT_OUTLINE, default on): the code a
  // cross-lane memo miss runs -- the function inlined between MEMO_GET and its
  // MEMO_PUT, e.g. K8sContainerLimits' canonify_mem with get_suffix's six
  // bodies -- becomes a __noinline__ function of its live-in registers, so the
  // predicate keeps only the memo probe and a call.  Misses are rare (a few
  // distinct arguments per launch), and the predicate shrinks: instruction
  // cache footprint and register pressure of the code every lane runs.
  std::map<uint32_t, uint32_t> outl;  // region start (MEMO_GET pc) -> its MEMO_PUT pc
  std::map<uint32_t, std::vector<uint32_t>> outl_in;  // live-in registers of the region
  {
    const char* ov = getenv("GKGPU_JIT_OUTLINE");
    const bool on = !ov || atoi(ov) != 0;
    // global liveness (backward may-analysis)
    const uint32_t nw = (p.nregs + 64) / 64;
    std::vector<std::vector<uint64_t>> live(p.code_len, std::vector<uint64_t>(nw, 0));
    std::vector<uint32_t> rd, wr, sc;
    auto reads_of = [&](uint32_t pc, std::vector<uint32_t>& r) {
      std::vector<uint32_t> w;
      ins_regs(bank.code[pc], r, w);
      const Ins& in = bank.code[pc];
      const uint32_t k = pc - b0;
      // lookups answered by an available register read that register
      if (in.op == OP_GETK) { const int h = LK.find(k, in.b, in.x); if (h >= 0) r.push_back((uint32_t)h); }
      if (in.op == OP_GET) {
        const int kc = LK.konst(k, in.c);
        const int h = kc >= 0 ? LK.find(k, in.b, (uint32_t)kc) : -1;
        if (h >= 0) r.push_back((uint32_t)h);
      }
    };
    for (bool changed = on; changed;) {
      changed = false;
      for (uint32_t k = p.code_len; k-- > 0;) {
        const uint32_t pc = b0 + k;
        std::vector<uint64_t> out(nw, 0);
        ins_succ(bank.code[pc], pc, sc);
        for (uint32_t t : sc)
          if (t >= b0 && t < b1) for (uint32_t w = 0; w < nw; ++w) out[w] |= live[t - b0][w];
        ins_regs(bank.code[pc], rd, wr);
        for (uint32_t r : wr) if (r < 64 * nw) out[r >> 6] &= ~(1ull << (r & 63));
        reads_of(pc, rd);
        for (uint32_t r : rd) if (r < 64 * nw) out[r >> 6] |= 1ull << (r & 63);
        if (out != live[k]) { live[k] = out; changed = true; }
      }
    }
    auto is_live = [&](uint32_t pc, uint32_t r) {
      return pc >= b0 && pc < b1 && r < 64 * nw && ((live[pc - b0][r >> 6] >> (r & 63)) & 1);
    };
    // jump targets from each instruction
    std::vector<std::pair<uint32_t, uint32_t>> jumps;  // (from, to)
    for (uint32_t pc = b0; pc < b1; ++pc)
      if (jump_op(bank.code[pc].op)) jumps.push_back({pc, bank.code[pc].x});
    for (uint32_t pc = b0; on && pc < b1; ++pc) {
      const Ins& in = bank.code[pc];
      if (in.op != OP_MEMO_GET || !gslots.count(in.y)) continue;
      const uint32_t x = in.x, put = x - 1;
      if (x <= pc + 1 || x > b1 || bank.code[put].op != OP_MEMO_PUT || bank.code[put].y != in.y) continue;
      if (put - (pc + 1) < 12) continue;  // small bodies stay inline
      // an argument that may be a deferred sprintf is no memo key (gm_key):
      // every call would miss and pay the out-of-line call
      {
        const uint32_t k = pc - b0;
        if (F.reached[k] && (F.has(k, in.b) || (in.c != 0xffff && F.has(k, in.c)))) continue;
      }
      bool ok = true;
      for (auto& j : jumps) {
        const bool from_in = j.first > pc && j.first < put, to_in = j.second > pc && j.second < put;
        if (from_in && !(to_in || j.second == put || j.second == x)) ok = false;  // leaves the region
        if (!from_in && to_in) ok = false;                                      // enters it
      }
      // what the region writes must be dead after it (its value register aside)
      std::set<uint32_t> wrs;
      for (uint32_t q = pc + 1; q < put && ok; ++q) {
        ins_regs(bank.code[q], rd, wr);
        wrs.insert(wr.begin(), wr.end());
        // register memo entries are the predicate's locals
        const Ins& qi = bank.code[q];
        if ((qi.op == OP_MEMO_GET || qi.op == OP_MEMO_PUT) && lslots.count(qi.y)) ok = false;
        // so are the computed-key CSE shadows (dkN) and a fused emission's
        // argument shadows (esS_i): a region that sets or reads one stays inline
        if (shadowed.count(q) || esites.count(q)) ok = false;
        if (qi.op == OP_GET && LK.konst(q - b0, qi.c) < 0) {
          const int dyn = LK.find_dyn(q - b0, qi.b, qi.c);
          if (dyn >= 0 && (uint32_t)dyn != q) ok = false;
        }
        if (qi.op == OP_EMIT && qi.b != qi.a) {
          const EmitFlow::FFact* ff = EFL.find(q - b0, qi.a);
          if (ff && ff->n > 0) ok = false;
        }
      }
      for (uint32_t r : wrs)
        if (r != in.a && (is_live(x, r) || r == in.b || r == in.c)) ok = false;
      if (!ok) continue;
      // live-in registers of the region (its exits read nothing)
      std::vector<std::vector<uint64_t>> rl(put - pc - 1, std::vector<uint64_t>(nw, 0));
      for (bool ch = true; ch;) {
        ch = false;
        for (uint32_t q = put; q-- > pc + 1;) {
          std::vector<uint64_t> out(nw, 0);
          ins_succ(bank.code[q], q, sc);
          for (uint32_t t : sc)
            if (t > pc && t < put) for (uint32_t w = 0; w < nw; ++w) out[w] |= rl[t - pc - 1][w];
          ins_regs(bank.code[q], rd, wr);
          for (uint32_t r : wr) if (r < 64 * nw) out[r >> 6] &= ~(1ull << (r & 63));
          reads_of(q, rd);
          for (uint32_t r : rd) if (r < 64 * nw) out[r >> 6] |= 1ull << (r & 63);
          if (out != rl[q - pc - 1]) { rl[q - pc - 1] = out; ch = true; }
        }
      }
      std::vector<uint32_t> lin;
      for (uint32_t r = 0; r < 64 * nw && r < p.nregs; ++r)
        if ((rl[0][r >> 6] >> (r & 63)) & 1) lin.push_back(r);
      if (std::find(lin.begin(), lin.end(), (uint32_t)in.a) == lin.end()) lin.insert(lin.begin(), in.a);
      outl[pc] = put;
      outl_in[pc] = lin;
      pc = put;  // outermost regions only
    }
  }
  // register memo sites inside an outlined body stay memo-only (their
  // registers are the predicate's locals)
  for (auto& kv : outl)
    for (uint32_t q = kv.first + 1; q < kv.second; ++q) {
      if (psite.erase(q)) put_site.erase(bank.code[q].x - 1);
    }
  for (uint32_t ps : psite)
    o << "  uint64_t psk0_" << ps << " = 0, psk1_" << ps << " = 0, psv_" << ps << " = 0; bool psok_" << ps << " = false;\n";
  std::ostringstream fo;  // the outlined functions (before the predicate)
  for (auto& kv : outl) {
    const uint32_t g0 = kv.first, put = kv.second;
    const Ins& gi = bank.code[g0];
    const std::vector<uint32_t>& lin = outl_in[g0];
    std::set<uint32_t> used;
    std::vector<uint32_t> rd, wr;
    for (uint32_t q = g0 + 1; q < put; ++q) {
      ins_regs(bank.code[q], rd, wr);
      used.insert(rd.begin(), rd.end());
      used.insert(wr.begin(), wr.end());
    }
    for (uint32_t r : lin) used.erase(r);
    fo << "__device__ __noinline__ uint64_t gk_o" << g0 << "(PLane& L, uint32_t plo, uint32_t pn";
    for (uint32_t r : lin) fo << ", uint64_t " << R(r);
    fo << ") {\n";
    if (!used.empty()) {
      fo << "  uint64_t ";
      bool first = true;
      for (uint32_t r : used) { fo << (first ? "" : ", ") << R(r); first = false; }
      fo << ";\n";
    }
    const std::string ret = "return " + R(gi.a) + ";";
    std::ostringstream ob;
    for (uint32_t q = g0 + 1; q < put; ++q) emit(q, ob, ret);
    fo << ob.str() << "L" << put << ":;\nL" << gi.x << ":;\n  " << ret << "\n}\n";
  }
  for (uint32_t pc = b0; pc < b1; ++pc) {
    emit(pc, o, "return;");
    auto ol = outl.find(pc);
    if (ol == outl.end()) continue;
    const Ins& in = bank.code[pc];
    o << "  " << R(in.a) << " = gk_o" << pc << "(L, plo, pn";
    for (uint32_t r : outl_in[pc]) o << ", " << R(r);
    o << "); if (L.fail) return;\n";
    pc = ol->second - 1;  // continue at the MEMO_PUT
  }
  g.pre += fo.str();
  o << "  lane_fallback(L, FB_UNSUPPORTED);\n";
  g.body = o.str();
  return g;
}

std::mutex g_mu;
std::map<std::string, std::string> g_cache;  // source -> code object

std::string cache_dir() {
  const char* d = getenv("GKGPU_JIT_CACHE");
  if (d && !strcmp(d, "0")) return "";
  if (d && *d) return d;
  const char* h = getenv("HOME");
  if (!h || !*h) return "";
  return std::string(h) + "/.cache/gkgpu-jit";
}

bool read_file(const std::string& path, std::string& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return !out.empty();
}

void write_file_atomic(const std::string& dir, const std::string& name, const std::string& data) {
  std::string cur;
  for (size_t i = 1; i <= dir.size(); ++i)
    if (i == dir.size() || dir[i] == '/') { cur = dir.substr(0, i); mkdir(cur.c_str(), 0755); }
  std::string tmp = dir + "/." + name + "." + std::to_string(getpid());
  {
    std::ofstream f(tmp, std::ios::binary);
    if (!f) return;
    f.write(data.data(), (std::streamsize)data.size());
    if (!f) { unlink(tmp.c_str()); return; }
  }
  if (rename(tmp.c_str(), (dir + "/" + name).c_str()) != 0) unlink(tmp.c_str());
}

}  // namespace

// Occupancy of a template kernel: minimum waves per SIMD it is compiled for
// (caps VGPRs at 512/n; the compiler spills beyond) and the lane-heap words it
// keeps in LDS (devrt.h GK_LDS_HWORDS; with the 8 KB of lane scalars, LDS
// caps the 256-thread blocks per CU).  History: round 1 measured 2 waves best
// for K8sContainerLimits (65 ms at the compiler's choice of 1, 41 ms at 2, 69
// at 4; later 11.0 / 8.4 / 12.5 ms at 1 / 2 / 3).  Round 2 (tools/gpu_r02s.sh,
// config 2 at 1M Pods, one call): K8sContainerLimits (64 registers) 4.70 ms
// at 2 waves + 32 heap words, 5.87 at 3 + 16, 6.55 at 4 + 16; K8sRequiredProbes
// (40 registers) 3.39 / 2.83 / 2.98.  So programs with at most 48 registers
// get 3 waves, larger ones 2.  Heap words: 16 for both since round 4 -- the
// per-iteration heap marks keep the config-2 templates' lane heaps inside 16
// words (CPU accounting build), and the 32 KB a 2-wave block no longer spends
// on heap words goes to the LDS stage (parameters, memo cache): config 4's
// K8sContainerLimits 7.8 -> 5.7 ms, config 2 unchanged (profiles/r04/
// r04s_ab.txt; all templates at 16 vs 32: config 4 1,774 vs 1,169 M evals/s,
// r04zd_ab.txt).  GKGPU_JIT_WPE and GKGPU_LDS_HEAP override both choices (WPE
// 0 = the compiler's choice).
// Round 5 (profiles/r05/r05h_wpe_ab.txt, r05i_wpe_ab.txt): 4 waves for small
// programs without regular expressions -- K8sRequiredProbes 1.55 -> 1.45 ms
// (config 2) and 4.29 -> 4.11 ms (config 4), K8sAllowedRepos 0.195 -> 0.179 /
// 4.12 -> 4.04 ms -- while the regex templates (their DFAs staged in LDS) and
// K8sContainerLimits lose at 4.  Re-checked at the end of round 5, after the
// emission changes (profiles/r05/r05ay_wpe_recheck_ab.txt): every template at 3
// or at 2 is slower on config 2 (1,000 -> 938 / 898 M evals/s), and the regex
// templates at 2 or 4 on config 3 (1,030 -> 762 / 749 M).
// Round 6, column form (profiles/r06/r06g_wpe_heap_grid.txt: every template at
// 2 / 3 / 4 waves and 4-16 heap words, configs 2 and 4 in one call): small
// programs at 3.  A 4-wave request leaves 40 KB of LDS, less than the 16 heap
// words, the lane scalars and the parameter stage need, so the compiler got
// no usable bound and K8sRequiredProbes read its parameters (probes x
// probeTypes, iterated per container) from the node store: 1.62 -> 1.23 ms
// (config 2) and 8.44 -> 3.43 ms (config 4) at 3; K8sAllowedRepos gives back
// 0.02 / 0.28 ms.  Fewer heap words at 4 waves stage the parameters too but
// lose elsewhere (K8sContainerLimits 1.29 -> 2.7 ms).
// Refined at the end of round 6: the small programs that need the parameter
// stage are those iterating a parameter collection inside a loop over another
// one (loop level >= 3: RequiredProbes' probeTypes inside probes inside
// containers) and those with regular expressions (their DFAs are staged too);
// they get 3 waves.  Other small programs keep round 5's 4: K8sAllowedRepos
// (one parameter loop per container) 0.157 -> 0.143 ms config 2, 3.17 -> 2.89
// ms config 4 (profiles/r06/r06g_wpe_heap_grid.txt, ab1 vs ab2).
static bool small_program(const Program& p) { return p.nregs <= 48; }
static int wpe_of(const Program& p, const Gen& g) {
  const char* w = getenv("GKGPU_JIT_WPE");
  if (w) return atoi(w);
  if (!small_program(p)) return 2;
  return (p.uses_regex || g.param_iter_depth >= 3) ? 3 : 4;
}
// (Launch bounds at 3 or 4 waves with the LDS plan of the default left
// unchanged measured slower for K8sContainerLimits -- 1.28 -> 1.56 / 2.71 ms
// -- and neutral elsewhere: profiles/r06/r06n_launch_bound_ab.txt.)
static std::string wpe_suffix(const Program& p, const Gen& g) {
  const int n = wpe_of(p, g);
  return n > 0 ? ", " + std::to_string(n) : std::string();
}
static int lds_heap_words(const Program& p) {
  const char* v = getenv("GKGPU_LDS_HEAP");
  int n = v ? atoi(v) : 16;
  return n < 0 ? 0 : (n > 64 ? 64 : n);
}

// Lane scalars in LDS (devrt.h GK_LDS_SCALARS): 8 KB per 256-thread block.
// GKGPU_LDS_SCALARS=0 keeps them in the private segment (A/B).
static bool lds_scalars() {
  const char* v = getenv("GKGPU_LDS_SCALARS");
  return !v || atoi(v) != 0;
}

// LDS stage (devrt.h GK_LDS_PARAMS / GK_LDS_DFA): what the kernel's block may
// add to the lane heap words and scalars and still fit the blocks per CU its
// waves-per-EU asks for (160 KB per CU).  2-wave kernels (32 heap words, 73 KB)
// take one of the two, 3-wave kernels (16 words, 41 KB) both.
constexpr uint32_t kMaxLoop = 16;  // devrt.h MAXLOOP
static int max_depth(const Program& p, const CodeBank& bank) {
  uint32_t m = 0;
  for (uint32_t k = 0; k < p.code_len; ++k) {
    const Ins& in = bank.code[p.code_off + k];
    uint32_t d = 0;
    switch (in.op) {
      case OP_ITER_INIT: case OP_ITER_NEXT: case OP_JNEXT: d = in.y < kMaxLoop ? in.y : 0; break;
      case OP_JPROBE: d = (in.y & 0xff) < kMaxLoop ? (in.y & 0xff) : 0; break;
      case OP_LIST_ADD: case OP_OBJ_PUT: case OP_YIELD: d = (in.y >> 8) & 0xff; break;
      default: break;
    }
    m = std::max(m, d);
  }
  return (int)std::min<uint32_t>(m + 1, kMaxLoop);
}

// LDS cache of the cross-lane memo (devrt.h GK_LDS_MEMO): entries per
// wavefront for a program with pure-function memo sites, 0 = none.
// GKGPU_JIT_LDSMEMO=0 disables it (A/B), =N sets the entries (a power of two).
static int lds_memo_entries(const Gen& g) {
  const char* v = getenv("GKGPU_JIT_LDSMEMO");
  int n = v ? atoi(v) : 32;
  if (n <= 0) return 0;
  if (n > 256) n = 256;
  while (n & (n - 1)) n &= n - 1;
  return (g.pre.find("gm_get(") != std::string::npos || g.body.find("gm_get(") != std::string::npos) ? n : 0;
}

struct StagePlan { bool params = false, dfa = false; int memo = 0; };
static StagePlan stage_plan(const Program& p, const Gen& g, int depth) {
  StagePlan sp;
  if (!lds_stage_on()) return sp;
  const int wpe = wpe_of(p, g);
  const uint32_t limit = (wpe > 0 ? 163840u / (uint32_t)wpe : 163840u) - 512u;  // allocation granularity slack
  // lane heap words, lane scalars and (with the scalars) the loop watermarks;
  // then, as they fit: the memo cache, the DFAs, the parameters
  uint32_t used = (uint32_t)lds_heap_words(p) * 8u * 256u + (lds_scalars() ? 9u * 4u * 256u + 4u * 256u * (uint32_t)depth : 0u);
  // (the memo cache before the parameters when the program probes the memo at
  // more sites than it reads parameters: K8sContainerLimits' canonify calls
  // per container against its two parameter reads per lane)
  auto count = [&](const char* w) {
    size_t n = 0;
    for (const std::string* t : {&g.pre, &g.body})
      for (size_t at = 0; (at = t->find(w, at)) != std::string::npos; ++at) ++n;
    return n;
  };
  const uint32_t mbytes = 4u * 32u * (uint32_t)lds_memo_entries(g);
  const bool memo_first = mbytes && count("gm_get(") > count("vget_p(") + count("op_iter_next_p(");
  auto memo = [&] { if (mbytes && used + mbytes <= limit) { sp.memo = lds_memo_entries(g); used += mbytes; } };
  const uint32_t pbytes = 4u * 64u * 16u, dbytes = 4u * 1024u + 4u * 17u * 4u;  // devrt.h LDS_PCAP / LDS_DFA_*
  if (memo_first) memo();
  if (g.param_regex && used + dbytes <= limit) { sp.dfa = true; used += dbytes; }
  if (g.param_reads && used + pbytes <= limit) { sp.params = true; used += pbytes; }
  if (!memo_first) memo();
  return sp;
}

// the loop levels a program's lane uses (devrt.h GK_MAXDEPTH): loop depths
// of its iterations and probes, and the ranges values escaping loops pin
static std::string inline_hot_tag(const Program& p) {
  const char* v = getenv("GKGPU_INLINE_HOT");
  std::string t = (!v || atoi(v) != 0) ? "h1" : "h0";
  t += "d" + std::to_string(lds_heap_words(p));
  if (!lds_scalars()) t += "s0";
  if (!lds_stage_on()) t += "p0";
  return t;
}

std::string jit_name(const Program& p, const CodeBank& bank, const Store& st) {
  Gen g = generate(p, bank, st);
  return "gk_t_" + hex16(fnv1a(g.pre + g.body + wpe_suffix(p, g) + inline_hot_tag(p) + "lm" + std::to_string(lds_memo_entries(g))));
}

std::string jit_source(const Program& p, const CodeBank& bank, const Store& st, const std::string& name) {
  Gen g = generate(p, bank, st);
  std::ostringstream o;
  o << "// generated by jit.cc from template bytecode (" << p.code_len << " instructions)\n";
  if (const char* pre = getenv("GKGPU_JIT_PRE")) {  // diagnostics: e.g. "GK_BCAP=1024,GK_HCAP=64"
    std::string d = pre;
    for (size_t i = 0, j; i < d.size(); i = j + 1) {
      j = d.find(',', i);
      if (j == std::string::npos) j = d.size();
      std::string kv = d.substr(i, j - i);
      size_t eq = kv.find('=');
      if (eq != std::string::npos) o << "#define " << kv.substr(0, eq) << " " << kv.substr(eq + 1) << "\n";
    }
  }
  // GKGPU_INLINE_HOT (A/B switch, default on): inline the per-container builtins
  if (!getenv("GKGPU_INLINE_HOT") || atoi(getenv("GKGPU_INLINE_HOT")) != 0) o << "#define GK_INLINE_HOT 1\n";
  if (lds_heap_words(p) > 0) o << "#define GK_LDS_HWORDS " << lds_heap_words(p) << "\n";
  if (lds_scalars()) o << "#define GK_LDS_SCALARS 1\n";
  const int depth = max_depth(p, bank);
  o << "#define GK_MAXDEPTH " << depth << "\n";
  const StagePlan sp = stage_plan(p, g, depth);
  if (sp.params) o << "#define GK_LDS_PARAMS 1\n";
  if (sp.dfa) o << "#define GK_LDS_DFA 1\n";
  if (sp.memo) o << "#define GK_LDS_MEMO " << sp.memo << "\n";
  o << "#include \"devrt.h\"\n"
    << "namespace gk {\n"
    << g.pre
    << (sp.params ? "" : "#define vget_p(L, c, k, lo, n) vget(L, c, k)\n"
                         "#define op_iter_next_p(L, c, st, y, k, v, lo, n) op_iter_next(L, c, st, y, k, v)\n")
    << "__device__ void " << name << "_pred(PLane& L, uint64_t review, uint64_t params, uint32_t plo, uint32_t pn) {\n"
    << g.body << "}\n"
    << "}  // namespace gk\n"
    << "extern \"C\" __global__ void __launch_bounds__(256" << wpe_suffix(p, g) << ") " << name << "(gk::DevArgs) {\n"
    << "  gk::audit_body([&](gk::PLane& L, uint64_t review, uint64_t params, uint32_t, uint32_t plo, uint32_t pn) {\n"
    << "    gk::" << name << "_pred(L, review, params, plo, pn);\n"
    << "  });\n"
    << "}\n";
  std::string src = o.str();
  // diagnostics (GPU probes of what a kernel's parts cost): GKGPU_JIT_PATCH =
  // "from=>to||from2=>to2" replaces text in every generated kernel source
  if (const char* pt = getenv("GKGPU_JIT_PATCH")) {
    std::string spec = pt;
    if (!spec.empty() && spec[0] == '@' && !read_file(spec.substr(1), spec)) spec.clear();  // @file: the spec in a file
    for (size_t i = 0; i < spec.size();) {
      size_t j = spec.find("||", i);
      if (j == std::string::npos) j = spec.size();
      const std::string item = spec.substr(i, j - i);
      const size_t arrow = item.find("=>");
      if (arrow != std::string::npos) {
        const std::string from = item.substr(0, arrow), to = item.substr(arrow + 2);
        for (size_t at = 0; !from.empty() && (at = src.find(from, at)) != std::string::npos; at += to.size())
          src.replace(at, from.size(), to);
      }
      i = j + 2;
    }
  }
  return src;
}

bool jit_compile(const std::string& src, std::string& code, std::string& log) {
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_cache.find(src);
    if (it != g_cache.end()) { code = it->second; return true; }
  }
  int ver_major = 0, ver_minor = 0;
  hiprtcVersion(&ver_major, &ver_minor);
  // GKGPU_JIT_OPTS (diagnostics): extra hipRTC options, space-separated
  std::vector<std::string> xopt;
  if (const char* xo = getenv("GKGPU_JIT_OPTS")) {
    std::istringstream is(xo);
    for (std::string t; is >> t;) xopt.push_back(t);
  }
  // the key covers every option the code object is compiled with (the base
  // options too: a changed base option must not reuse code built without it)
  std::vector<const char*> opts = base_opts();
  for (const auto& t : xopt) opts.push_back(t.c_str());
  std::string xkey;
  for (const char* t : opts) xkey += std::string(" ") + t;
  std::string key = hex16(fnv1a(src + xkey, fnv1a(std::string(gk_rt_common_h) + gk_rt_devrt_h +
                                                  std::to_string(ver_major) + "." + std::to_string(ver_minor))));
  std::string dir = cache_dir();
  std::string fname = key + ".co";
  if (!dir.empty() && read_file(dir + "/" + fname, code)) {
    std::lock_guard<std::mutex> g(g_mu);
    g_cache[src] = code;
    return true;
  }
  if (const char* dd = getenv("GKGPU_JIT_DUMP")) {  // diagnostics: keep the generated source
    if (*dd) write_file_atomic(dd, key + ".hip", src);
  }
  if (getenv("GKGPU_JIT_DUMP_ONLY")) {  // host tests of the generator: no hipRTC (the template stays on the VM)
    log = "GKGPU_JIT_DUMP_ONLY";
    return false;
  }
  hiprtcProgram prog;
  const char* hs[] = {gk_rt_common_h, gk_rt_devrt_h};
  const char* hn[] = {"common.h", "devrt.h"};
  if (hiprtcCreateProgram(&prog, src.c_str(), "gk_template.hip", 2, hs, hn) != HIPRTC_SUCCESS) {
    log = "hiprtcCreateProgram failed";
    return false;
  }
  hiprtcResult r = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  log.assign(ls, '\0');
  if (ls) hiprtcGetProgramLog(prog, &log[0]);
  bool ok = r == HIPRTC_SUCCESS;
  if (ok) {
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    code.assign(cs, '\0');
    ok = cs > 0 && hiprtcGetCode(prog, &code[0]) == HIPRTC_SUCCESS;
  }
  hiprtcDestroyProgram(&prog);
  if (!ok) return false;
  {
    std::lock_guard<std::mutex> g(g_mu);
    g_cache[src] = code;
  }
  if (!dir.empty()) write_file_atomic(dir, fname, code);
  return true;
}

// the bytecode's register reads / writes and successors, for analyses in
// other translation units (colplan.cc)
void bc_regs(const Ins& in, std::vector<uint32_t>& rd, std::vector<uint32_t>& wr) { ins_regs(in, rd, wr); }
void bc_succ(const Ins& in, uint32_t pc, std::vector<uint32_t>& out) { ins_succ(in, pc, out); }

}  // namespace gk
