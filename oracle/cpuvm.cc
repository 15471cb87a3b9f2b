// CPU baseline of the audit sweep -- TEST / MEASUREMENT INFRASTRUCTURE, NOT
// THE PRODUCT AND NOT OPA.
//
// The reference's own CPU path (Go OPA v0.21 topdown, drivers/local/local.go)
// cannot be built here (no Go toolchain), so bench.py's
// cpu_baseline times this native multi-threaded evaluator instead, labelled
// kind "port" with its thread count.  It runs the SAME compiled template
// bytecode and the same match / builtin / printing semantics as the device
// (the engine's devrt.h compiled for the host), one (review, constraint) pair
// per call, over std::thread workers -- i.e. an interpreter of the engine's
// own program, with none of OPA's per-Review JSON round trips
// (local.go:331, rego.go:1478-1496), so it is a much stronger baseline than
// the reference as deployed.  Messages are formatted, as the GPU format pass
// does.  Only bench.py's cpu_baseline leg and tests load it; the product
// (gatekeeper-1_amd/) never does.
//
// Per pair it follows devrt.h audit_body (autoreject, matching_constraints,
// template program) and kernels.hip run_program (the bytecode VM loop).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

// ---- host spellings of the device-language words devrt.h uses
namespace __hip_internal {
using ::int16_t;
using ::int32_t;
using ::int64_t;
using ::int8_t;
using ::uint16_t;
using ::uint32_t;
using ::uint64_t;
using ::uint8_t;
}  // namespace __hip_internal
#define __HIPCC_RTC__ 1
#define GK_HOST 1
#define GK_PRIV
#define __device__
#define __global__
#define __host__
// each worker thread evaluates with its own copy of the launch arguments,
// whose output buffers are that thread's (OutBufs below)
#define __constant__ thread_local
#define __forceinline__ inline __attribute__((always_inline))
#define __noinline__ __attribute__((noinline))
// single-lane stand-ins: the emission path's wave-level reservations see a
// wave of one lane (devrt.h GK_HOST); audit_body / finish_lane are compiled
// but never called here
template <class T> static inline T __shfl_up(T v, int, int) { return v; }
template <class T> static inline T __shfl(T v, int, int) { return v; }
template <class T> static inline T __shfl_xor(T v, int, int) { return v; }
template <class T, class U> static inline T atomicAdd(T* p, U v) { T o = *p; *p = (T)(o + v); return o; }
template <class T, class U> static inline T atomicOr(T* p, U v) { T o = *p; *p = (T)(o | v); return o; }
template <class T, class U> static inline T atomicMax(T* p, U v) { T o = *p; if ((T)v > o) *p = (T)v; return o; }
static inline uint64_t __umul64hi(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }
static inline void __threadfence() {}  // the host build has no memo arena (gk_args.mstr is null)
struct CpuDim3 { uint32_t x = 0, y = 0, z = 0; };
static CpuDim3 blockIdx, threadIdx, blockDim{64, 1, 1}, gridDim{1, 1, 1};

#ifdef GKCPU_TOUCH
// Reference accounting build (cpuvm_touch.cc): the same runtime in its own
// namespace, recording every document node and string the evaluation reads.
namespace gkcpu_touch {
thread_local uint64_t* node_bits = nullptr;
thread_local uint64_t* str_bits = nullptr;
thread_local uint64_t* pc_hist = nullptr;  // executions per bytecode instruction
}  // namespace gkcpu_touch
#define GK_TOUCH_NODE(i) (gkcpu_touch::node_bits[(uint32_t)(i) >> 6] |= 1ull << ((uint32_t)(i) & 63))
#define GK_TOUCH_STR(s) (gkcpu_touch::str_bits[(uint32_t)(s) >> 6] |= 1ull << ((uint32_t)(s) & 63))
// lane-state writes by heap word index (bucket: <16, <32, <64, the rest) and
// lane-buffer bytes: where a template kernel's lane state lands (LDS words vs
// the private segment; gkcpu_scratch_stats)
namespace gkcpu_touch {
thread_local uint64_t heap_w[4] = {0, 0, 0, 0};
thread_local uint64_t buf_b = 0;
}  // namespace gkcpu_touch
#define GK_HEAP_WRITE(w) (++gkcpu_touch::heap_w[(w) < 16 ? 0 : (w) < 32 ? 1 : (w) < 64 ? 2 : 3])
#define GK_BUF_WRITE(n) (gkcpu_touch::buf_b += (n))
#endif

// the launch arguments devrt.h reads (the device reads its kernarg segment)
#include "../gatekeeper-1_amd/csrc/common.h"
extern "C" {
__constant__ gk::DevArgs gk_args;
}
#include "../gatekeeper-1_amd/csrc/devrt.h"

namespace gk {
namespace cpu {

constexpr int NREG = 192;

// kernels.hip run_program on the host
static void run_program(Lane& L, uint32_t pc, uint64_t review, uint64_t params) {
  const uint64_t UND = mkv(V_UNDEF, 0);
  uint64_t R[NREG];
  for (int guard = 0; guard < (1 << 22); ++guard) {
    if (pc >= gk_args.ncode) { lane_fallback(L, FB_UNSUPPORTED); return; }
    const Ins in = gk_args.code[pc];
#ifdef GKCPU_TOUCH
    if (gkcpu_touch::pc_hist) ++gkcpu_touch::pc_hist[pc];
#endif
    ++pc;
    switch (in.op) {
      case OP_END: return;
      case OP_JMP: pc = in.x; break;
      case OP_JUNDEF: if (vtag(R[in.a]) == V_UNDEF) pc = in.x; break;
      case OP_JFALSE: if (vtag(R[in.a]) == V_BOOL && vpay(R[in.a]) == 0) pc = in.x; break;
      case OP_JTRUE: if (vtag(R[in.a]) == V_BOOL && vpay(R[in.a]) == 1) pc = in.x; break;
      case OP_LOADK: R[in.a] = gk_args.K[in.x]; break;
      case OP_LOADREV: R[in.a] = review; break;
      case OP_LOADPARAM: R[in.a] = params; break;
      case OP_MOV: R[in.a] = R[in.b]; break;
      case OP_GET: R[in.a] = vget(L, R[in.b], R[in.c]); break;
      case OP_GETK: R[in.a] = vget(L, R[in.b], gk_args.K[in.x]); break;
      case OP_ITER_INIT: op_iter_init(L, R[in.a], R[in.a + 1], R[in.b], in.y); break;
      case OP_ITER_NEXT: {
        uint64_t k = UND, v = UND;
        if (!op_iter_next(L, R[in.a], R[in.a + 1], in.y, k, v)) { pc = in.x; break; }
        if (in.b != 0xffff) R[in.b] = k;
        if (in.c != 0xffff) R[in.c] = v;
        break;
      }
      case OP_CMP: if (!op_cmp(L, in.y, R[in.b], R[in.c], R[in.a])) return; break;
      case OP_ARITH: R[in.a] = arith(L, in.y, R[in.b], R[in.c]); if (L.fail) return; break;
      case OP_LIST_NEW: R[in.a] = list_new(L, in.y, 4); if (L.fail) return; break;
      case OP_LIST_ADD: if (!op_list_add(L, R[in.a], R[in.b], in.y)) return; break;
      case OP_OBJ_PUT: if (!op_obj_put(L, R[in.a], R[in.b], R[in.c], in.y)) return; break;
      case OP_YIELD: if (!op_yield(L, R[in.a], R[in.b], in.y)) return; break;
      case OP_CALL: R[in.a] = call_builtin(L, in.y, &R[in.b]); if (L.fail) return; break;
      case OP_SPRINTF: R[in.a] = do_sprintf(L, in.x, R[in.b]); if (L.fail) return; break;
      case OP_LEN_EQ: R[in.a] = op_len_eq(L, R[in.b], in.y); break;
      case OP_EMIT: if (!op_emit(L, R[in.a], in.b == 0xffff ? UND : R[in.b], in.c, in.y)) return; break;
      case OP_TABLE: R[in.a] = op_table(L, gk_args.K + in.x, R[in.b]); break;
      case OP_MEMO_GET: {
        uint64_t k1 = in.c == 0xffff ? 0 : R[in.c];
        if (((L.memo_ok >> in.y) & 1) && L.memo_k0[in.y] == R[in.b] && L.memo_k1[in.y] == k1) {
          R[in.a] = L.memo_v[in.y];
          pc = in.x;
        }
        break;
      }
      case OP_MEMO_PUT: {
        uint64_t k1 = in.c == 0xffff ? 0 : R[in.c];
        if (memo_stable(R[in.b]) && memo_stable(k1) && memo_stable(R[in.a])) {
          L.memo_k0[in.y] = R[in.b];
          L.memo_k1[in.y] = k1;
          L.memo_v[in.y] = R[in.a];
          L.memo_ok |= 1u << in.y;
        }
        break;
      }
      case OP_FAIL_FALLBACK: lane_fallback(L, in.y); return;
      case OP_ORD: op_ord(L, in.y); break;
      // inventory joins: with gkcpu_build_joins' indexes the probe, else
      // (jdir null) the plain scan the compiler emits beside it
      case OP_JPROBE: if (!op_jprobe(L, R[in.a], R[in.a + 1], R[in.b], in.y)) pc = in.x; break;
      case OP_JNEXT: {
        uint64_t v = UND;
        if (!op_jnext(L, R[in.a], R[in.a + 1], in.y, v)) { pc = in.x; break; }
        R[in.b] = v;
        break;
      }
      case OP_JVAR: R[in.a] = op_jvar(R[in.b], R[in.b + 1], in.y); break;
      case OP_KEYOUT: op_keyout(L, R[in.a]); break;
      default: lane_fallback(L, FB_UNSUPPORTED); return;
    }
  }
  lane_fallback(L, FB_UNSUPPORTED);
}

struct Counts {
  uint64_t evals = 0, violations = 0, msg_bytes = 0, flagged = 0;
  uint64_t digest = 0;  // sum over result rows of row_hash (an order-free multiset digest)
};

// gkcpu_sweep_digest: rows are hashed as FNV-1a 64 over (u32 batch review index
// LE, u32 constraint LE, message bytes, 0xff, details JSON bytes); tests compute
// the same over the oracle's rows (oracle/cpu_baseline.py row_hash)
static bool g_digest = false;
static uint64_t g_last_digest = 0;
static uint64_t fnv_bytes(uint64_t h, const void* p, size_t n) {
  const unsigned char* b = (const unsigned char*)p;
  for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ull; }
  return h;
}

// A worker thread's output buffers: its copy of the launch arguments points
// the emission path (devrt.h op_emit / emit_eager) at them.  One pair emits
// at most EM_MAXIDX tuples (then it falls back), each staging at most BCAP
// bytes, so the per-pair capacities never overflow.
struct OutBufs {
  std::vector<Viol> out;
  std::vector<uint64_t> frec;
  std::vector<char> ebytes;
  unsigned long long counters[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t rflags[1] = {0};
  void bind(const void* args) {
    memcpy(&gk_args, args, sizeof(DevArgs));
    out.resize(EM_MAXIDX + 1);
    frec.resize((size_t)(EM_MAXIDX + 1) * FMT_MAXARGS);
    ebytes.resize((size_t)(EM_MAXIDX + 1) * (BCAP + 64) + 16);
    gk_args.out = out.data();
    gk_args.out_cap = out.size();
    gk_args.frec = frec.data();
    gk_args.ebytes = ebytes.data();
    gk_args.ebytes_cap = ebytes.size() - 16;
    gk_args.counters = counters;
    gk_args.rflags = rflags;
    gk_args.rreason = nullptr;
    gk_args.totals = nullptr;
  }
};

// devrt.h audit_body for one (review position, constraint), then the message
// bytes of every tuple it emitted (the size + format passes' work)
static void eval_pair(uint32_t rp, uint32_t c, Counts& k, char* fbuf, uint32_t fcap) {
  Lane L;
  L.hp = 0; L.bp = 0; L.ord = 0; L.ord_base = 0; L.fail = 0; L.reason = 0; L.en = 0; L.steps = 0; L.memo_ok = 0;
  for (int d = 0; d < MAXLOOP; ++d) { L.keepH[d] = 0; L.keepB[d] = 0; }
  L.rv = 0;  // the thread's one-slot flag word
  L.cn = c;
  gk_args.counters[0] = 0;
  gk_args.counters[1] = 0;
  const ReviewCol rc = gk_args.revs[rp];
  const MatchSpec m = gk_args.cons[c];
  ++k.evals;
  if (rc.flags & RC_FALLBACK) {
    L.fail = RF_FALLBACK;
  } else {
    if (!(rc.flags & RC_AUDIT) && (m.flags & MF_HAS_NSSEL) && (rc.flags & RC_HAS_NS) && rc.ns != NO_ID && !(rc.flags & RC_NS_EMPTY) &&
        !(rc.flags & RC_NS_CACHED) && !(rc.flags & RC_UNSTABLE_NS))
      emit_eager(L, true, RULE_AUTOREJECT, "Namespace is not cached in OPA.", 31, nullptr, 2);
    int mr = match_constraint(m, rc);
    if (mr == -1) L.fail = RF_ERROR;
    else if (mr == -2) L.fail = RF_FALLBACK;
    else if (mr == 1 && (m.flags & MF_FALLBACK)) lane_fallback(L, FB_TEMPLATE);
    else if (mr == 1 && m.prog != NO_ID) {
      uint64_t params = m.params == NO_ID ? mkv(V_NODE, 0) : nodeval(m.params);
      run_program(L, gk_args.prog_off[m.prog], gk_args.cv_on ? mkv(V_ROW, (uint64_t)rp) : mkv(V_NODE, rc.root), params);
    }
  }
  if (L.fail) { ++k.flagged; return; }
  const uint64_t n = gk_args.counters[0];
  const uint32_t review = rc.orig != NO_ID ? rc.orig : rp;
  std::vector<char> dbuf;
  for (uint64_t i = 0; i < n; ++i) {
    const Viol& v = gk_args.out[i];
    const char* mp = gk_args.ebytes + v.msg_off;
    uint32_t ml = v.msg_len;
    if (v.pad & VF_DEFER) {
      const uint32_t fidx = v.msg_len & 0xffffffu, na = v.msg_len >> 24;
      Out out{fbuf, 0, fcap, false};
      if (!fmt_run(L, out, fidx, [&](uint32_t j) { return j < na ? gk_args.frec[(uint64_t)j * gk_args.out_cap + i] : 0ull; })) {
        ++k.flagged;  // the size pass's outcome: the review goes to the CPU fallback
        return;
      }
      k.msg_bytes += out.n;
      mp = fbuf;
      ml = out.n;
    } else {
      k.msg_bytes += v.msg_len;
    }
    const char* dp = "{}";
    uint32_t dl = 2;
    if (v.pad & (VF_DET_VAL | VF_DET_KV)) {
      // details as frec words: VF_DET_VAL the JSON of one value, VF_DET_KV a
      // one-member object {k: v} (k at word di, v at di + 1) -- what the size
      // and format passes print (kernels.hip put_det_words)
      const uint32_t di = (v.pad & VF_DEFER) ? (v.msg_len >> 24) : 0u;
      const bool kv = (v.pad & VF_DET_KV) != 0;
      const uint64_t dk = kv ? gk_args.frec[(uint64_t)di * gk_args.out_cap + i] : 0ull;
      const uint64_t dv = gk_args.frec[(uint64_t)(di + (kv ? 1u : 0u)) * gk_args.out_cap + i];
      auto print = [&](auto& o) {
        if (kv) {
          put(o, '{');
          if (!put_json_str(o, sview(L, dk))) return false;
          put(o, ':');
        }
        if (!put_json(L, o, dv)) return false;
        if (kv) put(o, '}');
        return true;
      };
      Cnt cn{0, false};
      if (!print(cn)) {
        ++k.flagged;
        return;
      }
      if (g_digest) {
        dbuf.resize(cn.n + 1);
        Out o{dbuf.data(), 0, (uint32_t)dbuf.size(), false};
        print(o);
        dp = dbuf.data();
        dl = o.n;
      }
    } else if (!(v.pad & VF_DET_OBJ)) {
      dp = gk_args.ebytes + v.msg_off + ((v.pad & VF_DEFER) ? 0u : v.msg_len);
      dl = v.det_len;
    }
    if (g_digest) {
      uint64_t h = 1469598103934665603ull;
      const uint32_t rc4[2] = {review, v.constraint};
      h = fnv_bytes(h, rc4, 8);
      h = fnv_bytes(h, mp, ml);
      const unsigned char sep = 0xff;
      h = fnv_bytes(h, &sep, 1);
      h = fnv_bytes(h, dp, dl);
      k.digest += h;
    }
    ++k.violations;
  }
}

}  // namespace cpu
}  // namespace gk

#ifndef GKCPU_TOUCH
namespace gk {
namespace cpu {
// the checker's own join indexes (gkcpu_build_joins), same layout as the
// engine's device indexes (engine.cc build_joins)
static std::vector<uint32_t> j_dir, j_ord;
static std::vector<uint64_t> j_hash;
}  // namespace cpu
}  // namespace gk

extern "C" {

size_t gkcpu_devargs_size() { return sizeof(gk::DevArgs); }

// Builds the join indexes of the engine's join plan on the host -- the key
// programs run by this interpreter per leaf, (hash, leaf row) sorted per
// (constraint, site) -- and points `args` (gk_debug_host_args, whose jleaf
// holds the plan's leaf rows) at them, so the checker's sweeps probe as the
// device does.  sites: gk_debug_join_plan's records.  Returns the number of
// (constraint, site) pairs left unindexed (a failed key program).
int gkcpu_build_joins(void* args, const uint64_t* sites, uint64_t nsites, int threads) {
  using namespace gk;
  DevArgs& A = *(DevArgs*)args;
  A.jdir = nullptr;
  A.jhash = nullptr;
  A.jord = nullptr;
  if (!nsites || !A.jleaf) return 0;
  cpu::j_dir.assign((size_t)(A.ncons ? A.ncons : 1) * JMAX_SITES * 4, 0);
  cpu::j_hash.clear();
  cpu::j_ord.clear();
  if (threads < 1) threads = 1;
  int unindexed = 0;
  for (uint64_t q = 0; q < nsites; ++q) {
    const uint64_t* sr = sites + 8 * q;
    const uint32_t ci = (uint32_t)sr[0], site = (uint32_t)sr[1], pc = (uint32_t)sr[2], stride = (uint32_t)sr[3];
    const uint64_t row0 = sr[4], n = sr[5], params = sr[6];
    if (sr[7] & 1) { ++unindexed; continue; }  // a path variable over an array: the site scans
    std::vector<uint64_t> keys(n * JKEYS_MAX, KH_NONE);
    std::atomic<uint64_t> next{0};
    auto work = [&]() {
      memcpy(&gk_args, args, sizeof(DevArgs));
      gk_args.jkeys = keys.data();
      gk_args.jdir = nullptr;
      for (;;) {
        const uint64_t i = next.fetch_add(1);
        if (i >= n) break;
        Lane L;
        L.hp = 0; L.bp = 0; L.ord = 0; L.ord_base = 0; L.fail = 0; L.reason = 0; L.en = 0; L.steps = 0; L.memo_ok = 0;
        for (int d = 0; d < MAXLOOP; ++d) { L.keepH[d] = 0; L.keepB[d] = 0; }
        L.rv = (uint32_t)i;
        L.cn = 0;
        cpu::run_program(L, pc, A.jleaf[row0 + i * stride], params);
        if (L.fail) keys[i * JKEYS_MAX] = KH_FAIL;
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; ++t) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
    uint32_t* dir = &cpu::j_dir[((size_t)ci * JMAX_SITES + site) * 4];
    dir[0] = (uint32_t)cpu::j_hash.size();
    std::vector<std::pair<uint64_t, uint32_t>> ent;
    bool failed = false;
    for (uint64_t i = 0; i < n && !failed; ++i) {
      const uint64_t* k = &keys[i * JKEYS_MAX];
      if (k[0] == KH_FAIL) { failed = true; break; }
      for (uint32_t j = 0; j < JKEYS_MAX && k[j] != KH_NONE; ++j) {
        bool dup = false;
        for (uint32_t h = 0; h < j; ++h) dup = dup || k[h] == k[j];
        if (!dup) ent.push_back({k[j], (uint32_t)(row0 + i * stride)});
      }
    }
    if (failed) { ++unindexed; continue; }
    std::stable_sort(ent.begin(), ent.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    for (auto& e : ent) { cpu::j_hash.push_back(e.first); cpu::j_ord.push_back(e.second); }
    dir[1] = (uint32_t)ent.size();
    dir[2] = 1;
  }
  if (cpu::j_hash.empty()) { cpu::j_hash.push_back(0); cpu::j_ord.push_back(0); }
  A.jdir = cpu::j_dir.data();
  A.jhash = cpu::j_hash.data();
  A.jord = cpu::j_ord.data();
  return unindexed;
}

// Evaluates reviews [lo, hi) of the staged batch described by `args` (host
// pointers, gk_debug_host_args) against every constraint on `threads` threads.
// out4 = [evals, violations, message bytes, flagged pairs]; returns seconds.
double gkcpu_sweep(const void* args, uint32_t lo, uint32_t hi, int threads, uint64_t* out4) {
  memcpy(&gk_args, args, sizeof(gk::DevArgs));
  if (hi > gk_args.nrev) hi = gk_args.nrev;
  if (lo > hi) lo = hi;
  const uint32_t ncons = gk_args.ncons;
  const void* shared_args = args;
  if (threads < 1) threads = 1;
  std::vector<gk::cpu::Counts> per(threads);
  std::atomic<uint32_t> next{lo};
  auto t0 = std::chrono::steady_clock::now();
  auto work = [&](int t) {
    gk::cpu::OutBufs ob;
    ob.bind(shared_args);
    std::vector<char> fbuf(1 << 16);
    gk::cpu::Counts& k = per[t];
    for (;;) {
      uint32_t a = next.fetch_add(256);
      if (a >= hi) break;
      uint32_t b = a + 256 < hi ? a + 256 : hi;
      for (uint32_t rp = a; rp < b; ++rp)
        for (uint32_t c = 0; c < ncons; ++c) gk::cpu::eval_pair(rp, c, k, fbuf.data(), (uint32_t)fbuf.size());
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t tot[4] = {0, 0, 0, 0};
  uint64_t dig = 0;
  for (auto& k : per) { tot[0] += k.evals; tot[1] += k.violations; tot[2] += k.msg_bytes; tot[3] += k.flagged; dig += k.digest; }
  gk::cpu::g_last_digest = dig;
  if (out4) memcpy(out4, tot, sizeof tot);
  return s;
}

// gkcpu_sweep plus out5[4] = the digest of every result row (Counts::digest)
double gkcpu_sweep_digest(const void* args, uint32_t lo, uint32_t hi, int threads, uint64_t* out5) {
  gk::cpu::g_digest = true;
  uint64_t o4[4];
  const double s = gkcpu_sweep(args, lo, hi, threads, o4);
  gk::cpu::g_digest = false;
  memcpy(out5, o4, sizeof o4);
  out5[4] = gk::cpu::g_last_digest;
  return s;
}

// The same row digest over a device evaluation's raw output (the formatted
// gk_viol records and their message + details bytes, as
// gk_results_copy_device_output returns them), so a GPU test can compare every
// row of a 1M-review sweep with gkcpu_sweep_digest.  Records of flagged
// reviews (VF_NOPRINT) are skipped as every consumer drops them; returns the
// digest, *nrows the rows hashed.
uint64_t gkcpu_rows_digest(const void* viols, uint64_t n, const uint8_t* bytes, uint64_t nbytes, int threads,
                           uint64_t* nrows) {
  const gk::Viol* V = (const gk::Viol*)viols;
  if (threads < 1) threads = 1;
  std::vector<uint64_t> dig(threads, 0), cnt(threads, 0);
  std::atomic<uint64_t> next{0};
  auto work = [&](int t) {
    for (;;) {
      const uint64_t a = next.fetch_add(65536);
      if (a >= n) break;
      const uint64_t b = a + 65536 < n ? a + 65536 : n;
      for (uint64_t i = a; i < b; ++i) {
        const gk::Viol& v = V[i];
        if (v.pad & gk::VF_NOPRINT) continue;
        if (v.msg_off + v.msg_len + v.det_len > nbytes) { dig[t] ^= 0x5bd1e995ull * (i + 1); continue; }
        uint64_t h = 1469598103934665603ull;
        const uint32_t rc4[2] = {v.review, v.constraint};
        h = gk::cpu::fnv_bytes(h, rc4, 8);
        h = gk::cpu::fnv_bytes(h, bytes + v.msg_off, v.msg_len);
        const unsigned char sep = 0xff;
        h = gk::cpu::fnv_bytes(h, &sep, 1);
        h = gk::cpu::fnv_bytes(h, bytes + v.msg_off + v.msg_len, v.det_len);
        dig[t] += h;
        ++cnt[t];
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  uint64_t d = 0, c = 0;
  for (int t = 0; t < threads; ++t) { d += dig[t]; c += cnt[t]; }
  if (nrows) *nrows = c;
  return d;
}

}  // extern "C"
#else
extern "C" {

// SURVEY 8(d) reference accounting for the roofline: evaluates reviews
// [lo, hi) against constraint `only` (or all when only < 0) and reports
// out5 = [document nodes referenced, distinct strings whose bytes were read,
// their bytes, violations, flagged pairs].  n_nodes / n_strings: the host
// store's sizes (gk_debug_store_sizes).
int gkcpu_referenced(const void* args, uint64_t n_nodes, uint64_t n_strings, uint32_t lo, uint32_t hi, int only,
                     int threads, uint64_t* out5, uint64_t* pc_hist) {
  if (pc_hist) threads = 1;  // pc_hist: executions per bytecode instruction (diagnostics)
  memcpy(&gk_args_touch, args, sizeof(gk_touch::DevArgs));
  auto& A = gk_args_touch;
  if (hi > A.nrev) hi = A.nrev;
  if (lo > hi) lo = hi;
  if (threads < 1) threads = 1;
  const size_t nwords = (size_t)(n_nodes + 63) / 64, swords = (size_t)(n_strings + 63) / 64;
  std::vector<std::vector<uint64_t>> nb(threads), sb(threads);
  std::vector<gk_touch::cpu::Counts> per(threads);
  std::atomic<uint32_t> next{lo};
  auto work = [&](int t) {
    gk_touch::cpu::OutBufs ob;
    ob.bind(args);
    nb[t].assign(nwords, 0);
    sb[t].assign(swords, 0);
    gkcpu_touch::node_bits = nb[t].data();
    gkcpu_touch::str_bits = sb[t].data();
    gkcpu_touch::pc_hist = pc_hist;
    std::vector<char> fbuf(1 << 16);
    auto& k = per[t];
    for (;;) {
      uint32_t a = next.fetch_add(256);
      if (a >= hi) break;
      uint32_t b = a + 256 < hi ? a + 256 : hi;
      for (uint32_t rp = a; rp < b; ++rp)
        for (uint32_t c = 0; c < A.ncons; ++c)
          if (only < 0 || (uint32_t)only == c) gk_touch::cpu::eval_pair(rp, c, k, fbuf.data(), (uint32_t)fbuf.size());
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  uint64_t nodes = 0, strs = 0, sbytes = 0;
  for (size_t w = 0; w < nwords; ++w) {
    uint64_t x = 0;
    for (int t = 0; t < threads; ++t) x |= nb[t][w];
    nodes += (uint64_t)__builtin_popcountll(x);
  }
  for (size_t w = 0; w < swords; ++w) {
    uint64_t x = 0;
    for (int t = 0; t < threads; ++t) x |= sb[t][w];
    while (x) {
      int bit = __builtin_ctzll(x);
      x &= x - 1;
      uint64_t sid = w * 64 + (uint64_t)bit;
      ++strs;
      sbytes += A.strs[sid].len;
    }
  }
  uint64_t viol = 0, flagged = 0;
  for (auto& k : per) { viol += k.violations; flagged += k.flagged; }
  uint64_t o[5] = {nodes, strs, sbytes, viol, flagged};
  memcpy(out5, o, sizeof o);
  return 0;
}

// the heap-word writes (by word index bucket) and lane-buffer bytes of the
// last gkcpu_referenced call on this thread (threads = 1)
int gkcpu_scratch_stats(uint64_t* out5, int reset) {
  for (int i = 0; i < 4; ++i) out5[i] = gkcpu_touch::heap_w[i];
  out5[4] = gkcpu_touch::buf_b;
  if (reset) {
    for (int i = 0; i < 4; ++i) gkcpu_touch::heap_w[i] = 0;
    gkcpu_touch::buf_b = 0;
  }
  return 0;
}

}  // extern "C"
#endif
