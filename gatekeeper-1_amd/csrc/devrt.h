// Device runtime of the MI355X audit engine: value model, document access,
// comparisons, builtins, printing, regex DFA, match stage, staged emission and
// the per-instruction semantics of the predicate bytecode.
//
// Shared verbatim by the two evaluation back ends so they cannot drift apart:
//   * kernels.hip  — the bytecode VM kernel (any compiled template), and
//   * jit.cc       — per-template kernels: the template's bytecode translated to
//                    straight-line HIP (registers become VGPR locals, constants
//                    become immediates) and compiled with hipRTC for gfx950; this
//                    header is embedded into the library and handed to hipRTC.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "common.h"

// Launch arguments: every kernel takes the DevArgs BY VALUE as its ONLY
// parameter, so they sit at the start of the dispatch's kernarg segment,
// immediately followed by the hidden (implicit) kernel arguments.  Device
// functions receive the implicit-argument pointer as an SGPR input (the
// kernarg segment pointer itself reads as null outside the kernel), so every
// helper reads the launch arguments at implicitarg_ptr - sizeof(DevArgs), with
// wave-uniform scalar loads.  Per-launch arguments: concurrent evaluations on
// different streams never share them (a __constant__ copy per code object is
// overwritten by the next launch of the same kernel).  Passing them by
// reference to non-inlined helpers would copy them into every lane's scratch.
// The host build of this runtime (oracle/cpuvm.cc) declares a variable of that
// name instead.
#ifndef GK_HOST
static_assert(sizeof(gk::DevArgs) % 8 == 0, "the hidden kernel arguments follow DevArgs at an 8-byte boundary");
#define gk_args                                                                                                     \
  (*(const __attribute__((address_space(4))) gk::DevArgs*)((const __attribute__((address_space(4))) char*)        \
                                                              __builtin_amdgcn_implicitarg_ptr() -                 \
                                                          sizeof(gk::DevArgs)))
#endif

// Reference accounting hooks (empty on the device): the CPU build of this
// runtime (oracle/cpuvm.cc) defines them to record which document nodes and
// which strings' bytes an evaluation references -- SURVEY 8(d)'s algorithmic
// bytes for the roofline are counted from that record.
#ifndef GK_TOUCH_NODE
#define GK_TOUCH_NODE(i) ((void)0)
#endif
#ifndef GK_TOUCH_STR
#define GK_TOUCH_STR(s) ((void)0)
#endif
// heap word / lane-buffer byte writes (the accounting build counts where they
// would land: LDS or the private segment)
#ifndef GK_HEAP_WRITE
#define GK_HEAP_WRITE(w) ((void)0)
#endif
#ifndef GK_BUF_WRITE
#define GK_BUF_WRITE(n) ((void)0)
#endif

namespace gk {

// GK_INLINE_HOT: the builtins template bodies call per container (startswith /
// endswith / contains, to_number, substring, literal-regex DFAs, integer
// arithmetic) are inlined at their call sites.  An out-of-line call makes the
// caller save and restore its live VGPRs in scratch, which dominates these
// kernels' memory traffic; the JIT enables it per template (jit.cc).
#ifndef GK_INLINE_HOT
#define GK_INLINE_HOT 0
#endif
#if GK_INLINE_HOT
#define GK_HOT __forceinline__
#else
#define GK_HOT
#endif
#ifndef GK_HCAP
#define GK_HCAP 128
#endif
#ifndef GK_BCAP
#define GK_BCAP 4096
#endif
constexpr int HCAP = GK_HCAP;  // heap words per lane (lists, big floats)
#ifndef GK_LDS_HWORDS
#define GK_LDS_HWORDS 0
#endif
#define GK_LDS_HWORDS_DEF GK_LDS_HWORDS
static_assert(GK_LDS_HWORDS < GK_HCAP, "LDS heap words must leave a private-segment tail");
constexpr int MAXLOOP = 16;    // loop nesting levels with per-iteration heap reclamation
// loop levels a kernel's programs use (the template JIT defines it from the
// program's deepest loop; audit_body clears only those watermarks)
#ifndef GK_MAXDEPTH
#define GK_MAXDEPTH MAXLOOP
#endif
static_assert(GK_MAXDEPTH >= 1 && GK_MAXDEPTH <= MAXLOOP, "GK_MAXDEPTH: 1..MAXLOOP loop levels");
constexpr int BCAP = GK_BCAP;  // byte buffer per lane (computed strings; an emission's bytes in transit)
// emission order key of a tuple (Viol.seq): (OP_ORD key << 8) | the lane's
// emission index; a lane past either limit goes to the CPU fallback
constexpr uint32_t EM_MAXIDX = 256, EM_MAXORD = 256;

// Wave-level primitives of the emission path.  The host build of this runtime
// (oracle/cpuvm.cc, GK_HOST) evaluates one lane at a time: a wave of one.
#ifdef GK_HOST
__device__ __forceinline__ uint64_t gk_ballot(bool p) { return p ? 1ull : 0ull; }
__device__ __forceinline__ uint32_t gk_lane_id() { return 0u; }
__device__ __forceinline__ uint32_t gk_lanes_below(uint64_t) { return 0u; }
#else
__device__ __forceinline__ uint64_t gk_ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t gk_lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
// set bits of m below this lane
__device__ __forceinline__ uint32_t gk_lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
#endif


// ------------------------------------------------------------------ values
__device__ __forceinline__ uint32_t vtag(uint64_t v) { return (uint32_t)(v >> 60); }
__device__ __forceinline__ uint64_t vpay(uint64_t v) { return v & 0x0fffffffffffffffull; }
__device__ __forceinline__ uint64_t mkv(uint32_t t, uint64_t p) { return ((uint64_t)t << 60) | (p & 0x0fffffffffffffffull); }
__device__ __forceinline__ uint64_t mkint(int64_t i) { return mkv(V_INT, (uint64_t)i & 0x0000ffffffffffffull); }
// an int that came out of arithmetic: OPA turns big.Float results back into
// numbers with Text('g', -1), so from 1e6 up they print in exponent form
// (put_intv); comparisons and intof ignore the flag
constexpr uint64_t INT_G = 1ull << 48;
__device__ __forceinline__ uint64_t mkint_g(int64_t i) { return mkint(i) | INT_G; }
__device__ __forceinline__ int64_t intof(uint64_t v) {
  uint64_t p = vpay(v) & 0x0000ffffffffffffull;
  return (p & 0x0000800000000000ull) ? (int64_t)(p | 0xffff000000000000ull) : (int64_t)p;
}
__device__ __forceinline__ uint32_t list_kind(uint64_t v) { return (uint32_t)((v >> 56) & 0xf); }
__device__ __forceinline__ uint64_t mklist(uint32_t kind, uint32_t off) { return mkv(V_LIST, ((uint64_t)kind << 56) | off); }
__device__ __forceinline__ uint32_t list_off(uint64_t v) { return (uint32_t)(v & 0xffffffffu); }
__device__ __forceinline__ uint64_t mkhstr(uint32_t off, uint32_t len) { return mkv(V_HSTR, ((uint64_t)off << 16) | len); }
__device__ __forceinline__ uint64_t mkslice(uint32_t sid, uint32_t st, uint32_t len) {
  return mkv(V_SLICE, ((uint64_t)sid << 28) | ((uint64_t)st << 14) | len);
}
__device__ __forceinline__ bool is_strv(uint64_t v) {
  uint32_t t = vtag(v);
  return t == V_STR || t == V_HSTR || t == V_SLICE || t == V_GSTR;
}
__device__ __forceinline__ bool is_numv(uint64_t v) { uint32_t t = vtag(v); return t == V_NUM || t == V_INT || t == V_BFN; }

// GK_LDS_SCALARS (template kernels, jit.cc): the lane's hot scalars (heap and
// buffer tops, failure word, emission count and order keys) live in LDS, one
// 32-bit slot per thread and field (gk_lds_scal[field][threadIdx.x]), instead
// of the lane's private segment.  Every helper reads and writes them, and the
// private segment is reached through a generic pointer that byte stores into
// the lane buffer may alias, so in scratch they were reloaded from memory
// after almost every helper.  Fields keep their names: LdsField converts.
#ifndef GK_LDS_SCALARS
#define GK_LDS_SCALARS 0
#endif
#if GK_LDS_SCALARS
constexpr int LDS_NSCAL = 9;
__shared__ uint32_t gk_lds_scal[LDS_NSCAL][256];
template <class T, int F>
struct LdsField {
  __device__ __forceinline__ operator T() const { return (T)gk_lds_scal[F][threadIdx.x]; }
  __device__ __forceinline__ LdsField& operator=(uint32_t v) { gk_lds_scal[F][threadIdx.x] = (T)v; return *this; }
  __device__ __forceinline__ LdsField& operator=(const LdsField& o) { return *this = (uint32_t)(T)o; }
  __device__ __forceinline__ LdsField& operator+=(uint32_t v) { return *this = (uint32_t)(T)*this + v; }
  __device__ __forceinline__ LdsField& operator-=(uint32_t v) { return *this = (uint32_t)(T)*this - v; }
  __device__ __forceinline__ LdsField& operator|=(uint32_t v) { return *this = (uint32_t)(T)*this | v; }
  __device__ __forceinline__ LdsField& operator++() { return *this += 1u; }
  __device__ __forceinline__ T operator++(int) { T o = *this; *this += 1u; return o; }
};
#define GK_LSCAL(T, name, F) LdsField<T, F> name
// the loop watermarks (keepH / keepB per loop level, read at every iteration)
// likewise: GK_MAXDEPTH levels x 2 x 256 threads x 2 B in LDS
__shared__ uint16_t gk_lds_keep[2][GK_MAXDEPTH][256];
template <int F>
struct LdsKeep {
  struct Ref {
    uint32_t d;
    __device__ __forceinline__ operator uint16_t() const { return gk_lds_keep[F][d][threadIdx.x]; }
    __device__ __forceinline__ Ref& operator=(uint32_t v) { gk_lds_keep[F][d][threadIdx.x] = (uint16_t)v; return *this; }
  };
  __device__ __forceinline__ Ref operator[](uint32_t d) const { return Ref{d < GK_MAXDEPTH ? d : 0u}; }
};
#define GK_LKEEP(name, F) LdsKeep<F> name
#else
#define GK_LSCAL(T, name, F) T name
#define GK_LKEEP(name, F) uint16_t name[MAXLOOP]
#endif

struct Lane {
  uint64_t H[HCAP - GK_LDS_HWORDS_DEF];  // heap words GK_LDS_HWORDS_DEF.. (the first ones are in LDS)
  char B[BCAP];
  GK_LSCAL(uint32_t, hp, 0);
  GK_LSCAL(uint32_t, bp, 1);
  GK_LSCAL(uint32_t, fail, 2);  // fail: 0 ok, RF_ERROR, RF_FALLBACK
  // emission order key (OP_ORD, fused rule bodies): emissions are numbered by
  // (key, emission index) at flush, which is the reference's evaluation order
  GK_LSCAL(uint16_t, ord, 3);
  GK_LSCAL(uint16_t, ord_base, 4);
  GK_LSCAL(uint32_t, reason, 5);
  // per loop depth: heap / byte watermarks that values escaping the loop pinned
  GK_LKEEP(keepH, 0);
  GK_LKEEP(keepB, 1);
  GK_LSCAL(uint32_t, en, 6);  // tuples this lane emitted (written straight to the output)
  uint32_t steps;
  GK_LSCAL(uint32_t, rv, 7);  // the review's index in the caller's batch (Viol.review)
  GK_LSCAL(uint32_t, cn, 8);  // the constraint (Viol.constraint)
  uint32_t memo_ok;  // VM memo slots holding a value (bit per slot)
  uint64_t memo_k0[MEMO_SLOTS], memo_k1[MEMO_SLOTS], memo_v[MEMO_SLOTS];
};

// A lane's state lives in private (scratch) memory.  Helpers take it through
// PLane&.  A template kernel may be compiled with GK_PRIV set to
// __attribute__((address_space(5))) (GKGPU_PRIV=1), so the compiler emits
// scratch_load/store with a 32-bit offset instead of flat accesses through a
// 64-bit generic pointer; the default is the generic address space (the VM
// kernel does not compile in address space 5 with this toolchain).
#ifndef GK_PRIV
#define GK_PRIV
#endif
typedef GK_PRIV Lane PLane;

// The first GK_LDS_HWORDS words of each lane's heap live in LDS (template and
// VM kernels; 0 = all in the private segment, as in the CPU build).  Lists and
// big floats are allocated by bumping L.hp and reclaimed per loop iteration,
// so the hot words are the low ones: list headers and the short argument lists
// sprintf and the set builtins build per container.  Layout: word w of thread t
// at gk_lds_heap[w][t], so a wavefront's access to one word touches 64
// consecutive 8-byte slots (no bank conflicts).  256 threads per block.
#if GK_LDS_HWORDS_DEF > 0
__shared__ uint64_t gk_lds_heap[GK_LDS_HWORDS_DEF][256];
__device__ __forceinline__ uint64_t hget(const PLane& L, uint32_t w) {
  return w < GK_LDS_HWORDS_DEF ? gk_lds_heap[w][threadIdx.x] : L.H[w - GK_LDS_HWORDS_DEF];
}
__device__ __forceinline__ void hset(PLane& L, uint32_t w, uint64_t v) {
  if (w < GK_LDS_HWORDS_DEF) gk_lds_heap[w][threadIdx.x] = v;
  else L.H[w - GK_LDS_HWORDS_DEF] = v;
}
#else
__device__ __forceinline__ uint64_t hget(const PLane& L, uint32_t w) { return L.H[w]; }
__device__ __forceinline__ void hset(PLane& L, uint32_t w, uint64_t v) { GK_HEAP_WRITE(w); L.H[w] = v; }
#endif

// ------------------------------------------------------------------ LDS stage
// Template kernels stage, per wavefront and at kernel entry, what every lane
// of the wave reads again and again (the wave evaluates ONE constraint):
//   GK_LDS_PARAMS  the constraint's parameters subtree (a node window of its
//                  document, MatchSpec.plo/pn), read by the lookups the JIT
//                  proves parameter-derived (jit.cc param_flow: vget_p,
//                  op_iter_next_p) from LDS instead of the node store;
//   GK_LDS_DFA     the byte-class-compressed DFAs of the regex patterns in
//                  those parameters (MatchSpec.stage_off), walked by re_run
//                  from LDS (two LDS reads per subject byte instead of a
//                  dependent global load).
// One area per wavefront of the 256-thread block (threadIdx.x >> 6).
#ifndef GK_LDS_PARAMS
#define GK_LDS_PARAMS 0
#endif
#ifndef GK_LDS_DFA
#define GK_LDS_DFA 0
#endif
constexpr uint32_t LDS_PCAP = 64;          // parameter nodes per wave (1 KB)
constexpr uint32_t LDS_DFA_BYTES = 1024;   // compressed DFA bytes per wave (engine.cc rebuild_stage)
constexpr uint32_t LDS_DFA_MAX = 4;        // DFAs per wave
#if GK_LDS_PARAMS
__shared__ Node gk_lds_pnodes[4][LDS_PCAP];
__device__ __forceinline__ Node pnode(uint32_t idx, uint32_t plo, uint32_t pn) {
  GK_TOUCH_NODE(idx);
  const uint32_t off = idx - plo;
  if (off < pn) return gk_lds_pnodes[threadIdx.x >> 6][off];
  return gk_args.nodes[idx];
}
#endif
#if GK_LDS_DFA
__shared__ uint32_t gk_lds_dfa[4][LDS_DFA_BYTES / 4];
// per DFA: pattern sid, byte offset in the wave's area, nst | ncls << 16, start | sens << 16
__shared__ uint32_t gk_lds_dfadir[4][1 + 4 * LDS_DFA_MAX];
#endif

// GK_LDS_MEMO (template kernels, jit.cc): a direct-mapped cache in front of
// the cross-lane memo (gm_get / gm_put below), GK_LDS_MEMO entries of
// (key0, key1, value, check) per wavefront.  A pure call's arguments repeat
// within a wave -- K8sContainerLimits' canonify_cpu("2000m") at every
// container of the 64 Pods -- and each probe of the global table is a
// dependent L2 round trip; the wave's own copy answers in LDS.  Entries are
// guarded by the same check word as the global table, so racing lanes of
// the wave and collisions read as misses.  Cleared at wave start.
#ifndef GK_LDS_MEMO
#define GK_LDS_MEMO 0
#endif
static_assert((GK_LDS_MEMO & (GK_LDS_MEMO - 1)) == 0, "GK_LDS_MEMO: a power of two");
#if GK_LDS_MEMO && !defined(GK_HOST)
__shared__ uint64_t gk_lds_memo[4][GK_LDS_MEMO][4];
#endif
#ifndef GK_HOST
__shared__ unsigned long long gk_lds_chunk[4][6];  // per wave: tuple-slot chunk (slot_reserve), byte chunk (bytes_reserve)
__shared__ uint32_t gk_lds_bscan[4];                // per wave: bytes_reserve's running sum
#endif

// copies this wave's stage (all 64 lanes, wave-uniform m); the wave's own
// lanes read it after the wave barrier
__device__ __forceinline__ void stage_wave(const MatchSpec& m, uint32_t lane) {
#if GK_LDS_PARAMS || GK_LDS_DFA || (GK_LDS_MEMO && !defined(GK_HOST))
  const uint32_t wv = threadIdx.x >> 6;
#endif
#if GK_LDS_MEMO && !defined(GK_HOST)
  for (uint32_t k = lane; k < GK_LDS_MEMO * 4u; k += 64) (&gk_lds_memo[wv][0][0])[k] = 0;
#endif
#ifndef GK_HOST
  if (lane < 6) gk_lds_chunk[threadIdx.x >> 6][lane] = 0;  // no chunks yet (devrt.h slot_reserve, bytes_reserve)
  if (lane == 0) gk_lds_bscan[threadIdx.x >> 6] = 0;
#endif
#if GK_LDS_PARAMS
  const uint32_t pn = m.pn <= LDS_PCAP ? m.pn : 0;
  for (uint32_t k = lane; k < pn; k += 64) gk_lds_pnodes[wv][k] = gk_args.nodes[m.plo + k];
#endif
#if GK_LDS_DFA
  uint32_t nd = 0;
  if (m.stage_off != NO_ID) {
    const uint32_t* r = gk_args.stage + m.stage_off;
    nd = r[0] < LDS_DFA_MAX ? r[0] : LDS_DFA_MAX;
    uint32_t at = 0;
    for (uint32_t i = 0; i < nd; ++i) {
      const uint32_t* e = r + 1 + 5 * i;
      const uint32_t words = (e[2] + 3) / 4;
      if (at + words * 4 > LDS_DFA_BYTES) { nd = i; break; }
      for (uint32_t k = lane; k < words; k += 64) gk_lds_dfa[wv][at / 4 + k] = gk_args.dfa_c[e[1] + k];
      if (lane == 0) {
        gk_lds_dfadir[wv][1 + 4 * i] = e[0];
        gk_lds_dfadir[wv][2 + 4 * i] = at;
        gk_lds_dfadir[wv][3 + 4 * i] = e[3];
        gk_lds_dfadir[wv][4 + 4 * i] = e[4];
      }
      at += words * 4;
    }
  }
  if (lane == 0) gk_lds_dfadir[wv][0] = nd;
#endif
#ifndef GK_HOST
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
}

// a heap-resident value (must survive a loop's per-iteration heap reset when it
// escapes to a register that outlives the iteration)
__device__ __forceinline__ bool heap_val(uint64_t v) {
  uint32_t t = v >> 60;
  return t == V_LIST || t == V_BFN || t == V_HSTR || t == V_FMT;
}
__device__ __forceinline__ void pin_escape(PLane& L, uint32_t range) {
  uint32_t lo = range & 0xff, hi = (range >> 8) & 0xff;
  for (uint32_t d = lo; d <= hi && d < GK_MAXDEPTH; ++d) {
    if (L.keepH[d] < L.hp) L.keepH[d] = (uint16_t)L.hp;
    if (L.keepB[d] < L.bp) L.keepB[d] = (uint16_t)L.bp;
  }
}

__device__ __forceinline__ void lane_fallback(PLane& L, uint32_t reason) {
  if (!L.fail) { L.fail = RF_FALLBACK; L.reason = reason; }
}
__device__ __forceinline__ void lane_error(PLane& L) {
  if (!L.fail) { L.fail = RF_ERROR; L.reason = 0; }
}

// the value of node idx whose record n the caller has already loaded (an
// object scan reads whole member records: no second round trip)
__device__ __forceinline__ uint64_t nodeval_of(const Node& n, uint32_t idx) {
  GK_TOUCH_NODE(idx);
  switch (n.type) {
    case NT_NULL: return mkv(V_NULL, 0);
    case NT_FALSE: return mkv(V_BOOL, 0);
    case NT_TRUE: return mkv(V_BOOL, 1);
    case NT_NUM: return mkv(V_NUM, n.val);
    case NT_STR: return mkv(V_STR, n.val);
    case NT_ARR: case NT_OBJ: return mkv(V_NODE, idx);
  }
  return mkv(V_UNDEF, 0);
}
__device__ __forceinline__ uint64_t nodeval(uint32_t idx) {
  GK_TOUCH_NODE(idx);
  const Node& n = gk_args.nodes[idx];
  switch (n.type) {
    case NT_NULL: return mkv(V_NULL, 0);
    case NT_FALSE: return mkv(V_BOOL, 0);
    case NT_TRUE: return mkv(V_BOOL, 1);
    case NT_NUM: return mkv(V_NUM, n.val);
    case NT_STR: return mkv(V_STR, n.val);
    case NT_ARR: case NT_OBJ: return mkv(V_NODE, idx);
  }
  return mkv(V_UNDEF, 0);
}

// string bytes of a string value
struct SView { const char* p; uint32_t n; };
__device__ __forceinline__ SView sview(const PLane& L, uint64_t v) {
  uint32_t t = vtag(v);
  if (t == V_STR) { GK_TOUCH_STR((uint32_t)vpay(v)); const StrEnt& s = gk_args.strs[(uint32_t)vpay(v)]; return SView{(const char*)gk_args.pool + s.off, s.len}; }
  if (t == V_HSTR) { uint64_t p = vpay(v); return SView{L.B + (uint32_t)(p >> 16), (uint32_t)(p & 0xffff)}; }
  if (t == V_GSTR) { uint64_t p = vpay(v); return SView{gk_args.mstr + (p >> 20), (uint32_t)(p & 0xfffff)}; }
  if (t == V_SLICE) {
    uint64_t p = vpay(v);
    GK_TOUCH_STR((uint32_t)(p >> 28));
    const StrEnt& s = gk_args.strs[(uint32_t)(p >> 28)];
    return SView{(const char*)gk_args.pool + s.off + (uint32_t)((p >> 14) & 0x3fff), (uint32_t)(p & 0x3fff)};
  }
  return SView{nullptr, 0};
}
__device__ __forceinline__ int bytes_cmp(SView a, SView b) {
  uint32_t n = a.n < b.n ? a.n : b.n;
  for (uint32_t i = 0; i < n; ++i) {
    unsigned char x = (unsigned char)a.p[i], y = (unsigned char)b.p[i];
    if (x != y) return x < y ? -1 : 1;
  }
  return a.n == b.n ? 0 : (a.n < b.n ? -1 : 1);
}

// ------------------------------------------------------------------ numbers
// exact 64-bit-mantissa big-float view of a numeric value; returns false if unavailable
struct BF { uint64_t m; int32_t e; bool neg; bool zero; };
__device__ bool num_bf(const PLane& L, uint64_t v, BF& out) {
  uint32_t t = vtag(v);
  if (t == V_NUM) {
    const NumEnt& n = gk_args.nums[(uint32_t)vpay(v)];
    if (!(n.flags & NF_BF_OK)) return false;
    out.m = n.mant; out.e = n.exp; out.neg = n.neg != 0; out.zero = n.mant == 0;
    return true;
  }
  if (t == V_INT) {
    int64_t i = intof(v);
    out.neg = i < 0;
    uint64_t a = out.neg ? (uint64_t)(-i) : (uint64_t)i;
    out.zero = a == 0;
    if (out.zero) { out.m = 0; out.e = 0; return true; }
    int lz = __builtin_clzll(a);
    out.m = a << lz;
    out.e = -lz;
    return true;
  }
  if (t == V_BFN) {
    uint32_t o = (uint32_t)vpay(v);
    out.m = hget(L, o);
    uint64_t w = hget(L, o + 1);
    out.e = (int32_t)(uint32_t)w;
    out.neg = (w >> 32) & 1;
    out.zero = out.m == 0;
    return true;
  }
  return false;
}
__device__ int bf_cmp(const BF& a, const BF& b) {
  if (a.zero && b.zero) return 0;
  if (a.zero) return b.neg ? 1 : -1;
  if (b.zero) return a.neg ? -1 : 1;
  if (a.neg != b.neg) return a.neg ? -1 : 1;
  int mag;
  if (a.e != b.e) mag = a.e < b.e ? -1 : 1;
  else mag = a.m == b.m ? 0 : (a.m < b.m ? -1 : 1);
  return a.neg ? -mag : mag;
}
// integer view: true if the value is an exact integer representable in int64
__device__ bool num_int(const PLane& L, uint64_t v, int64_t& out) {
  uint32_t t = vtag(v);
  if (t == V_INT) { out = intof(v); return true; }
  if (t == V_NUM) {
    const NumEnt& n = gk_args.nums[(uint32_t)vpay(v)];
    if (n.flags & NF_INT64) { out = n.i; return true; }
    BF b;
    if (!num_bf(L, v, b)) return false;
    if (b.zero) { out = 0; return true; }
    if (b.e >= 0 || b.e < -63) return false;
    uint64_t sh = (uint64_t)(-b.e);
    if (b.m & ((1ull << sh) - 1)) return false;
    uint64_t mag = b.m >> sh;
    if (mag > (1ull << 62)) return false;
    out = b.neg ? -(int64_t)mag : (int64_t)mag;
    return true;
  }
  if (t == V_BFN) {
    BF b;
    num_bf(L, v, b);
    if (b.zero) { out = 0; return true; }
    if (b.e >= 0 || b.e < -63) return false;
    uint64_t sh = (uint64_t)(-b.e);
    if (b.m & ((1ull << sh) - 1)) return false;
    uint64_t mag = b.m >> sh;
    if (mag > (1ull << 62)) return false;
    out = b.neg ? -(int64_t)mag : (int64_t)mag;
    return true;
  }
  return false;
}
__device__ uint64_t heap_bf(PLane& L, const BF& b) {
  if (L.hp + 2 > HCAP) { lane_fallback(L, FB_HEAP); return mkv(V_UNDEF, 0); }
  uint32_t o = L.hp;
  L.hp += 2;
  hset(L, o, b.zero ? 0 : b.m);
  hset(L, o + 1, (uint64_t)(uint32_t)b.e | ((uint64_t)(b.neg ? 1 : 0) << 32));
  return mkv(V_BFN, o);
}
// big.Float Mul at prec 64, ToNearestEven
__device__ BF bf_mul(const BF& a, const BF& b) {
  BF r;
  r.neg = a.neg != b.neg;
  if (a.zero || b.zero) { r.zero = true; r.m = 0; r.e = 0; r.neg = false; return r; }
  r.zero = false;
  uint64_t lo = a.m * b.m;
  uint64_t hi = __umul64hi(a.m, b.m);
  int32_t e = a.e + b.e;
  // product in [2^126, 2^128): normalize hi to have top bit set
  uint64_t m;
  uint64_t rest;  // bits shifted out (as a 64-bit fraction, msb = half)
  if (hi >> 63) { m = hi; rest = lo; e += 64; }
  else { m = (hi << 1) | (lo >> 63); rest = lo << 1; e += 63; }
  bool half = rest >> 63;
  bool sticky = (rest << 1) != 0;
  if (half && (sticky || (m & 1))) {
    ++m;
    if (m == 0) { m = 1ull << 63; ++e; }
  }
  r.m = m;
  r.e = e;
  return r;
}

// ------------------------------------------------------------------ lists
__device__ __forceinline__ uint32_t list_len(const PLane& L, uint64_t v) { return (uint32_t)hget(L, list_off(v)); }
__device__ __forceinline__ uint64_t list_at(const PLane& L, uint64_t v, uint32_t i) { return hget(L, list_off(v) + 2 + i); }

__device__ __forceinline__ uint64_t list_new(PLane& L, uint32_t kind, uint32_t cap) {
  if (L.hp + 2 + cap > HCAP) { lane_fallback(L, FB_HEAP); return mkv(V_UNDEF, 0); }
  uint32_t o = L.hp;
  hset(L, o, 0);
  hset(L, o + 1, cap);
  L.hp += 2 + cap;
  return mklist(kind, o);
}

// value type ordering class (ast/compare.go sortOrder)
__device__ __forceinline__ int tclass(uint64_t v) {
  switch (vtag(v)) {
    case V_NULL: return 1;
    case V_BOOL: return 2;
    case V_NUM: case V_INT: case V_BFN: return 3;
    case V_STR: case V_HSTR: case V_SLICE: case V_GSTR: return 4;
    case V_NODE: GK_TOUCH_NODE((uint32_t)vpay(v)); return gk_args.nodes[(uint32_t)vpay(v)].type == NT_ARR ? 7 : 8;
    case V_LIST: case V_GLIST: { uint32_t k = list_kind(v); return k == LK_ARR ? 7 : k == LK_OBJ ? 8 : 9; }
    case V_ROW: return 8;
    case V_ROWS: return 7;
  }
  return 0;
}

// ------------------------------------------------------------------ path columns
// A columnar staged batch (colstore.cc) holds the paths its programs read as
// value columns: an object is V_ROW(view, row) -- its members are the view's
// slots, found by (view, key) in a small hash -- and an array V_ROWS(table,
// first row, length) of element-table rows.  Objects read whole (iterated,
// counted, compared, printed) stay document nodes (CW_NODE).
__device__ __forceinline__ uint32_t cv_find(uint32_t view, uint32_t key) {
  const uint32_t mask = gk_args.cv_hmask;
  uint32_t i = cv_hash_of(view, key) & mask;
  for (uint32_t p = 0; p <= mask; ++p, i = (i + 1) & mask) {
    const CvHash e = gk_args.cv_hash[i];
    if (e.view == view && e.key == key) return e.slot;
    if (e.view == NO_ID) return NO_ID;
  }
  return NO_ID;
}
__device__ __forceinline__ uint32_t row_view(uint64_t v) { return (uint32_t)(vpay(v) >> 40) & 0xfffu; }
__device__ __forceinline__ uint64_t row_row(uint64_t v) { return vpay(v) & ((1ull << 40) - 1); }
__device__ __forceinline__ uint32_t rows_tab(uint64_t v) { return (uint32_t)(vpay(v) >> 48) & 0xfffu; }
__device__ __forceinline__ uint32_t rows_first(uint64_t v) { return (uint32_t)(vpay(v) >> 16); }
__device__ __forceinline__ uint32_t rows_len(uint64_t v) { return (uint32_t)(vpay(v) & 0xffffu); }
// the value of slot `slot` at `row`
__device__ __forceinline__ uint64_t cv_value(uint32_t slot, uint64_t row) {
  const CvSlot sl = gk_args.cv_slots[slot];
  const uint32_t w = (sl.flags & CVS_BYTES) ? cv_byte_word(gk_args.cv_bytes[(uint64_t)sl.col + row])
                                            : gk_args.cv_words[(uint64_t)sl.col + row];
  const uint32_t p = w & CW_PAY;
  switch (w >> CW_SHIFT) {
    case CW_STR: return mkv(V_STR, p);
    case CW_NUM: return mkv(V_NUM, p);
    case CW_LIT: return p == 0 ? mkv(V_NULL, 0) : mkv(V_BOOL, p == 2 ? 1 : 0);
    case CW_OBJ: return mkv(V_ROW, ((uint64_t)sl.view << 40) | row);
    case CW_ARR:
      return mkv(V_ROWS, ((uint64_t)sl.tab << 48) | ((uint64_t)p << 16) | gk_args.cv_words[(uint64_t)sl.lencol + row]);
    case CW_NODE: return nodeval(p);
  }
  return mkv(V_UNDEF, 0);
}
// element i of a V_ROWS array
__device__ __forceinline__ uint64_t rows_at(uint64_t v, uint32_t i) {
  return cv_value(gk_args.cv_tabs[rows_tab(v)], (uint64_t)rows_first(v) + i);
}

// a list copied out at emission (gval_copy), read by the size / format passes
__device__ __forceinline__ const uint64_t* glist_words(uint64_t v) {
  return (const uint64_t*)gk_args.ebytes + list_off(v);
}

// collection view helpers (NODE arrays/objects and heap lists)
__device__ uint32_t coll_len(const PLane& L, uint64_t v) {
  if (vtag(v) == V_NODE) { GK_TOUCH_NODE((uint32_t)vpay(v)); return gk_args.nodes[(uint32_t)vpay(v)].n; }
  if (vtag(v) == V_ROWS) return rows_len(v);
  if (vtag(v) == V_ROW) {  // the staging keeps objects read as collections as nodes: not reached
    PLane& M = const_cast<PLane&>(L);
    if (!M.fail) { M.fail = RF_FALLBACK; M.reason = FB_UNSUPPORTED; }
    return 0;
  }
  if (vtag(v) == V_LIST) { uint32_t n = list_len(L, v); return list_kind(v) == LK_OBJ ? n / 2 : n; }
  if (vtag(v) == V_GLIST) { uint32_t n = (uint32_t)glist_words(v)[0]; return list_kind(v) == LK_OBJ ? n / 2 : n; }
  return 0;
}
// i-th (key, value) of a collection
__device__ void coll_at(const PLane& L, uint64_t v, uint32_t i, uint64_t& k, uint64_t& val) {
  if (vtag(v) == V_ROWS) { val = rows_at(v, i); k = mkint(i); return; }
  if (vtag(v) == V_ROW) { k = val = mkv(V_UNDEF, 0); return; }  // (coll_len flagged the lane)
  if (vtag(v) == V_NODE) {
    const Node& n = gk_args.nodes[(uint32_t)vpay(v)];
    uint32_t c = n.first + i;
    val = nodeval(c);
    k = n.type == NT_OBJ ? mkv(V_STR, gk_args.nodes[c].key) : mkint(i);
    return;
  }
  uint32_t kind = list_kind(v);
  if (vtag(v) == V_GLIST) {
    const uint64_t* w = glist_words(v) + 2;
    if (kind == LK_OBJ) { k = w[2 * i]; val = w[2 * i + 1]; return; }
    val = w[i];
    k = kind == LK_SET ? val : mkint(i);
    return;
  }
  if (kind == LK_OBJ) { k = list_at(L, v, 2 * i); val = list_at(L, v, 2 * i + 1); return; }
  val = list_at(L, v, i);
  k = kind == LK_SET ? val : mkint(i);
}

// scalar compare within one type class (1..4); 2 = undecidable (fallback set)
__device__ int scmp(PLane& L, uint64_t a, uint64_t b, int cls) {
  switch (cls) {
    case 1: return 0;
    case 2: { uint64_t x = vpay(a), y = vpay(b); return x == y ? 0 : (x < y ? -1 : 1); }
    case 3: {
      if (vtag(a) == V_NUM && vtag(b) == V_NUM && vpay(a) == vpay(b)) return 0;
      BF x, y;
      if (!num_bf(L, a, x) || !num_bf(L, b, y)) { lane_fallback(L, FB_NUMBER); return 2; }
      return bf_cmp(x, y);
    }
    case 4: {
      if (vtag(a) == V_STR && vtag(b) == V_STR && vpay(a) == vpay(b)) return 0;
      return bytes_cmp(sview(L, a), sview(L, b));
    }
  }
  return 2;
}

// element comparison inside a composite: scalars, or identical document nodes;
// anything deeper is served by the CPU fallback
__device__ int ecmp(PLane& L, uint64_t a, uint64_t b) {
  int ca = tclass(a), cb = tclass(b);
  if (ca != cb) return ca < cb ? -1 : 1;
  if (ca <= 4) return scmp(L, a, b, ca);
  if (vtag(a) == V_NODE && vtag(b) == V_NODE && vpay(a) == vpay(b)) return 0;
  if (vtag(a) >= V_ROW && a == b) return 0;
  if (vtag(a) == V_ROW || vtag(b) == V_ROW) { lane_fallback(L, FB_DEEP_EQ); return 2; }
  if (coll_len(L, a) == 0 && coll_len(L, b) == 0) return 0;
  lane_fallback(L, FB_DEEP_EQ);
  return 2;
}

// ast.Compare: -1/0/1; 3 = "not equal, order undefined here"; 2 = undecidable
__device__ int vcmp(PLane& L, uint64_t a, uint64_t b) {
  int ca = tclass(a), cb = tclass(b);
  if (ca != cb) return ca < cb ? -1 : 1;
  if (ca <= 4) return scmp(L, a, b, ca);
  if (vtag(a) == V_NODE && vtag(b) == V_NODE && vpay(a) == vpay(b)) return 0;
  if (vtag(a) >= V_ROW && a == b) return 0;
  if (vtag(a) == V_ROW || vtag(b) == V_ROW) { lane_fallback(L, FB_DEEP_EQ); return 2; }
  uint32_t na = coll_len(L, a), nb = coll_len(L, b);
  if (ca == 7) {
    uint32_t n = na < nb ? na : nb;
    for (uint32_t i = 0; i < n; ++i) {
      uint64_t k1, v1, k2, v2;
      coll_at(L, a, i, k1, v1);
      coll_at(L, b, i, k2, v2);
      int c = ecmp(L, v1, v2);
      if (c != 0) return c;
    }
    return na == nb ? 0 : (na < nb ? -1 : 1);
  }
  if (na != nb) return 3;
  // objects / sets of equal size: equal iff every member of a is in b
  for (uint32_t i = 0; i < na; ++i) {
    uint64_t k1, v1;
    coll_at(L, a, i, k1, v1);
    bool found = false;
    for (uint32_t j = 0; j < nb && !found; ++j) {
      uint64_t k2, v2;
      coll_at(L, b, j, k2, v2);
      int c = ecmp(L, k1, k2);
      if (c == 2) return 2;
      if (c != 0) continue;
      if (ca == 9) { found = true; break; }
      int d = ecmp(L, v1, v2);
      if (d == 2) return 2;
      if (d != 0) return 3;
      found = true;
    }
    if (!found) return 3;
  }
  return 0;
}

__device__ bool veq(PLane& L, uint64_t a, uint64_t b) {
  if (a == b) {
    uint32_t t = vtag(a);
    if (t != V_HSTR && t != V_BFN) return true;
  }
  if (is_strv(a) && is_strv(b)) {
    // interned strings: equal bytes <=> equal id; otherwise lengths first
    if (vtag(a) == V_STR && vtag(b) == V_STR) return false;
    SView x = sview(L, a), y = sview(L, b);
    if (x.n != y.n) return false;
    for (uint32_t i = 0; i < x.n; ++i) if (x.p[i] != y.p[i]) return false;
    return true;
  }
  int c = vcmp(L, a, b);
  return c == 0;
}

__device__ bool list_contains(PLane& L, uint64_t l, uint64_t v) {
  uint32_t n = list_len(L, l);
  for (uint32_t i = 0; i < n; ++i) if (veq(L, list_at(L, l, i), v)) return true;
  return false;
}
// append (sets dedupe); may relocate the list to the heap top when full
__device__ __noinline__ uint64_t list_add_slow(PLane& L, uint64_t l, uint64_t v) {
  if (vtag(l) != V_LIST) return l;
  if (list_kind(l) == LK_SET && list_contains(L, l, v)) return l;
  uint32_t o = list_off(l);
  uint32_t n = (uint32_t)hget(L, o), cap = (uint32_t)hget(L, o + 1);
  if (n == cap) {
    // grow: move to top of heap if this list is the last allocation, else copy
    uint32_t ncap = cap < 4 ? 8 : cap * 2;
    if (o + 2 + cap == L.hp) {
      if (o + 2 + ncap > HCAP) { lane_fallback(L, FB_HEAP); return l; }
      L.hp = o + 2 + ncap;
      hset(L, o + 1, ncap);
    } else {
      if (L.hp + 2 + ncap > HCAP) { lane_fallback(L, FB_HEAP); return l; }
      uint32_t no = L.hp;
      L.hp += 2 + ncap;
      for (uint32_t i = 0; i < n + 2; ++i) hset(L, no + i, hget(L, o + i));
      hset(L, no + 1, ncap);
      o = no;
      l = mklist(list_kind(l), o);
    }
  }
  hset(L, o + 2 + n, v);
  hset(L, o, n + 1);
  return l;
}
// Identity-decidable equality: 1 equal, 0 different, -1 undecided (needs veq).
// Interned strings are equal iff their ids are; booleans and nulls by bits;
// plain ints by value (the INT_G print flag does not take part).
__device__ __forceinline__ int id_eq(uint64_t a, uint64_t b) {
  if (a == b) { uint32_t t = vtag(a); return (t == V_STR || t == V_BOOL || t == V_NULL || t == V_INT) ? 1 : -1; }
  uint32_t ta = vtag(a), tb = vtag(b);
  if (ta != tb) return -1;
  if (ta == V_STR || ta == V_BOOL) return 0;
  if (ta == V_INT) return intof(a) == intof(b) ? 1 : 0;
  return -1;
}
// append fast path, inlined: AMDGPU calls save and restore the caller's live
// registers in scratch.  Arrays / objects with room append; a set with room
// appends after an inline duplicate scan when every member compares by
// identity (interned strings, booleans, ints: the set-comprehension case).
__device__ __forceinline__ uint64_t list_add(PLane& L, uint64_t l, uint64_t v) {
  if (vtag(l) == V_LIST) {
    uint32_t o = list_off(l);
    uint32_t n = (uint32_t)hget(L, o), cap = (uint32_t)hget(L, o + 1);
    if (n < cap) {
      if (list_kind(l) == LK_SET) {
        int found = 0;
        for (uint32_t i = 0; i < n && found == 0; ++i) found = id_eq(hget(L, o + 2 + i), v);
        if (found == 1) return l;
        if (found < 0) return list_add_slow(L, l, v);
      }
      hset(L, o + 2 + n, v);
      hset(L, o, n + 1);
      return l;
    }
  }
  return list_add_slow(L, l, v);
}

// ------------------------------------------------------------------ get
// a member / element of a column value: an object's member by interned key
// (a computed key string has no id to look up: CPU fallback), an array's
// element by index
__device__ __noinline__ uint64_t row_get_slow(PLane& L, uint64_t c, uint64_t key) {
  if (vtag(c) == V_ROW) {
    if (is_strv(key)) lane_fallback(L, FB_UNSUPPORTED);
    return mkv(V_UNDEF, 0);
  }
  if (!is_numv(key)) return mkv(V_UNDEF, 0);
  int64_t i;
  if (!num_int(L, key, i) || i < 0 || i >= (int64_t)rows_len(c)) return mkv(V_UNDEF, 0);
  return rows_at(c, (uint32_t)i);
}
__device__ __forceinline__ uint64_t row_get(PLane& L, uint64_t c, uint64_t key) {
  if (vtag(c) == V_ROW && vtag(key) == V_STR) {
    const uint32_t view = row_view(c);
    const uint32_t slot = cv_find(view, (uint32_t)vpay(key));
    if (slot != NO_ID) return cv_value(slot, row_row(c));
    // a key the batch never has at this path: undefined where the view holds
    // every key (the analysis gave the program's constant keys slots)
    if (!(gk_args.cv_views[view] & CV_COMPLETE)) lane_fallback(L, FB_UNSUPPORTED);
    return mkv(V_UNDEF, 0);
  }
  return row_get_slow(L, c, key);
}

__device__ __noinline__ uint64_t vget_slow(PLane& L, uint64_t c, uint64_t key) {
  uint32_t t = vtag(c);
  if (t >= V_ROW) return row_get(L, c, key);
  if (t == V_NODE) {
    GK_TOUCH_NODE((uint32_t)vpay(c));
    const Node& n = gk_args.nodes[(uint32_t)vpay(c)];
    if (n.flags & 1) { lane_fallback(L, FB_UNSUPPORTED); return mkv(V_UNDEF, 0); }
    if (n.type == NT_OBJ) {
      uint32_t kt = vtag(key);
      if (kt == V_STR) {
        uint32_t id = (uint32_t)vpay(key);
        for (uint32_t i = 0; i < n.n; ++i) if (gk_args.nodes[n.first + i].key == id) return nodeval(n.first + i);
        return mkv(V_UNDEF, 0);
      }
      if (kt == V_HSTR || kt == V_SLICE || kt == V_GSTR) {
        SView kv = sview(L, key);
        for (uint32_t i = 0; i < n.n; ++i) {
          const StrEnt& s = gk_args.strs[gk_args.nodes[n.first + i].key];
          if (bytes_cmp(kv, SView{(const char*)gk_args.pool + s.off, s.len}) == 0) return nodeval(n.first + i);
        }
      }
      return mkv(V_UNDEF, 0);
    }
    if (n.type == NT_ARR) {
      if (!is_numv(key)) return mkv(V_UNDEF, 0);
      int64_t i;
      if (!num_int(L, key, i)) return mkv(V_UNDEF, 0);
      if (i < 0 || i >= n.n) return mkv(V_UNDEF, 0);
      return nodeval(n.first + (uint32_t)i);
    }
    return mkv(V_UNDEF, 0);
  }
  if (t == V_LIST) {
    uint32_t kind = list_kind(c);
    uint32_t n = list_len(L, c);
    if (kind == LK_SET) return list_contains(L, c, key) ? key : mkv(V_UNDEF, 0);
    if (kind == LK_ARR) {
      if (!is_numv(key)) return mkv(V_UNDEF, 0);
      int64_t i;
      if (!num_int(L, key, i) || i < 0 || i >= n) return mkv(V_UNDEF, 0);
      return list_at(L, c, (uint32_t)i);
    }
    for (uint32_t i = 0; i + 1 < n; i += 2) if (veq(L, list_at(L, c, i), key)) return list_at(L, c, i + 1);
    return mkv(V_UNDEF, 0);
  }
  return mkv(V_UNDEF, 0);
}
// Inlined fast path of vget for the common document lookups (object member by
// interned key, array element by small int), and for containers that cannot
// be indexed at all (scalars, undefined: undefined).  Everything else,
// including fallback-flagged nodes, goes through vget_slow: an out-of-line
// call costs the caller a save/restore of its live registers in scratch.
__device__ __forceinline__ uint64_t vget(PLane& L, uint64_t c, uint64_t key) {
  if (vtag(c) >= V_ROW) return row_get(L, c, key);
  if (vtag(c) != V_NODE && vtag(c) != V_LIST) return mkv(V_UNDEF, 0);
  if (vtag(c) == V_NODE) {
    GK_TOUCH_NODE((uint32_t)vpay(c));
    const Node n = gk_args.nodes[(uint32_t)vpay(c)];
    if (!(n.flags & 1)) {
      uint32_t kt = vtag(key);
      if (n.type == NT_OBJ && kt == V_STR) {
        uint32_t id = (uint32_t)vpay(key);
        // whole member records: the match's value needs no second load
        for (uint32_t i = 0; i < n.n; ++i) {
          const Node m = gk_args.nodes[n.first + i];
          if (m.key == id) return nodeval_of(m, n.first + i);
        }
        return mkv(V_UNDEF, 0);
      }
      if (n.type == NT_ARR && kt == V_INT) {
        int64_t i = intof(key);
        if (i < 0 || i >= n.n) return mkv(V_UNDEF, 0);
        return nodeval(n.first + (uint32_t)i);
      }
    }
  }
  return vget_slow(L, c, key);
}

#if GK_LDS_PARAMS
// vget for a container the JIT proved parameter-derived (jit.cc param_flow):
// the constraint's parameter nodes come from the wave's LDS stage
__device__ __forceinline__ uint64_t vget_p(PLane& L, uint64_t c, uint64_t key, uint32_t plo, uint32_t pn) {
  if (vtag(c) == V_NODE && vtag(key) == V_STR) {
    const uint32_t ci = (uint32_t)vpay(c);
    const Node n = pnode(ci, plo, pn);
    if (!(n.flags & 1) && n.type == NT_OBJ) {
      const uint32_t id = (uint32_t)vpay(key);
      for (uint32_t i = 0; i < n.n; ++i) {
        const Node ch = pnode(n.first + i, plo, pn);
        if (ch.key == id) return nodeval_of(ch, n.first + i);
      }
      return mkv(V_UNDEF, 0);
    }
  }
  return vget(L, c, key);
}
#endif

// ------------------------------------------------------------------ printing
// Output sinks of the printers below (each has put(c); puts_/put_* dispatch on it):
//   Out  — the lane byte buffer (eagerly formatted strings, details JSON);
//   Cnt  — length only (sizing a deferred message before the wave reservation);
//   GOut — the global output bytes at a reserved offset, packed into dword
//          stores (byte stores only for the partial dwords at either end, which
//          neighbouring tuples share).
struct Out {
  char* p;
  uint32_t n, cap;
  bool ovf;
  __device__ __forceinline__ void put(char c) { if (n < cap) { GK_BUF_WRITE(1); p[n++] = c; } else ovf = true; }
};
struct Cnt {
  uint32_t n;
  bool ovf;
  __device__ __forceinline__ void put(char) { ++n; }
};
struct GOut {
  uint8_t* base;
  uint64_t start, pos;
  uint32_t acc;
  bool ovf;
  __device__ __forceinline__ void word(uint64_t w) {
    if (w >= start) *(uint32_t*)(base + w) = acc;
    else for (uint32_t i = (uint32_t)(start - w); i < 4; ++i) base[w + i] = (uint8_t)(acc >> (8 * i));
  }
  __device__ __forceinline__ void put(char c) {
    acc |= (uint32_t)(uint8_t)c << ((pos & 3) * 8);
    if ((++pos & 3) == 0) { word(pos - 4); acc = 0; }
  }
  __device__ __forceinline__ void finish() {
    if (pos & 3) {
      uint64_t w = pos & ~(uint64_t)3, lo = w > start ? w : start;
      for (uint64_t i = lo; i < pos; ++i) base[i] = (uint8_t)(acc >> (8 * (i - w)));
    }
  }
};
template <class O> __device__ __forceinline__ void put(O& o, char c) { o.put(c); }
// n bytes at s, read a dword at a time (the device string pool is padded past
// its end; lane buffers are dword-aligned arrays)
template <class O> __device__ __forceinline__ void puts_(O& o, const char* s, uint32_t n) {
  if (!n) return;
  uint64_t a = (uint64_t)s;
  const uint32_t* w = (const uint32_t*)(a & ~(uint64_t)3);
  uint32_t sh = (uint32_t)(a & 3);
  uint32_t cur = *w;
  for (uint32_t i = 0; i < n; ++i) {
    o.put((char)(cur >> (8 * sh)));
    if (++sh == 4 && i + 1 < n) { sh = 0; cur = *++w; }
  }
}
__device__ __forceinline__ void puts_(Cnt& o, const char*, uint32_t n) { o.n += n; }
template <class O> __device__ void put_cstr(O& o, const char* s) { while (*s) put(o, *s++); }
template <class O> __device__ void put_int(O& o, int64_t v) {
  uint64_t a = v < 0 ? (uint64_t)(-v) : (uint64_t)v;
  if (v < 0) put(o, '-');
  uint64_t p = 1;
  while (p <= a / 10) p *= 10;
  for (;;) {
    put(o, (char)('0' + (a / p) % 10));
    if (p == 1) break;
    p /= 10;
  }
}
// V_INT text: plain for counts and parsed integers; arithmetic results
// (INT_G) as big.Float.Text('g', -1) -- exponent form from 1e6 up, digits
// without trailing zeros (31457280 -> 3.145728e+07)
__device__ __forceinline__ bool intv_gform(uint64_t v) {
  int64_t i = intof(v);
  return (v & INT_G) && (i >= 1000000 || i <= -1000000);
}
template <class O> __device__ void put_intv(O& o, uint64_t v) {
  int64_t i = intof(v);
  if (!intv_gform(v)) { put_int(o, i); return; }
  uint64_t a = i < 0 ? (uint64_t)(-i) : (uint64_t)i;
  if (i < 0) put(o, '-');
  uint32_t e = 0;
  while (a % 10 == 0) { a /= 10; ++e; }
  uint64_t p = 1;
  uint32_t d = 1;
  while (p <= a / 10) { p *= 10; ++d; }
  e += d - 1;
  put(o, (char)('0' + a / p));
  a %= p;
  if (d > 1) {
    put(o, '.');
    for (p /= 10; p; p /= 10) { put(o, (char)('0' + a / p)); a %= p; }
  }
  put(o, 'e');
  put(o, '+');
  put(o, (char)('0' + e / 10));
  put(o, (char)('0' + e % 10));
}
template <class O> __device__ void put_sid(O& o, uint32_t sid) {
  GK_TOUCH_STR(sid);
  const StrEnt& s = gk_args.strs[sid];
  puts_(o, (const char*)gk_args.pool + s.off, s.len);
}
__device__ const char* hexd = "0123456789abcdef";

// strconv.Quote; returns false if a non-ASCII byte needs unicode.IsPrint
template <class O> __device__ bool put_quoted(O& o, SView s) {
  put(o, '"');
  for (uint32_t i = 0; i < s.n; ++i) {
    unsigned char c = (unsigned char)s.p[i];
    if (c >= 0x80) return false;
    if (c == '"' || c == '\\') { put(o, '\\'); put(o, (char)c); continue; }
    if (c >= 0x20 && c < 0x7f) { put(o, (char)c); continue; }
    switch (c) {
      case '\a': put_cstr(o, "\\a"); break;
      case '\b': put_cstr(o, "\\b"); break;
      case '\f': put_cstr(o, "\\f"); break;
      case '\n': put_cstr(o, "\\n"); break;
      case '\r': put_cstr(o, "\\r"); break;
      case '\t': put_cstr(o, "\\t"); break;
      case '\v': put_cstr(o, "\\v"); break;
      default: put_cstr(o, "\\x"); put(o, hexd[c >> 4]); put(o, hexd[c & 15]); break;
    }
  }
  put(o, '"');
  return true;
}

// encoding/json string (HTMLEscape); false on non-ASCII
template <class O> __device__ bool put_json_str(O& o, SView s) {
  put(o, '"');
  for (uint32_t i = 0; i < s.n; ++i) {
    unsigned char c = (unsigned char)s.p[i];
    if (c >= 0x80) return false;
    if (c == '"') { put_cstr(o, "\\\""); continue; }
    if (c == '\\') { put_cstr(o, "\\\\"); continue; }
    if (c == '\n') { put_cstr(o, "\\n"); continue; }
    if (c == '\r') { put_cstr(o, "\\r"); continue; }
    if (c == '\t') { put_cstr(o, "\\t"); continue; }
    if (c < 0x20 || c == '<' || c == '>' || c == '&') {
      put_cstr(o, "\\u00"); put(o, hexd[c >> 4]); put(o, hexd[c & 15]);
      continue;
    }
    put(o, (char)c);
  }
  put(o, '"');
  return true;
}

// scalar Term.String()/JSON; returns 0 not-scalar, 1 ok, -1 fallback
template <class O> __device__ int put_scalar(PLane& L, O& o, uint64_t v, bool json) {
  switch (vtag(v)) {
    case V_UNDEF: if (json) { put_cstr(o, "{}"); return 1; } return -1;
    case V_NULL: put_cstr(o, "null"); return 1;
    case V_BOOL: put_cstr(o, vpay(v) ? "true" : "false"); return 1;
    case V_NUM: put_sid(o, gk_args.nums[(uint32_t)vpay(v)].text); return 1;
    case V_INT: put_intv(o, v); return 1;
    case V_BFN: return -1;
    case V_STR: case V_HSTR: case V_SLICE: case V_GSTR:
      return (json ? put_json_str(o, sview(L, v)) : put_quoted(o, sview(L, v))) ? 1 : -1;
    case V_FMT: return -1;  // forced before any printing (jit.cc)
    case V_ROW: return -1;  // a column object (colstore.cc keeps printed paths as nodes)
    default: return 0;
  }
}

struct PFrame { uint64_t v; uint32_t i, n; uint64_t last; int cls; };

// ast.Term.String() (json=false) or encoding/json of ast.JSON (json=true, map
// keys in byte order), iterative with an explicit stack; false => fallback
template <class O> __device__ bool put_value(PLane& L, O& o, uint64_t v, bool json) {
  int r = put_scalar(L, o, v, json);
  if (r != 0) return r > 0;
  PFrame st[8];
  int sp = 0;
  st[0] = PFrame{v, 0, coll_len(L, v), 0, tclass(v)};
  if (!json && st[0].cls == 9 && st[0].n == 0) { put_cstr(o, "set()"); return true; }
  put(o, (st[0].cls == 7 || (json && st[0].cls == 9)) ? '[' : '{');
  while (sp >= 0) {
    PFrame& f = st[sp];
    if (f.i >= f.n) {
      put(o, (f.cls == 7 || (json && f.cls == 9)) ? ']' : '}');
      --sp;
      continue;
    }
    if (f.i) { put(o, ','); if (!json) put(o, ' '); }
    uint64_t k, val;
    if (json && f.cls == 8) {
      // next key in byte order after f.last
      int best = -1;
      uint64_t bk = 0;
      for (uint32_t j = 0; j < f.n; ++j) {
        uint64_t kk, vv;
        coll_at(L, f.v, j, kk, vv);
        if (!is_strv(kk)) return false;
        if (f.i && bytes_cmp(sview(L, kk), sview(L, f.last)) <= 0) continue;
        if (best < 0 || bytes_cmp(sview(L, kk), sview(L, bk)) < 0) { best = (int)j; bk = kk; }
      }
      if (best < 0) return false;
      coll_at(L, f.v, (uint32_t)best, k, val);
      f.last = k;
    } else {
      coll_at(L, f.v, f.i, k, val);
    }
    f.i++;
    if (f.cls == 8) {
      if (put_scalar(L, o, k, json) <= 0) return false;
      put(o, ':');
      if (!json) put(o, ' ');
    }
    int rs = put_scalar(L, o, val, json);
    if (rs < 0) return false;
    if (rs == 0) {
      if (sp + 1 >= 8) return false;
      int cls = tclass(val);
      uint32_t n = coll_len(L, val);
      if (!json && cls == 9 && n == 0) { put_cstr(o, "set()"); continue; }
      st[++sp] = PFrame{val, 0, n, 0, cls};
      put(o, (cls == 7 || (json && cls == 9)) ? '[' : '{');
    }
  }
  return true;
}

template <class O> __device__ __forceinline__ bool put_term(PLane& L, O& o, uint64_t v) { return put_value(L, o, v, false); }
template <class O> __device__ __forceinline__ bool put_json(PLane& L, O& o, uint64_t v) { return put_value(L, o, v, true); }

// Go fmt conversion of one sprintf argument (topdown/strings.go:355-367)
template <class O> __device__ bool put_fmt_arg(PLane& L, O& o, uint64_t v, uint32_t verb) {
  uint32_t t = vtag(v);
  if (t == V_STR || t == V_HSTR || t == V_SLICE || t == V_GSTR) {
    SView s = sview(L, v);
    if (verb == 'd') { put_cstr(o, "%!d(string="); puts_(o, s.p, s.n); put(o, ')'); return true; }
    puts_(o, s.p, s.n);
    return true;
  }
  if (t == V_NUM) {
    const NumEnt& n = gk_args.nums[(uint32_t)vpay(v)];
    if (n.flags & NF_INT64) {
      if (verb == 's') { put_cstr(o, "%!s(int="); put_int(o, n.i); put(o, ')'); return true; }
      put_int(o, n.i);
      return true;
    }
    if (verb != 'v') return false;
    put_sid(o, n.print);
    return true;
  }
  if (t == V_INT) {
    if (intv_gform(v)) {  // a float64 to Go fmt
      if (verb != 'v') return false;
      put_intv(o, v);
      return true;
    }
    if (verb == 's') { put_cstr(o, "%!s(int="); put_int(o, intof(v)); put(o, ')'); return true; }
    put_int(o, intof(v));
    return true;
  }
  if (t == V_BFN || t == V_FMT) return false;
  // everything else is formatted as Term.String() (a Go string)
  if (verb == 'd') return false;
  return put_term(L, o, v);
}

// the segments of format fidx (compiler.cc parse_format) with argument i = arg(i)
template <class O, class A> __device__ bool fmt_run(PLane& L, O& o, uint32_t fidx, A arg) {
  const uint32_t* f = gk_args.fmt + fidx;
  uint32_t nseg = f[0];
  for (uint32_t s = 0; s < nseg; ++s) {
    uint32_t kind = f[2 + 2 * s], a = f[3 + 2 * s];
    if (kind == 0) { put_sid(o, a); continue; }
    if (!put_fmt_arg(L, o, arg(a & 0xffff), a >> 16)) return false;
  }
  return true;
}

// ------------------------------------------------------------------ regex
// DFA layout at dfa_words[off]: [nstates, start, then per state: accept flags
// word, 256 transitions (u16 packed 2 per word)]; accept flags: bit0 = match
// already found (sticky), bit1 = accepting at end of text.
__device__ int re_lookup(uint32_t sid) {
  int lo = 0, hi = (int)gk_args.ndfa - 1;
  while (lo <= hi) {
    int mid = (lo + hi) >> 1;
    uint32_t k = gk_args.dfa_keys[mid];
    if (k == sid) return mid;
    if (k < sid) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}
#if GK_LDS_DFA
// the walk over a byte-class-compressed DFA the wave staged (regex.cc
// compress_regex_dfa layout); -3 when the pattern is not staged
__device__ __forceinline__ int re_run_lds(const PLane& L, uint32_t sid, uint64_t val) {
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t nd = gk_lds_dfadir[wv][0];
  for (uint32_t i = 0; i < nd; ++i) {
    if (gk_lds_dfadir[wv][1 + 4 * i] != sid) continue;
    const uint8_t* t = (const uint8_t*)gk_lds_dfa[wv] + gk_lds_dfadir[wv][2 + 4 * i];
    const uint32_t nc = gk_lds_dfadir[wv][3 + 4 * i], ss = gk_lds_dfadir[wv][4 + 4 * i];
    const uint32_t nst = nc & 0xffff, ncls = nc >> 16, sens = ss >> 16;
    const uint8_t* acc = t + 256 + nst * ncls;
    uint32_t s = ss & 0xffff;
    SView v = sview(L, val);
    for (uint32_t j = 0; j < v.n; ++j) {
      const uint32_t c = (uint8_t)v.p[j];
      if (c >= 0x80 && sens) return -2;
      if (acc[s] & 1) return 1;
      s = t[256 + s * ncls + t[c]];
      if (s >= nst) return 0;
    }
    return (acc[s] & 3) ? 1 : 0;
  }
  return -3;
}
#endif

// returns 1 match, 0 no match, -1 error (invalid pattern), -2 fallback
__device__ int re_run(const PLane& L, uint64_t pat, uint64_t val) {
  if (vtag(pat) != V_STR) return -2;
#if GK_LDS_DFA
  {
    const int r = re_run_lds(L, (uint32_t)vpay(pat), val);
    if (r != -3) return r;
  }
#endif
  int e = re_lookup((uint32_t)vpay(pat));
  if (e < 0) return -2;
  uint32_t meta = gk_args.dfa_meta[e];
  uint32_t status = meta >> 30;
  if (status == 1) return -1;
  if (status == 2) return -2;
  const uint32_t* d = gk_args.dfa_words + (meta & 0x3fffffffu);
  uint32_t nst = d[0];
  uint32_t s = d[1];
  uint32_t utf8_sensitive = d[2];
  const uint32_t* st = d + 3;
  SView v = sview(L, val);
  const uint32_t stride = 1 + 128;
  for (uint32_t i = 0; i < v.n; ++i) {
    unsigned char c = (unsigned char)v.p[i];
    if (c >= 0x80 && utf8_sensitive) return -2;
    const uint32_t* row = st + s * stride;
    if (row[0] & 1) return 1;
    uint32_t w = row[1 + (c >> 1)];
    s = (c & 1) ? (w >> 16) : (w & 0xffff);
    if (s >= nst) return 0;  // dead state
  }
  const uint32_t* row = st + s * stride;
  return (row[0] & 3) ? 1 : 0;
}

// ------------------------------------------------------------------ match
__device__ __forceinline__ bool label_lookup(uint32_t labels, uint32_t key, uint32_t& val) {
  if (labels == NO_ID) return false;
  GK_TOUCH_NODE(labels);
  const Node& n = gk_args.nodes[labels];
  for (uint32_t i = 0; i < n.n; ++i) {
    const Node& c = gk_args.nodes[n.first + i];
    if (c.key == key) { GK_TOUCH_NODE(n.first + i); val = c.val; return true; }
  }
  return false;
}

// matches_label_selector (target_template_source.go:185-230) over a labels node
// whose values are all strings (validated by the host).  Returns 1/0, or -1 error.
__device__ int sel_match(const uint32_t* w, uint32_t labels) {
  uint32_t flags = w[0];
  if (flags & 2) return -1;         // count() of a non-collection
  if (flags & 1) return 0;          // never satisfiable
  uint32_t nml = w[1];
  const uint32_t* p = w + 2;
  bool ok = true;
  for (uint32_t i = 0; i < nml; ++i) {
    uint32_t k = p[2 * i], v = p[2 * i + 1], lv;
    if (!(label_lookup(labels, k, lv) && lv == v)) ok = false;
  }
  p += 2 * nml;
  if (!ok) return 0;
  uint32_t nex = *p++;
  bool violated = false;
  for (uint32_t e = 0; e < nex; ++e) {
    uint32_t op = p[0], key = p[1], vflags = p[2], nv = p[3];
    const uint32_t* vals = p + 4;
    p += 4 + nv;
    uint32_t lv = 0;
    bool has = key != NO_ID && label_lookup(labels, key, lv);
    if (op == SO_IN || op == SO_NOTIN) {
      if (vflags & 2) return -1;      // count(values) type error
      bool nonempty = vflags & 1;
      bool inset = false;
      if (has) for (uint32_t j = 0; j < nv; ++j) if (vals[j] == lv) inset = true;
      if (op == SO_IN) {
        if (!has) violated = true;
        if (nonempty && has && !inset) violated = true;
      } else {
        if (nonempty && has && inset) violated = true;
      }
    } else if (op == SO_EXISTS) {
      if (!has) violated = true;
    } else if (op == SO_DOESNOTEXIST) {
      if (has) violated = true;
    }
  }
  return violated ? 0 : 1;
}

// any_labelselector_match over the review's object / oldObject labels
__device__ int any_sel(const uint32_t* w, const ReviewCol& rc) {
  bool uo = rc.flags & RC_LABELS_OBJ, ul = rc.flags & RC_LABELS_OLD;
  if (!uo && !ul) return sel_match(w, NO_ID);
  int r = 0;
  if (uo) { int x = sel_match(w, rc.labels); if (x < 0) return -1; r |= x; }
  if (ul) { int x = sel_match(w, rc.old_labels); if (x < 0) return -1; r |= x; }
  return r;
}

// 1 = match, 0 = no match, -1 = error (query fails), -2 = fallback
__device__ int match_constraint(const MatchSpec& m, const ReviewCol& rc) {
  if (!(rc.flags & RC_REVIEW_DEF)) return 0;
  const uint32_t* W = gk_args.mwords;
  // kinds
  {
    const uint32_t* k = W + m.kinds_off;
    uint32_t nsel = *k++;
    bool any = false;
    for (uint32_t s = 0; s < nsel; ++s) {
      uint32_t ng = *k++;
      bool gm = false;
      for (uint32_t i = 0; i < ng; ++i) { uint32_t g = k[i]; if (g == 0xfffffffeu || (g == rc.group && g != NO_ID)) gm = true; }
      k += ng;
      uint32_t nk = *k++;
      bool km = false;
      for (uint32_t i = 0; i < nk; ++i) { uint32_t x = k[i]; if (x == 0xfffffffeu || (x == rc.kind && x != NO_ID)) km = true; }
      k += nk;
      if (gm && km) any = true;
    }
    if (!any) return 0;
  }
  bool kind_def = rc.flags & RC_KIND_OK;
  bool is_ns = rc.flags & RC_IS_NS;
  bool always = kind_def && !is_ns && (rc.flags & RC_NS_EMPTY);
  // namespaces / excludedNamespaces
  if (m.flags & MF_HAS_NAMESPACES) {
    if (!always) {
      if (!kind_def || rc.nsname == NO_ID) return 0;
      const uint32_t* l = W + m.ns_off;
      bool in = false;
      for (uint32_t i = 0; i < l[0]; ++i) if (l[1 + i] == rc.nsname) in = true;
      if (!in) return 0;
    }
  }
  if (m.flags & MF_HAS_EXCLUDED) {
    if (!always) {
      if (!kind_def || rc.nsname == NO_ID) return 0;
      const uint32_t* l = W + m.exns_off;
      for (uint32_t i = 0; i < l[0]; ++i) if (l[1 + i] == rc.nsname) return 0;
    }
  }
  // namespaceSelector
  if (m.flags & MF_HAS_NSSEL) {
    if (!always) {
      if (!kind_def) return 0;
      const uint32_t* w = W + m.nssel_off;
      int r;
      if (is_ns) r = any_sel(w, rc);
      else {
        if (rc.ns_labels == NO_ID && !(rc.flags & (RC_UNSTABLE_NS | RC_NS_CACHED))) return 0;
        r = sel_match(w, rc.ns_labels);
      }
      if (r < 0) return -1;
      if (!r) return 0;
    }
  }
  // scope
  if (m.flags & MF_SCOPE_PRESENT) {
    bool ok = (m.flags & MF_SCOPE_ANY) || ((m.flags & MF_SCOPE_NS) && !(rc.flags & RC_NS_EMPTY)) ||
              ((m.flags & MF_SCOPE_CLUSTER) && (rc.flags & RC_NS_EMPTY));
    if (!ok) return 0;
  }
  // labelSelector
  {
    int r = any_sel(W + m.labelsel_off, rc);
    if (r < 0) return -1;
    if (!r) return 0;
  }
  return 1;
}

// ------------------------------------------------------------------ emit
// Violations go straight to the output at the emission site.  The lanes of a
// wavefront that emit at one site take consecutive tuple slots (one ballot +
// one atomic per wave and site), so their 32-B tuples land as one coalesced
// run; a deferred message's argument record goes to the structure-of-arrays
// `frec` at the same slot (word j of tuple i at frec[j * out_cap + i]).
// Message bytes that exist at emission time (an eager message, a details
// JSON) are copied to `ebytes`, reserved the same way.  The final byte layout
// (message, then details) is produced after the predicate kernels by the size
// and format passes (kernels.hip), which also size deferred messages.  A lane
// that fails after emitting leaves its tuples behind: the review's flag word
// (rflags) drops them in every consumer, as it drops the rows of reviews
// another constraint's lane flagged.

// Output reservations: a plain atomicAdd per emitting lane on the one
// counter.  The address is wave-uniform, so the compiler's atomic optimizer
// turns it into one atomic per wavefront (a scan over the active lanes, then a
// broadcast of the base): consecutive slots for the lanes that emit at a site.
__device__ __forceinline__ uint64_t wave_reserve(unsigned long long* ctr, bool want) {
  return want ? (uint64_t)atomicAdd(ctr, 1ull) : 0;
}

// Tuple slots by per-wavefront chunks (device build).  One same-address
// atomic per wavefront per emission site serialized the emitting kernels:
// K8sContainerLimits executes ~20-50 emission sites per wave, and a
// microbenchmark of that pattern (tools/atomic_probe.hip, 1M lanes x 48 sites)
// takes 9.3 ms against 1.1 ms with 64-slot chunks.  A wave now takes a chunk
// of slots (its size grows with what the wave has emitted, CHUNK_MIN ..
// CHUNK_MAX) and numbers its emitting lanes inside it; the slots a wave leaves
// unused -- a chunk's tail when the next emission does not fit, the last
// chunk's at the wave's end -- are marked as holes (Viol.review = VIOL_HOLE),
// and gk_compact (kernels.hip) packs the tuples of all launches before the
// size / format passes, which read a dense array as before.  Chunk state per
// wave in LDS: next slot, slots left, slots used so far.
constexpr uint32_t VIOL_HOLE = 0xffffffffu;
constexpr uint64_t CHUNK_MIN = 64, CHUNK_MAX = 1024;
// a new chunk takes the wave's slots so far divided by GK_CHUNK_DIV (clamped;
// 4 since round 5: compaction 0.33 -> 0.31 ms, profiles/r05/r05g_chunk_ab.txt):
// 1 doubles (a wave's last chunk leaves up to half its slots as holes, which
// the wave writes and the compaction reads); larger divisors trade holes for
// a few more atomics
#ifndef GK_CHUNK_DIV
#define GK_CHUNK_DIV 4
#endif
#ifndef GK_HOST
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
}
// holes at [from, from + k) of the tuple array, written by the active lanes
__device__ __forceinline__ void mark_holes(uint64_t from, uint64_t k) {
  const uint64_t act = __ballot(true);
  const uint32_t nact = (uint32_t)__popcll(act), rank = gk_lanes_below(act);
  for (uint64_t j = rank; j < k; j += nact)
    if (from + j < gk_args.out_cap) gk_args.out[from + j].review = VIOL_HOLE;
}
#endif
#ifndef GK_HOST
// The wave's chunk state is shared by its lanes, and divergent lane subsets
// update it at different emission sites.  Plain loads and stores of it are a
// data race to the compiler, which may then forward a lane's own earlier store
// to a later load (a phi over the emission sites its own path took) instead of
// reloading what another subset wrote: stale chunk state hands out slots twice
// and marks live tuples as holes.  Every access is a wave-scope atomic, which
// the compiler neither forwards nor caches, and is read back uniformly.
// GK_CHUNK_PLAIN=1 (diagnostic only, GKGPU_JIT_PRE): round 5's plain accesses,
// to reproduce the row loss (tools/diag_r06.sh).
#ifndef GK_CHUNK_PLAIN
#define GK_CHUNK_PLAIN 0
#endif
__device__ __forceinline__ uint64_t chunk_ld(unsigned long long* p) {
#if GK_CHUNK_PLAIN
  return *p;
#else
  return rfl64(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT));
#endif
}
__device__ __forceinline__ void chunk_st(unsigned long long* p, uint64_t v) {
#if GK_CHUNK_PLAIN
  *p = v;
#else
  __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
#endif
}
#endif
// a slot for each lane with `want` (every active lane calls it)
__device__ __forceinline__ uint64_t slot_reserve(bool want) {
#ifdef GK_HOST
  return wave_reserve(&gk_args.counters[0], want);
#else
  const uint64_t m = __ballot(want);
  if (!m) return 0;
  const uint64_t n = (uint64_t)__popcll(m);
  unsigned long long* st = gk_lds_chunk[threadIdx.x >> 6];
  uint64_t base = chunk_ld(&st[0]), left = chunk_ld(&st[1]);
  const uint64_t used = chunk_ld(&st[2]);
  if (n > left) {
    mark_holes(base, left);
    const uint64_t want = used / GK_CHUNK_DIV;
    uint64_t take = want < CHUNK_MIN ? CHUNK_MIN : want > CHUNK_MAX ? CHUNK_MAX : want;
    if (take < n) take = n;
    uint64_t b = 0;
    if (gk_lanes_below(__ballot(true)) == 0) b = (uint64_t)atomicAdd(&gk_args.counters[0], (unsigned long long)take);
    base = rfl64(b);
    left = take;
  }
  const uint64_t slot = base + gk_lanes_below(m);
  chunk_st(&st[0], base + n);
  chunk_st(&st[1], left - n);
  chunk_st(&st[2], used + n);
  return slot;
#endif
}
__device__ __forceinline__ uint64_t wave_reserve_bytes(unsigned long long* ctr, bool want, uint32_t n) {
  return (want && n) ? (uint64_t)atomicAdd(ctr, (unsigned long long)n) : 0;
}

// Staged bytes (ebytes) by per-wavefront chunks, as slot_reserve does for
// tuples: the slow emission path (details, eager messages) otherwise takes one
// same-address atomic on counters[1] per wave and site.  The lanes' byte
// counts are numbered by an LDS atomic (any active-lane subset); the tail of a
// chunk the next emission does not fit is left unused -- nothing reads
// ebytes except through a tuple's offsets.  Chunk size: the wave's bytes so
// far, BCHUNK_MIN .. BCHUNK_MAX.
constexpr uint64_t BCHUNK_MIN = 512, BCHUNK_MAX = 16384;
#ifndef GK_BCHUNK
#define GK_BCHUNK 1  // A/B switch (GKGPU_JIT_PRE=GK_BCHUNK=0: one atomic per wave and site)
#endif
__device__ __forceinline__ uint64_t bytes_reserve(bool want, uint32_t n) {
#if defined(GK_HOST) || !GK_BCHUNK
  return wave_reserve_bytes(&gk_args.counters[1], want, n);
#else
  const uint32_t nn = want ? n : 0u;
  if (!__ballot(nn != 0)) return 0;
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t o = nn ? __hip_atomic_fetch_add(&gk_lds_bscan[wv], nn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) : 0u;
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const uint64_t tot = (uint32_t)__builtin_amdgcn_readfirstlane((int)__hip_atomic_load(&gk_lds_bscan[wv], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT));
  unsigned long long* st = gk_lds_chunk[wv] + 3;
  uint64_t base = chunk_ld(&st[0]), left = chunk_ld(&st[1]);
  const uint64_t used = chunk_ld(&st[2]);
  if (tot > left) {
    uint64_t take = used < BCHUNK_MIN ? BCHUNK_MIN : used > BCHUNK_MAX ? BCHUNK_MAX : used;
    if (take < tot) take = tot;
    uint64_t b = 0;
    if (gk_lanes_below(__ballot(true)) == 0) b = (uint64_t)atomicAdd(&gk_args.counters[1], (unsigned long long)take);
    base = rfl64(b);
    left = take;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  if (gk_lanes_below(__ballot(true)) == 0) {
    chunk_st(&st[0], base + tot);
    chunk_st(&st[1], left - tot);
    chunk_st(&st[2], used + tot);
    __hip_atomic_store(&gk_lds_bscan[wv], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  return base + o;
#endif
}

// the tuple order key of the lane's next emission; false = over the limits
__device__ __forceinline__ bool next_seq(PLane& L, uint32_t& seq) {
  const uint32_t en = L.en, ord = L.ord;
  if (en >= EM_MAXIDX || ord >= EM_MAXORD) { lane_fallback(L, FB_MSG_LEN); return false; }
  seq = (ord << 8) | en;
  return true;
}

// an emission's bytes into the global staging buffer at `off` (slow path
// only): source read a dword at a time, destination written in dwords (byte
// stores only at the two ends, which neighbouring reservations share)
__device__ __forceinline__ void copy_out(uint64_t off, const char* src, uint32_t n) {
  GOut g{(uint8_t*)gk_args.ebytes, off, off, 0, false};
  puts_(g, src, n);
  g.finish();
}

__device__ __forceinline__ void slot_overflow(const PLane& L) { atomicOr(&gk_args.rflags[L.rv], (uint32_t)RF_OVERFLOW); }

// An emission whose message and details bytes exist now (an eager message,
// e.g. autoreject's constant or a string sprintf built in the lane buffer).
// det == nullptr: the details are the hook default `{}`.  Every active lane
// calls it (want = this lane emits).
__device__ __noinline__ void emit_eager(PLane& L, bool want, uint32_t rule, const char* msg, uint32_t mlen,
                                        const char* det, uint32_t dlen) {
  uint32_t seq = 0;
  if (want) want = next_seq(L, seq);
  const bool detobj = det == nullptr;
  const uint32_t eb = want ? mlen + (detobj ? 0u : dlen) : 0u;
  const uint64_t eoff = bytes_reserve(want, eb);
  const uint64_t slot = slot_reserve(want);
  if (!want) return;
  L.en = L.en + 1u;
  if (slot >= gk_args.out_cap || eoff + eb > gk_args.ebytes_cap) { slot_overflow(L); return; }
  copy_out(eoff, msg, mlen);
  if (!detobj) copy_out(eoff + mlen, det, dlen);
  Viol v;
  v.review = L.rv;
  v.constraint = L.cn;
  v.seq = (uint16_t)seq;
  v.rule = (uint16_t)rule;
  v.msg_len = mlen;
  v.msg_off = eoff;
  v.det_len = detobj ? 2u : dlen;
  v.pad = detobj ? VF_DET_OBJ : 0u;
  gk_args.out[slot] = v;
}

// ------------------------------------------------------------------ builtins
// One device function per builtin: template kernels call them directly with
// register operands (jit.cc); the VM dispatches through call_builtin.
__device__ __forceinline__ uint64_t bi_count(PLane& L, uint64_t a) {
  uint32_t t = vtag(a);
  if (t == V_NODE || t == V_LIST || t == V_ROWS || t == V_ROW) return mkint(coll_len(L, a));
  if (is_strv(a)) return mkint(sview(L, a).n);
  lane_error(L);
  return mkv(V_UNDEF, 0);
}

__device__ uint64_t bi_anyall(PLane& L, uint32_t id, uint64_t a) {
  int cls = tclass(a);
  if (cls != 7 && cls != 9) { lane_error(L); return mkv(V_UNDEF, 0); }
  uint32_t n = coll_len(L, a);
  bool any = false, all = true;
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t k, v;
    coll_at(L, a, i, k, v);
    bool t = vtag(v) == V_BOOL && vpay(v) == 1;
    any |= t;
    all &= t;
  }
  return mkv(V_BOOL, id == BI_ANY ? any : all);
}

// startswith / endswith / contains (topdown/strings.go:135-175, byte-wise)
__device__ GK_HOT uint64_t bi_strpred(PLane& L, uint32_t id, uint64_t a, uint64_t b) {
  if (!is_strv(a) || !is_strv(b)) { lane_error(L); return mkv(V_UNDEF, 0); }
  SView s = sview(L, a), p = sview(L, b);
  if (p.n > s.n) return mkv(V_BOOL, 0);
  if (id == BI_STARTSWITH) { for (uint32_t i = 0; i < p.n; ++i) if (s.p[i] != p.p[i]) return mkv(V_BOOL, 0); return mkv(V_BOOL, 1); }
  if (id == BI_ENDSWITH) { uint32_t o = s.n - p.n; for (uint32_t i = 0; i < p.n; ++i) if (s.p[o + i] != p.p[i]) return mkv(V_BOOL, 0); return mkv(V_BOOL, 1); }
  for (uint32_t o = 0; o + p.n <= s.n; ++o) {
    bool m = true;
    for (uint32_t i = 0; i < p.n && m; ++i) if (s.p[o + i] != p.p[i]) m = false;
    if (m) return mkv(V_BOOL, 1);
  }
  return mkv(V_BOOL, 0);
}

// re_run / a literal pattern's compiled DFA (jit.cc) -> value: 1/0 match,
// -1 invalid pattern (builtin error), -2 CPU fallback
__device__ __forceinline__ uint64_t re_result(PLane& L, int r) {
  if (r == -1) { lane_error(L); return mkv(V_UNDEF, 0); }
  if (r == -2) { lane_fallback(L, FB_REGEX); return mkv(V_UNDEF, 0); }
  return mkv(V_BOOL, r);
}
__device__ __forceinline__ uint64_t bi_re_match(PLane& L, uint64_t a, uint64_t b) {
  if (!is_strv(a) || !is_strv(b)) { lane_error(L); return mkv(V_UNDEF, 0); }
  return re_result(L, re_run(L, a, b));
}

// to_number (topdown/casts.go:14-33).  The number keeps the string's text, so
// only canonical integer texts become V_INT (no '+', no leading zero, no "-0":
// those print differently); other valid forms go to the CPU fallback.
__device__ GK_HOT uint64_t bi_to_number(PLane& L, uint64_t a) {
  const uint64_t UND = mkv(V_UNDEF, 0);
  uint32_t t = vtag(a);
  if (t == V_NULL) return mkint(0);
  if (t == V_BOOL) return mkint((int64_t)vpay(a));
  if (is_numv(a)) return a;
  if (!is_strv(a)) { lane_error(L); return UND; }
  SView s = sview(L, a);
  uint32_t i = 0;
  bool neg = false;
  if (i < s.n && (s.p[i] == '+' || s.p[i] == '-')) { neg = s.p[i] == '-'; ++i; }
  if (i >= s.n) { lane_error(L); return UND; }
  bool digits_only = true, any_digit = false, dot = false, ex = false, bad = false;
  for (uint32_t j = i; j < s.n; ++j) {
    char c = s.p[j];
    if (c >= '0' && c <= '9') { any_digit = true; continue; }
    digits_only = false;
    if (c == '.' && !dot && !ex) { dot = true; continue; }
    if ((c == 'e' || c == 'E') && any_digit && !ex) { ex = true; if (j + 1 < s.n && (s.p[j + 1] == '+' || s.p[j + 1] == '-')) ++j; continue; }
    if (c == 'i' || c == 'I' || c == 'n' || c == 'N' || c == 'x' || c == 'X' || c == '_' || c == 'p' || c == 'P') { lane_fallback(L, FB_NUMBER); return UND; }
    bad = true;
  }
  if (bad || !any_digit) { lane_error(L); return UND; }
  if (!digits_only || s.n - i > 15 || s.p[0] == '+' || (s.n - i > 1 && s.p[i] == '0')) { lane_fallback(L, FB_NUMBER); return UND; }
  int64_t v = 0;
  for (uint32_t j = i; j < s.n; ++j) v = v * 10 + (s.p[j] - '0');
  if (neg && v == 0) { lane_fallback(L, FB_NUMBER); return UND; }
  return mkint(neg ? -v : v);
}

// replace = strings.Replace(s, old, new, -1) (topdown/strings.go:212-229)
__device__ uint64_t bi_replace(PLane& L, uint64_t a0, uint64_t a1, uint64_t a2) {
  const uint64_t UND = mkv(V_UNDEF, 0);
  if (!is_strv(a0) || !is_strv(a1) || !is_strv(a2)) { lane_error(L); return UND; }
  SView s = sview(L, a0), old = sview(L, a1), nw = sview(L, a2);
  if (old.n == 0) { lane_fallback(L, FB_STRING); return UND; }
  // no occurrence: the result is the subject itself (no lane-buffer copy)
  bool any = false;
  for (uint32_t i = 0; i + old.n <= s.n && !any; ++i) {
    bool m = true;
    for (uint32_t j = 0; j < old.n && m; ++j) if (s.p[i + j] != old.p[j]) m = false;
    any = m;
  }
  if (!any) return a0;
  uint32_t start = L.bp;
  for (uint32_t i = 0; i < s.n;) {
    bool m = i + old.n <= s.n;
    for (uint32_t j = 0; j < old.n && m; ++j) if (s.p[i + j] != old.p[j]) m = false;
    if (m) {
      for (uint32_t j = 0; j < nw.n; ++j) { if (L.bp >= BCAP) { lane_fallback(L, FB_MSG_LEN); return UND; } L.B[L.bp++] = nw.p[j]; }
      i += old.n;
    } else {
      if (L.bp >= BCAP) { lane_fallback(L, FB_MSG_LEN); return UND; }
      L.B[L.bp++] = s.p[i++];
    }
  }
  return mkhstr(start, L.bp - start);
}

// substring(s, start, length), byte-indexed (topdown/strings.go:100-133)
__device__ GK_HOT uint64_t bi_substring(PLane& L, uint64_t a0, uint64_t a1, uint64_t a2) {
  const uint64_t UND = mkv(V_UNDEF, 0);
  if (!is_strv(a0)) { lane_error(L); return UND; }
  int64_t st, ln;
  if (!is_numv(a1) || !num_int(L, a1, st)) { lane_error(L); return UND; }
  SView s = sview(L, a0);
  if (st >= (int64_t)s.n) return mkv(V_STR, 0);  // "" is string id 0
  if (st < 0) { lane_error(L); return UND; }
  if (!is_numv(a2) || !num_int(L, a2, ln)) { lane_error(L); return UND; }
  uint32_t end = ln < 0 ? s.n : (uint32_t)((st + ln) < (int64_t)s.n ? (st + ln) : s.n);
  uint32_t len = end - (uint32_t)st;
  if (vtag(a0) == V_STR && s.n < 0x3fff) return mkslice((uint32_t)vpay(a0), (uint32_t)st, len);
  if (vtag(a0) == V_HSTR) return mkhstr((uint32_t)(s.p - L.B) + (uint32_t)st, len);
  if (vtag(a0) == V_GSTR) return mkv(V_GSTR, (((vpay(a0) >> 20) + (uint64_t)st) << 20) | len);
  if (vtag(a0) == V_SLICE) {
    uint64_t p = vpay(a0);
    return mkslice((uint32_t)(p >> 28), (uint32_t)((p >> 14) & 0x3fff) + (uint32_t)st, len);
  }
  lane_fallback(L, FB_STRING);
  return UND;
}

// the byte range [st, st+len) of string value a0 (s = its view) as a value
// that shares the bytes: a slice of an interned string or of the lane buffer
__device__ uint64_t str_sub(PLane& L, uint64_t a0, SView s, uint32_t st, uint32_t len) {
  if (st == 0 && len == s.n) return a0;
  if (len == 0) return mkv(V_STR, 0);
  if (vtag(a0) == V_STR && s.n < 0x3fff) return mkslice((uint32_t)vpay(a0), st, len);
  if (vtag(a0) == V_HSTR) return mkhstr((uint32_t)(s.p - L.B) + st, len);
  if (vtag(a0) == V_GSTR) return mkv(V_GSTR, (((vpay(a0) >> 20) + (uint64_t)st) << 20) | len);
  if (vtag(a0) == V_SLICE) {
    uint64_t p = vpay(a0);
    return mkslice((uint32_t)(p >> 28), (uint32_t)((p >> 14) & 0x3fff) + st, len);
  }
  lane_fallback(L, FB_STRING);
  return mkv(V_UNDEF, 0);
}

__device__ __forceinline__ bool bytes_at(SView s, uint32_t o, SView p) {
  if (o + p.n > s.n) return false;
  for (uint32_t i = 0; i < p.n; ++i) if (s.p[o + i] != p.p[i]) return false;
  return true;
}

// trim(s, cutset) = strings.Trim (topdown/strings.go:261-273).  The cutset is a
// set of runes; for an ASCII cutset byte-wise trimming is exact (UTF-8 lead and
// continuation bytes are >= 0x80), otherwise the review goes to the CPU.
__device__ uint64_t bi_trim(PLane& L, uint64_t a0, uint64_t a1) {
  if (!is_strv(a0) || !is_strv(a1)) { lane_error(L); return mkv(V_UNDEF, 0); }
  SView s = sview(L, a0), c = sview(L, a1);
  for (uint32_t i = 0; i < c.n; ++i) if ((unsigned char)c.p[i] >= 0x80) { lane_fallback(L, FB_UNICODE); return mkv(V_UNDEF, 0); }
  auto in_cut = [&](char ch) { for (uint32_t i = 0; i < c.n; ++i) if (c.p[i] == ch) return true; return false; };
  uint32_t i = 0, j = s.n;
  while (i < j && in_cut(s.p[i])) ++i;
  while (j > i && in_cut(s.p[j - 1])) --j;
  return str_sub(L, a0, s, i, j - i);
}

// trim_prefix / trim_suffix = strings.TrimPrefix / TrimSuffix (byte-wise)
__device__ uint64_t bi_trim_fix(PLane& L, uint32_t id, uint64_t a0, uint64_t a1) {
  if (!is_strv(a0) || !is_strv(a1)) { lane_error(L); return mkv(V_UNDEF, 0); }
  SView s = sview(L, a0), p = sview(L, a1);
  if (p.n > s.n) return a0;
  if (id == BI_TRIM_PREFIX) return bytes_at(s, 0, p) ? str_sub(L, a0, s, p.n, s.n - p.n) : a0;
  return bytes_at(s, s.n - p.n, p) ? str_sub(L, a0, s, 0, s.n - p.n) : a0;
}

// split(s, sep) = strings.Split (topdown/strings.go:195-210): an array of the
// pieces, each sharing the subject's bytes.  An empty separator splits into
// runes (ASCII subjects only; others go to the CPU).
__device__ uint64_t bi_split(PLane& L, uint64_t a0, uint64_t a1) {
  const uint64_t UND = mkv(V_UNDEF, 0);
  if (!is_strv(a0) || !is_strv(a1)) { lane_error(L); return UND; }
  SView s = sview(L, a0), d = sview(L, a1);
  uint32_t n = 1;
  if (d.n == 0) {
    for (uint32_t i = 0; i < s.n; ++i) if ((unsigned char)s.p[i] >= 0x80) { lane_fallback(L, FB_UNICODE); return UND; }
    n = s.n;
  } else {
    for (uint32_t i = 0; i + d.n <= s.n;) { if (bytes_at(s, i, d)) { ++n; i += d.n; } else ++i; }
  }
  uint64_t l = list_new(L, LK_ARR, n);
  if (vtag(l) != V_LIST) return UND;
  uint32_t o = list_off(l);
  if (d.n == 0) {
    for (uint32_t i = 0; i < n; ++i) hset(L, o + 2 + i, str_sub(L, a0, s, i, 1));
  } else {
    uint32_t k = 0, st = 0;
    for (uint32_t i = 0; i + d.n <= s.n;) {
      if (bytes_at(s, i, d)) { hset(L, o + 2 + k++, str_sub(L, a0, s, st, i - st)); i += d.n; st = i; } else ++i;
    }
    hset(L, o + 2 + k++, str_sub(L, a0, s, st, s.n - st));
  }
  hset(L, o, n);
  return l;
}

// lower / upper = strings.ToLower / ToUpper: ASCII subjects on the GPU
__device__ uint64_t bi_case(PLane& L, uint32_t id, uint64_t a0) {
  if (!is_strv(a0)) { lane_error(L); return mkv(V_UNDEF, 0); }
  SView s = sview(L, a0);
  bool change = false;
  for (uint32_t i = 0; i < s.n; ++i) {
    unsigned char ch = (unsigned char)s.p[i];
    if (ch >= 0x80) { lane_fallback(L, FB_UNICODE); return mkv(V_UNDEF, 0); }
    change |= id == BI_LOWER ? (ch >= 'A' && ch <= 'Z') : (ch >= 'a' && ch <= 'z');
  }
  if (!change) return a0;
  if (L.bp + s.n > BCAP) { lane_fallback(L, FB_MSG_LEN); return mkv(V_UNDEF, 0); }
  uint32_t st = L.bp;
  for (uint32_t i = 0; i < s.n; ++i) {
    char ch = s.p[i];
    if (id == BI_LOWER && ch >= 'A' && ch <= 'Z') ch = (char)(ch + 32);
    if (id == BI_UPPER && ch >= 'a' && ch <= 'z') ch = (char)(ch - 32);
    L.B[L.bp++] = ch;
  }
  return mkhstr(st, s.n);
}

// concat(delim, array|set) = strings.Join (topdown/strings.go:48-83); non-string
// elements and other collections are operand errors
__device__ uint64_t bi_concat(PLane& L, uint64_t a0, uint64_t a1) {
  const uint64_t UND = mkv(V_UNDEF, 0);
  int cls = tclass(a1);
  if (!is_strv(a0) || (cls != 7 && cls != 9)) { lane_error(L); return UND; }
  SView d = sview(L, a0);
  uint32_t n = coll_len(L, a1), st = L.bp;
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t k, v;
    coll_at(L, a1, i, k, v);
    if (!is_strv(v)) { L.bp = st; lane_error(L); return UND; }
    SView e = sview(L, v);
    if (L.bp + e.n + d.n > BCAP) { lane_fallback(L, FB_MSG_LEN); return UND; }
    if (i) for (uint32_t j = 0; j < d.n; ++j) L.B[L.bp++] = d.p[j];
    for (uint32_t j = 0; j < e.n; ++j) L.B[L.bp++] = e.p[j];
  }
  if (L.bp == st) return mkv(V_STR, 0);
  return mkhstr(st, L.bp - st);
}

// indexof(s, sub) = strings.Index: byte offset or -1 (topdown/strings.go:85-98)
__device__ uint64_t bi_indexof(PLane& L, uint64_t a0, uint64_t a1) {
  if (!is_strv(a0) || !is_strv(a1)) { lane_error(L); return mkv(V_UNDEF, 0); }
  SView s = sview(L, a0), p = sview(L, a1);
  for (uint32_t o = 0; o + p.n <= s.n; ++o) if (bytes_at(s, o, p)) return mkint(o);
  return mkint(-1);
}

// sort (topdown/sets.go builtinSort via ast.Compare, v0.21): an array or a
// set -> sorted array.  Insertion sort into a new heap array; elements whose
// order this runtime cannot decide (composites) go to the CPU fallback.
__device__ uint64_t bi_sort(PLane& L, uint64_t a) {
  const uint64_t UND = mkv(V_UNDEF, 0);
  const int cls = tclass(a);
  if (cls != 7 && cls != 9) { lane_error(L); return UND; }
  const uint32_t n = coll_len(L, a);
  uint64_t out = list_new(L, LK_ARR, n);
  if (vtag(out) == V_UNDEF) return UND;
  const uint32_t o = list_off(out);
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t k, v;
    coll_at(L, a, i, k, v);
    uint32_t j = i;
    while (j > 0) {
      const uint64_t p = hget(L, o + 2 + j - 1);
      const int c = vcmp(L, p, v);
      if (c == 2) return UND;
      if (c == 3) { lane_fallback(L, FB_DEEP_EQ); return UND; }
      if (c <= 0) break;
      hset(L, o + 2 + j, p);
      --j;
    }
    hset(L, o + 2 + j, v);
  }
  hset(L, o, n);
  return out;
}

// array.concat (topdown/array.go builtinArrayConcat): two arrays -> one new
// heap array (a type error otherwise)
__device__ uint64_t bi_array_concat(PLane& L, uint64_t a, uint64_t b) {
  const uint64_t UND = mkv(V_UNDEF, 0);
  if (tclass(a) != 7 || tclass(b) != 7) { lane_error(L); return UND; }
  const uint32_t na = coll_len(L, a), nb = coll_len(L, b);
  uint64_t out = list_new(L, LK_ARR, na + nb);
  if (vtag(out) == V_UNDEF) return UND;
  const uint32_t o = list_off(out);
  for (uint32_t i = 0; i < na + nb; ++i) {
    uint64_t k, v;
    if (i < na) coll_at(L, a, i, k, v);
    else coll_at(L, b, i - na, k, v);
    hset(L, o + 2 + i, v);
  }
  hset(L, o, na + nb);
  return out;
}

__device__ uint64_t call_builtin(PLane& L, uint32_t id, const uint64_t* a) {
  switch (id) {
    case BI_COUNT: return bi_count(L, a[0]);
    case BI_ANY: case BI_ALL: return bi_anyall(L, id, a[0]);
    case BI_STARTSWITH: case BI_ENDSWITH: case BI_CONTAINS: return bi_strpred(L, id, a[0], a[1]);
    case BI_RE_MATCH: return bi_re_match(L, a[0], a[1]);
    case BI_TO_NUMBER: return bi_to_number(L, a[0]);
    case BI_REPLACE: return bi_replace(L, a[0], a[1], a[2]);
    case BI_SUBSTRING: return bi_substring(L, a[0], a[1], a[2]);
    case BI_IS_NUMBER: return mkv(V_BOOL, is_numv(a[0]));
    case BI_IS_STRING: return mkv(V_BOOL, is_strv(a[0]));
    case BI_IS_BOOLEAN: return mkv(V_BOOL, vtag(a[0]) == V_BOOL);
    case BI_IS_NULL: return mkv(V_BOOL, vtag(a[0]) == V_NULL);
    case BI_IS_ARRAY: return mkv(V_BOOL, tclass(a[0]) == 7);
    case BI_IS_OBJECT: return mkv(V_BOOL, tclass(a[0]) == 8);
    case BI_IS_SET: return mkv(V_BOOL, tclass(a[0]) == 9);
    case BI_TRIM: return bi_trim(L, a[0], a[1]);
    case BI_TRIM_PREFIX: case BI_TRIM_SUFFIX: return bi_trim_fix(L, id, a[0], a[1]);
    case BI_SPLIT: return bi_split(L, a[0], a[1]);
    case BI_LOWER: case BI_UPPER: return bi_case(L, id, a[0]);
    case BI_CONCAT: return bi_concat(L, a[0], a[1]);
    case BI_INDEXOF: return bi_indexof(L, a[0], a[1]);
    case BI_SORT: return bi_sort(L, a[0]);
    case BI_ARRAY_CONCAT: return bi_array_concat(L, a[0], a[1]);
    default: break;
  }
  lane_fallback(L, FB_UNSUPPORTED);
  return mkv(V_UNDEF, 0);
}

__device__ __noinline__ uint64_t arith_slow(PLane& L, uint32_t kind, uint64_t x, uint64_t y);
// exact small-integer +, -, * inline (the common case: canonical quantities
// times a constant); everything else out of line
__device__ __forceinline__ uint64_t arith(PLane& L, uint32_t kind, uint64_t x, uint64_t y) {
  if (vtag(x) == V_INT && vtag(y) == V_INT && kind <= AR_MUL) {
    const int64_t LIM = (1ll << 46);
    int64_t a = intof(x), b = intof(y);
    if (a < LIM && a > -LIM && b < LIM && b > -LIM) {
      if (kind == AR_PLUS) return mkint_g(a + b);
      if (kind == AR_MINUS) return mkint_g(a - b);
      uint64_t ua = a < 0 ? (uint64_t)(-a) : (uint64_t)a, ub = b < 0 ? (uint64_t)(-b) : (uint64_t)b;
      if (__umul64hi(ua, ub) == 0 && ua * ub < (uint64_t)LIM) return mkint_g(a * b);
    }
  }
  // set difference of heap sets whose members compare by identity (e.g.
  // probe_type_set - {field | ctr[probe][field]}), inline
  if (kind == AR_MINUS && vtag(x) == V_LIST && vtag(y) == V_LIST && list_kind(x) == LK_SET && list_kind(y) == LK_SET) {
    const uint32_t nx = list_len(L, x), ny = list_len(L, y), hp0 = L.hp;
    uint64_t out = list_new(L, LK_SET, nx);
    if (vtag(out) == V_UNDEF) return out;
    const uint32_t oo = list_off(out);
    uint32_t n = 0;
    bool ok = true;
    for (uint32_t i = 0; i < nx && ok; ++i) {
      const uint64_t v = list_at(L, x, i);
      int found = 0;
      for (uint32_t j = 0; j < ny && found == 0; ++j) found = id_eq(list_at(L, y, j), v);
      if (found < 0) ok = false;
      else if (found == 0) hset(L, oo + 2 + n++, v);
    }
    if (ok) { hset(L, oo, n); return out; }
    L.hp = hp0;
  }
  return arith_slow(L, kind, x, y);
}
__device__ __noinline__ uint64_t arith_slow(PLane& L, uint32_t kind, uint64_t x, uint64_t y) {
  const uint64_t UND = mkv(V_UNDEF, 0);
  if (kind == AR_MINUS && tclass(x) == 9 && tclass(y) == 9) {
    uint64_t out = list_new(L, LK_SET, coll_len(L, x));
    if (vtag(out) == V_UNDEF) return UND;
    uint32_t n = coll_len(L, x);
    for (uint32_t i = 0; i < n; ++i) {
      uint64_t k, v;
      coll_at(L, x, i, k, v);
      if (!list_contains(L, y, v)) out = list_add(L, out, v);
    }
    return out;
  }
  if ((kind == AR_OR || kind == AR_AND)) {
    if (tclass(x) != 9 || tclass(y) != 9) { lane_error(L); return UND; }
    uint32_t nx = coll_len(L, x), ny = coll_len(L, y);
    uint64_t out = list_new(L, LK_SET, nx + ny);
    if (vtag(out) == V_UNDEF) return UND;
    for (uint32_t i = 0; i < nx; ++i) {
      uint64_t k, v;
      coll_at(L, x, i, k, v);
      if (kind == AR_OR || list_contains(L, y, v)) out = list_add(L, out, v);
    }
    if (kind == AR_OR)
      for (uint32_t i = 0; i < ny; ++i) { uint64_t k, v; coll_at(L, y, i, k, v); out = list_add(L, out, v); }
    return out;
  }
  if (!is_numv(x) || !is_numv(y)) { lane_error(L); return UND; }
  int64_t a, b;
  bool ints = num_int(L, x, a) && num_int(L, y, b);
  const int64_t LIM = (1ll << 46);
  switch (kind) {
    case AR_PLUS: if (ints && a < LIM && a > -LIM && b < LIM && b > -LIM) return mkint_g(a + b); break;
    case AR_MINUS: if (ints && a < LIM && a > -LIM && b < LIM && b > -LIM) return mkint_g(a - b); break;
    case AR_MUL: {
      // an integer product below 2^46 in magnitude is exact at any precision the
      // big.Float Mul rounds to (64-bit mantissa), so it stays a heap-free V_INT
      // (memoizable; e.g. to_number("1") * mem_multiple("Gi") = 2^30)
      if (ints && a < LIM && a > -LIM && b < LIM && b > -LIM) {
        uint64_t ua = a < 0 ? (uint64_t)(-a) : (uint64_t)a, ub = b < 0 ? (uint64_t)(-b) : (uint64_t)b;
        if (__umul64hi(ua, ub) == 0 && ua * ub < (uint64_t)LIM) return mkint_g(a * b);
      }
      BF p, q;
      if (!num_bf(L, x, p) || !num_bf(L, y, q)) { lane_fallback(L, FB_NUMBER); return UND; }
      return heap_bf(L, bf_mul(p, q));
    }
    case AR_REM: {
      if (!ints) { lane_error(L); return UND; }
      if (b == 0) { lane_error(L); return UND; }
      return mkint(a % b);
    }
    default: break;
  }
  lane_fallback(L, FB_NUMBER);
  return UND;
}

// ------------------------------------------------------------------ sprintf
__device__ __noinline__ uint64_t do_sprintf(PLane& L, uint32_t fidx, uint64_t args) {
  const uint32_t* f = gk_args.fmt + fidx;
  uint32_t want = f[1];
  if (tclass(args) != 7) { lane_error(L); return mkv(V_UNDEF, 0); }
  uint32_t nargs = coll_len(L, args);
  if (nargs != want) { lane_fallback(L, FB_PRINT); return mkv(V_UNDEF, 0); }
  Out o{L.B + L.bp, 0, (uint32_t)(BCAP - L.bp), false};
  bool ok = fmt_run(L, o, fidx, [&](uint32_t i) { uint64_t k, v; coll_at(L, args, i, k, v); return v; });
  if (!ok) { lane_fallback(L, FB_PRINT); return mkv(V_UNDEF, 0); }
  if (o.ovf) { lane_fallback(L, FB_MSG_LEN); return mkv(V_UNDEF, 0); }
  uint32_t start = L.bp;
  L.bp += o.n;
  return mkhstr(start, o.n);
}

// Deferred sprintf (template kernels): the message is not built in the lane
// buffer; the value records (format, argument array).  An emission hands the
// record to the format pass (kernels.hip), which prints it into the output
// bytes; anywhere else that reads the value forces it into the lane buffer
// first (jit.cc inserts force_fmt).
// The argument array is the heap list / document array sprintf received, so a
// V_FMT lives exactly as long as that array (heap_val: pinned like a list).
__device__ __forceinline__ uint64_t fmt_args(uint64_t f) {
  uint64_t p = vpay(f);
  uint32_t lo = (uint32_t)p;
  return (lo >> 31) ? mkv(V_NODE, lo & 0x7fffffffu) : mklist(LK_ARR, lo);
}
__device__ __forceinline__ uint32_t fmt_fidx(uint64_t f) { return (uint32_t)(vpay(f) >> 32) & 0xffffffu; }

__device__ __forceinline__ uint64_t lazy_sprintf(PLane& L, uint32_t fidx, uint64_t args) {
  if (tclass(args) != 7) { lane_error(L); return mkv(V_UNDEF, 0); }
  uint32_t t = vtag(args);
  if ((t == V_LIST && list_kind(args) != LK_ARR) || t == V_ROWS) return do_sprintf(L, fidx, args);
  uint32_t idx = t == V_NODE ? ((uint32_t)vpay(args) | 0x80000000u) : list_off(args);
  if (t == V_NODE && (uint32_t)vpay(args) >= 0x80000000u) return do_sprintf(L, fidx, args);
  if (coll_len(L, args) != gk_args.fmt[fidx + 1]) { lane_fallback(L, FB_PRINT); return mkv(V_UNDEF, 0); }
  return mkv(V_FMT, ((uint64_t)fidx << 32) | idx);
}

// lazy_sprintf with the format's argument count known at compile time (jit.cc)
__device__ __forceinline__ uint64_t lazy_sprintf_n(PLane& L, uint32_t fidx, uint64_t args, uint32_t want) {
  if (tclass(args) != 7) { lane_error(L); return mkv(V_UNDEF, 0); }
  uint32_t t = vtag(args);
  if ((t == V_LIST && list_kind(args) != LK_ARR) || t == V_ROWS) return do_sprintf(L, fidx, args);
  uint32_t idx = t == V_NODE ? ((uint32_t)vpay(args) | 0x80000000u) : list_off(args);
  if (t == V_NODE && (uint32_t)vpay(args) >= 0x80000000u) return do_sprintf(L, fidx, args);
  if (coll_len(L, args) != want) { lane_fallback(L, FB_PRINT); return mkv(V_UNDEF, 0); }
  return mkv(V_FMT, ((uint64_t)fidx << 32) | idx);
}

// the string a deferred sprintf denotes, built in the lane buffer
__device__ uint64_t force_fmt(PLane& L, uint64_t v) {
  if (vtag(v) != V_FMT) return v;
  return do_sprintf(L, fmt_fidx(v), fmt_args(v));
}

// ------------------------------------------------------------------ ops
// Per-instruction semantics (OP_* in common.h).  The VM dispatches to these
// from its switch; the JIT emits one call per instruction with register
// operands bound to locals.  A `false` return means "leave the program".
__device__ __forceinline__ void op_iter_init(PLane& L, uint64_t& it, uint64_t& st, uint64_t coll, uint32_t y) {
  it = coll;
  st = ((uint64_t)L.hp << 32) | ((uint64_t)L.bp << 48);
  uint32_t d = y < MAXLOOP ? y : 0;
  L.keepH[d] = 0;
  L.keepB[d] = 0;
}

// advances the iterator; false when exhausted (jump to the loop exit)
__device__ __forceinline__ bool op_iter_next(PLane& L, uint64_t coll, uint64_t& st, uint32_t y,
                                             uint64_t& k, uint64_t& v) {
  uint32_t pos = (uint32_t)st;
  // per-iteration reclamation: everything allocated by the previous
  // iteration is dead unless it escaped this loop
  uint32_t d = y < MAXLOOP ? y : 0;
  uint32_t mh = (uint32_t)((st >> 32) & 0xffff), mb = (uint32_t)(st >> 48);
  L.hp = mh > L.keepH[d] ? mh : L.keepH[d];
  L.bp = mb > L.keepB[d] ? mb : L.keepB[d];
  uint32_t t = vtag(coll);
  if ((t != V_NODE && t != V_LIST && t < V_ROW) || pos >= coll_len(L, coll)) return false;
  coll_at(L, coll, pos, k, v);
  st = (st & 0xffffffff00000000ull) | (pos + 1);
  return true;
}

// ------------------------------------------------------------------ inventory joins
// A join key's bucket: equal Rego values (ast.Compare == 0) get equal hashes.
// Strings hash their bytes (whatever the representation); every number falls
// in one bucket (1 == 1.0); composite values get none (KH_NONE: a composite
// key never equals a scalar probe, and a composite probe takes the scan path).
__device__ __forceinline__ uint64_t key_hash(const PLane& L, uint64_t v) {
  const uint32_t t = vtag(v);
  if (is_strv(v)) {
    const SView s = sview(L, v);
    uint64_t h = 1469598103934665603ull;
    for (uint32_t i = 0; i < s.n; ++i) { h ^= (uint8_t)s.p[i]; h *= 1099511628211ull; }
    return h | (1ull << 63);
  }
  if (t == V_NUM || t == V_INT || t == V_BFN) return KH_NUM;
  if (t == V_NULL) return KH_NULL;
  if (t == V_BOOL) return vpay(v) ? KH_TRUE : KH_FALSE;
  return KH_NONE;
}

// key pass: the leaf's next key value (the lane's emission counter counts
// them; a value past JKEYS_MAX fails the lane, and with it the index). A
// composite key value has no bucket and takes no slot: KH_NONE pads the unused
// slots, and the host stops reading a leaf's keys at the first one.
__device__ __forceinline__ void op_keyout(PLane& L, uint64_t v) {
  if (!gk_args.jkeys) return;
  const uint64_t h = key_hash(L, v);
  if (h == KH_NONE) return;
  const uint32_t j = L.en;
  if (j >= JKEYS_MAX) { lane_fallback(L, FB_HEAP); return; }
  L.en = j + 1;
  gk_args.jkeys[(uint64_t)L.rv * JKEYS_MAX + j] = h;
}

// opens a probe of the lane's constraint's index `site` (y >> 8) for R[b]:
// it = [lo, hi) of the matching hash entries; false when there is no index or
// the probe value has no bucket (the caller runs the plain scan instead)
__device__ __forceinline__ bool op_jprobe(PLane& L, uint64_t& it, uint64_t& st, uint64_t key, uint32_t y) {
  uint32_t d = (y & 0xff) < MAXLOOP ? (y & 0xff) : 0;
  L.keepH[d] = 0;
  L.keepB[d] = 0;
  st = ((uint64_t)L.hp << 32) | ((uint64_t)L.bp << 48);
  const uint32_t site = y >> 8;
  if (!gk_args.jdir || site >= JMAX_SITES) return false;
  const uint32_t* dir = gk_args.jdir + ((uint64_t)L.cn * JMAX_SITES + site) * 4;
  if (!dir[2]) return false;
  const uint64_t h = key_hash(L, key);
  if (h == KH_NONE) return false;
  uint32_t lo = dir[0], hi = dir[0] + dir[1];
  // lower bound of h
  uint32_t a = lo, b = hi;
  while (a < b) {
    const uint32_t m = (a + b) >> 1;
    if (gk_args.jhash[m] < h) a = m + 1; else b = m;
  }
  uint32_t e = a;
  while (e < hi && gk_args.jhash[e] == h) ++e;
  it = (uint64_t)a | ((uint64_t)e << 32);
  return true;
}

// next candidate leaf of a probe (per-iteration heap reclamation as op_iter_next)
__device__ __forceinline__ bool op_jnext(PLane& L, uint64_t it, uint64_t& st, uint32_t y, uint64_t& leaf) {
  const uint32_t pos = (uint32_t)st;
  const uint32_t d = y < MAXLOOP ? y : 0;
  const uint32_t mh = (uint32_t)((st >> 32) & 0xffff), mb = (uint32_t)(st >> 48);
  L.hp = mh > L.keepH[d] ? mh : L.keepH[d];
  L.bp = mb > L.keepB[d] ? mb : L.keepB[d];
  const uint32_t p = (uint32_t)it + pos;
  if (p >= (uint32_t)(it >> 32)) return false;
  leaf = gk_args.jleaf[gk_args.jord[p]];
  st = (st & 0xffffffff00000000ull) | (pos + 1);
  return true;
}

// the current candidate's key at path variable j
__device__ __forceinline__ uint64_t op_jvar(uint64_t it, uint64_t st, uint32_t j) {
  const uint32_t p = (uint32_t)it + (uint32_t)st - 1;
  return gk_args.jleaf[(uint64_t)gk_args.jord[p] + 1 + j];
}

#if GK_LDS_PARAMS
// op_iter_next over a collection the JIT proved parameter-derived
__device__ __forceinline__ bool op_iter_next_p(PLane& L, uint64_t coll, uint64_t& st, uint32_t y, uint64_t& k,
                                               uint64_t& v, uint32_t plo, uint32_t pn) {
  if (vtag(coll) != V_NODE) return op_iter_next(L, coll, st, y, k, v);
  const uint32_t pos = (uint32_t)st;
  const uint32_t d = y < MAXLOOP ? y : 0;
  const uint32_t mh = (uint32_t)((st >> 32) & 0xffff), mb = (uint32_t)(st >> 48);
  L.hp = mh > L.keepH[d] ? mh : L.keepH[d];
  L.bp = mb > L.keepB[d] ? mb : L.keepB[d];
  const uint32_t ci = (uint32_t)vpay(coll);
  const Node n = pnode(ci, plo, pn);
  if (pos >= n.n) return false;
  const uint32_t c = n.first + pos;
  const Node ch = pnode(c, plo, pn);
  v = nodeval_of(ch, c);
  k = n.type == NT_OBJ ? mkv(V_STR, ch.key) : mkint(pos);
  st = (st & 0xffffffff00000000ull) | (pos + 1);
  return true;
}
#endif

__device__ __forceinline__ bool op_cmp(PLane& L, uint32_t kind, uint64_t x, uint64_t y, uint64_t& out) {
  if (vtag(x) == V_UNDEF || vtag(y) == V_UNDEF) { out = mkv(V_UNDEF, 0); return true; }
  int cr;
  // inlined fast paths (exact ints, interned strings, booleans); the rest of
  // ast.Compare is out of line in vcmp
  uint32_t tx = vtag(x), ty = vtag(y);
  if (tx == V_INT && ty == V_INT) {
    int64_t a = intof(x), b = intof(y);
    cr = a == b ? 0 : (a < b ? -1 : 1);
  } else if ((tx == V_STR && ty == V_STR && x == y) || (tx == V_BOOL && ty == V_BOOL && x == y)) {
    cr = 0;
  } else if (tx == V_STR && ty == V_STR && (kind == CMP_EQ || kind == CMP_NE)) {
    cr = 3;  // distinct interned ids: distinct bytes
  } else {
    cr = vcmp(L, x, y);
  }
  if (cr == 2) return false;
  if (cr == 3 && kind != CMP_EQ && kind != CMP_NE) { lane_fallback(L, FB_DEEP_EQ); return false; }
  bool res = false;
  switch (kind) {
    case CMP_EQ: res = cr == 0; break;
    case CMP_NE: res = cr != 0; break;
    case CMP_LT: res = cr < 0; break;
    case CMP_LE: res = cr <= 0; break;
    case CMP_GT: res = cr > 0; break;
    case CMP_GE: res = cr >= 0; break;
  }
  out = mkv(V_BOOL, res);
  return true;
}

__device__ __forceinline__ bool op_list_add(PLane& L, uint64_t& l, uint64_t v, uint32_t y) {
  l = list_add(L, l, v);
  if (L.fail) return false;
  if (y) pin_escape(L, y);
  return true;
}

__device__ __forceinline__ bool op_obj_put(PLane& L, uint64_t& o, uint64_t k, uint64_t v, uint32_t y) {
  uint32_t n = list_len(L, o);
  bool found = false;
  for (uint32_t i = 0; i + 1 < n; i += 2) {
    if (veq(L, list_at(L, o, i), k)) {
      found = true;
      if (!veq(L, list_at(L, o, i + 1), v)) { lane_error(L); return false; }
    }
  }
  if (!found) { o = list_add(L, o, k); o = list_add(L, o, v); }
  if (L.fail) return false;
  if (y) pin_escape(L, y);
  return true;
}

__device__ __forceinline__ bool op_yield(PLane& L, uint64_t& out, uint64_t v, uint32_t y) {
  if (vtag(out) != V_UNDEF) {
    if (vtag(out) == V_FMT || vtag(v) == V_FMT) { out = force_fmt(L, out); v = force_fmt(L, v); if (L.fail) return false; }
    if (!veq(L, out, v)) { lane_error(L); return false; }  // conflicting function/rule outputs
    if (L.fail) return false;
  } else {
    out = v;
    if (y && heap_val(v)) pin_escape(L, y);
  }
  return true;
}

__device__ __forceinline__ uint64_t op_len_eq(PLane& L, uint64_t v, uint32_t y) {
  uint32_t want = y & 0xffffff, kind = y >> 24;
  int cls = tclass(v);
  bool ok = (kind == LK_ARR ? cls == 7 : cls == 8) && coll_len(L, v) == want;
  return mkv(V_BOOL, ok);
}

// OP_ORD (compiler.cc rule_group): rule bodies that share their first
// expression are evaluated in one pass over its solutions, body after body for
// each solution; the reference evaluates them body by body (topdown
// evalOneRule per rule), so each fused body's emissions carry key base + j and
// the group's exit moves the base past them.  A tuple's order key is
// (key, the lane's emission index) (next_seq), which sorts the lane's
// emissions in the reference's order.
__device__ __forceinline__ void op_ord(PLane& L, uint32_t y) {
  const uint32_t k = (uint32_t)L.ord_base + (y & 0x7fffffffu);
  if (k > 0xffffu) { lane_fallback(L, FB_MSG_LEN); return; }
  if (y & 0x80000000u) L.ord_base = (uint16_t)k;
  L.ord = (uint16_t)k;
}

// f("k1") = v1 {true} ... compiled to a table (compiler.cc table_func): the
// value of the (at most one) entry whose key equals the argument, else undefined
__device__ __forceinline__ uint64_t op_table(PLane& L, const uint64_t* T, uint64_t arg) {
  if (vtag(arg) == V_UNDEF) return mkv(V_UNDEF, 0);
  uint32_t n = (uint32_t)T[0];
  for (uint32_t i = 0; i < n; ++i)
    if (veq(L, T[1 + 2 * i], arg)) return T[2 + 2 * i];
  return mkv(V_UNDEF, 0);
}

// Function-call memo (compiler.cc memo_slot): within one lane a Rego function's
// value depends only on its arguments (templates with `with` fall back), so a
// call with the same arguments may reuse the last value.  Only heap-free values
// are keys or results: lane-heap lists / computed strings / big floats can be
// reclaimed and their handles reused by different contents.
__device__ __forceinline__ bool memo_stable(uint64_t v) {
  uint32_t t = vtag(v);
  return t != V_LIST && t != V_HSTR && t != V_BFN && t != V_FMT;
}

// Cross-lane memo of pure function calls (compiler.cc pure_func: no input,
// data or rule references anywhere under the function).  Such a call's value
// depends only on its heap-free arguments, so every lane of the launch may
// share it: canonify_mem("1Gi") is computed by the first lanes that meet it and
// read by the rest.  Entries are (k0, k1, value, check) with check a hash of
// (call site, key, value); a reader accepts an entry only if key and check
// match, so torn or racing writes, stale cache lines and collisions all read
// as misses (the lane then evaluates the call itself).  No atomics or fences:
// equal keys always carry equal values.  Cleared before each launch.
__device__ __forceinline__ uint64_t gm_mix(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 27; x *= 0x94d049bb133111ebull; x ^= x >> 31;
  return x;
}
// Two 64-bit multiplies for the slot hash and one for the check (the
// splitmix-style pair per word cost ~150 VALU instructions per probe): the
// check is a bijection of h ^ v, so any torn or foreign (key, value) pair
// that differs from the reader's reads as a miss.  A real key is never 0
// (every tagged value but undefined is non-zero), so empty entries never match.
__device__ __forceinline__ uint64_t gm_hash(uint32_t site, uint64_t k0, uint64_t k1) {
  uint64_t h = (k0 ^ ((uint64_t)(site + 1) << 44) ^ gk_args.gm_salt) * 0x9e3779b97f4a7c15ull;
  h ^= h >> 29;
  h += k1 * 0xbf58476d1ce4e5b9ull;
  return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t gm_check(uint64_t h, uint64_t v) {
  return (h ^ v) * 0x94d049bb133111ebull + 0x632be59bd9b4e019ull;
}
// keys are scalars and permanent nodes (constraint parameters, data.inventory
// objects: every lane of the launch meets the same ones, e.g. the Services a
// unique-selector join scans); a review document's node is met by one lane
// only and would just evict shared entries
__device__ __forceinline__ bool gm_key(uint64_t v) {
  return vtag(v) == V_NODE ? (uint32_t)vpay(v) < gk_args.nperm : vtag(v) < V_ROW && memo_stable(v);
}
// a memo value: heap-free as it is, or a lane-buffer string copied into the
// evaluation's memo-string arena (V_GSTR); 0 = not memoizable.  Each string
// gets cache lines of its own (128-B aligned), written and fenced before the
// memo entry that names it is stored: a reader on another CU learns the
// offset only from that entry, so its L1 cannot hold an older copy of the
// line (offsets are never reused within an evaluation; L1 is invalidated at
// every launch).
__device__ __noinline__ uint64_t gm_value_slow(const PLane& L, uint64_t v) {
  if (vtag(v) != V_HSTR || !gk_args.mstr) return 0;
  const SView s = sview(L, v);
  if (s.n > 0xfffff) return 0;
  const unsigned long long need = ((unsigned long long)s.n + 127) & ~127ull;
  const unsigned long long at = atomicAdd(gk_args.mstr_top, need ? need : 128ull);
  if (at + s.n > gk_args.mstr_cap) return 0;
  for (uint32_t i = 0; i < s.n; ++i) gk_args.mstr[at + i] = s.p[i];
  __threadfence();
  return mkv(V_GSTR, ((uint64_t)at << 20) | s.n);
}

#if GK_LDS_MEMO && !defined(GK_HOST)
__device__ __forceinline__ uint64_t* lds_memo_entry(uint64_t h) {
  return gk_lds_memo[threadIdx.x >> 6][(uint32_t)(h >> 40) & (GK_LDS_MEMO - 1)];
}
__device__ __forceinline__ void lds_memo_put(uint64_t h, uint64_t k0, uint64_t k1, uint64_t v, uint64_t c) {
  uint64_t* le = lds_memo_entry(h);
  le[0] = k0; le[1] = k1; le[2] = v; le[3] = c;
}
#endif

__device__ __forceinline__ bool gm_get(uint32_t site, uint64_t k0, uint64_t k1, uint64_t& out) {
  if (!gk_args.gmemo || !gm_key(k0) || !gm_key(k1)) return false;
  uint64_t h = gm_hash(site, k0, k1);
#if GK_LDS_MEMO && !defined(GK_HOST)
  {
    const uint64_t* le = lds_memo_entry(h);
    const uint64_t a = le[0], b = le[1], v = le[2], c = le[3];
    if (a == k0 && b == k1 && c == gm_check(h, v)) { out = v; return true; }
  }
#endif
  uint32_t i = (uint32_t)h & gk_args.gmemo_mask;
#pragma unroll
  for (uint32_t p = 0; p < 2; ++p) {
    const uint64_t* e = gk_args.gmemo + 4 * (i ^ p);
    uint64_t a = e[0], b = e[1], v = e[2], c = e[3];
    if (a == k0 && b == k1 && c == gm_check(h, v)) {
#if GK_LDS_MEMO && !defined(GK_HOST)
      lds_memo_put(h, a, b, v, c);
#endif
      out = v;
      return true;
    }
  }
  return false;
}

__device__ __forceinline__ void gm_put(const PLane& L, uint32_t site, uint64_t k0, uint64_t k1, uint64_t v) {
  if (L.fail || !gk_args.gmemo || !gm_key(k0) || !gm_key(k1)) return;
  if (!memo_stable(v) && (v = gm_value_slow(L, v)) == 0) return;
  uint64_t h = gm_hash(site, k0, k1);
  uint32_t i = (uint32_t)h & gk_args.gmemo_mask;
  if (gk_args.gmemo[4 * i + 3] != 0) i ^= 1;
  uint64_t* e = gk_args.gmemo + 4 * i;
  const uint64_t c = gm_check(h, v);
  e[0] = k0; e[1] = k1; e[2] = v; e[3] = c;
#if GK_LDS_MEMO && !defined(GK_HOST)
  lds_memo_put(h, k0, k1, v, c);
#endif
}

// ------------------------------------------------------------------ values copied out at emission
// A deferred message's argument or a details value that lives in the lane heap
// -- a set, array or object such as k8srequiredlabels' `missing` and
// {"missing_labels": missing} (demo/agilebank/templates/
// k8srequiredlabels_template.yaml:39-46) -- is copied out with its tuple
// instead of being printed into the lane's byte buffer: its words go to the
// emission's ebytes reservation as [len, 0, words...] and the tuple's frec word
// names them (V_GLIST); the size and format passes print it (coll_len /
// coll_at read V_GLIST).  Members must be heap-free (memo_stable: interned
// strings, numbers, document nodes) or, one level down, heap lists of such.
constexpr uint32_t GVAL_MAXWORDS = 64;
// words a copy of v takes (0: v is heap-free as it is); > GVAL_MAXWORDS: no copy
__device__ __forceinline__ uint32_t gval_words(const PLane& L, uint64_t v) {
  if (memo_stable(v)) return 0;
  if (vtag(v) != V_LIST) return GVAL_MAXWORDS + 1;
  const uint32_t n = list_len(L, v);
  uint32_t w = 2 + n;
  for (uint32_t i = 0; i < n && w <= GVAL_MAXWORDS; ++i) {
    const uint64_t e = list_at(L, v, i);
    if (memo_stable(e)) continue;
    if (vtag(e) != V_LIST) return GVAL_MAXWORDS + 1;
    const uint32_t m = list_len(L, e);
    w += 2 + m;
    for (uint32_t j = 0; j < m; ++j)
      if (!memo_stable(list_at(L, e, j))) return GVAL_MAXWORDS + 1;
  }
  return w;
}
// copies v (gval_words(v) words) to ebytes word `at` onwards; the heap-free value
__device__ __forceinline__ uint64_t gval_put(const PLane& L, uint64_t v, uint64_t* dst, uint32_t& at) {
  if (memo_stable(v)) return v;
  const uint32_t n = list_len(L, v), me = at;
  at += 2 + n;
  dst[me] = n;
  dst[me + 1] = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t e = list_at(L, v, i);
    if (memo_stable(e)) { dst[me + 2 + i] = e; continue; }
    const uint32_t m = list_len(L, e), ce = at;
    at += 2 + m;
    dst[ce] = m;
    dst[ce + 1] = 0;
    for (uint32_t j = 0; j < m; ++j) dst[ce + 2 + j] = list_at(L, e, j);
    dst[me + 2 + i] = mkv(V_GLIST, ((uint64_t)list_kind(e) << 56) | ce);
  }
  return mkv(V_GLIST, ((uint64_t)list_kind(v) << 56) | me);
}

// m: message register, d: details register (undefined when absent).  Every
// active lane at the emission site calls it (the output reservations are
// wave-level); a lane that already failed emits nothing.
__device__ __noinline__ bool op_emit_slow(PLane& L, uint64_t m, uint64_t d, uint32_t depth, uint32_t rule) {
  bool ok = !L.fail;
  bool defer = false;
  uint32_t fidx = 0, n = 0, gw = 0;
  uint64_t args = 0;
  if (ok && vtag(m) == V_FMT) {
    // a deferred message whose arguments are heap-free (or copied out,
    // gval_words) goes to the format pass as its record -- it outlives this
    // iteration's heap; otherwise it is built in the lane buffer now
    args = fmt_args(m);
    fidx = fmt_fidx(m);
    n = coll_len(L, args);
    defer = n <= FMT_MAXARGS;
    for (uint32_t i = 0; i < n && defer; ++i) {
      uint64_t k, v;
      coll_at(L, args, i, k, v);
      gw += gval_words(L, v);
      defer = gw <= GVAL_MAXWORDS;
    }
    if (!defer) { m = force_fmt(L, m); ok = !L.fail; gw = 0; }
  }
  if (ok && !defer && !is_strv(m)) { lane_error(L); ok = false; }  // types.Result.msg must unmarshal as a string
  // details: a value the passes print as JSON (VF_DET_VAL, in the frec word
  // after the message's arguments), else JSON in the lane buffer above
  // everything live (not kept: copied out below)
  const char* det = nullptr;
  uint32_t dlen = 2, dw = 0;
  bool dval = false;
  const uint32_t di = defer ? n : 0u;
  if (ok && vtag(d) != V_UNDEF) {
    if (di < FMT_MAXARGS) {
      dw = gval_words(L, d);
      dval = gw + dw <= GVAL_MAXWORDS;
    }
    if (!dval) {
      dw = 0;
      Out o{L.B + L.bp, 0, (uint32_t)(BCAP - L.bp), false};
      if (!put_json(L, o, d) || o.ovf) { lane_fallback(L, o.ovf ? FB_MSG_LEN : FB_PRINT); ok = false; }
      else if (!(o.n == 2 && o.p[0] == '{' && o.p[1] == '}')) { det = o.p; dlen = o.n; }
    }
  }
  SView ms{nullptr, 0};
  if (ok && !defer) ms = sview(L, m);
  uint32_t seq = 0;
  if (ok) ok = next_seq(L, seq);
  const uint32_t sb = ok ? (defer ? 0u : ms.n) + (det ? dlen : 0u) : 0u;  // staged bytes
  const uint32_t words = ok ? gw + dw : 0u;                               // copied-out words (8-B aligned)
  const uint32_t eb = sb + (words ? 8u * words + 7u : 0u);
  const uint64_t eoff = bytes_reserve(ok, eb);
  const uint64_t slot = slot_reserve(ok);
  if (!ok) return false;
  L.en = L.en + 1u;
  if (slot >= gk_args.out_cap || eoff + eb > gk_args.ebytes_cap) { slot_overflow(L); return true; }
  if (!defer) copy_out(eoff, ms.p, ms.n);
  if (det) copy_out(eoff + (defer ? 0u : ms.n), det, dlen);
  uint64_t* gdst = (uint64_t*)gk_args.ebytes;
  uint32_t at = (uint32_t)((eoff + sb + 7) >> 3);
  Viol v;
  v.review = L.rv;
  v.constraint = L.cn;
  v.seq = (uint16_t)seq;
  v.rule = (uint16_t)rule;
  v.msg_len = defer ? (fidx | (n << 24)) : ms.n;
  v.msg_off = eoff;
  v.det_len = dval ? 0u : dlen;
  v.pad = (defer ? VF_DEFER : 0u) | (dval ? VF_DET_VAL : det ? 0u : VF_DET_OBJ);
  gk_args.out[slot] = v;
  if (defer)
    for (uint32_t i = 0; i < n; ++i) {
      uint64_t k, a;
      coll_at(L, args, i, k, a);
      gk_args.frec[(uint64_t)i * gk_args.out_cap + slot] = gval_put(L, a, gdst, at);
    }
  if (dval) gk_args.frec[(uint64_t)di * gk_args.out_cap + slot] = gval_put(L, d, gdst, at);
  return true;
}

// Emission fast path, inlined at every emission site: a deferred sprintf
// message without details whose arguments are plain scalars (interned
// strings, ints) -- the common case -- is written as its 32-B tuple and its
// argument words, nothing else: no bytes, no sizing (the size pass prints
// its length, kernels.hip).  Lanes on other paths take op_emit_slow, which
// is out of line: a call saves and restores the predicate's live VGPRs in
// scratch.
#ifndef GK_EMIT_FAST
#define GK_EMIT_FAST 1
#endif
// GK_EMIT_WIDE (GKGPU_JIT_PRE=GK_EMIT_WIDE=0 turns it off): every heap-free
// argument (numbers, booleans, document and parameter nodes such as
// k8sallowedrepos' input.parameters.repos) on the fast path, not only
// interned strings and ints (profiles/r05/r05ah_prealloc_wide_ab.txt: config 4
// 1,995 -> 2,038 M evals/s).  Round 5 saw it lose rows: a miscompile cleared by
// -amdgpu-prealloc-sgpr-spill-vgprs (jit.cc kOpts).
#ifndef GK_EMIT_WIDE
#define GK_EMIT_WIDE 1
#endif
__device__ __forceinline__ bool plain_scalar(uint64_t v) {
#if GK_EMIT_WIDE
  return memo_stable(v) && vtag(v) != V_UNDEF && vtag(v) < V_ROW;
#else
  return vtag(v) == V_STR || vtag(v) == V_INT;
#endif
}
// Details the fast path carries: none (the hook default), or a one-member
// object whose key is an interned string and whose value is heap-free
// (VF_DET_KV: two frec words, no staged bytes, no out-of-line call)
#ifndef GK_DET_KV
#define GK_DET_KV 1  // A/B: GKGPU_JIT_PRE=GK_DET_KV=0
#endif
__device__ __forceinline__ bool det_fast(PLane& L, uint64_t d, bool& kv, uint64_t& dk, uint64_t& dv) {
  kv = false;
  if (vtag(d) == V_UNDEF) return true;
  if (!GK_DET_KV) return false;
  if (tclass(d) != 8 || coll_len(L, d) != 1) return false;
  coll_at(L, d, 0, dk, dv);
  kv = vtag(dk) == V_STR && plain_scalar(dv);
  return kv;
}
__device__ __forceinline__ void det_fast_put(Viol& v, bool kv, uint64_t slot, uint32_t n, uint64_t dk, uint64_t dv) {
  v.det_len = kv ? 0u : 2u;
  v.pad = VF_DEFER | (kv ? VF_DET_KV : VF_DET_OBJ);
  if (kv) {
    gk_args.frec[(uint64_t)n * gk_args.out_cap + slot] = dk;
    gk_args.frec[(uint64_t)(n + 1) * gk_args.out_cap + slot] = dv;
  }
}

__device__ __forceinline__ bool op_emit(PLane& L, uint64_t m, uint64_t d, uint32_t depth, uint32_t rule) {
#if GK_EMIT_FAST
  bool fast = false, kv = false;
  uint32_t n = 0, seq = 0;
  uint64_t args = 0, dk = 0, dv = 0;
  if (vtag(m) == V_FMT && !L.fail && L.en < EM_MAXIDX && L.ord < EM_MAXORD && det_fast(L, d, kv, dk, dv)) {
    args = fmt_args(m);
    if (vtag(args) == V_LIST) {
      n = list_len(L, args);
      fast = n + (kv ? 2u : 0u) <= FMT_MAXARGS;
      for (uint32_t i = 0; i < n && fast; ++i) fast = plain_scalar(list_at(L, args, i));
    }
  }
  if (fast) {
    seq = ((uint32_t)L.ord << 8) | (uint32_t)L.en;
    const uint64_t slot = slot_reserve(true);
    L.en = L.en + 1u;
    if (slot >= gk_args.out_cap) { slot_overflow(L); return true; }
    Viol v;
    v.review = L.rv;
    v.constraint = L.cn;
    v.seq = (uint16_t)seq;
    v.rule = (uint16_t)rule;
    v.msg_len = fmt_fidx(m) | (n << 24);
    v.msg_off = 0;
    det_fast_put(v, kv, slot, n, dk, dv);
    gk_args.out[slot] = v;
    for (uint32_t i = 0; i < n; ++i) gk_args.frec[(uint64_t)i * gk_args.out_cap + slot] = list_at(L, args, i);
    return true;
  }
#endif
  return op_emit_slow(L, m, d, depth, rule);
}

// the fast path's record: the tuple and its argument (and details) words
template <uint32_t N>
__device__ __forceinline__ bool emit_fast_write(PLane& L, uint64_t m, uint32_t rule, const uint64_t (&args)[N], bool kv,
                                                uint64_t dk, uint64_t dv) {
  const uint32_t seq = ((uint32_t)L.ord << 8) | (uint32_t)L.en;
  const uint64_t slot = slot_reserve(true);
  L.en = L.en + 1u;
  if (slot >= gk_args.out_cap) { slot_overflow(L); return true; }
  Viol v;
  v.review = L.rv;
  v.constraint = L.cn;
  v.seq = (uint16_t)seq;
  v.rule = (uint16_t)rule;
  v.msg_len = fmt_fidx(m) | (N << 24);
  v.msg_off = 0;
  det_fast_put(v, kv, slot, N, dk, dv);
  gk_args.out[slot] = v;
#pragma unroll
  for (uint32_t i = 0; i < N; ++i) gk_args.frec[(uint64_t)i * gk_args.out_cap + slot] = args[i];
  return true;
}

// op_emit for a deferred message whose argument registers the JIT knows
// (jit.cc emit_flow): the same record, the argument words taken from the
// registers instead of the lane heap's list
template <uint32_t N>
__device__ __forceinline__ bool op_emit_args(PLane& L, uint64_t m, uint64_t d, uint32_t depth, uint32_t rule,
                                             const uint64_t (&args)[N]) {
#if GK_EMIT_FAST
  bool kv = false;
  uint64_t dk = 0, dv = 0;
  bool fast = N <= FMT_MAXARGS && vtag(m) == V_FMT && !L.fail && L.en < EM_MAXIDX && L.ord < EM_MAXORD &&
              det_fast(L, d, kv, dk, dv) && N + (kv ? 2u : 0u) <= FMT_MAXARGS;
#pragma unroll
  for (uint32_t i = 0; i < N; ++i) fast = fast && plain_scalar(args[i]);
  if (fast) return emit_fast_write(L, m, rule, args, kv, dk, dv);
  // the list holds these same arguments: op_emit's fast path would fail too
  return op_emit_slow(L, m, d, depth, rule);
#else
  return op_emit(L, m, d, depth, rule);
#endif
}

// (out of line: the argument list is built only where an argument is not
// heap-free.  Arguments by value and the LIST_ADD escape ranges packed 16
// bits each: an array passed by address would be stored to the private
// segment at every emission, fast path included -- 0.4 GB of writes per
// K8sContainerLimits launch, profiles/r05/)
__device__ __forceinline__ uint64_t sel6(uint32_t i, uint64_t a0, uint64_t a1, uint64_t a2, uint64_t a3, uint64_t a4,
                                         uint64_t a5) {
  return i == 0 ? a0 : i == 1 ? a1 : i == 2 ? a2 : i == 3 ? a3 : i == 4 ? a4 : a5;
}
// an escape range (pin_escape: lo | hi << 8) packed in 10 bits as lo | hi << 5
__device__ __forceinline__ uint32_t esc_unpack(uint32_t p) { return (p & 0x1fu) | (((p >> 5) & 0x1fu) << 8); }
__device__ __noinline__ bool op_emit_build_slow(PLane& L, uint64_t m, uint64_t d, uint32_t depth, uint32_t rule,
                                                uint32_t n, uint64_t ys, uint64_t a0, uint64_t a1, uint64_t a2,
                                                uint64_t a3, uint64_t a4, uint64_t a5) {
  uint64_t l = list_new(L, LK_ARR, 4);
  for (uint32_t i = 0; i < n; ++i)
    if (!op_list_add(L, l, sel6(i, a0, a1, a2, a3, a4, a5), esc_unpack((uint32_t)(ys >> (10 * i)) & 0x3ffu)))
      return false;
  const uint64_t m2 = lazy_sprintf_n(L, fmt_fidx(m), l, n);
  if (L.fail) return false;
  return op_emit_slow(L, m2, d, depth, rule);
}

// op_emit_args for a sprintf whose argument list the JIT did not build
// (jit.cc dce_sites): the value carries the format only, so the slow path
// builds the list from the arguments first (the same LIST_ADDs the program
// would have run; ys: their escape ranges, 10 bits each)
template <uint32_t N>
__device__ __forceinline__ bool op_emit_args_build(PLane& L, uint64_t m, uint64_t d, uint32_t depth, uint32_t rule,
                                                   const uint64_t (&args)[N], uint64_t ys) {
  static_assert(N <= 6, "fused emissions take up to six arguments");
  bool kv = false;
  uint64_t dk = 0, dv = 0;
  bool fast = N <= FMT_MAXARGS && vtag(m) == V_FMT && !L.fail && L.en < EM_MAXIDX && L.ord < EM_MAXORD &&
              det_fast(L, d, kv, dk, dv) && N + (kv ? 2u : 0u) <= FMT_MAXARGS;
#pragma unroll
  for (uint32_t i = 0; i < N; ++i) fast = fast && plain_scalar(args[i]);
  if (fast) return op_emit_args(L, m, d, depth, rule, args);
  if (vtag(m) != V_FMT) return op_emit_slow(L, m, d, depth, rule);
  return op_emit_build_slow(L, m, d, depth, rule, N, ys, args[0], N > 1 ? args[N > 1 ? 1 : 0] : 0,
                            N > 2 ? args[N > 2 ? 2 : 0] : 0, N > 3 ? args[N > 3 ? 3 : 0] : 0,
                            N > 4 ? args[N > 4 ? 4 : 0] : 0, N > 5 ? args[N > 5 ? 5 : 0] : 0);
}

// A fused emission whose details are the one-member object literal {k: v}
// built right before it (jit.cc kv_sites): the object is not built unless the
// fast path fails -- then exactly as the program would have (list_new +
// op_obj_put, escape range yput) before the general path.  BUILD: the message's
// argument list was not built either (op_emit_args_build).
template <bool BUILD, uint32_t N>
__device__ __forceinline__ bool op_emit_args_kvd(PLane& L, uint64_t m, uint64_t k, uint64_t v, uint32_t yput,
                                                 uint32_t depth, uint32_t rule, const uint64_t (&args)[N], uint64_t ys) {
  bool fast = GK_DET_KV && N + 2 <= FMT_MAXARGS && vtag(m) == V_FMT && !L.fail && L.en < EM_MAXIDX &&
              L.ord < EM_MAXORD && vtag(k) == V_STR && plain_scalar(v);
#pragma unroll
  for (uint32_t i = 0; i < N; ++i) fast = fast && plain_scalar(args[i]);
  if (fast) return emit_fast_write(L, m, rule, args, true, k, v);
  uint64_t d = list_new(L, LK_OBJ, 4);
  if (!op_obj_put(L, d, k, v, yput)) return false;
  if (BUILD) return op_emit_args_build(L, m, d, depth, rule, args, ys);
  return op_emit_args(L, m, d, depth, rule, args);
}

// Printed length of a deferred message whose arguments are plain scalars:
// put_fmt_arg restricted to interned strings and ints, on a counter (the size
// pass's fast path; fmt_run on a counter serves every other record).
__device__ __forceinline__ bool size_plain(uint32_t fidx, const uint64_t* args, uint32_t& len) {
  const uint32_t* f = gk_args.fmt + fidx;
  const uint32_t nseg = f[0];
  Cnt o{0, false};
  for (uint32_t s = 0; s < nseg; ++s) {
    const uint32_t kind = f[2 + 2 * s], a = f[3 + 2 * s];
    if (kind == 0) { put_sid(o, a); continue; }
    const uint32_t verb = a >> 16;
    const uint64_t v = args[a & 0xffff];
    if (vtag(v) == V_STR) {
      const uint32_t n = gk_args.strs[(uint32_t)vpay(v)].len;
      GK_TOUCH_STR((uint32_t)vpay(v));
      if (verb == 'd') { put_cstr(o, "%!d(string="); o.n += n; put(o, ')'); } else o.n += n;
    } else if (vtag(v) != V_INT) {
      return false;
    } else if (intv_gform(v)) {
      if (verb != 'v') return false;
      put_intv(o, v);
    } else if (verb == 's') {
      put_cstr(o, "%!s(int="); put_int(o, intof(v)); put(o, ')');
    } else {
      put_int(o, intof(v));
    }
  }
  len = o.n;
  return true;
}

// end of a lane's evaluation (all 64 lanes of the wave, reconverged): flag a
// failed review, add the wave's clean emissions to the constraint's total
__device__ __noinline__ void finish_lane(PLane& L, uint32_t lane, uint32_t c, bool live) {
  if (live && L.fail) {
    atomicAdd(&gk_args.counters[2], 1ull);
    atomicOr(&gk_args.rflags[L.rv], L.fail);
    if (gk_args.rreason) atomicMax(&gk_args.rreason[L.rv], L.reason);
  }
  uint32_t k = (live && !L.fail) ? (uint32_t)L.en : 0u;
#pragma unroll
  for (int dd = 32; dd >= 1; dd >>= 1) k += (uint32_t)__shfl_xor(k, dd, 64);
  if (lane == 0 && k) atomicAdd(&gk_args.totals[c], (unsigned long long)k);
}

// ------------------------------------------------------------------ kernel body
// lane -> (review tile, constraint): a wave = 64 consecutive reviews x ONE
// constraint of the launch's list, so every lane runs the same predicate and
// the constraint's MatchSpec loads are wave-uniform.  `run(L, review,
// params, prog, plo, pn)` evaluates the template predicate for a matched lane
// ([plo, plo + pn): the parameter nodes staged in LDS, template kernels).
template <typename Run>
__device__ __forceinline__ void audit_body(Run run) {
  uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t wave = (uint32_t)(gid >> 6);
  uint32_t lane = (uint32_t)(gid & 63);
  uint32_t c = gk_args.clist[wave % gk_args.nclist];
  uint32_t tile = wave / gk_args.nclist;
  if (tile >= gk_args.ntiles) return;  // wave-uniform
  uint32_t rp = tile * 64 + lane;  // position in the (size-ordered) review columns
  uint32_t r = rp;                   // the review's index in the caller's batch
  Lane L0;
  PLane& L = *(PLane*)&L0;
  // the lane scalars (LDS in template kernels); the private-segment fields
  // the predicate reads (loop watermarks, VM memo flags) are set only for a
  // matched lane, right before it runs: a scratch store is HBM write traffic
  // once the line leaves L2, and most lanes of a wide constraint set fail the
  // match
  L.hp = 0; L.bp = 0; L.ord = 0; L.ord_base = 0; L.fail = 0; L.reason = 0; L.en = 0; L.steps = 0;
  bool live = rp < gk_args.nrev;
  ReviewCol rc{};
  if (live) {
    rc = gk_args.revs[rp];
    if (rc.orig != NO_ID) r = rc.orig;
  }
  L.rv = r;
  L.cn = c;
  const MatchSpec m = gk_args.cons[c];
  stage_wave(m, lane);
#if GK_LDS_PARAMS
  const uint32_t plo = m.plo, pn = m.pn <= LDS_PCAP ? m.pn : 0;
#else
  const uint32_t plo = 0, pn = 0;
#endif
  // autoreject_review (target_template_source.go:12-25); hooks.violation only
  // (regolib src.go:7-20): the hooks.audit rule (src.go:45-62) has no such join
  const bool autorej = live && !(rc.flags & (RC_FALLBACK | RC_AUDIT)) && (m.flags & MF_HAS_NSSEL) && (rc.flags & RC_HAS_NS) &&
                       rc.ns != NO_ID && !(rc.flags & RC_NS_EMPTY) && !(rc.flags & RC_NS_CACHED) &&
                       !(rc.flags & RC_UNSTABLE_NS);
  if (__builtin_expect(gk_ballot(autorej) != 0, 0))
    emit_eager(L, autorej, RULE_AUTOREJECT, "Namespace is not cached in OPA.", 31, nullptr, 2);
  if (live) {
    if (rc.flags & RC_FALLBACK) {
      L.fail = RF_FALLBACK;
    } else {
      int mr = match_constraint(m, rc);
      if (mr == -1) L.fail = RF_ERROR;
      else if (mr == -2) L.fail = RF_FALLBACK;
      else if (mr == 1 && (m.flags & MF_FALLBACK)) lane_fallback(L, FB_TEMPLATE);  // template served by CPU OPA
      else if (mr == 1 && m.prog != NO_ID) {
        L.memo_ok = 0;
        for (int d = 0; d < GK_MAXDEPTH; ++d) { L.keepH[d] = 0; L.keepB[d] = 0; }
        uint64_t params = m.params == NO_ID ? mkv(V_NODE, 0) : nodeval(m.params);
        run(L, gk_args.cv_on ? mkv(V_ROW, (uint64_t)rp) : mkv(V_NODE, rc.root), params, m.prog, plo, pn);
      }
    }
  }
  // every lane of the wave reaches here (reconverged): flag failed reviews,
  // count the clean emissions
  finish_lane(L, lane, c, live);
#ifndef GK_HOST
  {
    // the wave's unused slots become holes; its slot count for the per-launch
    // tuple statistics (counters[6])
    unsigned long long* st = gk_lds_chunk[threadIdx.x >> 6];
    const uint64_t base = chunk_ld(&st[0]), left = chunk_ld(&st[1]), used = chunk_ld(&st[2]);
    mark_holes(base, left);
    if (lane == 0 && used) atomicAdd(&gk_args.counters[6], (unsigned long long)used);
  }
#endif
  if (gk_args.prof) {
    uint32_t mx = L.steps;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) { uint32_t o = __shfl_xor(mx, d, 64); mx = o > mx ? o : mx; }
    if (L.steps) {
      atomicAdd(&gk_args.prof[c * 4 + 0], (unsigned long long)L.steps);
      atomicMax(&gk_args.prof[c * 4 + 1], (unsigned long long)L.steps);
      atomicAdd(&gk_args.prof[c * 4 + 2], 1ull);
    }
    if (lane == 0) atomicAdd(&gk_args.prof[c * 4 + 3], (unsigned long long)mx);
  }
}

}  // namespace gk
