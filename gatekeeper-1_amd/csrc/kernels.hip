// MI355X (gfx950) audit kernel: resource x constraint matrix evaluation by a
// bytecode VM (the back end for templates without a JIT kernel, see jit.cc).
//
// One lane evaluates one (review, constraint) pair; a wavefront holds 64
// consecutive reviews x ONE constraint (devrt.h audit_body):
//   stage 1  match    — pkg/target/target_template_source.go:12-44 (autoreject +
//                       matching_constraints) from per-review match columns and
//                       the constraint's compiled MatchSpec;
//   stage 2  predicate — the template's `violation` bytecode (compiler.cc) run
//                       by the register VM below over the review document in HBM;
//   stage 3  compact  — violations staged per lane, one output reservation per
//                       wavefront (wave prefix sum); messages are formatted on
//                       the GPU (Go fmt / ast.Term.String rules).
#include <algorithm>

#include "devrt.h"

namespace gk {

constexpr int NREG = 192;

__device__ void run_program(PLane& L, uint32_t pc, uint64_t review, uint64_t params) {
  const uint64_t UND = mkv(V_UNDEF, 0);
  uint64_t R[NREG];
  for (int guard = 0; guard < (1 << 22); ++guard) {
    if (pc >= gk_args.ncode) { lane_fallback(L, FB_UNSUPPORTED); return; }
    const Ins in = gk_args.code[pc];
    ++pc;
    ++L.steps;
    if (gk_args.pchist) atomicAdd(&gk_args.pchist[pc - 1], 1u);
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

__global__ void __launch_bounds__(256) audit_kernel(DevArgs) {
  audit_body([&](PLane& L, uint64_t review, uint64_t params, uint32_t prog, uint32_t, uint32_t) {
    run_program(L, gk_args.prog_off[prog], review, params);
  });
}

// Key pass of an inventory join (engine.cc build_joins): one lane per leaf of
// the site's data.inventory iteration runs the site's key program (the body
// literals that derive the join key from the leaf, compiler.cc join_site) with
// the leaf as its input document and the constraint's parameters, and writes
// the bucket hash of each of the key's values (OP_KEYOUT; KH_NONE-padded, none
// when the key is undefined; KH_FAIL first when the program errs, needs the
// CPU or yields more than JKEYS_MAX values).
__global__ void __launch_bounds__(256) gk_key_kernel(DevArgs) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= gk_args.nrev) return;
  Lane L0;
  PLane& L = *(PLane*)&L0;
  L.hp = 0; L.bp = 0; L.ord = 0; L.ord_base = 0; L.fail = 0; L.reason = 0; L.en = 0; L.steps = 0; L.memo_ok = 0;
  for (int d = 0; d < MAXLOOP; ++d) { L.keepH[d] = 0; L.keepB[d] = 0; }
  L.rv = (uint32_t)i;
  L.cn = 0;
  for (uint32_t j = 0; j < JKEYS_MAX; ++j) gk_args.jkeys[i * JKEYS_MAX + j] = KH_NONE;
  run_program(L, gk_args.jpc, gk_args.jleaf[gk_args.jrow0 + i * gk_args.jstride], gk_args.jparams);
  if (L.fail) gk_args.jkeys[i * JKEYS_MAX] = KH_FAIL;
}

// LDS-staged writer for one wavefront's message bytes
struct LOut {
  uint8_t* p;
  uint32_t pos;
  __device__ __forceinline__ void put(char c) { p[pos++] = (uint8_t)c; }
  // n bytes of the dword array b starting at byte off (a format literal in
  // LDS): whole dwords where the destination is dword-aligned -- the bytes of
  // a lane's own range, so no neighbour's byte is touched -- single bytes at
  // the two ends.  A byte at a time cost ~5 VALU + one LDS store per byte.
  __device__ __forceinline__ void put_lit(const uint32_t* b, uint32_t off, uint32_t n) {
    uint8_t* d = p + pos;
    pos += n;
    while (n && ((uint32_t)(uintptr_t)d & 3u)) {
      *d++ = (uint8_t)(b[off >> 2] >> (8 * (off & 3)));
      ++off;
      --n;
    }
    const uint32_t sh = off & 3;
    for (; n >= 4; n -= 4, off += 4, d += 4) {
      const uint32_t lo = b[off >> 2];
      *(uint32_t*)d = sh ? __builtin_amdgcn_alignbyte(b[(off >> 2) + 1], lo, sh) : lo;
    }
    for (; n; --n, ++off) *d++ = (uint8_t)(b[off >> 2] >> (8 * (off & 3)));
  }
};
// LOut whose string sources are read in 16-B blocks (puts_wide below)
struct LOutW : LOut {};
// LDS staging of one window [w0, w0 + n) of the output: the printer runs
// whole, bytes outside the window are dropped (pos: output byte address)
struct WOut {
  uint8_t* p;
  int64_t rel;  // the next byte's offset from the window's start
  uint32_t n;
  __device__ __forceinline__ void put(char c) {
    if ((uint64_t)rel < n) p[rel] = (uint8_t)c;
    ++rel;
  }
  __device__ __forceinline__ void put_lit(const uint32_t* b, uint32_t off, uint32_t k) {
    for (; k; --k, ++off) put((char)(b[off >> 2] >> (8 * (off & 3))));
  }
};

// The format pass's byte sources (string pool, memo strings, staged bytes)
// read in aligned 16-B blocks: the printers are chains of dependent loads,
// and a dword at a time made a 60-byte message ~15 round trips.  An
// aligned block that holds one byte of the string never leaves its page, so
// reading the whole block is always in bounds.
template <class O> __device__ __forceinline__ void puts_wide(O& o, const char* s, uint32_t n) {
  if (!n) return;
  const uint64_t a = (uint64_t)s, e = a + n;
  uint32_t k = (uint32_t)(a & 15);
  for (uint64_t b = a & ~(uint64_t)15; b < e; b += 16, k = 0) {
    const uint4 q = *(const uint4*)b;
    const uint32_t lim = b + 16 <= e ? 16u : (uint32_t)(e - b);
    for (; k < lim; ++k) {
      const uint32_t w = k < 8 ? (k < 4 ? q.x : q.y) : (k < 12 ? q.z : q.w);
      o.put((char)(w >> (8 * (k & 3))));
    }
  }
}
__device__ __forceinline__ void puts_(LOutW& o, const char* s, uint32_t n) { puts_wide(o, s, n); }

__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) { uint32_t o = __shfl_xor(x, d, 64); x = o < x ? o : x; }
  return x;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) { uint32_t o = __shfl_xor(x, d, 64); x = o > x ? o : x; }
  return x;
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) { uint64_t o = __shfl_xor(x, d, 64); x = o < x ? o : x; }
  return x;
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) { uint64_t o = __shfl_xor(x, d, 64); x = o > x ? o : x; }
  return x;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

// Size + format passes over the tuples the predicate kernels wrote (devrt.h
// emission): every tuple's output bytes are its message followed by its
// details JSON, laid out in tuple order, so a tuple's byte offset is the
// exclusive prefix sum of the byte counts before it.
//   gk_size_kernel  — per tuple, its byte count (a deferred message is printed
//                     on a counter from its argument words); per tile of FTILE
//                     tuples, the tile's sum.  A deferred message that cannot be
//                     printed (a verb / argument the GPU printer does not
//                     reproduce) flags its review for the CPU fallback, as at
//                     emission time.
//   gk_scan_spine   — one block: exclusive prefix over the tile sums; the total
//                     (bytes of the whole output) in counters[3].
//   gk_format_kernel — per tile, a block-level prefix over its tuples gives each
//                     tuple's offset; a wavefront's 64 consecutive tuples fill one
//                     dense byte range, built in LDS and written back with
//                     coalesced dword stores (byte stores for the two edge dwords,
//                     which neighbouring wavefronts share).  The tuple is rewritten
//                     with its final (msg_off, msg_len, det_len).
// The tuple count is read on the device (counters[0]): the passes follow the
// predicate kernels on the stream with no host round trip.

__device__ __forceinline__ uint64_t ntuples() {
  const uint64_t n = gk_args.counters[0];
  return n < gk_args.out_cap ? n : gk_args.out_cap;
}

// ---- the resolved format table in LDS (DevArgs.fmtr / fmtb, engine.cc
// sync_tables).  The size and format passes print most messages from their
// format's literals and argument strings; with the table staged per block,
// a literal costs no global round trip (before: the format word, the string
// entry, then the pool bytes -- three dependent loads per segment), and the
// argument strings' entries are loaded together up front.
constexpr uint32_t FMTR_LDS = 1024, FMTB_LDS = 4096;
struct FmtLds {
  uint32_t r[FMTR_LDS];
  uint32_t b[FMTB_LDS / 4];
};
__shared__ FmtLds gk_fmt_lds;
// every thread of the block calls it; true when the table is staged
__device__ __forceinline__ bool fmt_stage() {
  const bool on = gk_args.fmtr && gk_args.nfmt <= FMTR_LDS && gk_args.nfmtb <= FMTB_LDS;  // block-uniform
  if (on) {
    for (uint32_t k = threadIdx.x; k < gk_args.nfmt; k += blockDim.x) gk_fmt_lds.r[k] = gk_args.fmtr[k];
    const uint32_t nb = (gk_args.nfmtb + 3) / 4;
    for (uint32_t k = threadIdx.x; k < nb; k += blockDim.x) gk_fmt_lds.b[k] = ((const uint32_t*)gk_args.fmtb)[k];
  }
  __syncthreads();
  return on;
}
// argument j of a tuple held in registers (an unrolled select: a dynamic index
// into a local array would put it in the private segment)
template <class T> __device__ __forceinline__ T sel_arg(const T (&a)[FMT_MAXARGS], uint32_t j) {
  T r = a[0];
#pragma unroll
  for (uint32_t k = 1; k < FMT_MAXARGS; ++k) r = j == k ? a[k] : r;
  return r;
}
// A deferred message whose sprintf arguments are interned strings (verbs v /
// s) or ints not printed in g-form (verbs v / d): the resolved table's
// segments, the strings' entries loaded once.  false: another printer.
__device__ __forceinline__ bool plain_args(const uint32_t* f, const uint64_t (&a)[FMT_MAXARGS], StrEnt (&se)[FMT_MAXARGS],
                                           uint32_t na) {
#pragma unroll
  for (uint32_t j = 0; j < FMT_MAXARGS; ++j) {
    se[j] = StrEnt{};
    if (j < na && vtag(a[j]) == V_STR) se[j] = gk_args.strs[(uint32_t)vpay(a[j])];
  }
  const uint32_t nseg = f[0];
  for (uint32_t s = 0; s < nseg; ++s) {
    const uint32_t w0 = f[2 + 2 * s], w1 = f[3 + 2 * s];
    if ((w0 & 0xff) == 0) continue;
    const uint32_t verb = w1 >> 16, j = w1 & 0xffff;
    if (j >= na) return false;
    const uint64_t v = sel_arg(a, j);
    if (vtag(v) == V_STR) { if (verb == 'd') return false; continue; }
    if (vtag(v) == V_INT && !intv_gform(v) && verb != 's') continue;
    return false;
  }
  return true;
}
template <class O>
__device__ __forceinline__ void print_plain_r(O& o, const uint32_t* f, const uint64_t (&a)[FMT_MAXARGS],
                                              const StrEnt (&se)[FMT_MAXARGS]) {
  const uint32_t nseg = f[0];
  for (uint32_t s = 0; s < nseg; ++s) {
    const uint32_t w0 = f[2 + 2 * s], w1 = f[3 + 2 * s];
    if ((w0 & 0xff) == 0) {
      // the literal's bytes from LDS (dword stores where aligned, LOut::put_lit)
      o.put_lit(gk_fmt_lds.b, w1, w0 >> 8);
      continue;
    }
    const uint32_t j = w1 & 0xffff;
    const uint64_t v = sel_arg(a, j);
    if (vtag(v) == V_STR) {
      const StrEnt e = sel_arg(se, j);
      puts_(o, (const char*)gk_args.pool + e.off, e.len);
    } else {
      put_int(o, intof(v));
    }
  }
}

// a deferred tuple's printed message length; false = not printable here
// (the string table's lengths: the resolved table staged in LDS measured
// slower here, 0.20 -> 0.27 ms per config-2 sweep, profiles/r05/)
__device__ __forceinline__ bool size_deferred_msg(PLane& L, const Viol& v, uint64_t i, uint32_t& len) {
  const uint32_t fidx = v.msg_len & 0xffffffu, na = v.msg_len >> 24;
  uint64_t a[FMT_MAXARGS];
#pragma unroll
  for (uint32_t j = 0; j < FMT_MAXARGS; ++j) a[j] = j < na ? gk_args.frec[(uint64_t)j * gk_args.out_cap + i] : 0;
  if (size_plain(fidx, a, len)) return true;
  Cnt cn{0, false};
  if (!fmt_run(L, cn, fidx, [&](uint32_t j) { return a[j]; })) return false;
  len = cn.n;
  return true;
}

// a tuple's details bytes: the hook default `{}`, staged bytes, or (VF_DET_VAL)
// the length the size pass printed and stored in det_len
__device__ __forceinline__ uint32_t det_bytes(const Viol& v) {
  return (v.pad & VF_NOPRINT) ? 0u : (v.pad & VF_DET_OBJ) ? 2u : v.det_len;
}
// VF_DET_VAL: the frec word holding the details value
__device__ __forceinline__ uint64_t det_word(const Viol& v, uint64_t i) {
  const uint32_t di = (v.pad & VF_DEFER) ? (v.msg_len >> 24) : 0u;
  return gk_args.frec[(uint64_t)di * gk_args.out_cap + i];
}
// Details printed from frec words: VF_DET_VAL the JSON of one value, VF_DET_KV
// {k: v} as encoding/json prints a one-key map (k an interned string).  One
// put_json site for both: a second inlined copy of the printer pushed the
// format pass past its registers (spills).
template <class O>
__device__ __forceinline__ bool put_det_words(PLane& L, O& o, uint32_t pad, uint64_t k, uint64_t val) {
  const bool kv = (pad & VF_DET_KV) != 0;
  if (kv) {
    put(o, '{');
    if (!put_json_str(o, sview(L, k))) return false;
    put(o, ':');
  }
  if (!put_json(L, o, val)) return false;
  if (kv) put(o, '}');
  return true;
}

// The lane the size / format passes hand to the printers.  Deferred arguments
// are heap-free values, so nothing reads it; a failing print only sets its
// fail word, which nobody reads either (the print's own result decides).  A
// module global instead of a local object: a local Lane put ~6 KB of private
// segment on every lane, and the dispatch paid for it (~1 ms fixed per call).
__device__ Lane gk_pass_lane;

__global__ void __launch_bounds__(256) gk_size_kernel(DevArgs) {
  __shared__ unsigned long long wsum[4];
  // an overflowed evaluation is re-run whole by the host: an emission that
  // found its slot but not its staged bytes left that slot unwritten, so the
  // tuples must not be read (the format pass returns here too)
  if (gk_args.counters[0] > gk_args.out_cap || gk_args.counters[1] > gk_args.ebytes_cap) return;
  PLane& L = *(PLane*)&gk_pass_lane;
  const uint64_t n = ntuples();
  const uint64_t ntile = (n + FTILE - 1) / FTILE;
  for (uint64_t t = blockIdx.x; t < ntile; t += gridDim.x) {
    unsigned long long s = 0;
    for (uint32_t k = 0; k < FTILE; k += 256) {
      const uint64_t i = t * FTILE + k + threadIdx.x;
      if (i >= n) break;
      const Viol v = gk_args.out[i];
      uint32_t ml = v.msg_len, dl = det_bytes(v);
      bool printable = true;
      if (v.pad & VF_DEFER) printable = size_deferred_msg(L, v, i, ml);
      if (v.pad & (VF_DET_VAL | VF_DET_KV)) {
        const uint64_t di = (v.pad & VF_DEFER) ? (v.msg_len >> 24) : 0u;
        const bool kv = (v.pad & VF_DET_KV) != 0;
        const uint64_t k = kv ? gk_args.frec[di * gk_args.out_cap + i] : 0ull;
        const uint64_t val = gk_args.frec[(di + (kv ? 1u : 0u)) * gk_args.out_cap + i];
        Cnt cn{0, false};
        printable = put_det_words(L, cn, v.pad, k, val) && printable;
        dl = cn.n;
        gk_args.out[i].det_len = dl;  // the format pass's det_bytes
      }
      if (!printable) {
        // the emission-time outcome: this review goes to CPU OPA; the tuple
        // gets no bytes (the format pass prints nothing for it, and every
        // consumer drops the rows of a flagged review)
        atomicOr(&gk_args.rflags[v.review], (uint32_t)RF_FALLBACK);
        if (gk_args.rreason) atomicMax(&gk_args.rreason[v.review], (uint32_t)FB_PRINT);
        atomicAdd(&gk_args.counters[2], 1ull);
        gk_args.out[i].pad = v.pad | VF_NOPRINT;
        ml = dl = 0;
      }
      const uint32_t len = ml + dl;
      gk_args.lens[i] = len;
      s += len;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) gk_args.part[t] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
}

__global__ void __launch_bounds__(1024) gk_scan_spine(DevArgs) {
  __shared__ unsigned long long wtot[16];
  const uint64_t n = ntuples();
  const uint64_t ntile = (n + FTILE - 1) / FTILE;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long carry = 0;
  for (uint64_t b = 0; b < ntile; b += 1024) {
    const uint64_t i = b + threadIdx.x;
    const unsigned long long x = i < ntile ? gk_args.part[i] : 0ull;
    unsigned long long incl = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    unsigned long long before = 0, all = 0;
    for (uint32_t k = 0; k < 16; ++k) {
      if (k < w) before += wtot[k];
      all += wtot[k];
    }
    if (i < ntile) gk_args.part[i] = carry + before + incl - x;
    carry += all;
    __syncthreads();
  }
  if (threadIdx.x == 0) gk_args.counters[3] = carry;
}

// ------------------------------------------------------------------ compaction
// The predicate kernels write tuples into per-wave chunks of slots (devrt.h
// slot_reserve); unused slots are holes (review = VIOL_HOLE).  These three
// kernels pack the tuples of all launches, and their deferred-argument words,
// into the dense arrays the size / format passes and the readback use:
//   count   -- per tile of 256 raw slots, its tuples;
//   scan    -- one block: exclusive prefix over the tiles; the dense count
//              becomes counters[0] (counters[5] keeps the raw slot count);
//   scatter -- each tuple to its dense slot, in raw order (a wave's tuples stay
//              together, as they did on one counter).
// Kernel arguments: DevArgs last (devrt.h gk_args finds it right before the
// hidden arguments).  An overflowed evaluation (raw slots or staged bytes past capacity) is
// re-run by the host with larger buffers: nothing is packed, counters[0]
// keeps the raw count the host checks.
constexpr uint32_t CTILE = 256;
__device__ __forceinline__ bool compact_overflow(uint64_t raw) {
  return raw > gk_args.out_cap || gk_args.counters[1] > gk_args.ebytes_cap;
}
__device__ __forceinline__ uint32_t frec_words(const Viol& v) {
  const uint32_t na = (v.pad & VF_DEFER) ? (v.msg_len >> 24) : 0u;
  return na + ((v.pad & VF_DET_VAL) ? 1u : (v.pad & VF_DET_KV) ? 2u : 0u);
}

__global__ void __launch_bounds__(256) gk_compact_count(const Viol* raw, uint32_t* tcnt, DevArgs) {
  const uint64_t n = gk_args.counters[0];
  if (blockIdx.x == 0 && threadIdx.x == 0) gk_args.counters[5] = n;
  if (compact_overflow(n)) return;
  const uint64_t ntile = (n + CTILE - 1) / CTILE;
  for (uint64_t t = blockIdx.x; t < ntile; t += gridDim.x) {
    const uint64_t i = t * CTILE + threadIdx.x;
    const bool real = i < n && raw[i].review != VIOL_HOLE;
    const int c = __syncthreads_count(real);
    if (threadIdx.x == 0) tcnt[t] = (uint32_t)c;
  }
}

__global__ void __launch_bounds__(1024) gk_compact_scan(const uint32_t* tcnt, unsigned long long* toff, DevArgs) {
  __shared__ unsigned long long wtot[16];
  __syncthreads();  // (counters[5] is written by the previous kernel)
  const uint64_t n = gk_args.counters[5];
  if (compact_overflow(n)) return;
  const uint64_t ntile = (n + CTILE - 1) / CTILE;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long carry = 0;
  for (uint64_t b = 0; b < ntile; b += 1024) {
    const uint64_t i = b + threadIdx.x;
    const unsigned long long x = i < ntile ? tcnt[i] : 0ull;
    unsigned long long incl = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    unsigned long long before = 0, all = 0;
    for (uint32_t k = 0; k < 16; ++k) {
      if (k < w) before += wtot[k];
      all += wtot[k];
    }
    if (i < ntile) toff[i] = carry + before + incl - x;
    carry += all;
    __syncthreads();
  }
  if (threadIdx.x == 0) gk_args.counters[0] = carry;
}

__global__ void __launch_bounds__(256) gk_compact_scatter(const Viol* raw, const uint64_t* rfrec,
                                                          const unsigned long long* toff, DevArgs) {
  __shared__ uint32_t wc[4];
  const uint64_t n = gk_args.counters[5];
  if (compact_overflow(n)) return;
  const uint64_t ntile = (n + CTILE - 1) / CTILE;
  const uint64_t cap = gk_args.out_cap;
  const uint32_t w = threadIdx.x >> 6;
  for (uint64_t t = blockIdx.x; t < ntile; t += gridDim.x) {
    const uint64_t i = t * CTILE + threadIdx.x;
    Viol v{};
    bool real = false;
    if (i < n) { v = raw[i]; real = v.review != VIOL_HOLE; }
    const uint64_t m = __ballot(real);
    if ((threadIdx.x & 63) == 0) wc[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint64_t before = toff[t];
    for (uint32_t k = 0; k < w; ++k) before += wc[k];
    if (real) {
      const uint64_t d = before + gk_lanes_below(m);
      gk_args.out[d] = v;
      const uint32_t nw = frec_words(v);
      for (uint32_t j = 0; j < nw && j < FMT_MAXARGS; ++j) gk_args.frec[(uint64_t)j * cap + d] = rfrec[(uint64_t)j * cap + i];
    }
    __syncthreads();
  }
}

// LDS bytes per wavefront (dynamic shared memory, 4 waves per block): 8 KB
// for a sweep's output (occupancy), 16 KB for a micro-batch's, whose messages
// are long enough that 64 tuples overflow 8 KB (config 5: ~160 B per tuple)
constexpr uint32_t FSTAGE = 8192, FSTAGE_SMALL = 16384;
extern __shared__ uint32_t gk_fmt_stage[];

template <class LO>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) gk_format_kernel(uint32_t fstage, DevArgs) {
  __shared__ uint32_t wtot[4];
  const uint64_t n = ntuples();
  // an overflowed output buffer: the host grows it and runs the passes again
  // (the tuples stay as the predicate kernels wrote them)
  if (gk_args.counters[3] > gk_args.bytes_cap || gk_args.counters[0] > gk_args.out_cap ||
      gk_args.counters[1] > gk_args.ebytes_cap)
    return;
  PLane& L = *(PLane*)&gk_pass_lane;  // see gk_size_kernel
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t* st = gk_fmt_stage + wv * (fstage / 4);
  uint8_t* stb = (uint8_t*)st;
  uint32_t* gw = (uint32_t*)gk_args.bytes;
  const uint64_t ntile = (n + FTILE - 1) / FTILE;
  const bool fl = blockIdx.x < ntile ? fmt_stage() : false;  // block-uniform
  for (uint64_t t = blockIdx.x; t < ntile; t += gridDim.x) {  // block-uniform
    uint64_t run = gk_args.part[t];
    for (uint32_t k = 0; k < FTILE; k += 256) {
      const uint64_t tb = t * FTILE + k;
      if (tb >= n) break;  // block-uniform
      const uint64_t i = tb + threadIdx.x;
      const bool valid = i < n;
      const uint32_t len = valid ? gk_args.lens[i] : 0u;
      // block-level exclusive prefix of len
      uint32_t incl = len;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
      }
      if (lane == 63) wtot[wv] = incl;
      __syncthreads();
      uint64_t wbase = run;
      for (uint32_t q = 0; q < wv; ++q) wbase += wtot[q];
      const uint64_t all = (uint64_t)wtot[0] + wtot[1] + wtot[2] + wtot[3];
      __syncthreads();
      run += all;
      const uint64_t dst = wbase + incl - len;
      Viol v{};
      if (valid) v = gk_args.out[i];
      const bool defer = valid && (v.pad & VF_DEFER);
      const uint32_t dl = valid ? det_bytes(v) : 0u;
      const uint32_t ml = len - dl;
      uint64_t a[FMT_MAXARGS];
      const uint32_t na = defer ? (v.msg_len >> 24) : 0u;
      const uint32_t nw = na + ((valid && (v.pad & VF_DET_KV)) ? 2u : 0u);  // (the details' key and value)
#pragma unroll
      for (uint32_t j = 0; j < FMT_MAXARGS; ++j) a[j] = j < nw ? gk_args.frec[(uint64_t)j * gk_args.out_cap + i] : 0;
      // the wave's range [lo, hi): consecutive tuples, consecutive bytes
      const uint64_t lo = __shfl(dst, 0, 64);
      const uint64_t hi = __shfl(dst + len, 63, 64);
      const uint64_t lo4 = lo & ~(uint64_t)3, hi4 = (hi + 3) & ~(uint64_t)3;
      // the resolved-table printer for plain arguments (string entries loaded
      // before the window loop)
      StrEnt se[FMT_MAXARGS];
      const bool plain = fl && defer && len && plain_args(gk_fmt_lds.r + (v.msg_len & 0xffffffu), a, se, na);
      auto body = [&](auto& o) {
        if (plain) print_plain_r(o, gk_fmt_lds.r + (v.msg_len & 0xffffffu), a, se);
        else if (defer) fmt_run(L, o, v.msg_len & 0xffffffu, [&](uint32_t j) { return sel_arg(a, j); });
        else puts_(o, gk_args.ebytes + v.msg_off, ml);
        if (v.pad & VF_DET_OBJ) { o.put('{'); o.put('}'); }
        else if (v.pad & (VF_DET_VAL | VF_DET_KV)) {
          if (dl)
            put_det_words(L, o, v.pad, sel_arg(a, na),
                          (v.pad & VF_DET_KV) ? sel_arg(a, na + 1) : det_word(v, i));
        }
        else puts_(o, gk_args.ebytes + v.msg_off + (defer ? 0u : ml), dl);
      };
      // the wave's bytes go through LDS in windows of FSTAGE: each lane prints
      // into the windows its tuple overlaps (one, unless it straddles an edge
      // or is longer than a window), then the wave writes the window back with
      // coalesced dword stores (byte stores at the range's two edge dwords)
      if (hi > lo) {
        const bool one = hi4 - lo4 <= fstage;
        for (uint64_t w0 = lo4; w0 < hi4; w0 += fstage) {  // wave-uniform
          const uint64_t w1 = w0 + fstage < hi4 ? w0 + fstage : hi4;
          if (valid && len && dst < w1 && dst + len > w0) {
            if (one) {
              LO o;
              o.p = stb + (dst - lo4);
              o.pos = 0;
              body(o);
            } else {
              WOut o{stb, (int64_t)(dst - w0), (uint32_t)(w1 - w0)};
              body(o);
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          const uint32_t nw = (uint32_t)((w1 - w0) >> 2);
          for (uint32_t q = lane; q < nw; q += 64) {
            const uint64_t ad = w0 + 4 * (uint64_t)q;
            if (ad >= lo && ad + 4 <= hi) {
              gw[(w0 >> 2) + q] = st[q];
            } else {
              for (uint32_t b = 0; b < 4; ++b)
                if (ad + b >= lo && ad + b < hi) gk_args.bytes[ad + b] = (char)stb[4 * q + b];
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
      if (valid) {
        v.msg_off = dst;
        v.msg_len = ml;
        v.det_len = dl;
        v.pad = 0;
        gk_args.out[i] = v;
      }
    }
  }
}

}  // namespace gk

// ------------------------------------------------------------------ host launch
// the size, spine and format passes after the predicate kernels of a call
// (grids sized for the output capacity; the passes read the tuple count on the
// device).  ev (optional, 3 events): recorded after size, spine and format.
// (the passes loop over tiles with a grid stride: `hint`, an estimate of the
// tuple count (the context's last evaluation), sizes the grid so a
// micro-batch does not launch thousands of idle blocks; 0 = the capacity)
extern "C" int gk_launch_format(const gk::DevArgs* a, hipStream_t stream, hipEvent_t* ev, uint64_t hint) {
  const uint64_t tiles = ((hint && hint < a->out_cap ? hint : a->out_cap) + gk::FTILE - 1) / gk::FTILE;
  const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(tiles, 4096));
  if (getenv("GKGPU_LAUNCH_TRACE"))
    fprintf(stderr, "passes: hint %llu, out_cap %llu, tiles %llu, blocks %u\n", (unsigned long long)hint,
            (unsigned long long)a->out_cap, (unsigned long long)tiles, blocks);
  hipLaunchKernelGGL(gk::gk_size_kernel, dim3(blocks), dim3(256), 0, stream, *a);
  if (ev) hipEventRecord(ev[0], stream);
  hipLaunchKernelGGL(gk::gk_scan_spine, dim3(1), dim3(1024), 0, stream, *a);
  if (ev) hipEventRecord(ev[1], stream);
  uint32_t fstage = hint && hint <= 65536 ? gk::FSTAGE_SMALL : gk::FSTAGE;
  // GKGPU_FMT_STAGE (tests): a smaller LDS window, so every wave's bytes go
  // through several windows
  if (const char* fs = getenv("GKGPU_FMT_STAGE")) {
    const long v = atol(fs);
    if (v >= 256 && v <= (long)gk::FSTAGE_SMALL) fstage = (uint32_t)v & ~3u;
  }
  // GKGPU_FMT_WIDE (A/B switch, default on): 16-B source reads in the printers
  static const bool wide = !getenv("GKGPU_FMT_WIDE") || atoi(getenv("GKGPU_FMT_WIDE")) != 0;
  if (wide) hipLaunchKernelGGL(gk::gk_format_kernel<gk::LOutW>, dim3(blocks), dim3(256), 4 * fstage, stream, fstage, *a);
  else hipLaunchKernelGGL(gk::gk_format_kernel<gk::LOut>, dim3(blocks), dim3(256), 4 * fstage, stream, fstage, *a);
  if (ev) hipEventRecord(ev[2], stream);
  return (int)hipGetLastError();
}

// packs the predicate kernels' chunked tuples (raw, rfrec) into a->out /
// a->frec; tcnt: one u32 per CTILE raw slots of capacity, toff: one u64 each
extern "C" int gk_launch_compact(const gk::DevArgs* a, const gk::Viol* raw, const uint64_t* rfrec, uint32_t* tcnt,
                                 unsigned long long* toff, hipStream_t stream, uint64_t hint) {
  const uint64_t tiles = ((hint && hint < a->out_cap ? hint : a->out_cap) + gk::CTILE - 1) / gk::CTILE;
  const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(tiles, 4096));
  hipLaunchKernelGGL(gk::gk_compact_count, dim3(blocks), dim3(256), 0, stream, raw, tcnt, *a);
  hipLaunchKernelGGL(gk::gk_compact_scan, dim3(1), dim3(1024), 0, stream, (const uint32_t*)tcnt, toff, *a);
  hipLaunchKernelGGL(gk::gk_compact_scatter, dim3(blocks), dim3(256), 0, stream, raw, rfrec,
                     (const unsigned long long*)toff, *a);
  return (int)hipGetLastError();
}

extern "C" int gk_launch_keys(const gk::DevArgs* a, hipStream_t stream) {
  const uint32_t blocks = (uint32_t)(((uint64_t)a->nrev + 255) / 256);
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(gk::gk_key_kernel, dim3(blocks), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

extern "C" int gk_launch_audit(const gk::DevArgs* a, hipStream_t stream) {
  uint64_t waves = (uint64_t)a->ntiles * a->nclist;
  uint64_t threads = waves * 64;
  uint32_t blocks = (uint32_t)((threads + 255) / 256);
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(gk::audit_kernel, dim3(blocks), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

extern "C" size_t gk_devargs_size() { return sizeof(gk::DevArgs); }

// ------------------------------------------------------------------ audit samples
// The audit status keeps, per constraint, the first `limit` results in
// evaluation order (pkg/audit/manager.go:485, --constraint-violations-limit)
// and the exact total of results (:470).  The tuples are unordered (one
// reservation per wavefront), so the first `limit` by (batch review index,
// autoreject first, emission order) are found in three passes over them:
//   hist   — per constraint, a histogram of review indices in `nb` buckets
//            (reviews flagged error / fallback excluded: CPU OPA answers them);
//   cut    — one wavefront per constraint: the first bucket where the running
//            count reaches `limit`, and the filtered exact total;
//   select — tuples in buckets up to the cut are copied out with the first
//            GK_SAMPLE_MSG bytes of their message (enough for the status's
//            256-byte truncateString, manager.go:622-631).
namespace gk {

__global__ void __launch_bounds__(256) gk_mark_ea_error(const Viol* out, uint64_t n, const uint8_t* cerr,
                                                        uint32_t* rflags) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const Viol v = out[i];
    if (cerr[v.constraint]) atomicOr(&rflags[v.review], (uint32_t)RF_ERROR);
  }
}

// Two levels of review buckets per constraint, so that almost no tuple
// costs a global atomic (round 4: one per tuple into 8,192 buckets, 0.38 ms
// of a config-2 sweep):
//   h1     -- SB1 coarse buckets, counted in LDS per block and added to the
//             global counts once per block and bin;
//   c1     -- one wavefront per constraint: the coarse bucket where the running
//             count reaches `limit` (cut1), the count before it, the exact total;
//   h2     -- only the tuples in their constraint's cut1 bucket: one bin per
//             review of that bucket;
//   c2     -- the first review of the bucket where the running count reaches
//             `limit` (cut2);
//   select -- the tuples of reviews before that one, and of it (ties), copied
//             out with their message's first GK_SAMPLE_MSG bytes.
constexpr uint32_t SB1 = 256;
__device__ __forceinline__ uint32_t coarse_of(uint32_t review, uint32_t nrev) {
  return (uint32_t)(((uint64_t)review * SB1) / nrev);
}
// the first review of coarse bucket b (review r is in b iff
// b * nrev <= r * SB1 < (b + 1) * nrev)
__device__ __forceinline__ uint32_t coarse_lo(uint32_t b, uint32_t nrev) {
  return (uint32_t)(((uint64_t)b * nrev + SB1 - 1) / SB1);
}
extern __shared__ uint32_t gk_sample_lds[];
__global__ void __launch_bounds__(256) gk_sample_h1(const Viol* out, uint64_t n, const uint32_t* rflags, uint32_t nrev,
                                                    uint32_t ncons, int lds, uint32_t* h1) {
  const uint32_t nbin = ncons * SB1;
  if (lds) {
    for (uint32_t k = threadIdx.x; k < nbin; k += blockDim.x) gk_sample_lds[k] = 0;
    __syncthreads();
  }
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const Viol v = out[i];
    if (rflags && (rflags[v.review] & (RF_ERROR | RF_FALLBACK))) continue;
    const uint32_t bin = v.constraint * SB1 + coarse_of(v.review, nrev);
    if (lds) atomicAdd(&gk_sample_lds[bin], 1u);
    else atomicAdd(&h1[bin], 1u);
  }
  if (lds) {
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nbin; k += blockDim.x)
      if (gk_sample_lds[k]) atomicAdd(&h1[k], gk_sample_lds[k]);
  }
}

// one wavefront per constraint: the first of `nb` counts (after `before`)
// where the running count reaches `limit`; nb - 1 when it never does
__device__ __forceinline__ uint32_t first_reaching(const uint32_t* h, uint32_t nb, uint64_t before, uint32_t limit,
                                                   uint64_t* total) {
  const uint32_t lane = threadIdx.x & 63;
  uint64_t run = before;
  uint32_t cb = 0xffffffffu;
  for (uint32_t base = 0; base < nb; base += 64) {
    const uint32_t x = base + lane < nb ? h[base + lane] : 0u;
    uint32_t incl = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    const uint32_t tot = __shfl(incl, 63, 64);
    if (cb == 0xffffffffu && run + tot >= limit) {
      const unsigned long long m = __ballot(run + incl >= limit);
      cb = base + (uint32_t)__ffsll((long long)m) - 1;
    }
    run += tot;
  }
  *total = run;
  return cb == 0xffffffffu ? nb - 1 : cb;
}
// cut[2c] = coarse cut, cut[2c + 1] = the count before it (then c2's fine cut)
__global__ void __launch_bounds__(64) gk_sample_c1(const uint32_t* h1, uint32_t limit, uint32_t* cut,
                                                   unsigned long long* ftot) {
  const uint32_t c = blockIdx.x;
  const uint32_t* h = h1 + (uint64_t)c * SB1;
  uint64_t total = 0;
  const uint32_t cb = first_reaching(h, SB1, 0, limit, &total);
  uint32_t before = 0;
  for (uint32_t k = threadIdx.x; k < cb; k += 64) before += h[k];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) before += __shfl_xor(before, d, 64);
  if (threadIdx.x == 0) {
    cut[2 * c] = cb;
    cut[2 * c + 1] = before;
    ftot[c] = total;
  }
}
__global__ void __launch_bounds__(256) gk_sample_h2(const Viol* out, uint64_t n, const uint32_t* rflags, uint32_t nrev,
                                                    uint32_t nf, const uint32_t* cut, uint32_t* h2) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const Viol v = out[i];
    const uint32_t b = coarse_of(v.review, nrev);
    if (b != cut[2 * v.constraint]) continue;
    if (rflags && (rflags[v.review] & (RF_ERROR | RF_FALLBACK))) continue;
    atomicAdd(&h2[(uint64_t)v.constraint * nf + (v.review - coarse_lo(b, nrev))], 1u);
  }
}
__global__ void __launch_bounds__(64) gk_sample_c2(const uint32_t* h2, uint32_t nf, uint32_t limit, uint32_t* cut) {
  const uint32_t c = blockIdx.x;
  uint64_t total = 0;
  const uint32_t f = first_reaching(h2 + (uint64_t)c * nf, nf, cut[2 * c + 1], limit, &total);
  __syncthreads();
  if (threadIdx.x == 0) cut[2 * c + 1] = f;
}

__global__ void __launch_bounds__(256) gk_sample_select(const Viol* out, uint64_t n, const uint32_t* rflags, uint32_t nrev,
                                                        const uint32_t* cut, const char* bytes, SampleRec* cand,
                                                        uint32_t cap, unsigned int* ncand) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const Viol v = out[i];
    const uint32_t b = coarse_of(v.review, nrev), cb = cut[2 * v.constraint];
    if (b > cb || (b == cb && v.review - coarse_lo(b, nrev) > cut[2 * v.constraint + 1])) continue;
    if (rflags && (rflags[v.review] & (RF_ERROR | RF_FALLBACK))) continue;
    uint32_t slot = atomicAdd(ncand, 1u);
    if (slot >= cap) continue;  // the host grows the buffer and runs this pass again
    SampleRec& r = cand[slot];
    r.review = v.review;
    r.constraint = v.constraint;
    r.seq = v.seq;
    r.rule = v.rule;
    r.msg_len = v.msg_len;
    r.pad = 0;
    uint32_t m = v.msg_len < SAMPLE_MSG ? v.msg_len : SAMPLE_MSG;
    const char* src = bytes + v.msg_off;
    for (uint32_t k = 0; k < m; ++k) r.msg[k] = (uint8_t)src[k];
  }
}

// The raw-output copy (gk_results_copy_device_output): the tuples of reviews
// the engine answered, i.e. without those of reviews flagged error or
// fallback (the caller re-runs those on CPU OPA) -- the same set the totals
// count.  Order is not kept (a wave-aggregated atomic cursor); consumers sort
// by (review, autoreject first, constraint, seq).
__global__ void __launch_bounds__(256) gk_filter_viol(const Viol* out, uint64_t n, const uint32_t* rflags, Viol* dst,
                                                      unsigned long long* count) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < n; base += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = base + threadIdx.x;
    Viol v;
    bool keep = false;
    if (i < n) {
      v = out[i];
      keep = !(rflags[v.review] & (RF_ERROR | RF_FALLBACK));
    }
    const unsigned long long m = __ballot(keep);
    if (!m) continue;
    unsigned long long slot0 = 0;
    const uint32_t leader = (uint32_t)__ffsll((long long)m) - 1;
    if (lane == leader) slot0 = atomicAdd(count, (unsigned long long)__popcll(m));
    slot0 = __shfl(slot0, (int)leader, 64);
    if (keep) dst[slot0 + __popcll(m & ((1ull << lane) - 1))] = v;
  }
}

}  // namespace gk

namespace gk {

// Clock probe: one wavefront spins on dependent integer ops while reading the
// shader-clock counter (s_memtime) and the fixed 100 MHz reference counter
// (s_memrealtime); their ratio is the core clock the kernels actually ran at
// (box-to-box variance: MI355X boxes in a low-power state run the same code
// objects at a fraction of the clock).  Results are written by a vector store.
__global__ void __launch_bounds__(64) gk_clock_probe(unsigned long long* out, uint32_t iters) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = threadIdx.x;
  for (uint32_t i = 0; i < iters; ++i) x = x * 1664525u + 1013904223u;
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = r1 - r0;
    out[2] = x;
  }
}

}  // namespace gk

// Zeroes an evaluation's per-call device state in one dispatch: flags,
// reasons, totals, counters, the memo-string cursor and the cross-lane memo
// tables of every stream the launches use (round 3 issued one fill per buffer
// and one per template launch: ~10 dispatches ahead of a micro-batch's work).
namespace gk {
struct ZeroList {
  uint32_t* p[12];
  uint64_t words[12];  // 4-byte words
  uint32_t n;
};
__global__ void __launch_bounds__(256) gk_zero(ZeroList z) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t b = 0; b < z.n; ++b) {
    uint32_t* q = z.p[b];
    const uint64_t nw = z.words[b];
    for (uint64_t i = t0; i < nw; i += stride) q[i] = 0u;
  }
}
}  // namespace gk

extern "C" int gk_launch_clock_probe(unsigned long long* out, uint32_t iters, hipStream_t stream) {
  hipLaunchKernelGGL(gk::gk_clock_probe, dim3(1), dim3(64), 0, stream, out, iters);
  return (int)hipGetLastError();
}

// zero n buffers (bytes multiples of 4, at most 12) on the stream
extern "C" int gk_launch_zero(void* const* ptrs, const uint64_t* bytes, uint32_t n, hipStream_t stream) {
  if (n > 12) return (int)hipErrorInvalidValue;
  gk::ZeroList z{};
  uint64_t tot = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (!ptrs[i] || !bytes[i]) continue;
    z.p[z.n] = (uint32_t*)ptrs[i];
    z.words[z.n] = bytes[i] / 4;
    tot += bytes[i] / 4;
    ++z.n;
  }
  if (!z.n) return 0;
  const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((tot + 1023) / 1024, 2048));
  hipLaunchKernelGGL(gk::gk_zero, dim3(blocks), dim3(256), 0, stream, z);
  return (int)hipGetLastError();
}

extern "C" int gk_launch_filter(const gk::Viol* out, uint64_t n, uint32_t* rflags, const uint8_t* cerr,
                                gk::Viol* dst, unsigned long long* count, hipStream_t stream) {
  uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, 8192);
  if (blocks == 0) blocks = 1;
  if (cerr) hipLaunchKernelGGL(gk::gk_mark_ea_error, dim3(blocks), dim3(256), 0, stream, out, n, cerr, rflags);
  (void)hipMemsetAsync(count, 0, 8, stream);
  hipLaunchKernelGGL(gk::gk_filter_viol, dim3(blocks), dim3(256), 0, stream, out, n, (const uint32_t*)rflags, dst, count);
  return (int)hipGetLastError();
}

extern "C" int gk_launch_sample(const gk::Viol* out, uint64_t n, uint32_t* rflags, uint32_t nrev, const uint8_t* cerr,
                                uint32_t ncons, uint32_t nf, uint32_t limit, uint32_t* hist, uint32_t* cut,
                                unsigned long long* ftot, const char* bytes, gk::SampleRec* cand, uint32_t cap,
                                unsigned int* ncand, int select_only, hipStream_t stream) {
  // hist: ncons * SB1 coarse counts, then ncons * nf fine counts
  // (nf = gk_sample_fine(nrev)); cut: 2 words per constraint
  uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, 8192);
  if (blocks == 0) blocks = 1;
  if (!select_only) {
    if (cerr) hipLaunchKernelGGL(gk::gk_mark_ea_error, dim3(blocks), dim3(256), 0, stream, out, n, cerr, rflags);
    uint32_t* h1 = hist;
    uint32_t* h2 = hist + (size_t)ncons * gk::SB1;
    (void)hipMemsetAsync(hist, 0, (size_t)ncons * (gk::SB1 + nf) * 4, stream);
    const size_t lds = (size_t)ncons * gk::SB1 * 4;
    const bool use_lds = lds <= 65536;
    // fewer, longer-running blocks for the LDS histogram: each flushes its bins once
    const uint32_t hb = use_lds ? std::min<uint32_t>(blocks, 512) : blocks;
    hipLaunchKernelGGL(gk::gk_sample_h1, dim3(hb), dim3(256), use_lds ? lds : 0, stream, out, n, (const uint32_t*)rflags,
                       nrev, ncons, use_lds ? 1 : 0, h1);
    hipLaunchKernelGGL(gk::gk_sample_c1, dim3(ncons), dim3(64), 0, stream, (const uint32_t*)h1, limit, cut, ftot);
    hipLaunchKernelGGL(gk::gk_sample_h2, dim3(blocks), dim3(256), 0, stream, out, n, (const uint32_t*)rflags, nrev, nf,
                       (const uint32_t*)cut, h2);
    hipLaunchKernelGGL(gk::gk_sample_c2, dim3(ncons), dim3(64), 0, stream, (const uint32_t*)h2, nf, limit, cut);
  }
  (void)hipMemsetAsync(ncand, 0, 4, stream);
  hipLaunchKernelGGL(gk::gk_sample_select, dim3(blocks), dim3(256), 0, stream, out, n, (const uint32_t*)rflags, nrev,
                     (const uint32_t*)cut, bytes, cand, cap, ncand);
  return (int)hipGetLastError();
}
// fine bins per constraint for nrev reviews (the reviews of one coarse bucket)
extern "C" uint32_t gk_sample_fine(uint32_t nrev) { return nrev / gk::SB1 + 2; }
