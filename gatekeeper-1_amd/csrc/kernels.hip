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
      default: lane_fallback(L, FB_UNSUPPORTED); return;
    }
  }
  lane_fallback(L, FB_UNSUPPORTED);
}

__global__ void __launch_bounds__(256) audit_kernel() {
  audit_body([&](PLane& L, uint64_t review, uint64_t params, uint32_t prog, uint32_t r, uint32_t c) {
    run_program(L, gk_args.prog_off[prog], review, params);
  });
}

// Format pass: one lane per output tuple whose message the audit kernels
// deferred (devrt.h op_emit / flush_wave).  The arguments are heap-free values
// (interned strings, slices, numbers, document nodes), so formatting reads only
// the shared tables: the lane reference below is never dereferenced for them
// (sview / coll_at touch a lane's buffers only for lane-heap values).  Lanes
// write disjoint byte ranges [msg_off, msg_off + msg_len) reserved by the audit
// kernel, consecutive tuples to consecutive ranges.

// LDS-staged writer for one wavefront's message bytes
struct LOut {
  uint8_t* p;
  uint32_t pos;
  __device__ __forceinline__ void put(char c) { p[pos++] = (uint8_t)c; }
};

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

constexpr uint32_t FSTAGE = 8192;  // LDS bytes per wavefront

// A wavefront takes 64 consecutive tuples.  When their output bytes (messages
// and details) form one dense range that fits in LDS — the usual case, since a
// wave's tuples come from one audit-kernel reservation — the range is read
// into LDS, the live lanes format their messages into it, and it is written
// back with coalesced dword stores (byte stores for the two edge dwords, which
// may hold a neighbouring wave's bytes).  Otherwise each lane formats straight
// into HBM.
__global__ void __launch_bounds__(256) gk_format_kernel() {
  __shared__ uint32_t stage[4][FSTAGE / 4];
  const uint64_t n = gk_args.counters[0];
  // an overflowed call left some reservations unwritten; the host retries it
  if (n > gk_args.out_cap || gk_args.counters[1] > gk_args.bytes_cap) return;
  Lane L0;  // never dereferenced: the arguments are heap-free values
  PLane& L = *(PLane*)&L0;
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t* st = stage[wv];
  uint8_t* stb = (uint8_t*)st;
  uint32_t* gw = (uint32_t*)gk_args.bytes;
  for (uint64_t base = ((uint64_t)blockIdx.x * 4 + wv) * 64; base < n; base += (uint64_t)gridDim.x * 256) {  // wave-uniform
    uint64_t i = base + lane;
    bool valid = i < n;
    const uint64_t* w = gk_args.frec + i * FREC_WORDS;
    uint64_t h = valid ? w[0] : 0;
    Viol v{};
    if (valid) v = gk_args.out[i];
    uint64_t end = v.msg_off + v.msg_len + v.det_len;
    bool live = valid && (h & FREC_LIVE) && v.msg_off + v.msg_len <= gk_args.bytes_cap;
    if (!__any(live)) continue;
    uint64_t lo = wave_min64(valid ? v.msg_off : ~0ull);
    uint64_t hi = wave_max64(valid ? end : 0ull);
    uint32_t tot = wave_sum(valid ? v.msg_len + v.det_len : 0u);
    uint64_t lo4 = lo & ~(uint64_t)3, hi4 = (hi + 3) & ~(uint64_t)3;
    if (tot == hi - lo && hi4 - lo4 <= FSTAGE && hi4 <= gk_args.bytes_cap) {
      uint32_t nw = (uint32_t)((hi4 - lo4) >> 2);
      // the range's bytes are read first unless this pass writes all of them:
      // every tuple live with no details bytes from the audit kernel
      // (FREC_DET_OBJ or none); the edge dwords are written bytewise anyway
      const bool whole = __all(!valid || (live && ((h & FREC_DET_OBJ) || v.det_len == 0)));
      if (!whole)
        for (uint32_t k = lane; k < nw; k += 64) st[k] = gw[(lo4 >> 2) + k];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      if (live) {
        LOut o{stb + (v.msg_off - lo4), 0};
        fmt_run(L, o, (uint32_t)h & 0xffffffu, [&](uint32_t j) { return w[1 + j]; });
        if (h & FREC_DET_OBJ) { o.put('{'); o.put('}'); }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (uint32_t k = lane; k < nw; k += 64) {
        uint64_t a = lo4 + 4 * (uint64_t)k;
        if (a >= lo && a + 4 <= hi) {
          gw[(lo4 >> 2) + k] = st[k];
        } else {
          for (uint32_t b = 0; b < 4; ++b)
            if (a + b >= lo && a + b < hi) gk_args.bytes[a + b] = (char)stb[4 * k + b];
        }
      }
    } else if (live) {
      GOut g{(uint8_t*)gk_args.bytes, v.msg_off, v.msg_off, 0, false};
      fmt_run(L, g, (uint32_t)h & 0xffffffu, [&](uint32_t j) { return w[1 + j]; });
      if (h & FREC_DET_OBJ) { g.put('{'); g.put('}'); }
      g.finish();
    }
  }
}

}  // namespace gk

// ------------------------------------------------------------------ host launch
extern "C" int gk_launch_format(const gk::DevArgs* a, hipStream_t stream) {
  if (!a->frec) return 0;
  hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(gk_args), a, sizeof(*a), 0, hipMemcpyHostToDevice, stream);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(gk::gk_format_kernel, dim3(2048), dim3(256), 0, stream);
  return (int)hipGetLastError();
}

extern "C" int gk_launch_audit(const gk::DevArgs* a, hipStream_t stream) {
  uint64_t waves = (uint64_t)a->ntiles * a->nclist;
  uint64_t threads = waves * 64;
  uint32_t blocks = (uint32_t)((threads + 255) / 256);
  if (blocks == 0) return 0;
  hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(gk_args), a, sizeof(*a), 0, hipMemcpyHostToDevice, stream);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(gk::audit_kernel, dim3(blocks), dim3(256), 0, stream);
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

__device__ __forceinline__ uint32_t sample_bucket(uint32_t review, uint32_t nrev, uint32_t nb) {
  return (uint32_t)(((uint64_t)review * nb) / nrev);
}

__global__ void __launch_bounds__(256) gk_sample_hist(const Viol* out, uint64_t n, const uint32_t* rflags, uint32_t nrev,
                                                      uint32_t nb, uint32_t* hist) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const Viol v = out[i];
    if (rflags && (rflags[v.review] & (RF_ERROR | RF_FALLBACK))) continue;
    atomicAdd(&hist[(uint64_t)v.constraint * nb + sample_bucket(v.review, nrev, nb)], 1u);
  }
}

__global__ void __launch_bounds__(64) gk_sample_cut(const uint32_t* hist, uint32_t nb, uint32_t limit, uint32_t* cut,
                                                    unsigned long long* ftot) {
  const uint32_t c = blockIdx.x, lane = threadIdx.x;
  const uint32_t* h = hist + (uint64_t)c * nb;
  uint64_t run = 0;
  uint32_t cb = 0xffffffffu;
  for (uint32_t base = 0; base < nb; base += 64) {
    uint32_t x = base + lane < nb ? h[base + lane] : 0u;
    uint32_t incl = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    uint32_t tot = __shfl(incl, 63, 64);
    if (cb == 0xffffffffu && run + tot >= limit) {
      // first lane whose inclusive count reaches the limit
      unsigned long long m = __ballot(run + incl >= limit);
      cb = base + (uint32_t)__ffsll((long long)m) - 1;
    }
    run += tot;
  }
  if (lane == 0) {
    cut[c] = cb == 0xffffffffu ? nb - 1 : cb;
    ftot[c] = run;
  }
}

__global__ void __launch_bounds__(256) gk_sample_select(const Viol* out, uint64_t n, const uint32_t* rflags, uint32_t nrev,
                                                        uint32_t nb, const uint32_t* cut, const char* bytes,
                                                        SampleRec* cand, uint32_t cap, unsigned int* ncand) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const Viol v = out[i];
    if (rflags && (rflags[v.review] & (RF_ERROR | RF_FALLBACK))) continue;
    if (sample_bucket(v.review, nrev, nb) > cut[v.constraint]) continue;
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

extern "C" int gk_launch_clock_probe(unsigned long long* out, uint32_t iters, hipStream_t stream) {
  hipLaunchKernelGGL(gk::gk_clock_probe, dim3(1), dim3(64), 0, stream, out, iters);
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
                                uint32_t ncons, uint32_t nb, uint32_t limit, uint32_t* hist, uint32_t* cut,
                                unsigned long long* ftot, const char* bytes, gk::SampleRec* cand, uint32_t cap,
                                unsigned int* ncand, int select_only, hipStream_t stream) {
  uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, 8192);
  if (blocks == 0) blocks = 1;
  if (!select_only) {
    if (cerr) hipLaunchKernelGGL(gk::gk_mark_ea_error, dim3(blocks), dim3(256), 0, stream, out, n, cerr, rflags);
    (void)hipMemsetAsync(hist, 0, (size_t)ncons * nb * 4, stream);
    hipLaunchKernelGGL(gk::gk_sample_hist, dim3(blocks), dim3(256), 0, stream, out, n, (const uint32_t*)rflags, nrev, nb, hist);
    hipLaunchKernelGGL(gk::gk_sample_cut, dim3(ncons), dim3(64), 0, stream, (const uint32_t*)hist, nb, limit, cut, ftot);
  }
  (void)hipMemsetAsync(ncand, 0, 4, stream);
  hipLaunchKernelGGL(gk::gk_sample_select, dim3(blocks), dim3(256), 0, stream, out, n, (const uint32_t*)rflags, nrev, nb,
                     (const uint32_t*)cut, bytes, cand, cap, ncand);
  return (int)hipGetLastError();
}
