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
#include "devrt.h"

namespace gk {

constexpr int NREG = 192;

__device__ void run_program(const DevArgs& A, Lane& L, uint32_t pc, uint64_t review, uint64_t params) {
  const uint64_t UND = mkv(V_UNDEF, 0);
  uint64_t R[NREG];
  for (int guard = 0; guard < (1 << 22); ++guard) {
    if (pc >= A.ncode) { lane_fallback(L, FB_UNSUPPORTED); return; }
    const Ins in = A.code[pc];
    ++pc;
    ++L.steps;
    if (A.pchist) atomicAdd(&A.pchist[pc - 1], 1u);
    switch (in.op) {
      case OP_END: return;
      case OP_JMP: pc = in.x; break;
      case OP_JUNDEF: if (vtag(R[in.a]) == V_UNDEF) pc = in.x; break;
      case OP_JFALSE: if (vtag(R[in.a]) == V_BOOL && vpay(R[in.a]) == 0) pc = in.x; break;
      case OP_JTRUE: if (vtag(R[in.a]) == V_BOOL && vpay(R[in.a]) == 1) pc = in.x; break;
      case OP_LOADK: R[in.a] = A.K[in.x]; break;
      case OP_LOADREV: R[in.a] = review; break;
      case OP_LOADPARAM: R[in.a] = params; break;
      case OP_MOV: R[in.a] = R[in.b]; break;
      case OP_GET: R[in.a] = vget(A, L, R[in.b], R[in.c]); break;
      case OP_GETK: R[in.a] = vget(A, L, R[in.b], A.K[in.x]); break;
      case OP_ITER_INIT: op_iter_init(L, R[in.a], R[in.a + 1], R[in.b], in.y); break;
      case OP_ITER_NEXT: {
        uint64_t k = UND, v = UND;
        if (!op_iter_next(A, L, R[in.a], R[in.a + 1], in.y, k, v)) { pc = in.x; break; }
        if (in.b != 0xffff) R[in.b] = k;
        if (in.c != 0xffff) R[in.c] = v;
        break;
      }
      case OP_CMP: if (!op_cmp(A, L, in.y, R[in.b], R[in.c], R[in.a])) return; break;
      case OP_ARITH: R[in.a] = arith(A, L, in.y, R[in.b], R[in.c]); if (L.fail) return; break;
      case OP_LIST_NEW: R[in.a] = list_new(L, in.y, 4); if (L.fail) return; break;
      case OP_LIST_ADD: if (!op_list_add(A, L, R[in.a], R[in.b], in.y)) return; break;
      case OP_OBJ_PUT: if (!op_obj_put(A, L, R[in.a], R[in.b], R[in.c], in.y)) return; break;
      case OP_YIELD: if (!op_yield(A, L, R[in.a], R[in.b], in.y)) return; break;
      case OP_CALL: R[in.a] = call_builtin(A, L, in.y, &R[in.b]); if (L.fail) return; break;
      case OP_SPRINTF: R[in.a] = do_sprintf(A, L, in.x, R[in.b]); if (L.fail) return; break;
      case OP_LEN_EQ: R[in.a] = op_len_eq(A, L, R[in.b], in.y); break;
      case OP_EMIT: if (!op_emit(A, L, R[in.a], in.b == 0xffff ? UND : R[in.b], in.c, in.y)) return; break;
      case OP_TABLE: R[in.a] = op_table(A, L, A.K + in.x, R[in.b]); break;
      case OP_FAIL_FALLBACK: lane_fallback(L, in.y); return;
      default: lane_fallback(L, FB_UNSUPPORTED); return;
    }
  }
  lane_fallback(L, FB_UNSUPPORTED);
}

__global__ void __launch_bounds__(256) audit_kernel(DevArgs A) {
  audit_body(A, [&](Lane& L, uint64_t review, uint64_t params, uint32_t prog, uint32_t r, uint32_t c) {
    run_program(A, L, A.prog_off[prog], review, params);
  });
}

}  // namespace gk

// ------------------------------------------------------------------ host launch
extern "C" int gk_launch_audit(const gk::DevArgs* a, hipStream_t stream) {
  uint64_t waves = (uint64_t)a->ntiles * a->nclist;
  uint64_t threads = waves * 64;
  uint32_t blocks = (uint32_t)((threads + 255) / 256);
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(gk::audit_kernel, dim3(blocks), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

extern "C" size_t gk_devargs_size() { return sizeof(gk::DevArgs); }
