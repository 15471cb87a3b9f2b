// Microbenchmark: cost of the emission slot reservation pattern of the
// template kernels (devrt.h wave_reserve: one same-address atomicAdd with
// return per wavefront per emission site, the slot then used by a store),
// against per-wave chunked reservation.  1M threads (15,625 waves), K
// emission sites per lane, 2 waves per SIMD as K8sContainerLimits runs.
//   hipcc --offload-arch=gfx950 -O3 tools/atomic_probe.hip -o gpurun_out/atomic_probe
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>

struct Tup { uint32_t a, b, c, d; uint64_t e, f; };

__global__ void __launch_bounds__(256, 2) per_site(unsigned long long* ctr, Tup* out, uint64_t cap, int K, int pct) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  for (int k = 0; k < K; ++k) {
    // a lane emits at this site with probability pct% (hash of gid, k)
    const uint32_t h = (gid * 2654435761u) ^ (uint32_t)(k * 40503u);
    if ((h >> 8) % 100u < (uint32_t)pct) {
      const uint64_t slot = atomicAdd(ctr, 1ull);
      if (slot < cap) out[slot] = Tup{gid, (uint32_t)k, 0, 0, slot, 0};
    }
  }
}

// the wave takes CH slots at a time; lanes are numbered within the wave by mbcnt
__global__ void __launch_bounds__(256, 2) chunked(unsigned long long* ctr, Tup* out, uint64_t cap, int K, int pct, int CH) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t base = 0;
  uint32_t left = 0;  // wave-uniform
  for (int k = 0; k < K; ++k) {
    const uint32_t h = (gid * 2654435761u) ^ (uint32_t)(k * 40503u);
    const bool want = (h >> 8) % 100u < (uint32_t)pct;
    const uint64_t m = __ballot(want);
    const uint32_t n = __popcll(m);
    if (n > left) {
      uint64_t b = 0;
      const uint32_t take = n > (uint32_t)CH ? n : (uint32_t)CH;
      if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0) b = atomicAdd(ctr, (unsigned long long)take);
      base = __shfl(b, 0, 64);
      left = take;
    }
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (want) {
      const uint64_t slot = base + below;
      if (slot < cap) out[slot] = Tup{gid, (uint32_t)k, 0, 0, slot, 0};
    }
    base += n;
    left -= n;
  }
}

int main() {
  const uint32_t threads = 1u << 20;
  const int K = 48;
  const uint64_t cap = (uint64_t)threads * K;
  unsigned long long* ctr;
  Tup* out;
  if (hipMalloc(&ctr, 8) != hipSuccess || hipMalloc(&out, cap * sizeof(Tup)) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int pct : {10, 50}) {
    for (int mode = 0; mode < 4; ++mode) {
      const int CH = mode == 1 ? 64 : mode == 2 ? 256 : 1024;
      float best = 1e9f;
      unsigned long long n = 0;
      for (int rep = 0; rep < 5; ++rep) {
        hipMemset(ctr, 0, 8);
        hipEventRecord(e0);
        if (mode == 0) hipLaunchKernelGGL(per_site, dim3(threads / 256), dim3(256), 0, 0, ctr, out, cap, K, pct);
        else hipLaunchKernelGGL(chunked, dim3(threads / 256), dim3(256), 0, 0, ctr, out, cap, K, pct, CH);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
        hipMemcpy(&n, ctr, 8, hipMemcpyDeviceToHost);
      }
      printf("emit %2d%% of %d sites: %-10s chunk %4d: %.3f ms  (%llu slots)\n", pct, K, mode ? "chunked" : "per-site",
             mode ? CH : 0, best, n);
    }
  }
  return 0;
}
