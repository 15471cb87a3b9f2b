// Path-grouped node layout of a staged batch, built on the device (N1).
//
// The host flattener parses, interns and relocates each part's documents
// into one per-document arena D (every document's nodes contiguous, node ids
// global) and uploads it; every container node of D carries in its (otherwise
// unused) `val` field its document path -- object.spec.containers[*] and so on,
// interned while the part parsed (flatten.cc count_paths) -- or kSharedPath
// for the Namespace documents several reviews share.  This pass permutes D
// into the layout the kernels read (flatten.h): the live review roots in
// evaluation order, then one region per path holding the member runs of every
// instance of that path in evaluation order, the shared Namespace runs last.
// An object's members stay one run in document order, so every reader of the
// node store is unchanged; the wavefront's 64 consecutive reviews find their
// nodes at one path side by side.  On the host this placement was a
// depth-first walk per review with random writes into the regions (~2/3 of
// flatten time for 1M Pods); here it is a sort of the runs by (path,
// evaluation position) and a scatter, HBM-bound.
//
//   mark    -- per D node: is it the owner of a member run (a container with
//              members, not borrowing a shared run) -> (key, D index)
//   select  -- compaction of the owners (hipcub DeviceSelect)
//   sort    -- stable radix sort of (path << 32 | evaluation position) keys
//   scan    -- exclusive sum of run lengths: each run's new start
//   runs    -- newrun[first child] = new start
//   scatter -- every run's members to their new places, child links rewritten
//   roots   -- the live roots to [0, nroots)
//   cols    -- the review columns' node ids through newpos
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>

#include <algorithm>
#include <vector>

#include "common.h"

namespace gk {
namespace dlayout {

constexpr uint8_t kSharedFlag = 0x80;        // flatten.cc kShared
constexpr uint32_t kSharedPath = 0xffffffffu;

__device__ __forceinline__ bool container(const Node& x) { return (x.type == NT_OBJ || x.type == NT_ARR) && x.n; }

// the review (batch index) whose document holds D index i: ranges are sorted
// by start (documents are laid out in batch order, part by part)
__device__ __forceinline__ uint32_t review_of(const uint32_t* beg, uint32_t nrev, uint32_t i) {
  uint32_t lo = 0, hi = nrev;
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) >> 1;
    if (beg[m] <= i) lo = m; else hi = m;
  }
  return lo;
}

__global__ void mark(const Node* D, uint64_t nD, uint32_t base, const uint32_t* beg, uint32_t nrev,
                     const uint32_t* evalpos, uint8_t* flag, uint64_t* key) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nD) return;
  const Node x = D[i];
  bool owner = false;
  uint64_t k = 0;
  if (container(x) && x.first >= base && (uint64_t)(x.first - base) < nD) {
    const bool shared = x.flags & kSharedFlag;
    const bool borrows = !shared && (D[x.first - base].flags & kSharedFlag);
    if (!borrows) {
      owner = true;
      if (shared || x.val == kSharedPath) k = (uint64_t)0xffffffffull << 32;
      else k = ((uint64_t)x.val << 32) | evalpos[review_of(beg, nrev, (uint32_t)i)];
    }
  }
  flag[i] = owner ? 1 : 0;
  key[i] = k;
}

// the selected owners' keys (gathered by D index) and run lengths
__global__ void gather(const Node* D, const uint64_t* key, const uint32_t* items, uint64_t nitems, uint64_t* ksel) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < nitems) ksel[j] = key[items[j]];
}
__global__ void run_len(const Node* D, const uint32_t* items, uint64_t nitems, uint32_t* len) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < nitems) len[j] = D[items[j]].n;
}

__global__ void runs(const Node* D, uint32_t base, uint32_t nroots, const uint32_t* items, const uint32_t* start,
                     uint64_t nitems, uint32_t* newrun) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nitems) return;
  newrun[D[items[j]].first - base] = base + nroots + start[j];
}

__device__ __forceinline__ Node relink(Node y, uint32_t base, uint64_t nD, const uint32_t* newrun) {
  if (container(y) && y.first >= base && (uint64_t)(y.first - base) < nD) y.first = newrun[y.first - base];
  if (y.type == NT_OBJ || y.type == NT_ARR) y.val = 0;
  y.flags &= (uint8_t)~kSharedFlag;
  return y;
}

__global__ void scatter(const Node* D, uint64_t nD, uint32_t base, uint32_t nroots, const uint32_t* items,
                        const uint32_t* start, uint64_t nitems, const uint32_t* newrun, Node* N, uint32_t* newpos) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nitems) return;
  const Node x = D[items[j]];
  const uint32_t f = x.first - base;
  const uint32_t s = nroots + start[j];
  for (uint32_t c = 0; c < x.n; ++c) {
    N[s + c] = relink(D[f + c], base, nD, newrun);
    newpos[f + c] = base + s + c;
  }
}

__global__ void roots(const Node* D, uint64_t nD, uint32_t base, const uint32_t* root_d, const uint32_t* slot,
                      uint32_t nrev, const uint32_t* newrun, Node* N, uint32_t* newpos) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nrev || slot[b] == NO_ID || root_d[b] < base) return;
  const uint32_t r = root_d[b] - base;
  Node y = relink(D[r], base, nD, newrun);
  y.key = 0;
  N[slot[b]] = y;
  newpos[r] = base + slot[b];
}

__device__ __forceinline__ uint32_t moved(uint32_t id, uint32_t base, uint64_t nD, const uint32_t* newpos) {
  return (id != NO_ID && id >= base && (uint64_t)(id - base) < nD) ? newpos[id - base] : id;
}

__global__ void cols(ReviewCol* c, uint32_t n, uint32_t base, uint64_t nD, const uint32_t* newpos) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ReviewCol r = c[i];
  r.root = moved(r.root, base, nD, newpos);
  r.labels = moved(r.labels, base, nD, newpos);
  r.old_labels = moved(r.old_labels, base, nD, newpos);
  r.ns_labels = moved(r.ns_labels, base, nD, newpos);
  c[i] = r;
}

}  // namespace dlayout
}  // namespace gk

static unsigned grid_of(uint64_t n) { return (unsigned)((n + 255) / 256); }

// D (nD nodes, ids base..) on the device -> N (the path-grouped layout, ids
// base..) and the review columns (cols, in evaluation order, D ids) rewritten
// to N ids.  beg[b]: D index of review b's first node (batch order, sorted);
// evalpos[b]: its evaluation position; root_d[b]: its root's id in D and
// slot[b]: its root's N index (NO_ID: excluded).  Device pointers; the
// temporaries are allocated on the stream and freed before returning.
// *n_out: nodes written to N (nroots + the runs' members, <= nD).  0 = success.
extern "C" int gk_device_layout(const gk::Node* D, uint64_t nD, uint32_t base, const uint32_t* beg, const uint32_t* evalpos,
                                const uint32_t* root_d, const uint32_t* slot, uint32_t nrev, uint32_t nroots,
                                gk::Node* N, gk::ReviewCol* cols, uint32_t ncols, uint64_t* n_out, hipStream_t s) {
  using namespace gk::dlayout;
  if (n_out) *n_out = 0;
  if (nD == 0 || nD >= 0x7fffffffull || nrev == 0) return (int)hipErrorInvalidValue;
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (e == hipSuccess && x != hipSuccess) e = x; };
  std::vector<void*> owned;
  auto alloc = [&](size_t bytes) -> void* {
    void* p = nullptr;
    chk(hipMallocAsync(&p, bytes ? bytes : 8, s));
    if (p) owned.push_back(p);
    return p;
  };
  const int n = (int)nD;
  uint8_t* flag = (uint8_t*)alloc(nD);
  uint64_t* key = (uint64_t*)alloc(nD * 8);
  uint32_t* items = (uint32_t*)alloc(nD * 4);
  int* nsel = (int*)alloc(sizeof(int));
  uint32_t* newrun = (uint32_t*)alloc(nD * 4);
  uint32_t* newpos = (uint32_t*)alloc(nD * 4);
  uint64_t nitems = 0, total = nroots;
  if (e == hipSuccess) {
    hipLaunchKernelGGL(mark, dim3(grid_of(nD)), dim3(256), 0, s, D, nD, base, beg, nrev, evalpos, flag, key);
    chk(hipGetLastError());
    hipcub::CountingInputIterator<uint32_t> cnt(0);
    size_t tb = 0;
    chk(hipcub::DeviceSelect::Flagged(nullptr, tb, cnt, flag, items, nsel, n, s));
    void* tmp = alloc(tb);
    chk(hipcub::DeviceSelect::Flagged(tmp, tb, cnt, flag, items, nsel, n, s));
    int h_n = 0;
    chk(hipMemcpyAsync(&h_n, nsel, sizeof(int), hipMemcpyDeviceToHost, s));
    chk(hipStreamSynchronize(s));
    nitems = h_n > 0 ? (uint64_t)h_n : 0;
  }
  if (e == hipSuccess && nitems) {
    const int m = (int)nitems;
    uint64_t* ka = (uint64_t*)alloc(nitems * 8);
    uint64_t* kb = (uint64_t*)alloc(nitems * 8);
    uint32_t* ib = (uint32_t*)alloc(nitems * 4);
    uint32_t* len = (uint32_t*)alloc(nitems * 4);
    uint32_t* start = (uint32_t*)alloc((nitems + 1) * 4);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(gather, dim3(grid_of(nitems)), dim3(256), 0, s, D, key, items, nitems, ka);
      chk(hipGetLastError());
      // stable: within one (path, evaluation position) the runs keep D order
      size_t tb = 0;
      chk(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, ka, kb, items, ib, m, 0, 64, s));
      void* tmp = alloc(tb);
      chk(hipcub::DeviceRadixSort::SortPairs(tmp, tb, ka, kb, items, ib, m, 0, 64, s));
      hipLaunchKernelGGL(run_len, dim3(grid_of(nitems)), dim3(256), 0, s, D, ib, nitems, len);
      chk(hipGetLastError());
      size_t tb2 = 0;
      chk(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, len, start, m, s));
      void* tmp2 = alloc(tb2);
      chk(hipcub::DeviceScan::ExclusiveSum(tmp2, tb2, len, start, m, s));
      uint32_t last[2] = {0, 0};
      chk(hipMemcpyAsync(&last[0], start + (nitems - 1), 4, hipMemcpyDeviceToHost, s));
      chk(hipMemcpyAsync(&last[1], len + (nitems - 1), 4, hipMemcpyDeviceToHost, s));
      chk(hipStreamSynchronize(s));
      total = (uint64_t)nroots + last[0] + last[1];
      if (total > nD) e = hipErrorInvalidValue;  // every member is placed once
      if (e == hipSuccess) {
        hipLaunchKernelGGL(runs, dim3(grid_of(nitems)), dim3(256), 0, s, D, base, nroots, ib, start, nitems, newrun);
        hipLaunchKernelGGL(scatter, dim3(grid_of(nitems)), dim3(256), 0, s, D, nD, base, nroots, ib, start, nitems, newrun,
                           N, newpos);
        chk(hipGetLastError());
      }
    }
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(roots, dim3(grid_of(nrev)), dim3(256), 0, s, D, nD, base, root_d, slot, nrev, newrun, N, newpos);
    hipLaunchKernelGGL(gk::dlayout::cols, dim3(grid_of(ncols)), dim3(256), 0, s, cols, ncols, base, nD, newpos);
    chk(hipGetLastError());
    chk(hipStreamSynchronize(s));
  }
  for (void* p : owned) chk(hipFreeAsync(p, s));
  chk(hipStreamSynchronize(s));
  if (e == hipSuccess && n_out) *n_out = total;
  return (int)e;
}
