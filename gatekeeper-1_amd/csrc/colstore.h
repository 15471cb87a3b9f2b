// Columnar staged batches (north_star: "flattens resource JSON into
// columnar, path-interned string and offset arrays in HBM").
//
// The reference marshals every object whole, once per Review
// (pkg/target/target.go:145, drivers/local/local.go:331).  A staged batch in
// column form uploads only what the batch's compiled programs read
// (colplan.h): per referenced path, one 4-byte value word per row (common.h
// CW_*) -- strings and numbers as interned ids, objects as views whose members
// are the path's own columns, arrays as CSR ranges of an element table -- and
// document nodes only for the paths a program reads whole (label objects the
// match stage scans, objects a template iterates or prints).
#pragma once
#include <sys/mman.h>

#include <cstdint>
#include <cstdlib>
#include <new>
#include <utility>
#include <mutex>
#include <string>
#include <vector>

#include "colplan.h"
#include "common.h"
#include "store.h"

namespace gk {

// An uninitialised array (every element is written before it is read): the
// build's threads write their own chunks' rows, so the first touch of the
// pages -- and their zeroing -- is spread over them instead of one serial
// fill of ~250 MB.  Large buffers are 2 MB aligned and marked for huge pages.
template <class T>
struct RawBuf {
  T* p = nullptr;
  size_t n = 0;
  RawBuf() = default;
  RawBuf(const RawBuf&) = delete;
  RawBuf& operator=(const RawBuf&) = delete;
  ~RawBuf() { free(p); }
  void resize(size_t k) {
    free(p);
    p = nullptr;
    n = k;
    if (!k) return;
    const size_t bytes = k * sizeof(T);
    void* m = nullptr;
    if (bytes >= (32u << 20)) {
      if (posix_memalign(&m, 2u << 20, bytes) != 0) m = nullptr;
      if (m) madvise(m, bytes, MADV_HUGEPAGE);
    } else {
      m = malloc(bytes);
    }
    if (!m) throw std::bad_alloc();
    p = (T*)m;
  }
  size_t size() const { return n; }
  T* data() { return p; }
  const T* data() const { return p; }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
  T* begin() { return p; }
  T* end() { return p + n; }
  const T* begin() const { return p; }
  const T* end() const { return p + n; }
};
using WordBuf = RawBuf<uint32_t>;
using ByteBuf = RawBuf<uint8_t>;

struct ColStore {
  WordBuf words;                // every word column's values
  ByteBuf bytes;                // the byte columns (CVS_BYTES)
  std::vector<CvSlot> slots;
  std::vector<CvHash> hash;     // power-of-two size
  std::vector<uint32_t> views;  // per object view: CV_COMPLETE
  std::vector<uint32_t> tabs;   // per element table: the slot of its elements
  NodeArena nodes;              // the subtrees kept as nodes: ids node_begin + k
  RawBuf<ReviewCol> cols;       // the review columns with node ids into `nodes`
  uint32_t node_begin = 0;
  uint64_t rows = 0;            // rows of every table (reviews + elements)
  std::string schema;           // description (diagnostics)
  uint64_t total_bytes() const {
    return words.size() * 4 + bytes.size() + slots.size() * sizeof(CvSlot) + hash.size() * sizeof(CvHash) + views.size() * 4 +
           tabs.size() * 4 + nodes.size() * sizeof(Node) + cols.size() * sizeof(ReviewCol);
  }
};

// Builds the column form of a staged batch whose documents are `arena` (node
// id node_begin + k at arena[k]; ids below node_begin are the permanent
// region `perm`) and whose reviews, in evaluation order, are `cols`.  False
// (and `why`) when the batch does not fit the form: the node mode stays.
bool build_columns(const PathPlan& plan, const Node* perm, uint32_t node_begin, const Node* arena, size_t n_arena,
                   const std::vector<ReviewCol>& cols, const Store& st, std::mutex& smu, ColStore& out,
                   std::string& why);

}  // namespace gk
