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
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "colplan.h"
#include "common.h"
#include "store.h"

namespace gk {

struct ColStore {
  std::vector<uint32_t> words;  // every column's value words
  std::vector<CvSlot> slots;
  std::vector<CvHash> hash;     // power-of-two size
  std::vector<uint32_t> views;  // per object view: CV_COMPLETE
  std::vector<uint32_t> tabs;   // per element table: the slot of its elements
  std::vector<Node> nodes;      // the subtrees kept as nodes: ids node_begin + k
  std::vector<ReviewCol> cols;  // the review columns with node ids into `nodes`
  uint32_t node_begin = 0;
  uint64_t rows = 0;            // rows of every table (reviews + elements)
  std::string schema;           // description (diagnostics)
  uint64_t bytes() const {
    return words.size() * 4 + slots.size() * sizeof(CvSlot) + hash.size() * sizeof(CvHash) + views.size() * 4 +
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
