// Shared host/device definitions for the MI355X policy-evaluation engine.
//
// Everything the kernels read lives in flat, 16-byte-aligned arrays in HBM:
//   * Node      — one JSON value of a review / constraint-parameter / literal
//                 document (children of an object/array are contiguous);
//   * StrEnt    — interned string table (global ids; equal bytes == equal id);
//   * NumEnt    — number table (int64 + exact 64-bit-mantissa big.Float form);
//   * Ins       — predicate bytecode compiled from ConstraintTemplate Rego;
//   * MatchSpec — a constraint's compiled `spec.match` (kinds / namespaces /
//                 selectors / scope), evaluated by the match stage;
//   * ReviewCol — per-review match columns extracted by the host flattener.
#pragma once
#ifdef __HIPCC_RTC__
// runtime-compiled template kernels (jit.cc): hipRTC supplies the fixed-width types
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::uint16_t uint16_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::uint64_t uint64_t;
typedef __hip_internal::int8_t int8_t;
typedef __hip_internal::int16_t int16_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::int64_t int64_t;
#else
#include <stdint.h>
#endif

namespace gk {

// ----------------------------------------------------------------- documents
enum NodeType : uint8_t { NT_NONE = 0, NT_NULL = 1, NT_FALSE = 2, NT_TRUE = 3, NT_NUM = 4, NT_STR = 5, NT_ARR = 6, NT_OBJ = 7 };

struct Node {
  uint32_t key;    // object member: key string id; array element: index
  uint32_t val;    // NT_STR: string id; NT_NUM: number id
  uint32_t first;  // NT_ARR/NT_OBJ: absolute index of first child
  uint16_t n;      // child count
  uint8_t type;    // NodeType
  uint8_t flags;
};
static_assert(sizeof(Node) == 16, "Node must be 16 bytes");

struct StrEnt {
  uint32_t off;    // byte offset into the string pool
  uint32_t len;    // byte length
};

enum StrFlags : uint8_t { SF_ASCII_PRINT = 1, SF_NEEDS_ESC = 2, SF_NON_ASCII = 4 };

enum NumFlags : uint32_t { NF_INT64 = 1, NF_BF_OK = 2, NF_PRINT_OK = 4 };

struct NumEnt {
  int64_t i;        // value when NF_INT64 (json.Number.Int64 parses)
  uint64_t mant;    // big.Float at prec 64: mant in [2^63,2^64) (0 for zero)
  int32_t exp;      // value = mant * 2^exp
  uint32_t flags;
  uint32_t text;    // string id of the literal text (Term.String)
  uint32_t print;   // string id of the Go %v text (int / float64 conversion)
  uint32_t neg;
  uint32_t pad;
};
static_assert(sizeof(NumEnt) == 40, "NumEnt layout");

// ----------------------------------------------------------------- values
// 64-bit tagged VM values: tag in bits 60..63.
enum Tag : uint32_t {
  V_UNDEF = 0, V_NULL = 1, V_BOOL = 2, V_NUM = 3,  // NUM: number-table id
  V_STR = 4,                                       // STR: string id
  V_NODE = 5,                                      // NODE: node index (array/object)
  V_INT = 6,                                       // INT: computed int (48-bit two's complement)
  V_BFN = 7,                                       // BFN: heap word index of a computed big-float
  V_HSTR = 8,                                      // HSTR: lane byte-buffer string (off:16 | len:16)
  V_LIST = 9,                                      // LIST: heap list (set/array/object); kind in bits 56..59
  V_SLICE = 10,                                    // SLICE: string id:32 | start:14 | len:14
  V_FMT = 11,                                      // FMT: deferred sprintf (template kernels only): fidx:24 <<32 | args (bit31: node, else heap list offset)
  V_GSTR = 12,                                     // GSTR: string in the evaluation's memo-string arena (off:40 << 20 | len:20)
  V_GLIST = 13,                                    // GLIST: a list copied out at emission (devrt.h gval_copy): kind in bits
                                                   // 56..59, the word offset of [len, 0, words...] in ebytes
  // columnar staged batches (colstore.cc): a document object / array read from
  // the batch's path columns instead of the node store
  V_ROW = 14,                                      // ROW: object view:12 << 40 | row:40
  V_ROWS = 15,                                     // ROWS: array -- element table:12 << 48 | first row:32 << 16 | length:16
};
enum ListKind : uint32_t { LK_SET = 1, LK_ARR = 2, LK_OBJ = 3 };

// ----------------------------------------------------------------- bytecode
enum Op : uint16_t {
  OP_END = 0,
  OP_JMP,          // x
  OP_JUNDEF,       // a, x : jump if R[a] undefined
  OP_JFALSE,       // a, x : jump if R[a] == false
  OP_JTRUE,        // a, x : jump if R[a] == true
  OP_LOADK,        // a, x : R[a] = K[x]
  OP_LOADREV,      // a    : R[a] = review root
  OP_LOADPARAM,    // a    : R[a] = constraint parameters
  OP_MOV,          // a, b
  OP_GET,          // a, b, c : R[a] = R[b][R[c]]
  OP_GETK,         // a, b, x : R[a] = R[b][K[x]]
  OP_ITER_INIT,    // a(iter base: a=coll, a+1=pos), b=coll
  OP_ITER_NEXT,    // a(iter base), b(key dst|0xffff), c(val dst|0xffff), x=exit
  OP_CMP,          // a, b, c, y=cmp kind : R[a] = bool
  OP_ARITH,        // a, b, c, y=kind
  OP_LIST_NEW,     // a, y=kind
  OP_LIST_ADD,     // a(list), b(value)      : set/array append (set dedupes)
  OP_OBJ_PUT,      // a(obj), b(key), c(value)
  OP_YIELD,        // a(out), b(val) : conflict check + assign
  OP_CALL,         // a(dst), b(arg base), c(nargs), y=builtin id
  OP_SPRINTF,      // a(dst), b(args list), x=format index
  OP_EMIT,         // a(msg), b(details), y=rule index
  OP_LEN_EQ,       // a(dst bool), b(value), y=n : collection length test (array patterns)
  OP_FAIL_FALLBACK,// y=reason : unsupported construct reached at run time
  OP_TABLE,        // a = lookup(K[x..]: n, (key, value) x n ; R[b]) — constant-table function call
  OP_MEMO_GET,     // memo slot y holds (R[b], R[c]) -> R[a] = cached value, jump x   (c = 0xffff: one arg)
  OP_MEMO_PUT,     // memo slot y := (R[b], R[c]) -> R[a] when arguments and value are heap-free
  OP_ORD,          // y: emission order key of fused rule bodies (compiler.cc rule_group):
                   //    y < 2^31: key = base + y; else base += y & 0x7fffffff, key = base
  // inventory joins (compiler.cc join_site, devrt.h op_jprobe): an iteration
  // over data.inventory leaves whose key equals R[b] through the constraint's
  // join index, or a jump to the plain scan when there is none
  OP_JPROBE,       // a(iter base: a=range, a+1=pos), b(probe value), x=scan path, y=loop depth | site << 8
  OP_JNEXT,        // a(iter base), b(leaf dst), x=exit, y=loop depth : next candidate leaf
  OP_JVAR,         // a(dst), b(iter base), y=selector : the current leaf's key at path variable y
  OP_KEYOUT,       // a : key pass (gk_key_kernel) -- the leaf's join key hash
  OP_COUNT_
};

struct Ins {
  uint16_t op, a, b, c;
  uint32_t x, y;
};
static_assert(sizeof(Ins) == 16, "Ins must be 16 bytes");

enum CmpKind : uint32_t { CMP_EQ = 0, CMP_NE, CMP_LT, CMP_LE, CMP_GT, CMP_GE };
enum ArithKind : uint32_t { AR_PLUS = 0, AR_MINUS, AR_MUL, AR_DIV, AR_REM, AR_OR, AR_AND };

enum Builtin : uint32_t {
  BI_COUNT = 0, BI_ANY, BI_ALL, BI_STARTSWITH, BI_ENDSWITH, BI_CONTAINS, BI_RE_MATCH, BI_TO_NUMBER,
  BI_REPLACE, BI_SUBSTRING, BI_IS_NUMBER, BI_IS_STRING, BI_IS_BOOLEAN, BI_IS_ARRAY, BI_IS_OBJECT,
  BI_IS_SET, BI_IS_NULL, BI_LOWER, BI_UPPER, BI_TRIM, BI_SPLIT, BI_CONCAT, BI_INDEXOF,
  BI_TRIM_PREFIX, BI_TRIM_SUFFIX, BI_SORT, BI_ARRAY_CONCAT, BI_COUNT_
};

// per-(review) outcome flags
enum ReviewFlags : uint32_t {
  RF_ERROR = 1u,      // the reference Query would return an error for this review
  RF_FALLBACK = 2u,   // evaluation needs the CPU OPA driver (value/builtin outside the GPU subset)
  RF_OVERFLOW = 4u,   // output buffer overflow (host re-runs)
};

// fallback reason codes (diagnostics)
enum Reason : uint32_t {
  FB_NONE = 0, FB_HEAP, FB_MSG_LEN, FB_NUMBER, FB_UNICODE, FB_DEEP_EQ, FB_REGEX, FB_PRINT, FB_TYPE,
  FB_UNSUPPORTED, FB_MATCH, FB_STRING,
  FB_TEMPLATE,  // a template expression outside the GPU subset was reached (guard programs)
};

// ----------------------------------------------------------------- match
constexpr uint32_t NO_ID = 0xffffffffu;

// A label selector compiled for the match stage (target_template_source.go:185-230).
// Encoded in the constraint side table as u32 words:
//   [n_match_labels, (key, val)*n, n_exprs, (op, key, n_vals, vals...)*]
enum SelOp : uint32_t { SO_IN = 1, SO_NOTIN = 2, SO_EXISTS = 3, SO_DOESNOTEXIST = 4, SO_OTHER = 5 };

enum MatchFlags : uint32_t {
  MF_HAS_NAMESPACES = 1, MF_HAS_EXCLUDED = 2, MF_HAS_NSSEL = 4, MF_SCOPE_PRESENT = 8,
  MF_SCOPE_ANY = 16, MF_SCOPE_NS = 32, MF_SCOPE_CLUSTER = 64, MF_FALLBACK = 128, MF_ERROR = 256,
};

struct MatchSpec {
  uint32_t flags;
  uint32_t kinds_off;     // word offset in the match word table: [n_sel, (n_groups, g.., n_kinds, k..)*]
  uint32_t ns_off;        // [n, ids...]
  uint32_t exns_off;      // [n, ids...]
  uint32_t labelsel_off;  // selector words
  uint32_t nssel_off;     // selector words
  uint32_t prog;          // program index of the template
  uint32_t params;        // node index of spec.parameters (or NO_ID => {})
  // LDS staging (template kernels, devrt.h stage_wave): the node window
  // [plo, plo + pn) holding the whole parameters subtree (pn = 0: not staged),
  // and the offset of the constraint's regex stage record in `stage`
  // (NO_ID: none) -- [n, then per DFA: pattern sid, word offset in dfa_c,
  // bytes, nst | ncls << 16, start | sens << 16]
  uint32_t plo, pn;
  uint32_t stage_off;
  uint32_t pad_;
};
static_assert(sizeof(MatchSpec) == 48, "MatchSpec layout");

enum ReviewColFlags : uint32_t {
  RC_KIND_OK = 1,         // review.kind.{group,kind} are strings
  RC_IS_NS = 2,           // kind.group == "" && kind.kind == "Namespace"
  RC_HAS_NS = 4,          // review.namespace defined (string)
  RC_NS_EMPTY = 8,        // get_default(review, "namespace", "") == ""
  RC_UNSTABLE_NS = 16,    // review._unstable.namespace is truthy (object)
  RC_NS_CACHED = 32,      // namespace object found in data.external cluster cache
  RC_LABELS_OBJ = 64,     // any_labelselector_match uses object labels
  RC_LABELS_OLD = 128,    // any_labelselector_match uses oldObject labels
  RC_NAME_OK = 256,       // object.metadata.name defined (for Namespace kinds)
  RC_FALLBACK = 512,      // review shape outside the match fast path
  RC_REVIEW_DEF = 1024,   // input.review defined
  RC_EXCLUDED = 2048,     // namespace excluded for the audit process (excluder.go:82-86): not reviewed
  RC_AUDIT = 4096,        // a hooks.audit review (matching_reviews_and_constraints, regolib src.go:45-62):
                          // that rule never joins autoreject_review, so no "not cached" row
};

struct ReviewCol {
  uint32_t root;      // review document root node
  uint32_t group;     // string ids
  uint32_t kind;
  uint32_t ns;        // namespace string id (review.namespace) or NO_ID
  uint32_t nsname;    // is_ns ? object.metadata.name : review.namespace
  uint32_t labels;    // node of object labels ({} => NO_ID)
  uint32_t old_labels;
  uint32_t ns_labels; // labels node of the namespace object used by namespaceSelector
  uint32_t flags;
  uint32_t orig;      // index of the review in the caller's batch (NO_ID: its position);
                      // staged batches are evaluated in document-size order
  uint32_t pad[2];
};
static_assert(sizeof(ReviewCol) == 48, "ReviewCol layout");

// ----------------------------------------------------------------- output
// One violation tuple.  Byte offsets are 64-bit: a 10M-resource sweep can
// write more than 4 GiB of message bytes in one call.  The details JSON
// follows the message: [msg_off, +msg_len) then [msg_off + msg_len, +det_len).
struct Viol {
  uint32_t review;
  uint32_t constraint;
  uint16_t seq;       // emission order within (review, constraint)
  uint16_t rule;      // template rule index (0xffff = autoreject)
  uint32_t msg_len;
  uint64_t msg_off;
  uint32_t det_len;
  uint32_t pad;
};
static_assert(sizeof(Viol) == 32, "Viol layout");

constexpr uint32_t RULE_AUTOREJECT = 0xffffu;

// audit status sample record (kernels.hip gk_sample_select): a tuple plus the
// first SAMPLE_MSG bytes of its message
constexpr uint32_t SAMPLE_MSG = 256;
struct SampleRec {
  uint32_t review, constraint;
  uint16_t seq, rule;
  uint32_t msg_len, pad;
  uint8_t msg[SAMPLE_MSG];
};
static_assert(sizeof(SampleRec) == 276, "SampleRec layout");
constexpr uint32_t MEMO_SLOTS = 16;  // memoized function call sites per template (per lane)
constexpr uint32_t GMEMO_ENTRIES = 1u << 15;  // cross-lane memo table of a template launch (32 B entries)
constexpr uint64_t MSTR_BYTES = 16ull << 20;  // memo-string arena of an evaluation (V_GSTR)

// ------------------------------------------------------------------ launch
// Kernel arguments of one audit launch (passed by value; shared by the bytecode
// VM kernel in kernels.hip and the per-template kernels jit.cc compiles).
struct DevArgs {
  const Node* nodes;
  const StrEnt* strs;
  const uint8_t* pool;
  const uint8_t* sflags;
  const NumEnt* nums;
  const Ins* code;
  const uint64_t* K;
  const uint32_t* fmt;
  const MatchSpec* cons;
  const uint32_t* mwords;
  const uint32_t* prog_off;
  const ReviewCol* revs;
  const uint32_t* dfa_keys;   // sorted pattern string ids
  const uint32_t* dfa_meta;   // per entry: word offset into dfa_words | status<<30
  const uint32_t* dfa_words;
  uint32_t ndfa;
  uint32_t ncode;
  uint32_t ncons;
  uint32_t nrev;
  uint32_t ntiles;            // ceil(nrev / 64)
  const uint32_t* clist;      // constraints this launch evaluates (wave -> tile x clist[j])
  uint32_t nclist;
  Viol* out;
  uint64_t out_cap;
  unsigned long long* counters;  // [0] = tuples, [1] = bytes, [2] = lanes that flagged their review
  char* bytes;
  uint64_t bytes_cap;
  uint32_t* rflags;
  unsigned long long* totals;    // per constraint violation count
  uint32_t* rreason;          // per review fallback reason (diagnostic)
  unsigned int* pchist;       // optional (GKGPU_PROFILE=2): executions per bytecode pc
  unsigned long long* prof;   // optional: per constraint [sum steps, max lane steps, lanes run, sum wave-max steps]
  uint64_t* gmemo;            // template kernels: cross-lane memo of pure function calls (4 words per entry)
  uint32_t gmemo_mask;        // entries - 1 (power of two)
  uint32_t nperm;             // node ids below this are the permanent region (constraints, inventory):
                              // memo keys (devrt.h gm_key)
  char* mstr;                 // memo-string arena of the evaluation (V_GSTR bytes; null: off)
  unsigned long long* mstr_top;  // its bump cursor (bytes used)
  uint64_t mstr_cap;
  uint64_t gm_salt;           // per launch: mixed into memo hashes, so launches sharing a
                              // memo table (one clear per evaluation) never read each other's entries
  uint64_t* frec;             // per output tuple, a deferred message's argument words, structure
                              // of arrays: word j of tuple i at frec[j * out_cap + i]
  char* ebytes;               // bytes that existed at emission (eager messages, details JSON)
  uint64_t ebytes_cap;
  const uint32_t* stage;      // per-constraint LDS stage records (MatchSpec.stage_off)
  const uint32_t* dfa_c;      // byte-class-compressed DFAs the stage records point at
  uint32_t* lens;             // size pass: output bytes per tuple (message + details)
  unsigned long long* part;   // size pass: per tile of FTILE tuples, its bytes; then the
                              // exclusive prefix over tiles (spine)
  // inventory join indexes (engine.cc build_joins; null: every join site scans)
  const uint32_t* jdir;       // per (constraint, site): [hash offset, entries, ready, pad] (JMAX_SITES sites)
  const uint64_t* jhash;      // key hashes, sorted within each index
  const uint32_t* jord;       // per hash entry: word offset of its leaf row in jleaf (leaf order within a hash)
  const uint64_t* jleaf;      // leaf rows: [leaf value, key at each path variable...]
  // key pass (gk_key_kernel): leaf i = jleaf[jrow0 + i * jstride], its key
  // hashes -> jkeys[i * JKEYS_MAX ..] (KH_NONE-padded)
  uint64_t* jkeys;
  uint64_t jparams;           // the constraint's parameters value
  uint32_t jpc, jstride;
  uint64_t jrow0;
  // the format table with its literal segments resolved (engine.cc
  // sync_tables): same offsets as `fmt`; a literal segment is
  // (0 | len << 8, byte offset in fmtb) instead of (0, string id), so the
  // size / format passes print literals without the string table (null: off)
  const uint32_t* fmtr;
  const char* fmtb;           // the literals' bytes, padded to a dword
  uint32_t nfmt, nfmtb;       // words of fmtr, bytes of fmtb
  // columnar staged batch (colstore.cc; cv_on = 0: the review documents are
  // node trees).  The review at evaluation position r is V_ROW(view 0, row r).
  const uint32_t* cv_words;   // every path column's value words (CW_*), one per row of its table
  const uint8_t* cv_bytes;    // the byte columns (CVS_BYTES)
  const struct CvSlot* cv_slots;
  const struct CvHash* cv_hash;  // (object view, member key) -> slot, open addressing
  const uint32_t* cv_views;   // per object view: CV_COMPLETE
  const uint32_t* cv_tabs;    // per element table: the slot of its elements
  uint32_t cv_hmask;          // hash entries - 1
  uint32_t cv_on;
};

// ----------------------------------------------------------------- path columns
// A column's value word per row: tag in bits 29..31, payload below.
enum ColWord : uint32_t {
  CW_ABSENT = 0,  // undefined at this row
  CW_STR = 1,     // interned string id
  CW_NUM = 2,     // number-table id
  CW_LIT = 3,     // 0 null, 1 false, 2 true
  CW_OBJ = 4,     // an object: V_ROW(the slot's view, this row)
  CW_ARR = 5,     // an array: its elements are rows [payload, + length column) of the slot's table
  CW_NODE = 6,    // kept as document nodes (a path used whole): node index
};
constexpr uint32_t CW_SHIFT = 29, CW_PAY = (1u << 29) - 1;
struct CvSlot {
  uint32_t col;     // word offset of the value column (row r at col + r)
  uint32_t lencol;  // word offset of the array-length column (CW_ARR rows), NO_ID if none
  uint16_t view;    // CW_OBJ rows: the object view of this path
  uint16_t tab;     // CW_ARR rows: the element table of this path
  uint32_t flags;   // CVS_BYTES: the column is bytes in cv_bytes (cv_byte_word)
};
static_assert(sizeof(CvSlot) == 16, "CvSlot layout");
struct CvHash {
  uint32_t view, key, slot, pad;  // view == NO_ID: empty entry
};
static_assert(sizeof(CvHash) == 16, "CvHash layout");
constexpr uint32_t CV_COMPLETE = 1;  // every member key the batch has at this path has a slot
// A path whose values carry no payload (objects only tested or navigated,
// null / booleans, undefined) is a byte column: tag << 2 | the literal
constexpr uint32_t CVS_BYTES = 1;
constexpr uint32_t cv_byte_word(uint32_t b) { return ((b >> 2) << CW_SHIFT) | (b & 3u); }
constexpr uint8_t cv_word_byte(uint32_t w) { return (uint8_t)(((w >> CW_SHIFT) << 2) | (w & 3u)); }
constexpr uint32_t cv_hash_of(uint32_t view, uint32_t key) {  // (constexpr: host and device)
  uint32_t h = view * 0x9E3779B1u ^ key * 0x85EBCA77u;
  return h ^ (h >> 15);
}
// join sites per template program (compiler.cc join_site)
constexpr uint32_t JMAX_SITES = 4;
// keys one leaf may have (a key over a generator, `other.spec.rules[_].host`);
// a leaf with more leaves its site unindexed
constexpr uint32_t JKEYS_MAX = 8;
// gk_key_kernel results besides a hash (a string key's hash has bit 63 set)
constexpr uint64_t KH_NONE = 0;       // key undefined or composite: the leaf is in no bucket
constexpr uint64_t KH_FAIL = 1;       // the key program failed (error / fallback): no index, scan
constexpr uint64_t KH_NUM = 2, KH_NULL = 3, KH_FALSE = 4, KH_TRUE = 5;
// A deferred message's sprintf takes at most FMT_MAXARGS arguments (the
// argument words a tuple carries in frec)
constexpr uint32_t FMT_MAXARGS = 6;
// Viol.pad while the predicate kernels run (the format pass clears it):
//   VF_DEFER   msg_len = fidx | nargs << 24, the arguments in frec; the size
//              pass prints its length, the format pass the bytes
//   VF_DET_OBJ the details are the hook default `{}` (no staged bytes)
//   VF_DET_VAL the details are the JSON of one frec word (index: the message's
//              argument count when VF_DEFER, else 0), printed by the passes;
//              the size pass stores their length in det_len
// otherwise msg_len is the message length and ebytes[msg_off, ...) holds the
// message (eager) followed by the details (unless VF_DET_OBJ / VF_DET_VAL); a
// deferred message's details (unless VF_DET_*) are at ebytes[msg_off, +det_len)
//   VF_NOPRINT set by the size pass: the message or details cannot be printed
//              on the GPU (the review goes to the CPU); the tuple gets no bytes
//   VF_DET_KV  (with VF_DEFER) the details are a one-member object {k: v}: k
//              and v are the two frec words after the message's arguments
//              (k8sallowedlabelregex's {"label": key}); printed like VF_DET_VAL
constexpr uint32_t VF_DEFER = 1, VF_DET_OBJ = 2, VF_DET_VAL = 4, VF_NOPRINT = 8, VF_DET_KV = 16;
// the size / format passes work in tiles of FTILE consecutive tuples
constexpr uint32_t FTILE = 256;  // one block pass: a small output still spreads over many blocks

}  // namespace gk
