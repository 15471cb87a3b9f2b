/*
 * gkgpu — MI355X batch policy-evaluation engine for Gatekeeper's audit sweep.
 *
 * C ABI of libgkgpu.so.  The first block mirrors the constraint framework's
 * plugin boundary one-for-one, so a cgo shim can implement drivers.Driver on
 * top of it:
 *
 *   vendor/github.com/open-policy-agent/frameworks/constraint/pkg/client/
 *     drivers/interface.go:21-39   type Driver interface { Init; PutModule;
 *     PutModules; DeleteModule; DeleteModules; PutData; DeleteData; Query; Dump }
 *
 * replacing the local OPA driver selected at main.go:223-229
 * (local.New(local.Tracing(false))).  The second block adds the batch entry
 * points the audit loop (pkg/audit/manager.go:333-398) and the webhook
 * micro-batch use.  Ownership: every input buffer is borrowed for the
 * duration of the call only (the engine copies/flattens it); results are
 * engine-allocated and released with gk_results_free.  Every function
 * returns 0 on success or a GK_E* code; gk_last_error() holds the message of
 * the calling thread's last failure.
 *
 * Threading follows the local driver's RWMutex (drivers/local/local.go:62-68,
 * 117, 303-304): evaluations (gk_query, gk_query_batch, gk_review_*,
 * gk_batch_stage_*, gk_batch_eval*) run concurrently -- each on its own
 * evaluation context (HIP stream, output buffers, per-launch kernel
 * arguments) -- while mutations (gk_put_* / gk_delete_*, excluder changes)
 * are exclusive: a mutation waits for the evaluations in flight and new
 * evaluations wait for it, so every evaluation sees one engine state from
 * start to end (gk_results_generation names it).  A staged batch belongs to
 * the state it was staged in.
 */
#ifndef GKGPU_H
#define GKGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GK_OK 0
#define GK_EINVAL 1      /* bad argument / malformed JSON / bad path        */
#define GK_EPARSE 2      /* Rego parse / compile error (PutModule(s))      */
#define GK_EQUERY 3      /* unsupported query path                          */
#define GK_EDEVICE 4     /* HIP runtime failure / no MI355X visible         */
#define GK_ENOTFOUND 5
#define GK_ERANGE 6      /* a value did not fit the caller's fixed-size field   */

/* per-review status in gk_results (bit set) */
#define GK_REVIEW_ERROR 1u     /* reference Query would return an error    */
#define GK_REVIEW_FALLBACK 2u  /* route this review to the CPU OPA driver  */
#define GK_REVIEW_EXCLUDED 4u  /* namespace excluded for the audit process:
                                  not reviewed (manager.go:362-365)          */

typedef struct gk_engine gk_engine;
typedef struct gk_results gk_results;
typedef struct gk_batch gk_batch;

/* opts_json (may be NULL): {"device": 0, "max_violations": N,
 *   "coalesce_us": W, "coalesce_max": M}
 * coalesce_us > 0 turns on the webhook micro-batch coalescer:
 * concurrent gk_query(violation) calls -- one per admission request in the
 * reference, pkg/webhook/policy.go:371-387 -- are evaluated together in one
 * launch of up to M (default 256) reviews, or whatever arrived within W
 * microseconds of the first; each caller still gets its own gk_results. */
int gk_engine_create(const char* opts_json, gk_engine** out);
void gk_engine_destroy(gk_engine* e);
const char* gk_last_error(gk_engine* e);
/* 1 if a HIP device is usable by this engine */
int gk_device_available(void);

/* ---- drivers.Driver (interface.go:21-39) -------------------------------- */
/* Driver.Init — interface.go:22 */
int gk_init(gk_engine* e);
/* Driver.PutModule(ctx, name, src string) error — interface.go:24; the hooks
 * and target-library modules (client.go:667-722) are recognized and served
 * natively; template modules compile to GPU bytecode or are marked FALLBACK. */
int gk_put_module(gk_engine* e, const char* name, const char* src, size_t len);
/* Driver.PutModules(ctx, namePrefix string, srcs []string) error — interface.go:26 */
int gk_put_modules(gk_engine* e, const char* prefix, const char* const* srcs, const size_t* lens, size_t n);
/* Driver.DeleteModule(ctx, name) (bool, error) — interface.go:28 */
int gk_delete_module(gk_engine* e, const char* name, int* deleted);
/* Driver.DeleteModules(ctx, namePrefix) (int, error) — interface.go:30 */
int gk_delete_modules(gk_engine* e, const char* prefix, int* count);
/* Driver.PutData(ctx, path string, data interface{}) error — interface.go:32;
 * data passed as JSON text (constraints under /constraints/<target>/...,
 * synced inventory under /external/<target>/...; client.go:79-113, 498-510) */
int gk_put_data(gk_engine* e, const char* path, const char* json, size_t len);
/* Driver.DeleteData(ctx, path) (bool, error) — interface.go:34 */
int gk_delete_data(gk_engine* e, const char* path, int* deleted);
/* Driver.Query(ctx, path, input, opts...) (*types.Response, error) —
 * interface.go:36.  path: `hooks["admission.k8s.gatekeeper.sh"].violation`
 * (input = {"review": ...}) or `hooks["admission.k8s.gatekeeper.sh"].audit`
 * (input ignored).  Results carry (review index, constraint, msg, details,
 * enforcementAction) per types.Result (types/validation.go:11-29). */
int gk_query(gk_engine* e, const char* path, const char* input_json, size_t len, gk_results** out);
/* Driver.Dump(ctx) (string, error) — interface.go:38; caller frees with gk_free_string */
int gk_dump(gk_engine* e, char** out);
void gk_free_string(char* s);

/* ---- batch extensions ----------------------------------------------------- */
/* n independent Query(violation, inputs[i]) calls in one launch (webhook micro-batch) */
int gk_query_batch(gk_engine* e, const char* const* inputs, const size_t* lens, size_t n, gk_results** out);
/* the coalescer's launches and the gk_query calls they served (diagnostics) */
int gk_coalesce_stats(gk_engine* e, uint64_t* batches, uint64_t* requests);
/* hooks.audit (Client.Audit, client.go:805-833) keeps the synced inventory as a
 * device-resident staged batch, rebuilt after any mutation: how many times it
 * was built, and the reviews of the current one. */
int gk_audit_cache_stats(gk_engine* e, uint64_t* builds, uint64_t* reviews);
/* audit discovery mode: Review(AugmentedUnstructured{objs[i], ns(objs[i])}) for
 * every object (pkg/audit/manager.go:361-389, pkg/target/target.go:129-163).
 * ns_json[i] is the JSON of the object's corev1.Namespace (NULL / len 0 for
 * cluster-scoped objects, which the reference reviews with an empty Namespace{}). */
int gk_review_objects(gk_engine* e, const char* const* objs, const size_t* obj_lens, const char* const* ns_json,
                      const size_t* ns_lens, size_t n, gk_results** out);

/* staged (device-resident) batches for the audit sweep: flatten + upload once,
 * evaluate many times.  stage_objects has gk_review_objects' semantics. */
int gk_batch_stage_objects(gk_engine* e, const char* const* objs, const size_t* obj_lens, const char* const* ns_json,
                           const size_t* ns_lens, size_t n, gk_batch** out);
/* The same two entry points over one List page in bulk form (the audit loop's
 * objList.Items, manager.go:361-389): objects as concatenated JSON texts with
 * n + 1 byte offsets, the page's distinct Namespace objects (the nsCache,
 * manager.go:96-115) with n_ns + 1 offsets, and per object the index of its
 * Namespace (UINT32_MAX = cluster-scoped: reviewed with an empty
 * corev1.Namespace{}, target.go:137-139).  Objects are parsed and flattened on
 * GKGPU_THREADS host threads (default: the leased host cores -- the CPU affinity
 * set, capped by a cgroup CPU quota). */
int gk_review_page(gk_engine* e, const char* objs, const uint64_t* obj_offs, size_t n, const char* nss,
                   const uint64_t* ns_offs, size_t n_ns, const uint32_t* obj_ns, gk_results** out);
int gk_batch_stage_page(gk_engine* e, const char* objs, const uint64_t* obj_offs, size_t n, const char* nss,
                        const uint64_t* ns_offs, size_t n_ns, const uint32_t* obj_ns, gk_batch** out);
/* host milliseconds of staging: [parse + build documents, flatten total, upload] */
int gk_batch_timing(const gk_batch* b, double* ms3);
/* reviews of the batch the process excluder skipped */
uint64_t gk_batch_excluded(const gk_batch* b);

/* HandleViolation's Result.Resource identity for a review of the batch
 * (pkg/target/target.go:193-244): apiVersion = "<group>/<version>" or
 * "<version>" when the group is "", kind = review.kind.kind, and the object's
 * metadata name / namespace.  NUL-terminated; GK_ERANGE if a field was cut. */
#define GK_RESOURCE_FIELD 512
typedef struct {
  char api_version[GK_RESOURCE_FIELD];
  char kind[GK_RESOURCE_FIELD];
  char name[GK_RESOURCE_FIELD];
  char namespace_[GK_RESOURCE_FIELD];
} gk_resource;
int gk_batch_resource(gk_engine* e, const gk_batch* b, size_t review, gk_resource* out);

/* evaluate a staged batch; decode=0 keeps results on the device (counts only) */
int gk_batch_eval(gk_engine* e, gk_batch* b, int decode, gk_results** out);
void gk_batch_free(gk_batch* b);
/* bytes of review documents + match columns resident in HBM for the batch */
uint64_t gk_batch_device_bytes(const gk_batch* b);
/* algorithmic input of one sweep over the batch: reviews, document nodes (16 B
 * each), bytes of the distinct string values they reference, match-column bytes */
int gk_batch_stats(const gk_batch* b, uint64_t* reviews, uint64_t* nodes, uint64_t* str_bytes, uint64_t* col_bytes);

/* One audit sweep of a staged batch as the audit status needs it
 * (pkg/audit/manager.go:462-508): gk_results_constraint_total = exact
 * per-constraint totals over the reviews the engine answered (flagged reviews
 * excluded: CPU OPA answers them), and gk_results_sample_* = the first `limit`
 * results per constraint in evaluation order (batch review index, autoreject
 * first, emission order), selected on the device so that only
 * constraints x limit records leave it.  Messages carry their first
 * GK_SAMPLE_MSG bytes (the status truncates at 256, manager.go:622-631). */
#define GK_SAMPLE_MSG 256
int gk_batch_eval_audit(gk_engine* e, gk_batch* b, uint32_t limit, gk_results** out);
/* --audit-from-cache as the audit manager consumes it: Client.Audit
 * (hooks.audit, client.go:805-833) over the synced inventory's staged batch
 * (built as gk_query(hooks.audit) builds it, reused until a mutation), with
 * the sweep reduced on the device as gk_batch_eval_audit does -- exact
 * per-constraint totals and the first `limit` results per constraint
 * (manager.go:195-207 then addAuditResponsesToUpdateLists :462-508) -- so no
 * result row is decoded on the host.  Reviews are numbered in inventory path
 * order (gk_results_sample_* review indexes). */
int gk_audit_cache_sample(gk_engine* e, uint32_t limit, gk_results** out);
typedef struct {
  uint32_t review, constraint;
  uint16_t seq, rule;          /* rule 0xffff = autoreject */
  uint32_t msg_len;            /* full message length */
  const char* msg;             /* first msg_stored bytes (not NUL-terminated) */
  size_t msg_stored;
  const char* enforcement_action;
} gk_sample_view;
size_t gk_results_sample_count(const gk_results* r);
int gk_results_sample_get(const gk_results* r, size_t i, gk_sample_view* out);
/* every sample in one buffer: per sample u32 review, u32 constraint, u16 seq,
 * u16 rule, u32 msg_len, u32 stored, then `stored` message bytes.  *needed
 * receives the size; GK_EINVAL when cap is smaller (nothing written). */
int gk_results_samples_export(const gk_results* r, void* buf, size_t cap, size_t* needed);
/* the constraint's enforcementAction as results report it */
const char* gk_results_constraint_action(const gk_results* r, size_t constraint);

/* ---- process excluder (pkg/controller/config/process/excluder.go) --------- */
/* Excluder.Add(MatchEntry{ExcludedNamespaces: namespaces, Processes: processes})
 * — excluder.go:44-68; process "*" adds the namespaces to audit, webhook and
 * sync.  The audit entry points (gk_review_objects, gk_review_page, staged
 * batches) skip objects whose metadata.namespace is excluded for "audit"
 * (manager.go:362-365): no results, status GK_REVIEW_EXCLUDED.  Changing the
 * exclusions invalidates staged batches. */
int gk_excluder_add(gk_engine* e, const char* const* processes, size_t np, const char* const* namespaces, size_t nn);
/* Excluder.Replace(New()) */
int gk_excluder_clear(gk_engine* e);
/* Excluder.IsNamespaceExcluded(process, ns) — excluder.go:82-86 */
int gk_excluder_is_excluded(gk_engine* e, const char* process, const char* ns);

/* ---- results ------------------------------------------------------------- */
typedef struct {
  uint32_t review;          /* index of the input / object in the call */
  uint32_t constraint;      /* engine constraint index */
  const char* constraint_kind;
  const char* constraint_name;
  const char* msg;          /* UTF-8, not NUL-terminated */
  size_t msg_len;
  const char* details_json; /* json.Marshal of Result.Metadata["details"] */
  size_t details_len;
  const char* enforcement_action;
} gk_result_view;

size_t gk_results_count(const gk_results* r);
int gk_results_get(const gk_results* r, size_t i, gk_result_view* out);
/* every result row in one buffer (a caller's bulk copy instead of one
 * gk_results_get per row): per row, u32 review, u32 constraint, u32 msg_len,
 * u32 details_len, then the message and details bytes, unpadded.  *needed
 * receives the byte size; GK_EINVAL when cap is smaller (nothing written). */
int gk_results_export(const gk_results* r, void* buf, size_t cap, size_t* needed);
size_t gk_results_reviews(const gk_results* r);
uint32_t gk_results_review_status(const gk_results* r, size_t review);
uint32_t gk_results_review_reason(const gk_results* r, size_t review);
/* bulk copy of the per-review status / reason arrays (length gk_results_reviews) */
int gk_results_copy_status(const gk_results* r, uint32_t* status, uint32_t* reason);
/* number of reviews flagged GK_REVIEW_ERROR / GK_REVIEW_FALLBACK */
int gk_results_flag_counts(const gk_results* r, uint64_t* errors, uint64_t* fallbacks);
/* reviews the process excluder skipped */
uint64_t gk_results_excluded(const gk_results* r);
/* per-constraint violation totals (device-side counters), length = constraints */
size_t gk_results_constraints(const gk_results* r);
uint64_t gk_results_constraint_total(const gk_results* r, size_t constraint);
/* the engine state the results were evaluated in: bumps on every mutation
 * (module / data / excluder change), so concurrent callers can tell which
 * state of the constraints and templates each evaluation saw */
uint64_t gk_results_generation(const gk_results* r);
/* timings of the call in milliseconds: [flatten, upload, kernel, download, decode] */
int gk_results_timing(const gk_results* r, double* ms5);
/* violation tuples (32 B each) and message/details bytes the kernel wrote */
int gk_results_device_counts(const gk_results* r, uint64_t* tuples, uint64_t* bytes);
/* The device-resident output of the call: dev_tuples gk_viol records and
 * dev_bytes message/details bytes (unordered: one reservation per wavefront).
 * Copied device-to-device into caller buffers on the engine's device (e.g.
 * tensors handed to an RCCL gather).  Valid until the evaluation context that
 * produced the results runs another evaluation (for a single caller: the
 * engine's next evaluation) or the engine state changes; GK_EINVAL after that. */
typedef struct {
  uint32_t review, constraint;
  uint16_t seq, rule;    /* emission order key within (review, constraint): rows sort by it into the
                            reference's evaluation order (consecutive for templates without fused
                            rule bodies); rule 0xffff = autoreject */
  uint32_t msg_len;
  uint64_t msg_off;      /* message at [msg_off, +msg_len), details JSON right after it */
  uint32_t det_len, pad;
} gk_viol;
/* tuples_dst receives only the tuples of reviews the engine answered (not
 * those of reviews flagged GK_REVIEW_ERROR / GK_REVIEW_FALLBACK, nor rows of a
 * constraint with an invalid enforcementAction): *n_tuples of them, in no
 * particular order; size it for dev_tuples. */
int gk_results_copy_device_output(gk_engine* e, const gk_results* r, void* tuples_dst, void* bytes_dst,
                                  uint64_t* n_tuples);
/* kernels of the call in launch order: kernel name ("audit_kernel" = bytecode
 * VM, "gk_t_<hash>" = a template kernel), duration (HIP events), how many
 * constraints it evaluated and the violation tuples / message bytes it wrote */
size_t gk_results_launches(const gk_results* r);
int gk_results_launch(const gk_results* r, size_t i, const char** kernel, double* ms, uint32_t* nconstraints,
                      uint64_t* tuples, uint64_t* bytes);
void gk_results_free(gk_results* r);

/* ---- introspection --------------------------------------------------------- */
/* template status: 1 = compiled to GPU bytecode, 0 = CPU fallback, -1 unknown kind */
int gk_template_status(gk_engine* e, const char* kind, const char** reason);
/* evaluation back end of a template: 2 = template kernel (hipRTC-compiled for
 * gfx950; detail = kernel name), 1 = bytecode VM kernel (detail = why not
 * compiled), 3 = outside the subset, guard program on the GPU: the match and
 * every rule-body prefix before the first unsupported expression run on the
 * device, and only (review, constraint) pairs that reach that expression are
 * flagged GK_REVIEW_FALLBACK (detail = reason), 0 = CPU fallback for every
 * matched review (detail = reason).  Compiles on demand. */
int gk_template_backend(gk_engine* e, const char* kind, int* backend, const char** detail);
/* Prepares the engine's current state for evaluation now instead of at the
 * next staging / evaluation: rules and constraints compiled, match tables and
 * constants uploaded, template kernels compiled (hipRTC or the code-object
 * cache) and loaded, join indexes built.  The reference compiles a template's
 * Rego when it is added (client.go AddTemplate), not inside the audit sweep;
 * an audit loop calls this after syncing templates and constraints.
 * device = 0: host state only.  0 = success. */
int gk_engine_prepare(gk_engine* e, int device);
/* inventory join sites of a template (compiler.cc join_site): iterations of
 * data.inventory whose body filters on `A == key(leaf)` run as probes of a
 * per-constraint hash index built on the device (the reference scans:
 * k8suniqueserviceselector_template.yaml:40-44, k8suniquelabel_template.yaml:49-52).
 * Returns the number of sites (sites = their paths, ';'-separated) or < 0. */
int gk_template_joins(gk_engine* e, const char* kind, const char** sites);
/* the indexes of the last prepared state: (constraint, site) indexes built,
 * their entries, sites left to the scan (a key pass that failed), leaves keyed,
 * and the build time (key passes + sort + upload).  Prepares the device state. */
int gk_join_stats(gk_engine* e, uint64_t* indexes, uint64_t* entries, uint64_t* unindexed, uint64_t* leaves,
                  double* build_ms);
size_t gk_constraint_count(gk_engine* e);
int gk_constraint_info(gk_engine* e, size_t i, const char** kind, const char** name);

#ifdef __cplusplus
}
#endif
#endif /* GKGPU_H */
