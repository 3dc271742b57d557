/*
 * das_mi355x.h — C ABI of the MI355X-native DAS query hot path.
 *
 * This library replaces, behind the reference's own Python API, the storage
 * and evaluation layers of tanksha/das (reference snapshot 2025-02-09):
 *   - the Redis pattern/template index + Mongo link/node collections that
 *     `RedisMongoDB` reads          (das/database/redis_mongo_db.py:204-279)
 *   - their construction            (das/canonical_parser.py:132-183,
 *                                    das/parser_threads.py:141-253)
 *   - the ExpressionHasher handles  (das/expression_hasher.py:9-35)
 *   - the binding algebra of the pattern matcher for ordered assignments
 *                                   (das/pattern_matcher/pattern_matcher.py:73-156,
 *                                    :466-538, :591-614, :705-748)
 * The Python host package `das_amd` binds it with ctypes.
 *
 * Conventions: every entry point returns int (0 = DAS_OK, < 0 = error; the
 * message is in das_last_error(ctx)); no C++ exception crosses the ABI;
 * plain pointers and sizes only.  Device buffers are owned by the context
 * (index) or by a table handle (results) until das_table_free.  A digest is
 * the 16 raw MD5 bytes as 4 little-endian uint32 words (the reference handle
 * is its 32-char lowercase hex).  Atom ids are dense uint32 in handle order.
 */
#ifndef DAS_MI355X_H
#define DAS_MI355X_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct das_ctx das_ctx_t;
typedef struct das_table das_table_t;

#define DAS_OK 0
#define DAS_ERR_INVALID (-1)
#define DAS_ERR_HIP (-2)
#define DAS_ERR_NOT_BUILT (-3)
#define DAS_ERR_UNSUPPORTED (-4)
#define DAS_ERR_INTERNAL (-5)
#define DAS_ERR_ATTRIBUTE (-6)  /* where the reference raises AttributeError (:359-360) */
#define DAS_ERR_SYNTAX (-7)     /* malformed input where the reference asserts (canonical_parser.py:307-310) */

#define DAS_NONE 0xFFFFFFFFu   /* "no atom / wildcard" id */

#define DAS_TABLE_ORDERED 0    /* column c binds vars[c] (OrderedAssignment.mapping) */
#define DAS_TABLE_UNORDERED 1  /* vars = variable set, columns = sorted value set
                                  (UnorderedAssignment.symbols / .values)           */
#define DAS_TABLE_COMPOSITE 2  /* CompositeAssignment: ordered columns first (member -1,
                                  sorted vars), then each unordered member in join
                                  order (member m: sorted vars, sorted values)      */

/* ---- context ------------------------------------------------------------ */
/* stream: a hipStream_t (e.g. torch.cuda.current_stream().cuda_stream) or NULL
 * for a private blocking stream (ordered against the legacy null stream). */
int das_ctx_create(int device, void* stream, das_ctx_t** out);
int das_ctx_destroy(das_ctx_t* ctx);
const char* das_last_error(const das_ctx_t* ctx);
int das_ctx_sync(das_ctx_t* ctx);
/* Process-wide counters since load: out[0] = kernel launches (instrumented
 * scopes), out[1] = host read-backs waited on (per-query latency accounting). */
int das_counters(uint64_t out[2]);
int das_version(void);

/* ---- ExpressionHasher (expression_hasher.py:9-35) ------------------------ */
/* Host-side md5 of one UTF-8 string -> digest (query planning). */
int das_md5(const uint8_t* bytes, uint64_t n, uint32_t out_digest[4]);
/* Host-side composite_hash: md5(" ".join(hex(d_0), ..., hex(d_{k-1}))), k>=2;
 * k==1 returns d_0 (composite_hash([x]) == x). */
int das_composite_digest(const uint32_t* digests, uint32_t k, uint32_t out_digest[4]);
/* Device bulk: n strings (device bytes + n+1 offsets) -> n device digests. */
int das_hash_strings_dev(das_ctx_t* ctx, const uint8_t* d_bytes, const uint64_t* d_off,
                         uint64_t n, uint32_t* d_out);
/* Device bulk: n messages, message i = composite of elems[i*k .. i*k+k) (device
 * digests) -> n device digests.  This is the one-link-per-lane kernel the index
 * build uses, exposed for the bulk-hash benchmark. */
int das_hash_fixed_dev(das_ctx_t* ctx, const uint32_t* d_elems, uint32_t k, uint64_t n,
                       uint32_t* d_out);

/* ---- knowledge-base load + index build ----------------------------------- */
/* Parsed atoms, host arrays (das_amd.loader.AtomArrays).  "Leaves" are strings
 * hashed as md5(string): type names (md5(name), named_type_hash) and terminals
 * ("Type name", terminal_hash).  "Expressions" are composite_hash of their
 * children (child 0 = the type leaf), listed level by level (children first).
 * Indices are unified: < n_leaf is a leaf, otherwise n_leaf + expression. */
typedef struct {
  uint64_t n_leaf;
  const uint8_t* leaf_bytes;
  const uint64_t* leaf_off;        /* n_leaf + 1 */
  const uint8_t* leaf_kind;        /* 0 type name, 1 node (terminal in `nodes`), 2 other terminal */
  const uint32_t* leaf_ctype;      /* leaf whose digest is this leaf's composite type */
  const uint32_t* leaf_type_id;    /* named-type id of a type leaf, DAS_NONE otherwise */
  uint64_t n_expr;
  const uint64_t* expr_off;        /* n_expr + 1 */
  const uint32_t* expr_child;
  const uint8_t* expr_kind;        /* 1 link (`links_*` collections), 2 typedef (`atom_types`),
                                      3 link whose index rows live on another shard (multi-GPU:
                                      it gets its global id and outgoing set, no pattern rows) */
  const int32_t* expr_ctype_leaf;  /* -1: composite type from children; else that leaf's digest */
  uint32_t n_levels;
  const uint64_t* level_off;       /* n_levels + 1, expression ranges per nesting level */
  uint32_t n_types;
} das_atoms_t;

/* ---- Redis key-space export ---------------------------------------------- */
/* Writes outgoing_set.txt, incomming_set.txt, patterns.txt, templates.txt and
 * names.txt into `dir`: the key-value files CanonicalParser builds before it
 * populates Redis (canonical_parser.py:119-183, key_value_file.py:8-16), lines
 * sorted bytewise.  counts (optional) = lines per file in that order. */
int das_export_keyspace(das_ctx_t* ctx, const char* dir, uint64_t counts[5]);

/* ---- canonical MeTTa reader (host, multi-threaded) ----------------------- */
/* Parses n_texts canonical files -- `(: Name Type)` typedefs, `(: "name" Type)`
 * terminals, then one `(Type "T name" (Type ...) ...)` expression per line --
 * into the das_atoms_t layout (CanonicalParser.parse / _parse_expression,
 * canonical_parser.py:242-365).  n_threads 0 = up to 16.  Syntax errors return
 * DAS_ERR_SYNTAX with "line N: ..." in das_last_error(NULL). */
typedef struct das_parsed das_parsed_t;
int das_parse_canonical(const char* const* texts, const uint64_t* lens, uint32_t n_texts, uint32_t n_threads,
                        das_parsed_t** out);
/* Views into the parsed arrays (valid until das_parsed_free); name_start[i] is
 * the byte offset of a terminal's name inside its "Type name" leaf string. */
int das_parsed_atoms(const das_parsed_t* p, das_atoms_t* atoms, const uint32_t** name_start);
int das_parsed_type_name(const das_parsed_t* p, uint32_t type_id, const char** name, uint64_t* len);
int das_parsed_free(das_parsed_t* p);

/* The reference's `pattern_black_list` (distributed_atom_space.py:38, 346,
 * 409): named types (md5 of each type name, 4 words per type) whose links the
 * NEXT index build gives no pattern keys -- typed and '*' Link queries with a
 * wildcard (RedisMongoDB.get_matched_links :235-252) never return them --
 * while their template keys, outgoing / incoming sets and existence stay
 * (canonical_parser.py:144, 179-180; parser_threads.py:185).  (The reference
 * also writes each black-listed link under the previous link's keys, a bug
 * that depends on its load order; that is not reproduced: DESIGN.md §2.)
 * n = 0 clears the list. */
int das_set_pattern_black_list(das_ctx_t* ctx, const uint32_t* type_digests, uint32_t n);

typedef struct {
  uint64_t n_atoms, n_nodes, n_links, n_types, n_ctypes;
  uint64_t device_bytes;
  uint64_t links_by_arity[9];
} das_index_stats_t;

/* Loads + hashes every atom on the GPU and builds the HBM index (replaces the
 * Mongo insert + key-value files + sort + Redis SADD of canonical_parser.py:
 * 111-240).  Rebuilds from scratch if called again. */
int das_build_index(das_ctx_t* ctx, const das_atoms_t* atoms);
/* Same build from a KB whose expressions are already resident in HBM: with
 * DAS_BUILD_EXPR_ON_DEVICE, expr_off / expr_child / expr_kind / expr_ctype_leaf
 * are device pointers on ctx's device (read, not copied, not freed); the leaf
 * arrays and level_off stay host arrays.  flags 0 = das_build_index. */
#define DAS_BUILD_EXPR_ON_DEVICE 1u
int das_build_index_ex(das_ctx_t* ctx, const das_atoms_t* atoms, uint32_t flags);
int das_index_stats(das_ctx_t* ctx, das_index_stats_t* out);

/* ---- links hash-partitioned by handle across GPUs --------- */
/* The owning shard of a handle: int(handle[:8], 16) % world (its first four
 * digest bytes, big-endian).  The build for shard `rank` of `world`
 * indexes a link (expr kind 1 or 3) iff its handle's owner is `rank`; every
 * other link keeps its global id and outgoing set (directory only, like kind
 * 3).  Every copy of one expression has one handle, so each distinct link is
 * indexed on exactly one shard (canonical_parser.py:132-183 writes one entry
 * per handle).  world 1 = das_build_index_ex. */
int das_build_index_sharded(das_ctx_t* ctx, const das_atoms_t* atoms, uint32_t flags, uint32_t rank,
                            uint32_t world);
/* Owner shard of every expression's handle (hashes the KB as the build does):
 * d_owner = n_expr device bytes.  With das_partition_rows and an all-to-all of
 * the rows, a KB generated in ranges is regrouped on the owners of its
 * handles before the per-shard build (bench.py --workload build at N GPUs). */
int das_hash_owners(das_ctx_t* ctx, const das_atoms_t* atoms, uint32_t flags, uint32_t world, uint8_t* d_owner);
/* n device rows of K u32 regrouped by d_owner (stable inside an owner) into
 * d_out; counts[world] = rows per owner (host).  world <= 64. */
int das_partition_rows(das_ctx_t* ctx, const uint32_t* d_rows, uint64_t n, uint32_t K, const uint8_t* d_owner,
                       uint32_t world, uint32_t* d_out, uint64_t* counts);

/* ---- synthetic input (bench / tests) ---------- */
/* Writes n links of K-1 targets (K = 3 or 4 u32 per row: type leaf, then node
 * leaves) into device memory d_child, for global link indices first ..
 * first+n-1: type leaf = type_leaf0 + h % n_link_types, targets = node_leaf0 +
 * Zipf(s) rank over n_nodes, every field a counter-based hash of (seed, index),
 * so any split of the index range reproduces the same KB. */
int das_synth_powerlaw_links(das_ctx_t* ctx, uint32_t* d_child, uint64_t first, uint64_t n, uint32_t K,
                             uint32_t n_link_types, uint32_t type_leaf0, uint32_t node_leaf0, uint64_t n_nodes,
                             double s, uint64_t seed);

/* Host: the n strings prefix + decimal(first + i) back to back into `out`, and
 * n + 1 byte offsets (the configs 4-5 node leaves "Concept n<i>"). */
int das_numbered_strings(const char* prefix, uint64_t plen, uint64_t first, uint64_t n, uint8_t* out,
                         uint64_t* off);

/* digests -> atom ids (-1 if absent); cat: 0 other, 1 node, 2 link. */
int das_lookup(das_ctx_t* ctx, const uint32_t* digests, uint64_t n, int64_t* ids,
               uint8_t* cat, uint32_t* arity, uint32_t* type);
/* ids -> digests / category / arity / named type id / loader leaf of nodes */
int das_atoms_info(das_ctx_t* ctx, const uint32_t* ids, uint64_t n, uint32_t* digests,
                   uint8_t* cat, uint32_t* arity, uint32_t* type, uint32_t* name_leaf);
/* outgoing set of a link: targets in stored order (get_link_targets) */
int das_link_targets(das_ctx_t* ctx, uint32_t id, uint32_t* out, uint32_t cap, uint32_t* n);
/* The whole outgoing CSR to the host (a prefetch for per-link metadata calls,
 * replacing redis_mongo_db.py:222-227's per-call `outgoing_set:<handle>`
 * SMEMBERS): *n_off = n_atoms + 1 offsets, *n_tgt targets.  With null
 * buffers only the sizes are returned; else `off` / `tgt` must hold them. */
int das_export_outgoing(das_ctx_t* ctx, uint64_t* off, uint32_t* tgt, uint64_t* n_off, uint64_t* n_tgt);
/* incoming set of an atom: the links whose outgoing set contains it, ascending
 * link id (`incomming_set:<handle>`, canonical_parser.py:141-143).  *n = the set
 * size; min(*n, cap) ids are copied to `out`. */
int das_incoming(das_ctx_t* ctx, uint32_t id, uint32_t* out, uint64_t cap, uint64_t* n);
/* composite-type digest -> ctype id, or -1 (templates:<composite_type_hash>) */
int das_ctype_lookup(das_ctx_t* ctx, const uint32_t digest[4], int64_t* ctype_id);

/* ---- query operators ----------------------------------------------------- */
/* One Link with >= 1 wildcard, evaluated against the pattern index
 * (RedisMongoDB.get_matched_links :235-252 + Link._assign_variables :466-489).
 * `target[i]`: atom id or DAS_NONE for '*', in the position order the
 * reference builds its pattern key (sorted for Similarity/Set).  type_id
 * DAS_NONE means the '*' link type.
 * ordered: var[i] is the variable id bound at position i (-1 = grounded).
 * unordered: the variable set is var[0..n_vars) and values are the targets at
 * wildcard positions (sorted, must be distinct).
 * emit_link: prepend the link id column (var id -1) for get_matched_links. */
typedef struct {
  uint32_t arity;
  uint32_t type_id;
  uint32_t target[8];
  int32_t var[8];
  uint32_t n_vars;
  uint32_t ordered;
  uint32_t no_overload;
  uint32_t emit_link;
  int32_t order_pos;   /* >= 0: a typed all-wildcard scan returns its rows sorted by the
                          target at this position (the planner's join variable); -1 none */
} das_link_scan_t;

/* LinkTemplate (get_matched_type_template :269-275 + LinkTemplate._assign_variables
 * :591-601): all links of composite type `ctype_id`, var[i] bound at position i. */
typedef struct {
  uint32_t ctype_id;
  uint32_t arity;
  int32_t var[8];
  uint32_t ordered;
  uint32_t no_overload;
  uint32_t emit_link;
} das_template_scan_t;

int das_scan_link(das_ctx_t* ctx, const das_link_scan_t* q, das_table_t** out);
int das_scan_template(das_ctx_t* ctx, const das_template_scan_t* q, das_table_t** out);
/* All links of a named type, any arity (get_matched_type :277-279), as
 * (link id) tables per arity: out[a] for a in 0..8 (NULL where empty). */
int das_scan_type(das_ctx_t* ctx, uint32_t type_id, das_table_t** out9);

/* And's join step: ordered natural join (OrderedAssignment.join/_join_ordered
 * :105-139); with an unordered/composite operand the CompositeAssignment
 * algebra (:203-209, :316-351) -> DAS_TABLE_COMPOSITE. */
int das_join(das_ctx_t* ctx, const das_table_t* a, const das_table_t* b, uint32_t no_overload,
             das_table_t** out);
/* And's join of `a` with one Link term, evaluated through the pattern index
 * instead of a scan of the term: equal to das_join(a, das_scan_link(q)) when
 * it applies -- `a` ordered, q ordered and typed, arity <= 3, exactly one
 * target variable bound by `a`, every other target a fresh distinct variable,
 * no link column.  Each row of `a` looks its key up in P_{arity,p} and
 * expands that row range.  *out = NULL (status 0) when it does not apply. */
int das_index_join(das_ctx_t* ctx, const das_table_t* a, const das_link_scan_t* q, das_table_t** out);
/* Rows of `a` that pass check_negation against every row of `t` (:112-117,
 * :211-217, :353-362; And.matched :741-746). */
int das_antijoin(das_ctx_t* ctx, const das_table_t* a, const das_table_t* t, das_table_t** out);
/* Set semantics (Python set of assignments): unique rows. */
int das_dedup(das_ctx_t* ctx, const das_table_t* a, das_table_t** out);
/* Concatenate same-schema tables. */
int das_concat(das_ctx_t* ctx, const das_table_t* const* ts, uint32_t n, das_table_t** out);
/* Python-set identity across tables of any kinds and schemas (Assignment.__eq__
 * is hash equality, pattern_matcher.py:41-47; Composite hash = ordered.hash (or
 * 1) XOR member hashes, :279-286): keeps the first occurrence of every identity
 * in input order (table order, then row order); out[i] = rows kept of ts[i]. */
int das_set_dedup(das_ctx_t* ctx, const das_table_t* const* ts, uint32_t n, das_table_t** out);
/* out[i] = rows of a[i] whose identity occurs in no table of b (Or's
 * `term_answer.assignments - or_answer.assignments`, pattern_matcher.py:679). */
int das_set_minus(das_ctx_t* ctx, const das_table_t* const* a, uint32_t na, const das_table_t* const* b,
                  uint32_t nb, das_table_t** out);

int das_table_info(const das_table_t* t, int32_t* kind, int32_t* ncols, int32_t* vars,
                   uint64_t* nrows);
/* Copies rows [row0, row0+nrows) column-major into host `out` (ncols*nrows). */
int das_table_fetch(das_ctx_t* ctx, const das_table_t* t, uint64_t row0, uint64_t nrows,
                    uint32_t* out);
/* Device pointer of column c (valid until das_table_free). */
int das_table_column(const das_table_t* t, int32_t c, uint32_t** dptr);
/* Declares inclusive value bounds per column (NULL = unknown).  Joins size their
 * direct-address buckets from the build key's bound; every value must lie inside
 * it (values outside are dropped by the build).  Scan and join results carry
 * bounds derived from the index, so callers only set them on imported tables. */
int das_table_set_bounds(das_table_t* t, const uint32_t* lo, const uint32_t* hi);
/* Order-independent checksum of an ORDERED table under the reference's set
 * identity (pattern_matcher.py:41-51, 741-748), for parity checks at sizes no
 * host copy of the rows fits: out[0] = sum over rows of prod over columns c of
 * (splitmix64(d64(value) ^ salt[c]) | 1) mod 2^64, d64 = the value's first 8
 * digest bytes little-endian, salt[c] = the caller's key of column c's
 * variable name; out[1] = values that are not atom ids (0 for a valid table). */
int das_table_checksum(das_ctx_t* ctx, const das_table_t* t, const uint64_t* salt, uint64_t out[2]);
/* The declared / derived inclusive bounds per column ([0, DAS_NONE] = unknown). */
int das_table_get_bounds(const das_table_t* t, uint32_t* lo, uint32_t* hi);
/* Member id per column: -1 ordered, m = unordered member m (DAS_TABLE_COMPOSITE;
 * an UNORDERED table is member 0 throughout). */
int das_table_members(const das_table_t* t, int32_t* member);
/* New table from host columns (column-major ncols x nrows); member may be NULL
 * unless kind == DAS_TABLE_COMPOSITE. */
int das_table_from_host(das_ctx_t* ctx, int32_t kind, int32_t ncols, const int32_t* vars,
                        const int32_t* member, const uint32_t* cols, uint64_t nrows, das_table_t** out);
int das_table_free(das_table_t* t);

/* ---- whole-expression plans --------------------------------------------- */
/* An And / Or / Not tree of ordered Links, evaluated in one call with the
 * folding rules of the pattern matcher (And.matched pattern_matcher.py:705-748,
 * Or.matched :644-687, Not.matched :627-631) instead of one host call per
 * operator.  Nodes are in prefix order: an AND / OR node is followed by its
 * `nchild` subtrees, a NOT node by one.  Leaves: LINK = Link.matched's
 * wildcard branch (`scan` as das_scan_link, ordered; `dedup` when the
 * reference's set would merge rows: a '*' type, a repeated variable, the
 * sorted key of an ordered Similarity/Set query); CONST = a term the host
 * settled (node_exists / link_exists): matched = `value`, no assignments.
 * `index_join` (LINK) allows And to evaluate the term as das_index_join(`ij`)
 * against its running result, as the host path does.
 * The answer's tables (one per schema, rows distinct) go to out[0..*n_out);
 * DAS_ERR_INVALID if more than `cap`, with *n_out set to the number needed (call
 * again with that capacity). */
#define DAS_PLAN_LINK 1
#define DAS_PLAN_CONST 2
#define DAS_PLAN_NOT 3
#define DAS_PLAN_AND 4
#define DAS_PLAN_OR 5
/* TEMPLATE leaf: LinkTemplate.matched (:603-614), the scan_template of
 * composite type `scan.type_id` (arity, var, ordered, no_overload as in
 * das_template_scan_t); `dedup` when a variable repeats.
 * TVM node: a Link with LinkTemplate targets (Link._typed_variable_matched
 * :491-500), followed by its `nchild` targets (CONST node checks, TEMPLATE,
 * LINK, nested TVM): matched iff every target matches, in order; its
 * assignments are the last template / link target's. */
#define DAS_PLAN_TEMPLATE 7
#define DAS_PLAN_TVM 8
typedef struct {
  int32_t op;
  uint32_t nchild;
  uint32_t value;
  uint32_t dedup;
  uint32_t index_join;
  das_link_scan_t scan;
  das_link_scan_t ij;
} das_plan_node_t;
int das_plan_execute(das_ctx_t* ctx, const das_plan_node_t* nodes, uint32_t n, uint32_t no_overload,
                     das_table_t** out, uint32_t cap, uint32_t* n_out, int32_t* matched, int32_t* negation);
/* das_plan_execute + each answer table's (kind, ncols, nrows, 0, vars[16])
 * in info[20 * i ..] (NULL: not written), as das_plan_execute_many reports
 * them: the caller needs no das_table_info call per table. */
int das_plan_execute_info(das_ctx_t* ctx, const das_plan_node_t* nodes, uint32_t n, uint32_t no_overload,
                          das_table_t** out, uint32_t cap, uint32_t* n_out, int32_t* matched, int32_t* negation,
                          int64_t* info);

/* n_plans independent plans in one call (no reference counterpart: a batch of
 * the reference's Expression.matched calls, pattern_matcher.py:705-748 /
 * :644-687, one per plan): plan i is nodes[i][0 .. n[i]), its answer tables
 * out[sum(n_out[0..i)) ..], n_out[i] of them, matched[i] / negation[i] as
 * das_plan_execute's.  Every answer equals das_plan_execute's on that plan
 * alone; Ands one fused chain answers are launched before any other plan
 * runs and read back last, so the host work of the batch overlaps their GPU
 * time.  More than `cap` tables in all: DAS_ERR_INVALID with n_out set and
 * no table returned.  info (optional, 20 int64 per table): kind, ncols,
 * nrows, 0, vars[16] -- das_table_info's fields without a call per table. */
int das_plan_execute_many(das_ctx_t* ctx, uint32_t n_plans, const das_plan_node_t* const* nodes, const uint32_t* n,
                          uint32_t no_overload, das_table_t** out, uint32_t cap, uint32_t* n_out, int32_t* matched,
                          int32_t* negation, int64_t* info);

/* ---- sharded plans (links hash-partitioned by handle across GPUs) ---------- */
/* One GPU's part of a plan over a KB sharded across GPUs (das_amd.parallel
 * ShardedDB): an INPUT leaf (`value` = index into `inputs`, `scan` = the term
 * it stands for) is a relation every shard holds whole -- e.g. a term's rows
 * gathered from all shards -- and is read in place; a LINK leaf scans or
 * index-joins this shard's index, giving this shard's part of the term.  The
 * And fold assumes that such partial relations are non-empty where it tests
 * them; checks[j] = 1 if the running result of the top-level And holds rows
 * on this shard after its j-th positive term.  The caller verifies the
 * assumption (for every j after the first LINK leaf, some shard has rows) and
 * otherwise evaluates the expression another way.  No fused chain, no anti
 * index join (a negated link's owner may be another shard), no fused Or. */
#define DAS_PLAN_INPUT 6
int das_plan_execute_sharded(das_ctx_t* ctx, const das_plan_node_t* nodes, uint32_t n, uint32_t no_overload,
                             const das_table_t* const* inputs, uint32_t n_inputs, das_table_t** out, uint32_t cap,
                             uint32_t* n_out, int32_t* matched, int32_t* negation, uint8_t* checks,
                             uint32_t checks_cap, uint32_t* n_checks);
/* rows[i] = the index rows node i's scan would read (LINK / INPUT nodes; an
 * upper bound of its output on this shard), 0 for other nodes. */
int das_plan_estimates(das_ctx_t* ctx, const das_plan_node_t* nodes, uint32_t n, uint64_t* rows);
/* Per LINK / TEMPLATE node, an upper bound of das_plan_estimates over every
 * value of its grounded targets (its query shape): the largest pattern-key
 * range of its type at a grounded position; UINT64_MAX when unknown.  A
 * sharded plan caches these per shape, so a fresh anchor of a known shape
 * needs no estimate exchange. */
int das_plan_bounds(das_ctx_t* ctx, const das_plan_node_t* nodes, uint32_t n, uint64_t* rows);

/* ---- multi-GPU exchange (RCCL all-to-all of binding rows) ----- */
/* Rows of `t` regrouped by destination = mix(key columns) % nparts (stable
 * inside a destination); counts[nparts] receives the group sizes.  nkey == 0
 * keys on every column (global dedup / set difference). */
int das_partition(das_ctx_t* ctx, const das_table_t* t, const int32_t* key_vars, uint32_t nkey,
                  uint32_t nparts, das_table_t** out, uint64_t* counts);
/* Rows idx[0..n) of `t` (host indices) as a new table, same schema: the
 * heavy / light split of a skewed join's buckets. */
int das_table_gather(das_ctx_t* ctx, const das_table_t* t, const uint32_t* idx, uint64_t n, das_table_t** out);
/* Rows [begin[i], end[i]) of `t` for every range i, in range order (host range
 * arrays; the rows never pass through the host): the heavy / light buckets of
 * a partitioned table (das_partition groups rows by bucket). */
int das_table_gather_ranges(das_ctx_t* ctx, const das_table_t* t, const uint64_t* begin, const uint64_t* end,
                            uint32_t n_ranges, das_table_t** out);
/* Row-major (n x ncols u32) device copies for the collective buffers. */
int das_table_export_rows(das_ctx_t* ctx, const das_table_t* t, uint32_t* d_dst);
int das_table_import_rows(das_ctx_t* ctx, int32_t kind, int32_t ncols, const int32_t* vars,
                          const int32_t* member, const uint32_t* d_src, uint64_t nrows,
                          das_table_t** out);

/* ---- measurement ---------------------------------------------------------- */
/* Per-kernel HIP-event timing on the context stream (bench.py roofline):
 * totals of elapsed ms, launches and algorithmic bytes since the last reset. */
int das_prof_enable(das_ctx_t* ctx, int on);
/* Restrict event recording to the scopes named `name` (NULL or "" = every
 * scope): the bench times its dominant kernel live without paying two event
 * records per launch for every other kernel. */
int das_prof_only(das_ctx_t* ctx, const char* name);   /* name: one scope or a '|'-separated list */
/* Scopes recorded while a tag is set are named "<scope>@<tag>" (NULL or "" =
 * none): one query's launches of a kernel other queries launch too are timed
 * apart inside a step (bench.py's in-step And-join fraction). */
int das_prof_tag(das_ctx_t* ctx, const char* tag);
/* The tag applied only while plan `plan` of each following
 * das_plan_execute_many batch runs (its own launches, not those of other
 * plans launched inside its read-back waits); plan = UINT32_MAX or tag NULL
 * clears it: one query tagged inside a batched step. */
int das_prof_tag_plan(das_ctx_t* ctx, uint32_t plan, const char* tag);
int das_prof_reset(das_ctx_t* ctx);
/* The card's 16-byte nontemporal store ceiling: `bytes` written as six
 * columns of dwordx4 stores (k_cartesian's pattern), `reps` timed launches
 * after one warm one; GB/s out.  bench.py records it beside every run. */
int das_box_store_bw(das_ctx_t* ctx, uint64_t bytes, uint32_t reps, double* gbps);
/* One tiny kernel (k_prof_mark) on the context stream: brackets a region in a
 * rocprofv3 kernel trace (tools/step_split.py). */
int das_prof_mark(das_ctx_t* ctx, uint32_t id);
int das_prof_read(das_ctx_t* ctx, const char* name, double* ms, uint64_t* launches, double* bytes);
int das_prof_names(das_ctx_t* ctx, char* buf, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* DAS_MI355X_H */
