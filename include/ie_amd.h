/*
 * ie_amd.h — C ABI of the MI355X-native `{key}` interpolation resolver (libie_amd.so).
 *
 * This is the drop-in boundary for the reference's hot path:
 *
 *   Python  src/interpolation_engine/interpolation_engine.py
 *     interpolate_inserts(inserts, content)        py:497-541   -> ie_interpolate / ie_interpolate_batch
 *     get_interpdata(inserts, key)                 py:430-467   -> ie_table_build (lookup order baked in)
 *     get_simple_insertkey(content)                py:477-495   -> ie_simple_insertkey
 *     recursive_unescape / recursive_escape        py:1436-1460 -> ie_unescape_batch / ie_escape_batch
 *     InterpolationException / AssertionError      py:426, 519, 530 -> ie_status codes
 *     is_wildcard_match / get_wildcard_matches     py:553-567   -> ie_wildcards_build + ie_wildcard_match_*
 *   Rust    rust-project/src/interp.rs
 *     interpolate_inserts(&Map, &str, &ctx)        interp.rs:31-89  -> ie_interpolate (dialect IE_DIALECT_RS)
 *     get_interpdata                               interp.rs:91-137 -> ie_table_build
 *     get_simple_insertkey                         interp.rs:11-29  -> ie_simple_insertkey
 *     recursive_unescape / recursive_escape        interp.rs:147-177 -> ie_unescape_batch / ie_escape_batch
 *   Rust    rust-project/src/runtime.rs
 *     wildcard match / captures                    runtime.rs:1633-1647, 1754-1775 -> ie_wildcard_match_*
 *
 * Plain pointers and sizes only; no torch or HIP types appear in a signature (streams are void*).
 * Every entry point returns 0 (IE_SUCCESS) or a negative IE_ERR_* code; ie_last_error() gives text.
 * Per-string outcomes are ie_status bytes, one per input string.
 */
#ifndef IE_AMD_H
#define IE_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: ie_timing gained n_deferred; ie_unescape_cmd_device may report IE_RECURSE; IE_OPT_LEAN (6) was
 *    removed and IE_OPT_RESERVE (8) added. */
#define IE_ABI_VERSION 2

/* ---- dialects: which reference implementation's rules to follow ---- */
enum ie_dialect {
  IE_DIALECT_PY = 0, /* interpolation_engine.py (the default parity target) */
  IE_DIALECT_RS = 1  /* rust-project/src/interp.rs (restated; parity unpinned) */
};

/* ---- value kinds (the JSON type of an insert value) ---- */
enum ie_kind {
  IE_KIND_STR = 0,
  IE_KIND_INT = 1,
  IE_KIND_LIST = 2,
  IE_KIND_FLOAT = 3,
  IE_KIND_BOOL = 4,
  IE_KIND_NULL = 5,
  IE_KIND_DICT = 6
};

/* ---- per-string status (one byte per input string) ---- */
enum ie_status {
  IE_OK_STR = 0,          /* result is the string in the output arena                      */
  IE_OK_VALUE = 1,        /* whole-string "{key}": result is the raw insert, see value_id   */
  IE_E_INTERP = 2,        /* InterpolationException: missing key, '' key, missing ARGn      */
  IE_E_ASSERT_BRACES = 3, /* AssertionError: uneven '{' / '}' count (py:517-519)           */
  IE_E_ASSERT_TYPE = 4,   /* AssertionError: splice of a non str/int/list (py:530);
                             Rust: "unsupported type" error (interp.rs:76-79)               */
  IE_E_UNHASHABLE = 5,    /* TypeError: a list/dict raw value used as a key (py:512, 450)   */
  IE_E_RS_PANIC = 6,      /* Rust dialect: unwrap() panic on a '}{' leftover (interp.rs:63-66) */
  IE_NEEDS_HOST = 7,      /* key missing and an --inserts-dir is configured (py:452-461)   */
  IE_DIVERGED = 8,        /* iteration cap hit: the reference would loop forever           */
  IE_E_OVERFLOW = 9,      /* string over its single-pass scratch budget (host APIs retry)  */
  IE_E_NO_MATCH = 11,     /* ie_goto_map: no key matches the text (py:1708's AssertionError)   */
  IE_E_NO_NULL = 12,      /* ie_goto_map: the text failed to interpolate and no key is 'NULL'
                             (py:1703's AssertionError)                                        */
  IE_RECURSE = 10         /* ie_unescape_cmd_device, py dialect: the unescaped item is a whole-string
                             '{key}' as written, so recursive_interpolate walks its result again
                             (py:1463-1464); the result (a str, list or dict; value_id = the insert
                             when the result was one) is not final: the caller resolves the item
                             with recursive_interpolate itself, as the mirror does                */
};

/* ---- API return codes ---- */
#define IE_SUCCESS 0
#define IE_ERR_INVALID (-1)
#define IE_ERR_HIP (-2)
#define IE_ERR_NOMEM (-3)
#define IE_ERR_NO_DEVICE (-4)
#define IE_ERR_TIMEOUT (-5)
#define IE_ERR_CAPACITY (-6) /* caller-owned output buffer too small (see *total), or a table full (rebuild) */

/* Divergence caps. The reference loops forever on self-referential inserts (py:516 has no bound)
 * or grows without limit; both the oracle and the device path stop a string once its working
 * copy has taken more than IE_ITER_CAP substitutions or grown beyond IE_SIZE_CAP bytes, and report
 * IE_DIVERGED. `len` is the input string's byte length, `maxtext` the longest splice text in the
 * table (so any result without re-resolution, at most len/2 refs of maxtext bytes, fits). */
#define IE_ITER_CAP(len) (4096ull + 8ull * (uint64_t)(len))
#define IE_SIZE_CAP(len, maxtext) \
  ((1ull << 20) + 64ull * (uint64_t)(len) + (uint64_t)(maxtext) * ((uint64_t)(len) / 2ull + 1ull))

/* value_id sentinels (value_id is otherwise the index into the ie_kv array given to ie_table_build) */
#define IE_VID_NONE 0xFFFFFFFFu
#define IE_VID_CLOCK_HHMM 0xFFFFFFFEu   /* get_interpdata 'HH:MM'    (py:433-434) */
#define IE_VID_CLOCK_HHMMSS 0xFFFFFFFDu /* get_interpdata 'HH:MM:SS' (py:435-436) */

/* One insert. `text` is the splice rendering the binding computed on the host:
 *   py: str(v)  (list -> Python repr, int -> decimal; py:531)
 *   rs: value_to_string(v)  (interp.rs:314-322)
 * For IE_KIND_STR `text` is the string itself. */
typedef struct ie_kv {
  const char* key;
  uint64_t key_len;
  const char* text;
  uint64_t text_len;
  int32_t kind;
  uint32_t reserved;
} ie_kv;

/* Injected wall clock for 'HH:MM' / 'HH:MM:SS' (one clock per table build). */
typedef struct ie_clock {
  int32_t hour, minute, second;
} ie_clock;

#define IE_TABLE_HAS_INSERTS_DIR 1u /* missing keys report IE_NEEDS_HOST instead of IE_E_INTERP */
#define IE_TABLE_MUTABLE 2u         /* room for ie_table_set_update's new keys (entries at load 0.5, not 0.8) */

/* A table is read-only on the device. It may be used by several execs / host threads at once, EXCEPT
 * while ie_table_set_update or ie_table_set_clock rewrites it: those two patch the device copy in
 * place (after waiting for the device), so the caller must not run a batch on the table from
 * another thread while they run (they are not synchronised with other threads' launches). */
typedef struct ie_table ie_table;
typedef struct ie_exec ie_exec;   /* one per host thread: device, stream, workspace           */

/* Device-resident output of a batch call. All pointers are DEVICE pointers owned by the caller.
 * bytes_cap is the capacity of `bytes`. The call writes the required byte count to *total
 * (a device word); when it exceeds bytes_cap the byte payload is not written and the caller
 * re-runs with a larger buffer (offsets/status stay valid). value_id[i] is written only
 * where status[i] == IE_OK_VALUE. */
typedef struct ie_dev_out {
  uint8_t* bytes;
  uint64_t bytes_cap;
  uint64_t* offsets;  /* n + 1 */
  uint8_t* status;    /* n     */
  uint32_t* value_id; /* n     */
  uint64_t* total;    /* 1     */
} ie_dev_out;

/* Host-resident result owned by the library (free with ie_batch_free). */
typedef struct ie_batch {
  uint8_t* bytes;
  uint64_t bytes_len;
  uint64_t* offsets; /* n + 1 */
  uint8_t* status;   /* n     */
  uint32_t* value_id;/* n     */
  uint64_t n;
} ie_batch;

/* Kernel timing of the last device call on an exec (HIP events on the exec's stream). */
typedef struct ie_timing {
  float resolve_ms;      /* the resolve (or escape) kernel(s) of the last call */
  float complex_ms;      /* reserved: literal strings are resolved inside the resolve kernel */
  float total_ms;        /* setup memsets + kernels of the last call */
  uint64_t n_complex;    /* strings routed to the literal (wave-cooperative) path */
  uint64_t n_direct;     /* tiles that bypassed the LDS stages (long strings / many segments) */
  uint64_t n_polls;      /* look-back poll rounds that found a predecessor not yet published */
  uint64_t n_exact;      /* strings the level evaluator handed to the exact event evaluator */
  uint64_t n_chain_fail; /* strings whose chain evaluation met a miss or an unspliceable hit */
  uint64_t n_deferred;   /* views batches: strings left to a second pass (the fused unescape
                            command: strings left to its deferred pass) */
} ie_timing;

/* ---- library ---- */
int32_t ie_abi_version(void);
const char* ie_build_id(void); /* hash of the sources the library was built from */
const char* ie_last_error(void);
int32_t ie_device_count(void);

/* ---- table: get_interpdata (py:430-467 / interp.rs:91-137) ---- */
int ie_table_build(const ie_kv* kv, uint64_t n, int32_t dialect, const ie_clock* now,
                   uint32_t flags, int32_t device, ie_table** out);
/* A table set: n_tables inserts dicts in one device table, table t = kv[kv_start[t] .. kv_start[t+1]).
 * Strings pick their dict with a table id (ie_interpolate_*_ids); value ids index kv as a whole.
 * This is SURVEY §8b's `tables[] + table_id[]` batch for config 5's forked states (one dict per
 * state, the per-task map clone of rust-project/src/runtime.rs:700-701 made unnecessary) and for
 * replace_map's `inserts | extra_inserts` (py:1734). ie_table_build is the one-dict case. */
int ie_table_set_build(const ie_kv* kv, const uint64_t* kv_start, uint32_t n_tables, int32_t dialect,
                       const ie_clock* now, uint32_t flags, int32_t device, ie_table** out);
void ie_table_free(ie_table* t);
/* Multi-GPU (the path shards, no data-path collective). ie_table_replicate copies a
 * built table to another device (device-to-device, over xGMI between GPUs); ie_shard_bounds
 * splits a packed batch into n_shards byte-balanced contiguous string ranges,
 * first[k] .. first[k+1] (first has n_shards + 1 entries; binary search on offsets). */
int ie_table_replicate(const ie_table* t, int32_t device, ie_table** out);
int ie_shard_bounds(const uint64_t* offsets, uint64_t n, uint32_t n_shards, uint64_t* first);
/* Re-read the clock (py:433-436) without a rebuild: rewrites the 'HH:MM' / 'HH:MM:SS' entries in
 * place (values that read the clock, also through nested keys, are never pre-resolved at build,
 * so every lookup sees the new time). Waits for the device first: no batch may be in flight. */
int ie_table_set_clock(ie_table* t, const ie_clock* now);
/* set_interpdata on a built table or table set (py:470-471 `inserts[key] = value`, the replace_map /
 * user_input / set stores of py:1566-1568, 1770-1773; rust-project/src/runtime.rs:700-701 snapshots
 * the map per task): entry i sets kv[i] (kind < 0: deletes the key) in table table_id[i], value id
 * vid[i], without a rebuild: a key the table has is rewritten in place, a new key re-places its
 * pilot group (or, when that group has no free placement, the whole table is placed again at the
 * same capacity: entries and pilots uploaded whole). Waits for the device first (like ie_table_set_clock);
 * the patch kernel it ends with completes asynchronously, ordered before every later batch on the
 * table (the batches wait on its event in their own stream). A brace-bearing
 * value is not pre-resolved, and the pre-resolved values of every changed table return to their raw
 * text (both then resolve through the exact evaluator, in the reference's order). IE_ERR_CAPACITY:
 * a new key found no placement (the entries before it were applied, it and the rest were not:
 * rebuild the table; a table built with IE_TABLE_MUTABLE keeps room for about as many new keys as it
 * was built with). Every change is validated before any is applied (IE_ERR_INVALID leaves the table
 * unchanged). Texts: a rewrite whose new text fits the old one's room is written in place, any other
 * text is appended to the table's arena; the replaced bytes are counted dead, and the arena is
 * compacted (host mirror + one upload) when the dead bytes outnumber the live ones. A change that
 * would take an arena offset past the table's limit (2^32 - 16, or ie_table_set_arena_limit's) even
 * after a compaction returns IE_ERR_CAPACITY (the changes before it applied): rebuild the table. */
int ie_table_set_update(ie_table* t, const ie_kv* kv, const uint32_t* table_id, const uint32_t* vid, uint64_t n);
/* ie_table_set_update with the value ids handed out by the table (the caller keeps no (table, key) ->
 * id map): a rewrite keeps its key's id, a new key takes an id a delete freed or the next unused one
 * (a table set's build gives kv i the id i), a delete frees its key's id. vid_out[i] = the id change
 * i stored under (for a delete: the id it freed), IE_VID_NONE for a change that stored nothing (an
 * absent key deleted, the keys '', 'HH:MM', 'HH:MM:SS', or a change after an IE_ERR_CAPACITY stop).
 * Ids exhausted (2^32 - 3): IE_ERR_CAPACITY. */
int ie_table_set_store(ie_table* t, const ie_kv* kv, const uint32_t* table_id, uint64_t n, uint32_t* vid_out);
/* The stored value behind a value id (any table of a set: a set's ids are unique): its kind
 * (IE_KIND_*) and text (ie_kv.text as stored; a pre-resolved value's raw text), read from the table's
 * host mirror; the pointer is valid until the next update of the table. The clock ids have none. */
int ie_table_value(const ie_table* t, uint32_t vid, int32_t* kind, const char** text, uint64_t* len);
/* Arena bookkeeping: bytes in use, bytes of live entries, compactions so far (any may be NULL). */
int ie_table_arena_stats(const ie_table* t, uint64_t* bytes, uint64_t* live, uint64_t* compactions);
/* Lower the arena limit of ie_table_set_update (tests: force compaction and IE_ERR_CAPACITY early). */
int ie_table_set_arena_limit(ie_table* t, uint64_t bytes);
uint64_t ie_table_entries(const ie_table* t);
uint32_t ie_table_tables(const ie_table* t);
int32_t ie_table_dialect(const ie_table* t);

/* ---- exec context ---- */
int ie_exec_create(int32_t device, void* hip_stream /* NULL: a new non-blocking stream */,
                   ie_exec** out);
void ie_exec_destroy(ie_exec* x);
int ie_exec_sync(ie_exec* x);
int ie_exec_set_timing(ie_exec* x, int32_t enabled);
int ie_exec_timing(ie_exec* x, ie_timing* out); /* syncs */
/* Exec options (defaults from the environment at ie_exec_create: IE_FAIL_COMMIT, IE_FAST,
 * IE_DEBUG_NOEVAL, IE_TILE, IE_VIEWS). IE_OPT_FAIL_COMMIT: -1 adaptive (default), 0 / 1 forces the k_resolve
 * variant (both give the reference's results; tests run under both). IE_OPT_TILE: 0 (default)
 * 512-string tiles for the unescape command's second resolve and 256 elsewhere; 256 / 512 force one
 * size (same results; a performance choice). */
#define IE_OPT_FAIL_COMMIT 1
#define IE_OPT_FAST 2
#define IE_OPT_DEBUG_NOEVAL 3
#define IE_OPT_TILE 4
#define IE_OPT_VIEWS 5 /* 1 (default): the host batch APIs resolve into a views layout (no look-back) and
                          pack the results in input order on the host; 0: packed on the device */
#define IE_OPT_DEFER 7 /* views batches in two passes: a first pass without the exact evaluator and
                          the literal path (leaner registers and schedule), then the strings it could
                          not finish in tiles of their own. 2 (default): batches of >= 2^19 strings,
                          and any batch after one with > 0.4 % such strings; 1: always; -1: only the
                          latter; 0: never (one pass, every string in its tile) */
#define IE_OPT_RESERVE 8 /* views output of a packed batch: 0 (default): each tile claims its range on one
                          cursor (the bytes packed without gaps, *total = sum of lengths); F in 16..1024:
                          tile t writes at F/16 x its input span's offset from the batch's first byte
                          when its output fits the span x F/16 (no atomic), else in an overflow region
                          after the whole reservation (a claim on the cursor): gaps between tiles,
                          *total = sum of lengths still; a tile that did not fit bytes_cap makes
                          ie_exec_sync report IE_ERR_CAPACITY. Size bytes_cap >= F/16 x the input bytes
                          plus the overflow's share. */
#define IE_OPT_ERROR_KEYS 9 /* 1: every IE_E_INTERP string of an interpolation call also leaves the
                          missing key its message names (py:467, "Could not find variable '<key>'")
                          in ie_exec_host_keys; such strings take the literal path (0, the default:
                          no keys, misses stay on the fast evaluators) */
#define IE_OPT_SMALL_ZC 10 /* host calls of one tile (<= 256 strings, views) and small wildcard batches
                          without copies: 1: inputs and outputs in one mapped, coherent pinned block the
                          kernels read and write; 2: the outputs only; 0 (default; env IE_SMALL_ZC):
                          one pinned block copy each way (the same latency) */
int ie_exec_set_option(ie_exec* x, int32_t option, int64_t value);
/* Literal-path scratch pool size. Setting it makes ie_interpolate_device fully asynchronous: it no
 * longer waits to check the pool's demand, and strings that ran out of it report IE_E_OVERFLOW.
 * Without it the device calls wait only for the demand, which the call's last kernel publishes to
 * host memory as it starts (not for the stream): read their results through the exec's stream
 * (ie_copy_d2h) or after ie_exec_sync, as with the asynchronous form. */
int ie_exec_set_scratch(ie_exec* x, uint64_t bytes);
/* Keys only the host can look up (get_interpdata's file fallback for a key that is not a canonical
 * relative file name under the inserts directory, py:452-461): for every string of the exec's last
 * interpolation call that reported IE_NEEDS_HOST (and, with IE_OPT_ERROR_KEYS, IE_E_INTERP), the key
 * its failing lookup used (also one built from looked-up values), as records {uint32 string index,
 * uint32 key length, key bytes padded to 4}. Copies min(cap, *used) bytes of records to buf; *used = the records' size. Synchronous. */
int ie_exec_host_keys(ie_exec* x, uint8_t* buf, uint64_t cap, uint64_t* used);

/* Diagnostic (no reference counterpart): one key through the device lookups next to the host's
 * view of the same table; out[12] as documented in ie_host.cpp. */
int ie_debug_probe(const ie_table* t, const char* key, uint64_t len, uint64_t* out);

/* ---- device memory and stream markers for callers without their own HIP bindings (the Rust
 * shim, ctypes). Copies are ordered on the exec's stream; *_sync variants wait for it. ---- */
int ie_dev_alloc(int32_t device, uint64_t bytes, void** out);
void ie_dev_free(void* p);
int ie_copy_h2d(ie_exec* x, void* dst, const void* src, uint64_t bytes);  /* synchronous */
int ie_copy_d2h(ie_exec* x, void* dst, const void* src, uint64_t bytes);  /* synchronous */
int ie_memset_d(ie_exec* x, void* dst, int32_t value, uint64_t bytes);     /* asynchronous */
/* HIP events recorded on the exec's stream: slot in [0, 1024). */
int ie_exec_mark(ie_exec* x, uint32_t slot);
int ie_exec_elapsed(ie_exec* x, uint32_t from_slot, uint32_t to_slot, float* ms); /* syncs */

/* ---- interpolate_inserts over a packed batch (py:497-541 / interp.rs:31-89) ----
 * Input: UTF-8 bytes, offsets[n+1] (string i = bytes[offsets[i] .. offsets[i+1])).
 * _device: all pointers device-resident, enqueued on the exec's stream; ie_interpolate_device
 *          then waits for the stream to read the literal path's scratch demand and, when the pool
 *          was too small, grows it and re-runs the batch once (no IE_E_OVERFLOW from capacity),
 *          unless ie_exec_set_scratch sized the pool.
 * _batch:  host pointers; H2D + kernels + D2H, synchronous, retries capacity/overflow. */
int ie_interpolate_device(ie_exec* x, const ie_table* t, const uint8_t* d_bytes,
                          const uint64_t* d_offsets, uint64_t n, const ie_dev_out* out);
int ie_interpolate_batch(ie_exec* x, const ie_table* t, const uint8_t* bytes,
                         const uint64_t* offsets, uint64_t n, ie_batch** out);
/* The same over a table set: string i resolves against table table_id[i] (_device: a device array;
 * an id beyond the set finds no key, so such strings report IE_E_INTERP; _batch checks the ids). */
int ie_interpolate_device_ids(ie_exec* x, const ie_table* t, const uint32_t* d_table_id, const uint8_t* d_bytes,
                              const uint64_t* d_offsets, uint64_t n, const ie_dev_out* out);
int ie_interpolate_batch_ids(ie_exec* x, const ie_table* t, const uint32_t* table_id, const uint8_t* bytes,
                             const uint64_t* offsets, uint64_t n, ie_batch** out);
/* Views layout (no global order). The reference returns one object per string (py:497-541,
 * interp.rs:31-89); the order in which results are stored is not part of that contract. A views
 * output holds string i's result at bytes[offsets[i] .. offsets[i] + lengths[i]) (offsets has n
 * entries, no offsets[n]); tiles of consecutive strings claim their byte ranges in completion
 * order with one atomic each, so the device never waits for an earlier tile (no look-back), and
 * the bytes of the whole batch are packed without gaps: *total = sum of lengths. A string that
 * failed has length 0. d_lengths (nullable) makes the INPUT a views layout too (string i =
 * d_bytes[d_offsets[i] .. + d_lengths[i]), e.g. an earlier views output); null means packed input
 * (d_offsets[n + 1]). When *total exceeds bytes_cap, the tiles that did not fit wrote no bytes:
 * re-run with a larger buffer (offsets, lengths and statuses are valid either way). */
typedef struct ie_dev_views {
  uint8_t* bytes;
  uint64_t bytes_cap;
  uint64_t* offsets;  /* n */
  uint32_t* lengths;  /* n */
  uint8_t* status;    /* n */
  uint32_t* value_id; /* n */
  uint64_t* total;    /* 1 */
} ie_dev_views;
int ie_interpolate_device_views(ie_exec* x, const ie_table* t, const uint32_t* d_table_id, const uint8_t* d_bytes,
                                const uint64_t* d_offsets, const uint32_t* d_lengths, uint64_t n,
                                const ie_dev_views* out);
/* scalar drop-in: one string (a batch of one on the device) */
int ie_interpolate(ie_exec* x, const ie_table* t, const char* s, uint64_t len, ie_batch** out);

/* ---- recursive_unescape / recursive_escape on strings (py:1436-1460 / interp.rs:147-177) ---- */
int ie_unescape_device(ie_exec* x, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n,
                       const ie_dev_out* out);
int ie_escape_device(ie_exec* x, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n,
                     const ie_dev_out* out);
int ie_unescape_batch(ie_exec* x, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                      ie_batch** out);
/* The `unescape` command's transform of its item (py:1660-1667 / rust-project/src/runtime.rs:
 * 1044-1050): recursive_unescape, then recursive_interpolate, on a batch of strings (table ids
 * nullable). tmp receives the unescaped strings (caller-sized; IE_ERR_CAPACITY when too small).
 * d_status_in (nullable): the statuses of the step that produced the input; a string that failed
 * there keeps that status (a failed item never reaches the command). A tmp too small for the
 * unescaped strings: nothing past tmp->bytes_cap is read, the outputs are void and ie_exec_sync
 * reports IE_ERR_CAPACITY. Waits once for the literal path's scratch demand, as
 * ie_interpolate_device (not with ie_exec_set_scratch). */
int ie_unescape_cmd_device(ie_exec* x, const ie_table* t, const uint32_t* d_table_id, const uint8_t* d_bytes,
                           const uint64_t* d_offsets, uint64_t n, const uint8_t* d_status_in, const ie_dev_out* tmp,
                           const ie_dev_out* out);
/* The same command on a views batch (d_lengths nullable: packed input, d_offsets[n + 1]) into a views
 * output, fused: each tile is unescaped in the LDS stage and resolved there, without an unescaped
 * copy in HBM and without a look-back; the strings a tile cannot finish (not staged, or needing
 * the literal path) are unescaped into the exec's scratch pool and resolved in a second pass.
 * Statuses, bytes and IE_RECURSE as ie_unescape_cmd_device. */
int ie_unescape_cmd_device_views(ie_exec* x, const ie_table* t, const uint32_t* d_table_id, const uint8_t* d_bytes,
                                 const uint64_t* d_offsets, const uint32_t* d_lengths, uint64_t n,
                                 const uint8_t* d_status_in, const ie_dev_views* out);
int ie_escape_batch(ie_exec* x, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                    ie_batch** out);

void ie_batch_free(ie_batch* b);

/* ---- wildcard match / capture (py:553-567 is_wildcard_match / get_wildcard_matches; the matcher
 * of goto_map / replace_map / delete_except, py:1688-1773; rust-project/src/runtime.rs:1633-1647,
 * 1754-1775). A wildcard is literal text with '*' (and, as in the reference, U+3020) standing for
 * a DOTALL greedy group; the match is anchored at both ends ('$' also before a trailing '\n').
 * ie_wildcards_build compiles a LIST of wildcards (packed UTF-8, offsets[n_patterns + 1]) onto a
 * device. ie_wildcard_match_*: for each string i, the FIRST wildcard p of the list (or of
 * [range[2i], range[2i+1]) when range is given) that matches; match[i] = p or -1, ncap[i] the
 * number of captures and caps[i * 2 * IE_WC_MAX_CAP + 2c .. +1] = {byte start, byte length} of
 * capture c within string i (re.findall's groups; a wildcard without '*' captures its whole match,
 * as re.findall returns it). Wildcards with more than IE_WC_MAX_CAP groups are rejected.
 * IE_DIALECT_RS follows runtime.rs's regex-crate pattern instead: only '*' is a group, '$' matches
 * at the end only, and a wildcard without '*' has no captures (parity unpinned: no toolchain). ---- */
#define IE_WC_MAX_CAP 16
typedef struct ie_wildcards ie_wildcards;
int ie_wildcards_build(const uint8_t* bytes, const uint64_t* offsets, uint32_t n_patterns, int32_t dialect,
                       int32_t device, ie_wildcards** out);
void ie_wildcards_free(ie_wildcards* w);
int ie_wildcard_match_device(ie_exec* x, const ie_wildcards* w, const uint8_t* d_bytes, const uint64_t* d_offsets,
                             uint64_t n, const uint32_t* d_range, int32_t* d_match, uint8_t* d_ncap, uint32_t* d_caps);
int ie_wildcard_match_batch(ie_exec* x, const ie_wildcards* w, const uint8_t* bytes, const uint64_t* offsets,
                            uint64_t n, const uint32_t* range, int32_t* match, uint8_t* ncap, uint32_t* caps);

/* ---- the map commands over the states of a table set (py:1689-1773, 1843-1868;
 * rust-project/src/runtime.rs:1085-1169, 1649-1731, 1754-1775). State s is table s of the set;
 * every interpolation runs in the resolve kernels and every wildcard test in k_wildcard: a command
 * over any number of states is a few device batches (synchronous; results owned by the library
 * until ie_map_result_free). A map is one {key: value} pair of the task's target_maps /
 * wildcard_maps, raw (the task pre-pass skips them, py:1471-1477).
 *
 * Per item: status IE_OK_STR (the result in bytes/offsets), or why it failed. `where` names the
 * string whose failure the reference raises: 0 = the item itself (goto_map: its text; replace:
 * the leaf, bytes = the string that failed), 1 + j = map j's key, 1 + n_maps + j = map j's value
 * (replace: bytes = the text the key matched; its captures are that key's wildcard groups).
 * `chosen`: the map taken (-1 none). value_id: a typed whole-string result's insert (names). ---- */
typedef struct ie_map_pair {
  const char* key;
  uint64_t key_len;
  const char* value;
  uint64_t value_len;
} ie_map_pair;
typedef struct ie_map_result {
  uint8_t* bytes;
  uint64_t bytes_len;
  uint64_t* offsets;  /* n + 1 */
  uint8_t* status;    /* n     */
  uint32_t* where;    /* n     */
  int32_t* chosen;    /* n     */
  uint32_t* value_id; /* n     */
  uint64_t n;
} ie_map_result;
void ie_map_result_free(ie_map_result* r);
/* goto_map (py:1689-1711) in every state: text, keys and values interpolated and str()-ed; the text's
 * InterpolationException (IE_E_INTERP only) takes the 'NULL' key's value (IE_E_NO_NULL without
 * one), any other failure of the text, then the first failing key, then the first failing value
 * propagates; else the value of the first key that wildcard-matches the text (IE_E_NO_MATCH: none).
 * n = the number of tables; bytes: the target (the caller treats 'CONTINUE'). */
int ie_goto_map(ie_exec* x, const ie_table* t, const char* text, uint64_t text_len, const ie_map_pair* maps,
                uint32_t n_maps, ie_map_result** out);
/* replace_map (py:1713-1773): replace_str on n leaves (leaf i: a string of state table_id[i], the
 * caller's walk of the item, py:1748-1759): each pass interpolates the leaf, takes the first map whose
 * interpolated key matches (a key that fails before a match fails the leaf), interpolates its value
 * against inserts | {'1': capture 1, ...}; repeat_until_done repeats until nothing changes (the
 * reference's unbounded loop stops at 100000 passes: IE_DIVERGED). name (nullable): output_name,
 * interpolated per state (py:1715, no str(): typed results keep their value id) into *names. The
 * clock the keys read is the table's (ie_table_set_clock before the call). */
int ie_replace_map(ie_exec* x, const ie_table* t, const char* name, uint64_t name_len, const uint8_t* bytes,
                   const uint64_t* offsets, const uint32_t* table_id, uint64_t n, const ie_map_pair* maps,
                   uint32_t n_maps, int32_t repeat_until_done, ie_map_result** names, ie_map_result** out);
/* delete (except_matching = 0: the keys some wildcard matches, py:1843-1855) / delete_except (1: the
 * keys no wildcard matches, py:1857-1868) in the given states (NULL: every state): wildcards packed
 * (offsets[n + 1]), as the task pre-pass left them; the keys are removed from the table set
 * (ie_table_set_store: their value ids go back to the set's free list) and listed in out (bytes =
 * the key, where = its state, value_id = the id it freed). */
int ie_delete_keys(ie_exec* x, ie_table* t, const uint32_t* states, uint32_t n_states, const uint8_t* wbytes,
                   const uint64_t* woffsets, uint32_t n_wildcards, int32_t except_matching, ie_map_result** out);

/* ---- get_simple_insertkey (py:477-495 / interp.rs:11-29), host-side classifier used by the
 * callers' control flow (recursive_interpolate, validate_program). Returns 1 when the reference
 * returns a truthy key (py) / Some (rs), 0 otherwise; key_off and key_len locate the key. ---- */
int ie_simple_insertkey(const char* s, uint64_t len, int32_t dialect, uint64_t* key_off,
                        uint64_t* key_len);

/* ---- synthetic workloads of SURVEY §8d (configs 2-4): deterministic splitmix64 ---- */
typedef struct ie_synth ie_synth;
int ie_synth_create(int32_t config, uint64_t seed, ie_synth** out);
void ie_synth_free(ie_synth* s);
uint64_t ie_synth_kv(const ie_synth* s, const ie_kv** kv); /* the inserts, as ie_kv */
/* Strings [first, first+n). bytes may be NULL (offsets + *total only). offsets are relative
 * to string `first` (offsets[0] == 0). */
int ie_synth_strings_host(const ie_synth* s, uint64_t first, uint64_t n, uint8_t* bytes,
                          uint64_t bytes_cap, uint64_t* offsets, uint64_t* total);
int ie_synth_strings_device(ie_exec* x, const ie_synth* s, uint64_t first, uint64_t n,
                            uint8_t* d_bytes, uint64_t bytes_cap, uint64_t* d_offsets,
                            uint64_t* total /* host */);

#ifdef __cplusplus
}
#endif
#endif /* IE_AMD_H */
