// ie_kernels.h — launch interface between the host library (ie_host.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ie_amd.h"
#include "ie_common.h"

namespace ie {

constexpr int kBlock = 256;          // lanes per workgroup = strings per tile
constexpr int kMaxDepth = 6;         // fast-path nesting limit (deeper: literal path)
constexpr int kKeyCap = 32;          // exact-evaluator key bytes per lane (longer keys: literal path)

constexpr int kTileBytes = 17664;    // escape kernels: LDS input stage per 256-string tile
constexpr int kStageBytes = 20480;   // escape kernels: LDS output stage

// k_resolve's tile: IE_RBLOCK strings (one lane each); the stages scale with it
#ifndef IE_RBLOCK
#define IE_RBLOCK 256
#endif
constexpr int kRBlock = IE_RBLOCK;
constexpr int kRTileBytes = 17664 * IE_RBLOCK / 256;   // LDS input stage: the tile's first bytes
constexpr int kRStageBytes = 20480 * IE_RBLOCK / 256;  // LDS output stage; larger outputs: k_emit_windows

enum { kOpInterp = 0, kOpUnescape = 1, kOpEscape = 2 };

struct Batch {
  const uint8_t* bytes;     // input payload
  const uint64_t* in_off;   // n + 1 input offsets (packed), or n starts (views input: in_len set)
  uint64_t n;
  uint64_t* out_off;        // n + 1 output offsets (packed), or n starts (views output: out_len set)
  uint8_t* status;          // n
  uint32_t* value_id;       // n
  const uint32_t* table_id; // n: the table of the set each string is resolved against, or null (0)
  // views (k_resolve only): string i is bytes[in_off[i], + in_len[i]); any placement is accepted,
  // strings of one tile that lie together in order are staged together (what a views output is)
  const uint32_t* in_len;   // n or null
  // views output: no global order, so no look-back: each tile claims its output range with one
  // atomic on the exec's cursor; string i's result is out[out_off[i], + out_len[i])
  uint32_t* out_len;        // n or null
  // a deferred subset (the unescape command's second pass): string i's results go to position
  // out_index[i] of the output arrays, and only the first *n_dev strings exist (a device count;
  // the grid is sized for n)
  const uint32_t* out_index;  // n or null
  const uint32_t* n_dev;      // 1 or null
};

struct Work {
  uint64_t* total;       // 1   caller's total word
  // single-pass resolve
  uint32_t* tile_ticket; // 1   dynamic tile ids (zeroed per call)
  uint64_t* tile_state;  // tiles: look-back words (zeroed per call)
  uint32_t* err;         // 1   look-back timeout flag
  uint32_t* stats;       // 5   telemetry: literal strings, direct tiles, look-back polls, exact-path
                         //     strings, chain failures (the adaptive variant choice)
  uint64_t* stamps;      // diagnostic (IE_DEBUG_STAMPS): 8 words per tile, or null
  uint32_t debug_noeval; // diagnostic (IE_DEBUG_NOEVAL): bit 0 copy strings verbatim (pipeline floor),
                         // bit 1 views tiles claim no output range (the range at twice the input offset)
  uint32_t fast_mode;    // level evaluator: 1 on (default), 0 off; diagnostics 2 = parse only, 3 = no probes
  uint8_t* pool;         // literal-path scratch
  uint64_t* pool_used;   // 1
  uint64_t pool_bytes;
  uint32_t lit_cap_max;  // 1: literal strings get the full IE_SIZE_CAP working space
  uint32_t fail_commit;  // 1: chain failures commit in the chain evaluator (k_resolve<true>)
  // tiles whose output does not fit the LDS stage: k_emit_windows writes their bytes
  uint32_t* defer_count; // 1
  uint32_t* defer_tiles; // 8 words per deferred tile: {tile | kDeferSub, 0, base (u64), total (u64), 0, 0}
  uint4* defer_desc;     // tiles * kBlock * 4: each string's descriptor
  uint64_t* cursor;      // 1   views output: bytes claimed so far (zeroed per call)
  // the fused unescape command (k_resolve<.., UNESC>): strings it cannot finish in the stage (not
  // staged, or needing the literal path) are listed here for the deferred pass
  uint32_t* udefer_list;  // n
  uint32_t* udefer_count; // 1
  // a LEAN first pass (launch_resolve_deferring) writes each deferred string's view for the second
  // pass itself: its input offset, length and table id at the string's place in udefer_list
  uint64_t* sub_off;
  uint32_t* sub_len;
  uint32_t* sub_tid;
  uint64_t* shards;      // 16 u64 words 16 apart (reserved ranges' tile sums), zeroed per call
  uint32_t n_shards;
  uint32_t defer_slow;   // k_resolve on a views batch: strings the chain jobs cannot finish are listed
                         // in udefer_list for a second pass instead of evaluated in their tile
  // views output of a packed batch, reserved ranges (IE_OPT_RESERVE): a tile's output goes to
  // reserve16 / 16 times its input span's offset from the batch's first byte when it fits there (no
  // atomic), else to the overflow region after the whole batch's reservation (W.cursor); the tile
  // sums go to the 16 `shards` words (u64, 128 B apart) and k_emit_windows adds them into *total
  // keys only the host can look up (IE_NEEDS_HOST, inserts-dir tables) and, with err_keys
  // (IE_OPT_ERROR_KEYS), the missing key of every IE_E_INTERP string: records {u32 string index,
  // u32 length, bytes padded to 4} appended by the literal path (ie_exec_host_keys)
  uint8_t* host_keys;
  uint64_t host_keys_cap;
  uint64_t* host_keys_used;
  uint32_t err_keys;     // IE_E_INTERP strings go to the literal path, which records their key
  uint32_t reserve16;
  uint64_t* res_ovf;     // 1   the overflow region's start (written by the reserved pass)
  uint32_t recurse;      // k_resolve in the unescape command (py dialect): whole-string items whose
                         // result recursive_interpolate walks again report IE_RECURSE
  // the call's telemetry words (stats[0..4]) in host-mapped pinned memory, written by its last
  // k_emit_windows (no copy kernel after it); null: the host copies them itself
  uint32_t* stat_out;
  // grid hints from the exec's last completed call (0: the defaults): a deferred subset's bounded
  // grid and the emit kernel's (both stride over their work: any size is correct, a small one is
  // cheap when there is little to do)
  uint32_t sub_grid, emit_grid;
  // a two-pass call's emit kernel zeroes the exec's other counter set (zero_words words) for the next
  // call (no fill before it)
  uint32_t* zero_next;
  uint32_t zero_words;
  // the literal pool's demand (pool_used) with the call's number, seq << 40 | used, to host-mapped
  // memory by the call's last k_emit_windows (null: not this kernel)
  uint64_t* pool_out;
  uint32_t pool_seq;
  // a one-tile views call without copies (ie_host.cpp, run_host_small_zc): k_resolve's last
  // instructions put counter words 0-15 here (host-mapped) and zero them on the device (null: not)
  uint32_t* ctr_host;
  uint32_t zero_on_overflow; // escape kernels: when the output exceeds its capacity, write every
                             // offset as 0 (a step that reads these strings next then reads nothing)
  // escape pipeline
  uint32_t* out_len;     // n
  uint64_t* tile_sum;    // tiles
  uint64_t* tile_base;   // tiles
};

// compiled wildcard patterns (ie_wildcard.hip): pattern p = literals [pat_lit[p], pat_lit[p+1]),
// literal l = bytes[lit_off[l] .. lit_off[l] + lit_len[l]); the groups sit between the literals
constexpr uint32_t kWcMaxCap = IE_WC_MAX_CAP;
struct WcSet {
  const uint8_t* bytes;
  const uint32_t* lit_off;
  const uint32_t* lit_len;
  const uint32_t* pat_lit;  // n_pat + 1
  uint32_t n_pat;
  uint32_t rs;              // IE_DIALECT_RS: '$' at the end only, no capture without a group
};
hipError_t launch_wildcard(const WcSet& P, const uint8_t* bytes, const uint64_t* off, uint64_t n,
                           const uint32_t* range, int32_t* match, uint8_t* ncap, uint32_t* caps, hipStream_t st);

// no_emit: a one-tile views batch without the emit kernel (k_resolve writes the total; a tile it
// had to defer is left unwritten: the caller sees defer_count and runs the batch again in full)
hipError_t launch_resolve(const Batch& B, const Work& W, const DevTable& T, uint8_t* out,
                          uint64_t cap, hipStream_t st, bool no_emit = false);
// the same with 512-string tiles (ie_resolve512.hip)
hipError_t launch_resolve512(const Batch& B, const Work& W, const DevTable& T, uint8_t* out,
                             uint64_t cap, hipStream_t st);
hipError_t launch_escape(int op, const Batch& B, const Work& W, uint8_t* out, uint64_t cap,
                         hipStream_t st);
hipError_t launch_cap_check(const uint64_t* total, uint64_t cap, uint32_t* err, hipStream_t st);
// the unescape command, views in and out (ie_resolve.hip): the fused resolve (unescape while
// staging), then the deferred strings: unescaped into the pool (k_unesc_deferred), resolved again
hipError_t launch_unescape_cmd(const Batch& B, const Work& W, const DevTable& T, uint8_t* out, uint64_t cap,
                               uint64_t* sub_off, uint32_t* sub_len, uint32_t* sub_tid, hipStream_t st);
// k_resolve on a views batch in two passes: the heavy strings listed by the first (W.defer_slow)
// are resolved by the second as a subset (their views in sub_off / sub_len / sub_tid)
hipError_t launch_resolve_deferring(const Batch& B, const Work& W, const DevTable& T, uint8_t* out, uint64_t cap,
                                    uint64_t* sub_off, uint32_t* sub_len, uint32_t* sub_tid, hipStream_t st);
// patch k writes len[k] (<= 256) bytes of src + soff[k] to the device address dst[k]
// (ie_table_set_update / _set_clock)
hipError_t launch_patch(const uint8_t* src, const uint64_t* dst, const uint32_t* soff, const uint32_t* len, uint32_t n,
                        hipStream_t st);
// a small patch set carried in the kernel's arguments (no upload before the launch): a scalar
// set_interpdata's few entries, pilot and text, as up to kPatchInlineN pieces of <= 16 bytes
// (piece c: len[c] bytes of data[16c..] to dst[c]), one lane each
constexpr uint32_t kPatchInlineN = 128;
struct PatchInline {
  uint32_t data[kPatchInlineN][4];
  uint64_t dst[kPatchInlineN];
  uint8_t len[kPatchInlineN];
  uint32_t n;
};
hipError_t launch_patch_inline(const PatchInline& a, hipStream_t st);
// whether k_resolve (ie_resolve.hip) was compiled for the two-choice table experiment (-DIE_CUCKOO):
// the host places keys the same way or refuses to build (ie_host.cpp, upload_table)
bool kernels_cuckoo();
hipError_t launch_status_carry(const uint8_t* before, uint8_t* after, uint64_t n, hipStream_t st);
hipError_t launch_debug_probe(const DevTable& T, const uint8_t* key, uint32_t klen, uint64_t* out,
                              hipStream_t st);
hipError_t launch_synth(const SynthParams& P, uint64_t first, uint64_t n, uint64_t* d_lens,
                        uint64_t* d_part, uint64_t* d_offsets, uint64_t* d_total, uint8_t* d_bytes,
                        hipStream_t st);

}  // namespace ie
