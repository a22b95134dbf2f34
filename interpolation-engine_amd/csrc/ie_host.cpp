// ie_host.cpp — host side of libie_amd.so: the C ABI of include/ie_amd.h.
//
//   table build    get_interpdata (py:430-467 / interp.rs:91-137) frozen into a device hash table:
//                  dict semantics (last duplicate wins), '' never an entry, 'HH:MM' / 'HH:MM:SS'
//                  injected from one clock per build, per-entry splice/inert/key flags.
//   exec           one HIP stream + a grow-only device workspace; no allocation inside the
//                  device entry points once the workspace fits (graph-capturable).
//   batch calls    ie_interpolate_device (async, device pointers) and the synchronous host
//                  convenience ie_interpolate_batch (H2D, kernels, D2H, capacity/overflow retry).
// There is no CPU execution path for the resolver: every string is resolved by the kernels in
// ie_kernels.hip; when no device is present the entry points fail with IE_ERR_NO_DEVICE.
#include <emmintrin.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <iterator>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "../../include/ie_amd.h"
#include "ie_common.h"
#include "ie_kernels.h"
#include "ie_internal.h"

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

bool have_device() {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}


// ---- splice-text analysis for the fast path (see DESIGN.md "inert values") ----
// The rules look at the bytes around a brace, a backslash or U+3020's lead byte only: 16 bytes at a
// time are tested for those four bytes (SSE2), and the rules run at the hits (a store's history text
// is kilobytes without one).
uint32_t text_flags(const std::string_view t) {
  const uint8_t* p = (const uint8_t*)t.data();
  const size_t n = t.size();
  auto breaks = [&](size_t i) -> bool {  // does the byte at i make the text non-inert?
    const uint8_t c = p[i];
    if (c == '{' || c == '}') return i == 0 || p[i - 1] != '\\';  // re-resolves
    if (c == 0xE3) return i + 2 < n && p[i + 1] == 0x80 && p[i + 2] == 0xA0;  // U+3020 collides with the placeholders
    if (c == '\\' && i + 1 < n && p[i + 1] == '}')
      return i == 0 || p[i - 1] == '.' || p[i - 1] == '}';  // '.' + '\}' across the seam; '.\}' restores as '\{.'
    return false;
  };
  size_t i = 0;
  const __m128i lb = _mm_set1_epi8('{'), rb = _mm_set1_epi8('}'), bs = _mm_set1_epi8('\\'),
                e3 = _mm_set1_epi8((char)0xE3);
  for (; i + 16 <= n; i += 16) {
    const __m128i v = _mm_loadu_si128((const __m128i*)(p + i));
    uint32_t hit = (uint32_t)_mm_movemask_epi8(_mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, lb), _mm_cmpeq_epi8(v, rb)),
                                                            _mm_or_si128(_mm_cmpeq_epi8(v, bs), _mm_cmpeq_epi8(v, e3))));
    for (; hit; hit &= hit - 1)
      if (breaks(i + __builtin_ctz(hit))) return 0u;
  }
  for (; i < n; i++)
    if (breaks(i)) return 0u;
  if (n && p[n - 1] == '\\') return 0u;  // escapes a following brace (trailing backslash)
  return EF_INERT;
}

uint32_t kind_flags(int32_t kind, int32_t dialect) {
  uint32_t f = (uint32_t)kind & EF_KIND_MASK;
  bool splice;
  if (dialect == IE_DIALECT_PY)  // py:530
    splice = kind == IE_KIND_STR || kind == IE_KIND_INT || kind == IE_KIND_LIST;
  else  // interp.rs:71-80
    splice = kind == IE_KIND_STR || kind == IE_KIND_INT || kind == IE_KIND_FLOAT || kind == IE_KIND_LIST;
  if (splice) f |= EF_SPLICE_OK;
  if (dialect == IE_DIALECT_PY) {
    if (kind == IE_KIND_STR) f |= EF_KEY_STR;
    if (kind == IE_KIND_LIST || kind == IE_KIND_DICT) f |= EF_KEY_UNHASHABLE;
  } else {
    f |= EF_KEY_STR;  // value_to_string (interp.rs:48, 51)
  }
  return f;
}

uint64_t fmix64_host(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

uint64_t key_hash(const std::string_view k, uint64_t seed, uint32_t tid) {
  return hash_key((uint32_t)k.size(), [&](uint32_t j) { return (uint8_t)k[j]; }, seed, tid);
}

// Perfect-hash placement (hash-and-displace): keys are grouped by ph_group (about 4 per group);
// groups, largest first, each get the smallest 16-bit pilot that sends all their keys to free,
// distinct entries. Fails (false) when some group has no such pilot; the caller then grows the
// table or changes the seed.
bool ph_place(const std::vector<uint64_t>& hash, uint64_t m, uint32_t nb, std::vector<uint16_t>& pilots,
              std::vector<uint32_t>& slot_of) {
  std::vector<uint32_t> start(nb + 1, 0), order(hash.size());
  for (uint64_t h : hash) start[ph_group(h, nb) + 1]++;
  for (uint32_t g = 0; g < nb; g++) start[g + 1] += start[g];
  {
    std::vector<uint32_t> fill(start.begin(), start.end() - 1);
    for (uint32_t i = 0; i < (uint32_t)hash.size(); i++) order[fill[ph_group(hash[i], nb)]++] = i;
  }
  std::vector<uint32_t> groups(nb);
  for (uint32_t g = 0; g < nb; g++) groups[g] = g;
  std::stable_sort(groups.begin(), groups.end(), [&](uint32_t a, uint32_t b) {
    return start[a + 1] - start[a] > start[b + 1] - start[b];
  });
  std::vector<uint8_t> taken(m, 0);
  pilots.assign(nb, 0);
  slot_of.assign(hash.size(), 0);
  std::vector<uint32_t> cand;
  for (uint32_t g : groups) {
    const uint32_t lo = start[g], hi = start[g + 1];
    if (lo == hi) break;  // sorted by size: the rest are empty
    bool found = false;
    for (uint32_t p = 0; p < 65536 && !found; p++) {
      cand.clear();
      bool ok = true;
      for (uint32_t k = lo; k < hi && ok; k++) {
        const uint32_t s = ph_slot(hash[order[k]], p, (uint32_t)m);
        if (taken[s]) ok = false;
        for (uint32_t c : cand) ok &= c != s;
        cand.push_back(s);
      }
      if (!ok) continue;
      for (uint32_t k = lo; k < hi; k++) {
        taken[cand[k - lo]] = 1;
        slot_of[order[k]] = cand[k - lo];
      }
      pilots[g] = (uint16_t)p;
      found = true;
    }
    if (!found) return false;
  }
  return true;
}

int set_device(int32_t dev) {
  if (!have_device()) return fail(IE_ERR_NO_DEVICE, "no HIP device visible (libie_amd has no CPU path)");
  IE_HIP(hipSetDevice(dev));
  return IE_SUCCESS;
}

// workspace for a batch of n strings. counters (u32 words): [0] tile ticket, [1] look-back error,
// [2..3] pool bytes used (u64), [4..8] telemetry (literal strings, deferred tiles, look-back polls,
// exact-path strings, chain failures), [9] deferred-tile count, [10..11] views output cursor (u64),
// [12] the fused unescape command's deferred-string count; zeroed on every call.
// a views batch this large takes the two-pass path by default (IE_OPT_DEFER 2): the LEAN first pass
// saves more than the second pass's fixed cost (config 3 0.844 -> 0.815 ms, config 2 0.108 -> 0.106 ms,
// profiles/r05/ab/lean_two_pass.txt)
constexpr uint64_t kLeanMinN = 1ull << 19;
constexpr uint32_t kSumShards = 16;  // reserved-range tile sums (IE_OPT_RESERVE), 128 B apart after the counters
constexpr uint64_t kCounterBytes = 64 + kSumShards * 128;
// Two counter sets, used in turn: a two-pass views call's last kernel (k_emit_windows) zeroes the set
// it did not use, so the next call starts on a clean set without a fill of its own; every other call
// fills its set first. The look-back words of a packed interpolation follow both sets.
constexpr uint64_t kLookbackOff = 2 * kCounterBytes;
inline uint8_t* ctr_base(ie_exec* x) { return (uint8_t*)x->counters.p + x->ctr_cur * kCounterBytes; }
int ensure_work(ie_exec* x, int op, uint64_t n) {
  // (k_resolve tiles of 128 strings or more: enough look-back words and deferred-tile slots)
  const uint64_t tiles = (n + 127) / 128 + 1;
  // the counter sets, then (interpolation) the look-back words: one buffer (a new one is not clean)
  const void* const before = x->counters.p;
  IE_HIP(x->counters.ensure(kLookbackOff + (op == kOpInterp ? tiles * sizeof(uint64_t) : 0)));
  if (x->counters.p != before) x->ctr_next_clean = false;
  if (op == kOpInterp) {
    IE_HIP(x->pool.ensure(x->pool_request));
    // room for every tile to be deferred (64 B of descriptor per string; grow-only, never read
    // unless written, so only HBM capacity is spent), twice: a two-pass views call appends its
    // deferred subset's tiles to the first pass's list (one k_emit_windows for both)
    IE_HIP(x->defer_tiles.ensure(2 * tiles * 32));  // (a 32-byte record per deferred tile)
    IE_HIP(x->defer_desc.ensure(2 * tiles * 128 * 64));  // whole tiles of kRBlock >= 128 strings
  } else {
    IE_HIP(x->out_len.ensure((n + 1) * sizeof(uint32_t)));
    IE_HIP(x->tile_sum.ensure(tiles * sizeof(uint64_t)));
    IE_HIP(x->tile_base.ensure(tiles * sizeof(uint64_t)));
  }
  return IE_SUCCESS;
}

Work make_work(ie_exec* x, uint64_t* total) {
  Work W{};
  void* const C = x->ctr_override ? (void*)x->ctr_override : (void*)ctr_base(x);
  W.total = total;
  W.tile_ticket = (uint32_t*)C;
  W.err = (uint32_t*)C + 1;
  W.stats = (uint32_t*)C + 4;
  W.stamps = x->stamp_tiles ? (uint64_t*)x->stamps.p : nullptr;
  W.debug_noeval = x->opt_noeval;  // diagnostic hooks, see DESIGN.md
  W.fast_mode = x->opt_fast;       // 0: exact evaluator only
  W.pool_used = (uint64_t*)C + 1;
  W.defer_count = (uint32_t*)C + 9;
  W.defer_tiles = (uint32_t*)x->defer_tiles.p;
  W.defer_desc = (uint4*)x->defer_desc.p;
  // (the small host path's own block: its look-back words right after its counters)
  W.tile_state = (uint64_t*)(x->ctr_override ? (uint8_t*)C + kCounterBytes : (uint8_t*)x->counters.p + kLookbackOff);
  W.shards = (uint64_t*)((uint8_t*)C + 64);
  W.n_shards = kSumShards;
  W.cursor = (uint64_t*)C + 5;  // words 10-11
  W.udefer_count = (uint32_t*)C + 12;
  W.res_ovf = (uint64_t*)C + 7;  // words 14-15
  W.zero_on_overflow = x->cmd_first ? 1u : 0u;
  W.pool = (uint8_t*)x->pool.p;
  W.pool_bytes = x->pool.bytes;
  W.lit_cap_max = x->lit_cap_max;
  W.out_len = (uint32_t*)x->out_len.p;
  W.tile_sum = (uint64_t*)x->tile_sum.p;
  W.tile_base = (uint64_t*)x->tile_base.p;
  return W;
}

// d_out_len / d_in_len (k_resolve only): views output / views input (ie_interpolate_device_views)
// a device pass starts a new host-key list
int reset_host_keys(ie_exec* x) {
  if (x->host_keys.p && x->hk_dirty) IE_HIP(hipMemsetAsync(x->host_keys.p, 0, 16, x->stream));
  x->hk_dirty = false;
  return IE_SUCCESS;
}

// the device's host-key records of the last pass (synchronises)
int read_host_keys(ie_exec* x, std::vector<uint8_t>& out) {
  out.clear();
  if (!x->host_keys.p) return IE_SUCCESS;
  uint64_t used = 0;
  IE_HIP(hipMemcpyAsync(&used, x->host_keys.p, 8, hipMemcpyDeviceToHost, x->stream));
  IE_HIP(hipStreamSynchronize(x->stream));
  used = std::min<uint64_t>(used, x->host_keys.bytes - 16);  // (records past the list's end were dropped)
  out.resize(used);
  if (used) IE_HIP(hipMemcpy(out.data(), (uint8_t*)x->host_keys.p + 16, used, hipMemcpyDeviceToHost));
  // keep whole records only
  uint64_t k = 0;
  while (k + 8 <= out.size()) {
    uint32_t len;
    memcpy(&len, out.data() + k + 4, 4);
    const uint64_t next = k + 8 + ((len + 3ull) & ~3ull);
    if (next > out.size()) break;
    k = next;
  }
  out.resize(k);
  return IE_SUCCESS;
}

// reserve_ok: the caller is ie_interpolate_device_views (the only entry whose caller sized the output
// for IE_OPT_RESERVE; the host batch APIs read back *total bytes and keep one claim per tile)
int run_device(ie_exec* x, int op, const ie_table* t, const uint8_t* d_bytes, const uint64_t* d_off,
               uint64_t n, const ie_dev_out* out, const uint32_t* d_tid = nullptr, uint32_t* d_out_len = nullptr,
               const uint32_t* d_in_len = nullptr, bool reserve_ok = false) {
  if (!x || !d_off || !out || !out->offsets || !out->status || !out->total || (op == kOpInterp && !t))
    return fail(IE_ERR_INVALID, "null argument");
  if (n && !d_bytes) return fail(IE_ERR_INVALID, "null input bytes");
  if (n && (!out->value_id && op == kOpInterp)) return fail(IE_ERR_INVALID, "null value_id");
  if (op == kOpInterp && t->device != x->device)
    return fail(IE_ERR_INVALID, "table and exec live on different devices");
  int rc = set_device(x->device);
  if (rc) return rc;
  if (n > 0xFFFFFFF0ull) return fail(IE_ERR_INVALID, "batch larger than 2^32 strings");
  if (op == kOpInterp && t->patch_pending.load(std::memory_order_acquire)) {  // (an update's patch kernel)
    ie_table* tm = const_cast<ie_table*>(t);
    if (hipEventQuery(t->patched) == hipSuccess) tm->patch_pending.store(false, std::memory_order_relaxed);
    else IE_HIP(hipStreamWaitEvent(x->stream, t->patched, 0));
  }
  rc = ensure_work(x, op, n);
  if (rc) return rc;
  x->pool_pub = false;
  // the counter set of this call: the clean one the last two-pass call left, else the current one
  // (filled below)
  bool ctr_clean = false;
  if (!x->ctr_override && x->ctr_next_clean) {
    x->ctr_cur ^= 1u;
    x->ctr_next_clean = false;
    ctr_clean = true;
  }
  x->stamp_tiles = 0;
  x->no_emit_used = false;
  if (op == kOpInterp && !x->stamps_path.empty()) {  // diagnostic build hook, see DESIGN.md
    const uint64_t tiles = (n + kRBlock - 1) / kRBlock;
    IE_HIP(x->stamps.ensure(tiles * 128));
    x->stamp_tiles = tiles;
  }
  if (op != kOpInterp && (d_out_len || d_in_len)) return fail(IE_ERR_INVALID, "views are an interpolation layout");
  if (n && d_out_len == nullptr && out->offsets == nullptr) return fail(IE_ERR_INVALID, "null offsets");
  Batch B{d_bytes, d_off, n, out->offsets, out->status, out->value_id, d_tid, d_in_len, d_out_len};
  Work W = make_work(x, out->total);
  // the literal path records IE_NEEDS_HOST keys (and, IE_OPT_ERROR_KEYS, the missing keys of IE_E_INTERP)
  if (op == kOpInterp && ((t->dev.flags & TF_HAS_DIR) || x->opt_err_keys)) {
    if (!x->host_keys.p) {
      IE_HIP(x->host_keys.ensure(1ull << 20));
      IE_HIP(hipMemsetAsync(x->host_keys.p, 0, 16, x->stream));
    }
    W.host_keys = (uint8_t*)x->host_keys.p + 16;
    W.host_keys_used = (uint64_t*)x->host_keys.p;
    W.host_keys_cap = x->host_keys.bytes - 16;
    x->hk_dirty = true;
  }
  W.err_keys = op == kOpInterp && x->opt_err_keys ? 1u : 0u;
  W.recurse = op == kOpInterp && x->in_cmd && t->dialect == IE_DIALECT_PY ? 1u : 0u;
  // reserved output ranges: a views output of a packed interpolation batch (not the unescape command)
  W.reserve16 = reserve_ok && op == kOpInterp && d_out_len && !d_in_len && !x->in_cmd && !x->cmd_fused ? x->opt_reserve : 0u;
  hipStream_t st = x->stream;
  const uint64_t cap = out->bytes ? out->bytes_cap : 0;
  if (x->timing) IE_HIP(hipEventRecord(x->ev[0], st));
  // the counters and, for a packed interpolation, the look-back words (one fill instead of two)
  const uint64_t zero_tiles = (op == kOpInterp && n && !d_out_len) ? (n + 127) / 128 : 0;  // (ensure_work)
  if (!x->ctr_override && (!ctr_clean || zero_tiles)) {  // (one fill: from the set through the look-back words)
    uint8_t* const c0 = ctr_base(x);
    const uint64_t to = zero_tiles ? kLookbackOff + zero_tiles * sizeof(uint64_t) : (uint64_t)(c0 - (uint8_t*)x->counters.p) + kCounterBytes;
    IE_HIP(hipMemsetAsync(c0, 0, to - (uint64_t)(c0 - (uint8_t*)x->counters.p), st));
  }
  if (n == 0) {
    if (!d_out_len) IE_HIP(hipMemsetAsync(out->offsets, 0, sizeof(uint64_t), st));
    IE_HIP(hipMemsetAsync(out->total, 0, sizeof(uint64_t), st));
  } else if (op == kOpInterp) {
    // fail commit: forced by the option (diagnostics, tests), else adaptive on the count of chain
    // failures (misses / unspliceable hits) an earlier batch saw, in either variant
    const bool forced = x->opt_fail_commit >= 0;
    if (x->stat_pending && hipEventQuery(x->stat_ev) == hipSuccess) {
      x->stat_pending = false;
      const uint64_t fails = x->stat_host[4];  // counters word 8: chain failures
      if (fails * 1024 > x->stat_n) x->fail_commit = true;  // > 0.1 % of the strings
      else if (fails == 0) x->fail_commit = false;
      // heavy strings (exact evaluator, literal path): above 0.4 % of a views batch they go to a
      // second pass in tiles of their own; below 1/4096 they stay in their tiles again
      const uint64_t heavy = (uint64_t)x->stat_host[3] + x->stat_host[0];
      if (heavy * 256 > x->stat_n) x->defer_slow = true;
      else if (heavy * 4096 < x->stat_n) x->defer_slow = false;
      // the next two-pass call's grids, from the last two-pass call's telemetry: as many subset
      // workgroups as the strings it deferred need (8 per XCD when none), and a small emit grid
      // when no tile had to be windowed
      if (x->stat_two_pass) {
        const uint64_t need = (x->stat_host[3] + 255) / 256;
        x->hint_sub_grid = (uint32_t)std::min<uint64_t>(1024, std::max<uint64_t>(64, need));
        x->hint_emit_grid = x->stat_host[5] ? 512u : 32u;
        x->hint_fc = x->stat_fc;
      }
    }
    W.fail_commit = forced ? (uint32_t)x->opt_fail_commit : (uint32_t)x->fail_commit;
    if (W.err_keys) W.fail_commit = 0;  // misses go through the exact evaluator to the literal path
    // the adaptive choices' telemetry: written into pinned host words by the call's last emit kernel
    // (no copy after it), or copied below when the call has none (a one-tile no-emit call). The
    // unescape command's calls publish none: their counts (the deferred subset's, the interpolation
    // of unescaped output) misled the next plain batch (config 4: a step after a command took the
    // evaluator without fail commit, 3.3 ms instead of 1.4); the command takes the plain batches' choice
    const bool want_stats = !x->stat_pending && !x->no_stats && !x->in_cmd && !x->cmd_fused;
    bool two_pass = false;
    if (!x->stat_host) {  // (words 0-5 the telemetry, 8-9 the pool demand word)
      IE_HIP(hipHostMalloc((void**)&x->stat_host, 64, hipHostMallocMapped));
      IE_HIP(hipHostGetDevicePointer((void**)&x->stat_dev, x->stat_host, 0));
      IE_HIP(hipEventCreateWithFlags(&x->stat_ev, hipEventDisableTiming));
      memset(x->stat_host, 0, 64);
    }
    W.stat_out = want_stats ? x->stat_dev : nullptr;
    // the literal pool's demand, published to the host by the call's last emit kernel (the device
    // APIs wait for that word instead of synchronising the stream: pool_demand)
    W.pool_out = (uint64_t*)(x->stat_dev + 8);
    W.pool_seq = (uint32_t)(++x->pool_seq & 0xFFFFFFu);
    x->pool_pub = true;
    if (x->timing) IE_HIP(hipEventRecord(x->ev[1], st));
    // 512-string tiles halve the look-back hops: the unescape command's second resolve (its input
    // is interpolation output, so its evaluation is light and the look-back bounds it) takes them
    // by default; everything else the 256-string tiles (ie_resolve512.hip has the numbers)
    const bool wide = x->opt_tile == 512 || (x->opt_tile == 0 && x->in_cmd && !d_out_len && !d_in_len);
    if (x->cmd_fused) {
      IE_HIP(x->u_list.ensure(n * 4));
      IE_HIP(x->u_off.ensure(n * 8));
      IE_HIP(x->u_len.ensure(n * 4));
      if (d_tid) IE_HIP(x->u_tid.ensure(n * 4));
      W.udefer_list = (uint32_t*)x->u_list.p;
      IE_HIP(launch_unescape_cmd(B, W, t->dev, out->bytes, cap, (uint64_t*)x->u_off.p, (uint32_t*)x->u_len.p,
                                 d_tid ? (uint32_t*)x->u_tid.p : nullptr, st));
    } else if (d_out_len && !x->in_cmd && !x->opt_noeval &&
               (x->opt_defer == 1 || (x->opt_defer != 0 && x->defer_slow) || (x->opt_defer == 2 && n >= kLeanMinN))) {
      // a views batch with heavy strings: two passes (launch_resolve_deferring)
      IE_HIP(x->u_list.ensure(n * 4 + 4));
      IE_HIP(x->u_off.ensure(n * 8 + 8));
      IE_HIP(x->u_len.ensure(n * 4 + 4));
      if (d_tid) IE_HIP(x->u_tid.ensure(n * 4 + 4));
      W.udefer_list = (uint32_t*)x->u_list.p;
      // (a grid measured under the other fail-commit mode would be wrong by the failing strings: the
      // evaluator defers them without it, 490 tiles in config 4, and 64 workgroups took 1.1 ms)
      const bool hint_ok = x->hint_fc == (W.fail_commit != 0);
      W.sub_grid = hint_ok ? x->hint_sub_grid : 0u;
      W.emit_grid = hint_ok ? x->hint_emit_grid : 0u;
      two_pass = true;
      if (!x->ctr_override) {  // (the call's emit kernel zeroes the other counter set for the next call)
        W.zero_next = (uint32_t*)((uint8_t*)x->counters.p + (x->ctr_cur ^ 1u) * kCounterBytes);
        W.zero_words = (uint32_t)(kCounterBytes / 4);
      }
      IE_HIP(launch_resolve_deferring(B, W, t->dev, out->bytes, cap, (uint64_t*)x->u_off.p, (uint32_t*)x->u_len.p,
                                      d_tid ? (uint32_t*)x->u_tid.p : nullptr, st));
      if (W.zero_next) x->ctr_next_clean = true;
    } else {
      // (a one-string call: k_resolve alone, one launch and its emit kernel's ~5 µs fewer)
      const bool ne = x->small_no_emit && d_out_len && !wide && !W.reserve16 && !x->opt_noeval && n <= (uint64_t)kRBlock;
      x->no_emit_used = ne;
      if (ne) W.stat_out = nullptr, W.pool_out = nullptr, x->pool_pub = false, W.ctr_host = x->zc_ctr_host;
      IE_HIP(wide ? launch_resolve512(B, W, t->dev, out->bytes, cap, st) : launch_resolve(B, W, t->dev, out->bytes, cap, st, ne));
    }
    if (want_stats) {
      if (!W.stat_out) IE_HIP(hipMemcpyAsync(x->stat_host, W.stats, 6 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
      IE_HIP(hipEventRecord(x->stat_ev, st));
      x->stat_pending = true;
      x->stat_n = n;
      x->stat_two_pass = two_pass;
      x->stat_fc = W.fail_commit != 0;
    }
  } else {
    if (x->timing) IE_HIP(hipEventRecord(x->ev[1], st));
    x->pool_pub = false;
    IE_HIP(launch_escape(op, B, W, out->bytes, cap, st));
  }
  if (x->timing) {
    if (n == 0) IE_HIP(hipEventRecord(x->ev[1], st));
    IE_HIP(hipEventRecord(x->ev[2], st));
    x->ev_recorded = true;
  }
  return IE_SUCCESS;
}

// look-back timeout flag of the last call (after a sync)
int check_device_error(ie_exec* x) {
  uint32_t err = 0;
  if (x->counters.p) IE_HIP(hipMemcpy(&err, (uint32_t*)ctr_base(x) + 1, 4, hipMemcpyDeviceToHost));
  if (err & 2u) return fail(IE_ERR_CAPACITY, "a step's output did not fit its caller-sized buffer");
  if (err) return fail(IE_ERR_TIMEOUT, "look-back spin timed out (a predecessor tile never published)");
  return IE_SUCCESS;
}

// Small host batches (the mirror's one-string calls, reference py:1691-1697 / 1722-1734): the
// inputs packed into one pinned block and sent with one copy, every output array read back with
// one copy, one synchronisation (the generic path below issues a pageable copy per array and
// synchronises three times). Leaves b null when the output outgrew its first-guess capacity: the
// generic path then runs the batch.
constexpr uint64_t kSmallN = 1024, kSmallBytes = 1ull << 16;
inline uint64_t al256(uint64_t v) { return (v + 255) & ~255ull; }

// the exec's zero-copy block (pinned, mapped into the device's address space, coherent: the kernel
// reads what the host has just written and the host what the kernel wrote, with no cache between)
int ensure_zc(ie_exec* x, uint64_t need) {
  if (x->zc_bytes >= need) return IE_SUCCESS;
  if (x->zc_host) (void)hipHostFree(x->zc_host);
  x->zc_host = x->zc_dev = nullptr;
  x->zc_bytes = 0;
  const uint64_t want = std::max<uint64_t>(need, 1ull << 19);
  IE_HIP(hipHostMalloc((void**)&x->zc_host, want, hipHostMallocMapped | hipHostMallocCoherent));
  IE_HIP(hipHostGetDevicePointer((void**)&x->zc_dev, x->zc_host, 0));
  x->zc_bytes = want;
  return IE_SUCCESS;
}

// A one-tile views interpolation (the mirror's scalar call, py:497-541) without copies: the input
// written into the zero-copy block, k_resolve reading it there and writing its results there, the
// call's counters in device memory that k_resolve itself leaves zeroed after putting their words in
// the block (Work::ctr_host). One launch and one wait; run_host_small's two block copies (and the
// waits between the three stream operations) are gone. Same contract as run_host_small.
int run_host_small_zc(ie_exec* x, const ie_table* t, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                      const uint32_t* table_id, ie_batch*& b, std::vector<uint32_t>& lens, uint64_t& total) {
  const uint64_t base = offsets[0], in_bytes = offsets[n] - base, cap = 2 * in_bytes + 4096;
  const uint64_t i_tid = al256((n + 1) * 8), i_bytes = i_tid + al256(table_id ? n * 4 : 0);
  const uint64_t in_size = i_bytes + al256(in_bytes + 64);
  // outputs: total | offsets | lengths | statuses | value ids | bytes | the counter words
  const uint64_t o_off = 256, o_len = o_off + al256((n + 1) * 8), o_st = o_len + al256(n * 4),
                 o_vid = o_st + al256(n + 1), o_bytes = o_vid + al256((n + 1) * 4), o_ctr = o_bytes + al256(cap);
  int rc = ensure_zc(x, in_size + o_ctr + 256);
  if (rc) return rc;
  if (x->zc_dirty || !x->zc_ctr.p) {
    IE_HIP(x->zc_ctr.ensure(kCounterBytes + 256));  // (the counters, then the one-tile look-back words)
    IE_HIP(hipMemsetAsync(x->zc_ctr.p, 0, kCounterBytes + 256, x->stream));
    x->zc_dirty = false;
  }
  uint8_t* const h = x->zc_host;
  uint64_t* const hoff = (uint64_t*)h;
  for (uint64_t i = 0; i <= n; i++) hoff[i] = offsets[i] - base;
  if (table_id) memcpy(h + i_tid, table_id, n * 4);
  if (in_bytes) memcpy(h + i_bytes, bytes + base, in_bytes);
  // IE_SMALL_ZC=2: the input still goes over in one copy (device-memory reads in the kernel), only
  // the outputs are written straight to the host
  uint8_t* dv = x->zc_dev;
  if (x->opt_zc == 2) {
    IE_HIP(x->sm_dev.ensure(std::max<uint64_t>(in_size, 1ull << 19)));
    dv = (uint8_t*)x->sm_dev.p;
    IE_HIP(hipMemcpyAsync(dv, h, i_bytes + in_bytes, hipMemcpyHostToDevice, x->stream));
  }
  uint8_t* const ho = h + in_size;
  uint8_t* const dout = x->zc_dev + in_size;
  ie_dev_out o{dout + o_bytes, cap, (uint64_t*)(dout + o_off), dout + o_st, (uint32_t*)(dout + o_vid), (uint64_t*)dout};
  x->no_stats = true;
  x->ctr_override = (uint8_t*)x->zc_ctr.p;
  x->small_no_emit = true;
  x->zc_ctr_host = (uint32_t*)(dout + o_ctr);
  rc = run_device(x, kOpInterp, t, dv + i_bytes, (const uint64_t*)dv, n, &o,
                  table_id ? (const uint32_t*)(dv + i_tid) : nullptr, (uint32_t*)(dout + o_len));
  x->no_stats = false;
  x->ctr_override = nullptr;
  x->small_no_emit = false;
  x->zc_ctr_host = nullptr;
  const bool no_emit = x->no_emit_used;
  x->no_emit_used = false;
  if (rc) {
    x->zc_dirty = true;
    return rc;
  }
  if (!no_emit) {  // (another path ran, e.g. two passes: the counters stayed as it left them)
    IE_HIP(hipMemcpyAsync(ho + o_ctr, x->zc_ctr.p, 64, hipMemcpyDeviceToHost, x->stream));
    x->zc_dirty = true;
  }
  IE_HIP(hipStreamSynchronize(x->stream));
  const uint32_t* const ctr = (const uint32_t*)(ho + o_ctr);
  if (ctr[1] & 2u) return fail(IE_ERR_CAPACITY, "a step's output did not fit its caller-sized buffer");
  if (ctr[1]) return fail(IE_ERR_TIMEOUT, "look-back spin timed out (a predecessor tile never published)");
  if (no_emit && ctr[9] != 0) return IE_SUCCESS;  // a deferred tile: the generic path (run_host_small)
  total = *(const uint64_t*)ho;
  if (total > cap) return IE_SUCCESS;
  b = new ie_batch{};
  b->n = n;
  b->bytes_len = total;
  b->bytes = new uint8_t[total + 1];
  b->offsets = new uint64_t[n + 1];
  b->status = new uint8_t[n + 1];
  b->value_id = new uint32_t[n + 1];
  if (total) memcpy(b->bytes, ho + o_bytes, total);
  memcpy(b->offsets, ho + o_off, n * 8);
  lens.assign((const uint32_t*)(ho + o_len), (const uint32_t*)(ho + o_len) + n);
  memcpy(b->status, ho + o_st, n);
  memcpy(b->value_id, ho + o_vid, n * 4);
  return IE_SUCCESS;
}

int run_host_small(ie_exec* x, int op, const ie_table* t, const uint8_t* bytes, const uint64_t* offsets,
                   uint64_t n, const uint32_t* table_id, bool views, ie_batch*& b, std::vector<uint32_t>& lens,
                   uint64_t& total) {
  const uint64_t base = offsets[0], in_bytes = offsets[n] - base, cap = 2 * in_bytes + 4096;
  // input block: offsets | table ids | bytes (the device block keeps room for the loads' over-read)
  const uint64_t i_tid = al256((n + 1) * 8), i_bytes = i_tid + al256(table_id ? n * 4 : 0);
  const uint64_t in_size = i_bytes + al256(in_bytes + 64);
  // then the call's counters and look-back words (zeroed here, sent with the input, read back with
  // the output: no fill, one read-back); the exec's own counters when timing asks for its telemetry
  const bool own_ctr = !x->timing;
  const uint64_t ctr_size = own_ctr ? al256(kCounterBytes + ((n + 127) / 128 + 1) * sizeof(uint64_t)) : 0;
  // output block: total | offsets | lengths (views) | statuses | value ids | bytes; then the
  // device error word, read with a copy of its own
  const uint64_t o_off = 256, o_len = o_off + al256((n + 1) * 8), o_st = o_len + al256(views ? n * 4 : 0),
                 o_vid = o_st + al256(n + 1), o_bytes = o_vid + al256((n + 1) * 4), o_err = o_bytes + al256(cap);
  const uint64_t need = in_size + ctr_size + o_err + 256;
  if (x->opt_zc && own_ctr && views && op == kOpInterp && n <= (uint64_t)kRBlock && !x->in_cmd && !x->cmd_fused)
    return run_host_small_zc(x, t, bytes, offsets, n, table_id, b, lens, total);
  IE_HIP(x->sm_dev.ensure(std::max<uint64_t>(need, 1ull << 19)));
  if (x->sm_host_bytes < need) {
    if (x->sm_host) (void)hipHostFree(x->sm_host);
    x->sm_host = nullptr;
    x->sm_host_bytes = 0;
    const uint64_t want = std::max<uint64_t>(need, 1ull << 19);
    IE_HIP(hipHostMalloc((void**)&x->sm_host, want, hipHostMallocDefault));
    x->sm_host_bytes = want;
  }
  uint8_t* const h = x->sm_host;
  uint8_t* const ho = h + in_size + ctr_size;
  uint64_t* const hoff = (uint64_t*)h;
  for (uint64_t i = 0; i <= n; i++) hoff[i] = offsets[i] - base;
  if (table_id) memcpy(h + i_tid, table_id, n * 4);
  if (in_bytes) memcpy(h + i_bytes, bytes + base, in_bytes);
  if (ctr_size) memset(h + in_size, 0, ctr_size);
  uint8_t* const dv = (uint8_t*)x->sm_dev.p;
  uint8_t* const dout = dv + in_size + ctr_size;
  IE_HIP(hipMemcpyAsync(dv, h, ctr_size ? in_size + ctr_size : i_bytes + in_bytes, hipMemcpyHostToDevice, x->stream));
  ie_dev_out o{dout + o_bytes, cap, (uint64_t*)(dout + o_off), dout + o_st, (uint32_t*)(dout + o_vid), (uint64_t*)dout};
  // (the adaptive fail-commit / deferral statistics come from the larger batches)
  x->no_stats = true;
  x->ctr_override = ctr_size ? dv + in_size : nullptr;
  x->small_no_emit = ctr_size != 0 && views;  // (the deferred-tile count comes back with the counters)
  int rc = run_device(x, op, t, dv + i_bytes, (const uint64_t*)dv, n, &o,
                      table_id ? (const uint32_t*)(dv + i_tid) : nullptr, views ? (uint32_t*)(dout + o_len) : nullptr);
  x->no_stats = false;
  x->ctr_override = nullptr;
  x->small_no_emit = false;
  const bool no_emit = x->no_emit_used;
  x->no_emit_used = false;
  if (rc) return rc;
  if (ctr_size) {
    IE_HIP(hipMemcpyAsync(h + in_size, dv + in_size, ctr_size + o_err, hipMemcpyDeviceToHost, x->stream));
  } else {
    IE_HIP(hipMemcpyAsync(ho, dout, o_err, hipMemcpyDeviceToHost, x->stream));
    IE_HIP(hipMemcpyAsync(ho + o_err, (uint32_t*)ctr_base(x) + 1, 4, hipMemcpyDeviceToHost, x->stream));
  }
  IE_HIP(hipStreamSynchronize(x->stream));
  const uint32_t err = ctr_size ? ((const uint32_t*)(h + in_size))[1] : *(const uint32_t*)(ho + o_err);  // (check_device_error's rules)
  if (err & 2u) return fail(IE_ERR_CAPACITY, "a step's output did not fit its caller-sized buffer");
  if (err) return fail(IE_ERR_TIMEOUT, "look-back spin timed out (a predecessor tile never published)");
  // without the emit kernel a deferred tile's bytes were never written (counters word 9): the
  // generic path runs the batch (as for an output beyond the first-guess capacity)
  if (no_emit && ((const uint32_t*)(h + in_size))[9] != 0) return IE_SUCCESS;
  total = *(const uint64_t*)ho;
  if (total > cap) return IE_SUCCESS;
  b = new ie_batch{};
  b->n = n;
  b->bytes_len = total;
  b->bytes = new uint8_t[total + 1];
  b->offsets = new uint64_t[n + 1];
  b->status = new uint8_t[n + 1];
  b->value_id = new uint32_t[n + 1];
  if (total) memcpy(b->bytes, ho + o_bytes, total);
  memcpy(b->offsets, ho + o_off, (views ? n : n + 1) * 8);
  if (views) lens.assign((const uint32_t*)(ho + o_len), (const uint32_t*)(ho + o_len) + n);
  memcpy(b->status, ho + o_st, n);
  memcpy(b->value_id, ho + o_vid, n * 4);
  return IE_SUCCESS;
}

// synchronous host batch: H2D, run, D2H; grows the output buffer and re-runs overflowed
// literal-path strings with the full working space until every status is final.
int run_host(ie_exec* x, int op, const ie_table* t, const uint8_t* bytes, const uint64_t* offsets,
             uint64_t n, ie_batch** outp, const uint32_t* table_id) {
  if (!x || !outp || (n && (!bytes || !offsets))) return fail(IE_ERR_INVALID, "null argument");
  int rc = set_device(x->device);
  if (rc) return rc;
  if ((rc = reset_host_keys(x))) return rc;
  x->hk_host = true;
  x->hk.clear();
  if (table_id && t)
    for (uint64_t i = 0; i < n; i++)
      if (table_id[i] >= t->n_tables) return fail(IE_ERR_INVALID, "table id beyond the table set");
  const uint64_t base = n ? offsets[0] : 0;
  const uint64_t in_bytes = n ? offsets[n] - base : 0;
  // views: the device writes each string where its tile claimed room; packed on the host below
  const bool views = op == kOpInterp && x->opt_views && n;
  ie_batch* b = nullptr;
  std::vector<uint32_t> lens;
  uint64_t total = 0;
  if (x->opt_small && n && n <= kSmallN && in_bytes <= kSmallBytes) {
    rc = run_host_small(x, op, t, bytes, offsets, n, table_id, views, b, lens, total);
    if (rc) return rc;
  }
  if (!b) {
    const uint32_t* d_tid = nullptr;
    if (table_id && n) {
      IE_HIP(x->in_tid.ensure(n * 4));
      IE_HIP(hipMemcpyAsync(x->in_tid.p, table_id, n * 4, hipMemcpyHostToDevice, x->stream));
      d_tid = (const uint32_t*)x->in_tid.p;
    }
    std::vector<uint64_t> off(n + 1);
    for (uint64_t i = 0; i <= n; i++) off[i] = n ? offsets[i] - base : 0;
    IE_HIP(x->in_bytes.ensure(in_bytes + 16));
    IE_HIP(x->in_off.ensure((n + 1) * 8));
    IE_HIP(x->o_off.ensure((n + 1) * 8));
    IE_HIP(x->o_status.ensure(n + 1));
    IE_HIP(x->o_vid.ensure((n + 1) * 4));
    IE_HIP(x->o_total.ensure(8));
    if (in_bytes) IE_HIP(hipMemcpyAsync(x->in_bytes.p, bytes + base, in_bytes, hipMemcpyHostToDevice, x->stream));
    IE_HIP(hipMemcpyAsync(x->in_off.p, off.data(), (n + 1) * 8, hipMemcpyHostToDevice, x->stream));
    uint64_t cap = std::max<uint64_t>(2 * in_bytes + 4096, x->o_bytes.bytes);
    IE_HIP(x->o_bytes.ensure(cap));
    cap = x->o_bytes.bytes;
    ie_dev_out o{(uint8_t*)x->o_bytes.p, cap, (uint64_t*)x->o_off.p, (uint8_t*)x->o_status.p,
                 (uint32_t*)x->o_vid.p, (uint64_t*)x->o_total.p};
    uint32_t* d_len = nullptr;
    if (views) {
      IE_HIP(x->o_len.ensure(n * 4));
      d_len = (uint32_t*)x->o_len.p;
    }
    rc = run_device(x, op, t, (const uint8_t*)x->in_bytes.p, (const uint64_t*)x->in_off.p, n, &o, d_tid, d_len);
    if (rc) return rc;
    IE_HIP(hipMemcpyAsync(&total, o.total, 8, hipMemcpyDeviceToHost, x->stream));
    IE_HIP(hipStreamSynchronize(x->stream));
    if ((rc = check_device_error(x))) return rc;
    if (total > cap) {  // grow and re-run
      IE_HIP(x->o_bytes.ensure(total + 4096));
      o.bytes = (uint8_t*)x->o_bytes.p;
      o.bytes_cap = x->o_bytes.bytes;
      rc = run_device(x, op, t, (const uint8_t*)x->in_bytes.p, (const uint64_t*)x->in_off.p, n, &o, d_tid, d_len);
      if (rc) return rc;
      IE_HIP(hipMemcpyAsync(&total, o.total, 8, hipMemcpyDeviceToHost, x->stream));
      IE_HIP(hipStreamSynchronize(x->stream));
      if ((rc = check_device_error(x))) return rc;
      if (total > o.bytes_cap) return fail(IE_ERR_CAPACITY, "output grew between runs");
    }
    b = new ie_batch{};
    b->n = n;
    b->bytes_len = total;
    b->bytes = new uint8_t[total + 1];
    b->offsets = new uint64_t[n + 1];
    b->status = new uint8_t[n + 1];
    b->value_id = new uint32_t[n + 1];
    if (total) IE_HIP(hipMemcpyAsync(b->bytes, o.bytes, total, hipMemcpyDeviceToHost, x->stream));
    if (d_len) {
      lens.resize(n);
      IE_HIP(hipMemcpyAsync(b->offsets, o.offsets, n * 8, hipMemcpyDeviceToHost, x->stream));
      IE_HIP(hipMemcpyAsync(lens.data(), d_len, n * 4, hipMemcpyDeviceToHost, x->stream));
    } else {
      IE_HIP(hipMemcpyAsync(b->offsets, o.offsets, (n + 1) * 8, hipMemcpyDeviceToHost, x->stream));
    }
    if (n) IE_HIP(hipMemcpyAsync(b->status, o.status, n, hipMemcpyDeviceToHost, x->stream));
    if (n) IE_HIP(hipMemcpyAsync(b->value_id, o.value_id, n * 4, hipMemcpyDeviceToHost, x->stream));
    IE_HIP(hipStreamSynchronize(x->stream));
  }
  if (views) {  // views -> packed in input order
    uint8_t* packed = new uint8_t[total + 1];
    uint64_t w = 0;
    for (uint64_t i = 0; i < n; i++) {
      if (b->offsets[i] + lens[i] > total) {
        delete[] packed;
        ie_batch_free(b);
        return fail(IE_ERR_HIP, "views output outside the batch's bytes");
      }
      if (lens[i]) memcpy(packed + w, b->bytes + b->offsets[i], lens[i]);
      b->offsets[i] = w;
      w += lens[i];
    }
    b->offsets[n] = w;
    delete[] b->bytes;
    b->bytes = packed;
    b->bytes_len = w;
    if (w > total) {
      ie_batch_free(b);
      return fail(IE_ERR_HIP, "views output lengths exceed its total");
    }
  }
  for (uint64_t i = 0; i < n; i++)
    if (b->status[i] != IE_OK_VALUE && b->status[i] != IE_RECURSE) b->value_id[i] = IE_VID_NONE;
  std::vector<uint8_t> recs;  // this batch's host-key records (the device pass above)
  // (records exist only for strings that ended IE_NEEDS_HOST or IE_E_INTERP: no read-back, and no
  // reset before the next pass, when none did)
  bool any_keys = false;
  for (uint64_t i = 0; i < n && !any_keys; i++) any_keys = b->status[i] == IE_NEEDS_HOST || b->status[i] == IE_E_INTERP;
  if (!any_keys) x->hk_dirty = false;
  if (any_keys && op == kOpInterp && t && ((t->dev.flags & TF_HAS_DIR) || x->opt_err_keys) && (rc = read_host_keys(x, recs))) {
    ie_batch_free(b);
    return rc;
  }

  // literal-path strings that ran out of scratch: re-run them alone with the full working space
  if (op == kOpInterp) {
    std::vector<uint64_t> redo;
    for (uint64_t i = 0; i < n; i++)
      if (b->status[i] == IE_E_OVERFLOW) redo.push_back(i);
    if (!redo.empty() && !x->lit_cap_max) {
      std::vector<uint8_t> rb;
      std::vector<uint64_t> ro(1, 0);
      std::vector<uint32_t> rt;
      uint64_t need = 0;
      for (uint64_t i : redo) {
        const uint64_t len = offsets[i + 1] - offsets[i];
        rb.insert(rb.end(), bytes + offsets[i], bytes + offsets[i + 1]);
        ro.push_back(rb.size());
        rt.push_back(table_id ? table_id[i] : 0u);
        need += 4 * (IE_SIZE_CAP(len, t->dev.maxtext) + 4 * t->dev.maxtext + 80);
      }
      const uint64_t saved_pool = x->pool_request;
      x->lit_cap_max = 1;
      x->pool_request = std::max<uint64_t>(need + (1 << 20), saved_pool);
      ie_batch* sub = nullptr;
      rc = run_host(x, op, t, rb.data(), ro.data(), redo.size(), &sub, table_id ? rt.data() : nullptr);
      x->lit_cap_max = 0;
      x->pool_request = saved_pool;
      if (rc) {
        ie_batch_free(b);
        return rc;
      }
      for (uint64_t k = 0; k + 8 <= x->hk.size();) {  // the re-run's records, at their batch indices
        uint32_t idx, len;
        memcpy(&idx, x->hk.data() + k, 4);
        memcpy(&len, x->hk.data() + k + 4, 4);
        const uint64_t rl = 8 + ((len + 3ull) & ~3ull);
        const uint32_t at = idx < redo.size() ? (uint32_t)redo[idx] : idx;
        const size_t o = recs.size();
        recs.insert(recs.end(), x->hk.data() + k, x->hk.data() + k + rl);
        memcpy(recs.data() + o, &at, 4);
        k += rl;
      }
      // splice the re-run results back in
      std::vector<uint8_t> nb;
      std::vector<uint64_t> noff(n + 1, 0);
      nb.reserve(total + sub->bytes_len);
      size_t r = 0;
      for (uint64_t i = 0; i < n; i++) {
        noff[i] = nb.size();
        if (r < redo.size() && redo[r] == i) {
          b->status[i] = sub->status[r];
          b->value_id[i] = sub->value_id[r];
          nb.insert(nb.end(), sub->bytes + sub->offsets[r], sub->bytes + sub->offsets[r + 1]);
          r++;
        } else {
          nb.insert(nb.end(), b->bytes + b->offsets[i], b->bytes + b->offsets[i + 1]);
        }
      }
      noff[n] = nb.size();
      ie_batch_free(sub);
      delete[] b->bytes;
      b->bytes = new uint8_t[nb.size() + 1];
      if (!nb.empty()) memcpy(b->bytes, nb.data(), nb.size());
      b->bytes_len = nb.size();
      memcpy(b->offsets, noff.data(), (n + 1) * 8);
    }
  }
  x->hk.swap(recs);
  x->hk_host = true;
  *outp = b;
  return IE_SUCCESS;
}


#ifndef IE_BUILD_ID
#define IE_BUILD_ID "unstamped-build!"
#endif
// the source id __graft_entry__.build() stamps into the library (found in the file by its marker)
static const char kBuildId[] = "IE_BUILD_ID:" IE_BUILD_ID;

extern "C" {

int32_t ie_abi_version(void) { return IE_ABI_VERSION; }
const char* ie_build_id(void) { return kBuildId + 12; }
const char* ie_last_error(void) { return g_err.c_str(); }
int32_t ie_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

struct Ent {
  std::string_view key, text;
  uint32_t flags, vid;
  uint32_t tid;          // the entry's table within the set
  std::string_view raw;  // EF_RAWALT: the raw value behind a pre-resolved splice text
};

// Byte patches of device memory, applied by one upload and one kernel (k_patch): patch k writes
// len[k] (<= 256) bytes of data (at soff[k]) to the device address dst[k]. Synchronous. The upload
// goes through a grow-only staging buffer of the caller's (a table's); a set of at most
// kPatchInlineN 16-byte pieces goes in the kernel's arguments instead (k_patch_inline).
struct Patches {
  std::vector<uint8_t> data;
  std::vector<uint64_t> dst;
  std::vector<uint32_t> soff, len;
  void add(void* dst_ptr, const void* src, uint64_t n) {
    const uint8_t* s8 = (const uint8_t*)src;
    for (uint64_t k = 0; k < n; k += 256) {
      const uint32_t l = (uint32_t)std::min<uint64_t>(256, n - k);
      dst.push_back((uint64_t)(uintptr_t)dst_ptr + k);
      soff.push_back((uint32_t)data.size());
      len.push_back(l);
      data.insert(data.end(), s8 + k, s8 + k + l);
      while (data.size() & 15) data.push_back(0);
    }
  }
  bool empty() const { return dst.empty(); }
  // many ranges at once: pieces and places counted serially, the bytes copied across the host
  // threads (the ranges sit all over a mirror of tens of MB: the reads are cache misses)
  void add_many(const std::vector<CopyJob>& r) {
    const size_t nr = r.size();
    if (!nr) return;
    std::vector<uint64_t> pf(nr + 1), df(nr + 1);
    pf[0] = dst.size();
    df[0] = data.size();
    for (size_t k = 0; k < nr; k++) {
      const uint64_t np = (r[k].len + 255) / 256;
      pf[k + 1] = pf[k] + np;
      df[k + 1] = df[k] + (np ? (np - 1) * 256 + ((r[k].len - (np - 1) * 256 + 15) & ~15ull) : 0);
    }
    dst.resize(pf[nr]);
    soff.resize(pf[nr]);
    len.resize(pf[nr]);
    data.resize(df[nr]);
    parallel_for(nr, df[nr] - df[0], [&](uint64_t lo, uint64_t hi) {
      for (uint64_t k = lo; k < hi; k++) {
        uint64_t p = pf[k], d = df[k];
        for (uint64_t o = 0; o < r[k].len; o += 256, p++) {
          const uint32_t l = (uint32_t)std::min<uint64_t>(256, r[k].len - o);
          dst[p] = r[k].dst + o;
          soff[p] = (uint32_t)d;
          len[p] = l;
          memcpy(data.data() + d, r[k].src + o, l);
          d += (l + 15) & ~15u;
        }
      }
    });
  }
  void reserve(uint64_t pieces, uint64_t bytes) {
    dst.reserve(pieces);
    soff.reserve(pieces);
    len.reserve(pieces);
    data.reserve(bytes + 16 * pieces);
  }
};

// after the patch kernel: an event the table's next batches wait on (run_device), no device-wide
// synchronisation (the next update or clock set synchronises the device first anyway)
int patched_event(ie_table* t) {
  if (!t->patched) IE_HIP(hipEventCreateWithFlags(&t->patched, hipEventDisableTiming));
  IE_HIP(hipEventRecord(t->patched, nullptr));
  t->patch_pending.store(true, std::memory_order_release);
  return IE_SUCCESS;
}

int apply_patches(ie_table* t, const Patches& P) {
  DevBuf& staging = t->patch_staging;
  const uint64_t n = P.dst.size();
  if (!n) return IE_SUCCESS;
  if (P.data.size() >= (1ull << 32)) return fail(IE_ERR_INVALID, "patch set above 4 GiB");
  uint64_t pieces = 0;
  for (uint64_t k = 0; k < n; k++) pieces += (P.len[k] + 15) / 16;
  if (pieces <= kPatchInlineN) {  // no upload: the launch carries the bytes
    PatchInline a{};
    for (uint64_t k = 0; k < n; k++)
      for (uint32_t o = 0; o < P.len[k]; o += 16, a.n++) {
        a.dst[a.n] = P.dst[k] + o;
        a.len[a.n] = (uint8_t)std::min<uint32_t>(16, P.len[k] - o);
        memcpy(a.data[a.n], P.data.data() + P.soff[k] + o, a.len[a.n]);
      }
    hipError_t e = launch_patch_inline(a, nullptr);
    if (e != hipSuccess) return fail(IE_ERR_HIP, std::string("table patch: ") + hipGetErrorString(e));
    return patched_event(t);
  }
  const uint64_t o_dst = (P.data.size() + 15) & ~15ull, o_soff = o_dst + 8 * n, o_len = o_soff + 4 * n;
  std::vector<uint8_t> blob(o_len + 4 * n);
  memcpy(blob.data(), P.data.data(), P.data.size());
  memcpy(blob.data() + o_dst, P.dst.data(), 8 * n);
  memcpy(blob.data() + o_soff, P.soff.data(), 4 * n);
  memcpy(blob.data() + o_len, P.len.data(), 4 * n);
  IE_HIP(staging.ensure(blob.size()));
  hipError_t e = hipMemcpy(staging.p, blob.data(), blob.size(), hipMemcpyHostToDevice);
  const uint8_t* base = (const uint8_t*)staging.p;
  if (e == hipSuccess)
    e = launch_patch(base, (const uint64_t*)(base + o_dst), (const uint32_t*)(base + o_soff),
                     (const uint32_t*)(base + o_len), (uint32_t)n, nullptr);
  if (e != hipSuccess) return fail(IE_ERR_HIP, std::string("table patch: ") + hipGetErrorString(e));
  return patched_event(t);
}

extern "C++" {
// the key stored at a slot of the host mirror (inline up to kInlineKey bytes, else the arena copy)
std::string_view mirror_key(const ie_table* t, const Entry& e) {
  if (e.key_len <= kInlineKey) return std::string_view((const char*)e.key, e.key_len);
  return std::string_view((const char*)t->h_arena.data() + key_off_of(e.text_off, e.text_len), e.key_len);
}

// [text][pad to 4][key] appended to the mirror's arena: the new text's offset (kernels read a long
// key at key_off_of(text_off, text_len))
uint32_t arena_append(ie_table* t, std::string_view text, std::string_view key) {
  HostArena& a = t->h_arena;
  while (a.size() & 3) a.push_back(0);
  const uint32_t off = (uint32_t)a.size();
  if (t->defer && text.size() >= 256) {  // (placed now, copied with the others in parallel)
    t->defer->push_back(CopyJob{off, (const uint8_t*)text.data(), text.size()});
    a.grow(text.size());
  } else {
    a.insert(a.end(), text.begin(), text.end());
  }
  while (a.size() & 3) a.push_back(0);
  a.insert(a.end(), key.begin(), key.end());
  return off;
}

// the deferred text copies of ie_table_set_update, across the host threads
void flush_copies(ie_table* t) {
  if (!t->defer || t->defer->empty()) return;
  std::vector<CopyJob>& jobs = *t->defer;
  uint8_t* const a = t->h_arena.data();
  uint64_t bytes = 0;
  for (const CopyJob& j : jobs) bytes += j.len;
  parallel_for(jobs.size(), bytes, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t k = lo; k < hi; k++) memcpy(a + jobs[k].dst, jobs[k].src, jobs[k].len);
  });
  jobs.clear();
}

Entry make_entry(ie_table* t, std::string_view key, std::string_view text, uint32_t flags, uint32_t vid, uint32_t tb) {
  Entry b{};
  b.key_len = (uint32_t)key.size();
  b.text_len = (uint32_t)text.size();
  b.vid = vid;
  b.flags = flags | EF_OCCUPIED | (tb << kTidShift);
  b.text_off = arena_append(t, text, key);
  memcpy(b.key, key.data(), std::min<size_t>(key.size(), kInlineKey));
  memcpy(b.text, text.data(), std::min<size_t>(text.size(), kInlineText));
  t->arena_live += ((key_off_of(b.text_off, b.text_len) + b.key_len + 3ull) & ~3ull) - b.text_off;
  return b;
}

// [first, end) of an entry's bytes in the arena: [raw text, pad, u32 raw length] (EF_RAWALT),
// [splice text, pad, key], padded to 4
void arena_span(const ie_table* t, const Entry& e, uint64_t& first, uint64_t& end) {
  first = e.text_off;
  if (e.flags & EF_RAWALT) {
    uint32_t rl;
    memcpy(&rl, t->h_arena.data() + e.text_off - 4, 4);
    first -= 4 + ((rl + 3ull) & ~3ull);
  }
  end = (key_off_of(e.text_off, e.text_len) + e.key_len + 3ull) & ~3ull;
}

// an entry leaves the table or its texts are replaced: its arena bytes are dead
void arena_release(ie_table* t, const Entry& e) {
  if (!(e.flags & EF_OCCUPIED)) return;
  uint64_t a, b;
  arena_span(t, e, a, b);
  t->arena_live -= std::min<uint64_t>(t->arena_live, b - a);
}

// Rewrite of a present key (set_interpdata of a key the table has): the new text goes where the old
// one was when it fits there (the key moves up behind it; the freed tail is dead), else it is
// appended. False: no room in place (the caller appends).
bool rewrite_in_place(ie_table* t, Entry& e, std::string_view text, uint32_t flags, uint32_t vid) {
  if ((e.flags & EF_RAWALT) || ((text.size() + 3ull) & ~3ull) > ((e.text_len + 3ull) & ~3ull)) return false;
  uint64_t a, b;
  arena_span(t, e, a, b);
  uint8_t* base = t->h_arena.data();
  const std::string_view k0 = mirror_key(t, e);
  char kbuf[256];  // (the key moves: copied out first; a long key on the heap)
  std::string klong;
  std::string_view key;
  if (k0.size() <= sizeof kbuf) {
    memcpy(kbuf, k0.data(), k0.size());
    key = std::string_view(kbuf, k0.size());
  } else {
    klong.assign(k0);
    key = klong;
  }
  memset(base + a, 0, b - a);
  memcpy(base + e.text_off, text.data(), text.size());
  const uint32_t ko = key_off_of(e.text_off, (uint32_t)text.size());
  memcpy(base + ko, key.data(), key.size());
  t->arena_live -= (b - a) - ((((uint64_t)ko + key.size() + 3ull) & ~3ull) - e.text_off);
  e.text_len = (uint32_t)text.size();
  e.vid = vid;
  e.flags = flags | EF_OCCUPIED | (e.flags & ~((1u << kTidShift) - 1u));
  memset(e.text, 0, kInlineText);
  memcpy(e.text, text.data(), std::min<size_t>(text.size(), kInlineText));
  return true;
}

// Compaction: every live entry's bytes copied into a fresh arena, in slot order, offsets rewritten
// (the caller uploads the entries and the arena whole)
void compact_arena(ie_table* t) {
  flush_copies(t);
  HostArena na;
  na.swap(t->h_arena_spare);
  na.clear();
  na.reserve(t->arena_live + t->arena_live / 2 + 64);  // (room for the appends that follow)
  // the new places in slot order, then the bytes copied across the host threads
  std::vector<CopyJob> jobs;
  jobs.reserve(t->n_entries);
  uint64_t at = 0;
  for (Entry& e : t->h_entries) {
    if (!(e.flags & EF_OCCUPIED)) continue;
    uint64_t a, b;
    arena_span(t, e, a, b);  // (starts and ends 4-aligned)
    jobs.push_back(CopyJob{at, t->h_arena.data() + a, b - a});
    e.text_off = (uint32_t)(at + (e.text_off - a));
    at += b - a;
  }
  na.grow(at);
  uint8_t* const dst = na.data();
  parallel_for(jobs.size(), at, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t k = lo; k < hi; k++) memcpy(dst + jobs[k].dst, jobs[k].src, jobs[k].len);
  });
  t->h_arena.swap(na);
  t->h_arena_spare.swap(na);
  t->arena_live = t->h_arena.size();
  t->n_compactions++;
}

// Whole-table re-placement at the same capacity (ie_table_set_update, when a group found no pilot
// around a new key): every live entry and `extra` placed again under a new seed. The slot lists
// (groups, clock entries, pre-resolved values) follow their entries; the caller uploads entries
// and pilots whole. False when no seed of a few tried places them all (the table is too full).
bool replace_all(ie_table* t, const Entry& extra) {
  const uint32_t m = t->dev.m, nb = t->dev.nb;
  std::vector<Entry> live;
  std::vector<uint32_t> from;
  for (uint32_t s = 0; s < m; s++)
    if (t->h_entries[s].flags & EF_OCCUPIED) live.push_back(t->h_entries[s]), from.push_back(s);
  live.push_back(extra);
  from.push_back(UINT32_MAX);
  std::vector<std::string> keys(live.size());
  for (size_t i = 0; i < live.size(); i++) keys[i] = std::string(mirror_key(t, live[i]));
  std::vector<uint64_t> hs(live.size());
  std::vector<uint16_t> pilots;
  std::vector<uint32_t> slot_of;
  uint64_t seed = t->dev.seed;
  for (int attempt = 0; attempt < 8; attempt++) {
    seed = fmix64_host(seed + 0x9E3779B97F4A7C15ull);
    for (size_t i = 0; i < live.size(); i++) hs[i] = key_hash(keys[i], seed, live[i].flags >> kTidShift);
    if (!ph_place(hs, m, nb, pilots, slot_of)) continue;
    std::vector<Entry> ne(m);
    std::unordered_map<uint32_t, uint32_t> moved;
    t->groups.assign(nb, {});
    for (size_t i = 0; i < live.size(); i++) {
      ne[slot_of[i]] = live[i];
      if (from[i] != UINT32_MAX) moved[from[i]] = slot_of[i];
      t->groups[ph_group(hs[i], nb)].push_back(slot_of[i]);
    }
    for (uint32_t& cs : t->clock_slots)
      if (moved.count(cs)) cs = moved[cs];
    for (auto& kv : t->rawalt) {  // (a deleted entry's slot is dropped)
      std::vector<uint32_t> keep;
      for (uint32_t rs : kv.second)
        if (moved.count(rs)) keep.push_back(moved[rs]);
      kv.second = std::move(keep);
    }
    t->h_entries = std::move(ne);
    t->h_pilots = std::move(pilots);
    t->dev.seed = seed;
    return true;
  }
  return false;
}

}  // extern "C++"

// Entries -> perfect-hash table on the device.
// a placement to reuse (the pre-resolution's second upload: same keys, same slots)
struct Placement {
  uint64_t seed, m;
  uint32_t nb;
  std::vector<uint16_t> pilots;
  std::vector<uint32_t> slot_of;
};

int upload_table(const std::vector<Ent>& ents, uint32_t n_tables, int32_t dialect, uint32_t flags,
                 int32_t device, ie_table** out, const Placement* reuse = nullptr,
                 std::vector<uint32_t>* slots_out = nullptr) {
  // the arena's layout first (every entry's place, serially: a prefix sum), then the bytes, the
  // entries and the key hashes across the host threads
  const uint64_t ne = ents.size();
  std::vector<uint64_t> at(ne + 1, 0), toffs(ne);
  uint64_t maxtext = 8;
  bool long_keys = false;
  {
    uint64_t pos = 0;
    for (uint64_t i = 0; i < ne; i++) {
      const Ent& e = ents[i];
      long_keys |= e.key.size() > kInlineKey && e.key.size() <= 2 * kInlineKey;
      if (e.key.size() >= 0xFFFFFFF0ull || e.text.size() >= 0xFFFFFFF0ull) return fail(IE_ERR_INVALID, "key or text above 4 GiB");
      pos = (pos + 3) & ~3ull;  // texts 4-byte aligned (dword copies)
      at[i] = pos;
      if (e.flags & EF_RAWALT) {  // [raw text][u32 raw length] right before the splice text
        pos = ((pos + e.raw.size() + 3) & ~3ull) + 4;
        maxtext = std::max<uint64_t>(maxtext, e.raw.size());
      }
      toffs[i] = pos;
      pos = ((pos + e.text.size() + 3) & ~3ull) + e.key.size();  // the key follows at key_off_of(toff, len)
      maxtext = std::max<uint64_t>(maxtext, e.text.size());
      if (pos >= 0xFFFFFFF0ull) return fail(IE_ERR_INVALID, "table arena above 4 GiB");
    }
    at[ne] = pos;
  }
  HostArena arena;
  arena.grow(at[ne]);
  std::vector<Entry> items(ne);
  std::vector<uint64_t> hs0(ne);
  const uint64_t seed0 = reuse ? reuse->seed : 0xA0761D6478BD642Full;
  parallel_for(ne, at[ne] + 64 * ne, [&](uint64_t lo, uint64_t hi) {
    uint8_t* const a = arena.data();
    for (uint64_t i = lo; i < hi; i++) {
      const Ent& e = ents[i];
      uint64_t p = at[i];
      if (e.flags & EF_RAWALT) {
        memcpy(a + p, e.raw.data(), e.raw.size());
        const uint64_t q = (p + e.raw.size() + 3) & ~3ull;
        memset(a + p + e.raw.size(), 0, q - p - e.raw.size());
        const uint32_t rl = (uint32_t)e.raw.size();
        memcpy(a + q, &rl, 4);
        p = q + 4;
      }
      memcpy(a + p, e.text.data(), e.text.size());
      const uint64_t ko = (p + e.text.size() + 3) & ~3ull;
      memset(a + p + e.text.size(), 0, ko - p - e.text.size());
      memcpy(a + ko, e.key.data(), e.key.size());
      const uint64_t end = ko + e.key.size();
      memset(a + end, 0, at[i + 1] - end);  // (the pad before the next entry)
      Entry b{};
      b.key_len = (uint32_t)e.key.size();
      b.text_len = (uint32_t)e.text.size();
      b.vid = e.vid;
      b.flags = e.flags | EF_OCCUPIED | (e.tid << kTidShift);
      b.text_off = (uint32_t)toffs[i];
      memcpy(b.key, e.key.data(), std::min<size_t>(e.key.size(), kInlineKey));
      memcpy(b.text, e.text.data(), std::min<size_t>(e.text.size(), kInlineText));
      items[i] = b;
      hs0[i] = key_hash(e.key, seed0, e.tid);
    }
  });
  uint64_t hs_seed = seed0;  // (the seed hs0 was computed under)
  auto rehash = [&](uint64_t sd) {
    if (sd == hs_seed) return;
    parallel_for(ne, 32 * ne, [&](uint64_t lo, uint64_t hi) {
      for (uint64_t i = lo; i < hi; i++) hs0[i] = key_hash(ents[i].key, sd, ents[i].tid);
    });
    hs_seed = sd;
  };
  // perfect-hash placement: about 4 keys per pilot group at load 0.8 (entries 64 B: a 100k-key
  // table is 8 MB of entries and 50 KB of L2-resident pilots). A failed search changes the seed
  // (two keys with one 64-bit hash can never be separated) and then grows the table.
  const uint64_t nk = items.size();
  // (IE_TABLE_MUTABLE: load 0.5 and groups sized for the capacity, about 2 keys each at the build
  // and 4 when the table is full, so that a group can be placed again around new keys)
  const bool mut = (flags & IE_TABLE_MUTABLE) != 0;
  uint64_t m = std::max<uint64_t>(16, mut ? 2 * nk + 16 : nk + nk / 4 + 1);
  const uint32_t nb = reuse ? reuse->nb : (uint32_t)std::max<uint64_t>(1, ((mut ? m : nk) + 3) / 4);
  uint64_t seed = seed0;
  std::vector<uint16_t> pilots;
  std::vector<uint32_t> slot_of;
  // the one-trip table experiment (IE_CUCKOO=1 with a k_resolve built -DIE_CUCKOO): two-choice
  // placement at load 0.4, no pilots; such a table takes no ie_table_set_update
  // (the setting must match the kernels: a pilot-free table under kernels that read pilots would
  // miss every key, so a library built without -DIE_CUCKOO refuses the variable instead)
  static const bool cuckoo = getenv("IE_CUCKOO") && atoi(getenv("IE_CUCKOO")) == 1;
  if (cuckoo != kernels_cuckoo())
    return fail(IE_ERR_INVALID, cuckoo ? "IE_CUCKOO=1 needs a library whose k_resolve was built with -DIE_CUCKOO"
                                       : "this library's k_resolve was built with -DIE_CUCKOO: set IE_CUCKOO=1");
  bool placed = false;
  if (reuse && !cuckoo && reuse->slot_of.size() == items.size()) {
    placed = true;
    seed = reuse->seed;
    m = reuse->m;
    pilots = reuse->pilots;
    slot_of = reuse->slot_of;
  } else if (cuckoo) {
    m = std::max<uint64_t>(16, (5 * nk) / 2 + 16);
    pilots.assign(nb, 0);
    for (int attempt = 0;; attempt++) {
      if (attempt > 64) return fail(IE_ERR_INVALID, "cuckoo placement failed");
      std::vector<uint64_t> hs(items.size());
      for (size_t i = 0; i < items.size(); i++) hs[i] = key_hash(ents[i].key, seed, ents[i].tid);
      std::vector<int64_t> occ(m, -1);
      bool ok = true;
      for (size_t i = 0; i < items.size() && ok; i++) {
        int64_t cur = (int64_t)i;
        uint32_t a, b;
        ck_slots(hs[cur], (uint32_t)m, a, b);
        uint32_t pos = a;
        int kick = 0;
        for (; kick < 1000; kick++) {
          if (occ[pos] < 0) {
            occ[pos] = cur;
            break;
          }
          std::swap(cur, occ[pos]);
          ck_slots(hs[cur], (uint32_t)m, a, b);
          pos = pos == a ? b : a;
        }
        ok = kick < 1000;
      }
      if (ok) {
        slot_of.assign(items.size(), 0);
        for (uint64_t s2 = 0; s2 < m; s2++)
          if (occ[s2] >= 0) slot_of[occ[s2]] = (uint32_t)s2;
        break;
      }
      seed = fmix64_host(seed + 0x9E3779B97F4A7C15ull);
    }
  }
  for (int attempt = 0; !cuckoo && !placed; attempt++) {  // (a failed ph_place leaves slot_of sized: the flag ends the loop)
    if (m > (1ull << 31)) return fail(IE_ERR_INVALID, "table too large");
    rehash(seed);
    if ((placed = ph_place(hs0, m, nb, pilots, slot_of))) break;
    if (attempt & 1) m += m / 4;
    else seed = fmix64_host(seed + 0x9E3779B97F4A7C15ull);
  }
  rehash(seed);  // (the groups below: the hashes under the final seed)
  std::vector<Entry> entries(m);
  for (size_t i = 0; i < items.size(); i++) entries[slot_of[i]] = items[i];
  if (slots_out) *slots_out = slot_of;
  ie_table* t = new ie_table();
  t->groups.assign(nb, {});
  t->clock_slots.assign(2ull * n_tables, UINT32_MAX);
  for (size_t i = 0; i < items.size(); i++) {
    if (items[i].vid == IE_VID_CLOCK_HHMM || items[i].vid == IE_VID_CLOCK_HHMMSS)
      t->clock_slots[2ull * ents[i].tid + (items[i].vid == IE_VID_CLOCK_HHMMSS)] = slot_of[i];
    if (items[i].flags & EF_RAWALT) t->rawalt[ents[i].tid].push_back(slot_of[i]);
    t->groups[ph_group(hs0[i], nb)].push_back(slot_of[i]);
  }
  t->device = device;
  t->dialect = dialect;
  t->flags = flags;
  t->n_entries = ents.size();
  t->n_tables = n_tables;
  auto up = [&](DevBuf& b, const void* src, uint64_t bytes, uint64_t cap) -> hipError_t {
    hipError_t e = b.ensure(cap + 16);
    if (e != hipSuccess) return e;
    return bytes ? hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice) : hipSuccess;
  };
  // the arena keeps room for the texts ie_table_set_update appends (16 pad bytes past the end:
  // dword reads past the last text)
  t->arena_cap = arena.size() + std::max<uint64_t>(arena.size() / 4, 1ull << 16);
  hipError_t e1 = up(t->entries, entries.data(), entries.size() * sizeof(Entry), entries.size() * sizeof(Entry));
  hipError_t e2 = e1 == hipSuccess ? up(t->pilots, pilots.data(), pilots.size() * sizeof(uint16_t), pilots.size() * 2) : e1;
  hipError_t e3 = e2;
  if (e3 == hipSuccess) e3 = t->arena.ensure(t->arena_cap + 16);
  if (e3 == hipSuccess) e3 = hipMemset(t->arena.p, 0, t->arena_cap + 16);
  if (e3 == hipSuccess && !arena.empty()) e3 = hipMemcpy(t->arena.p, arena.data(), arena.size(), hipMemcpyHostToDevice);
  if (e3 != hipSuccess) {
    delete t;
    return fail(IE_ERR_HIP, std::string("table upload: ") + hipGetErrorString(e3));
  }
  t->dev.entries = (const Entry*)t->entries.p;
  t->dev.pilots = (const uint16_t*)t->pilots.p;
  t->dev.arena = (const uint8_t*)t->arena.p;
  t->dev.seed = seed;
  t->dev.nb = nb;
  t->dev.m = (uint32_t)m;
  t->dev.n_entries = (uint32_t)ents.size();
  t->dev.n_tables = n_tables;
  t->dev.dialect = (uint32_t)dialect;
  t->dev.flags = ((flags & IE_TABLE_HAS_INSERTS_DIR) ? TF_HAS_DIR : 0u) | (long_keys ? TF_LONG_KEYS : 0u) |
                 (cuckoo ? TF_CUCKOO : 0u);
  t->dev.maxtext = maxtext;
  t->h_entries = std::move(entries);
  t->h_pilots = std::move(pilots);
  t->arena_live = arena.size();
  t->h_arena = std::move(arena);
  *out = t;
  return IE_SUCCESS;
}

// Pre-resolution of brace-bearing splice texts (device work, at build time).
// The reference re-resolves a spliced value in place (py:516-535: the loop rescans the content).
// When the value V is balanced and carries no '\' or U+3020, splicing V and letting the loop
// continue equals splicing interpolate_inserts(V): rfind('{') always lands inside V until V is
// brace-free (the suffix after a resolved pair holds no '{', and V's pairs close inside V), no
// escape or placeholder can form across V's edges, and V's own errors would surface first.
// So V is resolved once here, on the device through the table itself, as the string "a" + V
// (never the whole-string simple form), and a result that is inert (no '{', '}', '\', U+3020)
// replaces the splice text; lookups that need the raw value (py:512 / interp.rs:48) read it
// from the arena (EF_RAWALT). Values whose resolution fails or stays structural keep the
// literal path, and so do values whose resolution reads the clock (py:433-436 reads it on every
// lookup, also through a nested key: '{{a}}' with a = 'HH:MM', '{HH:{m}}'): they are resolved
// under the build clock and under a second clock that differs in every field, and a value whose
// status or text differs stays raw, so ie_table_set_clock never leaves a stale time behind.
int preresolve(ie_table* t0, std::vector<Ent>& ents, uint32_t n_tables, int32_t dialect, uint32_t flags,
               int32_t device, const ie_clock& clock, ie_table** out, std::vector<uint32_t>& slots) {
  auto clean_value = [](std::string_view v, bool need_brace) {
    size_t opens = 0;
    int64_t depth = 0;
    for (size_t i = 0; i < v.size(); i++) {
      const uint8_t c = (uint8_t)v[i];
      if (c == '\\') return false;
      if (c == 0xE3 && i + 2 < v.size() && (uint8_t)v[i + 1] == 0x80 && (uint8_t)v[i + 2] == 0xA0) return false;
      if (c == '{') opens++, depth++;
      if (c == '}' && --depth < 0) return false;
    }
    return depth == 0 && (!need_brace || (opens > 0 && opens <= 64));
  };
  std::vector<size_t> cand;
  for (size_t i = 0; i < ents.size(); i++) {
    const Ent& e = ents[i];
    if ((e.flags & EF_INERT) || !(e.flags & EF_SPLICE_OK) || e.text.size() > (1u << 16)) continue;
    if (clean_value(e.text, true)) cand.push_back(i);
  }
  if (cand.empty()) return IE_SUCCESS;
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> offs(1, 0);
  std::vector<uint32_t> tids;
  for (size_t i : cand) {
    bytes.push_back('a');
    bytes.insert(bytes.end(), ents[i].text.begin(), ents[i].text.end());
    offs.push_back(bytes.size());
    tids.push_back(ents[i].tid);  // a value resolves against its own table of the set
  }
  // one exec per device kept for these passes (a table set built per map step would otherwise pay
  // an exec's stream and buffers each time); IE_PRE_EXEC_CACHE=0: a fresh exec per build
  static std::mutex mu;
  static ie_exec* kept[64] = {};
  static const bool keep = !(getenv("IE_PRE_EXEC_CACHE") && atoi(getenv("IE_PRE_EXEC_CACHE")) == 0);
  std::unique_lock<std::mutex> lk(mu, std::defer_lock);
  const bool use_kept = keep && device >= 0 && device < 64;
  ie_exec* x = nullptr;
  int rc = IE_SUCCESS;
  if (use_kept) {
    lk.lock();
    if (!kept[device]) rc = ie_exec_create(device, nullptr, &kept[device]);
    x = kept[device];
  } else {
    rc = ie_exec_create(device, nullptr, &x);
  }
  if (rc) return rc;
  ie_batch* b = nullptr;
  ie_batch* b2 = nullptr;
  const ie_clock other{(clock.hour + 12) % 24, (clock.minute + 30) % 60, (clock.second + 30) % 60};
  rc = run_host(x, kOpInterp, t0, bytes.data(), offs.data(), cand.size(), &b, tids.data());
  if (!rc) rc = ie_table_set_clock(t0, &other);
  if (!rc) rc = run_host(x, kOpInterp, t0, bytes.data(), offs.data(), cand.size(), &b2, tids.data());
  if (!rc) rc = ie_table_set_clock(t0, &clock);
  if (!use_kept) ie_exec_destroy(x);
  if (rc) {
    ie_batch_free(b);
    ie_batch_free(b2);
    return rc;
  }
  auto same = [&](uint64_t k) {
    const uint64_t l1 = b->offsets[k + 1] - b->offsets[k], l2 = b2->offsets[k + 1] - b2->offsets[k];
    return b->status[k] == b2->status[k] && l1 == l2 &&
           memcmp(b->bytes + b->offsets[k], b2->bytes + b2->offsets[k], l1) == 0;
  };
  std::vector<std::string> resolved(cand.size());
  size_t changed = 0;
  for (size_t k = 0; k < cand.size(); k++) {
    if (b->status[k] != IE_OK_STR || !same(k)) continue;
    const uint64_t o = b->offsets[k], len = b->offsets[k + 1] - o;
    if (len < 1 || b->bytes[o] != 'a') continue;
    std::string_view r((const char*)b->bytes + o + 1, len - 1);
    bool inert = true;
    for (size_t j = 0; j < r.size() && inert; j++) {
      const uint8_t c = (uint8_t)r[j];
      inert = c != '{' && c != '}' && c != '\\' &&
              !(c == 0xE3 && j + 2 < r.size() && (uint8_t)r[j + 1] == 0x80 && (uint8_t)r[j + 2] == 0xA0);
    }
    if (!inert) continue;
    resolved[k].assign(r);
    Ent& e = ents[cand[k]];
    e.raw = e.text;
    e.text = resolved[k];
    e.flags = (e.flags & ~EF_INERT) | text_flags(e.text) | EF_RAWALT;
    changed++;
  }
  ie_batch_free(b);
  ie_batch_free(b2);
  if (!changed) return IE_SUCCESS;
  // the same keys at the same slots: t0's placement, only the texts and the arena laid out again
  const Placement P{t0->dev.seed, t0->dev.m, t0->dev.nb, t0->h_pilots, std::move(slots)};
  ie_table* t1 = nullptr;
  rc = upload_table(ents, n_tables, dialect, flags, device, &t1, &P);
  if (rc) return rc;
  ie_table_free(t0);
  *out = t1;
  return IE_SUCCESS;
}

int ie_table_set_build(const ie_kv* kv, const uint64_t* kv_start, uint32_t n_tables, int32_t dialect,
                       const ie_clock* now, uint32_t flags, int32_t device, ie_table** out) {
  if (!out || !kv_start || (kv_start[n_tables] && !kv)) return fail(IE_ERR_INVALID, "null argument");
  if (dialect != IE_DIALECT_PY && dialect != IE_DIALECT_RS) return fail(IE_ERR_INVALID, "bad dialect");
  if (n_tables == 0 || n_tables > kMaxTables) return fail(IE_ERR_INVALID, "table count must be in [1, 2^20]");
  for (uint32_t t = 0; t < n_tables; t++)
    if (kv_start[t + 1] < kv_start[t]) return fail(IE_ERR_INVALID, "kv_start must be non-decreasing");
  int rc = set_device(device);
  if (rc) return rc;
  Trace tr("build");
  char hhmm[16], hhmmss[16];
  const int h = now ? now->hour : 0, mi = now ? now->minute : 0, se = now ? now->second : 0;
  snprintf(hhmm, sizeof hhmm, "%02d:%02d", h, mi);
  snprintf(hhmmss, sizeof hhmmss, "%02d:%02d:%02d", h, mi, se);
  // every table's entries (dict semantics per table: the last duplicate wins; '' is never looked up,
  // py:446 / interp.rs:105), tables split over the host threads, then concatenated in table order
  const unsigned T = (unsigned)std::min<uint64_t>(host_threads(), std::max<uint64_t>(1, n_tables / 256));
  std::vector<std::vector<Ent>> part(T);
  std::vector<int> part_rc(T, IE_SUCCESS);
  parallel_for(T, T > 1 ? ~0ull : 0ull, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t k = lo; k < hi; k++) {
      const uint32_t t_lo = (uint32_t)((uint64_t)n_tables * k / T), t_hi = (uint32_t)((uint64_t)n_tables * (k + 1) / T);
      std::vector<Ent>& out = part[k];
      out.reserve(kv_start[t_hi] - kv_start[t_lo] + 2ull * (t_hi - t_lo));
      std::unordered_map<std::string_view, uint64_t> last;
      std::vector<uint64_t> order;
      for (uint32_t tb = t_lo; tb < t_hi && part_rc[k] == IE_SUCCESS; tb++) {
        last.clear();
        order.clear();
        for (uint64_t i = kv_start[tb]; i < kv_start[tb + 1]; i++) {
          std::string_view key(kv[i].key ? kv[i].key : "", kv[i].key_len);
          if (key.empty()) continue;
          auto it = last.find(key);
          if (it == last.end()) {
            last.emplace(key, i);
            order.push_back(i);
          } else {
            it->second = i;
          }
        }
        for (uint64_t i : order) {
          std::string_view key(kv[i].key, kv[i].key_len);
          const uint64_t j = last[key];
          if (key == "HH:MM" || key == "HH:MM:SS") continue;  // py:433-436: the clock always wins
          if (kv[j].kind < 0 || kv[j].kind > IE_KIND_DICT) {
            part_rc[k] = IE_ERR_INVALID;  // (bad kind)
            break;
          }
          if (j >= IE_VID_CLOCK_HHMMSS) {
            part_rc[k] = IE_ERR_CAPACITY;  // (more inserts than value ids)
            break;
          }
          std::string_view tx(kv[j].text ? kv[j].text : "", kv[j].text_len);
          out.push_back(Ent{key, tx, kind_flags(kv[j].kind, dialect) | text_flags(tx), (uint32_t)j, tb, {}});
        }
        out.push_back(Ent{"HH:MM", hhmm, kind_flags(IE_KIND_STR, dialect) | text_flags(hhmm), IE_VID_CLOCK_HHMM, tb, {}});
        out.push_back(Ent{"HH:MM:SS", hhmmss, kind_flags(IE_KIND_STR, dialect) | text_flags(hhmmss), IE_VID_CLOCK_HHMMSS,
                          tb, {}});
      }
    }
  });
  for (unsigned k = 0; k < T; k++) {
    if (part_rc[k] == IE_ERR_INVALID) return fail(IE_ERR_INVALID, "bad kind");
    if (part_rc[k] != IE_SUCCESS) return fail(IE_ERR_INVALID, "more inserts than value ids");
  }
  std::vector<Ent> ents;
  {
    uint64_t total = 0;
    for (const auto& v : part) total += v.size();
    ents.reserve(total);
    for (auto& v : part) std::move(v.begin(), v.end(), std::back_inserter(ents));
  }
  tr.mark("entries", ents.size());
  ie_table* t0 = nullptr;
  std::vector<uint32_t> slots;
  rc = upload_table(ents, n_tables, dialect, flags, device, &t0, nullptr, &slots);
  tr.mark("upload", ents.size());
  if (rc || getenv("IE_NO_PRERESOLVE")) {  // diagnostic switch: raw splice texts only
    *out = t0;
    if (t0) t0->next_vid = (uint32_t)std::min<uint64_t>(kv_start[n_tables], IE_VID_CLOCK_HHMMSS);
    return rc;
  }
  *out = t0;
  const ie_clock clk{h, mi, se};
  rc = preresolve(t0, ents, n_tables, dialect, flags, device, clk, out, slots);
  tr.mark("pre-resolve", ents.size());
  if (rc) {
    ie_table_free(*out);
    *out = nullptr;
    return rc;
  }
  (*out)->next_vid = (uint32_t)std::min<uint64_t>(kv_start[n_tables], IE_VID_CLOCK_HHMMSS);  // (a kv's index is its id)
  return rc;
}

int ie_table_build(const ie_kv* kv, uint64_t n, int32_t dialect, const ie_clock* now,
                   uint32_t flags, int32_t device, ie_table** out) {
  if (!out || (n && !kv)) return fail(IE_ERR_INVALID, "null argument");
  const uint64_t start[2] = {0, n};
  return ie_table_set_build(kv, start, 1, dialect, now, flags, device, out);
}

// a copy of a built table on another device (or the same one): device-to-device copies of the
// entries, pilots and arena (hipMemcpyPeer: over xGMI between MI355X GPUs), no host placement or
// pre-resolution pass (the table is read-only and replicated per device)
int ie_table_replicate(const ie_table* t, int32_t device, ie_table** out) {
  if (!t || !out) return fail(IE_ERR_INVALID, "null argument");
  *out = nullptr;
  int rc = set_device(device);
  if (rc) return rc;
  ie_table* c = new ie_table();
  c->device = device;
  c->dialect = t->dialect;
  c->flags = t->flags;
  c->n_entries = t->n_entries;
  c->n_tables = t->n_tables;
  c->clock_slots = t->clock_slots;
  c->h_entries = t->h_entries;
  c->h_pilots = t->h_pilots;
  c->h_arena = t->h_arena;
  c->arena_cap = t->arena_cap;
  c->arena_live = t->arena_live;
  c->arena_limit = t->arena_limit;
  c->n_compactions = t->n_compactions;
  c->next_vid = t->next_vid;
  c->free_vids = t->free_vids;
  c->groups = t->groups;
  c->rawalt = t->rawalt;
  c->dev = t->dev;
  auto copy = [&](DevBuf& dst, const DevBuf& src) -> hipError_t {
    hipError_t e = dst.ensure(src.bytes);
    if (e != hipSuccess || !src.bytes) return e;
    return hipMemcpyPeer(dst.p, device, src.p, t->device, src.bytes);
  };
  hipError_t e = copy(c->entries, t->entries);
  if (e == hipSuccess) e = copy(c->pilots, t->pilots);
  if (e == hipSuccess) e = copy(c->arena, t->arena);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    delete c;
    return fail(IE_ERR_HIP, std::string("table replicate: ") + hipGetErrorString(e));
  }
  c->dev.entries = (const Entry*)c->entries.p;
  c->dev.pilots = (const uint16_t*)c->pilots.p;
  c->dev.arena = (const uint8_t*)c->arena.p;
  *out = c;
  return IE_SUCCESS;
}

// byte-balanced shards of a packed batch: shard k = strings [first[k], first[k+1]),
// first[k] = the first string whose offset reaches k/n_shards of the payload (binary search)
int ie_shard_bounds(const uint64_t* offsets, uint64_t n, uint32_t n_shards, uint64_t* first) {
  if (!offsets || !first || n_shards == 0) return fail(IE_ERR_INVALID, "null argument");
  const uint64_t lo = offsets[0], total = offsets[n] - lo;
  first[0] = 0;
  for (uint32_t k = 1; k < n_shards; k++) {
    const uint64_t target = lo + (uint64_t)((unsigned __int128)total * k / n_shards);
    first[k] = (uint64_t)(std::lower_bound(offsets, offsets + n, target) - offsets);
    if (first[k] < first[k - 1]) first[k] = first[k - 1];
  }
  first[n_shards] = n;
  return IE_SUCCESS;
}

void ie_table_free(ie_table* t) {
  if (t) {
    (void)hipSetDevice(t->device);
    delete t;
  }
}
int ie_table_set_clock(ie_table* t, const ie_clock* now) {
  if (!t || !now) return fail(IE_ERR_INVALID, "null argument");
  int rc = set_device(t->device);
  if (rc) return rc;
  // no batch may still read the table (exec streams are non-blocking: not ordered with these copies)
  IE_HIP(hipDeviceSynchronize());
  char hhmm[16], hhmmss[16];
  snprintf(hhmm, sizeof hhmm, "%02d:%02d", now->hour, now->minute);
  snprintf(hhmmss, sizeof hhmmss, "%02d:%02d:%02d", now->hour, now->minute, now->second);
  Patches pe;  // every table's two clock entries and their arena texts: one upload
  for (uint32_t slot : t->clock_slots) {
    if (slot == UINT32_MAX) continue;
    Entry& e = t->h_entries[slot];
    const char* txt = e.vid == IE_VID_CLOCK_HHMM ? hhmm : hhmmss;
    if (strlen(txt) != e.text_len) return fail(IE_ERR_INVALID, "clock field out of range");
    memcpy(e.text, txt, e.text_len);
    memcpy(t->h_arena.data() + e.text_off, txt, e.text_len);
    pe.add((Entry*)t->entries.p + slot, &e, sizeof(Entry));
    pe.add((uint8_t*)t->arena.p + e.text_off, txt, e.text_len);
  }
  return apply_patches(t, pe);
}

// set_interpdata on a built table (set): py:470-471 `inserts[key] = value` (and `del`) on state
// table_id[i], without a rebuild. A key already in that table is rewritten in place (its slot is
// fixed by the perfect hash); a new key re-places its pilot group (a few keys) around it, or, when
// the group finds no pilot, the whole table is placed again under a new seed at the same capacity
// (replace_all); only when that fails too IE_ERR_CAPACITY is reported and nothing of that key is
// applied (the caller rebuilds). Values are taken as given: a brace-bearing value is not pre-resolved (the
// exact evaluator resolves it in the reference's order), and the pre-resolved values of every
// table that changed go back to their raw text, since they were resolved against the old dict.
// a set of entry slots (bitmap): marked in any order, listed in slot order without a sort
struct SlotSet {
  std::vector<uint64_t> w;
  explicit SlotSet(uint32_t m) : w((m + 63) / 64, 0) {}
  void set(uint32_t s) { w[s >> 6] |= 1ull << (s & 63); }
  void set_atomic(uint32_t s) { __atomic_fetch_or(&w[s >> 6], 1ull << (s & 63), __ATOMIC_RELAXED); }
  void clear(uint32_t s) { w[s >> 6] &= ~(1ull << (s & 63)); }
  bool has(uint32_t s) const { return (w[s >> 6] >> (s & 63)) & 1; }
  uint64_t count() const {
    uint64_t c = 0;
    for (uint64_t x : w) c += (uint64_t)__builtin_popcountll(x);
    return c;
  }
  std::vector<uint32_t> slots() const {
    std::vector<uint32_t> out;
    for (size_t k = 0; k < w.size(); k++)
      for (uint64_t x = w[k]; x; x &= x - 1) out.push_back((uint32_t)(k * 64 + __builtin_ctzll(x)));
    return out;
  }
};

// ie_table_set_update (value ids given: vid_in) and ie_table_set_store (value ids handed out by the
// table: a rewrite keeps its key's id, a new key takes a freed id or the next one, a delete frees
// its key's id; vid_out[i] = the id, IE_VID_NONE for a key never stored)
static int table_update(ie_table* t, const ie_kv* kv, const uint32_t* table_id, const uint32_t* vid_in,
                        uint32_t* vid_out, uint64_t n) {
  const bool autov = vid_in == nullptr;
  if (!t || (n && (!kv || !table_id || (autov && !vid_out)))) return fail(IE_ERR_INVALID, "null argument");
  const uint32_t* const vid = vid_in;
  // every change is checked before any is applied: a rejected call leaves the table as it was
  for (uint64_t i = 0; i < n; i++) {
    if (table_id[i] >= t->n_tables) return fail(IE_ERR_INVALID, "table id beyond the table set");
    if (kv[i].key_len && !kv[i].key) return fail(IE_ERR_INVALID, "null key");
    if (kv[i].kind < 0) continue;
    if (kv[i].kind > IE_KIND_DICT) return fail(IE_ERR_INVALID, "bad kind");
    if (!autov && vid[i] >= IE_VID_CLOCK_HHMMSS) return fail(IE_ERR_INVALID, "value id out of range");
    if (kv[i].text_len && !kv[i].text) return fail(IE_ERR_INVALID, "null text");
    if (kv[i].key_len >= 0xFFFFFFF0ull || kv[i].text_len >= 0xFFFFFFF0ull) return fail(IE_ERR_INVALID, "key or text above 4 GiB");
  }
  if (t->dev.flags & TF_CUCKOO) return fail(IE_ERR_INVALID, "a two-choice (IE_CUCKOO) table takes no updates");
  Trace tr("update");
  int rc = set_device(t->device);
  if (rc) return rc;
  IE_HIP(hipDeviceSynchronize());  // no batch may still read the table
  tr.mark("sync", n);
  if (!t->occ_ok) {
    t->occ.assign((t->h_entries.size() + 63) / 64, 0);
    for (size_t s2 = 0; s2 < t->h_entries.size(); s2++)
      if (t->h_entries[s2].flags & EF_OCCUPIED) t->occ[s2 >> 6] |= 1ull << (s2 & 63);
    t->occ_ok = true;
  }
  auto occupy = [t](uint32_t s2, bool on) {
    if (on) t->occ[s2 >> 6] |= 1ull << (s2 & 63);
    else t->occ[s2 >> 6] &= ~(1ull << (s2 & 63));
  };
  uint64_t arena0 = t->h_arena.size();
  uint64_t seed = t->dev.seed;
  const uint32_t nb = t->dev.nb, m = t->dev.m;
  bool whole = false;                      // entries and pilots re-placed: upload them whole
  bool whole_arena = false;                // the arena was compacted: upload it whole
  SlotSet dirty(m);                        // entry slots to upload
  std::vector<uint32_t> dirty_groups;      // pilots to upload
  SlotSet rewritten(m);                    // slots whose arena bytes were rewritten in place
  std::vector<uint32_t> touched;           // tables whose pre-resolved values must go raw
  int status = IE_SUCCESS;
  uint64_t call_start = t->h_arena.size();  // (the texts placed since: maybe not copied yet)
  uint64_t n_tries = 0, n_replace_all = 0;  // (IE_HOST_TRACE)
  // room for an append of `need` bytes below the table's arena limit (offsets stay below 2^32):
  // compacted first when dead bytes would make the room; false: IE_ERR_CAPACITY
  auto room = [&](uint64_t need) -> bool {
    if (t->h_arena.size() + need + 8 <= t->arena_limit) return true;
    if (t->arena_live + need + 8 > t->arena_limit) return false;
    compact_arena(t);  // (flushes the deferred copies first)
    call_start = t->h_arena.size();
    whole = whole_arena = true;
    return t->h_arena.size() + need + 8 <= t->arena_limit;
  };
  // the texts' inert flags and the keys' hashes (under the current seed), across the host threads
  // before the (serial) placement
  std::vector<uint32_t> tflags(n, 0);
  std::vector<uint64_t> khash(n);
  const uint64_t seed0 = seed;
  uint64_t in_bytes = 0;
  for (uint64_t i = 0; i < n; i++) in_bytes += kv[i].key_len + (kv[i].kind >= 0 ? kv[i].text_len : 0) + 16;
  parallel_for(n, in_bytes, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; i++) {
      if (kv[i].kind >= 0) tflags[i] = text_flags(std::string_view(kv[i].text ? kv[i].text : "", kv[i].text_len));
      khash[i] = key_hash(std::string_view(kv[i].key ? kv[i].key : "", kv[i].key_len), seed0, table_id[i]);
    }
  });
  tr.mark("flags, hashes", n);
  // long texts are placed now and copied later, in parallel (flush_copies: before a compaction, a
  // rewrite of a text placed in this call, and the upload)
  std::vector<CopyJob> jobs;
  struct DeferScope {
    ie_table* t;
    ~DeferScope() { t->defer = nullptr; }
  } defer_scope{t};
  t->defer = &jobs;
  {  // room for the appends ahead in one reallocation (not a doubling copy in the middle of them)
    uint64_t est = 0;
    for (uint64_t i = 0; i < n; i++)
      if (kv[i].kind >= 0) est += kv[i].text_len + kv[i].key_len + 8;
    const uint64_t sz = t->h_arena.size();
    if (t->h_arena.capacity() < sz + est)
      t->h_arena.reserve(std::min<uint64_t>(std::max<uint64_t>(sz + est, sz + sz / 2), t->arena_limit + 64));
  }
  // (an applied store's id: reported, and taken from the free list or the counter)
  auto take = [&](uint64_t i, uint32_t v, bool kept) {
    if (!autov) return;
    vid_out[i] = v;
    if (kept) return;
    if (!t->free_vids.empty() && t->free_vids.back() == v) t->free_vids.pop_back();
    else if (v == t->next_vid) t->next_vid++;
  };
  if (autov)
    for (uint64_t i = 0; i < n; i++) vid_out[i] = IE_VID_NONE;
  else
    for (uint64_t i = 0; i < n; i++)
      if (kv[i].kind >= 0) t->next_vid = std::max(t->next_vid, vid[i] + 1);
  // A large call that only rewrites keys the tables have (a loop iteration's stores): the changes
  // split by table over the host threads (a key's changes stay in order on one thread), each thread
  // rewriting its entries in place or appending into an arena region of its own; anything else (a
  // new key, a delete, a pre-resolved entry) takes the serial placement below.
  bool parallel_done = false;
  if (n >= 4096 && host_threads() > 1) {
    std::vector<uint32_t> slot_of(n, UINT32_MAX);
    std::atomic<bool> all_present{true};
    parallel_for(n, in_bytes, [&](uint64_t lo, uint64_t hi) {
      for (uint64_t i = lo; i < hi && all_present.load(std::memory_order_relaxed); i++) {
        const std::string_view key(kv[i].key ? kv[i].key : "", kv[i].key_len);
        if (key.empty() || key == "HH:MM" || key == "HH:MM:SS") continue;
        const uint64_t h = khash[i];
        const uint32_t slot = ph_slot(h, t->h_pilots[ph_group(h, nb)], m);
        const Entry& e = t->h_entries[slot];
        if (kv[i].kind < 0 || !(e.flags & EF_OCCUPIED) || (e.flags >> kTidShift) != table_id[i] ||
            (e.flags & EF_RAWALT) || mirror_key(t, e) != key) {
          all_present.store(false, std::memory_order_relaxed);
          break;
        }
        slot_of[i] = slot;
      }
    });
    tr.mark("(pre-pass)", n);
    const unsigned T = host_threads();
    std::vector<std::vector<uint64_t>> mine(T);
    std::vector<uint64_t> region(T + 1, 0);
    if (all_present.load()) {
      for (uint64_t i = 0; i < n; i++) {
        if (slot_of[i] == UINT32_MAX) continue;
        const unsigned k = table_id[i] % T;
        mine[k].push_back(i);
        region[k + 1] += ((kv[i].text_len + 3ull) & ~3ull) + ((kv[i].key_len + 3ull) & ~3ull);
      }
      for (unsigned k = 0; k < T; k++) region[k + 1] += region[k];
    }
    const uint64_t start = (t->h_arena.size() + 3ull) & ~3ull;
    if (all_present.load() && start + region[T] + 8 <= t->arena_limit) {
      tr.mark("(lists)", T);
      while (t->h_arena.size() & 3) t->h_arena.push_back(0);
      t->h_arena.grow(region[T]);
      tr.mark("(grown)", region[T]);
      uint8_t* const base = t->h_arena.data();
      std::vector<int64_t> live_delta(T, 0);
      std::vector<uint64_t> maxtext(T, 0);
      std::vector<std::vector<uint32_t>> touched_k(T);
      parallel_for(T, ~0ull, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t k = lo; k < hi; k++) {
          uint64_t cursor = start + region[k];
          int64_t dl = 0;
          uint64_t mt = 0;
          std::vector<uint32_t> tk;  // (thread-local: the per-thread slots of shared vectors would share lines)
          tk.reserve(mine[k].size());
          for (uint64_t i : mine[k]) {
            const uint32_t slot = slot_of[i], tb = table_id[i];
            Entry& e = t->h_entries[slot];
            const std::string_view key(kv[i].key, kv[i].key_len);
            const std::string_view text(kv[i].text ? kv[i].text : "", kv[i].text_len);
            const uint32_t flags = kind_flags(kv[i].kind, t->dialect) | tflags[i];
            const uint32_t v = autov ? e.vid : vid[i];
            const uint64_t a = e.text_off, b = (key_off_of(e.text_off, e.text_len) + e.key_len + 3ull) & ~3ull;
            if (((text.size() + 3ull) & ~3ull) <= ((e.text_len + 3ull) & ~3ull)) {  // in place
              memset(base + a, 0, b - a);
              memcpy(base + a, text.data(), text.size());
              const uint32_t ko = key_off_of(e.text_off, (uint32_t)text.size());
              memcpy(base + ko, key.data(), key.size());
              dl -= (int64_t)(b - a) - (int64_t)((((uint64_t)ko + key.size() + 3ull) & ~3ull) - a);
              e.text_len = (uint32_t)text.size();
              e.vid = v;
              e.flags = flags | EF_OCCUPIED | (e.flags & ~((1u << kTidShift) - 1u));
              memset(e.text, 0, kInlineText);
              memcpy(e.text, text.data(), std::min<size_t>(text.size(), kInlineText));
              rewritten.set_atomic(slot);
            } else {  // appended in this thread's region: [text][pad][key][pad]
              dl -= (int64_t)(b - a);
              const uint64_t off = cursor;
              memcpy(base + off, text.data(), text.size());
              memset(base + off + text.size(), 0, ((text.size() + 3ull) & ~3ull) - text.size());
              const uint32_t ko = key_off_of((uint32_t)off, (uint32_t)text.size());
              memcpy(base + ko, key.data(), key.size());
              cursor = ((uint64_t)ko + key.size() + 3ull) & ~3ull;
              memset(base + ko + key.size(), 0, cursor - ko - key.size());
              dl += (int64_t)(cursor - off);
              Entry nb{};
              nb.key_len = (uint32_t)key.size();
              nb.text_len = (uint32_t)text.size();
              nb.vid = v;
              nb.flags = flags | EF_OCCUPIED | (tb << kTidShift);
              nb.text_off = (uint32_t)off;
              memcpy(nb.key, key.data(), std::min<size_t>(key.size(), kInlineKey));
              memcpy(nb.text, text.data(), std::min<size_t>(text.size(), kInlineText));
              e = nb;
            }
            dirty.set_atomic(slot);
            tk.push_back(tb);
            mt = std::max<uint64_t>(mt, text.size());
            if (autov) vid_out[i] = v;
          }
          memset(base + cursor, 0, start + region[k + 1] - cursor);  // (the region's unused tail: dead)
          live_delta[k] = dl;
          maxtext[k] = mt;
          touched_k[k] = std::move(tk);
        }
      });
      tr.mark("(placed)", region[T]);
      for (unsigned k = 0; k < T; k++) {
        t->arena_live = (uint64_t)((int64_t)t->arena_live + live_delta[k]);
        t->dev.maxtext = std::max<uint64_t>(t->dev.maxtext, maxtext[k]);
        touched.insert(touched.end(), touched_k[k].begin(), touched_k[k].end());
      }
      parallel_done = true;
      tr.mark("parallel rewrites", n);
    }
  }
  for (uint64_t i = 0; i < n && !parallel_done; i++) {
    const uint32_t tb = table_id[i];
    std::string_view key(kv[i].key ? kv[i].key : "", kv[i].key_len);
    if (key.empty() || key == "HH:MM" || key == "HH:MM:SS") continue;  // never looked up (py:433-446)
    // (the pilot a few changes ahead and the entry one step nearer pulled into the cache: the
    // mirror's entries are tens of MB and every change lands somewhere else in them)
    if (seed == seed0) {
      if (i + 16 < n) __builtin_prefetch(&t->h_pilots[ph_group(khash[i + 16], nb)]);
      if (i + 8 < n) {
        const uint64_t h8 = khash[i + 8];
        __builtin_prefetch(&t->h_entries[ph_slot(h8, t->h_pilots[ph_group(h8, nb)], m)]);
      }
      if (i + 4 < n) {  // (and the text a rewrite in place will overwrite)
        const uint64_t h4 = khash[i + 4];
        const Entry& e4 = t->h_entries[ph_slot(h4, t->h_pilots[ph_group(h4, nb)], m)];
        if (e4.text_off < t->h_arena.size()) __builtin_prefetch(t->h_arena.data() + e4.text_off, 1);
      }
    }
    const uint64_t h = seed == seed0 ? khash[i] : key_hash(key, seed, tb);
    const uint32_t g = ph_group(h, nb), slot = ph_slot(h, t->h_pilots[g], m);
    Entry& cur = t->h_entries[slot];
    const bool present = (cur.flags & EF_OCCUPIED) && (cur.flags >> kTidShift) == tb && mirror_key(t, cur) == key;
    // the change's value id
    uint32_t v = 0;
    if (!autov) {
      v = vid[i];
    } else if (kv[i].kind >= 0 && present) {
      v = cur.vid;
    } else if (kv[i].kind >= 0) {
      if (!t->free_vids.empty()) {
        v = t->free_vids.back();
      } else if (t->next_vid >= IE_VID_CLOCK_HHMMSS) {
        status = fail(IE_ERR_CAPACITY, "value ids exhausted: rebuild the table");
        break;
      } else {
        v = t->next_vid;
      }
    }
    if (kv[i].kind < 0) {  // del inserts[key]
      if (!present) continue;
      if (autov) {
        t->free_vids.push_back(cur.vid);
        vid_out[i] = cur.vid;
      }
      auto& gs = t->groups[g];
      gs.erase(std::remove(gs.begin(), gs.end(), slot), gs.end());
      arena_release(t, cur);
      cur = Entry{};
      occupy(slot, false);
      dirty.set(slot);
      t->n_entries--;
      touched.push_back(tb);
      continue;
    }
    std::string_view text(kv[i].text ? kv[i].text : "", kv[i].text_len);
    const uint32_t flags = kind_flags(kv[i].kind, t->dialect) | tflags[i];
    if (present && cur.text_off >= call_start && !jobs.empty()) flush_copies(t);  // (placed in this call)
    const uint64_t need = ((text.size() + 3ull) & ~3ull) + key.size() + 4;
    if (present) {
      // the new text where the old one was when it fits, else appended
      if (rewrite_in_place(t, cur, text, flags, v)) {
        rewritten.set(slot);
      } else {
        if (!room(need)) {
          status = fail(IE_ERR_CAPACITY, "table arena full (limit reached even after compaction): rebuild the table");
          break;
        }
        arena_release(t, t->h_entries[slot]);
        t->h_entries[slot] = make_entry(t, key, text, flags, v, tb);
      }
      dirty.set(slot);
      touched.push_back(tb);
    } else {
      if (!room(need)) {
        status = fail(IE_ERR_CAPACITY, "table arena full (limit reached even after compaction): rebuild the table");
        break;
      }
      touched.push_back(tb);
      // re-place the group with the new key: a pilot that sends every member to a distinct slot
      // that is free or one of the group's own
      std::vector<uint32_t>& gs = t->groups[g];
      std::vector<uint64_t> hs;
      for (uint32_t s2 : gs) {
        const Entry& e = t->h_entries[s2];
        hs.push_back(key_hash(mirror_key(t, e), seed, e.flags >> kTidShift));
      }
      hs.push_back(h);
      std::vector<uint32_t> cand(hs.size());
      bool found = false;
      uint32_t pilot = 0;
      for (uint32_t p = 0; p < 65536 && !found; p++) {
        n_tries++;
        bool ok = true;
        for (size_t k = 0; k < hs.size() && ok; k++) {
          const uint32_t c = ph_slot(hs[k], p, m);
          ok = !((t->occ[c >> 6] >> (c & 63)) & 1) || std::find(gs.begin(), gs.end(), c) != gs.end();
          for (size_t j = 0; j < k && ok; j++) ok = cand[j] != c;
          cand[k] = c;
        }
        if (ok) found = true, pilot = p;
      }
      if (!found) {
        // every entry placed again under a new seed, at the same capacity
        const Entry extra = make_entry(t, key, text, flags, v, tb);
        n_replace_all++;
        if (!replace_all(t, extra)) {
          arena_release(t, extra);
          status = fail(IE_ERR_CAPACITY, "no free placement for a new key: rebuild the table with more room");
          break;  // apply (upload) what came before, stop here
        }
        seed = t->dev.seed;
        whole = whole_arena = true;  // (the slots rewritten in place so far moved with the rest)
        std::fill(t->occ.begin(), t->occ.end(), 0ull);
        for (size_t s2 = 0; s2 < t->h_entries.size(); s2++)
          if (t->h_entries[s2].flags & EF_OCCUPIED) occupy((uint32_t)s2, true);
        {
          std::lock_guard<std::mutex> lock(t->vid_mu);
          t->vid_ok = false;
        }
        t->n_entries++;
        if (key.size() > kInlineKey && key.size() <= 2 * kInlineKey) t->dev.flags |= TF_LONG_KEYS;
        t->dev.maxtext = std::max<uint64_t>(t->dev.maxtext, text.size());
        take(i, v, false);
        continue;
      }
      // the group's members move together: one from -> to map, applied once to the slot lists (a
      // member may move into the old slot of another, so remapping member by member could move an
      // already remapped slot again)
      std::unordered_map<uint32_t, uint32_t> moved_to;
      std::vector<Entry> moved;
      for (uint32_t s2 : gs) moved.push_back(t->h_entries[s2]);
      for (uint32_t s2 : gs) {
        t->h_entries[s2] = Entry{};
        occupy(s2, false);
        dirty.set(s2);
      }
      for (size_t k = 0; k < moved.size(); k++) {
        const uint32_t from = gs[k], to = cand[k];
        t->h_entries[to] = moved[k];
        occupy(to, true);
        dirty.set(to);
        if (from != to) moved_to[from] = to;
      }
      if (!moved_to.empty()) {
        for (size_t k = 0; k < moved.size(); k++)  // (a clock entry's place in clock_slots: 2 * table + which)
          if (moved[k].vid == IE_VID_CLOCK_HHMM || moved[k].vid == IE_VID_CLOCK_HHMMSS)
            t->clock_slots[2ull * (moved[k].flags >> kTidShift) + (moved[k].vid == IE_VID_CLOCK_HHMMSS)] = cand[k];
        std::vector<uint32_t> tabs;  // the tables whose pre-resolved entries moved
        for (const Entry& e : moved)
          if (e.flags & EF_RAWALT) tabs.push_back(e.flags >> kTidShift);
        std::sort(tabs.begin(), tabs.end());
        tabs.erase(std::unique(tabs.begin(), tabs.end()), tabs.end());
        for (uint32_t tt : tabs) {
          auto it = t->rawalt.find(tt);
          if (it == t->rawalt.end()) continue;
          for (uint32_t& rs : it->second) {
            auto jt = moved_to.find(rs);
            if (jt != moved_to.end()) rs = jt->second;
          }
        }
        std::vector<uint32_t> rw;  // (all cleared first, then set at their new slots: see above)
        for (const auto& ft : moved_to)
          if (rewritten.has(ft.first)) rw.push_back(ft.second), rewritten.clear(ft.first);
        for (uint32_t to : rw) rewritten.set(to);
      }
      t->h_entries[cand.back()] = make_entry(t, key, text, flags, v, tb);
      occupy(cand.back(), true);
      dirty.set(cand.back());
      gs.assign(cand.begin(), cand.end());
      t->h_pilots[g] = (uint16_t)pilot;
      dirty_groups.push_back(g);
      t->n_entries++;
    }
    if (key.size() > kInlineKey && key.size() <= 2 * kInlineKey) t->dev.flags |= TF_LONG_KEYS;
    t->dev.maxtext = std::max<uint64_t>(t->dev.maxtext, text.size());
    take(i, v, present);
  }
  tr.mark("apply", n);
  tr.mark("(pilot tries)", n_tries);
  tr.mark("(re-placements)", n_replace_all);
  flush_copies(t);
  t->defer = nullptr;  // (the pre-resolved values below copy out of temporaries: no deferral)
  tr.mark("copies", t->h_arena.size() - call_start);
  // values pre-resolved against the old dict of a changed table: back to their raw text
  if (t->rawalt.empty()) {
    touched.clear();  // (no table holds a pre-resolved value any more: nothing to return to raw)
  } else {
    std::sort(touched.begin(), touched.end());
    touched.erase(std::unique(touched.begin(), touched.end()), touched.end());
  }
  for (uint32_t tb : touched) {
    auto it = t->rawalt.find(tb);
    if (it == t->rawalt.end()) continue;
    for (uint32_t s2 : it->second) {
      Entry& e = t->h_entries[s2];
      if (!(e.flags & EF_RAWALT)) continue;
      const uint8_t* a = t->h_arena.data();
      uint32_t rl;
      memcpy(&rl, a + e.text_off - 4, 4);
      const uint32_t roff = e.text_off - 4 - ((rl + 3u) & ~3u);
      const std::string raw((const char*)a + roff, rl), key(mirror_key(t, e));
      const uint32_t kflags = e.flags & (EF_KIND_MASK | EF_SPLICE_OK | EF_KEY_STR | EF_KEY_UNHASHABLE);
      if (!room(((raw.size() + 3ull) & ~3ull) + key.size() + 4)) {
        status = fail(IE_ERR_CAPACITY, "table arena full (limit reached even after compaction): rebuild the table");
        continue;
      }
      arena_release(t, e);
      e = make_entry(t, key, raw, kflags | text_flags(raw), e.vid, tb);
      t->dev.maxtext = std::max<uint64_t>(t->dev.maxtext, raw.size());
      dirty.set(s2);
    }
    t->rawalt.erase(it);
  }
  tr.mark("rawalt", touched.size());
  // dead bytes beyond the live ones (and beyond 64 KB): compact (one whole upload)
  const uint64_t dead = t->h_arena.size() - std::min<uint64_t>(t->h_arena.size(), t->arena_live);
  if (dead > t->arena_live && dead > (64u << 10)) {
    compact_arena(t);
    whole = whole_arena = true;
  }
  tr.mark("compact?", t->h_arena.size());
  // upload: the appended arena bytes, the changed entries, the changed pilots
  const bool grown = t->h_arena.size() > t->arena_cap;
  if (grown || whole_arena) {  // (re)allocate when grown; the whole mirror goes up
    if (grown) {
      DevBuf na;
      // (twice the mirror: a store loop appending tens of MB per call reallocates rarely)
      const uint64_t cap = std::min<uint64_t>(t->arena_limit, t->h_arena.size() + std::max<uint64_t>(t->h_arena.size(), 1ull << 16));
      IE_HIP(na.ensure(cap + 16));
      t->arena.release();
      t->arena = na;
      na.p = nullptr;
      t->arena_cap = cap;
      t->dev.arena = (const uint8_t*)t->arena.p;
    }
    IE_HIP(hipMemcpy(t->arena.p, t->h_arena.data(), t->h_arena.size(), hipMemcpyHostToDevice));
    IE_HIP(hipMemset((uint8_t*)t->arena.p + t->h_arena.size(), 0, t->arena_cap + 16 - t->h_arena.size()));
    arena0 = t->h_arena.size();
    tr.mark("arena upload", arena0);
  }
  // the appended texts in one copy; one upload and one kernel for the texts rewritten in place, the
  // changed entries and pilots (the whole entry array in one copy when many changed)
  Patches pe;
  if (t->h_arena.size() > arena0) {  // the appended texts: one contiguous copy
    IE_HIP(hipMemcpy((uint8_t*)t->arena.p + arena0, t->h_arena.data() + arena0, t->h_arena.size() - arena0,
                     hipMemcpyHostToDevice));
    tr.mark("tail upload", t->h_arena.size() - arena0);
  }
  {
    const uint64_t nd = dirty.count();
    pe.reserve(nd + dirty_groups.size() + 16, nd * sizeof(Entry));
  }
  if (!whole_arena) {
    const std::vector<uint32_t> rs = rewritten.slots();
    std::vector<CopyJob> rr(rs.size());
    parallel_for(rs.size(), rs.size() * 256, [&](uint64_t lo, uint64_t hi) {
      for (uint64_t k = lo; k < hi; k++) {
        const Entry& e = t->h_entries[rs[k]];
        rr[k] = CopyJob{0, nullptr, 0};
        if (!(e.flags & EF_OCCUPIED)) continue;
        uint64_t a, b2;
        arena_span(t, e, a, b2);
        if (a >= arena0) continue;  // inside the appended tail, sent whole above
        b2 = std::min<uint64_t>(b2, arena0);
        rr[k] = CopyJob{(uint64_t)(uintptr_t)((uint8_t*)t->arena.p + a), t->h_arena.data() + a, b2 - a};
      }
    });
    pe.add_many(rr);
  }
  // (the whole entry array in one copy when that is cheaper than a patch per entry: a copy moves
  // ~20 GB/s, a patch costs ~100 ns of host work)
  if (whole || dirty.count() * 32 > t->h_entries.size()) {
    IE_HIP(hipMemcpy(t->entries.p, t->h_entries.data(), t->h_entries.size() * sizeof(Entry), hipMemcpyHostToDevice));
  } else {
    const std::vector<uint32_t> ds = dirty.slots();
    std::vector<CopyJob> er(ds.size());
    for (size_t k = 0; k < ds.size(); k++)
      er[k] = CopyJob{(uint64_t)(uintptr_t)((Entry*)t->entries.p + ds[k]), (const uint8_t*)&t->h_entries[ds[k]],
                      sizeof(Entry)};
    pe.add_many(er);
  }
  if (whole) {
    IE_HIP(hipMemcpy(t->pilots.p, t->h_pilots.data(), t->h_pilots.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
  } else {
    std::sort(dirty_groups.begin(), dirty_groups.end());
    dirty_groups.erase(std::unique(dirty_groups.begin(), dirty_groups.end()), dirty_groups.end());
    for (uint32_t g : dirty_groups) pe.add((uint16_t*)t->pilots.p + g, &t->h_pilots[g], sizeof(uint16_t));
  }
  tr.mark("patch build", pe.data.size());
  if ((rc = apply_patches(t, pe))) return rc;
  tr.mark("patch apply", pe.dst.size());
  t->dev.n_entries = (uint32_t)t->n_entries;
  std::lock_guard<std::mutex> vid_lock(t->vid_mu);
  if (t->vid_ok) {  // the value ids of the changed slots (a stale one is caught on use)
    for (uint32_t s2 : dirty.slots()) {
      const Entry& e = t->h_entries[s2];
      if (!(e.flags & EF_OCCUPIED) || e.vid >= IE_VID_CLOCK_HHMMSS) continue;
      if (e.vid >= t->vid_slot.size()) t->vid_slot.resize(e.vid + 1, UINT32_MAX);
      t->vid_slot[e.vid] = s2;
    }
  }
  return status;
}

int ie_table_set_update(ie_table* t, const ie_kv* kv, const uint32_t* table_id, const uint32_t* vid, uint64_t n) {
  if (n && !vid) return fail(IE_ERR_INVALID, "null argument");
  return table_update(t, kv, table_id, vid, nullptr, n);
}

int ie_table_set_store(ie_table* t, const ie_kv* kv, const uint32_t* table_id, uint64_t n, uint32_t* vid_out) {
  return table_update(t, kv, table_id, nullptr, vid_out, n);
}

// arena bookkeeping of a table (ie_table_set_update): bytes in use, bytes of live entries, compactions
int ie_table_arena_stats(const ie_table* t, uint64_t* bytes, uint64_t* live, uint64_t* compactions) {
  if (!t) return fail(IE_ERR_INVALID, "null argument");
  if (bytes) *bytes = t->h_arena.size();
  if (live) *live = t->arena_live;
  if (compactions) *compactions = t->n_compactions;
  return IE_SUCCESS;
}

// the largest arena ie_table_set_update may grow the table to (default and maximum 2^32 - 16:
// every arena offset is a 32-bit word); a smaller limit makes IE_ERR_CAPACITY come earlier
int ie_table_set_arena_limit(ie_table* t, uint64_t bytes) {
  if (!t) return fail(IE_ERR_INVALID, "null argument");
  t->arena_limit = std::min<uint64_t>(bytes, 0xFFFFFFF0ull);
  return IE_SUCCESS;
}

int ie_exec_host_keys(ie_exec* x, uint8_t* buf, uint64_t cap, uint64_t* used) {
  if (!x || !used || (cap && !buf)) return fail(IE_ERR_INVALID, "null argument");
  int rc = set_device(x->device);
  if (rc) return rc;
  std::vector<uint8_t> dev;
  const std::vector<uint8_t>* src = &x->hk;
  if (!x->hk_host) {
    if ((rc = read_host_keys(x, dev))) return rc;
    src = &dev;
  }
  *used = src->size();
  if (!src->empty() && cap) memcpy(buf, src->data(), std::min<uint64_t>(cap, src->size()));
  return IE_SUCCESS;
}

uint64_t ie_table_entries(const ie_table* t) { return t ? t->n_entries : 0; }
uint32_t ie_table_tables(const ie_table* t) { return t ? t->n_tables : 0; }
int32_t ie_table_dialect(const ie_table* t) { return t ? t->dialect : -1; }

int ie_exec_create(int32_t device, void* hip_stream, ie_exec** out) {
  if (!out) return fail(IE_ERR_INVALID, "null argument");
  int rc = set_device(device);
  if (rc) return rc;
  ie_exec* x = new ie_exec();
  x->device = device;
  if (const char* e = getenv("IE_FAIL_COMMIT")) x->opt_fail_commit = atoi(e) != 0 ? 1 : 0;
  if (const char* e = getenv("IE_FAST")) x->opt_fast = (uint32_t)atoi(e);
  if (const char* e = getenv("IE_DEBUG_NOEVAL")) x->opt_noeval = (uint32_t)atoi(e);
  if (const char* e = getenv("IE_TILE")) x->opt_tile = atoi(e) == 512 ? 512 : atoi(e) == 256 ? 256 : 0;
  if (const char* e = getenv("IE_VIEWS")) x->opt_views = atoi(e) != 0;
  if (const char* e = getenv("IE_RESERVE")) {
    const int v = atoi(e);
    x->opt_reserve = v >= 16 && v <= 1024 ? (uint32_t)v : 0u;
  }
  if (const char* e = getenv("IE_SMALL_HOST")) x->opt_small = atoi(e) != 0;
  if (const char* e = getenv("IE_SMALL_ZC")) x->opt_zc = atoi(e);
  if (const char* e = getenv("IE_DEFER")) x->opt_defer = atoi(e) < 0 ? -1 : atoi(e) >= 2 ? 2 : atoi(e) != 0 ? 1 : 0;
  if (const char* e = getenv("IE_DEBUG_STAMPS")) x->stamps_path = e;
  if (hip_stream) {
    x->stream = (hipStream_t)hip_stream;
  } else {
    hipError_t e = hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete x;
      return fail(IE_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    x->own_stream = true;
  }
  for (auto& e : x->ev) {
    hipError_t r = hipEventCreate(&e);
    if (r != hipSuccess) {
      delete x;
      return fail(IE_ERR_HIP, std::string("hipEventCreate: ") + hipGetErrorString(r));
    }
  }
  *out = x;
  return IE_SUCCESS;
}

void ie_exec_destroy(ie_exec* x) {
  if (x) {
    (void)hipSetDevice(x->device);
    if (x->stream) (void)hipStreamSynchronize(x->stream);
    delete x;
  }
}

int ie_exec_sync(ie_exec* x) {
  if (!x) return fail(IE_ERR_INVALID, "null exec");
  IE_HIP(hipStreamSynchronize(x->stream));
  return check_device_error(x);
}

int ie_exec_set_timing(ie_exec* x, int32_t enabled) {
  if (!x) return fail(IE_ERR_INVALID, "null exec");
  x->timing = enabled != 0;
  x->ev_recorded = false;
  return IE_SUCCESS;
}

int ie_exec_timing(ie_exec* x, ie_timing* out) {
  if (!x || !out) return fail(IE_ERR_INVALID, "null argument");
  if (x->stamp_tiles && !x->stamps_path.empty()) {  // dump the last call's phase stamps
    IE_HIP(hipStreamSynchronize(x->stream));
    std::vector<uint64_t> h(x->stamp_tiles * 16);
    IE_HIP(hipMemcpy(h.data(), x->stamps.p, h.size() * 8, hipMemcpyDeviceToHost));
    if (FILE* f = fopen(x->stamps_path.c_str(), "wb")) {
      fwrite(h.data(), 8, h.size(), f);
      fclose(f);
    }
  }
  memset(out, 0, sizeof *out);
  if (!x->ev_recorded) return fail(IE_ERR_INVALID, "no timed call recorded");
  IE_HIP(hipStreamSynchronize(x->stream));
  float setup = 0, kern = 0;
  IE_HIP(hipEventElapsedTime(&setup, x->ev[0], x->ev[1]));
  IE_HIP(hipEventElapsedTime(&kern, x->ev[1], x->ev[2]));
  out->resolve_ms = kern;   // the resolve (or escape) kernels
  out->complex_ms = 0.0f;   // literal strings are resolved inside k_resolve
  out->total_ms = setup + kern;
  uint32_t st[6] = {0, 0, 0, 0, 0, 0};
  if (x->counters.p) IE_HIP(hipMemcpy(st, (uint32_t*)ctr_base(x) + 4, 24, hipMemcpyDeviceToHost));
  out->n_complex = st[0];
  out->n_direct = st[5];  // tiles deferred to the windowed emit (counter word 9)
  out->n_polls = st[2];
  out->n_exact = st[3];
  uint32_t nd = 0;
  if (x->counters.p) IE_HIP(hipMemcpy(&nd, (uint32_t*)ctr_base(x) + 12, 4, hipMemcpyDeviceToHost));
  out->n_deferred = nd;
  out->n_chain_fail = st[4];
  return check_device_error(x);
}

// diagnostic (not part of the reference surface): device vs host view of one key's lookup.
// out[0..1] device hash lo/hi, out[2] device slot, out[3] find_bytes, out[4] find_small (klen <= 16),
// out[5] entries, out[7..8] host hash lo/hi, out[9] host slot, out[10] the host's entry index holding
// the key (or -1), out[12] find_bytes by all 64 lanes, out[13] lane agreement ballot
int ie_debug_probe(const ie_table* t, const char* key, uint64_t len, uint64_t* out) {
  if (!t || !out || (len && !key) || len > 4096) return fail(IE_ERR_INVALID, "bad argument");
  int rc = set_device(t->device);
  if (rc) return rc;
  DevBuf dk, dout;
  IE_HIP(dk.ensure(len + 16));
  IE_HIP(dout.ensure(16 * 8));
  if (len) IE_HIP(hipMemcpy(dk.p, key, len, hipMemcpyHostToDevice));
  IE_HIP(launch_debug_probe(t->dev, (const uint8_t*)dk.p, (uint32_t)len, (uint64_t*)dout.p, 0));
  IE_HIP(hipDeviceSynchronize());
  IE_HIP(hipMemcpy(out, dout.p, 16 * 8, hipMemcpyDeviceToHost));
  const uint64_t h = key_hash(std::string_view(key ? key : "", len), t->dev.seed, 0);
  std::vector<uint16_t> pil(t->dev.nb);
  IE_HIP(hipMemcpy(pil.data(), t->dev.pilots, pil.size() * sizeof(uint16_t), hipMemcpyDeviceToHost));
  out[7] = h & 0xFFFFFFFFull;
  out[8] = h >> 32;
  out[9] = ph_slot(h, pil[ph_group(h, t->dev.nb)], t->dev.m);
  out[10] = (uint64_t)-1;
  std::vector<Entry> he(t->dev.m);
  IE_HIP(hipMemcpy(he.data(), t->dev.entries, he.size() * sizeof(Entry), hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < he.size(); i++)
    if ((he[i].flags & EF_OCCUPIED) && he[i].key_len == len && (he[i].flags >> kTidShift) == 0 &&
        memcmp(he[i].key, key, std::min<uint64_t>(len, kInlineKey)) == 0)
      out[10] = i;
  return IE_SUCCESS;
}

int ie_exec_set_option(ie_exec* x, int32_t option, int64_t value) {
  if (!x) return fail(IE_ERR_INVALID, "null exec");
  switch (option) {
    case IE_OPT_FAIL_COMMIT:
      if (value < -1 || value > 1) return fail(IE_ERR_INVALID, "fail commit must be -1, 0 or 1");
      x->opt_fail_commit = (int32_t)value;
      x->stat_pending = false;
      return IE_SUCCESS;
    case IE_OPT_FAST:
      x->opt_fast = value ? 1u : 0u;
      return IE_SUCCESS;
    case IE_OPT_DEBUG_NOEVAL:
      x->opt_noeval = value ? 1u : 0u;
      return IE_SUCCESS;
    case IE_OPT_TILE:
      if (value != 0 && value != 256 && value != 512) return fail(IE_ERR_INVALID, "tile must be 0, 256 or 512");
      x->opt_tile = (int32_t)value;
      return IE_SUCCESS;
    case IE_OPT_VIEWS:
      x->opt_views = value ? 1 : 0;
      return IE_SUCCESS;
    case IE_OPT_RESERVE:
      if (value != 0 && (value < 16 || value > 1024)) return fail(IE_ERR_INVALID, "reserve must be 0 or 16..1024");
      x->opt_reserve = (uint32_t)value;
      return IE_SUCCESS;
    case IE_OPT_DEFER:
      if (value < -1 || value > 2) return fail(IE_ERR_INVALID, "defer must be -1, 0, 1 or 2");
      x->opt_defer = (int32_t)value;
      return IE_SUCCESS;
    case IE_OPT_ERROR_KEYS:
      x->opt_err_keys = value ? 1 : 0;
      return IE_SUCCESS;
    case IE_OPT_SMALL_ZC:
      if (value < 0 || value > 2) return fail(IE_ERR_INVALID, "small zero-copy must be 0, 1 or 2");
      x->opt_zc = (int32_t)value;
      return IE_SUCCESS;
    default:
      return fail(IE_ERR_INVALID, "unknown exec option");
  }
}

int ie_exec_set_scratch(ie_exec* x, uint64_t bytes) {
  if (!x) return fail(IE_ERR_INVALID, "null exec");
  x->pool_request = std::max<uint64_t>(bytes, 1 << 20);
  x->pool_fixed = true;
  return IE_SUCCESS;
}

int ie_dev_alloc(int32_t device, uint64_t bytes, void** out) {
  if (!out) return fail(IE_ERR_INVALID, "null argument");
  int rc = set_device(device);
  if (rc) return rc;
  IE_HIP(hipMalloc(out, bytes ? bytes : 16));
  return IE_SUCCESS;
}

void ie_dev_free(void* p) {
  if (p) (void)hipFree(p);
}

int ie_copy_h2d(ie_exec* x, void* dst, const void* src, uint64_t bytes) {
  if (!x || (bytes && (!dst || !src))) return fail(IE_ERR_INVALID, "null argument");
  if (!bytes) return IE_SUCCESS;
  IE_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, x->stream));
  IE_HIP(hipStreamSynchronize(x->stream));
  return IE_SUCCESS;
}

int ie_copy_d2h(ie_exec* x, void* dst, const void* src, uint64_t bytes) {
  if (!x || (bytes && (!dst || !src))) return fail(IE_ERR_INVALID, "null argument");
  if (!bytes) return IE_SUCCESS;
  IE_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, x->stream));
  IE_HIP(hipStreamSynchronize(x->stream));
  return IE_SUCCESS;
}

int ie_memset_d(ie_exec* x, void* dst, int32_t value, uint64_t bytes) {
  if (!x || (bytes && !dst)) return fail(IE_ERR_INVALID, "null argument");
  if (bytes) IE_HIP(hipMemsetAsync(dst, value, bytes, x->stream));
  return IE_SUCCESS;
}

int ie_exec_mark(ie_exec* x, uint32_t slot) {
  if (!x || slot >= 1024) return fail(IE_ERR_INVALID, "bad exec or slot");
  if (x->marks.size() <= slot) x->marks.resize(slot + 1, nullptr);
  if (!x->marks[slot]) IE_HIP(hipEventCreate(&x->marks[slot]));
  IE_HIP(hipEventRecord(x->marks[slot], x->stream));
  return IE_SUCCESS;
}

int ie_exec_elapsed(ie_exec* x, uint32_t a, uint32_t b, float* ms) {
  if (!x || !ms || a >= x->marks.size() || b >= x->marks.size() || !x->marks[a] || !x->marks[b])
    return fail(IE_ERR_INVALID, "bad exec or unrecorded slot");
  IE_HIP(hipEventSynchronize(x->marks[b]));
  IE_HIP(hipEventElapsedTime(ms, x->marks[a], x->marks[b]));
  return IE_SUCCESS;
}

// the literal pool's demand of the last interpolation call: the word its last emit kernel published
// to pinned host memory (a wait of about a microsecond after the device wrote it, and the stream's
// later work already queued behind it), else a copy and a synchronisation
int pool_demand(ie_exec* x, uint64_t* used) {
  if (x->pool_pub) {
    const volatile uint64_t* w = (const volatile uint64_t*)(x->stat_host + 8);
    const uint64_t want = x->pool_seq & 0xFFFFFFu;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 1;; k++) {
      const uint64_t v = *w;
      if ((v >> 40) == want) {
        *used = v & ((1ull << 40) - 1);
        return IE_SUCCESS;
      }
      // (bounded: a call that never gets there, e.g. a fault, is reported by the synchronisation)
      if ((k & 4095u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
      __builtin_ia32_pause();
    }
  }
  IE_HIP(hipMemcpyAsync(used, (uint64_t*)ctr_base(x) + 1, 8, hipMemcpyDeviceToHost, x->stream));
  IE_HIP(hipStreamSynchronize(x->stream));
  return IE_SUCCESS;
}

int ie_interpolate_device_ids(ie_exec* x, const ie_table* t, const uint32_t* d_table_id, const uint8_t* d_bytes,
                              const uint64_t* d_offsets, uint64_t n, const ie_dev_out* out) {
  if (!x) return fail(IE_ERR_INVALID, "null exec");
  x->hk_host = false;
  int rc = reset_host_keys(x);
  if (!rc) rc = run_device(x, kOpInterp, t, d_bytes, d_offsets, n, out, d_table_id);
  if (rc || !n || x->pool_fixed) return rc;
  // The literal path reserves scratch with one atomic per string, so the counter ends at the
  // batch's whole demand even when the pool ran out. A demand above the pool means some strings
  // report IE_E_OVERFLOW: grow the pool to the demand and re-run the batch once (the look-back
  // fixed every later offset, so a partial fix-up is impossible). Strings over their own
  // single-pass budget stay IE_E_OVERFLOW here; ie_interpolate_batch re-runs those in max mode.
  uint64_t used = 0;
  if ((rc = pool_demand(x, &used))) return rc;
  if (used <= x->pool.bytes) return IE_SUCCESS;
  x->pool_request = std::max<uint64_t>(x->pool_request, used + used / 8 + (1ull << 20));
  if ((rc = reset_host_keys(x))) return rc;
  return run_device(x, kOpInterp, t, d_bytes, d_offsets, n, out, d_table_id);
}

int ie_interpolate_device(ie_exec* x, const ie_table* t, const uint8_t* d_bytes,
                          const uint64_t* d_offsets, uint64_t n, const ie_dev_out* out) {
  return ie_interpolate_device_ids(x, t, nullptr, d_bytes, d_offsets, n, out);
}

int ie_interpolate_device_views(ie_exec* x, const ie_table* t, const uint32_t* d_table_id, const uint8_t* d_bytes,
                                const uint64_t* d_offsets, const uint32_t* d_lengths, uint64_t n,
                                const ie_dev_views* out) {
  if (!out || (n && (!out->offsets || !out->lengths))) return fail(IE_ERR_INVALID, "null argument");
  const ie_dev_out o{out->bytes, out->bytes_cap, out->offsets, out->status, out->value_id, out->total};
  if (!x) return fail(IE_ERR_INVALID, "null exec");
  x->hk_host = false;
  int rc = reset_host_keys(x);
  if (!rc) rc = run_device(x, kOpInterp, t, d_bytes, d_offsets, n, &o, d_table_id, out->lengths, d_lengths, true);
  if (rc || !n || x->pool_fixed) return rc;
  // the literal path's scratch demand, as ie_interpolate_device_ids
  uint64_t used = 0;
  if ((rc = pool_demand(x, &used))) return rc;
  if (used <= x->pool.bytes) return IE_SUCCESS;
  x->pool_request = std::max<uint64_t>(x->pool_request, used + used / 8 + (1ull << 20));
  if ((rc = reset_host_keys(x))) return rc;
  return run_device(x, kOpInterp, t, d_bytes, d_offsets, n, &o, d_table_id, out->lengths, d_lengths, true);
}

int ie_interpolate_batch_ids(ie_exec* x, const ie_table* t, const uint32_t* table_id, const uint8_t* bytes,
                             const uint64_t* offsets, uint64_t n, ie_batch** out) {
  if (!t) return fail(IE_ERR_INVALID, "null table");
  if (n && !table_id) return fail(IE_ERR_INVALID, "null table ids");
  return run_host(x, kOpInterp, t, bytes, offsets, n, out, table_id);
}

int ie_interpolate_batch(ie_exec* x, const ie_table* t, const uint8_t* bytes,
                         const uint64_t* offsets, uint64_t n, ie_batch** out) {
  if (!t) return fail(IE_ERR_INVALID, "null table");
  return run_host(x, kOpInterp, t, bytes, offsets, n, out);
}

int ie_interpolate(ie_exec* x, const ie_table* t, const char* s, uint64_t len, ie_batch** out) {
  uint64_t off[2] = {0, len};
  return ie_interpolate_batch(x, t, (const uint8_t*)s, off, 1, out);
}

int ie_unescape_cmd_device(ie_exec* x, const ie_table* t, const uint32_t* d_table_id, const uint8_t* d_bytes,
                           const uint64_t* d_offsets, uint64_t n, const uint8_t* d_status_in, const ie_dev_out* tmp,
                           const ie_dev_out* out) {
  if (!tmp || !out || !tmp->bytes || !out->status) return fail(IE_ERR_INVALID, "null argument");
  x->cmd_first = true;
  int rc = run_device(x, kOpUnescape, nullptr, d_bytes, d_offsets, n, tmp);  // py:1665
  x->cmd_first = false;
  if (rc) return rc;
  // the unescaped bytes feed the interpolation (py:1666). Unescaping never lengthens a string, so
  // a tmp as large as the input always fits; a smaller one that overflowed is flagged on the
  // device (no wait here) and reported by ie_exec_sync as IE_ERR_CAPACITY. Its offsets are then
  // all 0 (k_emit, zero_on_overflow), so the interpolation below reads nothing past tmp->bytes.
  x->in_cmd = true;
  rc = ie_interpolate_device_ids(x, t, d_table_id, tmp->bytes, tmp->offsets, n, out);
  x->in_cmd = false;
  if (rc) return rc;
  IE_HIP(launch_cap_check(tmp->total, tmp->bytes_cap, (uint32_t*)ctr_base(x) + 1, x->stream));
  if (d_status_in) IE_HIP(launch_status_carry(d_status_in, out->status, n, x->stream));
  return IE_SUCCESS;
}

int ie_unescape_cmd_device_views(ie_exec* x, const ie_table* t, const uint32_t* d_table_id, const uint8_t* d_bytes,
                                 const uint64_t* d_offsets, const uint32_t* d_lengths, uint64_t n,
                                 const uint8_t* d_status_in, const ie_dev_views* out) {
  if (!x || !out || !out->status || (n && (!out->offsets || !out->lengths))) return fail(IE_ERR_INVALID, "null argument");
  const ie_dev_out o{out->bytes, out->bytes_cap, out->offsets, out->status, out->value_id, out->total};
  x->hk_host = false;
  auto run = [&]() -> int {
    const int r0 = reset_host_keys(x);
    if (r0) return r0;
    x->in_cmd = true;
    x->cmd_fused = true;
    const int r = run_device(x, kOpInterp, t, d_bytes, d_offsets, n, &o, d_table_id, out->lengths, d_lengths);
    x->in_cmd = false;
    x->cmd_fused = false;
    return r;
  };
  int rc = run();
  if (rc) return rc;
  if (n && !x->pool_fixed) {  // the pool's demand (deferred strings + literal path), as ie_interpolate_device
    uint64_t used = 0;
    if ((rc = pool_demand(x, &used))) return rc;
    if (used > x->pool.bytes) {
      x->pool_request = std::max<uint64_t>(x->pool_request, used + used / 8 + (1ull << 20));
      if ((rc = run())) return rc;
    }
  }
  if (d_status_in && n) IE_HIP(launch_status_carry(d_status_in, out->status, n, x->stream));
  return IE_SUCCESS;
}

int ie_unescape_device(ie_exec* x, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n,
                       const ie_dev_out* out) {
  return run_device(x, kOpUnescape, nullptr, d_bytes, d_offsets, n, out);
}
int ie_escape_device(ie_exec* x, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n,
                     const ie_dev_out* out) {
  return run_device(x, kOpEscape, nullptr, d_bytes, d_offsets, n, out);
}
int ie_unescape_batch(ie_exec* x, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                      ie_batch** out) {
  return run_host(x, kOpUnescape, nullptr, bytes, offsets, n, out);
}
int ie_escape_batch(ie_exec* x, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                    ie_batch** out) {
  return run_host(x, kOpEscape, nullptr, bytes, offsets, n, out);
}

// ---- wildcard match / capture (py:553-567; ie_wildcard.hip) ----
// A wildcard compiles to its literals: the text between consecutive group markers, where a marker
// is '*' or U+3020 (the reference's w.replace('*', '〠') then '〠' -> '(.*)', so a literal U+3020
// is a group as well); re.escape makes every other byte literal.
int ie_wildcards_build(const uint8_t* bytes, const uint64_t* offsets, uint32_t n_patterns, int32_t dialect,
                       int32_t device, ie_wildcards** out) {
  const bool rs = dialect == IE_DIALECT_RS;  // runtime.rs:1633-1647: only '*' is a group
  if (!out || (n_patterns && (!offsets || (!bytes && offsets[n_patterns])))) return fail(IE_ERR_INVALID, "null argument");
  *out = nullptr;
  int rc = set_device(device);
  if (rc) return rc;
  std::vector<uint32_t> lit_off, lit_len, pat_lit;
  const uint64_t base = n_patterns ? offsets[0] : 0;
  for (uint32_t p = 0; p < n_patterns; p++) {
    pat_lit.push_back((uint32_t)lit_off.size());
    const uint64_t a = offsets[p] - base, b = offsets[p + 1] - base;
    if (b < a || b >= 0xFFFFFFF0ull) return fail(IE_ERR_INVALID, "bad wildcard offsets");
    uint64_t start = a;
    uint32_t groups = 0;
    for (uint64_t k = a; k < b;) {
      const uint8_t* c = bytes + base + k;
      const uint32_t mk = c[0] == '*' ? 1u : (!rs && k + 2 < b && c[0] == 0xE3 && c[1] == 0x80 && c[2] == 0xA0) ? 3u : 0u;
      if (!mk) {
        k++;
        continue;
      }
      lit_off.push_back((uint32_t)start);
      lit_len.push_back((uint32_t)(k - start));
      groups++;
      k += mk;
      start = k;
    }
    lit_off.push_back((uint32_t)start);
    lit_len.push_back((uint32_t)(b - start));
    if (groups > IE_WC_MAX_CAP) return fail(IE_ERR_INVALID, "wildcard with more than IE_WC_MAX_CAP groups");
  }
  pat_lit.push_back((uint32_t)lit_off.size());
  ie_wildcards* w = new ie_wildcards();
  w->device = device;
  w->n_pat = n_patterns;
  const uint64_t nb = n_patterns ? offsets[n_patterns] - base : 0;
  auto up = [&](DevBuf& d, const void* src, uint64_t n) -> hipError_t {
    hipError_t e = d.ensure(n + 16);
    return e != hipSuccess ? e : n ? hipMemcpy(d.p, src, n, hipMemcpyHostToDevice) : hipSuccess;
  };
  hipError_t e = up(w->bytes, bytes ? bytes + base : nullptr, nb);
  if (e == hipSuccess) e = up(w->lit_off, lit_off.data(), lit_off.size() * 4);
  if (e == hipSuccess) e = up(w->lit_len, lit_len.data(), lit_len.size() * 4);
  if (e == hipSuccess) e = up(w->pat_lit, pat_lit.data(), pat_lit.size() * 4);
  if (e != hipSuccess) {
    delete w;
    return fail(IE_ERR_HIP, std::string("wildcard upload: ") + hipGetErrorString(e));
  }
  w->dev = WcSet{(const uint8_t*)w->bytes.p, (const uint32_t*)w->lit_off.p, (const uint32_t*)w->lit_len.p,
                 (const uint32_t*)w->pat_lit.p, n_patterns, rs ? 1u : 0u};
  *out = w;
  return IE_SUCCESS;
}

void ie_wildcards_free(ie_wildcards* w) { delete w; }

int ie_wildcard_match_device(ie_exec* x, const ie_wildcards* w, const uint8_t* d_bytes, const uint64_t* d_offsets,
                             uint64_t n, const uint32_t* d_range, int32_t* d_match, uint8_t* d_ncap, uint32_t* d_caps) {
  if (!x || !w || !d_offsets || !d_match || !d_ncap || !d_caps || (n && !d_bytes)) return fail(IE_ERR_INVALID, "null argument");
  if (w->device != x->device) return fail(IE_ERR_INVALID, "wildcards and exec live on different devices");
  int rc = set_device(x->device);
  if (rc) return rc;
  IE_HIP(launch_wildcard(w->dev, d_bytes, d_offsets, n, d_range, d_match, d_ncap, d_caps, x->stream));
  return IE_SUCCESS;
}

int ie_wildcard_match_batch(ie_exec* x, const ie_wildcards* w, const uint8_t* bytes, const uint64_t* offsets,
                            uint64_t n, const uint32_t* range, int32_t* match, uint8_t* ncap, uint32_t* caps) {
  if (!x || !w || !offsets || !match || !ncap || !caps || (n && !bytes && offsets[n] > offsets[0]))
    return fail(IE_ERR_INVALID, "null argument");
  int rc = set_device(x->device);
  if (rc) return rc;
  if (n == 0) return IE_SUCCESS;
  const uint64_t base = offsets[0], nb = offsets[n] - base;
  // a small batch (a map task over a few states): one pinned block each way, one synchronisation
  // (as run_host_small): [offsets | ranges | bytes] in, [match | ncap | caps] out
  const uint64_t i_rng = al256((n + 1) * 8), i_bytes = i_rng + al256(range ? n * 8 : 0),
                 in_size = i_bytes + al256(nb + 64);
  const uint64_t o_ncap = al256(n * 4), o_caps = o_ncap + al256(n), out_size = o_caps + al256(n * 8 * IE_WC_MAX_CAP);
  if (in_size + out_size <= (4ull << 20)) {
    const uint64_t need = in_size + out_size;
    // zero-copy (IE_SMALL_ZC): k_wildcard reads the block and writes its results into it, no copies
    const bool zc = x->opt_zc != 0;
    if (zc) {
      if ((rc = ensure_zc(x, need))) return rc;
    } else {
      IE_HIP(x->sm_dev.ensure(std::max<uint64_t>(need, 1ull << 19)));
      if (x->sm_host_bytes < need) {
        if (x->sm_host) (void)hipHostFree(x->sm_host);
        x->sm_host = nullptr;
        x->sm_host_bytes = 0;
        const uint64_t want = std::max<uint64_t>(need, 1ull << 19);
        IE_HIP(hipHostMalloc((void**)&x->sm_host, want, hipHostMallocDefault));
        x->sm_host_bytes = want;
      }
    }
    uint8_t* const h = zc ? x->zc_host : x->sm_host;
    uint8_t* const dv = zc ? x->zc_dev : (uint8_t*)x->sm_dev.p;
    uint64_t* const hoff = (uint64_t*)h;
    for (uint64_t i = 0; i <= n; i++) hoff[i] = offsets[i] - base;
    if (range) memcpy(h + i_rng, range, n * 8);
    if (nb) memcpy(h + i_bytes, bytes + base, nb);
    memset(h + i_bytes + nb, 0, 64);
    if (!zc) IE_HIP(hipMemcpyAsync(dv, h, in_size, hipMemcpyHostToDevice, x->stream));
    uint8_t* const dout = dv + in_size;
    rc = ie_wildcard_match_device(x, w, dv + i_bytes, (const uint64_t*)dv, n, range ? (const uint32_t*)(dv + i_rng) : nullptr,
                                  (int32_t*)dout, dout + o_ncap, (uint32_t*)(dout + o_caps));
    if (rc) return rc;
    if (!zc) IE_HIP(hipMemcpyAsync(h + in_size, dout, out_size, hipMemcpyDeviceToHost, x->stream));
    IE_HIP(hipStreamSynchronize(x->stream));
    memcpy(match, h + in_size, n * 4);
    memcpy(ncap, h + in_size + o_ncap, n);
    memcpy(caps, h + in_size + o_caps, n * 8 * IE_WC_MAX_CAP);
    return IE_SUCCESS;
  }
  std::vector<uint64_t> off(offsets, offsets + n + 1);
  for (auto& o : off) o -= base;
  IE_HIP(x->in_bytes.ensure(nb + 16));
  IE_HIP(x->in_off.ensure((n + 1) * 8));
  IE_HIP(x->wc_match.ensure(n * 4));
  IE_HIP(x->wc_ncap.ensure(n));
  IE_HIP(x->wc_caps.ensure(n * 8 * IE_WC_MAX_CAP));
  if (nb) IE_HIP(hipMemcpyAsync(x->in_bytes.p, bytes + base, nb, hipMemcpyHostToDevice, x->stream));
  IE_HIP(hipMemcpyAsync(x->in_off.p, off.data(), (n + 1) * 8, hipMemcpyHostToDevice, x->stream));
  const uint32_t* d_range = nullptr;
  if (range) {
    IE_HIP(x->wc_range.ensure(n * 8));
    IE_HIP(hipMemcpyAsync(x->wc_range.p, range, n * 8, hipMemcpyHostToDevice, x->stream));
    d_range = (const uint32_t*)x->wc_range.p;
  }
  rc = ie_wildcard_match_device(x, w, (const uint8_t*)x->in_bytes.p, (const uint64_t*)x->in_off.p, n, d_range,
                                (int32_t*)x->wc_match.p, (uint8_t*)x->wc_ncap.p, (uint32_t*)x->wc_caps.p);
  if (rc) return rc;
  IE_HIP(hipMemcpyAsync(match, x->wc_match.p, n * 4, hipMemcpyDeviceToHost, x->stream));
  IE_HIP(hipMemcpyAsync(ncap, x->wc_ncap.p, n, hipMemcpyDeviceToHost, x->stream));
  IE_HIP(hipMemcpyAsync(caps, x->wc_caps.p, n * 8 * IE_WC_MAX_CAP, hipMemcpyDeviceToHost, x->stream));
  IE_HIP(hipStreamSynchronize(x->stream));
  return IE_SUCCESS;
}

void ie_batch_free(ie_batch* b) {
  if (!b) return;
  delete[] b->bytes;
  delete[] b->offsets;
  delete[] b->status;
  delete[] b->value_id;
  delete b;
}

int ie_simple_insertkey(const char* s, uint64_t len, int32_t dialect, uint64_t* key_off,
                        uint64_t* key_len) {
  // py:477-495 / interp.rs:11-29 on the caller's string (callers pass protected text when they
  // mirror interpolate_inserts; recursive_interpolate passes the raw string, py:1463)
  if (key_off) *key_off = 0;
  if (key_len) *key_len = 0;
  if (!s && len) return 0;
  const uint8_t* p = (const uint8_t*)s;
  uint64_t ko = 0, kl = 0;
  if (!simple_insertkey([&](uint64_t k) { return p[k]; }, len, dialect == IE_DIALECT_RS ? 1u : 0u, ko, kl)) return 0;
  if (key_off) *key_off = ko;
  if (key_len) *key_len = kl;
  return 1;
}

// ---- synthetic workloads ----
int ie_synth_create(int32_t config, uint64_t seed, ie_synth** out) {
  if (!out) return fail(IE_ERR_INVALID, "null argument");
  if (config < 2 || config > 4) return fail(IE_ERR_INVALID, "synthetic config must be 2, 3 or 4");
  ie_synth* s = new ie_synth();
  s->P.config = config;
  s->P.seed = seed ? seed : (0x1E5EED00ull + (uint64_t)config);
  s->P.n_keys = 1000;
  s->P.n_q = 99000;
  s->P.n_i = 1000;
  uint64_t st = s->P.seed ^ 0xA5A5A5A5DEADBEEFull;
  auto filler_value = [&]() {
    uint32_t len = 4 + (uint32_t)(splitmix(st) % 21);
    std::string v(len, '\0');
    synth_filler(st, (uint8_t*)&v[0], len);
    return v;
  };
  if (config == 2) {
    for (uint32_t j = 0; j < s->P.n_keys; j++) {
      s->keys.push_back("k" + std::to_string(j));
      s->texts.push_back(filler_value());
    }
  } else if (config == 3) {
    for (uint32_t j = 0; j < s->P.n_q; j++) {
      s->keys.push_back("q-" + std::to_string(j));
      s->texts.push_back(filler_value());
    }
    for (uint32_t j = 0; j < s->P.n_i; j++) {
      s->keys.push_back("i" + std::to_string(j));
      s->texts.push_back(std::to_string(splitmix(st) % s->P.n_q));  // int value, str(int) splice
    }
  } else {
    // config 4: 100k entries = q-/a-/b- (32,666 each) + i (1,000) + c (1,000).
    // q- strings; i, a-, b- ints in [0, n_q) so every chain depth resolves; c- strings that
    // carry a {q-N} reference (re-resolved after the splice, py:516-535).
    s->P.n_q = 32666;
    s->P.n_chain = 1000;
    for (uint32_t j = 0; j < s->P.n_q; j++) {
      s->keys.push_back("q-" + std::to_string(j));
      s->texts.push_back(filler_value());
    }
    for (const char* pre : {"a-", "b-"})
      for (uint32_t j = 0; j < s->P.n_q; j++) {
        s->keys.push_back(pre + std::to_string(j));
        s->texts.push_back(std::to_string(splitmix(st) % s->P.n_q));
      }
    for (uint32_t j = 0; j < s->P.n_i; j++) {
      s->keys.push_back("i" + std::to_string(j));
      s->texts.push_back(std::to_string(splitmix(st) % s->P.n_q));
    }
    // the escaped segment \{lit\} of 10 % of the strings: after the unescape command's
    // recursive_unescape it is a live {lit} reference, resolved by its recursive_interpolate
    s->keys.push_back("lit");
    s->texts.push_back("LIT");
    for (uint32_t j = 0; j < s->P.n_chain; j++) {
      s->keys.push_back("c-" + std::to_string(j));
      std::string head(4, '\0'), tail(4, '\0');
      synth_filler(st, (uint8_t*)&head[0], 4);
      std::string ref = "{q-" + std::to_string(splitmix(st) % s->P.n_q) + "}";
      synth_filler(st, (uint8_t*)&tail[0], 4);
      s->texts.push_back(head + ref + tail);
    }
  }
  s->kv.resize(s->keys.size());
  for (size_t j = 0; j < s->keys.size(); j++) {
    const bool is_int = (config == 3 && j >= s->P.n_q) ||
                        (config == 4 && j >= s->P.n_q && j < 3ull * s->P.n_q + s->P.n_i);
    s->kv[j] = ie_kv{s->keys[j].data(), s->keys[j].size(), s->texts[j].data(), s->texts[j].size(),
                     is_int ? IE_KIND_INT : IE_KIND_STR, 0};
  }
  *out = s;
  return IE_SUCCESS;
}

void ie_synth_free(ie_synth* s) { delete s; }

uint64_t ie_synth_kv(const ie_synth* s, const ie_kv** kv) {
  if (!s) return 0;
  if (kv) *kv = s->kv.data();
  return s->kv.size();
}

int ie_synth_strings_host(const ie_synth* s, uint64_t first, uint64_t n, uint8_t* bytes,
                          uint64_t bytes_cap, uint64_t* offsets, uint64_t* total) {
  if (!s || !offsets) return fail(IE_ERR_INVALID, "null argument");
  uint64_t w = 0;
  for (uint64_t k = 0; k < n; k++) {
    offsets[k] = w;
    w += synth_len(s->P, first + k);
  }
  offsets[n] = w;
  if (total) *total = w;
  if (bytes) {
    if (w > bytes_cap) return fail(IE_ERR_CAPACITY, "synthetic bytes exceed capacity");
    for (uint64_t k = 0; k < n; k++) synth_string(s->P, first + k, bytes + offsets[k]);
  }
  return IE_SUCCESS;
}

int ie_synth_strings_device(ie_exec* x, const ie_synth* s, uint64_t first, uint64_t n,
                            uint8_t* d_bytes, uint64_t bytes_cap, uint64_t* d_offsets,
                            uint64_t* total) {
  if (!x || !s || !d_offsets) return fail(IE_ERR_INVALID, "null argument");
  int rc = set_device(x->device);
  if (rc) return rc;
  IE_HIP(x->s_lens.ensure((n + 1) * 8));
  IE_HIP(x->s_part.ensure(((n / (kBlock * 16)) + 2) * 8 + 64));
  uint64_t* d_total = (uint64_t*)((char*)x->s_part.p + x->s_part.bytes - 64);
  IE_HIP(launch_synth(s->P, first, n, (uint64_t*)x->s_lens.p, (uint64_t*)x->s_part.p, d_offsets,
                      d_total, nullptr, x->stream));
  uint64_t tot = 0;
  IE_HIP(hipMemcpyAsync(&tot, d_total, 8, hipMemcpyDeviceToHost, x->stream));
  IE_HIP(hipStreamSynchronize(x->stream));
  if (total) *total = tot;
  if (d_bytes) {
    if (tot > bytes_cap) return fail(IE_ERR_CAPACITY, "synthetic bytes exceed capacity");
    IE_HIP(launch_synth(s->P, first, n, nullptr, nullptr, d_offsets, nullptr, d_bytes, x->stream));
    IE_HIP(hipStreamSynchronize(x->stream));
  }
  return IE_SUCCESS;
}

}  // extern "C"
