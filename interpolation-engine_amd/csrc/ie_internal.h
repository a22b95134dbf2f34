// ie_internal.h — the host library's internal types, shared by its translation units (ie_host.cpp:
// tables, execs, batches; ie_maps.cpp: the map commands). Not part of the C ABI (include/ie_amd.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <new>

#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/ie_amd.h"
#include "ie_common.h"
#include "ie_kernels.h"

using namespace ie;

// the calling thread's last error text (ie_last_error); returns code
int fail(int code, const std::string& msg);

#define IE_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(IE_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));     \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  uint64_t bytes = 0;
  hipError_t ensure(uint64_t need) {
    if (need <= bytes && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    uint64_t n = std::max<uint64_t>(need, 256);
    hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess) bytes = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};


bool have_device();

// IE_HOST_TRACE=1: each phase's host wall time to stderr (where a map command's or an update's
// time goes); off: one branch per mark
struct Trace {
  const bool on = getenv("IE_HOST_TRACE") != nullptr;
  const char* cmd;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  explicit Trace(const char* c) : cmd(c) {}
  void mark(const char* what, uint64_t n = 0) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[ie_host] %-8s %-14s n=%-9llu %10.1f us\n", cmd, what, (unsigned long long)n,
            std::chrono::duration<double, std::micro>(now - t).count());
    t = now;
  }
};

// fn(lo, hi) over [0, n) split across up to IE_HOST_THREADS host threads (default: the cores, at
// most 8): the table mirror's bulk byte work (text scans, text copies, compaction, patches)
inline unsigned host_threads() {
  static const unsigned n = [] {
    const char* e = getenv("IE_HOST_THREADS");
    const long v = e ? atol(e) : 0;
    return v > 0 ? (unsigned)v : std::min(8u, std::max(1u, std::thread::hardware_concurrency()));
  }();
  return n;
}
// (`bytes`: about how much memory the whole loop touches; a thread per 256 KB at most, so a scalar
// caller's few stores never pay a thread start)
template <class F>
void parallel_for(uint64_t n, uint64_t bytes, F&& fn) {
  const unsigned T = (unsigned)std::min<uint64_t>(std::min<uint64_t>(host_threads(), n), bytes >> 18);
  if (T <= 1) {
    fn((uint64_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (unsigned k = 1; k < T; k++) th.emplace_back([&fn, n, k, T] { fn(n * k / T, n * (k + 1) / T); });
  fn((uint64_t)0, n / T);
  for (std::thread& x : th) x.join();
}

// a text copy ie_table_set_update defers until the appends are placed (then done in parallel)
struct CopyJob {
  uint64_t dst;
  const uint8_t* src;
  uint64_t len;
};

// The host mirror of a table's text arena: a growable byte buffer over an anonymous mapping, grown
// by mremap (the kernel moves page tables, not bytes: a 200 MB arena grows without a copy) and
// backed by transparent huge pages where the kernel gives them (a store appends tens of MB of
// history text per iteration: 2 MB faults, not 4 KB ones). Appends only; the subset of
// std::vector's interface the table code uses.
class HostArena {
 public:
  HostArena() = default;
  HostArena(const HostArena& o) { insert(end(), o.begin(), o.end()); }
  HostArena& operator=(const HostArena& o) {
    if (this != &o) {
      n_ = 0;
      insert(end(), o.begin(), o.end());
    }
    return *this;
  }
  HostArena(HostArena&& o) noexcept { swap(o); }
  HostArena& operator=(HostArena&& o) noexcept {
    swap(o);  // (o takes ours and frees it)
    return *this;
  }
  ~HostArena() {
    if (p_) munmap(p_, cap_);
  }
  void swap(HostArena& o) noexcept {
    std::swap(p_, o.p_);
    std::swap(n_, o.n_);
    std::swap(cap_, o.cap_);
  }
  uint8_t* data() { return p_; }
  const uint8_t* data() const { return p_; }
  uint8_t* begin() { return p_; }
  uint8_t* end() { return p_ + n_; }
  const uint8_t* begin() const { return p_; }
  const uint8_t* end() const { return p_ + n_; }
  uint64_t size() const { return n_; }
  uint64_t capacity() const { return cap_; }
  bool empty() const { return n_ == 0; }
  void clear() { n_ = 0; }
  void reserve(uint64_t want) {
    if (want <= cap_) return;
    const uint64_t kStep = 2ull << 20;
    const uint64_t cap = (std::max<uint64_t>(want, cap_ * 2) + kStep - 1) & ~(kStep - 1);
    void* q = p_ ? mremap(p_, cap_, cap, MREMAP_MAYMOVE)
                 : mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (q == MAP_FAILED) throw std::bad_alloc();
    madvise((uint8_t*)q + cap_, cap - cap_, MADV_HUGEPAGE);
    p_ = (uint8_t*)q;
    cap_ = cap;
  }
  void grow(uint64_t k) {  // k more bytes, written later (ie_table_set_update's deferred copies)
    reserve(n_ + k);
#ifdef MADV_POPULATE_WRITE
    if (k >= (1u << 20)) {  // (fresh pages faulted in by one call, not by the writers one at a time)
      const uintptr_t lo = ((uintptr_t)(p_ + n_) + 4095) & ~(uintptr_t)4095, hi = (uintptr_t)(p_ + n_ + k) & ~(uintptr_t)4095;
      if (hi > lo) (void)madvise((void*)lo, hi - lo, MADV_POPULATE_WRITE);
    }
#endif
    n_ += k;
  }
  void push_back(uint8_t b) {
    if (n_ == cap_) reserve(n_ + 1);
    p_[n_++] = b;
  }
  template <class It>
  void insert(uint8_t* /* end() only */, It first, It last) {
    const uint64_t k = (uint64_t)(last - first);
    if (!k) return;
    reserve(n_ + k);
    memcpy(p_ + n_, &*first, k);
    n_ += k;
  }

 private:
  uint8_t* p_ = nullptr;
  uint64_t n_ = 0, cap_ = 0;
};

struct ie_table {
  int32_t device = 0;
  int32_t dialect = 0;
  uint32_t flags = 0;
  uint64_t n_entries = 0;
  uint32_t n_tables = 1;  // inserts dicts in the set
  DevTable dev{};
  // the clock entries ('HH:MM', 'HH:MM:SS' of every table): their slots (ie_table_set_clock)
  std::vector<uint32_t> clock_slots;  // [2 * table + 0/1]: 'HH:MM' / 'HH:MM:SS' (UINT32_MAX: none)
  DevBuf entries, pilots, arena;
  // host mirror of the device table (ie_table_set_update, ie_table_set_clock): entries, pilots,
  // the arena (device capacity arena_cap), the slots of each pilot group, and per table of the set
  // the slots of its pre-resolved (EF_RAWALT) entries
  std::vector<Entry> h_entries;
  std::vector<uint16_t> h_pilots;
  HostArena h_arena;
  HostArena h_arena_spare;
  std::vector<CopyJob>* defer = nullptr;  // set inside ie_table_set_update: long texts copied later  // the buffer the next compaction copies into (pages already touched)
  uint64_t arena_cap = 0;
  // arena bookkeeping (ie_table_set_update): bytes the live entries occupy (the rest of h_arena is
  // dead: replaced texts), the largest arena the table may have (an offset must stay below 2^32;
  // ie_table_set_arena_limit lowers it), and how often it was compacted
  uint64_t arena_live = 0;
  uint64_t arena_limit = 0xFFFFFFF0ull;
  uint64_t n_compactions = 0;
  // value ids ie_table_set_store hands out: the next unused one (the build's kv count), and those
  // deleted keys gave back
  uint32_t next_vid = 0;
  std::vector<uint32_t> free_vids;
  std::vector<std::vector<uint32_t>> groups;
  // value id -> slot, built on demand (ie_maps.cpp: str() of a typed result), kept by the updates.
  // The lazy rebuild happens on the READ paths (ie_table_value, the map steps' value_str), which
  // several host threads may run on one table at once (the header's thread contract): vid_mu
  // guards the map and its flag
  mutable std::mutex vid_mu;
  mutable std::vector<uint32_t> vid_slot;  // value id -> slot (UINT32_MAX: none); checked on use
  mutable bool vid_ok = false;
  // occupied slots (bitmap) for ie_table_set_update's pilot searches: cache-resident where the
  // entries are tens of MB; built on the first update, kept by the updates, dropped by a re-placement
  std::vector<uint64_t> occ;
  bool occ_ok = false;
  std::unordered_map<uint32_t, std::vector<uint32_t>> rawalt;
  DevBuf patch_staging;  // ie_table_set_update / _set_clock uploads
  // the last patch kernel (null stream) of an update: batches wait for it on their own stream
  // (run_device) instead of the update synchronising the device after it
  hipEvent_t patched = nullptr;
  std::atomic<bool> patch_pending{false};
  ~ie_table() {
    if (patched) (void)hipEventDestroy(patched);
    entries.release();
    pilots.release();
    arena.release();
    patch_staging.release();
  }
};

struct ie_exec {
  // compiled wildcard lists of the map commands (ie_maps.cpp), most recent last: a map task's keys
  // are the same texts call after call, so their device copies are kept instead of re-uploaded
  std::vector<std::pair<std::string, struct ie_wildcards*>> wc_cache;
  int32_t device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  bool timing = false;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  std::vector<hipEvent_t> marks;  // ie_exec_mark slots
  bool ev_recorded = false;
  uint32_t lit_cap_max = 0;
  uint64_t pool_request = 256ull << 20;
  bool pool_fixed = false;  // set by ie_exec_set_scratch: the caller sized the pool, no wait/re-run
  // options (ie_exec_set_option); defaults read once from the environment at ie_exec_create
  int32_t opt_fail_commit = -1;   // -1 adaptive, 0 / 1 forced (IE_FAIL_COMMIT)
  uint32_t opt_fast = 1;          // 0: exact evaluator only (IE_FAST)
  int32_t opt_tile = 0;           // k_resolve tile: 0 by call site, 256 or 512 forced (IE_TILE)
  int32_t opt_views = 1;          // host batch APIs resolve into a views layout (IE_VIEWS; 0: packed on the device)
  int32_t opt_defer = 2;          // views batches in two passes (a LEAN first pass, the strings it cannot
                                  // finish in a second): 2 (default) batches of >= kLeanMinN strings or
                                  // with many heavy strings, -1 the latter only, 0 never, 1 always (IE_DEFER)
  bool defer_slow = false;        // the adaptive choice (from an earlier batch's counts)
  int32_t opt_small = 1;          // host batches of <= 1024 strings / 64 KB: one pinned copy each way (IE_SMALL_HOST)
  int32_t opt_err_keys = 0;       // IE_OPT_ERROR_KEYS: record the missing key of every IE_E_INTERP string
  uint32_t opt_reserve = 0;       // views output of a packed batch: reserved ranges at opt_reserve / 16 x the
                                  // input offsets (IE_OPT_RESERVE; 0: one claim per tile on one cursor)
  bool in_cmd = false;            // inside the unescape command's second resolve
  bool cmd_first = false;         // the unescape command's unescape step (offsets zeroed on overflow)
  bool cmd_fused = false;         // the fused unescape command (views): launch_unescape_cmd
  uint32_t opt_noeval = 0;        // diagnostic verbatim copy (IE_DEBUG_NOEVAL)
  std::string stamps_path;        // diagnostic phase stamps (IE_DEBUG_STAMPS)
  // fail commit (k_resolve<true>): chosen from the chain-failure count of an earlier batch, read
  // back asynchronously (never a wait): > 0.1 % of a batch switches to it, a batch with none back
  bool fail_commit = false;
  bool stat_pending = false;
  bool no_stats = false;  // run_host_small: no statistics copy (two stream operations of a scalar call)
  bool small_no_emit = false;  // run_host_small: a one-tile views batch may skip k_emit_windows
  bool no_emit_used = false;   // (run_device: it did; a deferred tile then needs the full path)
  uint8_t* ctr_override = nullptr;  // run_host_small: the counters in its own block, zeroed by its input copy
  uint64_t stat_n = 0;
  uint32_t* stat_host = nullptr;  // pinned, mapped: the last emit kernel of a call writes it (stat_dev)
  uint32_t* stat_dev = nullptr;
  uint32_t hint_sub_grid = 0, hint_emit_grid = 0;  // (0: the defaults until a call's telemetry is in)
  bool stat_two_pass = false;                        // (the pending telemetry is a two-pass call's)
  bool stat_fc = false, hint_fc = false;             // (the fail-commit mode they were measured in)
  uint32_t ctr_cur = 0;        // the counter set of the last call (ie_host.cpp, kCounterBytes)
  uint64_t pool_seq = 0;       // the last interpolation call's number (its published pool word)
  bool pool_pub = false;       // its last emit kernel publishes the pool demand (pool_demand)
  bool ctr_next_clean = false; // the other set was zeroed by the last call's emit kernel
  hipEvent_t stat_ev = nullptr;
  // workspace
  DevBuf counters, pool, out_len, tile_sum, tile_base, defer_tiles, defer_desc;
  // keys only the host can look up (IE_NEEDS_HOST): [u64 bytes used | pad][records] (ie_exec_host_keys);
  // a host batch call keeps its records (all its device passes, indices of its own batch) in hk
  DevBuf host_keys;
  std::vector<uint8_t> hk;
  bool hk_host = false;
  bool hk_dirty = true;  // the device list may hold records (a pass with host keys enabled ran since the reset)
  // the fused unescape command's deferred pass: list, views into the pool, table ids
  DevBuf u_list, u_off, u_len, u_tid;
  // host-API staging
  DevBuf in_bytes, in_off, in_tid, o_bytes, o_off, o_len, o_status, o_vid, o_total, wc_range, wc_match, wc_ncap, wc_caps;
  // synth scratch
  DevBuf s_lens, s_part;
  DevBuf stamps;        // diagnostic phase stamps (env IE_DEBUG_STAMPS=<file>)
  uint64_t stamp_tiles = 0;
  // small host batches: one device block and one pinned host block (inputs, then outputs)
  DevBuf sm_dev;
  uint8_t* sm_host = nullptr;
  uint64_t sm_host_bytes = 0;
  // small calls without copies (IE_SMALL_ZC=1; 2: the outputs only): one pinned block, mapped and
  // coherent, the kernels read their inputs from and write their outputs to; the counters of such a
  // call in device memory, left zeroed by its k_resolve (zc_dirty: a call that took another path did
  // not). Off by default: the scalar call measured the same with and without it (32.2-33.3 µs in
  // every mode, profiles/r06/scalar_zc/): what the two copies saved, the kernel's reads and writes
  // across the host link cost
  int32_t opt_zc = 0;
  uint8_t* zc_host = nullptr;
  uint8_t* zc_dev = nullptr;  // (the block's device address)
  uint64_t zc_bytes = 0;
  DevBuf zc_ctr;
  bool zc_dirty = true;
  uint32_t* zc_ctr_host = nullptr;  // (run_device: a one-tile no-emit call's counter words go here)
  ~ie_exec() {
    for (auto& kv : wc_cache) ie_wildcards_free(kv.second);
    sm_dev.release();
    zc_ctr.release();
    if (sm_host) (void)hipHostFree(sm_host);
    if (zc_host) (void)hipHostFree(zc_host);
    for (DevBuf* b : {&u_list, &u_off, &u_len, &u_tid, &host_keys}) b->release();
    for (DevBuf* b : {&counters, &pool, &out_len, &tile_sum, &tile_base, &defer_tiles, &defer_desc, &in_bytes,
                      &in_off, &in_tid, &o_bytes, &o_off, &o_len, &o_status, &o_vid, &o_total, &wc_range, &wc_match, &wc_ncap, &wc_caps,
                      &s_lens, &s_part, &stamps})
      b->release();
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : marks)
      if (e) (void)hipEventDestroy(e);
    if (stat_ev) (void)hipEventDestroy(stat_ev);
    if (stat_host) (void)hipHostFree(stat_host);
    if (own_stream && stream) (void)hipStreamDestroy(stream);
  }
};

struct ie_wildcards {
  int32_t device = 0;
  uint32_t n_pat = 0;
  DevBuf bytes, lit_off, lit_len, pat_lit;
  WcSet dev{};
  ~ie_wildcards() {
    for (DevBuf* b : {&bytes, &lit_off, &lit_len, &pat_lit}) b->release();
  }
};

struct ie_synth {
  SynthParams P{};
  std::vector<std::string> keys, texts;
  std::vector<ie_kv> kv;
};

// helpers of ie_host.cpp used by the other translation units
int set_device(int32_t dev);
uint32_t text_flags(const std::string_view t);
uint32_t kind_flags(int32_t kind, int32_t dialect);
uint64_t key_hash(const std::string_view k, uint64_t seed, uint32_t tid);
// the key stored at a slot of a table's host mirror
std::string_view mirror_key(const ie_table* t, const ie::Entry& e);
// a batch through the device from host memory (H2D, kernels, D2H): op kOpInterp / kOpUnescape / kOpEscape
int run_host(ie_exec* x, int op, const ie_table* t, const uint8_t* bytes, const uint64_t* offsets,
             uint64_t n, ie_batch** outp, const uint32_t* table_id = nullptr);
