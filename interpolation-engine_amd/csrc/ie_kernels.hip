// ie_kernels.hip — gfx950 kernels of the `{key}` resolver (interpolate_inserts, py:497-541 /
// rust-project/src/interp.rs:31-89) and of recursive_(un)escape on strings (py:1436-1460).
//
// Pipeline for one packed batch (bytes + offsets[n+1]), all on one HIP stream:
//   k_measure<OP>   one 256-thread workgroup per tile of 256 consecutive strings. The tile's bytes
//                   are staged in LDS with 16-byte coalesced loads; every lane then runs the
//                   per-string evaluator on its own string out of LDS (fast path) and writes the
//                   string's status and output length; strings the fast path cannot prove equal
//                   to the reference are queued for k_literal. Per-tile output sums -> tile_sum.
//   k_literal       a literal emulation of py:505-540 for the queued ("complex") strings in a
//                   global scratch pool: rfind/find loop, placeholder protocol, re-protect after
//                   every splice, exact error order. Results stay in the pool.
//   k_scan_tiles    exclusive scan of tile sums -> tile bases, grand total.
//   k_emit<OP>      re-stages each tile, scans its string lengths in the workgroup, re-runs the
//                   evaluator in emit mode into an LDS output stage aligned like the destination,
//                   copies complex results from the pool, and streams the stage out with 16-byte
//                   stores; writes offsets[] (and value ids for typed results).
//
// The fast path handles strings whose brace structure is properly nested and whose spliced
// values are inert: for them the reference's rightmost-innermost loop equals one
// left-to-right stack evaluation, with the failure reported for the failing pair of largest
// opening offset. Everything else (re-resolving values, '}{' leftovers, U+3020 placeholder
// collisions, '.\}' restore collisions, trailing-backslash hazards, depth > kMaxDepth) is routed
// to k_literal, so results are identical to the reference on every input.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ie_amd.h"
#include "ie_common.h"
#include "ie_kernels.h"

namespace ie {

// ------------------------------------------------------------------------------------------
// table lookup: get_interpdata (py:430-467 / interp.rs:91-137) against the device table.
// 'HH:MM' / 'HH:MM:SS' are entries injected by the builder; '' is never an entry.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t j = 0; j < n; j++)
    if (a[j] != b[j]) return false;
  return true;
}

__device__ __forceinline__ uint64_t hash_bytes(const uint8_t* k, uint32_t n) {
  uint64_t h = 0;
  for (uint32_t j = 0; j < n; j++) h = hash_step(h, k[j]);
  return h;
}

__device__ int32_t table_find(const DevTable& T, const uint8_t* key, uint32_t klen) {
  const uint64_t h = hash_bytes(key, klen);
  uint32_t s = slot_of(h, klen, T.mask);
  for (uint32_t probes = 0; probes <= T.mask; probes++) {
    const uint32_t e = T.slots[s];
    if (!e) return -1;
    const DevEntry& E = T.entries[e - 1];
    if (E.hash == h && E.key_len == klen && bytes_eq(T.arena + E.key_off, key, klen))
      return (int32_t)(e - 1);
    s = (s + 1) & T.mask;
  }
  return -1;
}

// status of a key that is not in the table (py:437-467 / interp.rs:105-136)
__device__ uint8_t missing_status(const DevTable& T, const uint8_t* k, uint32_t n) {
  if (n == 0) return IE_E_INTERP;
  if (!(T.flags & TF_HAS_DIR)) return IE_E_INTERP;
  bool is_arg = n >= 3 && k[0] == 'A' && k[1] == 'R' && k[2] == 'G';
  if (T.dialect == IE_DIALECT_PY && n == 3) is_arg = false;  // ''.isdigit() is False
  for (uint32_t j = 3; is_arg && j < n; j++) is_arg = k[j] >= '0' && k[j] <= '9';
  return is_arg ? (uint8_t)IE_E_INTERP : (uint8_t)IE_NEEDS_HOST;
}

// lookup with a RAW value as the key (nested whole-string form, py:511-512 / interp.rs:47-48)
__device__ int32_t table_find_raw(const DevTable& T, int32_t e_prev, uint8_t& st) {
  const DevEntry& W = T.entries[e_prev];
  if (!(W.flags & EF_KEY_STR)) {
    st = (W.flags & EF_KEY_UNHASHABLE) ? (uint8_t)IE_E_UNHASHABLE
         : (T.flags & TF_HAS_DIR)      ? (uint8_t)IE_NEEDS_HOST
                                       : (uint8_t)IE_E_INTERP;
    return -1;
  }
  const int32_t e = table_find(T, T.arena + W.text_off, W.text_len);
  if (e < 0) st = missing_status(T, T.arena + W.text_off, W.text_len);
  return e;
}

// ------------------------------------------------------------------------------------------
// The fast evaluator: one lane, one string (in LDS or global memory).
// ------------------------------------------------------------------------------------------
struct LaneScratch {
  uint8_t* kbuf;        // kKeyCap bytes: keys under construction, innermost at the top
  uint32_t* st_open;    // [kMaxDepth] stride kBlock: opening offset of each open pair
  uint16_t* st_kstart;  // [kMaxDepth] stride kBlock: kbuf fill when the pair opened
};

template <bool EMIT>
__device__ uint8_t eval_fast(const DevTable& T, const uint8_t* __restrict__ s, uint32_t n,
                             const LaneScratch& L, uint8_t* __restrict__ out, uint32_t& out_len,
                             uint32_t& vid) {
  uint32_t depth = 0, klen = 0, olen = 0;
  uint32_t nopen = 0, nclose = 0;
  bool negclose = false;
  uint32_t poison = 0;  // bit d: the pair open at level d contains a failed pair
  int64_t err_off = -1;
  uint8_t err_cls = 0;
  int32_t wrap_e = -1;  // entry returned by the innermost whole-string pair resolved so far
  uint8_t prev = 0;
  uint32_t i = 0;

#define IE_PUT(ch)                          \
  do {                                      \
    if (depth) {                            \
      if (klen >= kKeyCap) return kStatusPending; \
      L.kbuf[klen++] = (ch);                \
    } else {                                \
      if (EMIT) out[olen] = (ch);           \
      olen++;                               \
    }                                       \
  } while (0)

  while (i < n) {
    const uint8_t c = s[i];
    if (c == '\\' && i + 1 < n) {
      const uint8_t c2 = s[i + 1];
      if (c2 == '{' || c2 == '}') {
        // '\}' right after '.' or '}' can restore as '\{' (py:537-540 replace order): literal path
        if (c2 == '}' && (prev == '.' || prev == '}')) return kStatusPending;
        IE_PUT(c);
        IE_PUT(c2);
        prev = c2;
        i += 2;
        continue;
      }
    }
    if (c == 0xE3 && i + 2 < n && s[i + 1] == 0x80 && s[i + 2] == 0xA0)
      return kStatusPending;  // a literal U+3020 collides with the placeholders (py:502-503)
    if (c == '{') {
      nopen++;
      if (depth >= kMaxDepth) return kStatusPending;
      L.st_open[depth * kBlock] = i;
      L.st_kstart[depth * kBlock] = (uint16_t)klen;
      poison &= ~(1u << depth);
      depth++;
      prev = c;
      i++;
      continue;
    }
    if (c == '}') {
      nclose++;
      if (depth == 0) {  // unmatched: literal text unless the counts check fails
        negclose = true;
        IE_PUT(c);
        prev = c;
        i++;
        continue;
      }
      depth--;
      const uint32_t open = L.st_open[depth * kBlock];
      const uint32_t ks = L.st_kstart[depth * kBlock];
      const uint32_t kl = klen - ks;
      klen = ks;
      if ((poison >> depth) & 1u) {  // an inner pair failed first: this pair is never evaluated
        if (depth) poison |= 1u << (depth - 1);
        prev = c;
        i++;
        continue;
      }
      // a "whole-string" pair (get_simple_insertkey truthy at this nesting level, py:510-514)
      const bool wrapping = (open == depth) && (i == n - 1 - depth) && (i - open >= 2);
      uint8_t st = 0;
      int32_t e;
      if (wrapping && wrap_e >= 0) {
        e = table_find_raw(T, wrap_e, st);
      } else {
        e = table_find(T, L.kbuf + ks, kl);
        if (e < 0) st = missing_status(T, L.kbuf + ks, kl);
      }
      if (e >= 0 && !wrapping) {
        const DevEntry& E = T.entries[e];
        if (!(E.flags & EF_SPLICE_OK)) {
          e = -1;
          st = IE_E_ASSERT_TYPE;
        } else if (!(E.flags & EF_INERT)) {
          return kStatusPending;  // re-resolution / escape hazard: literal path
        } else {
          const uint8_t* t = T.arena + E.text_off;
          for (uint32_t j = 0; j < E.text_len; j++) IE_PUT(t[j]);
        }
      }
      if (e < 0) {
        if ((int64_t)open > err_off) {
          err_off = open;
          err_cls = st;
        }
        if (depth) poison |= 1u << (depth - 1);
      } else if (wrapping) {
        wrap_e = e;
      }
      prev = c;
      i++;
      continue;
    }
    IE_PUT(c);
    prev = c;
    i++;
  }
#undef IE_PUT
  out_len = olen;
  if (nopen == 0) return IE_OK_STR;                  // no loop at all (py:516)
  if (nopen != nclose) return IE_E_ASSERT_BRACES;    // py:517-519
  if (negclose) return kStatusPending;               // balanced but '}{': py break / rs panic
  if (err_off >= 0) return err_cls;
  if (wrap_e >= 0) {
    vid = T.entries[wrap_e].vid;
    out_len = 0;
    return IE_OK_VALUE;
  }
  return IE_OK_STR;
}

// recursive_unescape / recursive_escape on one string (py:1436-1460). Both replace passes are
// fused into one: neither pass can create or destroy a match of the other.
template <int OP>
__device__ uint8_t eval_escape(const uint8_t* __restrict__ s, uint32_t n, uint8_t* __restrict__ out,
                               uint32_t& out_len, bool emit) {
  uint32_t w = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t c = s[i];
    if (OP == kOpUnescape) {
      if (c == '\\' && i + 1 < n && (s[i + 1] == '{' || s[i + 1] == '}')) {
        if (emit) out[w] = s[i + 1];
        w++;
        i++;
        continue;
      }
    } else {
      if (c == '{' || c == '}') {
        if (emit) out[w] = '\\';
        w++;
      }
    }
    if (emit) out[w] = c;
    w++;
  }
  out_len = w;
  return IE_OK_STR;
}

// ------------------------------------------------------------------------------------------
// workgroup helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// exclusive scan over the workgroup; returns this lane's prefix, *total = sum
__device__ uint64_t block_excl_scan(uint64_t v, uint64_t* lds_w /*kBlock/64*/, uint64_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t inc = wave_incl_scan(v);
  if (lane == 63) lds_w[wid] = inc;
  __syncthreads();
  uint64_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kBlock / 64; w++) {
    const uint64_t x = lds_w[w];
    if (w < wid) base += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

// Stage bytes [lo, hi) of the batch into LDS so that LDS position p holds byte (lo16 + p) where
// lo16 = lo rounded down to 16 B. Body with 16-byte loads, ragged head/tail byte by byte (never
// touches bytes outside [lo, hi)). Returns the LDS offset of byte `lo`.
__device__ uint32_t stage_tile(const uint8_t* __restrict__ bytes, uint64_t lo, uint64_t hi,
                               uint8_t* lds) {
  const uintptr_t plo = (uintptr_t)(bytes + lo), phi = (uintptr_t)(bytes + hi);
  const uintptr_t a_down = plo & ~(uintptr_t)15;
  const uintptr_t a_up = (plo + 15) & ~(uintptr_t)15;
  const uintptr_t b_down = phi & ~(uintptr_t)15;
  const uint32_t shift = (uint32_t)(plo - a_down);
  if (a_up >= b_down) {  // tiny tile: bytewise
    for (uint32_t j = threadIdx.x; j < (uint32_t)(phi - plo); j += kBlock)
      lds[shift + j] = ((const uint8_t*)plo)[j];
  } else {
    const uint32_t head = (uint32_t)(a_up - plo), tail = (uint32_t)(phi - b_down);
    if (threadIdx.x < head) lds[shift + threadIdx.x] = ((const uint8_t*)plo)[threadIdx.x];
    if (threadIdx.x < tail) lds[(uint32_t)(b_down - a_down) + threadIdx.x] = ((const uint8_t*)b_down)[threadIdx.x];
    const uint4* src = (const uint4*)a_up;
    uint4* dst = (uint4*)(lds + (a_up - a_down));
    const uint32_t nv = (uint32_t)((b_down - a_up) >> 4);
    for (uint32_t j = threadIdx.x; j < nv; j += kBlock) dst[j] = src[j];
  }
  return shift;
}

// ------------------------------------------------------------------------------------------
// k_measure
// ------------------------------------------------------------------------------------------
template <int OP>
__global__ __launch_bounds__(kBlock) void k_measure(Batch B, Work W, DevTable T) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kTileBytes + 32];
  __shared__ __attribute__((aligned(16))) uint8_t s_key[kBlock * kKeyCap];
  __shared__ uint32_t s_open[kMaxDepth * kBlock];
  __shared__ uint16_t s_kstart[kMaxDepth * kBlock];
  __shared__ uint64_t s_red[kBlock / 64];

  const uint64_t tile = blockIdx.x;
  const uint64_t first = tile * kBlock;
  const uint64_t i = first + threadIdx.x;
  const uint64_t last = min(first + kBlock, B.n);  // exclusive
  const uint64_t lo = B.in_off[first], hi = B.in_off[last];
  const bool staged = (hi - lo) <= kTileBytes;
  uint32_t shift = 0;
  if (staged) shift = stage_tile(B.bytes, lo, hi, s_in);
  __syncthreads();

  uint64_t my_len = 0;
  if (i < B.n) {
    const uint64_t so = B.in_off[i], eo = B.in_off[i + 1];
    const uint8_t* s = staged ? s_in + shift + (so - lo) : B.bytes + so;
    const uint64_t n = eo - so;
    uint32_t olen = 0, vid = IE_VID_NONE;
    uint8_t st;
    if (OP == kOpInterp) {
      if (n >= 0xFFFF0000ull) {
        st = kStatusPending;
      } else {
        LaneScratch L{s_key + threadIdx.x * kKeyCap, s_open + threadIdx.x, s_kstart + threadIdx.x};
        st = eval_fast<false>(T, s, (uint32_t)n, L, nullptr, olen, vid);
      }
    } else {
      st = eval_escape<OP>(s, (uint32_t)n, nullptr, olen, false);
    }
    if (st == kStatusPending) {
      const uint32_t slot = atomicAdd(W.cx_count, 1u);
      W.cx_list[slot] = (uint32_t)i;
      W.out_len[i] = 0;
    } else {
      W.out_len[i] = (st == IE_OK_STR) ? olen : 0;
      if (st == IE_OK_STR) my_len = olen;
      if (st == IE_OK_VALUE) B.value_id[i] = vid;
    }
    B.status[i] = st;
  }
  uint64_t total;
  block_excl_scan(my_len, s_red, &total);
  if (threadIdx.x == 0) W.tile_sum[tile] = total;
}

// ------------------------------------------------------------------------------------------
// k_literal: py:497-541 restated on bytes, ONE WAVE per complex string, global scratch.
// Every str method the reference applies is a wave-parallel pass, 64 bytes per step: the
// patterns involved ('\{', '\}', '.〠', '〠.') cannot overlap themselves, so "non-overlapping,
// left to right" equals "every occurrence" and each byte decides its fate locally; a wave
// prefix sum then places the output. The two restore passes stay sequential (their order
// matters: '.〠.' must become '\{.').
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ uint64_t w_sum(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}
__device__ __forceinline__ int64_t w_max(int64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const int64_t o = __shfl_xor(v, d, 64);
    v = o > v ? o : v;
  }
  return v;
}
// the lanes' global stores become visible to the other lanes' loads of the next pass
__device__ __forceinline__ void w_phase() { __threadfence_block(); }

__device__ __forceinline__ bool is_ph_start(const uint8_t* p, uint64_t k, uint64_t n) {
  return k + 4 <= n && p[k] == '.' && p[k + 1] == 0xE3 && p[k + 2] == 0x80 && p[k + 3] == 0xA0;
}
__device__ __forceinline__ bool is_ph_stop(const uint8_t* p, uint64_t k, uint64_t n) {
  return k + 4 <= n && p[k] == 0xE3 && p[k + 1] == 0x80 && p[k + 2] == 0xA0 && p[k + 3] == '.';
}
__device__ __forceinline__ bool is_brace(uint8_t c) { return c == '{' || c == '}'; }

enum { kPatProtect = 0, kPatRestoreOpen = 1, kPatRestoreClose = 2 };
constexpr uint64_t kOverflow = ~0ull;

// dst = src.replace(...) for one pattern family; returns the length or kOverflow (> cap).
//   kPatProtect:      '\{' -> '.〠' and '\}' -> '〠.'  (py:505-508, fused: see DESIGN.md)
//   kPatRestoreOpen:  '.〠' -> '\{'                     (py:526, 538)
//   kPatRestoreClose: '〠.' -> '\}'                     (py:527, 539)
// kPatProtect may look one byte past n at `seam` (the next byte of a virtual concatenation);
// *seam_used reports that a trailing '\' consumed it.
template <int PAT>
__device__ uint64_t w_replace(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap,
                              int seam = -1, bool* seam_used = nullptr) {
  const uint32_t lane = lane_id();
  uint64_t w = 0;
  for (uint64_t base = 0; base < n; base += 64) {
    const uint64_t k = base + lane;
    uint32_t len = 0;
    uint8_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
    if (k < n) {
      const uint8_t c = src[k];
      if (PAT == kPatProtect) {
        const int nx = (k + 1 < n) ? (int)src[k + 1] : seam;
        if (c == '\\' && (nx == '{' || nx == '}')) {
          len = 4;
          if (nx == '{') { r0 = '.'; r1 = 0xE3; r2 = 0x80; r3 = 0xA0; }
          else { r0 = 0xE3; r1 = 0x80; r2 = 0xA0; r3 = '.'; }
        } else if (k >= 1 && src[k - 1] == '\\' && is_brace(c)) {
          len = 0;  // second byte of a match ('\' is never the second byte of one)
        } else {
          len = 1;
          r0 = c;
        }
      } else {
        const bool open = PAT == kPatRestoreOpen;
        if (open ? is_ph_start(src, k, n) : is_ph_stop(src, k, n)) {
          len = 2;
          r0 = '\\';
          r1 = open ? '{' : '}';
        } else {
          bool inside = false;
          for (uint64_t j = 1; j <= 3 && j <= k; j++)
            inside |= open ? is_ph_start(src, k - j, n) : is_ph_stop(src, k - j, n);
          len = inside ? 0 : 1;
          r0 = c;
        }
      }
    }
    const uint64_t incl = wave_incl_scan(len);
    const uint64_t tot = __shfl(incl, 63, 64);
    if (w + tot > cap) return kOverflow;
    const uint64_t pos = w + incl - len;
    if (len >= 1) dst[pos] = r0;
    if (len >= 2) dst[pos + 1] = r1;
    if (len >= 4) { dst[pos + 2] = r2; dst[pos + 3] = r3; }
    w += tot;
  }
  if (PAT == kPatProtect && seam_used) {
    *seam_used = n > 0 && src[n - 1] == '\\' && (seam == '{' || seam == '}');
  }
  w_phase();
  return w;
}

__device__ void w_copy(uint8_t* dst, const uint8_t* src, uint64_t n) {
  for (uint64_t k = lane_id(); k < n; k += 64) dst[k] = src[k];
}

// content.find('{') / count('{') / count('}') / rfind('{') in one pass
struct BraceScan {
  uint64_t n_open, n_close;
  int64_t last_open;
};
__device__ BraceScan w_scan_braces(const uint8_t* p, uint64_t n) {
  uint64_t no = 0, nc = 0;
  int64_t lo = -1;
  for (uint64_t k = lane_id(); k < n; k += 64) {
    const uint8_t c = p[k];
    if (c == '{') { no++; lo = (int64_t)k; }
    if (c == '}') nc++;
  }
  return BraceScan{w_sum(no), w_sum(nc), w_max(lo)};
}

// content.find(ch, from)
__device__ int64_t w_find(const uint8_t* p, uint64_t from, uint64_t n, uint8_t ch) {
  for (uint64_t base = from; base < n; base += 64) {
    const uint64_t k = base + lane_id();
    const uint64_t m = __ballot(k < n && p[k] == ch);
    if (m) return (int64_t)(base + (uint64_t)__ffsll((long long)m) - 1);
  }
  return -1;
}

// get_simple_insertkey on protected bytes (py:477-495 / interp.rs:11-29): truthy / Some.
// Byte-level equals the code-point loop: only ASCII '{' / '}' positions matter.
__device__ bool w_simple(uint32_t dialect, const uint8_t* p, uint64_t n) {
  if (dialect == IE_DIALECT_RS) {
    if (n < 2 || p[0] != '{' || p[n - 1] != '}') return false;
    if (n == 2) return true;  // Some("")
  } else if (n < 3 || p[0] != '{' || p[n - 1] != '}') {
    return false;
  }
  uint64_t carry = 0;  // signed sums in two's complement
  for (uint64_t base = 0; base < n; base += 64) {
    const uint64_t k = base + lane_id();
    uint64_t e = 0;
    bool close = false;
    if (k < n) {
      const uint8_t c = p[k];
      e = c == '{' ? 1ull : (c == '}' ? ~0ull : 0ull);
      close = c == '}';
    }
    const uint64_t incl = wave_incl_scan(e);
    const uint64_t depth = carry + incl - e - (close ? 1ull : 0ull);  // after the decrement at k
    const bool edge = (k == 0 || k == n - 1);
    if (__ballot(k < n && ((depth == 0) != edge))) return false;
    carry += __shfl(incl, 63, 64);
  }
  return true;
}

struct LitOut {
  uint8_t status;
  uint64_t res_off;  // pool offset of the result bytes
  uint64_t res_len;
  uint32_t vid;
};

// One complex string, executed by all 64 lanes of a wave with uniform control flow.
// Scratch: four regions of `cap` bytes at R[0..3] (pool offset `pool_off` of R[0]).
__device__ LitOut w_literal(const DevTable& T, const uint8_t* s, uint64_t n, uint8_t* R0,
                            uint64_t cap, uint64_t pool_off) {
  LitOut r{0, 0, 0, IE_VID_NONE};
  uint8_t* R[4] = {R0, R0 + cap, R0 + 2 * cap, R0 + 3 * cap};
  uint8_t* K = R[2];
  uint8_t* K2 = R[3];
  const uint64_t alen = w_replace<kPatProtect>(s, n, R[0], cap);  // py:505-508
  if (alen == kOverflow) { r.status = IE_E_OVERFLOW; return r; }
  // whole-string levels (py:510-514): each is get_interpdata(interpolate_inserts(inner))
  uint64_t cur = 0, clen = alen;
  uint32_t W = 0;
  for (;;) {
    if (W > 900) { r.status = IE_DIVERGED; return r; }  // CPython's recursion limit (oracle twin)
    if (!w_simple(T.dialect, R[0] + cur, clen)) break;
    cur += 1;
    clen -= 2;
    W++;
  }
  const uint64_t n0 = W ? clen : n;
  const uint64_t iter_cap = IE_ITER_CAP(n0);
  const uint64_t size_cap = IE_SIZE_CAP(n0, T.maxtext);
  int si = 0;
  uint8_t* src = R[0] + cur;
  uint64_t slen = clen;
  uint64_t iters = 0;
  for (;;) {
    const BraceScan bs = w_scan_braces(src, slen);
    if (bs.n_open == 0) break;  // py:516
    if (++iters > iter_cap || slen > size_cap) { r.status = IE_DIVERGED; return r; }
    // count('\\{') is 0 on protected content, so py:517-518 reduce to the raw counts
    if (bs.n_open != bs.n_close) { r.status = IE_E_ASSERT_BRACES; return r; }
    const uint64_t outer_from = (uint64_t)bs.last_open;                 // py:520
    const int64_t inner_to = w_find(src, outer_from + 1, slen, '}');    // py:521
    if (inner_to < 0) {
      if (T.dialect == IE_DIALECT_RS) { r.status = IE_E_RS_PANIC; return r; }  // interp.rs:63-66
      break;                                                                    // py:522
    }
    // py:525-528 the key with placeholders restored
    const uint64_t k1 = w_replace<kPatRestoreOpen>(src + outer_from + 1, (uint64_t)inner_to - outer_from - 1, K, cap);
    const uint64_t k2 = w_replace<kPatRestoreClose>(K, k1, K2, cap);
    const int32_t e = table_find(T, K2, (uint32_t)k2);                  // py:529
    if (e < 0) { r.status = missing_status(T, K2, (uint32_t)k2); return r; }
    const DevEntry& E = T.entries[e];
    if (!(E.flags & EF_SPLICE_OK)) { r.status = IE_E_ASSERT_TYPE; return r; }  // py:530
    // py:531-535: prefix (protected already, never ends in '\') + protect(text | seam) + suffix
    uint8_t* dst = R[si ^ 1];
    const uint8_t* suf = src + inner_to + 1;
    const uint64_t sl = slen - (uint64_t)inner_to - 1;
    w_copy(dst, src, outer_from);
    bool seam_used = false;
    const uint64_t tw = w_replace<kPatProtect>(T.arena + E.text_off, E.text_len, dst + outer_from,
                                               cap - outer_from, sl ? (int)suf[0] : -1, &seam_used);
    if (tw == kOverflow) { r.status = IE_E_OVERFLOW; return r; }
    const uint64_t skip = seam_used ? 1 : 0;
    if (outer_from + tw + sl - skip > cap) { r.status = IE_E_OVERFLOW; return r; }
    w_copy(dst + outer_from + tw, suf + skip, sl - skip);
    w_phase();
    si ^= 1;
    src = dst;
    slen = outer_from + tw + sl - skip;
  }
  // py:537-540: restore into the other buffer, then into K
  uint8_t* other = R[si ^ 1];
  const uint64_t f1 = w_replace<kPatRestoreOpen>(src, slen, other, cap);
  const uint64_t f2 = w_replace<kPatRestoreClose>(other, f1, K, cap);
  if (W == 0) {
    r.status = IE_OK_STR;
    r.res_off = pool_off + 2 * cap;
    r.res_len = f2;
    return r;
  }
  // typed result: W lookups, the first on the string, then on raw values (py:512 / interp.rs:48)
  uint8_t st = 0;
  int32_t e = table_find(T, K, (uint32_t)f2);
  if (e < 0) { r.status = missing_status(T, K, (uint32_t)f2); return r; }
  for (uint32_t k = 1; k < W; k++) {
    if (T.dialect == IE_DIALECT_PY) {
      e = table_find_raw(T, e, st);
    } else {
      const DevEntry& P = T.entries[e];
      const int32_t e2 = table_find(T, T.arena + P.text_off, P.text_len);
      if (e2 < 0) st = missing_status(T, T.arena + P.text_off, P.text_len);
      e = e2;
    }
    if (e < 0) { r.status = st; return r; }
  }
  r.status = IE_OK_VALUE;
  r.vid = T.entries[e].vid;
  return r;
}

__global__ __launch_bounds__(kBlock) void k_literal(Batch B, Work W, DevTable T) {
  const uint32_t count = *W.cx_count;
  const uint32_t waves = gridDim.x * (kBlock / 64);
  const uint32_t wid = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  for (uint32_t j = wid; j < count; j += waves) {
    const uint32_t i = W.cx_list[j];
    const uint64_t so = B.in_off[i], n = B.in_off[i + 1] - so;
    uint64_t cap = W.lit_cap_max ? IE_SIZE_CAP(n, T.maxtext) + 4 * T.maxtext + 64
                                 : 4 * n + 4 * T.maxtext + 256;
    cap = (cap + 15) & ~15ull;
    const uint64_t need = 4 * cap;
    uint64_t base = 0;
    if (lane_id() == 0) base = atomicAdd((unsigned long long*)W.pool_used, (unsigned long long)need);
    base = __shfl(base, 0, 64);
    LitOut r;
    if (base + need > W.pool_bytes) {
      r = LitOut{IE_E_OVERFLOW, 0, 0, IE_VID_NONE};
    } else {
      r = w_literal(T, B.bytes + so, n, W.pool + base, cap, base);
    }
    if (lane_id() == 0) {
      W.cx_status[i] = r.status;
      if (r.status == IE_OK_STR) {
        W.out_len[i] = (uint32_t)r.res_len;
        W.res_off[i] = r.res_off;
        atomicAdd((unsigned long long*)&W.tile_sum[i / kBlock], (unsigned long long)r.res_len);
      } else {
        W.out_len[i] = 0;
        if (r.status == IE_OK_VALUE) B.value_id[i] = r.vid;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// k_scan_tiles: one workgroup, exclusive scan of tile sums (chunked), grand total.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_scan_tiles(Work W, uint64_t n_tiles, uint64_t* total,
                                                       uint64_t* offsets_n) {
  __shared__ uint64_t s_red[kBlock / 64];
  const uint64_t per = (n_tiles + kBlock - 1) / kBlock;
  const uint64_t b = threadIdx.x * per, e = min(b + per, n_tiles);
  uint64_t sum = 0;
  for (uint64_t t = b; t < e; t++) sum += W.tile_sum[t];
  uint64_t tot;
  uint64_t run = block_excl_scan(sum, s_red, &tot);
  for (uint64_t t = b; t < e; t++) {
    const uint64_t v = W.tile_sum[t];
    W.tile_base[t] = run;
    run += v;
  }
  if (threadIdx.x == 0) {
    *total = tot;
    *offsets_n = tot;
  }
}

// ------------------------------------------------------------------------------------------
// k_emit
// ------------------------------------------------------------------------------------------
template <int OP>
__global__ __launch_bounds__(kBlock) void k_emit(Batch B, Work W, DevTable T, uint8_t* out_bytes,
                                                 uint64_t out_cap, const uint64_t* total) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kTileBytes + 32];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kStageBytes + 32];
  __shared__ __attribute__((aligned(16))) uint8_t s_key[kBlock * kKeyCap];
  __shared__ uint32_t s_open[kMaxDepth * kBlock];
  __shared__ uint16_t s_kstart[kMaxDepth * kBlock];
  __shared__ uint64_t s_red[kBlock / 64];

  const uint64_t tile = blockIdx.x;
  const uint64_t first = tile * kBlock;
  const uint64_t i = first + threadIdx.x;
  const uint64_t last = min(first + kBlock, B.n);
  const uint64_t base = W.tile_base[tile];
  const bool write_bytes = *total <= out_cap;

  const uint32_t my_len = (i < B.n) ? W.out_len[i] : 0;
  uint64_t tile_out;
  const uint64_t local = block_excl_scan(my_len, s_red, &tile_out);
  bool was_cx = false;
  uint8_t st = 0;
  if (i < B.n) {
    B.out_off[i] = base + local;
    st = B.status[i];
    if (OP == kOpInterp && st == kStatusPending) {  // final status of a literal-path string
      was_cx = true;
      st = W.cx_status[i];
      B.status[i] = st;
    }
  }
  if (!write_bytes) return;  // uniform across the workgroup

  const uint64_t lo = B.in_off[first], hi = B.in_off[last];
  const bool staged_in = (hi - lo) <= kTileBytes;
  const uint32_t oshift = (uint32_t)(((uintptr_t)(out_bytes + base)) & 15);
  const bool staged_out = tile_out + oshift <= kStageBytes;
  uint32_t shift = 0;
  if (staged_in) shift = stage_tile(B.bytes, lo, hi, s_in);
  __syncthreads();

  if (i < B.n && my_len) {
    uint8_t* dst = staged_out ? s_out + oshift + local : out_bytes + base + local;
    if (was_cx) {  // the literal kernel left the result in the pool
      const uint8_t* src = W.pool + W.res_off[i];
      for (uint32_t j = 0; j < my_len; j++) dst[j] = src[j];
    } else {
      const uint64_t so = B.in_off[i], n = B.in_off[i + 1] - so;
      const uint8_t* s = staged_in ? s_in + shift + (so - lo) : B.bytes + so;
      uint32_t olen = 0, vid = 0;
      if (OP == kOpInterp) {
        LaneScratch L{s_key + threadIdx.x * kKeyCap, s_open + threadIdx.x, s_kstart + threadIdx.x};
        eval_fast<true>(T, s, (uint32_t)n, L, dst, olen, vid);
      } else {
        eval_escape<OP>(s, (uint32_t)n, dst, olen, true);
      }
    }
  }
  if (!staged_out) return;
  __syncthreads();
  // stream the stage out: LDS position oshift + k holds output byte base + k
  uint8_t* g = out_bytes + base;
  const uintptr_t pg = (uintptr_t)g, pe = pg + tile_out;
  const uintptr_t a_up = (pg + 15) & ~(uintptr_t)15, b_down = pe & ~(uintptr_t)15;
  if (a_up >= b_down) {
    for (uint32_t k = threadIdx.x; k < tile_out; k += kBlock) g[k] = s_out[oshift + k];
  } else {
    const uint32_t head = (uint32_t)(a_up - pg), tail = (uint32_t)(pe - b_down);
    if (threadIdx.x < head) g[threadIdx.x] = s_out[oshift + threadIdx.x];
    if (threadIdx.x < tail) {
      const uint32_t k = (uint32_t)(b_down - pg) + threadIdx.x;
      g[k] = s_out[oshift + k];
    }
    const uint32_t nv = (uint32_t)((b_down - a_up) >> 4);
    const uint4* src = (const uint4*)(s_out + oshift + head);
    uint4* dstv = (uint4*)a_up;
    for (uint32_t j = threadIdx.x; j < nv; j += kBlock) dstv[j] = src[j];
  }
}

// ------------------------------------------------------------------------------------------
// synthetic string generation on the device
// ------------------------------------------------------------------------------------------
__global__ void k_synth_len(SynthParams P, uint64_t first, uint64_t n, uint64_t* lens) {
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x)
    lens[k] = synth_len(P, first + k);
}

__global__ void k_synth_fill(SynthParams P, uint64_t first, uint64_t n, const uint64_t* offsets,
                             uint8_t* bytes) {
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x)
    synth_string(P, first + k, bytes + offsets[k]);
}

// generic exclusive scan of n u64 values into out[0..n] (out[n] = total), 3 phases
__global__ __launch_bounds__(kBlock) void k_scan_a(const uint64_t* in, uint64_t n, uint64_t* part) {
  __shared__ uint64_t s_red[kBlock / 64];
  const uint64_t per = kBlock * 16;
  const uint64_t b = blockIdx.x * per;
  uint64_t sum = 0;
  for (uint64_t k = b + threadIdx.x; k < min(b + per, n); k += kBlock) sum += in[k];
  uint64_t tot;
  block_excl_scan(sum, s_red, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_scan_b(uint64_t* part, uint64_t nparts, uint64_t* total) {
  __shared__ uint64_t s_red[kBlock / 64];
  const uint64_t per = (nparts + kBlock - 1) / kBlock;
  const uint64_t b = threadIdx.x * per, e = min(b + per, nparts);
  uint64_t sum = 0;
  for (uint64_t t = b; t < e; t++) sum += part[t];
  uint64_t tot;
  uint64_t run = block_excl_scan(sum, s_red, &tot);
  for (uint64_t t = b; t < e; t++) {
    const uint64_t v = part[t];
    part[t] = run;
    run += v;
  }
  if (threadIdx.x == 0) *total = tot;
}

__global__ __launch_bounds__(kBlock) void k_scan_c(const uint64_t* in, uint64_t n, const uint64_t* part,
                                                   uint64_t* out) {
  __shared__ uint64_t s_red[kBlock / 64];
  const uint64_t per = kBlock * 16;
  const uint64_t b = blockIdx.x * per;
  uint64_t run = part[blockIdx.x];
  for (uint64_t c = b; c < min(b + per, n); c += kBlock) {
    const uint64_t k = c + threadIdx.x;
    const uint64_t v = k < n ? in[k] : 0;
    uint64_t tot;
    const uint64_t ex = block_excl_scan(v, s_red, &tot);
    if (k < n) out[k] = run + ex;
    run += tot;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = run;
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
hipError_t launch_measure(int op, const Batch& B, const Work& W, const DevTable& T, hipStream_t st) {
  const uint64_t tiles = (B.n + kBlock - 1) / kBlock;
  if (!tiles) return hipSuccess;
  if (op == kOpInterp) hipLaunchKernelGGL(k_measure<kOpInterp>, dim3((uint32_t)tiles), dim3(kBlock), 0, st, B, W, T);
  else if (op == kOpUnescape) hipLaunchKernelGGL(k_measure<kOpUnescape>, dim3((uint32_t)tiles), dim3(kBlock), 0, st, B, W, T);
  else hipLaunchKernelGGL(k_measure<kOpEscape>, dim3((uint32_t)tiles), dim3(kBlock), 0, st, B, W, T);
  return hipGetLastError();
}

hipError_t launch_literal(const Batch& B, const Work& W, const DevTable& T, hipStream_t st) {
  hipLaunchKernelGGL(k_literal, dim3(1024), dim3(kBlock), 0, st, B, W, T);
  return hipGetLastError();
}

hipError_t launch_scan_tiles(const Batch& B, const Work& W, uint64_t* total, hipStream_t st) {
  const uint64_t tiles = (B.n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, st, W, tiles, total, B.out_off + B.n);
  return hipGetLastError();
}

hipError_t launch_emit(int op, const Batch& B, const Work& W, const DevTable& T, uint8_t* out,
                       uint64_t cap, const uint64_t* total, hipStream_t st) {
  const uint64_t tiles = (B.n + kBlock - 1) / kBlock;
  if (!tiles) return hipSuccess;
  if (op == kOpInterp) hipLaunchKernelGGL(k_emit<kOpInterp>, dim3((uint32_t)tiles), dim3(kBlock), 0, st, B, W, T, out, cap, total);
  else if (op == kOpUnescape) hipLaunchKernelGGL(k_emit<kOpUnescape>, dim3((uint32_t)tiles), dim3(kBlock), 0, st, B, W, T, out, cap, total);
  else hipLaunchKernelGGL(k_emit<kOpEscape>, dim3((uint32_t)tiles), dim3(kBlock), 0, st, B, W, T, out, cap, total);
  return hipGetLastError();
}

hipError_t launch_synth(const SynthParams& P, uint64_t first, uint64_t n, uint64_t* d_lens,
                        uint64_t* d_part, uint64_t* d_offsets, uint64_t* d_total, uint8_t* d_bytes,
                        hipStream_t st) {
  if (!n) return hipSuccess;
  const uint64_t g0 = (n + 255) / 256;
  const uint32_t g = (uint32_t)(g0 < 4096 ? g0 : 4096);
  if (!d_bytes) {
    hipLaunchKernelGGL(k_synth_len, dim3(g), dim3(256), 0, st, P, first, n, d_lens);
    const uint64_t per = kBlock * 16, nparts = (n + per - 1) / per;
    hipLaunchKernelGGL(k_scan_a, dim3((uint32_t)nparts), dim3(kBlock), 0, st, d_lens, n, d_part);
    hipLaunchKernelGGL(k_scan_b, dim3(1), dim3(kBlock), 0, st, d_part, nparts, d_total);
    hipLaunchKernelGGL(k_scan_c, dim3((uint32_t)nparts), dim3(kBlock), 0, st, d_lens, n, d_part, d_offsets);
  } else {
    hipLaunchKernelGGL(k_synth_fill, dim3(g), dim3(256), 0, st, P, first, n, d_offsets, d_bytes);
  }
  return hipGetLastError();
}

}  // namespace ie
