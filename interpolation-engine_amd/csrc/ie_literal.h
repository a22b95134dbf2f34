// ie_literal.h — the literal path: interpolate_inserts (py:497-541 / interp.rs:31-89)
// restated on bytes for ONE string, executed by all 64 lanes of a wave with uniform control
// flow, working copies in global scratch (four regions of `cap` bytes).
#pragma once
#include "ie_device.h"

namespace ie {

constexpr uint64_t kLitIterBudget = 2048;  // substitutions allowed outside max mode

// ------------------------------------------------------------------------------------------
// py:497-541 restated on bytes, ONE WAVE per complex string, global scratch.
// Every str method the reference applies is a wave-parallel pass, 64 bytes per step: the
// patterns involved ('\{', '\}', '.〠', '〠.') cannot overlap themselves, so "non-overlapping,
// left to right" equals "every occurrence" and each byte decides its fate locally; a wave
// prefix sum then places the output. The two restore passes stay sequential (their order
// matters: '.〠.' must become '\{.').
// ------------------------------------------------------------------------------------------
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

// get_simple_insertkey on protected bytes (py:477-495 / interp.rs:11-29): truthy / Some, with
// l0 / ll the byte lengths of the first and the last character (content[1:-1] drops them). The
// py rule has no brace test at the edges ('a}b{c' is simple: ie_common.h simple_insertkey), so
// the depth test skips continuation bytes and treats the first and last CHARACTER as the edges.
// Wave-uniform; every lane returns the same.
__device__ bool w_simple(uint32_t dialect, const uint8_t* p, uint64_t n, uint64_t& l0, uint64_t& ll) {
  l0 = ll = 0;
  if (n == 0) return false;
  if (dialect == IE_DIALECT_RS && (n < 2 || p[0] != '{' || p[n - 1] != '}')) return false;
  // the first character's bytes and the last character's first byte (at most 3 bytes back)
  const uint8_t c0 = p[0];
  const uint64_t f = c0 < 0x80u ? 1u : (c0 & 0xE0u) == 0xC0u ? 2u : (c0 & 0xF0u) == 0xE0u ? 3u : 4u;
  uint64_t last = n - 1;
  while (last > 0 && last + 3 >= n && (p[last] & 0xC0u) == 0x80u) last--;
  // py: content[1:-1] must be non-empty (3+ characters); rs: Some("") for "{}"
  if (dialect != IE_DIALECT_RS && last <= f) return false;
  uint64_t carry = 0;  // signed sums in two's complement
  for (uint64_t base = 0; base < n; base += 64) {
    const uint64_t k = base + lane_id();
    uint64_t e = 0;
    bool close = false, lead = false;
    if (k < n) {
      const uint8_t c = p[k];
      lead = (c & 0xC0u) != 0x80u;
      e = c == '{' ? 1ull : (c == '}' ? ~0ull : 0ull);
      close = c == '}';
    }
    const uint64_t incl = wave_incl_scan(e);
    const uint64_t depth = carry + incl - e - (close ? 1ull : 0ull);  // after the decrement at k
    const bool edge = (k == 0 || k == last);
    if (__ballot(k < n && lead && ((depth == 0) != edge))) return false;
    carry += __shfl(incl, 63, 64);
  }
  l0 = f < n ? f : n;
  ll = n - last;
  return true;
}

struct LitOut {
  uint8_t status;
  uint64_t res_off;  // pool offset of the result bytes
  uint64_t res_len;
  uint32_t vid;
  uint32_t flags;    // the entry flags of an IE_OK_VALUE result
  const uint8_t* key;  // IE_NEEDS_HOST / IE_E_INTERP: the missing key's bytes (pool or arena), key_len
  uint32_t key_len;
};

// One complex string, executed by all 64 lanes of a wave with uniform control flow.
// Scratch: four regions of `cap` bytes at R[0..3] (pool offset `pool_off` of R[0]).
__device__ LitOut w_literal(const DevTable T, uint32_t tid, const uint8_t* s, uint64_t n, uint8_t* R0,
                            uint64_t cap, uint64_t pool_off, bool max_mode) {
  LitOut r{0, 0, 0, IE_VID_NONE, 0, nullptr, 0};
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
    uint64_t l0, ll;
    if (!w_simple(T.dialect, R[0] + cur, clen, l0, ll)) break;
    cur += l0;
    clen -= l0 + ll;
    W++;
  }
  const uint64_t n0 = W ? clen : n;
  const uint64_t iter_cap = IE_ITER_CAP(n0);
  const uint64_t size_cap = IE_SIZE_CAP(n0, T.maxtext);
  // outside max mode a string gets a small budget so one runaway string cannot hold up the
  // single-pass chain; exceeding it (before the reference's own caps) reports IE_E_OVERFLOW and
  // the host API re-runs the string in max mode
  const uint64_t iter_budget = max_mode ? iter_cap : (iter_cap < kLitIterBudget ? iter_cap : kLitIterBudget);
  int si = 0;
  uint8_t* src = R[0] + cur;
  uint64_t slen = clen;
  uint64_t iters = 0;
  for (;;) {
    const BraceScan bs = w_scan_braces(src, slen);
    if (bs.n_open == 0) break;  // py:516
    if (++iters > iter_cap || slen > size_cap) { r.status = IE_DIVERGED; return r; }
    if (iters > iter_budget) { r.status = IE_E_OVERFLOW; return r; }
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
    Hit E;
    const int32_t e = find_bytes(T, tid, K2, (uint32_t)k2, E);                // py:529
    if (e < 0) {  // (the key stays in K2: k_resolve records it for the host)
      r.status = missing_status(T, K2, (uint32_t)k2);
      r.key = K2, r.key_len = (uint32_t)k2;
      return r;
    }
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
  Hit cur_hit;
  int32_t e = find_bytes(T, tid, K, (uint32_t)f2, cur_hit);
  if (e < 0) {
    r.status = missing_status(T, K, (uint32_t)f2);
    r.key = K, r.key_len = (uint32_t)f2;
    return r;
  }
  for (uint32_t k = 1; k < W; k++) {
    Hit nh;
    e = find_raw(T, tid, cur_hit, st, nh);  // rs: every raw value has EF_KEY_STR (value_to_string)
    if (e < 0) {  // (the key: the raw value, as the message shows it)
      r.status = st;
      if (st == IE_E_INTERP) r.key = raw_text(T, cur_hit, r.key_len);
      return r;
    }
    cur_hit = nh;
  }
  r.status = IE_OK_VALUE;
  r.vid = cur_hit.vid;
  r.flags = cur_hit.flags;
  return r;
}

}  // namespace ie
