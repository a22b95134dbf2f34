// ie_bytes.h — byte and event-mask building blocks of the gfx950 kernels (k_resolve,
// k_emit_windows): LDS-typed views, unaligned LDS moves, chunk classification, 128-bit event masks.
#pragma once
#include "ie_device.h"

namespace ie {

// LDS-typed views: accesses through them compile to ds_* (not flat_*) instructions
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;
typedef __attribute__((address_space(3))) u32x4 lds_u128;

// ------------------------------------------------------------------------------------------
// Unaligned LDS access (gfx950 runs in unaligned mode: ds_read/ds_write_b32/b64/b128 take any
// byte address). Pieces are moved in 16-byte units; the last partial unit is stored with exact
// 8/4/2/1-byte stores so no lane ever writes past its own bytes.
// ------------------------------------------------------------------------------------------
typedef u32x4 __attribute__((aligned(1))) u32x4_ua;
typedef uint64_t __attribute__((aligned(1))) u64_ua;
typedef uint32_t __attribute__((aligned(1))) u32_ua;
typedef uint16_t __attribute__((aligned(1))) u16_ua;
typedef __attribute__((address_space(3))) u32x4_ua lds_v4u;
typedef __attribute__((address_space(3))) u64_ua lds_u64u;
typedef __attribute__((address_space(3))) u32_ua lds_u32u;
typedef __attribute__((address_space(3))) u16_ua lds_u16u;

__device__ __forceinline__ u32x4 ld16(const lds_u8* p) { return *(const lds_v4u*)p; }
__device__ __forceinline__ void st16(lds_u8* p, u32x4 v) { *(lds_v4u*)p = v; }

// the first len (0..16) bytes of v to p
__device__ __forceinline__ void st_part(lds_u8* p, u32x4 v, uint32_t len) {
  uint64_t lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
  const uint64_t hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
  if (len >= 16) {
    st16(p, v);
    return;
  }
  if (len & 8) {
    *(lds_u64u*)p = lo;
    lo = hi;
    p += 8;
  }
  if (len & 4) {
    *(lds_u32u*)p = (uint32_t)lo;
    lo >>= 32;
    p += 4;
  }
  if (len & 2) {
    *(lds_u16u*)p = (uint16_t)lo;
    lo >>= 16;
    p += 2;
  }
  if (len & 1) *p = (uint8_t)lo;
}

// len bytes LDS -> LDS, any alignments (reads up to 15 bytes past the source; the arrays are
// padded). Wave-uniform call.
__device__ __forceinline__ void lds_move(lds_u8* dst, const lds_u8* src, uint32_t len) {
  for (uint32_t k = 0; __any(k + 16 <= len); k += 16)
    if (k + 16 <= len) st16(dst + k, ld16(src + k));
  const uint32_t kt = len & ~15u;  // this lane's partial unit
  if (kt < len) st_part(dst + kt, ld16(src + kt), len - kt);
}

// v with the bytes at and past len (0..16) cleared
__device__ __forceinline__ u32x4 keep_bytes(u32x4 v, uint32_t len) {
  u32x4 r;
  const int32_t l = (int32_t)len;
  r.x = l >= 4 ? v.x : l > 0 ? v.x & ((1u << (8 * l)) - 1u) : 0u;
  r.y = l >= 8 ? v.y : l > 4 ? v.y & ((1u << (8 * (l - 4))) - 1u) : 0u;
  r.z = l >= 12 ? v.z : l > 8 ? v.z & ((1u << (8 * (l - 8))) - 1u) : 0u;
  r.w = l >= 16 ? v.w : l > 12 ? v.w & ((1u << (8 * (l - 12))) - 1u) : 0u;
  return r;
}

// v moved up by sh (0..16) bytes: byte i of the result is byte i - sh of v (zero below sh; bytes
// moved past 16 are dropped)
__device__ __forceinline__ u32x4 shl_bytes(u32x4 v, uint32_t sh) {
  const uint32_t q = sh >> 2, r = sh & 3u;
  const uint32_t w0 = q == 0 ? v.x : 0u;
  const uint32_t w1 = q == 0 ? v.y : q == 1 ? v.x : 0u;
  const uint32_t w2 = q == 0 ? v.z : q == 1 ? v.y : q == 2 ? v.x : 0u;
  const uint32_t w3 = q == 0 ? v.w : q == 1 ? v.z : q == 2 ? v.y : q == 3 ? v.x : 0u;
  if (r == 0) return u32x4{w0, w1, w2, w3};
  const uint32_t a = 4u - r;  // v_alignbyte: ({hi, lo} >> 8a)[31:0] = hi << 8r | lo >> (32 - 8r)
  return u32x4{__builtin_amdgcn_alignbyte(w0, 0u, a), __builtin_amdgcn_alignbyte(w1, w0, a),
               __builtin_amdgcn_alignbyte(w2, w1, a), __builtin_amdgcn_alignbyte(w3, w2, a)};
}

// 16 bytes at any LDS address from five aligned dword reads and v_alignbyte (a 16-byte access off
// its natural alignment is replayed at 64 cycles per wave-instruction; aligned dwords are not)
__device__ __forceinline__ u32x4 ld16a(const lds_u8* p) {
  const uint32_t sh = (uint32_t)(uintptr_t)p & 3u;
  const lds_u32* q = (const lds_u32*)(p - sh);
  const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
  return u32x4{__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
               __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
}

// the first n (< 16) bytes of v to a 4-aligned LDS address: dwords, then a short and a byte
__device__ __forceinline__ void put_tail4(lds_u8* p, u32x4 v, uint32_t n) {
  lds_u32* q = (lds_u32*)p;
  if (n >= 4) q[0] = v.x;
  if (n >= 8) q[1] = v.y;
  if (n >= 12) q[2] = v.z;
  const uint32_t nw = n >> 2, r = n & 3u;
  const uint32_t x = nw == 0 ? v.x : nw == 1 ? v.y : nw == 2 ? v.z : v.w;
  lds_u8* b = p + (n & ~3u);
  if (r & 2u) *(lds_u16*)b = (uint16_t)x;
  if (r & 1u) b[r & 2u] = (uint8_t)(x >> (8u * (r & 2u)));
}

// len bytes LDS -> LDS at any alignments with aligned accesses only: up to 3 head bytes until the
// destination is 4-aligned, then 4-aligned dwords from aligned source dwords. Wave-uniform call.
__device__ __forceinline__ void lds_copy(lds_u8* dst, const lds_u8* src, uint32_t len) {
  const uint32_t h0 = (0u - (uint32_t)(uintptr_t)dst) & 3u, h = h0 < len ? h0 : len;
  if (h > 0) dst[0] = src[0];
  if (h > 1) dst[1] = src[1];
  if (h > 2) dst[2] = src[2];
  const uint32_t body = (len - h) & ~15u;  // whole 16-byte units after the head
  for (uint32_t k = 0; __any(k < body); k += 16u) {
    if (k < body) {
      const u32x4 v = ld16a(src + h + k);
      lds_u32* q = (lds_u32*)(dst + h + k);
      q[0] = v.x, q[1] = v.y, q[2] = v.z, q[3] = v.w;
    }
  }
  const uint32_t kt = h + body;
  if (kt < len) put_tail4(dst + kt, ld16a(src + kt), len - kt);
}

// len (<= 28) bytes held as 8 little-endian words (zero past the text) to any LDS address:
// head bytes, then 4-aligned dwords realigned in registers
__device__ __forceinline__ void put_words(lds_u8* dst, const uint32_t (&t)[8], uint32_t len) {
  const uint32_t h0 = (0u - (uint32_t)(uintptr_t)dst) & 3u, h = h0 < len ? h0 : len;
  if (h > 0) dst[0] = (uint8_t)t[0];
  if (h > 1) dst[1] = (uint8_t)(t[0] >> 8);
  if (h > 2) dst[2] = (uint8_t)(t[0] >> 16);
  const uint32_t rest = len - h, nfull = rest >> 2, r = rest & 3u;
  lds_u32* q = (lds_u32*)(dst + h);
  uint32_t last = 0;
#pragma unroll
  for (int k = 0; k < 7; k++) {
    const uint32_t a = __builtin_amdgcn_alignbyte(t[k + 1], t[k], h);  // text bytes h+4k .. h+4k+3
    if ((uint32_t)k < nfull) q[k] = a;
    last = (uint32_t)k == nfull ? a : last;
  }
  lds_u8* b = dst + h + 4u * nfull;
  if (r & 2u) *(lds_u16*)b = (uint16_t)last;
  if (r & 1u) b[r & 2u] = (uint8_t)(last >> (8u * (r & 2u)));
}
// ------------------------------------------------------------------------------------------
// Classification of a staged tile: per 16-byte chunk, bits 0-15 = '{' bytes, bits 16-31 = '}'
// bytes (exact per-byte tests, no carries across bytes), and an "odd" flag for '\' or 0xE3.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t nib(uint32_t v) {  // bit k: byte k of v has its top bit
  return ((v & 0x80808080u) * 0x00204081u) >> 28;
}
__device__ __forceinline__ uint32_t chunk_classify(const lds_u32* w, bool& odd, bool& esc) {
  uint32_t op = 0, cl = 0, od = 0, bs = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t x = w[k];
    const uint32_t x7 = x & 0x7F7F7F7Fu;
    // top bit of each byte CLEAR exactly where the byte equals the target
    const uint32_t no = ((x7 ^ 0x7B7B7B7Bu) + 0x7F7F7F7Fu) | x;
    const uint32_t nc = ((x7 ^ 0x7D7D7D7Du) + 0x7F7F7F7Fu) | x;
    const uint32_t nb = ((x7 ^ 0x5C5C5C5Cu) + 0x7F7F7F7Fu) | x;
    const uint32_t ne = ((x7 ^ 0x63636363u) + 0x7F7F7F7Fu) | ~x;
    od |= ~ne;
    bs |= ~nb;
    op |= nib(~no) << (4 * k);
    cl |= nib(~nc) << (4 * k);
  }
  odd = (od & 0x80808080u) != 0;
  esc = (bs & 0x80808080u) != 0;
  return op | (cl << 16);
}

// bits 0-15: '\' bytes, bits 16-31: '.' bytes of one staged 16-byte chunk
__device__ __forceinline__ uint32_t chunk_bs_dot(const lds_u32* w) {
  uint32_t bs = 0, dt = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t x = w[k];
    const uint32_t x7 = x & 0x7F7F7F7Fu;
    const uint32_t nb = ((x7 ^ 0x5C5C5C5Cu) + 0x7F7F7F7Fu) | x;
    const uint32_t nd = ((x7 ^ 0x2E2E2E2Eu) + 0x7F7F7F7Fu) | x;
    bs |= nib(~nb) << (4 * k);
    dt |= nib(~nd) << (4 * k);
  }
  return bs | (dt << 16);
}

// 128-bit event masks of one string (bit i = byte i)
struct Ev {
  uint64_t lo, hi;
};
__device__ __forceinline__ Ev ev_from(Ev m, uint32_t p) {  // the bits at or after p
  Ev r;
  r.lo = p >= 64u ? 0ull : m.lo & (~0ull << p);
  r.hi = p <= 64u ? m.hi : p >= 128u ? 0ull : m.hi & (~0ull << (p - 64u));
  return r;
}
__device__ __forceinline__ Ev ev_below(Ev m, uint32_t p) {  // the bits before p
  Ev r;
  r.lo = p >= 64u ? m.lo : m.lo & ((1ull << p) - 1ull);
  r.hi = p <= 64u ? 0ull : p >= 128u ? m.hi : m.hi & ((1ull << (p - 64u)) - 1ull);
  return r;
}
__device__ __forceinline__ uint32_t ev_first(Ev m) {  // lowest set bit, 128 if none
  return m.lo ? (uint32_t)__builtin_ctzll(m.lo) : m.hi ? 64u + (uint32_t)__builtin_ctzll(m.hi) : 128u;
}
__device__ __forceinline__ uint32_t ev_last(Ev m) {  // highest set bit, 128 if none
  return m.hi ? 127u - (uint32_t)__builtin_clzll(m.hi) : m.lo ? 63u - (uint32_t)__builtin_clzll(m.lo) : 128u;
}
__device__ __forceinline__ uint32_t ev_count(Ev m) { return (uint32_t)(__popcll(m.lo) + __popcll(m.hi)); }

__device__ __forceinline__ uint32_t w_max32(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d, 64));
  return v;
}

// ------------------------------------------------------------------------------------------
// Chains (the chain evaluator's string shape): every top-level pair has at most one
// child ({a}, {q-{i}}, {a-{b-{c-{d}}}}); at most kMaxTop chains of depth <= kChainDepth in a
// string of <= kChainMax bytes (the 128-bit event window).
// ------------------------------------------------------------------------------------------
constexpr int kMaxTop = 3;
constexpr int kChainDepth = 4;
constexpr uint32_t kChainMax = 112;

// A chain record: first open | first close << 8 | innermost open << 16 | last close << 24 (strings
// of <= kChainMax bytes), or, for a flat pair of a long string, kLongRec | open | close << 14.
constexpr uint32_t kLongRec = 1u << 31;
__device__ __forceinline__ uint32_t cr_first_open(uint32_t r) { return (r & kLongRec) ? r & 0x3FFFu : r & 0xFFu; }
__device__ __forceinline__ uint32_t cr_first_close(uint32_t r) { return (r & kLongRec) ? (r >> 14) & 0x3FFFu : (r >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t cr_inner_open(uint32_t r) { return (r & kLongRec) ? r & 0x3FFFu : (r >> 16) & 0xFFu; }
__device__ __forceinline__ uint32_t cr_last_close(uint32_t r) { return (r & kLongRec) ? (r >> 14) & 0x3FFFu : r >> 24; }

// The open / close events of a string of <= kChainMax bytes at p0 of the staged tile, as 128-bit
// windows (bit i = byte i), from the chunk masks: braces right after a '\\' are not events (escapes,
// py:505-508). ok in: the string is a candidate; out: false when a chunk of it holds a U+3020 lead
// byte or an escape that the restore may misread (the exact evaluator's strings). parse_chains'
// first step; the LEAN k_resolve also recomputes it for a chain's middle levels.
__device__ __forceinline__ void string_events(const lds_u8* tile, uint32_t p0, uint32_t n, const lds_u32* cm,
                                              const lds_u32* oddbits, const lds_u32* escbits, bool& ok, bool& any_esc,
                                              Ev& Om, Ev& Cm) {
  uint32_t O[4], C[4];
  any_esc = false;
  {
    const uint32_t c0 = ok ? p0 >> 4 : 0u, o = p0 & 15u;
    const uint32_t cl = ok && n ? (p0 + n - 1) >> 4 : c0;
    // any odd chunk in [c0, cl] (<= 8 chunks): U+3020 needs the exact evaluator
    const uint64_t span_m = (2ull << (cl - c0)) - 1ull;
    const uint64_t ob = ((uint64_t)oddbits[(c0 >> 5) + 1] << 32) | oddbits[c0 >> 5];
    if ((ob >> (c0 & 31)) & span_m) ok = false;
    const uint64_t eb = ((uint64_t)escbits[(c0 >> 5) + 1] << 32) | escbits[c0 >> 5];
    const bool esc = ok && ((eb >> (c0 & 31)) & span_m) != 0;
    any_esc = esc;
    uint32_t Wo[5], Wc[5];
#pragma unroll
    for (int j = 0; j < 5; j++) {
      const uint32_t x = cm[c0 + 2 * j], y = j < 4 ? cm[c0 + 2 * j + 1] : 0u;
      Wo[j] = (x & 0xFFFFu) | (y << 16);
      Wc[j] = (x >> 16) | (y & 0xFFFF0000u);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int32_t r = (int32_t)n - 32 * j;
      const uint32_t keep = !ok ? 0u : r >= 32 ? 0xFFFFFFFFu : r > 0 ? (1u << r) - 1u : 0u;
      O[j] = __builtin_amdgcn_alignbit(Wo[j + 1], Wo[j], o) & keep;
      C[j] = __builtin_amdgcn_alignbit(Wc[j + 1], Wc[j], o) & keep;
    }
    // Escapes (py:505-508): a brace right after a '\' is protected, i.e. plain text to the loop,
    // and comes back unchanged (py:537-540) unless the restore misreads it: '\}' right after a
    // '.' or a '}' (a value may end in '.') restores as '\{...' (py:538 runs before py:539), so
    // such strings stay with the exact evaluator.
    if (__any(esc)) {
      uint32_t Wb[5], Wd[5];
#pragma unroll
      for (int j = 0; j < 5; j++) {
        const uint32_t ca = c0 + 2 * j, cb = ca + 1;
        const uint32_t x = esc && ca <= cl ? chunk_bs_dot(((const lds_u32*)tile) + 4 * ca) : 0u;
        const uint32_t y = esc && j < 4 && cb <= cl ? chunk_bs_dot(((const lds_u32*)tile) + 4 * cb) : 0u;
        Wb[j] = (x & 0xFFFFu) | (y << 16);
        Wd[j] = (x >> 16) | (y & 0xFFFF0000u);
      }
      uint32_t B[4], D[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int32_t r = (int32_t)n - 32 * j;
        const uint32_t keep = !esc ? 0u : r >= 32 ? 0xFFFFFFFFu : r > 0 ? (1u << r) - 1u : 0u;
        B[j] = __builtin_amdgcn_alignbit(Wb[j + 1], Wb[j], o) & keep;
        D[j] = __builtin_amdgcn_alignbit(Wd[j + 1], Wd[j], o) & keep;
      }
      uint32_t EC[4];
      bool hazard = false;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t b1 = (B[j] << 1) | (j ? B[j - 1] >> 31 : 0u);  // bytes right after a '\'
        EC[j] = C[j] & b1;
        O[j] &= ~b1;
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t before = (EC[j] >> 2) | (j < 3 ? EC[j + 1] << 30 : 0u);  // the byte before the '\'
        hazard |= (before & (D[j] | C[j])) != 0u;
      }
#pragma unroll
      for (int j = 0; j < 4; j++) C[j] &= ~EC[j];
      if (hazard) ok = false;
    }
  }
  Om = Ev{O[0] | ((uint64_t)O[1] << 32), O[2] | ((uint64_t)O[3] << 32)};
  Cm = Ev{C[0] | ((uint64_t)C[1] << 32), C[2] | ((uint64_t)C[3] << 32)};
}

// the string's chains (<= kMaxTop, depth <= kChainDepth; records as in ChainJobs::crec). False:
// the string is not a chain-only clean string (the exact evaluator decides it).
__device__ __forceinline__ bool parse_chains(const lds_u8* tile, uint32_t p0, uint32_t n, const lds_u32* cm,
                                             const lds_u32* oddbits, const lds_u32* escbits, bool active,
                                             uint32_t (&crec)[kMaxTop], uint32_t (&cdep)[kMaxTop], uint32_t& nch,
                                             Ev& Om_out, Ev& Cm_out, uint32_t& maxd_out, bool& whole_out) {
  whole_out = false;
  if (active && n > kChainMax) {
    // A long string (a prompt template): copied verbatim when none of its bytes is a brace and its
    // chunks hold no U+3020 lead byte (py:505-540 leave it unchanged). One with up to kMaxTop FLAT
    // pairs ({key} with no brace inside, no '\\' near any of them) is chain-shaped too: each pair is
    // a one-level chain whose record holds 14-bit positions (kLongRec). Anything else: the exact
    // evaluator.
    nch = 0;
#pragma unroll
    for (int c = 0; c < kMaxTop; c++) crec[c] = cdep[c] = 0;
    const uint32_t c0 = p0 >> 4, cl = (p0 + n - 1) >> 4;
    bool ok = n < (1u << 14), braces = false, esc = false, inside = false;
    uint32_t a = 0;
    for (uint32_t c = c0; c <= cl && ok; c++) {
      const uint32_t b_lo = c == c0 ? (p0 & 15u) : 0u, b_hi = c == cl ? ((p0 + n - 1) & 15u) : 15u;
      const uint32_t bm = ((2u << b_hi) - 1u) & ~((1u << b_lo) - 1u);  // the string's bytes in the chunk
      uint32_t op = cm[c] & bm, cls = (cm[c] >> 16) & bm;  // '{' / '}' bytes of the chunk
      if ((oddbits[c >> 5] >> (c & 31u)) & 1u) ok = false;
      esc |= ((escbits[c >> 5] >> (c & 31u)) & 1u) != 0u;
      braces |= (op | cls) != 0u;
      while ((op | cls) && ok) {  // the chunk's events in byte order
        const uint32_t k = (uint32_t)__builtin_ctz(op | cls), pos = 16u * c + k - p0;
        if ((op >> k) & 1u) {
          ok = !inside;  // a brace inside a pair: nesting (the exact evaluator)
          inside = true;
          a = pos;
          op &= op - 1u;
        } else {
          ok = inside && nch < (uint32_t)kMaxTop;  // a '}' before its '{', or too many pairs
          if (ok) {
            crec[nch] = kLongRec | a | (pos << 14);
            cdep[nch] = 1u;
            nch++;
          }
          inside = false;
          cls &= cls - 1u;
        }
      }
    }
    ok = ok && !inside && !(braces && esc);
    // a single pair that is the whole string: get_simple_insertkey's typed result (exact evaluator)
    ok = ok && !(nch == 1u && (crec[0] & 0x3FFFu) == 0u && ((crec[0] >> 14) & 0x3FFFu) == n - 1u);
    if (!ok) nch = 0;
    Om_out = Cm_out = Ev{0ull, 0ull};
    maxd_out = ok && nch ? 1u : 0u;
    return ok;
  }
  bool ok = active && n <= kChainMax;
  // ---- 1. the string's open / close events as 128-bit windows ----
  bool any_esc = false;
  Ev Om, Cm;
  string_events(tile, p0, n, cm, oddbits, escbits, ok, any_esc, Om, Cm);
  // ---- 2. chains: the events of a chain-only string are blocks O^d C^d (each pair has at most
  //      one child), so chain c is located by a few mask scans: its first '{' (a), its first '}'
  //      (c1), the opens in [a, c1) (its depth), the closes before the next '{' (as many). ----
  // per chain: first open | first close << 8 | innermost open << 16 | last close << 24, depth
  uint32_t pos = 0, maxd = 0;
  nch = 0;
  bool bad = !ok, whole = false;
#pragma unroll
  for (int c = 0; c < kMaxTop; c++) {
    crec[c] = cdep[c] = 0;
    const Ev Oa = ev_from(Om, pos), Ca = ev_from(Cm, pos);
    const uint32_t a = ev_first(Oa), c1 = ev_first(Ca);
    const bool has = !bad && (a < 128u || c1 < 128u);
    if (!__any(has)) continue;
    const uint32_t dd = ev_count(ev_below(Oa, c1));
    const Ev Cb = ev_below(Ca, ev_first(ev_from(Om, c1)));
    const uint32_t end = ev_last(Cb);
    // a '}' before its '{', a second child or an unbalanced block, too deep: exact evaluator
    const bool cbad = c1 < a || dd != ev_count(Cb) || dd > (uint32_t)kChainDepth;
    const bool take = has && !cbad;
    bad |= has && cbad;
    if (c == 0) whole = take && a == 0 && end == n - 1;
    const uint32_t o0 = ev_last(ev_below(Oa, c1));
    crec[c] = take ? (a | (c1 << 8) | (o0 << 16) | (end << 24)) : 0u;
    cdep[c] = take ? dd : 0u;
    maxd = take && dd > maxd ? dd : maxd;
    nch += take ? 1u : 0u;
    pos = take ? end + 1u : pos;
  }
  bad |= ev_first(ev_from(Ev{Om.lo | Cm.lo, Om.hi | Cm.hi}, pos)) < 128u;  // more than kMaxTop chains
  // A whole-string pair is get_simple_insertkey-truthy (py:477-495, typed result py:510-514). The
  // plain form -- one pair, no nesting, a non-empty key, no '\\' anywhere near (an escaped brace
  // inside would break py's depth walk) -- is one lookup whose raw value is the result: the jobs
  // take it (whole_out); every other whole-string pair goes to the exact evaluator.
  const bool whole1 = !bad && nch == 1 && whole && cdep[0] == 1u && !any_esc && ((crec[0] >> 8) & 0xFFu) > 1u;
  ok = !bad && (!(nch == 1 && whole) || whole1);
  whole_out = ok && whole1;
  Om_out = Om, Cm_out = Cm;  // middle levels (depth > 2) are found from these masks in their round
  maxd_out = ok ? maxd : 0u;
  return ok;
}


}  // namespace ie
