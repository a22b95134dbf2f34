// ie_resolve.hip — k_resolve: interpolate_inserts (py:497-541 / rust-project/src/interp.rs:31-89)
// over a packed batch in ONE pass over HBM.
//
// One 256-lane workgroup per tile of 256 consecutive strings; tiles are taken from an atomic
// ticket (so every tile a workgroup waits on is already running) and chained with a decoupled
// look-back over 8-byte {flag, value} words published by agent-scope atomics. Per tile:
//   1. stage the tile's input bytes in LDS (16-byte loads);
//   2. every lane evaluates its string (eval_rounds): a skip-ahead scan that only visits the
//      special bytes at depth 0 ('{', '}', '\', and >= 0x7B for U+3020), builds keys of open
//      pairs in a lane-private LDS buffer, probes the bucketed table, and records the depth-0
//      output as <= kMaxSeg segments (template runs and splice texts) — no bytes move yet;
//   3. strings the fast path cannot prove equal to the reference are resolved by the tile's
//      waves with the literal emulator (ie_literal.h), results in the scratch pool;
//   4. workgroup scan of output lengths, look-back for the tile's global offset;
//   5. each lane copies its segments (dword copies) into an LDS stage aligned like the
//      destination; the stage streams out with 16-byte stores; offsets/status/value ids.
//
// Fast-path correctness (DESIGN.md "fast path"): for properly nested strings whose
// spliced values are inert, the reference's rightmost-innermost loop equals this left-to-right
// stack evaluation, and its first failure is the failing pair with the largest opening offset
// (pairs enclosing a failed pair are never evaluated). Everything else is PENDING -> literal.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ie_device.h"
#include "ie_kernels.h"
#include "ie_literal.h"

namespace ie {

// segment sources: template bytes (string offset), arena text (offset), literal-path pool
// (16-byte units), a bucket's inline text (bucket index; splice texts <= kInlineText)
enum : uint32_t { kSegTemplate = 0, kSegValue = 1, kSegPool = 2, kSegBucket = 3 };

__device__ __forceinline__ uint64_t seg_make(uint32_t kind, uint32_t len, uint32_t src) {
  return ((uint64_t)kind << 62) | ((uint64_t)len << 32) | (uint64_t)src;
}

// LDS-typed views: reads through them compile to ds_* (not flat_*) instructions
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;

// the string being evaluated: in the tile's LDS stage (STAGED) or in global memory
template <bool STAGED>
struct Src {
  const uint8_t* p;
  __device__ __forceinline__ uint8_t operator[](uint32_t i) const {
    if (STAGED) return ((const lds_u8*)p)[i];
    return gld(p + i);
  }
  __device__ __forceinline__ uint32_t word_at(uintptr_t aligned_addr) const {
    if (STAGED) return *(const lds_u32*)(const lds_u8*)(const uint8_t*)aligned_addr;
    return gld((const uint32_t*)aligned_addr);
  }
};

// bytes the skip-ahead scan must look at: '\\' and everything >= 0x7B ('{', '}', U+3020's 0xE3,
// other non-ASCII, '|', '~'). The lowest flagged byte is always a true candidate.
__device__ __forceinline__ uint32_t special_mask(uint32_t w) {
  const uint32_t ge = ((w + 0x05050505u) | w) & 0x80808080u;
  const uint32_t x = w ^ 0x5C5C5C5Cu;
  return ge | ((x - 0x01010101u) & ~x & 0x80808080u);
}

// first index j in [i, n) whose byte is a candidate, else n. Reads aligned dwords (an aligned
// dword never crosses a page, so bytes around the string are safe to read and ignored).
template <bool STAGED>
__device__ __forceinline__ uint32_t next_special(const Src<STAGED>& s, uint32_t i, uint32_t n) {
  while (i < n) {
    const uintptr_t a = (uintptr_t)(s.p + i);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t m = special_mask(s.word_at(a - sh)) & (0xFFFFFFFFu << (8 * sh));
    if (m) {
      const uint32_t j = i + ((uint32_t)__builtin_ctz(m) >> 3) - sh;
      return j < n ? j : n;
    }
    i += 4 - sh;
  }
  return n;
}

// copy len bytes src -> dst: byte head until dst is 4-aligned, dword body with v_alignbyte over
// the source's aligned dwords, byte tail. SRC_LDS / DST_LDS select ds_* vs global access.
template <bool DST_LDS, bool SRC_LDS>
__device__ __forceinline__ void copy_bytes(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                           uint32_t len) {
  auto rd8 = [&](uint32_t k) -> uint8_t {
    if (SRC_LDS) return ((const lds_u8*)src)[k];
    return gld(src + k);
  };
  auto rd32 = [&](const uint32_t* p, uint32_t q) -> uint32_t {
    if (SRC_LDS) return ((const lds_u32*)(const lds_u8*)(const uint8_t*)p)[q];
    return gld(p + q);
  };
  auto wr8 = [&](uint32_t k, uint8_t v) {
    if (DST_LDS) ((lds_u8*)dst)[k] = v;
    else gst(dst + k, v);
  };
  auto wr32 = [&](uint32_t* p, uint32_t q, uint32_t v) {
    if (DST_LDS) ((lds_u32*)(lds_u8*)(uint8_t*)p)[q] = v;
    else gst(p + q, v);
  };
  uint32_t k = 0;
  while (k < len && (((uintptr_t)(dst + k)) & 3)) {
    wr8(k, rd8(k));
    k++;
  }
  if (k + 4 <= len) {
    const uintptr_t a = (uintptr_t)(src + k);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t* s32 = (const uint32_t*)(a - sh);
    uint32_t* d32 = (uint32_t*)(dst + k);
    const uint32_t nw = (len - k) >> 2;
    if (sh == 0) {
      for (uint32_t q = 0; q < nw; q++) wr32(d32, q, rd32(s32, q));
    } else {
      uint32_t w0 = rd32(s32, 0);
      for (uint32_t q = 0; q < nw; q++) {
        const uint32_t w1 = rd32(s32, q + 1);
        wr32(d32, q, __builtin_amdgcn_alignbyte(w1, w0, sh));
        w0 = w1;
      }
    }
    k += nw << 2;
  }
  for (; k < len; k++) wr8(k, rd8(k));
}

// Branch-free LDS writers: a lane that has nothing to write for some step stores to its own
// sink dword instead (an address select, no exec-mask branch); trip counts are wave-uniform.
__device__ __forceinline__ void st8(lds_u8* p, bool on, lds_u8* sink, uint8_t v) { *(on ? p : sink) = v; }
__device__ __forceinline__ void st32(lds_u32* p, bool on, lds_u8* sink, uint32_t v) {
  *(on ? p : (lds_u32*)sink) = v;
}

// a bucket's inline text (16-byte aligned, len <= kInlineText) -> LDS at any byte offset: the
// four 16-byte loads go out together (one memory latency), dwords are re-aligned with alignbyte
__device__ __forceinline__ void put_bucket_text(lds_u8* dst, const Bucket* b, uint32_t len, lds_u8* sink) {
  const uint4* tp = (const uint4*)b->text;
  const uint4 t0 = gld4(tp), t1 = gld4(tp + 1), t2 = gld4(tp + 2), t3 = gld4(tp + 3);  // one line
  const uint32_t tw[17] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w,
                           t2.x, t2.y, t2.z, t2.w, t3.x, t3.y, t3.z, t3.w, 0u};
  const uint32_t a = (uint32_t)(uintptr_t)dst & 3u;
  const uint32_t head = min(len, (4u - a) & 3u);
#pragma unroll
  for (uint32_t k = 0; k < 3; k++) st8(dst + k, k < head, sink, (uint8_t)(tw[0] >> (8 * k)));
  // dword q of the aligned body = text bytes head + 4q .. head + 4q + 3
  lds_u32* d32 = (lds_u32*)(dst + head);
  const uint32_t rest = len - head, nq = rest >> 2, tail = rest & 3u;
  uint32_t x = 0;
#pragma unroll
  for (uint32_t q = 0; q < 16; q++) {
    if (!__any(q <= nq)) break;  // wave-uniform exit
    const uint32_t v = __builtin_amdgcn_alignbyte(tw[q + 1], tw[q], head);
    st32(d32 + q, q < nq, sink, v);
    x = q == nq ? v : x;
  }
  lds_u8* t = dst + head + 4 * nq;
#pragma unroll
  for (uint32_t k = 0; k < 3; k++) st8(t + k, k < tail, sink, (uint8_t)(x >> (8 * k)));
}

// len bytes LDS -> LDS, any alignments: dst-aligned dword body built with alignbyte from the
// source's aligned dwords (reads may touch up to 3 bytes around the source; the tile is padded)
__device__ __forceinline__ void lds_copy(lds_u8* dst, const lds_u8* src, uint32_t len, lds_u8* sink) {
  const uint32_t a = (uint32_t)(uintptr_t)dst & 3u;
  const uint32_t head = min(len, (4u - a) & 3u);
#pragma unroll
  for (uint32_t k = 0; k < 3; k++) st8(dst + k, k < head, sink, src[k]);
  const uint32_t s2 = (uint32_t)(uintptr_t)(src + head);
  const uint32_t sh = s2 & 3u;
  const lds_u32* sw = (const lds_u32*)(lds_u8*)(uintptr_t)(s2 - sh);
  lds_u32* d32 = (lds_u32*)(dst + head);
  const uint32_t rest = len - head, nq = rest >> 2, tail = rest & 3u;
  uint32_t prev = sw[0];
  for (uint32_t q = 0; __any(q < nq); q++) {  // wave-uniform trip count
    const uint32_t nx = sw[q + 1];
    st32(d32 + q, q < nq, sink, __builtin_amdgcn_alignbyte(nx, prev, sh));
    prev = nx;
  }
  const lds_u8* ts = src + head + 4 * nq;
  lds_u8* td = dst + head + 4 * nq;
#pragma unroll
  for (uint32_t k = 0; k < 3; k++) st8(td + k, k < tail, sink, ts[k]);
}

struct LaneLds {
  lds_u8* kbuf;     // kKeyCap bytes, 4-aligned
  lds_u32* stack;   // [kMaxDepth] stride kBlock: (enclosing key length << 24) | opening offset
  lds_u64* seg;     // [kMaxSeg] stride kBlock
};

// Evaluate one string in ROUNDS: every lane scans (LDS only) up to its next closing brace, then
// all lanes that reached one probe the table in the same instructions, so a wave pays one memory
// latency per lookup round instead of one per special byte of any of its lanes.
// RECORD mode (WRITE = false) stores depth-0 output segments in L.seg and returns their count in
// nseg (may exceed kMaxSeg: then only the count is valid). WRITE mode copies every segment's
// bytes to dst as it is produced (only for strings already known to be OK_STR).
// `active` lanes take part; the call is wave-uniform (all lanes must call it).
template <bool STAGED, bool WRITE>
__device__ uint8_t eval_rounds(const DevTable& T, const Src<STAGED> s, uint32_t n, bool active,
                               const LaneLds& L, uint8_t* __restrict__ dst, uint32_t& out_len,
                               uint32_t& vid, uint32_t& nseg) {
  constexpr uint8_t kRunning = 0xFF;
  uint8_t status = active ? kRunning : (uint8_t)IE_OK_STR;
  uint32_t depth = 0, klen = 0, olen = 0, ns = 0;
  uint32_t nopen = 0, nclose = 0;
  bool negclose = false;
  uint32_t poison = 0;  // bit d: the pair open at level d contains a failed pair
  int64_t err_off = -1;
  uint8_t err_cls = 0;
  bool wrapped = false;  // a whole-string pair resolved (typed result so far in wrap_h)
  Hit wrap_h{0, 0, IE_VID_NONE, 0};
  uint32_t run_start = 0;
  uint32_t i = 0;
  // the close waiting for its lookup
  uint32_t c_open = 0, c_ks = 0, c_kl = 0;
  bool c_wrapping = false;

  auto emit = [&](uint32_t kind, uint32_t len, uint32_t src) {
    if (!len) return;
    if (WRITE) {
      if (kind == kSegTemplate) copy_bytes<false, STAGED>(dst + olen, s.p + src, len);
      else copy_bytes<false, false>(dst + olen, T.arena + src, len);
    } else if (ns < (uint32_t)kMaxSeg) {
      L.seg[ns * kBlock] = seg_make(kind, len, src);
    }
    ns++;
    olen += len;
  };
  auto kput = [&](uint8_t c) -> bool {
    if (klen >= (uint32_t)kKeyCap) return false;
    L.kbuf[klen++] = c;
    return true;
  };
  // end of string: the reference's checks in order (py:516-519, 522, 540)
  auto finish = [&]() -> uint8_t {
    if (nopen == 0) {
      emit(kSegTemplate, n - run_start, run_start);
      return IE_OK_STR;
    }
    if (nopen != nclose) return IE_E_ASSERT_BRACES;
    if (negclose) return kStatusPending;  // balanced but '}{': py break / rs panic
    if (err_off >= 0) return err_cls;
    if (wrapped) {
      vid = wrap_h.vid;
      return IE_OK_VALUE;
    }
    emit(kSegTemplate, n - run_start, run_start);
    return IE_OK_STR;
  };

  for (;;) {
    // ---- scan phase: LDS only, up to this lane's next closing brace ----
    bool need = false;
    while (status == kRunning) {
      if (depth == 0) {
        i = next_special(s, i, n);
      } else {
        const uint32_t j = next_special(s, i, n);
        if (klen + (j - i) > (uint32_t)kKeyCap) {  // long key: literal path
          status = kStatusPending;
          break;
        }
        for (; i < j; i++) L.kbuf[klen++] = s[i];
      }
      if (i >= n) {
        status = finish();
        break;
      }
      const uint8_t c = s[i];
      if (c == '\\') {
        const uint8_t nx = i + 1 < n ? s[i + 1] : 0;
        if (nx == '{' || nx == '}') {  // an escape pair (py:505-508): plain text
          // '.\}' and '}\}' can restore as '\{...' (py:537-540 replace order): literal path
          if ((nx == '}' && i > 0 && (s[i - 1] == '.' || s[i - 1] == '}')) ||
              (depth && !(kput(c) && kput(nx)))) {
            status = kStatusPending;
            break;
          }
          i += 2;
          continue;
        }
        if (depth && !kput(c)) {
          status = kStatusPending;
          break;
        }
        i++;
        continue;
      }
      if (c == '{') {
        nopen++;
        const uint32_t ks = (klen + 3) & ~3u;  // keys start dword-aligned (pad bytes are not key)
        if (depth >= (uint32_t)kMaxDepth || i >= (1u << 24) || ks > (uint32_t)kKeyCap) {
          status = kStatusPending;
          break;
        }
        if (depth == 0) emit(kSegTemplate, i - run_start, run_start);
        L.stack[depth * kBlock] = (klen << 24) | i;  // the enclosing key resumes at klen
        klen = ks;
        poison &= ~(1u << depth);
        depth++;
        i++;
        continue;
      }
      if (c == '}') {
        nclose++;
        if (depth == 0) {  // unmatched '}': text, unless the count check fails (py:517-519)
          negclose = true;
          i++;
          continue;
        }
        depth--;
        const uint32_t st = L.stack[depth * kBlock];
        const uint32_t open = st & 0xFFFFFFu, resume = st >> 24, ks = (resume + 3) & ~3u;
        c_kl = klen - ks;
        c_ks = ks;
        c_open = open;
        klen = resume;
        if ((poison >> depth) & 1u) {  // an inner pair failed first: never evaluated
          if (depth) poison |= 1u << (depth - 1);
          i++;
          continue;
        }
        // a whole-string pair at this level (get_simple_insertkey truthy, py:510-514)
        c_wrapping = (open == depth) && (i == n - 1 - depth) && (i - open >= 2);
        need = true;
        break;
      }
      if (c == 0xE3 && i + 2 < n && s[i + 1] == 0x80 && s[i + 2] == 0xA0) {
        status = kStatusPending;  // a literal U+3020 collides with the placeholders (py:502-503)
        break;
      }
      if (depth && !kput(c)) {  // other flagged bytes are plain text
        status = kStatusPending;
        break;
      }
      i++;
    }
    if (!__any(need)) break;  // every lane is finished (or pending)
    // ---- lookup phase: all lanes with a pending close probe together ----
    if (need) {
      uint8_t est = 0;
      Hit h;
      int32_t b;
      if (c_wrapping && wrapped) {
        b = find_raw(T, wrap_h, est, h);  // the key is the inner level's raw value
      } else {
        b = c_kl <= kInlineKey ? find_small(T, (const lds_u32*)(L.kbuf + c_ks), c_kl, h)
                               : find_bytes(T, (const uint8_t*)(L.kbuf + c_ks), c_kl, h);
        if (b < 0) est = missing_status(T, (const uint8_t*)(L.kbuf + c_ks), c_kl);
      }
      if (b >= 0 && !c_wrapping) {
        if (!(h.flags & EF_SPLICE_OK)) {  // py:530 / interp.rs:76-79
          b = -1;
          est = IE_E_ASSERT_TYPE;
        } else if (!(h.flags & EF_INERT)) {
          status = kStatusPending;  // re-resolution / escape hazard
        } else if (depth) {         // splice into the enclosing key
          if (klen + h.text_len > (uint32_t)kKeyCap) {
            status = kStatusPending;
          } else {
            const uint8_t* t = h.text_len <= kInlineText ? T.buckets[b].text : T.arena + h.text_off;
            copy_bytes<true, false>((uint8_t*)(L.kbuf + klen), t, h.text_len);
            klen += h.text_len;
          }
        } else {
          emit(kSegValue, h.text_len, h.text_off);
          run_start = i + 1;
        }
      }
      if (b < 0) {
        if ((int64_t)c_open > err_off) {
          err_off = c_open;
          err_cls = est;
        }
        if (depth) poison |= 1u << (depth - 1);
      } else if (c_wrapping) {
        wrapped = true;
        wrap_h = h;
      }
      i++;
    }
  }
  nseg = ns;
  out_len = status == IE_OK_STR ? olen : 0;
  return status;
}

// ------------------------------------------------------------------------------------------
// Cooperative classification of a staged tile: one 16-bit mask per 16-byte LDS chunk, bit k set
// when byte k is '{', '}', '\' or 0xE3 (U+3020's lead byte): the only bytes that can change the
// reference's result. Exact per-byte test: no carries cross bytes.
// ------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) uint16_t lds_u16;

__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {  // 0x80 in every zero byte of x
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t nibble_of(uint32_t z) {  // bit k: byte k of z has its top bit
  return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}
// chunk mask: bits 0-15 '{' / '}', bits 16-31 '\' / 0xE3 ("odd" bytes) of the 16-byte chunk
__device__ __forceinline__ uint32_t chunk_mask(const lds_u32* w) {
  uint32_t br = 0, odd = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t x = w[k];
    br |= nibble_of(zero_bytes(x ^ 0x7B7B7B7Bu) | zero_bytes(x ^ 0x7D7D7D7Du)) << (4 * k);
    odd |= nibble_of(zero_bytes(x ^ 0x5C5C5C5Cu) | zero_bytes(x ^ 0xE3E3E3E3u)) << (4 * k);
  }
  return br | (odd << 16);
}

// Event-driven evaluation of a staged string: the same rounds and the same semantics as
// eval_rounds, but the lane visits only its event bytes (from the chunk masks) and copies key
// text between events with dword copies. s = the string in LDS at stage position p0.
__device__ uint8_t eval_events(const DevTable& T, const lds_u8* s, uint32_t p0, uint32_t n,
                               const lds_u32* cm, bool active, const LaneLds& L, uint32_t& out_len,
                               uint32_t& vid, uint32_t& nseg) {
  constexpr uint8_t kRunning = 0xFF;
  uint8_t status = active ? kRunning : (uint8_t)IE_OK_STR;
  uint32_t depth = 0, klen = 0, olen = 0, ns = 0;
  uint32_t nopen = 0, nclose = 0;
  bool negclose = false;
  uint32_t poison = 0;
  int64_t err_off = -1;
  uint8_t err_cls = 0;
  bool wrapped = false;
  Hit wrap_h{0, 0, IE_VID_NONE, 0};
  uint32_t run_start = 0;
  uint32_t c_open = 0, c_ks = 0, c_kl = 0, c_pos = 0;
  bool c_wrapping = false;
  // event cursor over the chunk masks
  const uint32_t end = p0 + n;
  uint32_t ch = p0 >> 4, m = 0, skip_below = 0, last = 0;
  bool m_loaded = false;

  auto next_event = [&]() -> uint32_t {  // string-relative position of the next event, or n
    for (;;) {
      if (!m_loaded) {
        const uint32_t cb = ch << 4;
        if (cb >= end) return n;
        m = cm[ch];
        m = (m | (m >> 16)) & 0xFFFFu;
        if (cb < p0) m &= 0xFFFFu << (p0 - cb);
        if (cb + 16 > end) m &= (1u << (end - cb)) - 1u;
        m_loaded = true;
      }
      if (m) {
        const uint32_t e = (ch << 4) + (uint32_t)__builtin_ctz(m) - p0;
        m &= m - 1;
        if (e < skip_below) continue;
        return e;
      }
      ch++;
      m_loaded = false;
    }
  };
  auto emit = [&](uint32_t kind, uint32_t len, uint32_t src) {
    if (!len) return;
    if (ns < (uint32_t)kMaxSeg) L.seg[ns * kBlock] = seg_make(kind, len, src);
    ns++;
    olen += len;
  };
  auto kput = [&](uint8_t c) -> bool {
    if (klen >= (uint32_t)kKeyCap) return false;
    L.kbuf[klen++] = c;
    return true;
  };
  auto finish = [&]() -> uint8_t {
    if (nopen == 0) {
      emit(kSegTemplate, n - run_start, run_start);
      return IE_OK_STR;
    }
    if (nopen != nclose) return IE_E_ASSERT_BRACES;  // py:517-519
    if (negclose) return kStatusPending;             // balanced but '}{'
    if (err_off >= 0) return err_cls;
    if (wrapped) {
      vid = wrap_h.vid;
      return IE_OK_VALUE;
    }
    emit(kSegTemplate, n - run_start, run_start);
    return IE_OK_STR;
  };

  for (;;) {
    bool need = false;
    while (status == kRunning) {
      const uint32_t e = next_event();
      if (depth) {  // the template bytes since the last event are key text
        const uint32_t len = e - last;
        if (klen + len > (uint32_t)kKeyCap) {
          status = kStatusPending;
          break;
        }
        copy_bytes<true, true>((uint8_t*)(L.kbuf + klen), (const uint8_t*)(s + last), len);
        klen += len;
      }
      if (e >= n) {
        status = finish();
        break;
      }
      const uint8_t c = s[e];
      last = e + 1;
      if (c == '\\') {
        const uint8_t nx = e + 1 < n ? s[e + 1] : 0;
        if (nx == '{' || nx == '}') {  // escape pair (py:505-508)
          if ((nx == '}' && e > 0 && (s[e - 1] == '.' || s[e - 1] == '}')) ||
              (depth && !(kput(c) && kput(nx)))) {
            status = kStatusPending;
            break;
          }
          skip_below = e + 2;
          last = e + 2;
          continue;
        }
        if (depth && !kput(c)) {
          status = kStatusPending;
          break;
        }
        continue;
      }
      if (c == 0xE3) {
        if ((e + 2 < n && s[e + 1] == 0x80 && s[e + 2] == 0xA0) || (depth && !kput(c))) {
          status = kStatusPending;  // U+3020 collides with the placeholders (py:502-503)
          break;
        }
        continue;
      }
      if (c == '{') {
        nopen++;
        const uint32_t ks = (klen + 3) & ~3u;
        if (depth >= (uint32_t)kMaxDepth || ks > (uint32_t)kKeyCap) {
          status = kStatusPending;
          break;
        }
        if (depth == 0) emit(kSegTemplate, e - run_start, run_start);
        L.stack[depth * kBlock] = (klen << 24) | e;
        klen = ks;
        poison &= ~(1u << depth);
        depth++;
        continue;
      }
      // '}'
      nclose++;
      if (depth == 0) {
        negclose = true;
        continue;
      }
      depth--;
      const uint32_t st = L.stack[depth * kBlock];
      const uint32_t open = st & 0xFFFFFFu, resume = st >> 24, ks = (resume + 3) & ~3u;
      c_kl = klen - ks;
      c_ks = ks;
      c_open = open;
      c_pos = e;
      klen = resume;
      if ((poison >> depth) & 1u) {
        if (depth) poison |= 1u << (depth - 1);
        continue;
      }
      c_wrapping = (open == depth) && (e == n - 1 - depth) && (e - open >= 2);
      need = true;
      break;
    }
    if (!__any(need)) break;
    if (need) {
      uint8_t est = 0;
      Hit h;
      int32_t b;
      if (c_wrapping && wrapped) {
        b = find_raw(T, wrap_h, est, h);
      } else {
        b = c_kl <= kInlineKey ? find_small(T, (const lds_u32*)(L.kbuf + c_ks), c_kl, h)
                               : find_bytes(T, (const uint8_t*)(L.kbuf + c_ks), c_kl, h);
        if (b < 0) est = missing_status(T, (const uint8_t*)(L.kbuf + c_ks), c_kl);
      }
      if (b >= 0 && !c_wrapping) {
        if (!(h.flags & EF_SPLICE_OK)) {
          b = -1;
          est = IE_E_ASSERT_TYPE;
        } else if (!(h.flags & EF_INERT)) {
          status = kStatusPending;
        } else if (depth) {
          if (klen + h.text_len > (uint32_t)kKeyCap) {
            status = kStatusPending;
          } else {
            const uint8_t* t = h.text_len <= kInlineText ? T.buckets[b].text : T.arena + h.text_off;
            copy_bytes<true, false>((uint8_t*)(L.kbuf + klen), t, h.text_len);
            klen += h.text_len;
          }
        } else {
          if (h.text_len <= kInlineText) emit(kSegBucket, h.text_len, (uint32_t)b);
          else emit(kSegValue, h.text_len, h.text_off);
          run_start = c_pos + 1;
        }
      }
      if (b < 0) {
        if ((int64_t)c_open > err_off) {
          err_off = c_open;
          err_cls = est;
        }
        if (depth) poison |= 1u << (depth - 1);
      } else if (c_wrapping) {
        wrapped = true;
        wrap_h = h;
      }
    }
  }
  nseg = ns;
  out_len = status == IE_OK_STR ? olen : 0;
  return status;
}

// ------------------------------------------------------------------------------------------
// Level evaluator for CLEAN strings (the common case): only '{' / '}' events, properly nested to
// depth <= kFastDepth, <= kFastPairs pairs, <= 3 top-level pairs, no whole-string pair, every
// lookup a hit on an inert splice-able value with keys <= kInlineKey bytes. For such strings every
// order of evaluation gives the reference's result (the values never create braces), so pairs are
// resolved by HEIGHT: round h looks up every pair whose children are all resolved, up to two
// probes in flight per lane. A lane whose string breaks any condition returns false with nothing
// committed, and the caller re-evaluates it with eval_events (exact reference semantics).
// ------------------------------------------------------------------------------------------
constexpr int kFastDepth = 4;
constexpr int kFastPairs = 6;
constexpr int kFastVb = 32;  // bytes of resolved inner values per lane

struct FastLds {
  lds_u8* kbuf;   // lane-private key buffer (kKeyCap bytes, 4-aligned)
  lds_u64* pair;  // [kFastPairs] stride kBlock: pair records
  lds_u8* vbuf;   // lane-private kFastVb bytes: texts of resolved inner pairs
};

// pair record: open:16 | close:16 | depth:4 | height:4 | vb_off:8 | vlen:8 | top ordinal:8
__device__ __forceinline__ uint32_t pr_open(uint64_t r) { return (uint32_t)r & 0xFFFFu; }
__device__ __forceinline__ uint32_t pr_close(uint64_t r) { return (uint32_t)(r >> 16) & 0xFFFFu; }
__device__ __forceinline__ uint32_t pr_depth(uint64_t r) { return (uint32_t)(r >> 32) & 0xFu; }
__device__ __forceinline__ uint32_t pr_height(uint64_t r) { return (uint32_t)(r >> 36) & 0xFu; }
__device__ __forceinline__ uint32_t pr_vboff(uint64_t r) { return (uint32_t)(r >> 40) & 0xFFu; }
__device__ __forceinline__ uint32_t pr_vlen(uint64_t r) { return (uint32_t)(r >> 48) & 0xFFu; }
__device__ __forceinline__ uint32_t pr_top(uint64_t r) { return (uint32_t)(r >> 56); }

struct FastKey {
  uint32_t w[8];  // key bytes, zero padded like the buckets' inline keys
  uint32_t len;
  uint64_t hash;
};

// key of pair `idx` (string s in LDS): a leaf pair's key is its template bytes, read as dwords
// straight from the staged tile; a chain pair's key is template + its one child's text (vbuf) +
// template, assembled bytewise in the lane's key buffer. Wave-uniform call (early exits vote).
__device__ __forceinline__ bool fast_key(const lds_u8* s, const FastLds& F, uint32_t idx, bool on,
                                         FastKey& K) {
  const uint64_t rec = on ? F.pair[idx * kBlock] : 0ull;
  const uint32_t open = pr_open(rec), close = pr_close(rec);
  const bool leaf = pr_height(rec) <= 1;
  uint32_t len = 0, la = 0, lv = 0, vb = 0, b0 = 0;
  if (on) {
    if (leaf) {
      len = close - open - 1;
    } else {
      const uint64_t c = F.pair[(idx - 1) * kBlock];  // postorder: the only child closes just before
      la = pr_open(c) - open - 1;
      lv = pr_vlen(c);
      vb = pr_vboff(c);
      b0 = pr_close(c) + 1;
      len = la + lv + (close - b0);
    }
  }
  const bool fits = len <= (uint32_t)kInlineKey;
  if (!fits) len = 0;
  const lds_u8* src = s + open + 1;
  if (on && fits && !leaf) {  // assemble: A | child text | B
    for (uint32_t k = 0; k < len; k++) {
      const uint8_t c = k < la ? src[k] : k < la + lv ? F.vbuf[vb + k - la] : s[b0 + (k - la - lv)];
      F.kbuf[k] = c;
    }
  }
  // dwords of the key: from the tile (leaf, any alignment) or the key buffer (chain, aligned)
  const uint32_t addr = (uint32_t)(uintptr_t)src;
  const uint32_t sh = addr & 3u;
  const lds_u32* lw = (const lds_u32*)(lds_u8*)(uintptr_t)(addr - sh);
  const lds_u32* kw = (const lds_u32*)F.kbuf;
  uint64_t hash = 0xA0761D6478BD642Full ^ (uint64_t)len;
  uint32_t prev = leaf && on && fits ? lw[0] : 0u;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    K.w[q] = 0;
    if (!__any(4 * q < (int)len)) continue;  // wave-uniform: no lane has this word
    const int32_t rem = (int32_t)len - 4 * q;
    if (rem > 0) {
      uint32_t x;
      if (leaf) {
        const uint32_t nx = lw[q + 1];
        x = __builtin_amdgcn_alignbyte(nx, prev, sh);
        prev = nx;
      } else {
        x = kw[q];
      }
      if (rem < 4) x &= (1u << (8 * rem)) - 1u;
      K.w[q] = x;
      hash = hash_word(hash, x);
    }
  }
  K.len = len;
  K.hash = hash;
  return fits;
}

struct FastProbe {
  uint4 q0, q1, q2, q3, q4, q5;
};

// one probe = the bucket's first 96 bytes (header, inline key, inline text 0..31): unconditional,
// so the loop carries no partially-defined registers (idle lanes read slot 0)
__device__ __forceinline__ void fast_load(const DevTable& T, uint32_t slot, FastProbe& P) {
  const uint4* bp = (const uint4*)(T.buckets + slot);
  P.q0 = gld4(bp);
  P.q1 = gld4(bp + 1);
  P.q2 = gld4(bp + 2);
  P.q3 = gld4(bp + 3);
  P.q4 = gld4(bp + 4);
  P.q5 = gld4(bp + 5);
}

// does the bucket hold key K (branch-free)
__device__ __forceinline__ bool fast_match(const FastProbe& P, const FastKey& K) {
  return ((P.q1.y & EF_OCCUPIED) != 0) & ((((uint64_t)P.q0.y << 32) | P.q0.x) == K.hash) &
         (P.q0.z == K.len) & (P.q2.x == K.w[0]) & (P.q2.y == K.w[1]) & (P.q2.z == K.w[2]) &
         (P.q2.w == K.w[3]) & (P.q3.x == K.w[4]) & (P.q3.y == K.w[5]) & (P.q3.z == K.w[6]) &
         (P.q3.w == K.w[7]);
}

// commit a hit for pair idx; false when the value is not fast-path material
__device__ __forceinline__ bool fast_commit(const FastLds& F, const LaneLds& L, uint32_t idx, uint32_t slot,
                                            const FastProbe& P, uint32_t& vb_used, uint32_t& vsum) {
  const uint32_t flags = P.q1.y, tlen = P.q0.w;
  if (!(flags & EF_SPLICE_OK) || !(flags & EF_INERT)) return false;
  uint64_t rec = F.pair[idx * kBlock];
  if (pr_depth(rec) == 0) {
    L.seg[(2 * pr_top(rec) + 1) * kBlock] =
        tlen <= kInlineText ? seg_make(kSegBucket, tlen, slot) : seg_make(kSegValue, tlen, P.q1.w);
    vsum += tlen;
    return true;
  }
  if (tlen > (uint32_t)kInlineKey || vb_used + tlen > (uint32_t)kFastVb) return false;
  const uint32_t tw[8] = {P.q4.x, P.q4.y, P.q4.z, P.q4.w, P.q5.x, P.q5.y, P.q5.z, P.q5.w};
  lds_u32* v32 = (lds_u32*)(F.vbuf + vb_used);
#pragma unroll
  for (int q = 0; q < 8; q++) {
    if (!__any(4 * q < (int)tlen)) break;  // wave-uniform exit
    if (4 * q < (int)tlen) v32[q] = tw[q];
  }
  rec = (rec & ~(0xFFFFull << 40)) | ((uint64_t)vb_used << 40) | ((uint64_t)tlen << 48);
  F.pair[idx * kBlock] = rec;
  vb_used += (tlen + 3) & ~3u;
  return true;
}

constexpr uint32_t kLeanMax = 112;  // strings the 128-bit event window covers

// Wave-uniform call. tile = the staged tile; the string starts at stage position p0; cm = chunk
// masks. On success: depth-0 segments in L.seg (2 * top pairs + 1 of them), nseg, out_len.
// Shape rules on top of the clean-string rules above: n <= kLeanMax, every pair has at most one
// child (chains such as {q-{i}}), so a chain pair's key is template + child text + template.
__device__ bool eval_fast(const DevTable& T, const lds_u8* tile, uint32_t p0, uint32_t n,
                          const lds_u32* cm, bool active, uint32_t mode, const FastLds& F,
                          const LaneLds& L, uint32_t& out_len, uint32_t& nseg) {
  bool ok = active && n <= kLeanMax;
  const lds_u8* s = tile + p0;
  // ---- 1. the string's brace events as a 128-bit window (straight-line) ----
  uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  {
    const uint32_t c0 = ok ? p0 >> 4 : 0u, o = p0 & 15u;
    uint32_t Wb[5], Wd[5];
#pragma unroll
    for (int j = 0; j < 5; j++) {
      const uint32_t x = cm[c0 + 2 * j], y = j < 4 ? cm[c0 + 2 * j + 1] : 0u;
      Wb[j] = (x & 0xFFFFu) | (y << 16);
      Wd[j] = (x >> 16) | (y & 0xFFFF0000u);
    }
    uint32_t odd = 0;
    uint32_t* wp[4] = {&w0, &w1, &w2, &w3};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int32_t r = (int32_t)n - 32 * j;
      const uint32_t keep = r >= 32 ? 0xFFFFFFFFu : r > 0 ? (1u << r) - 1u : 0u;
      *wp[j] = __builtin_amdgcn_alignbit(Wb[j + 1], Wb[j], o) & keep;
      odd |= __builtin_amdgcn_alignbit(Wd[j + 1], Wd[j], o) & keep;
    }
    if (odd) ok = false;  // '\' or 0xE3: escapes / U+3020 need the exact evaluator
    if (!ok) w0 = w1 = w2 = w3 = 0;
  }
  // ---- 2. pairs: one wave-uniform pass over the events, predicated push / pop ----
  const uint32_t E = __builtin_popcount(w0) + __builtin_popcount(w1) + __builtin_popcount(w2) +
                     __builtin_popcount(w3);
  const uint32_t Ew = (uint32_t)w_max((int64_t)E);
  uint32_t depth = 0, np = 0, H = 0, ntop = 0, run = 0, tmpl = 0;
  uint32_t hm1 = 0, hm2 = 0, hm3 = 0, hm4 = 0;
  uint32_t st0 = 0, st1 = 0, st2 = 0, st3 = 0;  // open | height << 16 | children << 20
  for (uint32_t k = 0; k < Ew; k++) {
    const bool z0 = w0 == 0, z1 = w1 == 0, z2 = w2 == 0;
    const uint32_t e = !z0 ? (uint32_t)__builtin_ctz(w0 | 0x80000000u * z0)
                     : !z1 ? 32u + (uint32_t)__builtin_ctz(w1 | 0x80000000u * z1)
                     : !z2 ? 64u + (uint32_t)__builtin_ctz(w2 | 0x80000000u * z2)
                           : 96u + (uint32_t)__builtin_ctz(w3 | 0x80000000u);
    if (!z0) w0 &= w0 - 1;
    else if (!z1) w1 &= w1 - 1;
    else if (!z2) w2 &= w2 - 1;
    else w3 &= w3 - 1;
    const bool valid = ok && k < E;
    const uint8_t c = valid ? s[e] : (uint8_t)0;
    if (valid && c == '{') {
      if (depth == (uint32_t)kFastDepth) ok = false;
      st0 = depth == 0 ? e : st0;
      st1 = depth == 1 ? e : st1;
      st2 = depth == 2 ? e : st2;
      st3 = depth == 3 ? e : st3;
      depth++;
    } else if (valid) {  // '}'
      const uint32_t d1 = depth - 1;
      const uint32_t sv = d1 == 0 ? st0 : d1 == 1 ? st1 : d1 == 2 ? st2 : st3;
      const uint32_t open = sv & 0xFFFFu, h = ((sv >> 16) & 0xFu) + 1, nch = sv >> 20;
      // '}{', too many pairs, two children, a whole-string pair (typed-result rules), > 3 top pairs
      if (depth == 0 || np == (uint32_t)kFastPairs || nch > 1 || (open == d1 && e == n - 1 - d1) ||
          (d1 == 0 && ntop == 3))
        ok = false;
      if (ok) {
        uint64_t rec = (uint64_t)open | ((uint64_t)e << 16) | ((uint64_t)d1 << 32) | ((uint64_t)h << 36);
        if (d1 == 0) {
          rec |= (uint64_t)ntop << 56;
          L.seg[2 * ntop * kBlock] = seg_make(kSegTemplate, open - run, run);
          tmpl += open - run;
          run = e + 1;
          ntop++;
        }
        F.pair[np * kBlock] = rec;
        const uint32_t bit = 1u << np;
        hm1 |= h == 1 ? bit : 0u;
        hm2 |= h == 2 ? bit : 0u;
        hm3 |= h == 3 ? bit : 0u;
        hm4 |= h == 4 ? bit : 0u;
        np++;
        H = h > H ? h : H;
        // the parent (level d1 - 1) gains a child of height h
        auto raise = [h](uint32_t v) {
          const uint32_t hh = ((v >> 16) & 0xFu) > h ? ((v >> 16) & 0xFu) : h;
          return (v & 0xFFFFu) | (hh << 16) | (((v >> 20) + 1u) << 20);
        };
        st0 = d1 == 1 ? raise(st0) : st0;
        st1 = d1 == 2 ? raise(st1) : st1;
        st2 = d1 == 3 ? raise(st2) : st2;
      }
      depth = d1;
    }
  }
  if (depth) ok = false;  // unbalanced: the exact evaluator reports it
  // ---- 3. rounds by height: every probe of a round in flight together ----
  uint32_t vb_used = 0, vsum = 0;
  if (mode == 2) {  // diagnostic: parse only (output = template)
    if (ok) nseg = 1, out_len = n, L.seg[0] = seg_make(kSegTemplate, n, 0);
    return ok;
  }
  const uint32_t Hw = (uint32_t)w_max(ok ? (int64_t)H : 0);
  for (uint32_t h = 1; h <= Hw; h++) {
    uint32_t hm = !ok ? 0u : h == 1 ? hm1 : h == 2 ? hm2 : h == 3 ? hm3 : hm4;
    while (__any(hm != 0)) {
      const uint32_t a = hm ? (uint32_t)__builtin_ctz(hm) : 0u;
      bool pa = hm != 0;
      hm &= hm - 1;
      const uint32_t b = hm ? (uint32_t)__builtin_ctz(hm) : 0u;
      bool pb = hm != 0;
      hm &= hm - 1;
      FastKey ka, kb;
      if (!fast_key(s, F, a, pa, ka) && pa) ok = false;
      if (!fast_key(s, F, b, pb, kb) && pb) ok = false;
      if (!ok || mode == 3) pa = pb = false, hm = ok ? hm : 0;  // mode 3: keys only
      // both cuckoo slots of both keys in flight together: one memory latency per sub-round
      const SlotPair xa = slots_of(ka.hash, T.mask), xb = slots_of(kb.hash, T.mask);
      FastProbe A1, A2, B1, B2;
      fast_load(T, pa ? xa.s1 : 0u, A1);
      fast_load(T, pa ? xa.s2 : 0u, A2);
      fast_load(T, pb ? xb.s1 : 0u, B1);
      fast_load(T, pb ? xb.s2 : 0u, B2);
      if (pa) {
        const bool h1 = fast_match(A1, ka), h2 = fast_match(A2, ka);
        if (!(h1 || h2) || !fast_commit(F, L, a, h1 ? xa.s1 : xa.s2, h1 ? A1 : A2, vb_used, vsum))
          ok = false;  // a miss: the exact evaluator decides the error
      }
      if (pb) {
        const bool h1 = fast_match(B1, kb), h2 = fast_match(B2, kb);
        if (!(h1 || h2) || !fast_commit(F, L, b, h1 ? xb.s1 : xb.s2, h1 ? B1 : B2, vb_used, vsum))
          ok = false;
      }
      if (!ok) hm = 0;
    }
  }
  if (ok && mode == 3) {
    nseg = 1, out_len = n, L.seg[0] = seg_make(kSegTemplate, n, 0);
    return ok;
  }
  if (ok) {
    L.seg[2 * ntop * kBlock] = seg_make(kSegTemplate, n - run, run);
    tmpl += n - run;
    nseg = 2 * ntop + 1;
    out_len = tmpl + vsum;
  }
  return ok;
}

// ------------------------------------------------------------------------------------------
// decoupled look-back (wave 0 of the workgroup, all 64 lanes). Words: flag<<62 | value.
// ------------------------------------------------------------------------------------------
constexpr uint64_t kFlagAgg = 1ull << 62, kFlagIncl = 2ull << 62, kValMask = (1ull << 62) - 1;

__device__ __forceinline__ void publish(uint64_t* state, uint32_t tile, uint64_t word) {
  __hip_atomic_store(state + tile, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ uint64_t look_back(uint64_t* state, uint32_t tile, uint64_t agg, uint32_t* err,
                              uint32_t* polls) {
  const uint32_t lane = lane_id();
  if (tile == 0) {
    if (lane == 0) publish(state, 0, kFlagIncl | agg);
    return 0;
  }
  if (lane == 0) publish(state, tile, kFlagAgg | agg);
  uint64_t excl = 0;
  int64_t pos = (int64_t)tile - 1;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  // each poll reads a window of 4 x 64 predecessors (one memory round trip): sub-window q holds
  // distances 64q .. 64q+63 from pos, lane l at distance 64q + l
  for (;;) {
    uint64_t w[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int64_t idx = pos - 64 * q - (int64_t)lane;
      w[q] = idx >= 0 ? __hip_atomic_load(state + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagIncl;
    }
    bool done = false, wait = false;
    uint64_t sum = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (done || wait) continue;  // uniform across the wave
      const uint64_t flag = w[q] >> 62;
      const uint64_t incl_m = __ballot(flag == 2);
      const uint64_t wait_m = __ballot(flag == 0);
      const uint32_t first = incl_m ? (uint32_t)__builtin_ctzll(incl_m) : 64u;
      const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
      if (wait_m & need) {
        wait = true;
        continue;
      }
      sum += w_sum(lane <= first ? (w[q] & kValMask) : 0ull);
      if (first < 64) done = true;
    }
    if (wait) {
      // consume what was complete before the gap: windows before it are final
      // (re-read from the same pos next time, so nothing is double counted)
      if (lane == 0) atomicAdd(polls, 1u);
      __builtin_amdgcn_s_sleep(1);
      // bounded spin: 60 s of s_memrealtime (100 MHz); a missing predecessor is a bug
      if (__builtin_amdgcn_s_memrealtime() - t0 > 6000000000ull) {
        if (lane == 0) atomicOr(err, 1u);
        break;
      }
      continue;
    }
    excl += sum;
    if (done) break;
    pos -= 256;
  }
  if (lane == 0) publish(state, tile, kFlagIncl | (excl + agg));
  return excl;
}

// ------------------------------------------------------------------------------------------
// workgroup scan helper
// ------------------------------------------------------------------------------------------
__device__ uint64_t block_scan(uint64_t v, uint64_t* lds_w, uint64_t* total) {
  const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
  const uint64_t inc = wave_incl_scan(v);
  if (lane == 63) lds_w[wid] = inc;
  __syncthreads();
  uint64_t base = 0, tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < kBlock / 64; w++) {
    const uint64_t x = lds_w[w];
    if (w < wid) base += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

// eval region: key buffers | eval_events' stacks | pair records | inner values. Every lane owns
// one column of each; nothing may alias across columns of different width (waves run the fast
// and the exact evaluator at different times).
constexpr uint32_t kKbufLds = kBlock * kKeyCap;
constexpr uint32_t kStackLds = kMaxDepth * kBlock * 4;
constexpr uint32_t kPairLds = kFastPairs * kBlock * 8;
constexpr uint32_t kEvalLds = kKbufLds + kStackLds + kPairLds + kBlock * kFastVb;
constexpr uint32_t kUnionLds = (kEvalLds > (uint32_t)kStageBytes + 32 ? kEvalLds : (uint32_t)kStageBytes + 32);

__global__ __launch_bounds__(kBlock) void k_resolve(Batch B, Work W, DevTable T, uint8_t* out,
                                                    uint64_t cap) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kTileBytes + 32];
  __shared__ __attribute__((aligned(16))) uint8_t s_u[kUnionLds];  // eval: keys+stacks; emit: stage
  __shared__ __attribute__((aligned(16))) uint64_t s_seg[kMaxSeg * kBlock];
  __shared__ uint32_t s_olen[kBlock];  // output length; the value id for IE_OK_VALUE strings
  __shared__ uint8_t s_st[kBlock];
  __shared__ uint8_t s_nseg[kBlock];
  __shared__ uint16_t s_pend[kBlock];
  __shared__ uint32_t s_misc[4];  // tile, pending count
  __shared__ uint64_t s_red[kBlock / 64 + 2];
  __shared__ uint32_t s_sink[kBlock];  // per-lane write sink of the branch-free LDS writers
  __shared__ uint32_t s_cm[(kTileBytes + 32) / 16 + 10];  // event masks of the staged chunks (+ window pad)

  const uint32_t tid = threadIdx.x, wave = tid >> 6;
  uint64_t t_start = 0;
  if (tid == 0) {
    if (W.stamps) t_start = __builtin_amdgcn_s_memrealtime();
    s_misc[0] = atomicAdd(W.tile_ticket, 1u);
    s_misc[1] = 0;
  }
  __syncthreads();
  const uint32_t tile = s_misc[0];
  // diagnostic phase stamps (100 MHz s_memrealtime), one row of 8 words per tile
  uint64_t* const stamp_row = W.stamps ? W.stamps + (uint64_t)tile * 8 : nullptr;
#define IE_STAMP(k)                                                                  \
  do {                                                                               \
    if (stamp_row && tid == 0) stamp_row[k] = __builtin_amdgcn_s_memrealtime();      \
  } while (0)
  if (stamp_row && tid == 0) {
    stamp_row[0] = t_start;
    uint32_t hw = 0, xcc = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    stamp_row[7] = ((uint64_t)xcc << 32) | hw;
  }
  const uint64_t first = (uint64_t)tile * kBlock;
  const uint64_t last = min(first + (uint64_t)kBlock, B.n);
  const uint64_t i = first + tid;
  const uint64_t lo = gld(B.in_off + first), hi = gld(B.in_off + last);
  const bool staged = (hi - lo) <= (uint64_t)kTileBytes;
  const uintptr_t plo = (uintptr_t)(B.bytes + lo);
  const uint32_t shift = (uint32_t)(plo & 15);
  if (staged) {  // whole 16-byte chunks covering [lo, hi): an aligned chunk never crosses a page
    const uint4* src = (const uint4*)(plo - shift);
    uint4* dst = (uint4*)s_in;
    const uint32_t nv = (uint32_t)((shift + (hi - lo) + 15) >> 4);
    for (uint32_t j = tid; j < nv; j += kBlock) dst[j] = gld4(src + j);
    __syncthreads();
    for (uint32_t c = tid; c < nv; c += kBlock) {  // classify: one event mask per chunk
      ((lds_u32*)s_cm)[c] = chunk_mask((const lds_u32*)(lds_u8*)s_in + 4 * c);
    }
  }
  __syncthreads();
  IE_STAMP(1);

  // ---- 2. evaluate (fast path) ----
  uint64_t so = 0, sn = 0;
  const LaneLds L{(lds_u8*)(s_u + tid * kKeyCap), (lds_u32*)(lds_u8*)(s_u + kKbufLds) + tid,
                  (lds_u64*)s_seg + tid};
  const uint8_t* s = nullptr;
  {
    uint8_t st = IE_OK_STR;
    uint32_t olen = 0, vid = IE_VID_NONE, ns = 0;
    bool active = false;
    if (i < B.n) {
      so = gld(B.in_off + i);
      sn = gld(B.in_off + i + 1) - so;
      s = staged ? s_in + shift + (so - lo) : B.bytes + so;
      active = sn < 0xFFFF0000ull;
      if (!active) st = kStatusPending;
    }
    // wave-uniform calls (the rounds vote across the wave); idle lanes ride along. Clean strings
    // take the level evaluator; the rest (and its failures) the exact event evaluator.
    const uint32_t p0 = shift + (uint32_t)(so - lo);
    uint8_t r = IE_OK_STR;
    if (W.debug_noeval) {
      ns = 1;
      olen = (uint32_t)sn;
      L.seg[0] = seg_make(kSegTemplate, (uint32_t)sn, 0);
    } else if (staged) {
      const FastLds F{(lds_u8*)(s_u + tid * kKeyCap), (lds_u64*)(lds_u8*)(s_u + kKbufLds + kStackLds) + tid,
                      (lds_u8*)(s_u + kKbufLds + kStackLds + kPairLds + tid * kFastVb)};
      const bool fast = eval_fast(T, (const lds_u8*)s_in, p0, (uint32_t)sn, (const lds_u32*)s_cm,
                                  active && W.fast_mode, W.fast_mode, F, L, olen, ns);
      const bool slow = active && !fast;
      const uint64_t slow_m = __ballot(slow);
      if (slow_m) {
        if (lane_id() == 0 && W.fast_mode) atomicAdd(W.stats + 3, (uint32_t)__popcll(slow_m));
        uint32_t o2 = 0, n2 = 0;
        const uint8_t r2 = eval_events(T, (const lds_u8*)s_in + p0, p0, (uint32_t)sn, (const lds_u32*)s_cm,
                                       slow, L, o2, vid, n2);
        if (slow) r = r2, olen = o2, ns = n2;
      }
    } else {
      r = eval_rounds<false, false>(T, Src<false>{s}, (uint32_t)sn, active, L, nullptr, olen, vid, ns);
    }
    if (active) st = r;
    if (i < B.n) {
      if (st == IE_OK_STR && ns > (uint32_t)kMaxSeg) st = kStatusPending;  // too many segments
      if (st == kStatusPending) s_pend[atomicAdd(&s_misc[1], 1u)] = (uint16_t)tid;
    }
    s_st[tid] = st;
    s_olen[tid] = st == IE_OK_STR ? olen : (st == IE_OK_VALUE ? vid : 0u);
    s_nseg[tid] = (uint8_t)(ns > 255u ? 255u : ns);
  }
  __syncthreads();
  IE_STAMP(2);

  // ---- 3. literal path for the pending strings, one wave each ----
  const uint32_t npend = s_misc[1];
  if (tid == 0 && npend) atomicAdd(W.stats, npend);
  for (uint32_t k = wave; k < npend; k += kBlock / 64) {
    const uint32_t j = s_pend[k];
    const uint64_t gi = first + j;
    const uint64_t po = gld(B.in_off + gi), pn = gld(B.in_off + gi + 1) - po;
    uint64_t rcap = W.lit_cap_max ? IE_SIZE_CAP(pn, T.maxtext) + 4 * T.maxtext + 64
                                  : 4 * pn + 4 * T.maxtext + 256;
    rcap = (rcap + 15) & ~15ull;
    uint64_t pbase = 0;
    if (lane_id() == 0) pbase = atomicAdd((unsigned long long*)W.pool_used, (unsigned long long)(4 * rcap));
    pbase = __shfl(pbase, 0, 64);
    LitOut r{IE_E_OVERFLOW, 0, 0, IE_VID_NONE};
    if (pbase + 4 * rcap <= W.pool_bytes)
      r = w_literal(T, B.bytes + po, pn, W.pool + pbase, rcap, pbase, W.lit_cap_max != 0);
    if (lane_id() == 0) {
      s_st[j] = r.status;
      s_olen[j] = r.status == IE_OK_STR ? (uint32_t)r.res_len : (r.status == IE_OK_VALUE ? r.vid : 0u);
      s_seg[j] = seg_make(kSegPool, (uint32_t)r.res_len, (uint32_t)(r.res_off >> 4));
      s_nseg[j] = 1;
    }
  }
  __syncthreads();
  IE_STAMP(3);

  // ---- 4. offsets: workgroup scan + decoupled look-back ----
  const uint8_t st = s_st[tid];
  const uint32_t olen = st == IE_OK_STR ? s_olen[tid] : 0u;
  uint64_t tile_total;
  const uint64_t local = block_scan(olen, s_red, &tile_total);
  if (tid == 128) s_red[kBlock / 64 + 1] = local;  // output offset where the second half starts
  if (wave == 0) {
    const uint64_t b = look_back(W.tile_state, tile, tile_total, W.err, W.stats + 2);
    if (tid == 0) s_red[kBlock / 64] = b;
  }
  __syncthreads();
  IE_STAMP(4);
  const uint64_t base = s_red[kBlock / 64];
  if (i < B.n) {
    gst(B.out_off + i, base + local);
    gst(B.status + i, st);
    if (st == IE_OK_VALUE) gst(B.value_id + i, s_olen[tid]);
  }
  if (last == B.n && tid == 0) {
    B.out_off[B.n] = base + tile_total;
    *W.total = base + tile_total;
  }
  if (base + tile_total > cap) return;  // caller's buffer too small: offsets only
  __syncthreads();  // s_red[kBlock / 64 + 1] (the half boundary) is visible

  // ---- 5. bytes: the tile (or, if it does not fit, each half) through the LDS output stage,
  //      then 16-byte stores ----
  const uint32_t whole = tile_total + 15 <= (uint64_t)kStageBytes;
  const uint32_t half = whole ? 0u : tid >> 7;
  for (uint32_t hsel = 0; hsel < (whole ? 1u : 2u); hsel++) {
    // the part's output range [h_lo, h_hi) relative to the tile
    const uint64_t h_lo = whole || hsel == 0 ? 0 : s_red[kBlock / 64 + 1];
    const uint64_t h_hi = whole ? tile_total : (hsel == 0 ? s_red[kBlock / 64 + 1] : tile_total);
    uint8_t* g = out + base + h_lo;
    const uint64_t h_len = h_hi - h_lo;
    const uint32_t oshift = (uint32_t)(((uintptr_t)g) & 15);
    const bool direct = !staged || h_len + oshift > (uint64_t)kStageBytes;
    const bool mine = half == hsel && i < B.n && st == IE_OK_STR && olen;
    const uint32_t ns = s_nseg[tid];
    if (direct) {  // rare (long strings): lanes store their own bytes straight to HBM
      if (tid == 0) atomicAdd(W.stats + 1, 1u);
      if (mine) {
        uint8_t* d = g + (local - h_lo);
        uint32_t w = 0;
        for (uint32_t k = 0; k < ns; k++) {
          const uint64_t sg = ((const lds_u64*)s_seg)[k * kBlock + tid];
          const uint32_t kind = (uint32_t)(sg >> 62), len = (uint32_t)(sg >> 32) & 0x3FFFFFFFu,
                         src = (uint32_t)sg;
          const uint8_t* p = kind == kSegTemplate ? s + src
                             : kind == kSegValue  ? T.arena + src
                             : kind == kSegBucket ? T.buckets[src].text
                                                  : W.pool + ((uint64_t)src << 4);
          for (uint32_t q = 0; q < len; q++) gst(d + w + q, p[q]);
          w += len;
        }
      }
      continue;
    }
    __syncthreads();  // the union region becomes the output stage (keys/stacks are dead)
    {
      // wave-uniform loop over segment indices; lanes without that segment write nothing
      lds_u8* const sink = (lds_u8*)(s_sink + tid);
      lds_u8* const d = (lds_u8*)(s_u + oshift + (mine ? local - h_lo : 0));
      const uint32_t nsl = mine ? ns : 0u;
      uint32_t w = 0;
      for (uint32_t k = 0; __any(k < nsl); k++) {
        const bool has = k < nsl;
        const uint64_t sg = has ? ((const lds_u64*)s_seg)[k * kBlock + tid] : 0ull;
        const uint32_t kind = (uint32_t)(sg >> 62), len = (uint32_t)(sg >> 32) & 0x3FFFFFFFu,
                       src = (uint32_t)sg;
        const bool tpl = has && kind == kSegTemplate, bkt = has && kind == kSegBucket;
        if (__any(tpl))
          lds_copy(d + w, tpl ? (const lds_u8*)s + src : (const lds_u8*)s_in, tpl ? len : 0u, sink);
        if (__any(bkt)) put_bucket_text(d + w, T.buckets + (bkt ? src : 0u), bkt ? len : 0u, sink);
        if (has && kind == kSegValue)
          copy_bytes<true, false>((uint8_t*)(d + w), T.arena + src, len);
        else if (has && kind == kSegPool)
          copy_bytes<true, false>((uint8_t*)(d + w), W.pool + ((uint64_t)src << 4), len);
        w += has ? len : 0u;
      }
    }
    __syncthreads();
    // stream the stage out: LDS position oshift + k holds output byte h_lo + k
    const uintptr_t pg = (uintptr_t)g, pe = pg + h_len;
    const uintptr_t a_up = (pg + 15) & ~(uintptr_t)15, b_down = pe & ~(uintptr_t)15;
    if (a_up >= b_down) {
      for (uint32_t k = tid; k < h_len; k += kBlock) gst(g + k, s_u[oshift + k]);
    } else {
      const uint32_t head = (uint32_t)(a_up - pg), tail = (uint32_t)(pe - b_down);
      if (tid < head) gst(g + tid, s_u[oshift + tid]);
      if (tid < tail) {
        const uint32_t k = (uint32_t)(b_down - pg) + tid;
        gst(g + k, s_u[oshift + k]);
      }
      const uint32_t nv = (uint32_t)((b_down - a_up) >> 4);
      const uint4* src = (const uint4*)(s_u + oshift + head);
      uint4* dstv = (uint4*)a_up;
      for (uint32_t j = tid; j < nv; j += kBlock) gst4(dstv + j, src[j]);
    }
  }
  IE_STAMP(5);
#undef IE_STAMP
}

// diagnostic: one key through the device lookups. out[0..1] hash, out[2] s1, out[3] s2,
// out[4] find_bytes, out[5] find_small (klen <= kInlineKey), out[6] mask
__global__ void k_debug_probe(DevTable T, const uint8_t* key, uint32_t klen, uint64_t* out) {
  __shared__ uint32_t kb[16];
  const uint32_t lane = threadIdx.x;
  if (lane < 16) kb[lane] = 0;
  __syncthreads();
  if (lane == 0)
    for (uint32_t j = 0; j < klen && j < 64; j++) ((uint8_t*)kb)[j] = key[j];
  __syncthreads();
  // all 64 lanes, uniformly (as the literal path calls it)
  Hit hw{0, 0, 0, 0};
  const int32_t fw = find_bytes(T, key, klen, hw);
  const uint64_t agree = __ballot(fw == __shfl(fw, 0, 64) && hw.text_off == __shfl(hw.text_off, 0, 64));
  if (lane != 0) return;
  const uint64_t hash = hash_key(klen, [&](uint32_t j) { return key[j]; });
  const SlotPair sp = slots_of(hash, T.mask);
  Hit h;
  const int32_t fb = find_bytes(T, key, klen, h);
  const int32_t fs = klen <= kInlineKey ? find_small(T, (const lds_u32*)(lds_u8*)(uint8_t*)kb, klen, h) : -2;
  out[0] = hash;
  out[1] = hash >> 32;
  out[2] = sp.s1;
  out[3] = sp.s2;
  out[4] = (uint64_t)(int64_t)fb;
  out[5] = (uint64_t)(int64_t)fs;
  out[6] = T.mask;
  out[12] = (uint64_t)(int64_t)fw;
  out[13] = agree;
  out[14] = hw.text_off;
  out[15] = h.text_off;
}

hipError_t launch_debug_probe(const DevTable& T, const uint8_t* key, uint32_t klen, uint64_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_debug_probe, dim3(1), dim3(64), 0, st, T, key, klen, out);
  return hipGetLastError();
}

hipError_t launch_resolve(const Batch& B, const Work& W, const DevTable& T, uint8_t* out, uint64_t cap,
                          hipStream_t st) {
  const uint64_t tiles = (B.n + kBlock - 1) / kBlock;
  if (!tiles) return hipSuccess;
  hipLaunchKernelGGL(k_resolve, dim3((uint32_t)tiles), dim3(kBlock), 0, st, B, W, T, out, cap);
  return hipGetLastError();
}

}  // namespace ie
