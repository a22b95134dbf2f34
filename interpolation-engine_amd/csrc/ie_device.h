// ie_device.h — device-side building blocks shared by the kernels: wave primitives, the
// get_interpdata lookup (py:430-467 / interp.rs:91-137) against the perfect-hash device table.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ie_amd.h"
#include "ie_common.h"

// once-streamed input and output with the non-temporal policy (keeps the table in L2; config 3
// k_resolve 0.975 -> 0.937 ms)
#ifndef IE_NT
#define IE_NT 1
#endif

namespace ie {

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// explicit address spaces: loads through these compile to global_* / ds_* instead of flat_*
template <class T>
__device__ __forceinline__ T gld(const T* p) {
  return *(const __attribute__((address_space(1))) T*)p;
}
template <class T>
__device__ __forceinline__ void gst(T* p, T v) {
  *(__attribute__((address_space(1))) T*)p = v;
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gld4(const uint4* p) {
  const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)(const void*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gst4(uint4* p, uint4 v) {
  u32x4 w;
  w.x = v.x; w.y = v.y; w.z = v.z; w.w = v.w;
  *(__attribute__((address_space(1))) u32x4*)(void*)p = w;
}

// once-streamed bytes (batch input, output): non-temporal with IE_NT, so that the scattered
// table lines keep their place in L2
__device__ __forceinline__ uint4 gld4s(const uint4* p) {
#if IE_NT
  const u32x4 v = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4*)(const void*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return gld4(p);
#endif
}
__device__ __forceinline__ void gst4s(uint4* p, uint4 v) {
#if IE_NT
  u32x4 w;
  w.x = v.x; w.y = v.y; w.z = v.z; w.w = v.w;
  __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x4*)(void*)p);
#else
  gst4(p, v);
#endif
}
template <class T>
__device__ __forceinline__ void gsts(T* p, T v) {
#if IE_NT
  __builtin_nontemporal_store(v, (__attribute__((address_space(1))) T*)p);
#else
  gst(p, v);
#endif
}

// Tile staging: nv 16-byte chunks src -> dst (LDS), every load of the thread in flight before
// the first LDS write (a plain strided loop waits for each load before issuing the next).
template <int BLOCK, int MAXV>
__device__ __forceinline__ void stage_chunks(uint4* dst, const uint4* src, uint32_t nv, uint32_t tid) {
  uint4 v[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; k++) {
    const uint32_t j = tid + (uint32_t)k * BLOCK;
    if (j < nv) v[k] = gld4(src + j);
  }
#pragma unroll
  for (int k = 0; k < MAXV; k++) {
    const uint32_t j = tid + (uint32_t)k * BLOCK;
    if (j < nv) dst[j] = v[k];
  }
}

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t t = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}

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

// ------------------------------------------------------------------------------------------
// lookups: perfect hash (ie_common.h) -> one candidate entry, full byte compare
// ------------------------------------------------------------------------------------------
struct Hit {
  uint32_t text_len, text_off, vid, flags;
};

__device__ __forceinline__ uint32_t ph_lookup_slot(const DevTable& T, uint64_t h) {
#ifdef IE_CUCKOO
  uint32_t s1, s2;
  ck_slots(h, T.m, s1, s2);
  return s1;
#else
  const uint32_t pilot = gld(T.pilots + ph_group(h, T.nb));
  return ph_slot(h, pilot, T.m);
#endif
}

// the rest of a long key (bytes 16..klen) against the arena copy; b in any address space
__device__ __forceinline__ bool long_key_eq(const DevTable& T, uint4 q0, const uint8_t* b, uint32_t klen) {
  const uint8_t* a = T.arena + key_off_of(q0.w, q0.y);
  bool eq = true;
  for (uint32_t j = kInlineKey; j < klen; j++) eq &= gld(a + j) == b[j];
  return eq;
}

__device__ __forceinline__ bool entry_head_ok(uint4 q0, uint32_t klen, uint32_t tid) {
  return ((q0.z & EF_OCCUPIED) != 0) & (q0.x == klen) & ((q0.z >> kTidShift) == tid);
}

// Lookup of a key whose bytes are at `key` (generic pointer: LDS or global) in table `tid` of the
// set. Returns the entry index or -1.
__device__ int32_t find_bytes(const DevTable& T, uint32_t tid, const uint8_t* key, uint32_t klen, Hit& h) {
  const uint64_t hash = hash_key(klen, [&](uint32_t j) { return key[j]; }, T.seed, tid);
#ifdef IE_CUCKOO
  uint32_t cs[2];
  ck_slots(hash, T.m, cs[0], cs[1]);
  for (int c = 0; c < 2; c++) {
    const uint32_t slot = cs[c];
#else
  {
    const uint32_t slot = ph_lookup_slot(T, hash);
#endif
    const Entry* e = T.entries + slot;
    const uint4 q0 = gld4((const uint4*)e), q1 = gld4((const uint4*)e + 1);
    const uint32_t kw[4] = {q1.x, q1.y, q1.z, q1.w};
    bool eq = entry_head_ok(q0, klen, tid);
    const uint32_t ni = klen < kInlineKey ? klen : kInlineKey;
    for (uint32_t j = 0; j < ni; j++) eq &= (uint8_t)(kw[j >> 2] >> (8 * (j & 3))) == key[j];
    if (eq && klen > kInlineKey) eq = long_key_eq(T, q0, key, klen);
    h = Hit{q0.y, q0.w, gld(&e->vid), q0.z};
    if (eq) return (int32_t)slot;
  }
  return -1;
}

// Lookup of a key held as dwords at a 4-byte aligned address (generic pointer),
// klen <= kInlineKey: hashed word-wise, compared against the entry's inline key in registers.
__device__ __forceinline__ int32_t find_small(const DevTable& T, uint32_t tid, const uint32_t* key32, uint32_t klen,
                                             Hit& h) {
  uint64_t hash = hash_init(klen, T.seed, tid);
  uint32_t kw[4];
#pragma unroll
  for (int d = 0; d < 4; d++) {
    const int32_t rem = (int32_t)klen - 4 * d;
    kw[d] = 0;
    if (rem > 0) {
      const uint32_t w = key32[d];
      kw[d] = rem >= 4 ? w : (w & ((1u << (8 * rem)) - 1u));  // entries are zero padded
      hash = hash_word(hash, kw[d]);
    }
  }
#ifdef IE_CUCKOO
  uint32_t s1, s2;
  ck_slots(hash, T.m, s1, s2);
  const Entry* e = T.entries + s1;
  const Entry* e2 = T.entries + s2;
  const uint4 a0 = gld4((const uint4*)e), a1 = gld4((const uint4*)e + 1);
  const uint4 b0 = gld4((const uint4*)e2), b1 = gld4((const uint4*)e2 + 1);
  const bool eqb = entry_head_ok(b0, klen, tid) & (b1.x == kw[0]) & (b1.y == kw[1]) & (b1.z == kw[2]) & (b1.w == kw[3]);
  const uint4 q0 = eqb ? b0 : a0, q1 = eqb ? b1 : a1;
  const uint32_t slot = eqb ? s2 : s1;
  e = eqb ? e2 : e;
#else
  const uint32_t slot = ph_lookup_slot(T, hash);
  const Entry* e = T.entries + slot;
  const uint4 q0 = gld4((const uint4*)e), q1 = gld4((const uint4*)e + 1);
#endif
  const bool eq = entry_head_ok(q0, klen, tid) & (q1.x == kw[0]) & (q1.y == kw[1]) & (q1.z == kw[2]) & (q1.w == kw[3]);
  h = Hit{q0.y, q0.w, gld(&e->vid), q0.z};
  return eq ? (int32_t)slot : -1;
}

// status of a key that is not in the table (py:437-467 / interp.rs:105-136). A table built with
// IE_TABLE_HAS_INSERTS_DIR holds the inserts directory's snapshot after the inserts
// (get_interpdata's file fallback, py:452-461, for every key a file answers), so a key it lacks
// is missing there too, unless it is not a canonical relative file name (absolute, an empty, '.'
// or '..' component, a NUL): os.path.join may then reach outside the directory, and the host
// decides (IE_NEEDS_HOST).
__device__ uint8_t missing_status(const DevTable& T, const uint8_t* k, uint32_t n) {
  if (n == 0 || !(T.flags & TF_HAS_DIR)) return IE_E_INTERP;
  // a canonical relative path (components separated by single '/', none empty, '.' or '..',
  // no NUL) names a file inside the directory, which the snapshot covers; anything else is
  // the host's
  bool odd = false;
  uint32_t c0 = 0;
  for (uint32_t j = 0; j <= n && !odd; j++) {
    if (j < n && k[j] == 0) odd = true;
    if (j == n || k[j] == '/') {
      const uint32_t cl = j - c0;
      odd |= cl == 0 || (cl == 1 && k[c0] == '.') || (cl == 2 && k[c0] == '.' && k[c0 + 1] == '.');
      c0 = j + 1;
    }
  }
  return odd ? (uint8_t)IE_NEEDS_HOST : (uint8_t)IE_E_INTERP;
}

// lookup with the RAW value of bucket `prev` as the key (nested whole-string form,
// py:511-512: the object itself; interp.rs:47-48: value_to_string of it)
// the raw value's text: a str value as it is (a pre-resolved one: its raw text), any other the
// text the reference's message shows for it (str() of the object, py:467)
__device__ __forceinline__ const uint8_t* raw_text(const DevTable& T, const Hit& prev, uint32_t& kl) {
  const uint8_t* k = T.arena + prev.text_off;
  kl = prev.text_len;
  if (prev.flags & EF_RAWALT) {  // a pre-resolved splice text: the key is the raw value
    kl = gld((const uint32_t*)(k - 4));
    k -= 4 + ((kl + 3u) & ~3u);
  }
  return k;
}

__device__ int32_t find_raw(const DevTable& T, uint32_t tid, const Hit& prev, uint8_t& st, Hit& h) {
  if (!(prev.flags & EF_KEY_STR)) {
    st = (prev.flags & EF_KEY_UNHASHABLE) ? (uint8_t)IE_E_UNHASHABLE
         : (T.flags & TF_HAS_DIR)         ? (uint8_t)IE_NEEDS_HOST
                                          : (uint8_t)IE_E_INTERP;
    return -1;
  }
  uint32_t kl;
  const uint8_t* k = raw_text(T, prev, kl);
  const int32_t b = find_bytes(T, tid, k, kl, h);
  if (b < 0) st = missing_status(T, k, kl);
  return b;
}

}  // namespace ie
