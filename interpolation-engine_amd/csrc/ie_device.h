// ie_device.h — device-side building blocks shared by the kernels: wave primitives, the
// get_interpdata lookup (py:430-467 / interp.rs:91-137) against the bucketed device table.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ie_amd.h"
#include "ie_common.h"

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
// lookups
// ------------------------------------------------------------------------------------------
struct Hit {
  uint32_t text_len, text_off, vid, flags;
};

// a: table arena (global), b: any address space
__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  bool eq = true;
  for (uint32_t j = 0; j < n; j++) eq &= gld(a + j) == b[j];
  return eq;
}

__device__ __forceinline__ Hit hit_of(uint4 q0, uint4 q1) {
  return Hit{q0.w, q1.w, q1.x, q1.y};
}

// Lookup of a key whose bytes are at `key` (any address space): both cuckoo slots. Returns the
// bucket or -1.
// (Written without a loop: an unrolled two-iteration loop with an early return compiled to code
// that returned the second slot's index without writing `h`.)
__device__ int32_t find_bytes(const DevTable& T, const uint8_t* key, uint32_t klen, Hit& h) {
  const uint64_t hash = hash_key(klen, [&](uint32_t j) { return key[j]; });
  const SlotPair sp = slots_of(hash, T.mask);
  const uint4* b1 = (const uint4*)(T.buckets + sp.s1);
  const uint4* b2 = (const uint4*)(T.buckets + sp.s2);
  const uint4 a0 = gld4(b1), a1 = gld4(b1 + 1), c0 = gld4(b2), c1 = gld4(b2 + 1);
  const bool ma = ((a1.y & EF_OCCUPIED) != 0) & ((((uint64_t)a0.y << 32) | a0.x) == hash) & (a0.z == klen);
  const bool mc = ((c1.y & EF_OCCUPIED) != 0) & ((((uint64_t)c0.y << 32) | c0.x) == hash) & (c0.z == klen);
  const bool ha = ma && bytes_eq(T.arena + a1.z, key, klen);
  const bool hc = !ha && mc && bytes_eq(T.arena + c1.z, key, klen);
  h = ha ? hit_of(a0, a1) : hit_of(c0, c1);
  return ha ? (int32_t)sp.s1 : hc ? (int32_t)sp.s2 : -1;
}

// Lookup of a key held in LDS at a 4-byte aligned address, klen <= kInlineKey: the key is read
// as dwords and hashed word-wise; both slots' 64-byte bursts (header + inline key) go out
// together and are compared dword-wise in registers.
__device__ __forceinline__ int32_t find_small(const DevTable& T, const __attribute__((address_space(3))) uint32_t* key32,
                                              uint32_t klen, Hit& h) {
  uint64_t hash = 0xA0761D6478BD642Full ^ (uint64_t)klen;
  uint32_t kw[8];
#pragma unroll
  for (int d = 0; d < 8; d++) {
    const int32_t rem = (int32_t)klen - 4 * d;
    kw[d] = 0;
    if (rem > 0) {
      const uint32_t w = key32[d];
      kw[d] = rem >= 4 ? w : (w & ((1u << (8 * rem)) - 1u));  // buckets are zero padded
      hash = hash_word(hash, kw[d]);
    }
  }
  const SlotPair sp = slots_of(hash, T.mask);
  const uint4* b1 = (const uint4*)(T.buckets + sp.s1);
  const uint4* b2 = (const uint4*)(T.buckets + sp.s2);
  const uint4 a0 = gld4(b1), a1 = gld4(b1 + 1), a2 = gld4(b1 + 2), a3 = gld4(b1 + 3);
  const uint4 c0 = gld4(b2), c1 = gld4(b2 + 1), c2 = gld4(b2 + 2), c3 = gld4(b2 + 3);
  auto eq = [&](uint4 q0, uint4 q1, uint4 q2, uint4 q3) {
    return ((q1.y & EF_OCCUPIED) != 0) & ((((uint64_t)q0.y << 32) | q0.x) == hash) & (q0.z == klen) &
           (q2.x == kw[0]) & (q2.y == kw[1]) & (q2.z == kw[2]) & (q2.w == kw[3]) &
           (q3.x == kw[4]) & (q3.y == kw[5]) & (q3.z == kw[6]) & (q3.w == kw[7]);
  };
  if (eq(a0, a1, a2, a3)) {
    h = hit_of(a0, a1);
    return (int32_t)sp.s1;
  }
  if (eq(c0, c1, c2, c3)) {
    h = hit_of(c0, c1);
    return (int32_t)sp.s2;
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

// lookup with the RAW value of bucket `prev` as the key (nested whole-string form,
// py:511-512: the object itself; interp.rs:47-48: value_to_string of it)
__device__ int32_t find_raw(const DevTable& T, const Hit& prev, uint8_t& st, Hit& h) {
  if (!(prev.flags & EF_KEY_STR)) {
    st = (prev.flags & EF_KEY_UNHASHABLE) ? (uint8_t)IE_E_UNHASHABLE
         : (T.flags & TF_HAS_DIR)         ? (uint8_t)IE_NEEDS_HOST
                                          : (uint8_t)IE_E_INTERP;
    return -1;
  }
  const uint8_t* k = T.arena + prev.text_off;
  const int32_t b = find_bytes(T, k, prev.text_len, h);
  if (b < 0) st = missing_status(T, k, prev.text_len);
  return b;
}

}  // namespace ie
