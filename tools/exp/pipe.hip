// Pipeline-floor experiment (diagnostic, not product): verbatim copy of a packed string batch
// through (A) the round-1 tile structure (one tile per workgroup, register staging) and
// (B) a persistent workgroup loop with LDS-DMA prefetch of the next tile. Both keep the
// decoupled look-back, the LDS output stage and the aligned 16-byte stream-out.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kBlock = 256;
#ifndef TILE_BYTES
#define TILE_BYTES 17408
#endif
constexpr int kTileBytes = TILE_BYTES;
constexpr int kStageBytes = 20480;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u128;

template <class T> __device__ __forceinline__ T gld(const T* p) { return *(const __attribute__((address_space(1))) T*)p; }
template <class T> __device__ __forceinline__ void gst(T* p, T v) { *(__attribute__((address_space(1))) T*)p = v; }
__device__ __forceinline__ uint4 gld4(const uint4* p) { const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)(const void*)p; return make_uint4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ void gst4(uint4* p, uint4 v) { u32x4 w; w.x=v.x; w.y=v.y; w.z=v.z; w.w=v.w; *(__attribute__((address_space(1))) u32x4*)(void*)p = w; }
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

struct Args { const uint8_t* in; const uint64_t* off; uint64_t n; uint8_t* out; uint64_t* ooff; uint8_t* st; uint64_t* state; uint32_t* err; uint64_t* stamps; uint64_t* sstate; };
__device__ uint32_t g_polls;

constexpr uint64_t kFlagAgg = 1ull << 62, kFlagIncl = 2ull << 62, kValMask = (1ull << 62) - 1;
__device__ __forceinline__ void publish(uint64_t* s, uint32_t t, uint64_t w) { __hip_atomic_store(s + t, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint64_t lb_poll(const uint64_t* s, int64_t pos) {
  const int64_t idx = pos - (int64_t)lane_id();
  return idx >= 0 ? __hip_atomic_load(s + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagIncl;
}
__device__ __forceinline__ uint64_t w_sum(uint64_t v) { for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64); return v; }
__device__ uint64_t look_back(uint64_t* state, uint32_t tile, uint64_t agg, uint32_t* err, uint64_t early) {
  const uint32_t lane = lane_id();
  if (tile == 0) return 0;
  uint64_t excl = 0; int64_t pos = (int64_t)tile - 1;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t nap = 1, npoll = 0;
  for (bool use_early = true;; use_early = false) {
    const uint64_t w = use_early ? early : lb_poll(state, pos);
    const uint64_t flag = w >> 62;
    const uint64_t incl_m = __ballot(flag == 2), wait_m = __ballot(flag == 0);
    const uint32_t first = incl_m ? (uint32_t)__builtin_ctzll(incl_m) : 64u;
    const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
    if (wait_m & need) {
      npoll++;
      if (use_early) continue;
      for (uint32_t k = 0; k < nap; k++) __builtin_amdgcn_s_sleep(1);
      nap = nap < 32 ? 2 * nap : 32;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { if (lane == 0) atomicOr(err, 1u); break; }
      continue;
    }
    excl += w_sum(lane <= first ? (w & kValMask) : 0ull);
    if (first < 64) break;
    pos -= 64;
  }
  if (lane == 0) publish(state, tile, kFlagIncl | (excl + agg));
  if (lane == 0 && npoll) atomicAdd(&g_polls, npoll);
  return excl;
}
// look-back over a 256-tile window per poll: lane l reads the words of predecessors
// pos-4l .. pos-4l-3 (all four loads in flight together)
template <int SLEEP>
__device__ uint64_t look_back4(uint64_t* state, uint32_t tile, uint64_t agg, uint32_t* err) {
  const uint32_t lane = lane_id();
  if (tile == 0) return 0;
  uint64_t excl = 0; int64_t pos = (int64_t)tile - 1;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    uint64_t w[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int64_t idx = pos - 4 * (int64_t)lane - k;
      w[k] = idx >= 0 ? __hip_atomic_load(state + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagIncl;
    }
    // per lane: the first inclusive among its 4 (nearest first), a gap before it, the sum up to it
    uint32_t fi = 4; bool gap = false; uint64_t sum = 0;
#pragma unroll
    for (int k = 3; k >= 0; k--) {
      const uint64_t f = w[k] >> 62;
      if (f == 2) { fi = k; gap = false; sum = 0; }
      if (f == 0) gap = true;
      sum += w[k] & kValMask;
    }
    // recompute exactly: sum over k <= fi, gap over k <= fi
    sum = 0; gap = false;
#pragma unroll
    for (int k = 0; k < 4; k++) if ((uint32_t)k <= fi) { sum += w[k] & kValMask; gap |= (w[k] >> 62) == 0; }
    const uint64_t incl_m = __ballot(fi < 4);
    const uint32_t first = incl_m ? (uint32_t)__builtin_ctzll(incl_m) : 64u;
    const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
    if (__ballot(gap) & need) {
      if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { if (lane == 0) atomicOr(err, 1u); break; }
      continue;
    }
    excl += w_sum(lane <= first ? sum : 0ull);
    if (first < 64) break;
    pos -= 256;
  }
  if (lane == 0) publish(state, tile, kFlagIncl | (excl + agg));
  return excl;
}
// look-back over R x 64 predecessors per poll: row k, lane l reads the word of tile pos-64k-l
// (each row one coalesced 512-byte read); early = the first row, polled before the build
template <int R, int NAPMAX>
__device__ uint64_t look_back_rows(uint64_t* state, uint32_t tile, uint64_t agg, uint32_t* err, uint64_t early) {
  const uint32_t lane = lane_id();
  if (tile == 0) return 0;
  uint64_t excl = 0; int64_t pos = (int64_t)tile - 1;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t nap = 1;
  for (bool first_poll = true;; first_poll = false) {
    uint64_t w[R];
#pragma unroll
    for (int k = 0; k < R; k++) {
      const int64_t idx = pos - 64 * k - (int64_t)lane;
      w[k] = (k == 0 && first_poll) ? early
           : idx >= 0 ? __hip_atomic_load(state + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagIncl;
    }
    bool gap = false, done = false;
    uint64_t part = 0;
#pragma unroll
    for (int k = 0; k < R; k++) {
      if (!done && !gap) {
        const uint64_t flag = w[k] >> 62;
        const uint64_t incl_m = __ballot(flag == 2), wait_m = __ballot(flag == 0);
        const uint32_t first = incl_m ? (uint32_t)__builtin_ctzll(incl_m) : 64u;
        const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
        if (wait_m & need) gap = true;
        else { part += w_sum(lane <= first ? (w[k] & kValMask) : 0ull); done = first < 64; }
      }
    }
    if (gap) {
      for (uint32_t k = 0; k < nap; k++) __builtin_amdgcn_s_sleep(1);
      nap = nap < NAPMAX ? 2 * nap : NAPMAX;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { if (lane == 0) atomicOr(err, 1u); break; }
      continue;
    }
    excl += part;
    if (done) break;
    pos -= 64 * R;
  }
  if (lane == 0) publish(state, tile, kFlagIncl | (excl + agg));
  return excl;
}
// two-level look-back: tiles publish only aggregates; the last tile of each super-tile of 64
// publishes the super-tile's aggregate, then its inclusive prefix. A tile's exclusive prefix =
// (the aggregates of its super-tile's earlier tiles: one 64-word window) + (the super-tile's
// exclusive prefix: a look-back over super words, 64 super-tiles = 4096 tiles per poll).
constexpr uint32_t kSuper = 64;
__device__ uint32_t g_polls2;
template <int NAPMAX>
__device__ uint64_t look_back2(uint64_t* state, uint64_t* sstate, uint32_t tile, uint32_t ntiles, uint64_t agg, uint32_t* err) {
  const uint32_t lane = lane_id();
  const uint32_t S = tile / kSuper, j = tile % kSuper;
  const bool last = j == kSuper - 1 || tile == ntiles - 1;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  // in-super prefix: tiles S*64 .. tile-1 (lane l reads tile-1-l, l < j)
  uint64_t in_s = 0, ex_s = 0;
  bool have_in = j == 0, have_ex = S == 0;
  int64_t spos = (int64_t)S - 1;
  uint32_t nap = 1, npoll = 0;
  for (;;) {
    uint64_t w = 0, v = 0;
    if (!have_in) w = lane < j ? __hip_atomic_load(state + tile - 1 - lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagAgg;
    if (!have_ex) v = spos - (int64_t)lane >= 0 ? __hip_atomic_load(sstate + spos - lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagIncl;
    bool again = false;
    if (!have_in) {
      if (__ballot((w >> 62) == 0)) again = true;
      else { in_s = w_sum(w & kValMask); have_in = true;
        if (last && lane == 0) publish(sstate, S, (S == 0 ? kFlagIncl : kFlagAgg) | (in_s + agg)); }
    }
    if (!have_ex) {
      const uint64_t flag = v >> 62;
      const uint64_t incl_m = __ballot(flag == 2), wait_m = __ballot(flag == 0);
      const uint32_t first = incl_m ? (uint32_t)__builtin_ctzll(incl_m) : 64u;
      const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
      if (wait_m & need) again = true;
      else { ex_s += w_sum(lane <= first ? (v & kValMask) : 0ull); if (first < 64) have_ex = true; else spos -= 64; }
    }
    if (have_in && have_ex) break;
    if (again) {
      npoll++;
      for (uint32_t k = 0; k < nap; k++) __builtin_amdgcn_s_sleep(1);
      nap = nap < NAPMAX ? 2 * nap : NAPMAX;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { if (lane == 0) atomicOr(err, 1u); break; }
    }
  }
  if (last && S > 0 && lane == 0) publish(sstate, S, kFlagIncl | (ex_s + in_s + agg));
  if (lane == 0 && npoll) atomicAdd(&g_polls2, npoll);
  return ex_s + in_s;
}
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  const uint32_t lane = lane_id();
  for (int d = 1; d < 64; d <<= 1) { const uint64_t t = __shfl_up(v, d, 64); if (lane >= (uint32_t)d) v += t; }
  return v;
}
__device__ __forceinline__ void raw_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
template <bool RAW>
__device__ uint64_t block_scan(uint64_t v, uint64_t* lds_w, uint64_t* total) {
  const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
  const uint64_t inc = wave_incl_scan(v);
  if (lane == 63) lds_w[wid] = inc;
  if (RAW) raw_barrier(); else __syncthreads();
  uint64_t base = 0, tot = 0;
  for (uint32_t w = 0; w < kBlock / 64; w++) { const uint64_t x = lds_w[w]; if (w < wid) base += x; tot += x; }
  if (RAW) raw_barrier(); else __syncthreads();
  *total = tot;
  return base + inc - v;
}
__device__ __forceinline__ u32x4 ld16a(const lds_u8* p) {
  const uint32_t sh = (uint32_t)(uintptr_t)p & 3u;
  const lds_u32* q = (const lds_u32*)(p - sh);
  const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
  return u32x4{__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
               __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
}
__device__ __forceinline__ void put_tail4(lds_u8* p, u32x4 v, uint32_t n) {
  lds_u32* q = (lds_u32*)p;
  if (n >= 4) q[0] = v.x; if (n >= 8) q[1] = v.y; if (n >= 12) q[2] = v.z;
  const uint32_t nw = n >> 2, r = n & 3u;
  const uint32_t x = nw == 0 ? v.x : nw == 1 ? v.y : nw == 2 ? v.z : v.w;
  lds_u8* b = p + (n & ~3u);
  if (r & 2u) *(__attribute__((address_space(3))) uint16_t*)b = (uint16_t)x;
  if (r & 1u) b[r & 2u] = (uint8_t)(x >> (8u * (r & 2u)));
}
__device__ __forceinline__ void lds_copy(lds_u8* dst, const lds_u8* src, uint32_t len) {
  const uint32_t h0 = (0u - (uint32_t)(uintptr_t)dst) & 3u, h = h0 < len ? h0 : len;
  if (h > 0) dst[0] = src[0]; if (h > 1) dst[1] = src[1]; if (h > 2) dst[2] = src[2];
  const uint32_t body = (len - h) & ~15u;
  for (uint32_t k = 0; __any(k < body); k += 16u) {
    if (k < body) { const u32x4 v = ld16a(src + h + k); lds_u32* q = (lds_u32*)(dst + h + k); q[0] = v.x, q[1] = v.y, q[2] = v.z, q[3] = v.w; }
  }
  const uint32_t kt = h + body;
  if (kt < len) put_tail4(dst + kt, ld16a(src + kt), len - kt);
}
__device__ __forceinline__ uint4 bytes_at(u32x4 x, u32x4 y, uint32_t r) {
  const uint32_t sb = r & 3u; uint32_t a0, a1, a2, a3, a4;
  switch (r >> 2) {
    case 0: a0 = x.x, a1 = x.y, a2 = x.z, a3 = x.w, a4 = y.x; break;
    case 1: a0 = x.y, a1 = x.z, a2 = x.w, a3 = y.x, a4 = y.y; break;
    case 2: a0 = x.z, a1 = x.w, a2 = y.x, a3 = y.y, a4 = y.z; break;
    default: a0 = x.w, a1 = y.x, a2 = y.y, a3 = y.z, a4 = y.w; break;
  }
  return make_uint4(__builtin_amdgcn_alignbyte(a1, a0, sb), __builtin_amdgcn_alignbyte(a2, a1, sb),
                    __builtin_amdgcn_alignbyte(a3, a2, sb), __builtin_amdgcn_alignbyte(a4, a3, sb));
}
// stream the stage s_out[0, total) to g (16-byte aligned stores)
__device__ __forceinline__ void stream_out(uint8_t* g, const uint8_t* s_out, uint32_t total, uint32_t tid) {
  const uintptr_t pg = (uintptr_t)g, pe = pg + total;
  const uintptr_t a_up = (pg + 15) & ~(uintptr_t)15, b_down = pe & ~(uintptr_t)15;
  if (a_up >= b_down) { for (uint32_t k = tid; k < total; k += kBlock) gst(g + k, s_out[k]); return; }
  const uint32_t head = (uint32_t)(a_up - pg), tail = (uint32_t)(pe - b_down);
  if (tid < head) gst(g + tid, s_out[tid]);
  if (tid < tail) { const uint32_t k = (uint32_t)(b_down - pg) + tid; gst(g + k, s_out[k]); }
  const uint32_t nv = (uint32_t)((b_down - a_up) >> 4);
  constexpr int kOutV = (kStageBytes + kBlock * 16 - 1) / (kBlock * 16);
  uint4 v[kOutV];
#pragma unroll
  for (int k = 0; k < kOutV; k++) { const uint32_t c = tid + (uint32_t)k * kBlock;
    if (c < nv) { const lds_u128* blk = (const lds_u128*)(lds_u8*)s_out + c; v[k] = bytes_at(blk[0], blk[1], head); } }
  uint4* dstv = (uint4*)a_up;
#pragma unroll
  for (int k = 0; k < kOutV; k++) { const uint32_t c = tid + (uint32_t)k * kBlock; if (c < nv) gst4(dstv + c, v[k]); }
}

// ---- (A) one tile per workgroup, register staging ----
template <bool LB, bool BUILD, int LBW = 1, int SLEEP = 1, int EARLYPUB = 0>
__global__ __launch_bounds__(kBlock) void kA(Args a) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kTileBytes + 48];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kStageBytes + 32];
  __shared__ uint64_t s_red[6];
  const uint32_t tid = threadIdx.x, wave = tid >> 6, tile = blockIdx.x;
  const uint64_t tstart = __builtin_amdgcn_s_memrealtime();
  const uint64_t first = (uint64_t)tile * kBlock, last = min(first + kBlock, a.n), i = first + tid;
  const uint64_t lo = gld(a.off + first), hi = gld(a.off + last);
  uint64_t so = 0, sn = 0;
  if (i < a.n) { so = gld(a.off + i); sn = gld(a.off + i + 1) - so; }
  uint64_t early0 = 0;
  if (EARLYPUB && wave == 0) {  // the aggregate is known from the offsets alone (verbatim copy)
    if (lane_id() == 0) publish(a.state, tile, (tile == 0 && LBW != 2 ? kFlagIncl : kFlagAgg) | (hi - lo));
    if (EARLYPUB == 2 && tile) early0 = lb_poll(a.state, (int64_t)tile - 1);
  }
  const uintptr_t plo = (uintptr_t)(a.in + lo); const uint32_t shift = plo & 15;
  const uint4* src = (const uint4*)(plo - shift);
  const uint32_t nv = (uint32_t)((shift + (hi - lo) + 15) >> 4);
  constexpr int MAXV = (kTileBytes + 31) / 16 / kBlock + 1;
  uint4 v[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; k++) { const uint32_t j = tid + k * kBlock; if (j < nv) v[k] = gld4(src + j); }
#pragma unroll
  for (int k = 0; k < MAXV; k++) { const uint32_t j = tid + k * kBlock; if (j < nv) ((uint4*)s_in)[j] = v[k]; }
  __syncthreads();
  uint64_t tot; const uint64_t local = block_scan<false>(sn, s_red, &tot);
  uint64_t early = 0;
  if (LB && wave == 0) {
    if (!EARLYPUB && lane_id() == 0) publish(a.state, tile, (tile == 0 && LBW != 2 ? kFlagIncl : kFlagAgg) | tot);
    if (tile && LBW != 2) early = EARLYPUB == 2 ? early0 : lb_poll(a.state, (int64_t)tile - 1);
  }
  if (BUILD && __any(sn != 0)) lds_copy((lds_u8*)s_out + local, (const lds_u8*)s_in + shift + (so - lo), (uint32_t)sn);
  const uint64_t tlb0 = __builtin_amdgcn_s_memrealtime();
  if (LB && wave == 0) { const uint64_t b = LBW == 2 ? look_back2<SLEEP>(a.state, a.sstate, tile, (uint32_t)((a.n + kBlock - 1) / kBlock), tot, a.err) : LBW == 4 ? look_back4<SLEEP>(a.state, tile, tot, a.err) : LBW > 4 ? look_back_rows<(LBW >= 64 ? LBW / 64 : 1), SLEEP>(a.state, tile, tot, a.err, early) : look_back(a.state, tile, tot, a.err, early); if (tid == 0) s_red[4] = b; }
  if (!LB && tid == 0) s_red[4] = lo;
  __syncthreads();
  const uint64_t base = s_red[4];
  if (a.stamps && tid == 0) { const uint64_t t1 = __builtin_amdgcn_s_memrealtime(); a.stamps[4 * tile] = tstart; a.stamps[4 * tile + 1] = tlb0; a.stamps[4 * tile + 2] = t1; }
  if (i < a.n) { gst(a.ooff + i, base + local); gst(a.st + i, (uint8_t)0); }
  if (last == a.n && tid == 0) a.ooff[a.n] = base + tot;
  if (BUILD) stream_out(a.out + base, s_out, (uint32_t)tot, tid);
  else stream_out(a.out + base, s_in + shift, (uint32_t)tot, tid);
  if (a.stamps && tid == 0) a.stamps[4 * tile + 3] = __builtin_amdgcn_s_memrealtime();
}

// ---- (C) plain streaming copy (the hardware floor for these bytes) ----
__global__ __launch_bounds__(kBlock) void kC(const uint4* in, uint4* out, uint64_t nv, const uint64_t* off, uint64_t* ooff, uint8_t* st, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < nv; j += stride) gst4(out + j, gld4(in + j));
  for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < n; j += stride) { gst(ooff + j, gld(off + j)); gst(st + j, (uint8_t)0); }
}

// ---- (B) persistent workgroups, LDS-DMA prefetch of the next tile ----
__global__ __launch_bounds__(kBlock) void kB(Args a, uint32_t ntiles) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[2][kTileBytes + 48];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kStageBytes + 32];
  __shared__ uint32_t s_off[2][kBlock + 1];
  __shared__ uint64_t s_red[6];
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = lane_id(), G = gridDim.x;
  uint32_t tile = blockIdx.x;
  if (tile >= ntiles) return;
  auto geo = [&](uint32_t t, uint64_t& lo, uint64_t& hi) {
    const uint64_t f = (uint64_t)t * kBlock, l = min(f + kBlock, a.n);
    lo = gld(a.off + f); hi = gld(a.off + l);
  };
  auto dma = [&](uint32_t b, uint64_t lo, uint64_t hi) {
    const uintptr_t plo = (uintptr_t)(a.in + lo); const uint32_t shift = plo & 15;
    const uint8_t* src = (const uint8_t*)(plo - shift);
    const uint32_t nv = (uint32_t)((shift + (hi - lo) + 15) >> 4);
    for (uint32_t c0 = wave * 64; c0 < nv; c0 += kBlock) {
      const uint32_t c = c0 + lane;
      if (c < nv)
        __builtin_amdgcn_global_load_lds((const void*)(src + 16 * c), (__attribute__((address_space(3))) void*)(s_in[b] + 16 * c0), 16, 0, 0);
    }
  };
  // prologue: tile's offsets and bytes, next tile's geometry
  uint64_t lo, hi, lo_n = 0, hi_n = 0;
  geo(tile, lo, hi);
  {
    const uint64_t f = (uint64_t)tile * kBlock, i = f + tid;
    s_off[0][tid] = (uint32_t)(gld(a.off + min(i, a.n)) - lo);
    if (tid == 0) s_off[0][kBlock] = (uint32_t)(hi - lo);
  }
  dma(0, lo, hi);
  if (tile + G < ntiles) geo(tile + G, lo_n, hi_n);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (uint32_t it = 0; tile < ntiles; it++, tile += G) {
    const uint32_t b = it & 1;
    raw_barrier();  // s_in[b], s_off[b] ready; s_in[b^1], s_out free
    const uint32_t nxt = tile + G;
    uint64_t offn = 0, lo_nn = 0, hi_nn = 0;
    if (nxt < ntiles) {
      dma(b ^ 1, lo_n, hi_n);
      offn = gld(a.off + min((uint64_t)nxt * kBlock + tid, a.n));
      if (nxt + G < ntiles) geo(nxt + G, lo_nn, hi_nn);
    }
    const uint64_t first = (uint64_t)tile * kBlock, last = min(first + kBlock, a.n), i = first + tid;
    const uint32_t shift = (uint32_t)((uintptr_t)(a.in + lo) & 15);
    const uint32_t so = s_off[b][tid], sn = i < a.n ? s_off[b][tid + 1] - so : 0u;
    uint64_t tot; const uint64_t local = block_scan<true>(sn, s_red, &tot);
    uint64_t early = 0;
    if (wave == 0) { if (lane == 0) publish(a.state, tile, (tile == 0 ? kFlagIncl : kFlagAgg) | tot); if (tile) early = lb_poll(a.state, (int64_t)tile - 1); }
    if (__any(sn != 0)) lds_copy((lds_u8*)s_out + local, (const lds_u8*)s_in[b] + shift + so, sn);
    if (wave == 0) { const uint64_t bb = look_back(a.state, tile, tot, a.err, early); if (tid == 0) s_red[4] = bb; }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA and prefetch loads have landed
    raw_barrier();
    const uint64_t base = s_red[4];
    if (nxt < ntiles) {  // the next tile's offsets, relative to its first byte
      s_off[b ^ 1][tid] = (uint32_t)(offn - lo_n);
      if (tid == 0) s_off[b ^ 1][kBlock] = (uint32_t)(hi_n - lo_n);
    }
    if (i < a.n) { gst(a.ooff + i, base + local); gst(a.st + i, (uint8_t)0); }
    if (last == a.n && tid == 0) a.ooff[a.n] = base + tot;
    stream_out(a.out + base, s_out, (uint32_t)tot, tid);
    lo = lo_n; hi = hi_n; lo_n = lo_nn; hi_n = hi_nn;
  }
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 10000000ull;
  const int reps = 20;
  std::vector<uint64_t> off(n + 1);
  uint64_t s = 0x1234567, tot = 0;
  for (uint64_t i = 0; i < n; i++) { s = s * 6364136223846793005ull + 1442695040888963407ull; off[i] = tot; tot += 48 + (s >> 33) % 33; }
  off[n] = tot;
  std::vector<uint8_t> in(tot + 64);
  for (uint64_t k = 0; k < tot; k++) { s = s * 6364136223846793005ull + 1442695040888963407ull; in[k] = 'a' + (s >> 40) % 26; }
  Args a{};
  uint8_t *din, *dout, *dst; uint64_t *doff, *dooff, *dstate; uint32_t* derr;
  const uint64_t ntiles = (n + kBlock - 1) / kBlock;
  CHECK(hipMalloc(&din, tot + 64)); CHECK(hipMalloc(&dout, tot + 64)); CHECK(hipMalloc(&dst, n + 16));
  CHECK(hipMalloc(&doff, (n + 1) * 8)); CHECK(hipMalloc(&dooff, (n + 1) * 8)); CHECK(hipMalloc(&dstate, ntiles * 8)); uint64_t* dsstate; CHECK(hipMalloc(&dsstate, (ntiles / kSuper + 2) * 8)); CHECK(hipMalloc(&derr, 4));
  CHECK(hipMemcpy(din, in.data(), tot, hipMemcpyHostToDevice)); CHECK(hipMemcpy(doff, off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
  CHECK(hipMemset(derr, 0, 4));
  uint64_t* dstamps; CHECK(hipMalloc(&dstamps, ntiles * 32));
  a = Args{din, doff, n, dout, dooff, dst, dstate, derr, nullptr, dsstate};
  int dev = 0, cus = 0; CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  int occB = 0; CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occB, kB, kBlock, 0));
  int occA = 0; CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occA, kA<true, true>, kBlock, 0));
  printf("n=%llu bytes=%llu tiles=%llu cus=%d occA=%d occB=%d\n", (unsigned long long)n, (unsigned long long)tot, (unsigned long long)ntiles, cus, occA, occB);
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  std::vector<uint8_t> out(tot);
  std::vector<uint64_t> oo(n + 1);
  auto run = [&](const char* name, auto launch) {
    float sum = 0, best = 1e9;
    for (int r = 0; r < reps + 2; r++) {
      CHECK(hipMemsetAsync(dstate, 0, ntiles * 8)); CHECK(hipMemsetAsync(dsstate, 0, (ntiles / kSuper + 2) * 8)); CHECK(hipMemsetAsync(dout, 0, 64));
      CHECK(hipEventRecord(e0)); launch(); CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) { best = ms < best ? ms : best; sum += ms; }
    }
    uint32_t err = 0; CHECK(hipMemcpy(&err, derr, 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(out.data(), dout, tot, hipMemcpyDeviceToHost)); CHECK(hipMemcpy(oo.data(), dooff, (n + 1) * 8, hipMemcpyDeviceToHost));
    const bool ok = !err && memcmp(out.data(), in.data(), tot) == 0 && memcmp(oo.data(), off.data(), n * 8) == 0;
    const double bytes = 2.0 * tot + 17.0 * n;
    printf("%-28s mean %.4f ms  best %.4f ms  %.0f GB/s  ok=%d err=%u\n", name, sum / reps, best, bytes / (sum / reps * 1e-3) / 1e9, (int)ok, err);
    CHECK(hipMemset(derr, 0, 4));
  };
  const uint32_t gA = (uint32_t)ntiles;
  auto stamped = [&](const char* name, auto launch) {
    a.stamps = dstamps; uint32_t z = 0; CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_polls), &z, 4));
    CHECK(hipMemsetAsync(dstate, 0, ntiles * 8)); CHECK(hipMemsetAsync(dsstate, 0, (ntiles / kSuper + 2) * 8)); launch(); CHECK(hipDeviceSynchronize());
    std::vector<uint64_t> h(ntiles * 4); CHECK(hipMemcpy(h.data(), dstamps, ntiles * 32, hipMemcpyDeviceToHost));
    uint32_t polls; CHECK(hipMemcpyFromSymbol(&polls, HIP_SYMBOL(g_polls), 4));
    double pre = 0, lb = 0, post = 0; uint64_t t0 = ~0ull, t1 = 0;
    for (uint64_t t = 0; t < ntiles; t++) { pre += h[4*t+1] - h[4*t]; lb += h[4*t+2] - h[4*t+1]; post += h[4*t+3] - h[4*t+2]; t0 = std::min(t0, h[4*t]); t1 = std::max(t1, h[4*t+3]); }
    printf("  stamps %-24s per tile (us): pre-lookback %.2f  lookback+barrier %.2f  stream-out %.2f  life %.2f | span %.3f ms  gap polls %.2f/tile\n", name,
           pre / ntiles / 100, lb / ntiles / 100, post / ntiles / 100, (pre + lb + post) / ntiles / 100, (t1 - t0) / 1e5, (double)polls / ntiles);
    a.stamps = nullptr;
  };
  stamped("lookback+build", [&] { hipLaunchKernelGGL((kA<true, true>), dim3(gA), dim3(kBlock), 0, 0, a); });
  stamped("early publish, poll late", [&] { hipLaunchKernelGGL((kA<true, true, 1, 1, 1>), dim3(gA), dim3(kBlock), 0, 0, a); });
  stamped("no lookback", [&] { hipLaunchKernelGGL((kA<false, true>), dim3(gA), dim3(kBlock), 0, 0, a); });
  stamped("2level+build", [&] { hipLaunchKernelGGL((kA<true, true, 2, 32>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A 2level nap32 +build", [&] { hipLaunchKernelGGL((kA<true, true, 2, 32>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A 2level nap4 +build", [&] { hipLaunchKernelGGL((kA<true, true, 2, 4>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A 2level nap1 +build", [&] { hipLaunchKernelGGL((kA<true, true, 2, 1>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A 2level early publish", [&] { hipLaunchKernelGGL((kA<true, true, 2, 4, 1>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A lookback+build", [&] { hipLaunchKernelGGL((kA<true, true>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A early publish, poll late", [&] { hipLaunchKernelGGL((kA<true, true, 1, 1, 1>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A early publish+poll", [&] { hipLaunchKernelGGL((kA<true, true, 1, 1, 2>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A rows1 nap32", [&] { hipLaunchKernelGGL((kA<true, true, 64, 32>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A rows2 nap32", [&] { hipLaunchKernelGGL((kA<true, true, 128, 32>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A rows4 nap32", [&] { hipLaunchKernelGGL((kA<true, true, 256, 32>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A rows4 nap4", [&] { hipLaunchKernelGGL((kA<true, true, 256, 4>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A rows8 nap4", [&] { hipLaunchKernelGGL((kA<true, true, 512, 4>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A rows4 nap4 earlypub", [&] { hipLaunchKernelGGL((kA<true, true, 256, 4, 1>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A lookback4 s1 +build", [&] { hipLaunchKernelGGL((kA<true, true, 4, 1>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A lookback4 s0 +build", [&] { hipLaunchKernelGGL((kA<true, true, 4, 0>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A lookback4 s4 +build", [&] { hipLaunchKernelGGL((kA<true, true, 4, 4>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A lookback, no build", [&] { hipLaunchKernelGGL((kA<true, false>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A no lookback, build", [&] { hipLaunchKernelGGL((kA<false, true>), dim3(gA), dim3(kBlock), 0, 0, a); });
  run("A no lookback, no build", [&] { hipLaunchKernelGGL((kA<false, false>), dim3(gA), dim3(kBlock), 0, 0, a); });
  for (int gm = 1; gm <= occB; gm++)
    run(gm == 1 ? "B persistent x1/CU" : "B persistent x2/CU", [&] { hipLaunchKernelGGL(kB, dim3(cus * gm), dim3(kBlock), 0, 0, a, (uint32_t)ntiles); });
  for (int gm : {4, 8, 16}) {
    char nm[64]; snprintf(nm, sizeof nm, "C copy grid %d/CU", gm);
    run(nm, [&] { hipLaunchKernelGGL(kC, dim3(cus * gm), dim3(kBlock), 0, 0, (const uint4*)din, (uint4*)dout, (tot + 15) / 16, doff, dooff, dst, n); });
  }
  return 0;
}
