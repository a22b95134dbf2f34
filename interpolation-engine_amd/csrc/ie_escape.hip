// ie_escape.hip — recursive_unescape / recursive_escape on strings (py:1436-1460 /
// rust-project/src/interp.rs:147-177) as a byte map with length change, plus the synthetic
// workload generator and a generic exclusive scan.
//
// Escape pipeline, one 256-lane workgroup per tile of 256 strings staged in LDS:
//   k_measure<OP>  output length per string, tile sums
//   k_scan_tiles   exclusive scan of tile sums -> tile bases, grand total
//   k_emit<OP>     re-stage, workgroup scan, write into an LDS stage aligned like the
//                  destination, stream out with 16-byte stores
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ie_device.h"
#include "ie_kernels.h"

namespace ie {

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

// The same map on one string by the whole wave (arguments uniform; generic pointers: LDS or
// global): 64 bytes per step, each lane decides its byte and places it by a ballot prefix count.
// Unescape drops position p iff s[p] == '\\' and s[p + 1] is a brace (a pair's second byte is a
// brace, never a '\\', so the decisions are independent); escape puts a '\\' before each brace.
template <int OP>
__device__ void wave_escape(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint32_t n) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t lower = (1ull << lane) - 1ull;
  uint32_t w = 0;
  for (uint32_t p0 = 0; p0 < n; p0 += 64) {
    const uint32_t p = p0 + lane;
    const bool in = p < n;
    const uint8_t c = in ? src[p] : 0;
    if (OP == kOpUnescape) {
      const uint8_t nx = p + 1 < n ? src[p + 1] : 0;
      const bool keep = in && !(c == '\\' && (nx == '{' || nx == '}'));
      const uint64_t km = __ballot(keep);
      if (keep) dst[w + (uint32_t)__popcll(km & lower)] = c;
      w += (uint32_t)__popcll(km);
    } else {
      const bool br = in && (c == '{' || c == '}');
      const uint64_t bm = __ballot(br);
      uint32_t pos = w + lane + (uint32_t)__popcll(bm & lower);
      if (br) dst[pos++] = '\\';
      if (in) dst[pos] = c;
      w += (n - p0 < 64u ? n - p0 : 64u) + (uint32_t)__popcll(bm);
    }
  }
}

// Output length of one string staged in LDS, a dword at a time: unescape drops one byte per '\'
// followed by a brace (such pairs never overlap: the second byte of one is never a '\'), escape
// adds one per brace. Same result as eval_escape's byte loop (measure mode).
__device__ __forceinline__ uint32_t nib4(uint32_t v) {  // bit k: byte k of v has its top bit
  return ((v & 0x80808080u) * 0x00204081u) >> 28;
}
template <int OP>
__device__ uint32_t escape_len_lds(const uint8_t* s, uint32_t n) {
  const uintptr_t p = (uintptr_t)s;
  const uint32_t* w = (const uint32_t*)(p & ~(uintptr_t)3);
  const uint32_t off = (uint32_t)(p & 3), end = off + n;
  uint32_t cnt = 0, carry = 0;  // carry: a valid '\' in the previous dword's top byte
  for (uint32_t j = 0; 4 * j < end; j++) {
    const uint32_t x = w[j], x7 = x & 0x7F7F7F7Fu;
    const uint32_t bs = nib4(~(((x7 ^ 0x5C5C5C5Cu) + 0x7F7F7F7Fu) | x));
    const uint32_t br = nib4(~(((x7 ^ 0x7B7B7B7Bu) + 0x7F7F7F7Fu) | x)) | nib4(~(((x7 ^ 0x7D7D7D7Du) + 0x7F7F7F7Fu) | x));
    const uint32_t lo = 4 * j < off ? off - 4 * j : 0u, hi = end - 4 * j < 4u ? end - 4 * j : 4u;
    const uint32_t valid = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
    if (OP == kOpUnescape) {
      const uint32_t b = bs & valid, r = br & valid;
      cnt += (uint32_t)__popc(b & (r >> 1)) + (carry & r & 1u);
      carry = b >> 3;
    } else {
      cnt += (uint32_t)__popc(br & valid);
    }
  }
  return OP == kOpUnescape ? n - cnt : n + cnt;
}

// LDS views (ds_* accesses) and an LDS -> LDS copy at any alignments with aligned accesses only
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// 16 bytes at any LDS address: five aligned dword reads and v_alignbyte (reads up to 19 bytes
// past p)
__device__ __forceinline__ u32x4 esc_ld16a(const lds_u8* p) {
  const uint32_t sh = (uint32_t)(uintptr_t)p & 3u;
  const lds_u32* q = (const lds_u32*)(p - sh);
  const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
  return u32x4{__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
               __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
}

// len bytes LDS -> LDS: head bytes until dst is 4-aligned, 16-byte units as aligned dwords, then
// the tail as dwords, a short and a byte. Wave-uniform call (lanes with len 0 copy nothing).
__device__ __forceinline__ void lds_copy_any(lds_u8* dst, const lds_u8* src, uint32_t len) {
  const uint32_t h0 = (0u - (uint32_t)(uintptr_t)dst) & 3u, h = h0 < len ? h0 : len;
  if (h > 0) dst[0] = src[0];
  if (h > 1) dst[1] = src[1];
  if (h > 2) dst[2] = src[2];
  const uint32_t body = (len - h) & ~15u;
  for (uint32_t k = 0; __any(k < body); k += 16u) {
    if (k < body) {
      const u32x4 v = esc_ld16a(src + h + k);
      lds_u32* q = (lds_u32*)(dst + h + k);
      q[0] = v.x, q[1] = v.y, q[2] = v.z, q[3] = v.w;
    }
  }
  const uint32_t kt = h + body;
  if (kt < len) {
    const u32x4 v = esc_ld16a(src + kt);
    const uint32_t n = len - kt;
    lds_u32* q = (lds_u32*)(dst + kt);
    if (n >= 4) q[0] = v.x;
    if (n >= 8) q[1] = v.y;
    if (n >= 12) q[2] = v.z;
    const uint32_t nw = n >> 2, r = n & 3u;
    const uint32_t x = nw == 0 ? v.x : nw == 1 ? v.y : nw == 2 ? v.z : v.w;
    lds_u8* b = dst + kt + (n & ~3u);
    if (r & 2u) *(lds_u16*)b = (uint16_t)x;
    if (r & 1u) b[r & 2u] = (uint8_t)(x >> (8u * (r & 2u)));
  }
}

// ------------------------------------------------------------------------------------------
// workgroup helpers
// ------------------------------------------------------------------------------------------
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

// Stage bytes [lo, hi) of the batch (hi - lo <= kTileBytes) into LDS so that LDS position p holds
// byte (lo16 + p) where lo16 = lo rounded down to 16 B: whole aligned 16-byte chunks (one never
// crosses a page; the bytes around [lo, hi) it carries are ignored), every load of the thread in
// flight before the first LDS write, with the non-temporal policy (read once). Returns the LDS
// offset of byte `lo`.
__device__ uint32_t stage_tile(const uint8_t* __restrict__ bytes, uint64_t lo, uint64_t hi, uint8_t* lds) {
  const uintptr_t plo = (uintptr_t)(bytes + lo);
  const uint32_t shift = (uint32_t)(plo & 15);
  const uint32_t nv = (uint32_t)((shift + (hi - lo) + 15) >> 4);
  constexpr int MAXV = (kTileBytes + 30) / 16 / kBlock + 1;
  const uint4* src = (const uint4*)(plo - shift);
  uint4 v[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; k++) {
    const uint32_t j = threadIdx.x + (uint32_t)k * kBlock;
    if (j < nv) v[k] = gld4s(src + j);
  }
#pragma unroll
  for (int k = 0; k < MAXV; k++) {
    const uint32_t j = threadIdx.x + (uint32_t)k * kBlock;
    if (j < nv) ((uint4*)lds)[j] = v[k];
  }
  return shift;
}

// ------------------------------------------------------------------------------------------
// Sub-batches: a tile's strings go through the LDS stage in runs [start, end) whose bytes fit it
// (a tile of resolve outputs averages 17.4 KB in config 4, so one tile in seven needs two runs);
// a single string longer than the stage is handled from global memory by its own lane.
// ------------------------------------------------------------------------------------------
struct SubBatch {
  uint64_t start, end, lo, hi;  // strings [start, end), bytes [lo, hi)
  bool staged;
};
// the run that starts at string `start` of the tile [.., last); every lane calls it (barrier)
__device__ __forceinline__ SubBatch next_run(const Batch& B, uint64_t start, uint64_t last, uint64_t i, uint64_t eo) {
  SubBatch r;
  r.start = start;
  r.lo = B.in_off[start];
  const bool fits = i >= start && i < last && eo - r.lo <= (uint64_t)kTileBytes;
  const uint64_t cnt = (uint64_t)__syncthreads_count(fits);  // fits is monotone in i
  r.staged = cnt > 0;
  r.end = start + (cnt > 0 ? cnt : 1);
  r.hi = B.in_off[r.end];
  return r;
}

// ------------------------------------------------------------------------------------------
// k_measure
// ------------------------------------------------------------------------------------------
template <int OP>
__global__ __launch_bounds__(kBlock) void k_measure(Batch B, Work W) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kTileBytes + 64];
  __shared__ uint64_t s_red[kBlock / 64];

  const uint64_t tile = blockIdx.x;
  const uint64_t first = tile * kBlock;
  const uint64_t i = first + threadIdx.x;
  const uint64_t last = min(first + kBlock, B.n);  // exclusive
  const uint64_t so = i < B.n ? B.in_off[i] : 0, eo = i < B.n ? B.in_off[i + 1] : 0;
  uint32_t olen = 0;
  for (uint64_t start = first; start < last;) {  // uniform
    const SubBatch r = next_run(B, start, last, i, eo);
    const bool mine = i >= r.start && i < r.end;
    if (r.staged) {
      const uint32_t shift = stage_tile(B.bytes, r.lo, r.hi, s_in);
      __syncthreads();
      if (mine) olen = escape_len_lds<OP>(s_in + shift + (so - r.lo), (uint32_t)(eo - so));
    } else if (mine) {
      eval_escape<OP>(B.bytes + so, (uint32_t)(eo - so), nullptr, olen, false);
    }
    __syncthreads();  // the stage is free for the next run
    start = r.end;
  }
  if (i < B.n) {
    W.out_len[i] = olen;
    gsts(B.status + i, (uint8_t)IE_OK_STR);
  }
  uint64_t total;
  block_excl_scan(olen, s_red, &total);
  if (threadIdx.x == 0) W.tile_sum[tile] = total;
}

// ------------------------------------------------------------------------------------------
// k_scan_tiles: one 1024-lane workgroup, exclusive scan of the tile sums (a contiguous chunk per
// lane, its loads in flight together), grand total.
// ------------------------------------------------------------------------------------------
constexpr int kScanLanes = 1024;
__global__ __launch_bounds__(kScanLanes) void k_scan_tiles(Work W, uint64_t n_tiles, uint64_t* total,
                                                           uint64_t* offsets_n) {
  __shared__ uint64_t s_w[kScanLanes / 64];
  const uint32_t t = threadIdx.x, lane = t & 63u, wid = t >> 6;
  const uint64_t per = (n_tiles + kScanLanes - 1) / kScanLanes;
  const uint64_t b = min((uint64_t)t * per, n_tiles), e = min(b + per, n_tiles);
  uint64_t sum = 0;
#pragma unroll 8
  for (uint64_t k = b; k < e; k++) sum += W.tile_sum[k];
  const uint64_t inc = wave_incl_scan(sum);
  if (lane == 63) s_w[wid] = inc;
  __syncthreads();
  uint64_t run = 0, tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < kScanLanes / 64; w++) {
    const uint64_t x = s_w[w];
    if (w < wid) run += x;
    tot += x;
  }
  run += inc - sum;
#pragma unroll 8
  for (uint64_t k = b; k < e; k++) {
    const uint64_t v = W.tile_sum[k];
    W.tile_base[k] = run;
    run += v;
  }
  if (t == 0) {
    *total = tot;
    *offsets_n = tot;
  }
}

// ------------------------------------------------------------------------------------------
// k_emit
// ------------------------------------------------------------------------------------------
// the LDS stage [0, len) -> g (any alignment; stage position p holds output byte p - oshift is
// NOT assumed: the stage is laid out tile-relative and realigned here), 16-byte aligned stores
__device__ __forceinline__ void stream_out(uint8_t* g, const uint8_t* stage, uint32_t oshift, uint32_t len) {
  const uintptr_t pg = (uintptr_t)g, pe = pg + len;
  const uintptr_t a_up = (pg + 15) & ~(uintptr_t)15, b_down = pe & ~(uintptr_t)15;
  if (a_up >= b_down) {
    for (uint32_t k = threadIdx.x; k < len; k += kBlock) g[k] = stage[oshift + k];
    return;
  }
  const uint32_t head = (uint32_t)(a_up - pg), tail = (uint32_t)(pe - b_down);
  if (threadIdx.x < head) g[threadIdx.x] = stage[oshift + threadIdx.x];
  if (threadIdx.x < tail) {
    const uint32_t k = (uint32_t)(b_down - pg) + threadIdx.x;
    g[k] = stage[oshift + k];
  }
  const uint32_t nv = (uint32_t)((b_down - a_up) >> 4);
  const uint4* src = (const uint4*)(stage + oshift + head);  // 16-aligned: oshift = pg & 15
  uint4* dstv = (uint4*)a_up;
  for (uint32_t j = threadIdx.x; j < nv; j += kBlock) gst4s(dstv + j, src[j]);
}

template <int OP>
__global__ __launch_bounds__(kBlock) void k_emit(Batch B, Work W, uint8_t* out_bytes, uint64_t out_cap,
                                                 const uint64_t* total) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kTileBytes + 64];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kStageBytes + 32];
  __shared__ uint64_t s_red[kBlock / 64];
  __shared__ uint32_t s_loc[kBlock + 1];  // tile-relative output offsets

  const uint64_t tile = blockIdx.x;
  const uint64_t first = tile * kBlock;
  const uint64_t i = first + threadIdx.x;
  const uint64_t last = min(first + kBlock, B.n);
  const uint64_t base = W.tile_base[tile];
  const bool write_bytes = *total <= out_cap;

  const uint32_t my_len = (i < B.n) ? W.out_len[i] : 0;
  uint64_t tile_out;
  const uint64_t local = block_excl_scan(my_len, s_red, &tile_out);
  // over capacity inside a multi-step command: offsets all 0 (empty strings), so that the next
  // step reads nothing past the caller's buffer; the error is reported at the exec's sync
  const bool zero = !write_bytes && W.zero_on_overflow;
  if (i < B.n) gsts(B.out_off + i, zero ? (uint64_t)0 : base + local);
  if (zero && i + 1 == B.n) gsts(B.out_off + B.n, (uint64_t)0);
  if (!write_bytes) return;  // uniform across the workgroup
  s_loc[threadIdx.x] = (uint32_t)local;
  if (threadIdx.x == 0) s_loc[kBlock] = (uint32_t)tile_out;
  const uint64_t so = i < B.n ? B.in_off[i] : 0, eo = i < B.n ? B.in_off[i + 1] : 0, n = eo - so;

  for (uint64_t start = first; start < last;) {  // uniform (next_run's barrier publishes s_loc)
    const SubBatch r = next_run(B, start, last, i, eo);
    const bool mine = i >= r.start && i < r.end && my_len;
    const uint32_t o_lo = s_loc[r.start - first], o_hi = s_loc[r.end - first];
    const uint64_t gb = base + o_lo;  // the run's first output byte
    const uint32_t oshift = (uint32_t)(((uintptr_t)(out_bytes + gb)) & 15);
    const bool staged_out = r.staged && o_hi - o_lo + oshift <= (uint32_t)kStageBytes;
    uint32_t shift = 0;
    if (r.staged) shift = stage_tile(B.bytes, r.lo, r.hi, s_in);
    __syncthreads();
    // a string the map leaves as it is (most of them): aligned LDS moves instead of the byte loop
    const bool same = staged_out && mine && my_len == n;
    if (__any(same))
      lds_copy_any((lds_u8*)(s_out + oshift + (same ? (uint32_t)local - o_lo : 0)),
                   (const lds_u8*)(s_in + shift + (same ? so - r.lo : 0)), same ? my_len : 0u);
    // the others (a brace pair to drop or a brace to escape) one at a time by the whole wave
    const bool slow = mine && !same;
    uint8_t* const dst = staged_out ? s_out + oshift + ((uint32_t)local - o_lo) : out_bytes + base + local;
    const uint8_t* const src = r.staged ? s_in + shift + (so - r.lo) : B.bytes + so;
    for (uint64_t m = __ballot(slow); m; m &= m - 1) {
      const int l = __builtin_ctzll(m);
      const uint64_t d64 = (uint64_t)(uintptr_t)dst, s64 = (uint64_t)(uintptr_t)src;
      uint8_t* const d = (uint8_t*)(uintptr_t)(((uint64_t)__shfl((uint32_t)(d64 >> 32), l, 64) << 32) |
                                                __shfl((uint32_t)d64, l, 64));
      const uint8_t* const q = (const uint8_t*)(uintptr_t)(((uint64_t)__shfl((uint32_t)(s64 >> 32), l, 64) << 32) |
                                                           __shfl((uint32_t)s64, l, 64));
      wave_escape<OP>(d, q, (uint32_t)__shfl((uint32_t)n, l, 64));
    }
    __syncthreads();
    if (staged_out) stream_out(out_bytes + gb, s_out, oshift, o_hi - o_lo);
    __syncthreads();  // the stages are free for the next run
    start = r.end;
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

// A step of a multi-step batch that failed earlier stays failed: strings whose earlier status
// is not IE_OK_STR take that status (their bytes are empty: a failed string has no output)
__global__ void k_status_carry(const uint8_t* before, uint8_t* after, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t b = before[i];
    if (b != IE_OK_STR) after[i] = b;
  }
}

// device-side capacity check between two steps: flags the exec's error word (reported at sync)
__global__ void k_cap_check(const uint64_t* total, uint64_t cap, uint32_t* err) {
  if (threadIdx.x == 0 && *total > cap) atomicOr(err, 2u);
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
hipError_t launch_cap_check(const uint64_t* total, uint64_t cap, uint32_t* err, hipStream_t st) {
  hipLaunchKernelGGL(k_cap_check, dim3(1), dim3(64), 0, st, total, cap, err);
  return hipGetLastError();
}

hipError_t launch_status_carry(const uint8_t* before, uint8_t* after, uint64_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  const uint64_t g0 = (n + 255) / 256;
  hipLaunchKernelGGL(k_status_carry, dim3((uint32_t)(g0 < 8192 ? g0 : 8192)), dim3(256), 0, st, before, after, n);
  return hipGetLastError();
}

hipError_t launch_escape(int op, const Batch& B, const Work& W, uint8_t* out, uint64_t cap, hipStream_t st) {
  const uint64_t tiles = (B.n + kBlock - 1) / kBlock;
  if (!tiles) return hipSuccess;
  if (op == kOpUnescape) hipLaunchKernelGGL(k_measure<kOpUnescape>, dim3((uint32_t)tiles), dim3(kBlock), 0, st, B, W);
  else hipLaunchKernelGGL(k_measure<kOpEscape>, dim3((uint32_t)tiles), dim3(kBlock), 0, st, B, W);
  hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kScanLanes), 0, st, W, tiles, W.total, B.out_off + B.n);
  if (op == kOpUnescape) hipLaunchKernelGGL(k_emit<kOpUnescape>, dim3((uint32_t)tiles), dim3(kBlock), 0, st, B, W, out, cap, W.total);
  else hipLaunchKernelGGL(k_emit<kOpEscape>, dim3((uint32_t)tiles), dim3(kBlock), 0, st, B, W, out, cap, W.total);
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
