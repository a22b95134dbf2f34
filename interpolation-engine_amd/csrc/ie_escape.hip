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
__global__ __launch_bounds__(kBlock) void k_measure(Batch B, Work W) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kTileBytes + 32];
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
    uint32_t olen = 0;
    uint8_t st = IE_OK_STR;
    if (staged) olen = escape_len_lds<OP>(s, (uint32_t)(eo - so));
    else st = eval_escape<OP>(s, (uint32_t)(eo - so), nullptr, olen, false);
    W.out_len[i] = olen;
    my_len = olen;
    B.status[i] = st;
  }
  uint64_t total;
  block_excl_scan(my_len, s_red, &total);
  if (threadIdx.x == 0) W.tile_sum[tile] = total;
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
__global__ __launch_bounds__(kBlock) void k_emit(Batch B, Work W, uint8_t* out_bytes, uint64_t out_cap,
                                                 const uint64_t* total) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kTileBytes + 32];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kStageBytes + 32];
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
  if (i < B.n) B.out_off[i] = base + local;
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
    const uint64_t so = B.in_off[i], n = B.in_off[i + 1] - so;
    const uint8_t* s = staged_in ? s_in + shift + (so - lo) : B.bytes + so;
    uint32_t olen = 0;
    eval_escape<OP>(s, (uint32_t)n, dst, olen, true);
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
  hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kBlock), 0, st, W, tiles, W.total, B.out_off + B.n);
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
