// Microbenchmark (diagnostic, not product): LDS access forms the k_resolve build and key assembly
// could use, on gfx950. Each 256-lane workgroup keeps 16 KB of LDS; every lane moves 16 bytes per
// iteration from a byte-granular source offset to a byte-granular destination offset.
//   mode 0: 5 aligned ds_read_b32 + 4 v_alignbyte, 4 aligned ds_write_b32 (dst 4-aligned)  [ld16a]
//   mode 1: 4 ds_read_b32 at the unaligned source, 4 aligned ds_write_b32
//   mode 2: 4 ds_read_b32 unaligned source, 4 ds_write_b32 at an unaligned destination
//   mode 3: 1 ds_read_b128 unaligned source, 1 ds_write_b128 aligned dst
//   mode 4: integer mix: v_mul_lo_u32 chain (hash_word-like), 8 per iteration
//   mode 5: the same work with v_mul_u32_u24
//   modes 6 / 7 / 8: throughput of 32 independent v_mul_lo_u32 / v_mul_u32_u24 / (xor + add) per iteration
// Prints cycles per iteration per wave (median over workgroups) and checks the copies.
// Build: hipcc --offload-arch=gfx950 -O3 tools/exp/lds_ubench.hip -o tools/exp/lds_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef uint32_t __attribute__((aligned(1))) u32_ua;
typedef __attribute__((address_space(3))) u32_ua lds_u32u;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(1))) u32x4_ua;
typedef __attribute__((address_space(3))) u32x4_ua lds_v4u;

constexpr int kIters = 256;

__device__ __forceinline__ uint32_t mul24_asm(uint32_t x) {
  uint32_t r;
  asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(x), "v"(0x9E3779u));
  return r;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_bench(uint64_t* cyc, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[16384 + 64];
  const uint32_t tid = threadIdx.x;
  for (uint32_t k = tid; k < 16384 / 4; k += 256) ((uint32_t*)buf)[k] = k * 0x9E3779B1u;
  __syncthreads();
  uint32_t acc = tid;
  uint32_t so = (tid * 37u + 5u) & 8191u, dof = 8192u + ((tid * 29u) & 4095u);
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; it++) {
    if (MODE == 0) {
      const lds_u8* p = (const lds_u8*)buf + so;
      const uint32_t sh = (uint32_t)(uintptr_t)p & 3u;
      const lds_u32* q = (const lds_u32*)(p - sh);
      const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
      lds_u32* d = (lds_u32*)((lds_u8*)buf + (dof & ~3u));
      d[0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
      d[1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
      d[2] = __builtin_amdgcn_alignbyte(w3, w2, sh);
      d[3] = __builtin_amdgcn_alignbyte(w4, w3, sh);
    } else if (MODE == 1 || MODE == 2) {
      // separate ds_read_b32 at byte addresses (asm: hipcc would merge four into one ds_read_b128)
      const uint32_t sa = (uint32_t)(uintptr_t)((const lds_u8*)buf + so);
      uint32_t a, b, c, e;
      asm volatile("ds_read_b32 %0, %4\n\tds_read_b32 %1, %4 offset:4\n\tds_read_b32 %2, %4 offset:8\n\t"
                   "ds_read_b32 %3, %4 offset:12\n\ts_waitcnt lgkmcnt(0)"
                   : "=v"(a), "=v"(b), "=v"(c), "=v"(e) : "v"(sa) : "memory");
      if (MODE == 1) {
        lds_u32* d = (lds_u32*)((lds_u8*)buf + (dof & ~3u));
        d[0] = a, d[1] = b, d[2] = c, d[3] = e;
      } else {
        const uint32_t da = (uint32_t)(uintptr_t)((lds_u8*)buf + dof);
        asm volatile("ds_write_b32 %0, %1\n\tds_write_b32 %0, %2 offset:4\n\tds_write_b32 %0, %3 offset:8\n\t"
                     "ds_write_b32 %0, %4 offset:12"
                     :: "v"(da), "v"(a), "v"(b), "v"(c), "v"(e) : "memory");
      }
    } else if (MODE == 3) {
      const u32x4 v = *(const lds_v4u*)((const lds_u8*)buf + so);
      *(__attribute__((address_space(3))) u32x4*)((lds_u8*)buf + (dof & ~15u)) = v;
    } else if (MODE == 4) {
#pragma unroll
      for (int k = 0; k < 8; k++) acc = (acc ^ (uint32_t)k) * 0x9E3779B1u;
    } else if (MODE == 5) {
#pragma unroll
      for (int k = 0; k < 8; k++) acc = ((acc ^ (uint32_t)k) & 0xFFFFFFu) * 0x9E3779u + (acc >> 24);
    } else if (MODE == 6 || MODE == 7) {
      // throughput: 8 independent chains of 4 multiplies (v_mul_lo_u32 / v_mul_u32_u24)
      uint32_t a[8];
#pragma unroll
      for (int k = 0; k < 8; k++) a[k] = acc + (uint32_t)k;
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int k = 0; k < 8; k++) {
          if (MODE == 6) a[k] = a[k] * 0x9E3779B1u;
          else a[k] = mul24_asm(a[k]);
        }
#pragma unroll
      for (int k = 0; k < 8; k++) acc ^= a[k];
    } else {
      // throughput: 8 independent chains of 4 xor-add pairs (full-rate reference)
      uint32_t a[8];
#pragma unroll
      for (int k = 0; k < 8; k++) a[k] = acc + (uint32_t)k;
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int k = 0; k < 8; k++) a[k] = (a[k] ^ 0x9E3779B1u) + 0x7F4A7C15u;
#pragma unroll
      for (int k = 0; k < 8; k++) acc ^= a[k];
    }
    so = (so + 13u) & 8191u;
    dof = 8192u + ((dof + 7u) & 4095u);
    if (MODE <= 3) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): per-iteration round trip, as in the build
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
  if (acc == 0x12345678u) sink[0] = acc + ((uint32_t*)buf)[tid];
}

template <int MODE>
double run(int blocks) {
  uint64_t* d_cyc;
  uint32_t* d_sink;
  hipMalloc(&d_cyc, blocks * 8);
  hipMalloc(&d_sink, 64);
  hipLaunchKernelGGL(k_bench<MODE>, dim3(blocks), dim3(256), 0, 0, d_cyc, d_sink);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_bench<MODE>, dim3(blocks), dim3(256), 0, 0, d_cyc, d_sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  std::vector<uint64_t> c(blocks);
  hipMemcpy(c.data(), d_cyc, blocks * 8, hipMemcpyDeviceToHost);
  std::sort(c.begin(), c.end());
  printf("mode %d: %.1f cycles/iteration/wave (median WG), %.3f ms per launch\n", MODE, (double)c[blocks / 2] / kIters,
         ms / 5);
  hipFree(d_cyc);
  hipFree(d_sink);
  return (double)c[blocks / 2] / kIters;
}

int main() {
  const int blocks = 256 * 4;  // 4 workgroups per CU
  run<0>(blocks);
  run<1>(blocks);
  run<2>(blocks);
  run<3>(blocks);
  run<4>(blocks);
  run<5>(blocks);
  run<6>(blocks);
  run<7>(blocks);
  run<8>(blocks);
  return 0;
}
