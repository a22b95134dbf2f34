// Microbenchmark (diagnostic, not product): how rocprofv3's FETCH_SIZE tallies the two read
// patterns k_resolve has, on gfx950, against known byte counts:
//   k_stream        coalesced 16 B/lane streaming reads (the input stage)
//   k_gather<HEAD>  per-lane random reads of 64-B table entries, as find_small does them
//                   (HEAD=1: two 16-B loads at +0/+16 and the dword at +60; HEAD=0: the whole
//                   64 B, four 16-B loads), from tables of 1k, 100k and 10M entries
// Launch order (one dispatch per line printed); compare FETCH_SIZE per dispatch with `bytes`.
// Build: hipcc --offload-arch=gfx950 -O3 tools/exp/gather_ubench.hip -o tools/exp/gather_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

constexpr int kBlocks = 2048, kThreads = 256, kPerLane = 8;

__global__ __launch_bounds__(256) void k_stream(const u32x4* src, uint64_t n16, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)kThreads + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * kThreads) {
    const u32x4 v = __builtin_nontemporal_load(src + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

template <int HEAD>
__global__ __launch_bounds__(256) void k_gather(const uint8_t* table, uint32_t nent, uint32_t salt, uint32_t* sink) {
  uint32_t acc = 0;
  const uint32_t g = blockIdx.x * kThreads + threadIdx.x;
#pragma unroll
  for (int k = 0; k < kPerLane; k++) {
    const uint32_t e = mix(g * kPerLane + k + salt) % nent;
    const u32x4* p = (const u32x4*)(table + (uint64_t)e * 64);
    const u32x4 a = p[0], b = p[1];
    acc ^= a.x ^ a.y ^ b.z ^ b.w;
    if (HEAD) {
      acc ^= ((const uint32_t*)p)[15];
    } else {
      const u32x4 c = p[2], d = p[3];
      acc ^= c.x ^ d.w;
    }
  }
  if (acc == 0x12345678u) sink[g] = acc;
}

int main() {
  const uint64_t stream_bytes = 512ull << 20;
  const uint32_t sizes[3] = {1000u, 100000u, 10000000u};
  uint8_t *src, *table;
  uint32_t* sink;
  CHECK(hipMalloc(&src, stream_bytes));
  CHECK(hipMalloc(&table, (uint64_t)sizes[2] * 64));
  CHECK(hipMalloc(&sink, (uint64_t)kBlocks * kThreads * 4));
  CHECK(hipMemset(src, 1, stream_bytes));
  CHECK(hipMemset(table, 2, (uint64_t)sizes[2] * 64));
  CHECK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const uint64_t gathers = (uint64_t)kBlocks * kThreads * kPerLane;
  int line = 0;
  for (int rep = 0; rep < 2; rep++) {  // the second round is the one to read (warm caches)
    CHECK(hipEventRecord(a));
    k_stream<<<kBlocks, kThreads>>>((const u32x4*)src, stream_bytes / 16, sink);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("%d k_stream bytes=%llu ms=%.4f GB/s=%.1f\n", line++, (unsigned long long)stream_bytes, ms,
           stream_bytes / (ms * 1e-3) / 1e9);
    for (int s = 0; s < 3; s++) {
      for (int head = 1; head >= 0; head--) {
        CHECK(hipEventRecord(a));
        if (head)
          k_gather<1><<<kBlocks, kThreads>>>(table, sizes[s], 977u * rep, sink);
        else
          k_gather<0><<<kBlocks, kThreads>>>(table, sizes[s], 977u * rep + 1, sink);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("%d k_gather<%d> entries=%u table_MB=%.1f gathers=%llu bytes=%llu ms=%.4f\n", line++, head, sizes[s],
               sizes[s] * 64 / 1e6, (unsigned long long)gathers, (unsigned long long)(gathers * 64), ms);
      }
    }
  }
  CHECK(hipFree(src));
  CHECK(hipFree(table));
  CHECK(hipFree(sink));
  return 0;
}
