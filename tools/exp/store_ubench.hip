// Microbenchmark (diagnostic, not product): how rocprofv3's WRITE_SIZE tallies the store patterns
// k_resolve has, on gfx950, against known byte counts (the FETCH_SIZE
// counterpart is gather_ubench.hip):
//   k_st<W>         coalesced W-byte stores, lane i at dst + i*W (W = 16, 8, 4, 2, 1): the per-string
//                   offset (8), length / value id (4) and status (1) arrays, the 16-B stream-out
//   k_st_nt<W>      the same stores, non-temporal (k_resolve's gst4s / gsts)
//   k_st_half<4>    every other lane stores (a predicated per-string store)
//   k_st_line<W>    one W-byte store per 64-B line (lane i at dst + i*64): partial-line writes
//   k_st_run<W,R>   each lane writes R consecutive W-byte elements of its own (a per-string record
//                   laid out lane-major: lanes write 64 R W apart)
// Launch order (one dispatch per line printed, two rounds: read the second); compare WRITE_SIZE
// (KB) per dispatch with `bytes`.
// Build: hipcc --offload-arch=gfx950 -O3 tools/exp/store_ubench.hip -o tools/exp/store_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

template <int W>
struct Elem;
template <>
struct Elem<16> {
  typedef u32x4 T;
};
template <>
struct Elem<8> {
  typedef uint64_t T;
};
template <>
struct Elem<4> {
  typedef uint32_t T;
};
template <>
struct Elem<2> {
  typedef uint16_t T;
};
template <>
struct Elem<1> {
  typedef uint8_t T;
};

template <int W>
__device__ __forceinline__ typename Elem<W>::T val(uint64_t i) {
  typedef typename Elem<W>::T T;
  if constexpr (W == 16) {
    return u32x4{(uint32_t)i, (uint32_t)(i >> 32), 7u, 9u};
  } else {
    return (T)(i * 2654435761u + 1);
  }
}

template <int W>
__global__ __launch_bounds__(256) void k_st(uint8_t* dst, uint64_t n) {
  typedef typename Elem<W>::T T;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) ((T*)dst)[i] = val<W>(i);
}

__global__ __launch_bounds__(256) void k_st_nt16(uint8_t* dst, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    __builtin_nontemporal_store(val<16>(i), (u32x4*)dst + i);
}

template <int W>
__global__ __launch_bounds__(256) void k_st_nt(uint8_t* dst, uint64_t n) {  // narrow non-temporal (gsts)
  typedef typename Elem<W>::T T;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    __builtin_nontemporal_store(val<W>(i), (T*)dst + i);
}

template <int W>
__global__ __launch_bounds__(256) void k_st_half(uint8_t* dst, uint64_t n) {  // every other lane stores
  typedef typename Elem<W>::T T;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    if (i & 1) ((T*)dst)[i] = val<W>(i);
}

template <int W>
__global__ __launch_bounds__(256) void k_st_line(uint8_t* dst, uint64_t n) {
  typedef typename Elem<W>::T T;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    *(T*)(dst + i * 64) = val<W>(i);
}

template <int W, int R>
__global__ __launch_bounds__(256) void k_st_run(uint8_t* dst, uint64_t n) {  // n lanes, R elements each
  typedef typename Elem<W>::T T;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    T* p = (T*)dst + i * R;
#pragma unroll
    for (int r = 0; r < R; r++) p[r] = val<W>(i * R + r);
  }
}

int main() {
  const uint64_t bytes = 256ull << 20;
  uint8_t* dst;
  CHECK(hipMalloc(&dst, bytes * 64));  // (the one-store-per-line kernels span 64x their bytes)
  CHECK(hipMemset(dst, 0, bytes * 64));
  CHECK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const dim3 grid(4096), block(256);
  int line = 0;
  auto run = [&](const char* name, auto launch, uint64_t nbytes, uint64_t span) -> int {
    CHECK(hipEventRecord(a));
    launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("%d %s bytes=%llu span=%llu ms=%.4f\n", line++, name, (unsigned long long)nbytes, (unsigned long long)span, ms);
    return 0;
  };
  for (int rep = 0; rep < 2; rep++) {
    if (run("k_st<16>", [&] { k_st<16><<<grid, block>>>(dst, bytes / 16); }, bytes, bytes)) return 1;
    if (run("k_st_nt<16>", [&] { k_st_nt16<<<grid, block>>>(dst, bytes / 16); }, bytes, bytes)) return 1;
    if (run("k_st<8>", [&] { k_st<8><<<grid, block>>>(dst, bytes / 8); }, bytes, bytes)) return 1;
    if (run("k_st<4>", [&] { k_st<4><<<grid, block>>>(dst, bytes / 4); }, bytes, bytes)) return 1;
    if (run("k_st<2>", [&] { k_st<2><<<grid, block>>>(dst, bytes / 2); }, bytes, bytes)) return 1;
    if (run("k_st<1>", [&] { k_st<1><<<grid, block>>>(dst, bytes); }, bytes, bytes)) return 1;
    const uint64_t nl = bytes / 64;  // lines touched by the one-store-per-line kernels
    if (run("k_st_line<8>", [&] { k_st_line<8><<<grid, block>>>(dst, nl); }, nl * 8, nl * 64)) return 1;
    if (run("k_st_line<4>", [&] { k_st_line<4><<<grid, block>>>(dst, nl); }, nl * 4, nl * 64)) return 1;
    if (run("k_st_line<1>", [&] { k_st_line<1><<<grid, block>>>(dst, nl); }, nl, nl * 64)) return 1;
    if (run("k_st_nt<8>", [&] { k_st_nt<8><<<grid, block>>>(dst, bytes / 8); }, bytes, bytes)) return 1;
    if (run("k_st_nt<4>", [&] { k_st_nt<4><<<grid, block>>>(dst, bytes / 4); }, bytes, bytes)) return 1;
    if (run("k_st_nt<1>", [&] { k_st_nt<1><<<grid, block>>>(dst, bytes); }, bytes, bytes)) return 1;
    if (run("k_st_half<4>", [&] { k_st_half<4><<<grid, block>>>(dst, bytes / 4); }, bytes / 2, bytes)) return 1;
    if (run("k_st_run<8,2>", [&] { k_st_run<8, 2><<<grid, block>>>(dst, bytes / 16); }, bytes, bytes)) return 1;
    if (run("k_st_run<4,4>", [&] { k_st_run<4, 4><<<grid, block>>>(dst, bytes / 16); }, bytes, bytes)) return 1;
  }
  CHECK(hipFree(dst));
  return 0;
}
