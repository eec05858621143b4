// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950
// for the access widths the bounding kernels use (MI355X_MICROARCH.md "HBM":
// only 16-byte streaming loads are calibrated there, at FETCH = 1/2 of the
// bytes).  Each kernel touches a known set of distinct cache lines of a
// buffer far larger than the 256 MiB Infinity Cache, once:
//   k_stream16    16-byte loads over 2 GiB, coalesced                (2 GiB)
//   k_gather8     one 8-byte load in each of G distinct 128-byte lines (G lines)
//   k_gather4     one 4-byte load in each of G distinct 128-byte lines
//   k_gather8x2   two 8-byte loads 64 bytes apart in each of G lines
//   k_gather8h    one 8-byte load in each of G distinct 64-byte halves
//                 (every other half of G/2... lines: two per line, 64 B apart,
//                 issued by different waves)
//   k_scatter8    one 8-byte store in each of G distinct 128-byte lines
//   k_stream16w   16-byte stores over 2 GiB
// (k_flush, between them, streams 512 MiB of stores to evict the cache)
// Run: rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib, then --pmc WRITE_SIZE;
// FETCH_SIZE / WRITE_SIZE are in KiB.  tools/fetch_calib.py prints the ratio
// counter bytes / line bytes per kernel.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                       \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr size_t kBytes = (size_t)4 << 30;        // buffer: 4 GiB
constexpr size_t kLines = kBytes / 128;           // 128-byte lines
constexpr size_t kGathers = (size_t)8 << 20;      // 8 Mi distinct lines per gather kernel (1 GiB of lines)
constexpr unsigned long long kStride = 2654435761ULL;  // odd: i -> (i * kStride) mod kLines is a bijection

// lines of the lower 2 GiB only (k_flush writes the upper half)
__device__ __forceinline__ size_t line_of(size_t i) { return (i * kStride) & (kLines / 2 - 1); }

__global__ void k_stream16(const uint4* __restrict__ src, size_t n, unsigned* out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;  // keeps the loads
}

__global__ void k_gather8(const unsigned long long* __restrict__ src, size_t g, unsigned* out) {
  unsigned long long acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < g; i += (size_t)gridDim.x * blockDim.x)
    acc ^= src[line_of(i) * 16];
  if (acc == 0x12345678ULL) out[0] = (unsigned)acc;
}

__global__ void k_gather4(const unsigned* __restrict__ src, size_t g, unsigned* out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < g; i += (size_t)gridDim.x * blockDim.x)
    acc ^= src[line_of(i) * 32];
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_gather8x2(const unsigned long long* __restrict__ src, size_t g, unsigned* out) {
  unsigned long long acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < g; i += (size_t)gridDim.x * blockDim.x)
    acc ^= src[line_of(i) * 16] ^ src[line_of(i) * 16 + 8];
  if (acc == 0x12345678ULL) out[0] = (unsigned)acc;
}

// lines i and its 64-byte halves from two different threads far apart in the grid
__global__ void k_gather8h(const unsigned long long* __restrict__ src, size_t g, unsigned* out) {
  unsigned long long acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < g; i += (size_t)gridDim.x * blockDim.x) {
    const size_t half = i & 1, j = i >> 1;
    acc ^= src[line_of(j) * 16 + half * 8];
  }
  if (acc == 0x12345678ULL) out[0] = (unsigned)acc;
}

__global__ void k_scatter8(unsigned long long* __restrict__ dst, size_t g) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < g; i += (size_t)gridDim.x * blockDim.x)
    dst[line_of(i) * 16] = i;
}

__global__ void k_flush(uint4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = make_uint4((unsigned)i, 7u, 8u, 9u);
}

__global__ void k_stream16w(uint4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}

int main() {
  char* buf = nullptr;
  unsigned* out = nullptr;
  CHECK(hipMalloc(&buf, kBytes));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(buf, 1, kBytes));
  // evict the 256 MiB Infinity Cache between kernels by streaming stores over
  // the upper half of the buffer (k_flush, reported separately)
  auto flush = [&]() {
    hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, (uint4*)(buf + kBytes / 2), (size_t)(512 << 20) / 16);
    CHECK(hipDeviceSynchronize());
  };
  const size_t n16 = ((size_t)2 << 30) / 16;
  flush();
  hipLaunchKernelGGL(k_stream16, dim3(4096), dim3(256), 0, 0, (const uint4*)buf, n16, out);
  CHECK(hipDeviceSynchronize());
  flush();
  hipLaunchKernelGGL(k_gather8, dim3(4096), dim3(256), 0, 0, (const unsigned long long*)buf, kGathers, out);
  CHECK(hipDeviceSynchronize());
  flush();
  hipLaunchKernelGGL(k_gather4, dim3(4096), dim3(256), 0, 0, (const unsigned*)buf, kGathers, out);
  CHECK(hipDeviceSynchronize());
  flush();
  hipLaunchKernelGGL(k_gather8x2, dim3(4096), dim3(256), 0, 0, (const unsigned long long*)buf, kGathers, out);
  CHECK(hipDeviceSynchronize());
  flush();
  hipLaunchKernelGGL(k_gather8h, dim3(4096), dim3(256), 0, 0, (const unsigned long long*)buf, 2 * kGathers, out);
  CHECK(hipDeviceSynchronize());
  flush();
  hipLaunchKernelGGL(k_scatter8, dim3(4096), dim3(256), 0, 0, (unsigned long long*)buf, kGathers);
  CHECK(hipDeviceSynchronize());
  hipLaunchKernelGGL(k_stream16w, dim3(4096), dim3(256), 0, 0, (uint4*)buf, n16);
  CHECK(hipDeviceSynchronize());
  printf("fetch_calib: stream 2 GiB; gathers %zu lines of 128 B (%.3f GB of lines)\n", kGathers,
         kGathers * 128.0 / 1e9);
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
