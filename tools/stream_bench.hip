// stream_bench.hip -- achievable read bandwidth of streaming-load shapes on
// gfx950, to choose the shape of the privacy-id rescan (pdp_bound.hip
// k_sieve_rescan) and the level-1 sieve.  Reads an 8 GiB int64 column (the
// C3 privacy-id column) and prints GB/s per variant (hipEvent timing, best of
// 5 after a warm-up).  Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/stream_bench tools/stream_bench.hip
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

constexpr size_t kRows = (size_t)1 << 30;  // 1 Gi int64 = 8 GiB

// A: grid-stride, U independent 16-byte loads per thread per iteration
template <int U>
__global__ void __launch_bounds__(256) k_grid(const longlong2* __restrict__ p, size_t n2, unsigned* out) {
  long long acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x * U;
  for (size_t i = blockIdx.x * (size_t)blockDim.x * U + threadIdx.x; i < n2; i += stride) {
    longlong2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + (size_t)u * blockDim.x < n2 ? p[i + (size_t)u * blockDim.x] : longlong2{0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y;
  }
  if (acc == 0x1234567) out[0] = 1;
}

// B: each block one contiguous span (blocks in order), U loads per thread per step
template <int U>
__global__ void __launch_bounds__(256) k_span(const longlong2* __restrict__ p, size_t n2, unsigned* out) {
  long long acc = 0;
  const size_t per = (n2 + gridDim.x - 1) / gridDim.x;
  const size_t b0 = blockIdx.x * per, b1 = b0 + per < n2 ? b0 + per : n2;
  for (size_t i = b0 + threadIdx.x; i < b1; i += (size_t)blockDim.x * U) {
    longlong2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + (size_t)u * blockDim.x < b1 ? p[i + (size_t)u * blockDim.x] : longlong2{0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y;
  }
  if (acc == 0x1234567) out[0] = 1;
}

// C: B + one random LDS probe per row (the rescan's Bloom filter, W words)
template <int U, int W = 16384>
__global__ void __launch_bounds__(512) k_span_lds(const longlong2* __restrict__ p, size_t n2, unsigned* out) {
  __shared__ unsigned bloom[W];
  for (int i = threadIdx.x; i < W; i += blockDim.x) bloom[i] = i * 2654435761u;
  __syncthreads();
  unsigned acc = 0;
  const size_t per = (n2 + gridDim.x - 1) / gridDim.x;
  const size_t b0 = blockIdx.x * per, b1 = b0 + per < n2 ? b0 + per : n2;
  for (size_t i = b0 + threadIdx.x; i < b1; i += (size_t)blockDim.x * U) {
    longlong2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + (size_t)u * blockDim.x < b1 ? p[i + (size_t)u * blockDim.x] : longlong2{0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned h0 = (unsigned)v[u].x * 0x9E3779B1u, h1 = (unsigned)v[u].y * 0x9E3779B1u;
      acc += bloom[(h0 >> 14) & (W - 1)] & (1u << (h0 & 31));
      acc += bloom[(h1 >> 14) & (W - 1)] & (1u << (h1 & 31));
    }
  }
  if (acc == 0x1234567) out[0] = 1;
}

// D: the level-1 shape -- one 1,024-thread block per 65,536-row tile reading
// TWO int64 columns (pid, pk) with 16-byte loads, Q rows per thread per chunk
template <int Q>
__global__ void __launch_bounds__(1024) k_tiles2(const long long* __restrict__ a, const long long* __restrict__ b,
                                                 size_t n, unsigned* out) {
  long long acc = 0;
  const size_t t0 = (size_t)blockIdx.x * 65536, t1 = t0 + 65536 < n ? t0 + 65536 : n;
  for (size_t c0 = t0; c0 < t1; c0 += (size_t)1024 * Q) {
#pragma unroll
    for (int q = 0; q < Q; q += 2) {
      const size_t i = c0 + 2 * (threadIdx.x + (size_t)(q / 2) * 1024);
      if (i + 1 < t1) {
        const longlong2 x = *reinterpret_cast<const longlong2*>(a + i);
        const longlong2 y = *reinterpret_cast<const longlong2*>(b + i);
        acc ^= x.x ^ x.y ^ y.x ^ y.y;
      }
    }
  }
  if (acc == 0x1234567) out[0] = 1;
}

// E: two columns, grid-stride 256-thread blocks (the best one-column shape)
__global__ void __launch_bounds__(256) k_grid2(const longlong2* __restrict__ a, const longlong2* __restrict__ b,
                                               size_t n2, unsigned* out) {
  long long acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x * 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x * 4 + threadIdx.x; i < n2; i += stride) {
    longlong2 v[8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t j = i + (size_t)u * blockDim.x;
      v[2 * u] = j < n2 ? a[j] : longlong2{0, 0};
      v[2 * u + 1] = j < n2 ? b[j] : longlong2{0, 0};
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y;
  }
  if (acc == 0x1234567) out[0] = 1;
}


// F: the level-1 skeleton -- 1,024 threads per 65,536-row tile, two int64
// columns, Q = 4 rows per thread per chunk in a ring of B register buffers
// (the next loads issued right after a chunk is consumed), dynamic LDS to
// pin one workgroup per CU, optionally a barrier per chunk (BAR) and the
// pair hash + a wave-compacted LDS append of ~15 % of rows (WORK)
template <int B, bool BAR, bool WORK>
__global__ void __launch_bounds__(1024) k_l1sim(const long long* __restrict__ a, const long long* __restrict__ b,
                                                size_t n, unsigned* out) {
  extern __shared__ unsigned long long stage[];
  __shared__ unsigned fill;
  if (threadIdx.x == 0) fill = 0;
  __syncthreads();
  const size_t t0 = (size_t)blockIdx.x * 65536, t1 = t0 + 65536 < n ? t0 + 65536 : n;
  if (t1 - t0 < 65536) return;
  constexpr int Q = 4, CH = 1024 * Q, NCH = 65536 / CH;
  long long u[B][Q], k[B][Q];
  auto load = [&](int c, long long (&uu)[Q], long long (&kk)[Q]) {
    const size_t c0 = t0 + (size_t)(c < NCH ? c : NCH - 1) * CH;
#pragma unroll
    for (int q = 0; q < Q; q += 2) {
      const size_t i = c0 + 2 * (threadIdx.x + (size_t)(q / 2) * 1024);
      const longlong2 x = *reinterpret_cast<const longlong2*>(a + i);
      const longlong2 y = *reinterpret_cast<const longlong2*>(b + i);
      uu[q] = x.x; uu[q + 1] = x.y; kk[q] = y.x; kk[q + 1] = y.y;
    }
  };
#pragma unroll
  for (int j = 0; j < B; ++j) load(j, u[j], k[j]);
  unsigned acc = 0;
  const int lane = threadIdx.x & 63;
  for (int c = 0; c < NCH; c += B) {
#pragma unroll
    for (int j = 0; j < B; ++j) {
      unsigned ul[Q], kl[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) { ul[q] = (unsigned)u[j][q] ^ (unsigned)(u[j][q] >> 32); kl[q] = (unsigned)k[j][q]; }
      load(c + j + B, u[j], k[j]);
      if (WORK) {
        bool cand[Q];
        unsigned long long m[Q];
        unsigned nw = 0;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          unsigned h = (ul[q] ^ 0x1234567u) * 0x9E3779B1u;
          h = h ^ (kl[q] * 0xC2B2AE3Du + 77u);
          h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
          cand[q] = h < 0x26000000u;
          m[q] = __ballot(cand[q]);
          nw += (unsigned)__popcll(m[q]);
        }
        unsigned base = 0;
        if (lane == 0 && nw) base = atomicAdd(&fill, nw);
        base = __shfl(base, 0, 64) & 8191u;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          if (cand[q]) stage[(base + (unsigned)__popcll(m[q] & ((1ULL << lane) - 1))) & 8191u] = ((unsigned long long)ul[q] << 32) | kl[q];
          base += (unsigned)__popcll(m[q]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < Q; ++q) acc ^= ul[q] ^ kl[q];
      }
      if (BAR) __syncthreads();
    }
  }
  if (acc == 0x1234567 || fill == 0x7654321) out[0] = 1;
}

template <typename F>
double time_it(F&& launch) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(a));
    launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  return best;
}

int main() {
  longlong2* p;
  unsigned* out;
  CHECK(hipMalloc(&p, kRows * 8));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(p, 3, kRows * 8));
  const size_t n2 = kRows / 2;
  const double gb = kRows * 8 / 1e9;
  auto report = [&](const char* name, double ms) { printf("%-28s %8.3f ms %8.1f GB/s\n", name, ms, gb / (ms * 1e-3)); };
#define RUN(NAME, KERNEL, GRID)                                                                           \
  report(NAME, time_it([&] { hipLaunchKernelGGL(KERNEL, dim3(GRID), dim3(256), 0, 0, p, n2, out); }))
  RUN("grid U=4 g=2048", k_grid<4>, 2048);
  RUN("grid U=8 g=2048", k_grid<8>, 2048);
  RUN("grid U=4 g=8192", k_grid<4>, 8192);
  RUN("grid U=8 g=1024", k_grid<8>, 1024);
  RUN("span U=4 g=2048", k_span<4>, 2048);
  RUN("span U=8 g=2048", k_span<8>, 2048);
  RUN("span U=4 g=8192", k_span<4>, 8192);
  RUN("span U=8 g=1024", k_span<8>, 1024);
  RUN("span+lds64K U=8 g=1024", k_span_lds<8>, 1024);
  RUN("span+lds64K U=8 g=2048", k_span_lds<8>, 2048);
#define RUN2(NAME, KERNEL, GRID, TH)                                                                      \
  report(NAME, time_it([&] { hipLaunchKernelGGL(KERNEL, dim3(GRID), dim3(TH), 0, 0, p, n2, out); }))
  RUN2("span+lds16K U=8 g=2048 t256", (k_span_lds<8, 4096>), 2048, 256);
  RUN2("span+lds16K U=8 g=2048 t512", (k_span_lds<8, 4096>), 2048, 512);
  RUN2("span+lds8K U=8 g=2048 t256", (k_span_lds<8, 2048>), 2048, 256);
  RUN2("span+lds8K U=8 g=2048 t512", (k_span_lds<8, 2048>), 2048, 512);
  RUN2("span+lds4K U=8 g=4096 t256", (k_span_lds<8, 1024>), 4096, 256);
  RUN2("span+lds8K U=4 g=4096 t256", (k_span_lds<4, 2048>), 4096, 256);
  {  // two 4 GiB columns (the level-1 pid / pk pair): 8 GiB read per call
    const size_t n = kRows / 2;
    const long long* a = (const long long*)p;
    const long long* b = a + n;
    const unsigned tiles = (unsigned)((n + 65535) / 65536);
    auto rep2 = [&](const char* name, double ms) { printf("%-28s %8.3f ms %8.1f GB/s\n", name, ms, gb / (ms * 1e-3)); };
    rep2("tiles2 Q=4 (level-1 shape)", time_it([&] { hipLaunchKernelGGL((k_tiles2<4>), dim3(tiles), dim3(1024), 0, 0, a, b, n, out); }));
    rep2("tiles2 Q=8", time_it([&] { hipLaunchKernelGGL((k_tiles2<8>), dim3(tiles), dim3(1024), 0, 0, a, b, n, out); }));
    const size_t lds = 150 * 1024;
#define SIM(NAME, ...)                                                                                   \
    CHECK(hipFuncSetAttribute((const void*)(__VA_ARGS__), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    rep2(NAME, time_it([&] { hipLaunchKernelGGL((__VA_ARGS__), dim3(tiles), dim3(1024), lds, 0, a, b, n, out); }))
    SIM("l1sim B2", k_l1sim<2, false, false>);
    SIM("l1sim B3", k_l1sim<3, false, false>);
    SIM("l1sim B2 bar", k_l1sim<2, true, false>);
    SIM("l1sim B2 bar work", k_l1sim<2, true, true>);
    SIM("l1sim B3 bar work", k_l1sim<3, true, true>);
    SIM("l1sim B2 work", k_l1sim<2, false, true>);
    SIM("l1sim B4", k_l1sim<4, false, false>);
    rep2("grid2 U=4 g=2048", time_it([&] { hipLaunchKernelGGL(k_grid2, dim3(2048), dim3(256), 0, 0, (const longlong2*)a,
                                                               (const longlong2*)b, n / 2, out); }));
  }
  CHECK(hipFree(p));
  CHECK(hipFree(out));
  return 0;
}
