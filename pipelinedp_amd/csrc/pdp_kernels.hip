// pdp_kernels.hip — gfx950 kernels + C ABI for the DPEngine.aggregate hot path.
//
// Stage map (reference = lagodiuk/PipelineDP 0.2.2rc2, pure Python):
//   k_pair_sketch      per-privacy-id bottom-L0 sketch of pair priorities
//                      == "Sample per privacy_id" (contribution_bounders.py:96-98)
//   k_pair_rows        per-(pid, pk) row count + bottom-Linf row sketch
//                      == "Sample per (privacy_id, partition_key)" (:80-82)
//   k_reduce_pairs     per-pair accumulators merged per partition
//                      == create_accumulator (combiners.py:749-753) +
//                         combine_accumulators_per_key (pipeline_backend.py:555-565)
//   k_select           private partition selection (dp_engine.py:315-371)
//   k_compact_*        ascending compaction of kept partitions
//   k_noise_metrics    CompoundCombiner.compute_metrics (combiners.py:766-788)
//
// Sampling: a uniform sample without replacement of k out of m items equals
// "the k items with the smallest i.i.d. uniform priorities".  Priorities are
// counter-based (SplitMix64 finaliser keyed by the seed), so the sampled set
// does not depend on thread scheduling and the CPU oracle can reproduce it
// bit-for-bit.  The per-pid and per-pair sketches are sorted arrays kept by a
// lock-free atomicMin cascade (values only ever decrease, so a plain load of
// the last slot is a safe early reject).
//
// Noise / selection randomness: Philox4x32-10 keyed by the seed, counter =
// (global partition index, mechanism slot).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <cstring>
#include <cstdio>

#include "../../include/pipelinedp_amd.h"

namespace {

thread_local std::string g_last_error;

int set_error(int code, const char* msg) {
  g_last_error = msg;
  return code;
}

#define PDP_HIP_CHECK(expr)                                                      \
  do {                                                                           \
    hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess) {                                                      \
      char buf_[256];                                                            \
      snprintf(buf_, sizeof(buf_), "%s failed: %s", #expr, hipGetErrorString(e_)); \
      return set_error(PDP_E_HIP, buf_);                                         \
    }                                                                            \
  } while (0)

constexpr uint64_t kEmpty = ~0ULL;
constexpr int kBlock = 256;

// ---------------------------------------------------------------- hashing --
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// Priority of the pair (pid, pk): random high bits, pk in the low bits, so
// that equal pairs collide exactly and the partition is recoverable.
__device__ __forceinline__ uint64_t pair_priority(uint64_t seed, int64_t pid, int64_t pk,
                                                  uint64_t pk_mask) {
  uint64_t h = mix64(seed ^ ((uint64_t)pid * 0x9E3779B97F4A7C15ULL));
  h = mix64(h + (uint64_t)pk * 0xC2B2AE3D27D4EB4FULL + 0x165667B19E3779F9ULL);
  if ((h | pk_mask) == kEmpty) h ^= (pk_mask + 1);  // never the EMPTY sentinel
  return (h & ~pk_mask) | (uint64_t)pk;
}

// Priority of row `i` of the shard: 32 random bits over the local row index.
__device__ __forceinline__ uint64_t row_priority(uint64_t row_seed, int64_t global_row,
                                                 uint32_t local_row) {
  uint64_t h = mix64(row_seed ^ ((uint64_t)global_row * 0xD6E8FEB86659FD93ULL));
  return (h & 0xFFFFFFFF00000000ULL) | (uint64_t)local_row;
}

__host__ __device__ __forceinline__ uint64_t derive_row_seed(uint64_t seed) {
  return mix64(seed ^ 0x5851F42D4C957F2DULL);
}

// ---------------------------------------------------------------- philox --
struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x;
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// uniform double in (0, 1) from 64 random bits (53-bit grid, open interval)
__device__ __forceinline__ double u01(uint32_t hi, uint32_t lo) {
  const uint64_t x = (((uint64_t)hi << 32) | lo) >> 11;
  return ((double)x + 0.5) * (1.0 / 9007199254740992.0);
}

// counter = (global partition index, stream slot)
__device__ __forceinline__ U4 philox_for(uint64_t seed, int64_t gidx, uint32_t slot) {
  U4 c{(uint32_t)((uint64_t)gidx), (uint32_t)((uint64_t)gidx >> 32), slot, 0x50445021u};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

__device__ __forceinline__ double laplace_noise(double b, U4 r) {
  const double u = u01(r.x, r.y) - 0.5;  // (-0.5, 0.5)
  const double a = fabs(u);
  const double mag = -b * log1p(-2.0 * a);
  return u < 0.0 ? -mag : mag;
}

__device__ __forceinline__ double gaussian_noise(double sigma, U4 r) {
  const double u1 = u01(r.x, r.y);
  const double u2 = u01(r.z, r.w);
  return sigma * sqrt(-2.0 * log(u1)) * cos(6.283185307179586476925286766559 * u2);
}

__device__ __forceinline__ double draw_noise(int kind, double scale, U4 r) {
  return kind == PDP_NOISE_GAUSSIAN ? gaussian_noise(scale, r) : laplace_noise(scale, r);
}

// ------------------------------------------------- sorted-sketch insertion --
// Insert x into the ascending array s[0..k) keeping the k smallest DISTINCT
// values.  Lock-free: every atomicMin keeps the array sorted; a value equal
// to x met on the way means x is already present.
__device__ __forceinline__ void sketch_insert(unsigned long long* s, int k, uint64_t x) {
  for (int j = 0; j < k; ++j) {
    const uint64_t old = atomicMin(s + j, (unsigned long long)x);
    if (old == x) return;      // duplicate
    if (old > x) {
      if (old == kEmpty) return;  // filled an empty slot
      x = old;                    // carry the displaced value right
    }
  }
}

// position of x in the ascending s[0..k), -1 if absent
__device__ __forceinline__ int sketch_find(const unsigned long long* s, int k, uint64_t x) {
  int lo = 0, hi = k;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const uint64_t v = s[mid];
    if (v < x) lo = mid + 1; else hi = mid;
  }
  return (lo < k && s[lo] == x) ? lo : -1;
}

struct BoundParams {
  int64_t n, U, P;
  int l0, linf;
  uint64_t pk_mask, seed, row_seed;
  int64_t row_offset;
};

__device__ __forceinline__ bool key_ok(const BoundParams& bp, int64_t u, int64_t k,
                                       unsigned int* err) {
  if (u < 0 || u >= bp.U || k < 0 || k >= bp.P) {
    atomicOr(err, 1u);
    return false;
  }
  return true;
}

// ------------------------------------------------------------- kernels --
__global__ void __launch_bounds__(kBlock) k_pair_sketch(BoundParams bp,
                                                        const int64_t* __restrict__ pid,
                                                        const int64_t* __restrict__ pk,
                                                        const uint8_t* __restrict__ allowed,
                                                        unsigned long long* sketch,
                                                        unsigned int* err) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < bp.n; i += stride) {
    const int64_t u = pid[i];
    const int64_t k = pk[i];
    if (!key_ok(bp, u, k, err)) continue;
    if (allowed != nullptr && allowed[k] == 0) continue;
    const uint64_t x = pair_priority(bp.seed, u, k, bp.pk_mask);
    unsigned long long* s = sketch + u * bp.l0;
    if (x >= s[bp.l0 - 1]) continue;  // not among the l0 smallest (or duplicate)
    sketch_insert(s, bp.l0, x);
  }
}

// LINF > 0: bottom-linf row sketch per kept pair.  LINF == 0: keep every row
// of a kept pair and accumulate the pair sums directly.
template <int VALUE_KIND, bool KEEP_ALL_ROWS>
__global__ void __launch_bounds__(kBlock) k_pair_rows(BoundParams bp, const int64_t* __restrict__ pid,
                                                      const int64_t* __restrict__ pk,
                                                      const void* __restrict__ value,
                                                      const uint8_t* __restrict__ allowed,
                                                      const unsigned long long* __restrict__ sketch,
                                                      unsigned int* pair_cnt,
                                                      unsigned long long* pair_rows,
                                                      double* pair_fsum, long long* pair_isum,
                                                      double* pair_nsum, double* pair_nsum2,
                                                      double lo, double hi, double mid, int flags,
                                                      unsigned int* err) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < bp.n; i += stride) {
    const int64_t u = pid[i];
    const int64_t k = pk[i];
    if (u < 0 || u >= bp.U || k < 0 || k >= bp.P) continue;  // flagged by k_pair_sketch
    if (allowed != nullptr && allowed[k] == 0) continue;
    const uint64_t x = pair_priority(bp.seed, u, k, bp.pk_mask);
    const unsigned long long* s = sketch + u * bp.l0;
    if (x > s[bp.l0 - 1]) continue;
    const int j = sketch_find(s, bp.l0, x);
    if (j < 0) continue;
    const int64_t slot = u * bp.l0 + j;
    atomicAdd(pair_cnt + slot, 1u);
    if (!KEEP_ALL_ROWS) {
      const uint64_t y = row_priority(bp.row_seed, bp.row_offset + i, (uint32_t)i);
      unsigned long long* r = pair_rows + slot * bp.linf;
      if (y < r[bp.linf - 1]) sketch_insert(r, bp.linf, y);
    } else if (VALUE_KIND != PDP_VALUE_NONE) {
      double v;
      long long iv = 0;
      if (VALUE_KIND == PDP_VALUE_I64) {
        iv = ((const long long*)value)[i];
        v = (double)iv;
      } else {
        v = ((const double*)value)[i];
      }
      if (flags & PDP_SUM_PER_PARTITION) {
        // raw pair sum; clipped per pair in k_reduce_pairs
        if (flags & PDP_SUM_INT) atomicAdd((unsigned long long*)(pair_isum + slot), (unsigned long long)iv);
        else unsafeAtomicAdd(pair_fsum + slot, v);
      } else if (flags & PDP_ACC_SUM) {
        if (flags & PDP_SUM_INT) {
          const long long ilo = (long long)lo, ihi = (long long)hi;
          const long long c = iv < ilo ? ilo : (iv > ihi ? ihi : iv);
          atomicAdd((unsigned long long*)(pair_isum + slot), (unsigned long long)c);
        } else {
          unsafeAtomicAdd(pair_fsum + slot, fmin(fmax(v, lo), hi));
        }
      }
      if (flags & (PDP_ACC_NSUM | PDP_ACC_NSUM2)) {
        const double c = fmin(fmax(v, lo), hi) - mid;
        if (flags & PDP_ACC_NSUM) unsafeAtomicAdd(pair_nsum + slot, c);
        if (flags & PDP_ACC_NSUM2) unsafeAtomicAdd(pair_nsum2 + slot, c * c);
      }
    }
  }
}

template <int VALUE_KIND, bool KEEP_ALL_ROWS>
__global__ void __launch_bounds__(kBlock) k_reduce_pairs(BoundParams bp, const void* __restrict__ value,
                                                         const unsigned long long* __restrict__ sketch,
                                                         const unsigned int* __restrict__ pair_cnt,
                                                         const unsigned long long* __restrict__ pair_rows,
                                                         const double* __restrict__ pair_fsum,
                                                         const long long* __restrict__ pair_isum,
                                                         const double* __restrict__ pair_nsum,
                                                         const double* __restrict__ pair_nsum2,
                                                         double lo, double hi, double mid,
                                                         double min_sum, double max_sum, int flags,
                                                         pdp_partition_accumulators acc) {
  const int64_t n_slots = bp.U * bp.l0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_slots; s += stride) {
    const uint64_t x = sketch[s];
    if (x == kEmpty) continue;
    const int64_t p = (int64_t)(x & bp.pk_mask);
    const unsigned int c = pair_cnt[s];
    if (c == 0) continue;  // cannot happen for a kept pair; defensive
    long long m;
    double fsum = 0.0, nsum = 0.0, nsum2 = 0.0;
    long long isum = 0;
    if (!KEEP_ALL_ROWS) {
      m = c < (unsigned)bp.linf ? (long long)c : (long long)bp.linf;
      if (VALUE_KIND != PDP_VALUE_NONE) {
        const unsigned long long* r = pair_rows + s * bp.linf;
        double raw = 0.0;
        long long iraw = 0;
        for (long long t = 0; t < m; ++t) {
          const uint32_t row = (uint32_t)r[t];
          double v;
          long long iv = 0;
          if (VALUE_KIND == PDP_VALUE_I64) {
            iv = ((const long long*)value)[row];
            v = (double)iv;
          } else {
            v = ((const double*)value)[row];
          }
          const double cv = fmin(fmax(v, lo), hi);
          if (flags & PDP_SUM_PER_PARTITION) {
            raw += v;
            iraw += iv;
          } else if (flags & PDP_SUM_INT) {
            const long long ilo = (long long)lo, ihi = (long long)hi;
            isum += iv < ilo ? ilo : (iv > ihi ? ihi : iv);
          } else {
            fsum += cv;
          }
          const double nc = cv - mid;
          nsum += nc;
          nsum2 += nc * nc;
        }
        if (flags & PDP_SUM_PER_PARTITION) {
          if (flags & PDP_SUM_INT) {
            const long long ilo = (long long)min_sum, ihi = (long long)max_sum;
            isum = iraw < ilo ? ilo : (iraw > ihi ? ihi : iraw);
          } else {
            fsum = fmin(fmax(raw, min_sum), max_sum);
          }
        }
      }
    } else {
      m = (long long)c;
      if (VALUE_KIND != PDP_VALUE_NONE) {
        if (flags & PDP_SUM_PER_PARTITION) {
          if (flags & PDP_SUM_INT) {
            const long long ilo = (long long)min_sum, ihi = (long long)max_sum;
            const long long raw = pair_isum[s];
            isum = raw < ilo ? ilo : (raw > ihi ? ihi : raw);
          } else {
            fsum = fmin(fmax(pair_fsum[s], min_sum), max_sum);
          }
        } else if (flags & PDP_ACC_SUM) {
          if (flags & PDP_SUM_INT) isum = pair_isum[s];
          else fsum = pair_fsum[s];
        }
        if (flags & PDP_ACC_NSUM) nsum = pair_nsum[s];
        if (flags & PDP_ACC_NSUM2) nsum2 = pair_nsum2[s];
      }
    }
    atomicAdd((unsigned long long*)(acc.privacy_id_count + p), 1ULL);
    if (acc.count) atomicAdd((unsigned long long*)(acc.count + p), (unsigned long long)m);
    if (acc.sum && (flags & (PDP_ACC_SUM | PDP_SUM_PER_PARTITION))) {
      if (flags & PDP_SUM_INT) atomicAdd((unsigned long long*)acc.sum + p, (unsigned long long)isum);
      else unsafeAtomicAdd((double*)acc.sum + p, fsum);
    }
    if (acc.normalized_sum && (flags & PDP_ACC_NSUM)) unsafeAtomicAdd(acc.normalized_sum + p, nsum);
    if (acc.normalized_sum_sq && (flags & PDP_ACC_NSUM2)) unsafeAtomicAdd(acc.normalized_sum_sq + p, nsum2);
  }
}

__global__ void __launch_bounds__(kBlock) k_select(pdp_select_config cfg, const int64_t* __restrict__ row_count,
                                                   uint8_t* __restrict__ keep, double* __restrict__ noised) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < cfg.n_partitions; p += stride) {
    const int64_t rc = row_count[p];
    uint8_t kp = 0;
    double nz = __builtin_nan("");
    if (cfg.strategy == PDP_SELECT_PUBLIC) {
      kp = cfg.public_mask[p] != 0;
    } else if (cfg.strategy == PDP_SELECT_ALL_NONEMPTY) {
      kp = rc > 0;
    } else if (rc > 0) {
      const int64_t mr = cfg.max_rows_per_privacy_id > 0 ? cfg.max_rows_per_privacy_id : 1;
      int64_t n = (rc + mr - 1) / mr;
      bool pre_ok = true;
      int64_t shift = 0;
      if (cfg.pre_threshold > 0) {
        if (n < cfg.pre_threshold) pre_ok = false;
        shift = cfg.pre_threshold - 1;
        n -= shift;
      }
      if (pre_ok) {
        const U4 r = philox_for(cfg.seed, cfg.partition_offset + p, 0x53454C00u);
        if (cfg.strategy == PDP_SELECT_TRUNCATED_GEOMETRIC) {
          const int64_t t = n < cfg.keep_table_len ? n : (int64_t)cfg.keep_table_len - 1;
          kp = u01(r.x, r.y) < cfg.keep_prob[t];
        } else {
          const double v = (double)n + (cfg.strategy == PDP_SELECT_GAUSSIAN_THRESHOLDING
                                            ? gaussian_noise(cfg.noise_scale, r)
                                            : laplace_noise(cfg.noise_scale, r));
          kp = v > cfg.threshold;
          if (kp) nz = v + (double)shift;
        }
      }
    }
    keep[p] = kp;
    if (noised) noised[p] = nz;
  }
}

constexpr int kCompactItems = 16;
constexpr int kCompactChunk = kBlock * kCompactItems;

__global__ void __launch_bounds__(kBlock) k_compact_count(const uint8_t* __restrict__ keep, int64_t n,
                                                          int64_t* __restrict__ block_counts) {
  __shared__ int64_t red[kBlock / 64];
  const int64_t base = (int64_t)blockIdx.x * kCompactChunk + (int64_t)threadIdx.x * kCompactItems;
  int c = 0;
#pragma unroll
  for (int t = 0; t < kCompactItems; ++t) {
    const int64_t i = base + t;
    c += (i < n && keep[i]) ? 1 : 0;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t s = 0;
    for (int w = 0; w < kBlock / 64; ++w) s += red[w];
    block_counts[blockIdx.x] = s;
  }
}

// exclusive scan of block_counts in place (single workgroup), total -> *out_count
__global__ void __launch_bounds__(kBlock) k_compact_scan(int64_t* block_counts, int64_t nb,
                                                         int64_t* out_count) {
  __shared__ int64_t part[kBlock];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < nb; base += kBlock) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < nb ? block_counts[i] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < kBlock; off <<= 1) {
      const int64_t t = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < nb) block_counts[i] = carry + part[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == kBlock - 1) carry += part[kBlock - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out_count = carry;
}

__global__ void __launch_bounds__(kBlock) k_compact_write(const uint8_t* __restrict__ keep, int64_t n,
                                                          const int64_t* __restrict__ block_offsets,
                                                          int64_t* __restrict__ out_index) {
  __shared__ int part[kBlock];
  const int64_t base = (int64_t)blockIdx.x * kCompactChunk + (int64_t)threadIdx.x * kCompactItems;
  int c = 0;
#pragma unroll
  for (int t = 0; t < kCompactItems; ++t) {
    const int64_t i = base + t;
    c += (i < n && keep[i]) ? 1 : 0;
  }
  part[threadIdx.x] = c;
  __syncthreads();
  for (int off = 1; off < kBlock; off <<= 1) {
    const int t = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += t;
    __syncthreads();
  }
  int64_t pos = block_offsets[blockIdx.x] + part[threadIdx.x] - c;
  for (int t = 0; t < kCompactItems; ++t) {
    const int64_t i = base + t;
    if (i < n && keep[i]) out_index[pos++] = i;
  }
}

struct OpsPack {
  pdp_metric_op op[PDP_MAX_OPS];
};

__device__ __forceinline__ void put(double* out, int64_t stride, int col, int64_t i, double v) {
  if (col >= 0) out[(int64_t)col * stride + i] = v;
}

__global__ void __launch_bounds__(kBlock) k_noise_metrics(OpsPack ops, int n_ops,
                                                          const int64_t* __restrict__ index,
                                                          int64_t n_kept, const int64_t* __restrict__ n_kept_dev,
                                                          int64_t partition_offset,
                                                          pdp_partition_accumulators acc, int sum_is_int,
                                                          const double* __restrict__ noised_count,
                                                          double* __restrict__ out, int64_t out_stride,
                                                          uint64_t seed) {
  int64_t n = n_kept;
  if (n_kept_dev != nullptr) {
    const int64_t d = *n_kept_dev;
    n = d < n ? d : n;
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t p = index[i];
    const int64_t g = partition_offset + p;
    for (int o = 0; o < n_ops; ++o) {
      const pdp_metric_op& op = ops.op[o];
      const uint32_t slot = (uint32_t)o << 4;
      switch (op.kind) {
        case PDP_OP_COUNT: {
          const double v = (double)acc.count[p] + draw_noise(op.noise_kind, op.scale[0], philox_for(seed, g, slot));
          put(out, out_stride, op.out_col[0], i, v);
          break;
        }
        case PDP_OP_SUM: {
          const double s = sum_is_int ? (double)((const long long*)acc.sum)[p] : ((const double*)acc.sum)[p];
          put(out, out_stride, op.out_col[0], i, s + draw_noise(op.noise_kind, op.scale[0], philox_for(seed, g, slot)));
          break;
        }
        case PDP_OP_PRIVACY_ID_COUNT: {
          const double v = (double)acc.privacy_id_count[p] +
                           draw_noise(op.noise_kind, op.scale[0], philox_for(seed, g, slot));
          put(out, out_stride, op.out_col[0], i, v);
          break;
        }
        case PDP_OP_MEAN: {
          const double dp_count = (double)acc.count[p] + draw_noise(op.noise_kind, op.scale[0], philox_for(seed, g, slot));
          const double denom = fmax(1.0, dp_count);
          const double dp_nsum = acc.normalized_sum[p] + draw_noise(op.noise_kind, op.scale[1], philox_for(seed, g, slot + 1));
          const double mean = op.middle + dp_nsum / denom;
          put(out, out_stride, op.out_col[0], i, mean);
          put(out, out_stride, op.out_col[1], i, dp_count);
          put(out, out_stride, op.out_col[2], i, mean * dp_count);
          break;
        }
        case PDP_OP_VARIANCE: {
          const double dp_count = (double)acc.count[p] + draw_noise(op.noise_kind, op.scale[0], philox_for(seed, g, slot));
          double dp_mean, dp_mean_sq;
          if (op.degenerate) {
            dp_mean = op.min_value;
            dp_mean_sq = op.sq_min_value;
          } else {
            const double denom = fmax(1.0, dp_count);
            dp_mean = (acc.normalized_sum[p] + draw_noise(op.noise_kind, op.scale[1], philox_for(seed, g, slot + 1))) / denom;
            dp_mean_sq = (acc.normalized_sum_sq[p] + draw_noise(op.noise_kind, op.scale[2], philox_for(seed, g, slot + 2))) / denom;
          }
          const double dp_var = dp_mean_sq - dp_mean * dp_mean;
          if (!op.degenerate) dp_mean += op.middle;
          put(out, out_stride, op.out_col[0], i, dp_var);
          put(out, out_stride, op.out_col[1], i, dp_count);
          put(out, out_stride, op.out_col[2], i, dp_mean * dp_count);
          put(out, out_stride, op.out_col[3], i, dp_mean);
          break;
        }
        case PDP_OP_THRESHOLDED_PID: {
          put(out, out_stride, op.out_col[0], i, noised_count[p]);
          break;
        }
        default:
          break;
      }
    }
  }
}

// ------------------------------------------------------------ helpers --
int pk_bits(int64_t P) {
  int b = 1;
  while (b < 63 && ((int64_t)1 << b) < P) ++b;
  return b;
}

unsigned grid_for(int64_t n, int64_t cap = 1 << 16) {
  int64_t g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

struct WsLayout {
  uint64_t err, sketch, cnt, rows, fsum, isum, nsum, nsum2, total;
};

uint64_t align256(uint64_t x) { return (x + 255) & ~(uint64_t)255; }

WsLayout layout_for(const pdp_bound_config* c) {
  WsLayout w{};
  const uint64_t slots = (uint64_t)c->n_privacy_ids * (uint64_t)c->l0;
  uint64_t off = 0;
  w.err = off; off = align256(off + 16);
  w.sketch = off; off = align256(off + slots * 8);
  w.cnt = off; off = align256(off + slots * 4);
  if (c->linf > 0) {
    w.rows = off; off = align256(off + slots * (uint64_t)c->linf * 8);
    w.fsum = w.isum = w.nsum = w.nsum2 = 0;
  } else {
    w.rows = 0;
    w.fsum = off; off = align256(off + slots * 8);  // also used as int64 (isum)
    w.isum = w.fsum;
    w.nsum = off; off = align256(off + slots * 8);
    w.nsum2 = off; off = align256(off + slots * 8);
  }
  w.total = off;
  return w;
}

int validate(const pdp_bound_config* c) {
  if (c == nullptr) return set_error(PDP_E_INVALID, "config is NULL");
  if (c->n_rows < 0 || c->n_rows >= ((int64_t)1 << 32))
    return set_error(PDP_E_INVALID, "n_rows must be in [0, 2^32)");
  if (c->n_privacy_ids < 1) return set_error(PDP_E_INVALID, "n_privacy_ids must be >= 1");
  if (c->n_partitions < 1 || c->n_partitions >= ((int64_t)1 << 32))
    return set_error(PDP_E_INVALID, "n_partitions must be in [1, 2^32)");
  if (c->l0 < 1 || c->l0 > PDP_MAX_L0) return set_error(PDP_E_UNSUPPORTED, "l0 out of supported range [1, 256]");
  if (c->linf < 0 || c->linf > PDP_MAX_LINF)
    return set_error(PDP_E_UNSUPPORTED, "linf out of supported range [0, 256]");
  if (c->value_kind < PDP_VALUE_NONE || c->value_kind > PDP_VALUE_I64)
    return set_error(PDP_E_INVALID, "bad value_kind");
  if (c->value_kind != PDP_VALUE_I64 && (c->flags & PDP_SUM_INT))
    return set_error(PDP_E_INVALID, "PDP_SUM_INT requires int64 values");
  return PDP_OK;
}

BoundParams make_params(const pdp_bound_config* c) {
  BoundParams bp;
  bp.n = c->n_rows;
  bp.U = c->n_privacy_ids;
  bp.P = c->n_partitions;
  bp.l0 = c->l0;
  bp.linf = c->linf;
  bp.pk_mask = (((uint64_t)1) << pk_bits(c->n_partitions)) - 1;
  bp.seed = c->seed;
  bp.row_seed = derive_row_seed(c->seed);
  bp.row_offset = c->row_offset;
  return bp;
}

template <int VK, bool KA>
void launch_rows(unsigned g, hipStream_t st, const BoundParams& bp, const pdp_bound_config* c,
                 const int64_t* pid, const int64_t* pk, const void* value, const uint8_t* allowed,
                 char* ws, const WsLayout& w) {
  hipLaunchKernelGGL((k_pair_rows<VK, KA>), dim3(g), dim3(kBlock), 0, st, bp, pid, pk, value, allowed,
                     (const unsigned long long*)(ws + w.sketch), (unsigned int*)(ws + w.cnt),
                     KA ? nullptr : (unsigned long long*)(ws + w.rows),
                     KA ? (double*)(ws + w.fsum) : nullptr, KA ? (long long*)(ws + w.isum) : nullptr,
                     KA ? (double*)(ws + w.nsum) : nullptr, KA ? (double*)(ws + w.nsum2) : nullptr,
                     c->min_value, c->max_value, c->middle, c->flags, (unsigned int*)(ws + w.err));
}

template <int VK, bool KA>
void launch_reduce(unsigned g, hipStream_t st, const BoundParams& bp, const pdp_bound_config* c,
                   const void* value, const char* ws, const WsLayout& w,
                   const pdp_partition_accumulators& acc) {
  hipLaunchKernelGGL((k_reduce_pairs<VK, KA>), dim3(g), dim3(kBlock), 0, st, bp, value,
                     (const unsigned long long*)(ws + w.sketch), (const unsigned int*)(ws + w.cnt),
                     KA ? nullptr : (const unsigned long long*)(ws + w.rows),
                     KA ? (const double*)(ws + w.fsum) : nullptr,
                     KA ? (const long long*)(ws + w.isum) : nullptr,
                     KA ? (const double*)(ws + w.nsum) : nullptr,
                     KA ? (const double*)(ws + w.nsum2) : nullptr, c->min_value, c->max_value,
                     c->middle, c->min_sum, c->max_sum, c->flags, acc);
}

}  // namespace

// ================================================================ C ABI ==
extern "C" {

int pdp_abi_version(void) { return PDP_ABI_VERSION; }

const char* pdp_last_error(void) { return g_last_error.c_str(); }

int pdp_bound_workspace_bytes(const pdp_bound_config* cfg, uint64_t* bytes) {
  const int rc = validate(cfg);
  if (rc != PDP_OK) return rc;
  if (bytes == nullptr) return set_error(PDP_E_INVALID, "bytes is NULL");
  *bytes = layout_for(cfg).total;
  return PDP_OK;
}

namespace {
int check_bound_args(const pdp_bound_config* cfg, const int64_t* privacy_id,
                     const int64_t* partition_key, const void* value, void* workspace,
                     uint64_t workspace_bytes, WsLayout* w, bool need_value) {
  int rc = validate(cfg);
  if (rc != PDP_OK) return rc;
  *w = layout_for(cfg);
  if (workspace == nullptr || workspace_bytes < w->total)
    return set_error(PDP_E_WORKSPACE, "workspace too small (see pdp_bound_workspace_bytes)");
  if (cfg->n_rows > 0 && (privacy_id == nullptr || partition_key == nullptr))
    return set_error(PDP_E_INVALID, "key columns are NULL");
  if (need_value && cfg->value_kind != PDP_VALUE_NONE && cfg->n_rows > 0 && value == nullptr)
    return set_error(PDP_E_INVALID, "value column is NULL");
  return PDP_OK;
}
}  // namespace

int pdp_bound_sketch(const pdp_bound_config* cfg, const int64_t* privacy_id,
                     const int64_t* partition_key, const uint8_t* pk_allowed, void* workspace,
                     uint64_t workspace_bytes, void* stream) {
  WsLayout w;
  int rc = check_bound_args(cfg, privacy_id, partition_key, nullptr, workspace, workspace_bytes, &w,
                            /*need_value=*/false);
  if (rc != PDP_OK) return rc;
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  const uint64_t slots = (uint64_t)cfg->n_privacy_ids * (uint64_t)cfg->l0;
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.err, 0, 16, st));
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.sketch, 0xFF, slots * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.cnt, 0, slots * 4, st));
  if (cfg->linf > 0) {
    PDP_HIP_CHECK(hipMemsetAsync(ws + w.rows, 0xFF, slots * (uint64_t)cfg->linf * 8, st));
  } else {
    PDP_HIP_CHECK(hipMemsetAsync(ws + w.fsum, 0, w.total - w.fsum, st));
  }
  if (cfg->n_rows == 0) return PDP_OK;
  const BoundParams bp = make_params(cfg);
  hipLaunchKernelGGL(k_pair_sketch, dim3(grid_for(cfg->n_rows)), dim3(kBlock), 0, st, bp, privacy_id,
                     partition_key, pk_allowed, (unsigned long long*)(ws + w.sketch),
                     (unsigned int*)(ws + w.err));
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

int pdp_bound_rows(const pdp_bound_config* cfg, const int64_t* privacy_id,
                   const int64_t* partition_key, const void* value, const uint8_t* pk_allowed,
                   void* workspace, uint64_t workspace_bytes, void* stream) {
  WsLayout w;
  int rc = check_bound_args(cfg, privacy_id, partition_key, value, workspace, workspace_bytes, &w,
                            /*need_value=*/true);
  if (rc != PDP_OK) return rc;
  if (cfg->n_rows == 0) return PDP_OK;
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  const BoundParams bp = make_params(cfg);
  const unsigned g = grid_for(cfg->n_rows);
  const bool keep_all = cfg->linf == 0;
  switch (cfg->value_kind) {
    case PDP_VALUE_NONE:
      if (keep_all) launch_rows<PDP_VALUE_NONE, true>(g, st, bp, cfg, privacy_id, partition_key, value, pk_allowed, ws, w);
      else launch_rows<PDP_VALUE_NONE, false>(g, st, bp, cfg, privacy_id, partition_key, value, pk_allowed, ws, w);
      break;
    case PDP_VALUE_F64:
      if (keep_all) launch_rows<PDP_VALUE_F64, true>(g, st, bp, cfg, privacy_id, partition_key, value, pk_allowed, ws, w);
      else launch_rows<PDP_VALUE_F64, false>(g, st, bp, cfg, privacy_id, partition_key, value, pk_allowed, ws, w);
      break;
    default:
      if (keep_all) launch_rows<PDP_VALUE_I64, true>(g, st, bp, cfg, privacy_id, partition_key, value, pk_allowed, ws, w);
      else launch_rows<PDP_VALUE_I64, false>(g, st, bp, cfg, privacy_id, partition_key, value, pk_allowed, ws, w);
      break;
  }
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

int pdp_bound_contributions(const pdp_bound_config* cfg, const int64_t* privacy_id,
                            const int64_t* partition_key, const void* value,
                            const uint8_t* pk_allowed, void* workspace, uint64_t workspace_bytes,
                            void* stream) {
  int rc = pdp_bound_sketch(cfg, privacy_id, partition_key, pk_allowed, workspace, workspace_bytes, stream);
  if (rc != PDP_OK) return rc;
  return pdp_bound_rows(cfg, privacy_id, partition_key, value, pk_allowed, workspace, workspace_bytes, stream);
}

int pdp_reduce_partitions(const pdp_bound_config* cfg, const void* value, const void* workspace,
                          uint64_t workspace_bytes, const pdp_partition_accumulators* acc,
                          void* stream) {
  int rc = validate(cfg);
  if (rc != PDP_OK) return rc;
  const WsLayout w = layout_for(cfg);
  if (workspace == nullptr || workspace_bytes < w.total)
    return set_error(PDP_E_WORKSPACE, "workspace too small (see pdp_bound_workspace_bytes)");
  if (acc == nullptr || acc->privacy_id_count == nullptr)
    return set_error(PDP_E_INVALID, "accumulators.privacy_id_count is required");
  if ((cfg->flags & (PDP_ACC_SUM | PDP_SUM_PER_PARTITION)) && acc->sum == nullptr)
    return set_error(PDP_E_INVALID, "accumulators.sum is required by flags");
  if ((cfg->flags & PDP_ACC_NSUM) && acc->normalized_sum == nullptr)
    return set_error(PDP_E_INVALID, "accumulators.normalized_sum is required by flags");
  if ((cfg->flags & PDP_ACC_NSUM2) && acc->normalized_sum_sq == nullptr)
    return set_error(PDP_E_INVALID, "accumulators.normalized_sum_sq is required by flags");
  if (cfg->value_kind == PDP_VALUE_NONE &&
      (cfg->flags & (PDP_ACC_SUM | PDP_ACC_NSUM | PDP_ACC_NSUM2 | PDP_SUM_PER_PARTITION)))
    return set_error(PDP_E_INVALID, "value sums requested without a value column");
  hipStream_t st = (hipStream_t)stream;
  const BoundParams bp = make_params(cfg);
  const unsigned g = grid_for((int64_t)cfg->n_privacy_ids * cfg->l0);
  const bool keep_all = cfg->linf == 0;
  const char* ws = (const char*)workspace;
  switch (cfg->value_kind) {
    case PDP_VALUE_NONE:
      if (keep_all) launch_reduce<PDP_VALUE_NONE, true>(g, st, bp, cfg, value, ws, w, *acc);
      else launch_reduce<PDP_VALUE_NONE, false>(g, st, bp, cfg, value, ws, w, *acc);
      break;
    case PDP_VALUE_F64:
      if (keep_all) launch_reduce<PDP_VALUE_F64, true>(g, st, bp, cfg, value, ws, w, *acc);
      else launch_reduce<PDP_VALUE_F64, false>(g, st, bp, cfg, value, ws, w, *acc);
      break;
    default:
      if (keep_all) launch_reduce<PDP_VALUE_I64, true>(g, st, bp, cfg, value, ws, w, *acc);
      else launch_reduce<PDP_VALUE_I64, false>(g, st, bp, cfg, value, ws, w, *acc);
      break;
  }
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

int pdp_select_partitions(const pdp_select_config* cfg, const int64_t* row_count, uint8_t* keep,
                          double* noised_count, void* stream) {
  if (cfg == nullptr || keep == nullptr) return set_error(PDP_E_INVALID, "NULL argument");
  if (cfg->n_partitions < 0) return set_error(PDP_E_INVALID, "n_partitions < 0");
  if (cfg->strategy < PDP_SELECT_ALL_NONEMPTY || cfg->strategy > PDP_SELECT_PUBLIC)
    return set_error(PDP_E_INVALID, "bad strategy");
  if (cfg->strategy == PDP_SELECT_PUBLIC && cfg->public_mask == nullptr)
    return set_error(PDP_E_INVALID, "public_mask is required");
  if (cfg->strategy == PDP_SELECT_TRUNCATED_GEOMETRIC && (cfg->keep_prob == nullptr || cfg->keep_table_len < 1))
    return set_error(PDP_E_INVALID, "keep_prob table is required");
  if (cfg->strategy != PDP_SELECT_PUBLIC && row_count == nullptr)
    return set_error(PDP_E_INVALID, "row_count is required");
  if (cfg->n_partitions == 0) return PDP_OK;
  hipLaunchKernelGGL(k_select, dim3(grid_for(cfg->n_partitions)), dim3(kBlock), 0, (hipStream_t)stream,
                     *cfg, row_count, keep, noised_count);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

int pdp_compact_workspace_bytes(int64_t n, uint64_t* bytes) {
  if (bytes == nullptr || n < 0) return set_error(PDP_E_INVALID, "bad argument");
  const int64_t nb = (n + kCompactChunk - 1) / kCompactChunk;
  *bytes = align256((uint64_t)(nb > 0 ? nb : 1) * 8);
  return PDP_OK;
}

int pdp_compact(const uint8_t* keep, int64_t n, int64_t* out_index, int64_t* out_count, void* workspace,
                uint64_t workspace_bytes, void* stream) {
  if (n < 0 || out_count == nullptr) return set_error(PDP_E_INVALID, "bad argument");
  uint64_t need = 0;
  pdp_compact_workspace_bytes(n, &need);
  if (workspace == nullptr || workspace_bytes < need) return set_error(PDP_E_WORKSPACE, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    PDP_HIP_CHECK(hipMemsetAsync(out_count, 0, 8, st));
    return PDP_OK;
  }
  if (keep == nullptr || out_index == nullptr) return set_error(PDP_E_INVALID, "NULL argument");
  const int64_t nb = (n + kCompactChunk - 1) / kCompactChunk;
  int64_t* bc = (int64_t*)workspace;
  hipLaunchKernelGGL(k_compact_count, dim3((unsigned)nb), dim3(kBlock), 0, st, keep, n, bc);
  PDP_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_compact_scan, dim3(1), dim3(kBlock), 0, st, bc, nb, out_count);
  PDP_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_compact_write, dim3((unsigned)nb), dim3(kBlock), 0, st, keep, n, bc, out_index);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

int pdp_noise_metrics(const pdp_metric_op* ops, int32_t n_ops, const int64_t* index, int64_t n_kept,
                      const int64_t* n_kept_dev, int64_t partition_offset,
                      const pdp_partition_accumulators* acc, int32_t sum_is_int,
                      const double* noised_count, double* out, int64_t out_stride, uint64_t seed,
                      void* stream) {
  if (ops == nullptr || n_ops < 0 || n_ops > PDP_MAX_OPS || acc == nullptr)
    return set_error(PDP_E_INVALID, "bad ops");
  if (n_kept < 0 || out_stride < n_kept) return set_error(PDP_E_INVALID, "bad n_kept / out_stride");
  if (n_kept == 0 || n_ops == 0) return PDP_OK;
  if (index == nullptr || out == nullptr) return set_error(PDP_E_INVALID, "NULL argument");
  OpsPack pack;
  memset(&pack, 0, sizeof(pack));
  for (int i = 0; i < n_ops; ++i) {
    const pdp_metric_op& o = ops[i];
    switch (o.kind) {
      case PDP_OP_COUNT:
        if (!acc->count) return set_error(PDP_E_INVALID, "COUNT needs accumulators.count");
        break;
      case PDP_OP_SUM:
        if (!acc->sum) return set_error(PDP_E_INVALID, "SUM needs accumulators.sum");
        break;
      case PDP_OP_PRIVACY_ID_COUNT:
        if (!acc->privacy_id_count) return set_error(PDP_E_INVALID, "needs privacy_id_count");
        break;
      case PDP_OP_MEAN:
        if (!acc->count || !acc->normalized_sum) return set_error(PDP_E_INVALID, "MEAN needs count, normalized_sum");
        break;
      case PDP_OP_VARIANCE:
        if (!acc->count || !acc->normalized_sum || !acc->normalized_sum_sq)
          return set_error(PDP_E_INVALID, "VARIANCE needs count, normalized sums");
        break;
      case PDP_OP_THRESHOLDED_PID:
        if (!noised_count) return set_error(PDP_E_INVALID, "THRESHOLDED_PID needs noised_count");
        break;
      default:
        return set_error(PDP_E_INVALID, "unknown op kind");
    }
    pack.op[i] = o;
  }
  hipLaunchKernelGGL(k_noise_metrics, dim3(grid_for(n_kept)), dim3(kBlock), 0, (hipStream_t)stream, pack,
                     n_ops, index, n_kept, n_kept_dev, partition_offset, *acc, sum_is_int, noised_count,
                     out, out_stride, seed);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

int pdp_bound_error_flags(const void* workspace, uint32_t* flags, void* stream) {
  if (workspace == nullptr || flags == nullptr) return set_error(PDP_E_INVALID, "NULL argument");
  hipStream_t st = (hipStream_t)stream;
  PDP_HIP_CHECK(hipMemcpyAsync(flags, workspace, 4, hipMemcpyDeviceToHost, st));
  PDP_HIP_CHECK(hipStreamSynchronize(st));
  return PDP_OK;
}

}  // extern "C"
