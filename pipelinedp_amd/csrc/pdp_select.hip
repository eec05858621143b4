// pdp_select.hip — partition selection, compaction and noisy metrics.
//
//   k_select          private partition selection (dp_engine.py:315-371 ->
//                     PyDP create_partition_strategy(...).should_keep,
//                     partition_selection.py:29-44); thresholding strategies
//                     also emit the noised privacy-unit count
//                     (PostAggregationThresholdingCombiner, combiners.py:328-382)
//   k_compact_*       ascending stream compaction of the kept partitions
//   k_noise_metrics   CompoundCombiner.compute_metrics (combiners.py:766-788)
//                     for Count/Sum/PrivacyIdCount/Mean/Variance children
#include <cmath>
#include <cstring>

#include "pdp_internal.h"

namespace pdp {

// host-side validation of one mechanism's parameters (pdp_noise_params)
int check_noise(const pdp_noise_params* np) {
  if (np == nullptr) return set_error(PDP_E_INVALID, "noise params are NULL");
  if (np->kind != PDP_NOISE_LAPLACE && np->kind != PDP_NOISE_GAUSSIAN) return set_error(PDP_E_INVALID, "bad noise kind");
  if (!(np->granularity >= 0.0) || !std::isfinite(np->granularity))
    return set_error(PDP_E_INVALID, "noise granularity must be finite and >= 0");
  if (!(np->scale >= 0.0) || !std::isfinite(np->scale))
    return set_error(PDP_E_INVALID, "noise scale must be finite and >= 0");
  if (np->granularity == 0.0) {  // no noise: only for a scale of exactly 0 (fail closed)
    if (np->scale != 0.0) return set_error(PDP_E_INVALID, "noise granularity 0 with a nonzero scale");
    return PDP_OK;
  }
  if (np->kind == PDP_NOISE_LAPLACE && !(np->lambda > 0.0 && std::isfinite(np->lambda)))
    return set_error(PDP_E_INVALID, "Laplace noise needs a finite lambda > 0");
  if (np->kind == PDP_NOISE_GAUSSIAN &&
      (np->step < 1 || np->step >= ((int64_t)1 << 32) || !(np->n > 1.0) || !(np->bound > 0.0) || !(np->coef > 0.0)))
    return set_error(PDP_E_INVALID, "Gaussian noise needs 1 <= step < 2^32, n > 1, bound > 0, coef > 0");
  return PDP_OK;
}

namespace {

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
        if (cfg.strategy == PDP_SELECT_TRUNCATED_GEOMETRIC) {
          const U4 r = philox_for(cfg.seed, cfg.partition_offset + p, 0x53454C00u);
          const int64_t t = n < cfg.keep_table_len ? n : (int64_t)cfg.keep_table_len - 1;
          kp = u01(r.x, r.y) < cfg.keep_prob[t];
        } else {  // PyDP Laplace/GaussianPartitionSelection: mechanism.AddNoise(n) > threshold
          const double v = secure_add_noise(cfg.noise, (double)n, cfg.seed, cfg.partition_offset + p, 0x53454C00u);
          kp = v > cfg.threshold;
          if (kp) nz = v + (double)shift;
        }
      }
    }
    keep[p] = kp;
    if (noised) noised[p] = nz;
  }
}

// Laplace / Gaussian thresholding with Gaussian noise: the rejection sampler
// takes ~16 attempts per sample (geometric), so a lane per partition leaves a
// wave waiting ~74 attempts for its slowest lane.  Here each loop trip is one
// attempt, and a lane whose sample was accepted takes the wave's next
// partition: every wave owns one contiguous chunk of partitions and hands
// them out in order (ballot + prefix count, no atomics), so its lanes stay
// busy until the chunk runs dry (a fixed grid stride left each lane its own
// ~20 partitions, and the wave the slowest lane's sum of attempts).  Same
// Philox blocks per partition as secure_add_noise, so the same draws.
__global__ void __launch_bounds__(kBlock) k_select_gauss(pdp_select_config cfg, const int64_t* __restrict__ row_count,
                                                         uint8_t* __restrict__ keep, double* __restrict__ noised) {
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ULL << lane) - 1;
  const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t chunk = (cfg.n_partitions + n_waves - 1) / n_waves;
  const int64_t c0 = wave * chunk < cfg.n_partitions ? wave * chunk : cfg.n_partitions;
  const int64_t c1 = c0 + chunk < cfg.n_partitions ? c0 + chunk : cfg.n_partitions;
  const double g = cfg.noise.granularity;
  const int64_t mr = cfg.max_rows_per_privacy_id > 0 ? cfg.max_rows_per_privacy_id : 1;
  // a fresh partition's set-up runs on some lane of nearly every trip, so it
  // avoids the int64 division (mr == 1) and the fmod (a power-of-two grid
  // <= 1 leaves an integer count where it is): both paths give the same value
  int g_exp = 0;
  const bool unit_grid = g > 0.0 && g <= 1.0 && frexp(g, &g_exp) == 0.5;
  int64_t p = c0 + lane;
  int64_t cursor = c0 + 64;  // wave-uniform: the chunk's next partition to hand out
  bool fresh = true;
  uint32_t k = 0;
  double base = 0.0, shift = 0.0;
  while (__ballot(p < c1) != 0) {  // wave-uniform trip count
    bool done = false;
    if (p < c1) {
      if (fresh) {
        fresh = false;
        k = 0;
        const int64_t rc = row_count[p];
        int64_t n = mr == 1 ? rc : (rc + mr - 1) / mr;  // mr: uniform
        bool live = rc > 0;
        int64_t sh = 0;
        if (live && cfg.pre_threshold > 0) {
          if (n < cfg.pre_threshold) live = false;
          sh = cfg.pre_threshold - 1;
          n -= sh;
        }
        if (!live) {
          keep[p] = 0;
          if (noised) noised[p] = __builtin_nan("");
          done = true;
        } else {
          base = unit_grid ? (double)n : round_to_multiple((double)n, g);
          shift = (double)sh;
        }
      }
      double md;
      if (!done && gaussian_attempt(cfg.noise, cfg.seed, cfg.partition_offset + p, 0x53454C00u, k, &md)) {
        const double v = base + md * g;
        const bool kp = v > cfg.threshold;
        keep[p] = kp;
        if (noised) noised[p] = kp ? v + shift : __builtin_nan("");
        done = true;
      }
    }
    const unsigned long long m = __ballot(done);
    if (done) {
      p = cursor + __popcll(m & below);
      fresh = true;
    }
    cursor += __popcll(m);
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


// DPEngine.add_dp_noise (dp_engine.py:551-607): y[i] = mechanism.add_noise(
// float(x[i])), the secure sampler reading the Philox streams (seed,
// index_offset + i).  One 16-byte load + one 16-byte store per thread step (2
// elements); the samplers' fp64 transcendentals, not HBM, set its rate.
constexpr uint32_t kAddNoiseSlot = 0x41444E00u;  // "ADN"

template <int VALUE_KIND>
__global__ void __launch_bounds__(kBlock) k_add_noise(const void* __restrict__ x, int64_t n,
                                                      pdp_noise_params np, uint64_t seed, int64_t index_offset,
                                                      double* __restrict__ y) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t pairs = n >> 1;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < pairs; t += stride) {
    const int64_t i = 2 * t;
    double a, b;
    if (VALUE_KIND == PDP_VALUE_I64) {
      const longlong2 v = reinterpret_cast<const longlong2*>(x)[t];
      a = (double)v.x;
      b = (double)v.y;
    } else {
      const double2 v = reinterpret_cast<const double2*>(x)[t];
      a = v.x;
      b = v.y;
    }
    double2 o;
    o.x = secure_add_noise(np, a, seed, index_offset + i, kAddNoiseSlot);
    o.y = secure_add_noise(np, b, seed, index_offset + i + 1, kAddNoiseSlot);
    reinterpret_cast<double2*>(y)[t] = o;
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t i = n - 1;
    const double a = VALUE_KIND == PDP_VALUE_I64 ? (double)((const long long*)x)[i] : ((const double*)x)[i];
    y[i] = secure_add_noise(np, a, seed, index_offset + i, kAddNoiseSlot);
  }
}

struct OpsPack {
  pdp_metric_op op[PDP_MAX_OPS];
};

__device__ __forceinline__ void put(double* out, int64_t stride, int col, int64_t i, double v) {
  if (col >= 0) out[(int64_t)col * stride + i] = v;
}

// mechanism draws of an op (each its own Philox stream (seed, partition, o << 4 | m))
__host__ __device__ inline int op_draws(int kind) {
  return kind == PDP_OP_MEAN ? 2 : (kind == PDP_OP_VARIANCE ? 3 : 1);  // THRESHOLDED_PID: a copy
}

// One lane per (kept partition, draw): a secure sample is a serial bisection
// of ~60 fp64 steps, so the draws of one partition run on G neighbouring lanes
// (G = draws per partition rounded up to a power of two) and the lane of each
// op's first draw combines the op's draws by __shfl and writes its columns.
// Same streams and arithmetic as one thread per partition.
__global__ void __launch_bounds__(kBlock) k_noise_metrics(OpsPack ops, int n_ops, int log2_g,
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
  const int G = 1 << log2_g;
  const int lane = (int)(threadIdx.x & 63);
  const int d = lane & (G - 1);
  // this lane's draw: op o, mechanism m (o < 0: a padding lane)
  int o = -1, m = 0;
  for (int q = 0, c = 0; q < n_ops; ++q) {
    const int k = op_draws(ops.op[q].kind);
    if (d >= c && d < c + k) {
      o = q;
      m = d - c;
    }
    c += k;
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;  // a multiple of 64: groups stay whole
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; (t >> log2_g) < n; t += stride) {
    const int64_t i = t >> log2_g;
    const int64_t p = index[i];
    const int64_t g = partition_offset + p;
    double v = 0.0;
    if (o >= 0) {
      const pdp_metric_op& op = ops.op[o];
      const uint32_t slot = ((uint32_t)o << 4) + (uint32_t)m;
      switch (op.kind) {
        case PDP_OP_COUNT:
          v = secure_add_noise(op.noise[0], (double)acc.count[p], seed, g, slot);
          break;
        case PDP_OP_SUM:
          v = secure_add_noise(op.noise[0],
                               sum_is_int ? (double)((const long long*)acc.sum)[p] : ((const double*)acc.sum)[p],
                               seed, g, slot);
          break;
        case PDP_OP_PRIVACY_ID_COUNT:
          v = secure_add_noise(op.noise[0], (double)acc.privacy_id_count[p], seed, g, slot);
          break;
        case PDP_OP_MEAN:
          v = secure_add_noise(op.noise[m], m == 0 ? (double)acc.count[p] : acc.normalized_sum[p], seed, g, slot);
          break;
        case PDP_OP_VARIANCE:
          if (m == 0) v = secure_add_noise(op.noise[0], (double)acc.count[p], seed, g, slot);
          else if (!op.degenerate)  // a degenerate variance draws the count only
            v = secure_add_noise(op.noise[m], m == 1 ? acc.normalized_sum[p] : acc.normalized_sum_sq[p], seed, g, slot);
          break;
        case PDP_OP_THRESHOLDED_PID:
          v = noised_count[p];
          break;
        default:
          break;
      }
    }
    // every lane takes part in the shuffles (the op's later draws sit on lanes + 1, + 2)
    const double v1 = __shfl(v, (lane + 1) & 63, 64);
    const double v2 = __shfl(v, (lane + 2) & 63, 64);
    if (o < 0 || m != 0) continue;
    const pdp_metric_op& op = ops.op[o];
    switch (op.kind) {
      case PDP_OP_COUNT:
      case PDP_OP_SUM:
      case PDP_OP_PRIVACY_ID_COUNT:
      case PDP_OP_THRESHOLDED_PID:
        put(out, out_stride, op.out_col[0], i, v);
        break;
      case PDP_OP_MEAN: {
        const double dp_count = v;
        const double mean = op.middle + v1 / fmax(1.0, dp_count);
        put(out, out_stride, op.out_col[0], i, mean);
        put(out, out_stride, op.out_col[1], i, dp_count);
        put(out, out_stride, op.out_col[2], i, mean * dp_count);
        break;
      }
      case PDP_OP_VARIANCE: {
        const double dp_count = v;
        double dp_mean, dp_mean_sq;
        if (op.degenerate) {
          dp_mean = op.min_value;
          dp_mean_sq = op.sq_min_value;
        } else {
          const double denom = fmax(1.0, dp_count);
          dp_mean = v1 / denom;
          dp_mean_sq = v2 / denom;
        }
        const double dp_var = dp_mean_sq - dp_mean * dp_mean;
        if (!op.degenerate) dp_mean += op.middle;
        put(out, out_stride, op.out_col[0], i, dp_var);
        put(out, out_stride, op.out_col[1], i, dp_count);
        put(out, out_stride, op.out_col[2], i, dp_mean * dp_count);
        put(out, out_stride, op.out_col[3], i, dp_mean);
        break;
      }
      default:
        break;
    }
  }
}

}  // namespace
}  // namespace pdp

using namespace pdp;

extern "C" {

int pdp_select_partitions(const pdp_select_config* cfg, const int64_t* row_count, uint8_t* keep,
                          double* noised_count, void* stream) {
  if (cfg == nullptr || keep == nullptr) return pdp::set_error(PDP_E_INVALID, "NULL argument");
  if (cfg->n_partitions < 0) return pdp::set_error(PDP_E_INVALID, "n_partitions < 0");
  if (cfg->strategy < PDP_SELECT_ALL_NONEMPTY || cfg->strategy > PDP_SELECT_PUBLIC)
    return pdp::set_error(PDP_E_INVALID, "bad strategy");
  if (cfg->strategy == PDP_SELECT_PUBLIC && cfg->public_mask == nullptr)
    return pdp::set_error(PDP_E_INVALID, "public_mask is required");
  if (cfg->strategy == PDP_SELECT_TRUNCATED_GEOMETRIC && (cfg->keep_prob == nullptr || cfg->keep_table_len < 1))
    return pdp::set_error(PDP_E_INVALID, "keep_prob table is required");
  if (cfg->strategy != PDP_SELECT_PUBLIC && row_count == nullptr)
    return pdp::set_error(PDP_E_INVALID, "row_count is required");
  if (cfg->strategy == PDP_SELECT_LAPLACE_THRESHOLDING || cfg->strategy == PDP_SELECT_GAUSSIAN_THRESHOLDING) {
    const int rc = pdp::check_noise(&cfg->noise);
    if (rc != PDP_OK) return rc;
  }
  if (cfg->n_partitions == 0) return PDP_OK;
  const bool gauss = (cfg->strategy == PDP_SELECT_LAPLACE_THRESHOLDING ||
                      cfg->strategy == PDP_SELECT_GAUSSIAN_THRESHOLDING) &&
                     cfg->noise.kind == PDP_NOISE_GAUSSIAN && cfg->noise.granularity != 0.0;
  PDP_PROF_BEGIN("k_select", (hipStream_t)stream);
  if (gauss)  // ~20 partitions per lane (a full chip: 2,048 workgroups of 4 waves)
    hipLaunchKernelGGL(k_select_gauss, dim3(grid_for(cfg->n_partitions, 2048)), dim3(kBlock), 0, (hipStream_t)stream,
                       *cfg, row_count, keep, noised_count);
  else
    hipLaunchKernelGGL(k_select, dim3(grid_for(cfg->n_partitions)), dim3(kBlock), 0, (hipStream_t)stream,
                       *cfg, row_count, keep, noised_count);
  PDP_PROF_END((hipStream_t)stream);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

int pdp_compact_workspace_bytes(int64_t n, uint64_t* bytes) {
  if (bytes == nullptr || n < 0) return pdp::set_error(PDP_E_INVALID, "bad argument");
  const int64_t nb = (n + kCompactChunk - 1) / kCompactChunk;
  *bytes = align256((uint64_t)(nb > 0 ? nb : 1) * 8);
  return PDP_OK;
}

int pdp_compact(const uint8_t* keep, int64_t n, int64_t* out_index, int64_t* out_count, void* workspace,
                uint64_t workspace_bytes, void* stream) {
  if (n < 0 || out_count == nullptr) return pdp::set_error(PDP_E_INVALID, "bad argument");
  uint64_t need = 0;
  pdp_compact_workspace_bytes(n, &need);
  if (workspace == nullptr || workspace_bytes < need) return pdp::set_error(PDP_E_WORKSPACE, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    PDP_HIP_CHECK(hipMemsetAsync(out_count, 0, 8, st));
    return PDP_OK;
  }
  if (keep == nullptr || out_index == nullptr) return pdp::set_error(PDP_E_INVALID, "NULL argument");
  const int64_t nb = (n + kCompactChunk - 1) / kCompactChunk;
  int64_t* bc = (int64_t*)workspace;
  PDP_PROF_BEGIN("k_compact_count", st);
  hipLaunchKernelGGL(k_compact_count, dim3((unsigned)nb), dim3(kBlock), 0, st, keep, n, bc);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  PDP_PROF_BEGIN("k_compact_scan", st);
  hipLaunchKernelGGL(k_compact_scan, dim3(1), dim3(kBlock), 0, st, bc, nb, out_count);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  PDP_PROF_BEGIN("k_compact_write", st);
  hipLaunchKernelGGL(k_compact_write, dim3((unsigned)nb), dim3(kBlock), 0, st, keep, n, bc, out_index);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

int pdp_noise_metrics(const pdp_metric_op* ops, int32_t n_ops, const int64_t* index, int64_t n_kept,
                      const int64_t* n_kept_dev, int64_t partition_offset,
                      const pdp_partition_accumulators* acc, int32_t sum_is_int,
                      const double* noised_count, double* out, int64_t out_stride, uint64_t seed,
                      void* stream) {
  if (ops == nullptr || n_ops < 0 || n_ops > PDP_MAX_OPS || acc == nullptr)
    return pdp::set_error(PDP_E_INVALID, "bad ops");
  if (n_kept < 0 || out_stride < n_kept) return pdp::set_error(PDP_E_INVALID, "bad n_kept / out_stride");
  if (n_kept == 0 || n_ops == 0) return PDP_OK;
  if (index == nullptr || out == nullptr) return pdp::set_error(PDP_E_INVALID, "NULL argument");
  OpsPack pack;
  memset(&pack, 0, sizeof(pack));
  for (int i = 0; i < n_ops; ++i) {
    const pdp_metric_op& o = ops[i];
    switch (o.kind) {
      case PDP_OP_COUNT:
        if (!acc->count) return pdp::set_error(PDP_E_INVALID, "COUNT needs accumulators.count");
        break;
      case PDP_OP_SUM:
        if (!acc->sum) return pdp::set_error(PDP_E_INVALID, "SUM needs accumulators.sum");
        break;
      case PDP_OP_PRIVACY_ID_COUNT:
        if (!acc->privacy_id_count) return pdp::set_error(PDP_E_INVALID, "needs privacy_id_count");
        break;
      case PDP_OP_MEAN:
        if (!acc->count || !acc->normalized_sum) return pdp::set_error(PDP_E_INVALID, "MEAN needs count, normalized_sum");
        break;
      case PDP_OP_VARIANCE:
        if (!acc->count || !acc->normalized_sum || !acc->normalized_sum_sq)
          return pdp::set_error(PDP_E_INVALID, "VARIANCE needs count, normalized sums");
        break;
      case PDP_OP_THRESHOLDED_PID:
        if (!noised_count) return pdp::set_error(PDP_E_INVALID, "THRESHOLDED_PID needs noised_count");
        break;
      default:
        return pdp::set_error(PDP_E_INVALID, "unknown op kind");
    }
    const int nmech = o.kind == PDP_OP_MEAN ? 2 : (o.kind == PDP_OP_VARIANCE ? 3 : (o.kind == PDP_OP_THRESHOLDED_PID ? 0 : 1));
    for (int m = 0; m < nmech; ++m) {
      const int rc = pdp::check_noise(&o.noise[m]);
      if (rc != PDP_OK) return rc;
    }
    pack.op[i] = o;
  }
  int draws = 0;
  for (int i = 0; i < n_ops; ++i) draws += op_draws(ops[i].kind);
  int log2_g = 0;
  while ((1 << log2_g) < draws) ++log2_g;  // <= 24 draws: groups of at most 32 lanes
  // n_kept is an upper bound when the count is on the device (n_kept_dev,
  // usually P): a grid-stride loop over at most 2,048 blocks, not one block per
  // 256 draws of every partition (C3: 7,813 mostly idle blocks, 34 us)
  const unsigned grid = grid_for(n_kept << log2_g) < 2048u ? grid_for(n_kept << log2_g) : 2048u;
  PDP_PROF_BEGIN("k_noise_metrics", (hipStream_t)stream);
  hipLaunchKernelGGL(k_noise_metrics, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, pack,
                     n_ops, log2_g, index, n_kept, n_kept_dev, partition_offset, *acc, sum_is_int, noised_count,
                     out, out_stride, seed);
  PDP_PROF_END((hipStream_t)stream);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

int pdp_add_noise(const void* values, int32_t value_kind, int64_t n, const pdp_noise_params* noise,
                  uint64_t seed, int64_t index_offset, double* out, void* stream) {
  if (n < 0) return pdp::set_error(PDP_E_INVALID, "n must be >= 0");
  if (value_kind != PDP_VALUE_F64 && value_kind != PDP_VALUE_I64)
    return pdp::set_error(PDP_E_INVALID, "value_kind must be PDP_VALUE_F64 or PDP_VALUE_I64");
  const int rc = pdp::check_noise(noise);
  if (rc != PDP_OK) return rc;
  if (n == 0) return PDP_OK;
  if (values == nullptr || out == nullptr) return pdp::set_error(PDP_E_INVALID, "NULL argument");
  if (((uintptr_t)values | (uintptr_t)out) & 15)
    return pdp::set_error(PDP_E_INVALID, "values and out must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  const int64_t pairs = (n + 1) >> 1;
  PDP_PROF_BEGIN("k_add_noise", st);
  if (value_kind == PDP_VALUE_I64)
    hipLaunchKernelGGL(k_add_noise<PDP_VALUE_I64>, dim3(grid_for(pairs)), dim3(kBlock), 0, st, values, n,
                       *noise, seed, index_offset, out);
  else
    hipLaunchKernelGGL(k_add_noise<PDP_VALUE_F64>, dim3(grid_for(pairs)), dim3(kBlock), 0, st, values, n,
                       *noise, seed, index_offset, out);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

}  // extern "C"
