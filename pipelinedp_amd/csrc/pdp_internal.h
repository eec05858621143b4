// pdp_internal.h — device helpers shared by the gfx950 kernels of the
// DPEngine.aggregate hot path (hashing, Philox, noise, sorted sketches).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <string>

#include "../../include/pipelinedp_amd.h"

namespace pdp {

// ------------------------------------------------------------ errors (host) --
int set_error(int code, const char* msg);

#define PDP_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) {                                                        \
      char buf_[256];                                                              \
      snprintf(buf_, sizeof(buf_), "%s failed: %s", #expr, hipGetErrorString(e_)); \
      return ::pdp::set_error(PDP_E_HIP, buf_);                                    \
    }                                                                              \
  } while (0)

constexpr uint64_t kEmpty = ~0ULL;
constexpr int kBlock = 256;

inline unsigned grid_for(int64_t n, int64_t cap = 1 << 16) {
  int64_t g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

inline uint64_t align256(uint64_t x) { return (x + 255) & ~(uint64_t)255; }

// Non-temporal ("streaming") loads of data a kernel reads exactly once: the
// lines are not kept in L2, which then holds the kernel's partially written
// output lines until they are whole (k_sieve_l1: C2 level 1 0.385 -> 0.349
// ms, profiles/r05/ab/ab4_fix_list_nt_loads.txt)
__device__ __forceinline__ longlong2 ld_nt(const longlong2* p) {
  typedef long long v2 __attribute__((ext_vector_type(2)));
  const v2 v = __builtin_nontemporal_load(reinterpret_cast<const v2*>(p));
  return make_longlong2(v.x, v.y);
}
__device__ __forceinline__ ulonglong2 ld_nt(const ulonglong2* p) {
  typedef unsigned long long v2 __attribute__((ext_vector_type(2)));
  const v2 v = __builtin_nontemporal_load(reinterpret_cast<const v2*>(p));
  return make_ulonglong2(v.x, v.y);
}
__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
  typedef unsigned v4 __attribute__((ext_vector_type(4)));
  const v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ld_nt(const uint2* p) {
  typedef unsigned v2 __attribute__((ext_vector_type(2)));
  const v2 v = __builtin_nontemporal_load(reinterpret_cast<const v2*>(p));
  return make_uint2(v.x, v.y);
}
template <typename T>
__device__ __forceinline__ T ld_nt(const T* p) {
  return __builtin_nontemporal_load(p);
}
// a load that is non-temporal when NT is set (a compile-time choice per site)
template <bool NT, typename T>
__device__ __forceinline__ T ld_maybe_nt(const T* p) {
  if constexpr (NT) return ld_nt(p);
  else return *p;
}

inline int bits_for(int64_t n) {  // smallest b >= 1 with 2^b >= n
  int b = 1;
  while (b < 63 && ((int64_t)1 << b) < n) ++b;
  return b;
}

// ---------------------------------------------------------------- hashing --
// SplitMix64 finaliser: a bijective 64-bit mixer; keyed by the seed it is a
// counter-based generator for sampling priorities.
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// MurmurHash3 32-bit finaliser
__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6BU;
  h ^= h >> 13;
  h *= 0xC2B2AE35U;
  return h ^ (h >> 16);
}

// 32 random bits of the pair (pid, pk) under `seed`: a per-pid word (the id
// keyed by the seed's low half, one odd multiply: a bijection of the id's low
// 32 bits), then the partition folded in as an odd-multiplier progression and
// the MurmurHash3 finaliser, which mixes both.  Within one pid distinct
// partitions (< 2^32) give distinct finaliser inputs, so they never tie.
// Four 32-bit multiplies per row (quarter rate on gfx950): the level-1 sieve
// hashes every row.
__host__ __device__ __forceinline__ uint32_t pid_hash(uint64_t seed, int64_t pid) {
  const uint32_t hi = (uint32_t)((uint64_t)pid >> 32);
  return ((uint32_t)pid ^ ((hi << 16) | (hi >> 16)) ^ (uint32_t)seed) * 0x9E3779B1U;
}

__host__ __device__ __forceinline__ uint32_t pair_hash_from(uint32_t hpid, uint64_t seed, int64_t pk) {
  return fmix32(hpid ^ ((uint32_t)pk * 0xC2B2AE3DU + (uint32_t)(seed >> 32)));
}

__host__ __device__ __forceinline__ uint32_t pair_hash(uint64_t seed, int64_t pid, int64_t pk) {
  return pair_hash_from(pid_hash(seed, pid), seed, pk);
}

// pair_key (below) with the pid's hash already computed (pid_hash)
__host__ __device__ __forceinline__ uint64_t pair_key_from(uint32_t hpid, uint64_t seed, int64_t pk,
                                                           uint64_t mid_bits, int rand_shift) {
  const uint64_t h = (uint64_t)pair_hash_from(hpid, seed, pk) << 32;
  const uint64_t low = (1ULL << rand_shift) - 1;
  uint64_t x = (h & ~low) | mid_bits | (uint64_t)pk;
  if ((x | low) == ~0ULL) x &= ~(1ULL << rand_shift);
  return x;
}

// Sampling key of the pair (pid, pk): bits [rand_shift, 64) are random (the
// pair hash from bit 32 up, zero below), bits [pk_bits, rand_shift) carry
// `mid` (the bucket-local pid, or 0) and bits [0, pk_bits) the partition.
// Within one privacy id keys order by (random part, partition) whatever `mid`
// is, so every execution path samples the same pairs.  Never equal to kEmpty.
__host__ __device__ __forceinline__ uint64_t pair_key(uint64_t seed, int64_t pid, int64_t pk,
                                                      uint64_t mid_bits, int rand_shift) {
  return pair_key_from(pid_hash(seed, pid), seed, pk, mid_bits, rand_shift);
}

__host__ __device__ __forceinline__ uint64_t derive_row_seed(uint64_t seed) {
  return mix64(seed ^ 0x5851F42D4C957F2DULL);
}

// Sampling key of row `local_row` (global index global_row): 32 random bits,
// then the local row index (unique, < 2^32, never kEmpty).
__device__ __forceinline__ uint64_t row_key(uint64_t row_seed, int64_t global_row, uint32_t local_row) {
  const uint64_t h = mix64(row_seed ^ ((uint64_t)global_row * 0xD6E8FEB86659FD93ULL));
  return (h & 0xFFFFFFFF00000000ULL) | (uint64_t)local_row;
}

// ---------------------------------------------------------------- philox --
struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
  // each 32 x 32 -> 64 product as one v_mad_u64_u32 (one quarter-rate
  // instruction for both halves, not a v_mul_lo_u32 + v_mul_hi_u32 pair)
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// uniform double in (0, 1): 53-bit grid, open interval
__device__ __forceinline__ double u01(uint32_t hi, uint32_t lo) {
  const uint64_t x = (((uint64_t)hi << 32) | lo) >> 11;
  return ((double)x + 0.5) * (1.0 / 9007199254740992.0);
}

// counter = (global partition index, mechanism slot, "PDP!")
__device__ __forceinline__ U4 philox_for(uint64_t seed, int64_t gidx, uint32_t slot) {
  U4 c{(uint32_t)((uint64_t)gidx), (uint32_t)((uint64_t)gidx >> 32), slot, 0x50445021u};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// ------------------------------------------------------- secure noise --
// Granularity-snapped samplers of Google's differential-privacy library
// (what PyDP's numerical_mechanisms call; restated from its published
// algorithm, see pdp_noise_params in pipelinedp_amd.h).  Every draw reads the
// Philox blocks k = 0, 1, ... of the stream (seed, gidx, slot); the oracle
// (oracle/columnar.py secure_noise) consumes them in the same order.
__device__ __forceinline__ U4 noise_block(uint64_t seed, int64_t gidx, uint32_t slot, uint32_t k) {
  U4 c{(uint32_t)((uint64_t)gidx), (uint32_t)((uint64_t)gidx >> 32), slot, 0x4E000000u + k};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// RoundToNearestDoubleMultiple: exact for a power-of-two base; ties go toward
// zero (|remainder| == base / 2 keeps n - remainder)
__device__ __forceinline__ double round_to_multiple(double x, double base) {
  if (base == 0.0) return x;
  const double r = fmod(x, base);
  if (fabs(r) > base / 2) return x - r + copysign(base, r);
  return x - r;
}

// Geometric sample P(X = j) = (1 - e^-lambda) e^(-lambda j), j >= 0: bisection
// of (lo, hi] over the integers; each step keeps the lower half with its exact
// conditional mass q = expm1(-lambda (mid - lo)) / expm1(-lambda (hi - lo)).
// Steps with q == 1 (the far tail has no mass at fp64) draw nothing; the
// others each read one uniform (two per Philox block).
__device__ __forceinline__ int64_t secure_geometric(double lambda, uint64_t seed, int64_t gidx, uint32_t slot,
                                                    uint32_t& k) {
  int64_t lo = 0, hi = INT64_MAX;
  // The far tail, without an expm1: while lambda (mid - lo) >= 40 both
  // expm1 terms round to exactly -1 (e^-40 < 2^-54), so q == 1 and the step
  // only halves hi -- the (lo, hi) sequence of the loop below, bit for bit
  // (C3's Laplace draws skip ~20 of their ~60 steps here)
  while (lo + 1 < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (!(lambda * (double)(lo - mid) <= -40.0)) break;
    hi = mid;
  }
  U4 blk{0, 0, 0, 0};
  int half = 0;  // 0: next uniform from a fresh block's (x, y); 1: from (z, w)
  // den = expm1(lambda (lo - hi)) of the current (lo, hi): after hi = mid it
  // is the step's numerator (same expression), so only lo = mid recomputes it
  double den = expm1(lambda * (double)(lo - hi));
  while (lo + 1 < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    const double num = expm1(lambda * (double)(lo - mid));
    const double q = num / den;
    if (q >= 1.0) {
      hi = mid;
      den = num;
      continue;
    }
    double u;
    if (half == 0) {
      blk = noise_block(seed, gidx, slot, k++);
      u = u01(blk.x, blk.y);
    } else {
      u = u01(blk.z, blk.w);
    }
    half ^= 1;
    if (u <= q) {
      hi = mid;
      den = num;
    } else {
      lo = mid;
      den = lo + 1 < hi ? expm1(lambda * (double)(lo - hi)) : den;
    }
  }
  return hi - 1;
}

// LaplaceDistribution::Sample: g * two-sided geometric (a zero with a
// negative sign is redrawn, so 0 is not counted twice)
__device__ __forceinline__ double secure_laplace(const pdp_noise_params& np, uint64_t seed, int64_t gidx,
                                                 uint32_t slot) {
  uint32_t k = 0;
  for (;;) {
    const U4 a = noise_block(seed, gidx, slot, k++);
    const bool positive = (a.x >> 31) != 0;
    const int64_t s = secure_geometric(np.lambda, seed, gidx, slot, k);
    if (s == 0 && !positive) continue;
    return (positive ? (double)s : -(double)s) * np.granularity;
  }
}

// GaussianDistribution::Sample: g * (Binomial(n, 1/2) - n/2) by rejection from
// a two-sided geometric(1/2) over blocks of `step` integers; acceptance
// uses Google's approximate binomial probability (Secure Noise Generation,
// Lemma 7).  ONE Philox block per attempt (k advances by 1), its 128 bits
// split as: x[31:24] geometric bits (leading ones; eight ones = geometric 8),
// x[23] sign, (y, z) the 64 bits of the uniform offset in [0, step), and
// (w, x[20:0]) the 53 bits of the acceptance uniform.  Eight geometric bits
// suffice: every proposal with geometric >= 4 lies beyond `bound` (bound /
// step = sqrt(ln n) / 2 < 3.4 for any n < 2^64) and is rejected, so lumping
// geometric >= 8 into 8 leaves the accepted distribution unchanged.  Returns
// true and *md = the binomial offset if accepted.  About 1 in 16 attempts is
// accepted, so a kernel drawing many samples runs attempts, not samples, per
// loop trip (k_select_gauss) to keep a wave's lanes busy.  The Philox block is
// ~3/4 of an attempt's instructions (20 v_mad_u64_u32 at quarter rate).
__device__ __forceinline__ bool gaussian_attempt(const pdp_noise_params& np, uint64_t seed, int64_t gidx,
                                                 uint32_t slot, uint32_t& k, double* md_out) {
  const uint64_t step = (uint64_t)np.step;
  const U4 a = noise_block(seed, gidx, slot, k++);
  const int geom = __clz((~a.x & 0xFF000000u) | 0x00800000u);  // leading ones of x[31:24], at most 8
  const int64_t two_sided = ((a.x >> 23) & 1u) ? (int64_t)geom : -(int64_t)geom - 1;
  // floor(r * step / 2^64) for the 64 random bits r = (y, z); step < 2^32
  const uint64_t hi_part = (uint64_t)a.y * step + (((uint64_t)a.z * step) >> 32);
  const int64_t uni = (int64_t)(hi_part >> 32);
  const int64_t m = (int64_t)step * two_sided + uni;
  const uint64_t u53 = ((uint64_t)a.w << 21) | (a.x & 0x1FFFFFu);
  const double accept_u = ((double)u53 + 0.5) * (1.0 / 9007199254740992.0);
  const double md = (double)m;
  *md_out = md;
  if (fabs(md) > np.bound) return false;
  // squeeze: the fp32 threshold is within 1e-4 (relative) of the fp64 one
  // below (|md| <= bound keeps 2 md^2 / n <= ln n < 45, so fp32's ~1e-7
  // relative errors on md, 1/n and the exponent cost at most ~2e-5); only an
  // acceptance uniform within 1e-3 of it takes the exact fp64 test, so the
  // decision is the exact test's and a wave rarely pays the fp64 exp and
  // division
  {
    const float mf = (float)md;
    const float xf = 2.0f * mf * mf * __frcp_rn((float)np.n);
    const float tf = (float)(np.coef * np.corr * (double)np.step * 0.25) * __expf(-xf) * (float)(1u << geom);
    if (accept_u < (double)tf * (1.0 - 1e-3)) return true;
    if (accept_u >= (double)tf * (1.0 + 1e-3)) return false;
  }
  const double prob = np.coef * exp(-2.0 * md * md / np.n) * np.corr;
  return prob > 0.0 && accept_u < prob * (double)np.step * ldexp(1.0, geom) / 4.0;
}

__device__ __forceinline__ double secure_gaussian(const pdp_noise_params& np, uint64_t seed, int64_t gidx,
                                                  uint32_t slot) {
  uint32_t k = 0;
  double md;
  while (!gaussian_attempt(np, seed, gidx, slot, k, &md)) {
  }
  return md * np.granularity;
}

// mechanism.add_noise(x): x snapped to the grid plus a grid-valued sample
__device__ __forceinline__ double secure_add_noise(const pdp_noise_params& np, double x, uint64_t seed,
                                                   int64_t gidx, uint32_t slot) {
  if (np.granularity == 0.0) return x;
  const double noise = np.kind == PDP_NOISE_GAUSSIAN ? secure_gaussian(np, seed, gidx, slot)
                                                     : secure_laplace(np, seed, gidx, slot);
  return round_to_multiple(x, np.granularity) + noise;
}

// ------------------------------------------------- sorted-sketch insertion --
// Keep in the ascending array s[0..k) the k smallest DISTINCT keys ever
// inserted (kEmpty = free).  Lock-free: each atomicMin keeps the array
// sorted and hands the displaced key to the next slot; meeting an equal key
// means it is already present.  Works on LDS and global pointers.
// Sorted bottom-k sketches of u64 keys (kEmpty = free), lock-free under
// concurrent inserts: the array stays sorted and every position only ever
// decreases.  Insert x (no-op if present or not among the k smallest) by an
// atomicMin cascade carrying the displaced key one position up.
__device__ __forceinline__ void sketch_insert(unsigned long long* s, int k, uint64_t x) {
  for (int j = 0; j < k; ++j) {
    const uint64_t old = atomicMin(s + j, (unsigned long long)x);
    if (old == x) return;
    if (old > x) {
      if (old == kEmpty) return;
      x = old;
    }
  }
}

// The same on a sketch whose entries are `stride` apart (structure-of-arrays
// LDS layout: entry j of sketch p at s[j * stride + p], so that the lanes of a
// wave touching different sketches hit different LDS banks).
__device__ __forceinline__ void sketch_insert_strided(unsigned long long* s, int k, int64_t stride, uint64_t x) {
  for (int j = 0; j < k; ++j) {
    const uint64_t old = atomicMin(s + j * stride, (unsigned long long)x);
    if (old == x) return;
    if (old > x) {
      if (old == kEmpty) return;
      x = old;
    }
  }
}

__device__ __forceinline__ int sketch_find_strided(const unsigned long long* s, int k, int64_t stride, uint64_t x) {
  int lo = 0, hi = k;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (s[mid * stride] < x) lo = mid + 1; else hi = mid;
  }
  return (lo < k && s[lo * stride] == x) ? lo : -1;
}

// Position of x in a quiescent sorted sketch, or -1.
__device__ __forceinline__ int sketch_find(const unsigned long long* s, int k, uint64_t x) {
  int lo = 0, hi = k;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (s[mid] < x) lo = mid + 1; else hi = mid;
  }
  return (lo < k && s[lo] == x) ? lo : -1;
}

// ------------------------------------------------ per-pair accumulation --
struct PairSums {
  long long count;
  long long isum;
  double fsum, nsum, nsum2;
};

template <int VALUE_KIND>
__device__ __forceinline__ void load_value(const void* value, uint32_t row, double* v, long long* iv) {
  if (VALUE_KIND == PDP_VALUE_I64) {
    *iv = ((const long long*)value)[row];
    *v = (double)*iv;
  } else {
    *iv = 0;
    *v = ((const double*)value)[row];
  }
}

__device__ __forceinline__ long long clamp_ll(long long v, long long lo, long long hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}

struct ClipParams {
  double lo, hi, mid, min_sum, max_sum;
  int flags;
};

// CompoundCombiner.create_accumulator on the sampled rows of one pair
// (combiners.py:749-753 with the Count/Sum/Mean/Variance children).
template <int VALUE_KIND>
__device__ __forceinline__ PairSums pair_sums_from_rows(const unsigned long long* rows, long long m,
                                                        const void* value, const ClipParams& cp,
                                                        int64_t stride = 1) {
  PairSums s{m, 0, 0.0, 0.0, 0.0};
  if (VALUE_KIND == PDP_VALUE_NONE) return s;
  double raw = 0.0;
  long long iraw = 0;
  for (long long t = 0; t < m; ++t) {
    double v;
    long long iv;
    if (value != nullptr) {
      load_value<VALUE_KIND>(value, (uint32_t)rows[t * stride], &v, &iv);
    } else {  // rows[] already holds the values' bits (bucket kernel B2.5)
      iv = (long long)rows[t * stride];
      v = VALUE_KIND == PDP_VALUE_I64 ? (double)iv : __longlong_as_double(iv);
    }
    const double cv = fmin(fmax(v, cp.lo), cp.hi);
    if (cp.flags & PDP_SUM_PER_PARTITION) {
      raw += v;
      iraw += iv;
    } else if (cp.flags & PDP_SUM_INT) {
      s.isum += clamp_ll(iv, (long long)cp.lo, (long long)cp.hi);
    } else {
      s.fsum += cv;
    }
    const double nc = cv - cp.mid;
    s.nsum += nc;
    s.nsum2 += nc * nc;
  }
  if (cp.flags & PDP_SUM_PER_PARTITION) {
    if (cp.flags & PDP_SUM_INT) s.isum = clamp_ll(iraw, (long long)cp.min_sum, (long long)cp.max_sum);
    else s.fsum = fmin(fmax(raw, cp.min_sum), cp.max_sum);
  }
  return s;
}

// Adds row `row`'s contribution to the running per-pair sums f0 (clipped or,
// with PDP_SUM_PER_PARTITION, raw sum; int64 bits with PDP_SUM_INT), f1
// (normalized sum), f2 (normalized sum of squares) with device atomics — the
// keep-every-row form of create_accumulator, finished by pair_sums_from_totals.
template <int VALUE_KIND>
__device__ __forceinline__ void accumulate_row(const void* value, uint32_t row, int64_t slot, double* f0,
                                               double* f1, double* f2, const ClipParams& cp) {
  if (VALUE_KIND == PDP_VALUE_NONE) return;
  double v;
  long long iv;
  load_value<VALUE_KIND>(value, row, &v, &iv);
  const int flags = cp.flags;
  if (flags & PDP_SUM_PER_PARTITION) {
    if (flags & PDP_SUM_INT) atomicAdd((unsigned long long*)(f0 + slot), (unsigned long long)iv);
    else unsafeAtomicAdd(f0 + slot, v);
  } else if (flags & PDP_ACC_SUM) {
    if (flags & PDP_SUM_INT)
      atomicAdd((unsigned long long*)(f0 + slot), (unsigned long long)clamp_ll(iv, (long long)cp.lo, (long long)cp.hi));
    else unsafeAtomicAdd(f0 + slot, fmin(fmax(v, cp.lo), cp.hi));
  }
  if (flags & (PDP_ACC_NSUM | PDP_ACC_NSUM2)) {
    const double c = fmin(fmax(v, cp.lo), cp.hi) - cp.mid;
    if (flags & PDP_ACC_NSUM) unsafeAtomicAdd(f1 + slot, c);
    if (flags & PDP_ACC_NSUM2) unsafeAtomicAdd(f2 + slot, c * c);
  }
}

// pair accumulator of a keep-every-row pair from its summed slots
__device__ __forceinline__ PairSums pair_sums_from_totals(long long cnt, double fsum_or_bits, double nsum,
                                                          double nsum2, const ClipParams& cp) {
  PairSums s{cnt, 0, 0.0, nsum, nsum2};
  const long long ibits = __double_as_longlong(fsum_or_bits);
  if (cp.flags & PDP_SUM_PER_PARTITION) {
    if (cp.flags & PDP_SUM_INT) s.isum = clamp_ll(ibits, (long long)cp.min_sum, (long long)cp.max_sum);
    else s.fsum = fmin(fmax(fsum_or_bits, cp.min_sum), cp.max_sum);
  } else if (cp.flags & PDP_SUM_INT) {
    s.isum = ibits;
  } else {
    s.fsum = fsum_or_bits;
  }
  return s;
}

// merge one pair's accumulator into the partition accumulators
__device__ __forceinline__ void add_pair_to_partition(const pdp_partition_accumulators& acc, int64_t p,
                                                      const PairSums& s, int flags) {
  atomicAdd((unsigned long long*)(acc.privacy_id_count + p), 1ULL);
  if (acc.count) atomicAdd((unsigned long long*)(acc.count + p), (unsigned long long)s.count);
  if (acc.sum && (flags & (PDP_ACC_SUM | PDP_SUM_PER_PARTITION))) {
    if (flags & PDP_SUM_INT) atomicAdd((unsigned long long*)acc.sum + p, (unsigned long long)s.isum);
    else unsafeAtomicAdd((double*)acc.sum + p, s.fsum);
  }
  if (acc.normalized_sum && (flags & PDP_ACC_NSUM)) unsafeAtomicAdd(acc.normalized_sum + p, s.nsum);
  if (acc.normalized_sum_sq && (flags & PDP_ACC_NSUM2)) unsafeAtomicAdd(acc.normalized_sum_sq + p, s.nsum2);
}

// ------------------------------------------- host helpers across files --
// Device-wide exclusive scan of v[0..n) in place, total -> v[n] (u32; every
// caller's totals are < 2^32).  chunk_sums needs scan_chunk_sums_len(n) words.
int64_t scan_chunk_sums_len(int64_t n);
int scan_u32(unsigned* v, int64_t n, unsigned* chunk_sums, hipStream_t st);

// Pair-table path (pdp_pairs.hip): LinfSampler / NoOpSampler (l0 == 0),
// SamplingPerPrivacyIdContributionBounder (max_contributions > 0) and
// contribution_bounds_already_enforced (rows_are_units).
// Bounds above this go to the pair-table path, where a cap beyond it selects
// by radix select instead of an atomicMin-cascade sketch (pdp_pairs.hip).
#define PDP_SKETCH_MAX 256

inline bool pairs_mode(const pdp_bound_config* c) {
  return c->l0 == 0 || c->max_contributions > 0 || c->rows_are_units != 0 || c->l0 > PDP_SKETCH_MAX ||
         c->linf > PDP_SKETCH_MAX || c->algorithm == PDP_ALGO_PAIR_TABLE;
}
int pairs_validate(const pdp_bound_config* c);
uint64_t pairs_workspace_bytes(const pdp_bound_config* c);
int pairs_bound(const pdp_bound_config* c, const int64_t* pid, const int64_t* pk, const void* value,
                const uint8_t* allowed, char* ws, hipStream_t st);
int pairs_reduce(const pdp_bound_config* c, const void* value, char* ws, const pdp_partition_accumulators& acc,
                 hipStream_t st);

}  // namespace pdp

// ------------------------------------------------------------ profiler --
// Optional per-launch HIP-event timing (pdp_profiler_enable / _report):
// PDP_PROF_BEGIN/END bracket a launch on its own stream; disabled = no-op.
namespace pdp {
bool profiler_enabled();
void profiler_begin(const char* name, hipStream_t stream);
void profiler_end(hipStream_t stream);
}  // namespace pdp

#define PDP_PROF_BEGIN(name, stream) \
  do { if (::pdp::profiler_enabled()) ::pdp::profiler_begin(name, stream); } while (0)
#define PDP_PROF_END(stream) \
  do { if (::pdp::profiler_enabled()) ::pdp::profiler_end(stream); } while (0)
