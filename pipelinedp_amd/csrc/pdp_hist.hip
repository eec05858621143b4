// pdp_hist.hip — dataset histograms (gfx950): the contribution and partition
// statistics of pipeline_dp/dataset_histograms/computing_histograms.py
// (compute_dataset_histograms, :456-513) over one shard of dense columns.
//
// The reference builds seven histograms with five group-bys and a distinct
// (count_per_element / sum_per_key over pids, pairs and partitions).  Here the
// dense codes turn every group-by but the (pid, pk) one into direct indexing:
//   k_h_region_count, k_h_region_caps, scan
//               rows per partition-range region (4,096 partitions each) ->
//               region slot bases (1.5 slots per row + 64)
//   k_h_rows    per row: (pid, pk) into an open-addressing pair table (HBM,
//               linear probing inside the row's region) whose 32-byte slots
//               hold key, value sum and rows - 1, so a row's CAS and atomics
//               touch one cache line and the creating row skips the count
//   k_h_pairs   per live pair: one packed 64-bit atomic per pid (distinct
//               partitions << 32 | rows: L0, L1); per partition (distinct pids
//               << 32 | rows, value sum) summed in LDS over the region and
//               flushed with contiguous atomics; the Linf histogram, min/max
//               of the pair sums
//   k_h_ids     per pid: L0 / L1 histograms; per partition: count and
//               privacy-id-count histograms, min/max of the partition sums
//   k_h_lowers  np.linspace(min, max, 10001) bin lowers (_min_max_lowers,
//               :346-370), bit-exact: separate fp64 multiply and add
//   k_h_float   Linf-sum and sum-per-partition histograms (bisect_right over
//               the lowers, _bin_lower_index :50-59); the pair histogram's
//               counts and sums are privatised in LDS (120 KB per workgroup);
//               k_h_float_max, a second pass, its bin maxima (80 KB)
//   k_h_final   derived sums / maxima of the width-1 bins, fp64 maxima decoded
//
// Integer histograms use the logarithmic bins of
// _to_bin_lower_upper_logarithmic (:28-47), indexed densely: lower < 1000 ->
// index = lower (width 1, so bin sum = count * lower and max = lower, which
// k_h_final fills in: the hot small bins only count, privatised in LDS);
// lower = q * 10^e (q in [100, 999], e >= 1) -> 1000 + (e - 1) * 900 + q - 100.
#include "pdp_internal.h"

namespace pdp {
namespace {

constexpr int kLogBins = PDP_HIST_LOG_BINS;
constexpr int kSumBuckets = PDP_HIST_SUM_BUCKETS;
constexpr int kNLowers = kSumBuckets + 1;
constexpr int kSmallBins = 1000;  // width-1 bins, counted in LDS
constexpr uint64_t kMinTable = 1024;

enum { H_L0 = 0, H_L1 = 1, H_LINF = 2, H_COUNT = 3, H_PIDS = 4 };
enum { F_LINF_SUM = 0, F_PART_SUM = 1 };

// pair-table slot: key + 1 (0 = empty, so the table clears with a memset);
// cnt holds rows - 1, so the row whose CAS creates the pair skips the count
// atomic (most pairs have one row)
struct alignas(32) Slot {
  unsigned long long key;
  double sum;
  unsigned cnt, pad;
};

// a pair's contribution to its partition (privacy-id buckets), grouped by
// partition range
struct alignas(16) PRec {
  unsigned pk, rows;
  double sum;
};

uint64_t table_capacity(int64_t n_rows) {
  uint64_t c = (uint64_t)n_rows + (uint64_t)n_rows / 2;
  c = (c + 255) & ~(uint64_t)255;
  return c < kMinTable ? kMinTable : c;
}

// the pair table is split into regions of kRegionW partitions (pk >> 12),
// each sized from its row count, so that k_h_pairs can sum per-partition
// statistics of one region in LDS and flush them with contiguous atomics
constexpr int kRegionBits = 12;
constexpr int kRegionW = 1 << kRegionBits;
constexpr int kRegionLdsMax = 16384;  // region count histogram in LDS up to here
constexpr int kPairsBlock = 512;
constexpr int kPairsChunk = 16384;    // slots per k_h_pairs workgroup

int64_t n_regions(int64_t P) { return P > 0 ? (P + kRegionW - 1) >> kRegionBits : 1; }

// slots: 1.5 per row + 64 of slack per region (every region with rows gets them)
uint64_t slots_capacity(int64_t n_rows, int64_t P) {
  return table_capacity(n_rows) + 64 * (uint64_t)n_regions(P);
}

struct HWs {
  uint64_t err, slots, rbase, rchunks, pidstat, pkstat, psum, minmax, fmax;
  // bucketed pairs (hb_*): per (tile, super-bucket) row counts -> offsets,
  // super-bucket bases, rows per pair bucket -> starts (+ scan scratch), write
  // cursors, the pair sums, {mode, pairs, overflow}; the level-1 / level-2
  // records reuse the pair-table region
  uint64_t hb_cts, hb_sbase, hb_bcnt, hb_bchunks, hb_bcur, hb_pairsum, hb_ctl;
  // privacy-id buckets with partition ranges: each bucket's run start per
  // range (k_hb_pid_pairs -> k_hb_prange)
  uint64_t hb_pruns;
  uint64_t total;
};

// ---- bucketed pairs (the raw-row pairs phase) -------
// Rows are partitioned by a hash of their (privacy id, partition) pair into
// NB pair buckets (two LDS counting-sort levels: <= 256 super-buckets of <=
// 256 buckets), and one workgroup per bucket finds the bucket's distinct
// pairs in an LDS hash table: no pair table in HBM, no global CAS.  A bucket
// holds ~kHbRowsPerBucket rows, an upper bound of its pairs, so its table
// (kHbSlots) stays at most ~60 % full; a table that would pass kHbFill falls
// back to the pair-table path for the whole call (never for hashed real data).
constexpr int kHbTileRows = 65536;
constexpr int kHbThreads = 1024;         // count / level-1 workgroups
constexpr int kHbStage = 8192;           // level-1 rows per LDS stage (8 per thread; 4,096: 1.32 vs 1.16 ms)
constexpr int kHbFan = 256;              // buckets per super-bucket
constexpr int kHbL2Threads = 1024;
// level-2 records per window (8 per thread; 139 KB of LDS, one workgroup per
// CU): windows of 2,048 / 4,096 records ran 1.35 / 1.12 ms against 0.95 ms
// at 1e8 rows -- fewer, longer runs per bucket write more whole lines
// (profiles/r05/ab/ab10_hist_latency.txt)
constexpr int kHbWin = 8192;
constexpr int kHbK = 8;                  // level-2 workgroups per super-bucket
constexpr int kHbSlots = 3072;           // LDS pair table per bucket
constexpr int kHbFill = 2760;            // 90 % of kHbSlots: more distinct pairs -> fallback
constexpr int64_t kHbRowsPerBucket = 1536;
constexpr int64_t kHbMaxBuckets = (int64_t)kHbFan * 256;
constexpr int kHbPairThreads = 512;
// Privacy-id buckets (the default, round 3): the same two levels keyed by a
// hash of the privacy id alone, so one workgroup (k_hb_pid_pairs) sees every
// row of its privacy ids and finishes their L0 / L1 counts in LDS; its pairs
// leave as (partition, rows, sum) records grouped by 2,048-partition range,
// which k_hb_prange sums per partition in LDS: no per-pair global atomics.
// Each thread keeps its <= 4 table slots in registers after the pair phase,
// so the 20-byte slots' LDS is reused by the pid table and the range
// counters: 80,640 B + a few words, two 1,024-thread workgroups per CU.
constexpr int kHbPidThreads = 1024;
constexpr int kHbPidSlots = 4032;
constexpr int kHbPidFill = 3628;         // 90 % of kHbPidSlots
constexpr int kHbPidPer = (kHbPidSlots + kHbPidThreads - 1) / kHbPidThreads;
#ifndef PDP_HB_PID_PRE
#define PDP_HB_PID_PRE 2
#endif
constexpr int kHbPidPre = PDP_HB_PID_PRE;  // rows per thread loaded together in k_hb_pid_pairs
constexpr int kHbRangeBits = 11;
constexpr int kHbRangeW = 1 << kHbRangeBits;
constexpr int kHbRangeMax = 128;         // more ranges (P > 262,144): per-pair partition atomics
constexpr int kHbRangeThreads = 1024;
#ifndef PDP_HB_RANGE_U
#define PDP_HB_RANGE_U 4
#endif
constexpr int kHbRangeU = PDP_HB_RANGE_U;
#ifndef PDP_HB_RANGE_WAVE
#define PDP_HB_RANGE_WAVE 1  // k_hb_prange: one wave per 64 buckets' runs (else a workgroup scan + search per record)
#endif  // records per thread in flight in k_hb_prange
static_assert(kHbPidSlots * 12 + kSmallBins * 4 + 3 * (kHbRangeMax + 1) * 4 <= kHbPidSlots * 20,
              "the pid table, Linf bins and range counters reuse the pair table's LDS");

inline int64_t hb_ranges(int64_t P) {
  const int64_t R = (P + kHbRangeW - 1) >> kHbRangeBits;
  return R >= 1 && R <= kHbRangeMax ? R : 0;
}

inline int64_t hb_buckets(int64_t n) {
  const int64_t nb = (n + kHbRowsPerBucket - 1) / kHbRowsPerBucket;
  return nb < 1 ? 1 : nb;
}
inline bool hb_eligible(int64_t n) { return n > 0 && hb_buckets(n) <= kHbMaxBuckets; }

// err first: pdp_bound_error_flags reads the error word at offset 0
HWs hlayout(int64_t n, int64_t U, int64_t P) {
  HWs w{};
  uint64_t off = 0;
  const uint64_t C = slots_capacity(n, P);
  const int64_t R = n_regions(P);
  w.err = off; off = align256(off + 16);
  w.slots = off; off = align256(off + C * sizeof(Slot));
  w.rbase = off; off = align256(off + (uint64_t)(R + 1) * 4);  // region rows -> slot bases (exclusive scan)
  w.rchunks = off; off = align256(off + (uint64_t)scan_chunk_sums_len(R + 1) * 4);
  // packed counters, one 64-bit atomic per pair: per pid (distinct
  // partitions << 32 | rows), per partition (distinct pids << 32 | rows)
  w.pidstat = off; off = align256(off + (uint64_t)U * 8);
  w.pkstat = off; off = align256(off + (uint64_t)P * 8);
  w.psum = off; off = align256(off + (uint64_t)P * 8);
  w.minmax = off; off = align256(off + 4 * 8);        // ordered u64: pair min, max; partition min, max
  w.fmax = off; off = align256(off + 2 * kSumBuckets * 8);  // ordered u64 bin maxima
  if (hb_eligible(n)) {
    const int64_t nb = hb_buckets(n);
    const int64_t ns = (nb + kHbFan - 1) / kHbFan;
    const int64_t nt = (n + kHbTileRows - 1) / kHbTileRows;
    w.hb_cts = off; off = align256(off + (uint64_t)(nt * ns) * 4);
    w.hb_sbase = off; off = align256(off + (uint64_t)(ns + 1) * 4);
    w.hb_bcnt = off; off = align256(off + (uint64_t)(nb + 1) * 4);
    w.hb_bchunks = off; off = align256(off + (uint64_t)scan_chunk_sums_len(nb + 1) * 4);
    w.hb_bcur = off; off = align256(off + (uint64_t)nb * 4);
    w.hb_pairsum = off; off = align256(off + (uint64_t)n * 8);
    const int64_t R = hb_ranges(P);
    if (R > 0) { w.hb_pruns = off; off = align256(off + (uint64_t)nb * (R + 1) * 4); }
  }
  // {mode (1: pair buckets' pair-sum list, 2: privacy-id buckets' records),
  //  pairs (mode 1), overflow, ranges (mode 2)}
  w.hb_ctl = off; off = align256(off + 16);
  w.total = off;
  return w;
}

struct HT {
  int64_t n, U, P;
  int pk_bits, has_value, do_parts;  // do_parts: per-partition histograms (multi-rank: one rank)
  uint64_t cap, pk_mask;             // cap: allocated slots (regions use a prefix of them)
  int64_t R;                         // regions
  int64_t nb, n_supers, n_tiles;     // bucketed pairs: pair buckets, super-buckets, tiles
  int hb_pid;                        // buckets keyed by privacy id (else by the pair)
  int64_t hb_R;                      // privacy-id buckets: partition ranges (0: per-pair atomics)
};

// order-preserving u64 image of an fp64 (for atomicMin/atomicMax)
__device__ __forceinline__ unsigned long long ord(double x) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}
__device__ __forceinline__ double unord(unsigned long long o) {
  const unsigned long long b = (o >> 63) ? (o & 0x7FFFFFFFFFFFFFFFULL) : ~o;
  return __longlong_as_double((long long)b);
}

// _to_bin_lower_upper_logarithmic's lower as a dense bin index
__device__ __forceinline__ int log_bin_index(unsigned long long v) {
  unsigned long long bound = 1000;
  while (v > bound) bound *= 10;
  const unsigned long long rb = bound / 1000;
  unsigned long long q = v / rb * rb;
  if (q < kSmallBins) return (int)q;
  int e = 0;
  while (q >= 1000) { q /= 10; ++e; }
  return kSmallBins + (e - 1) * 900 + (int)(q - 100);
}

struct IntHists {  // [5][kLogBins] each
  unsigned long long* count;
  unsigned long long* sum;
  unsigned long long* max;
};

// one element of value v into integer histogram h: small bins count in LDS
__device__ __forceinline__ void int_hist_add(const IntHists& H, unsigned* lds_counts, int h, int slot,
                                             unsigned long long v) {
  const int b = log_bin_index(v);
  if (b < kSmallBins) {
    atomicAdd(lds_counts + slot * kSmallBins + b, 1u);
  } else {
    const int64_t g = (int64_t)h * kLogBins + b;
    atomicAdd(H.count + g, 1ULL);
    atomicAdd(H.sum + g, v);
    atomicMax(H.max + g, v);
  }
}

// n elements of value v (one wave's elements that share a value)
__device__ __forceinline__ void int_hist_add_n(const IntHists& H, unsigned* lds_counts, int h, int slot,
                                               unsigned long long v, unsigned n) {
  const int b = log_bin_index(v);
  if (b < kSmallBins) {
    atomicAdd(lds_counts + slot * kSmallBins + b, n);
  } else {
    const int64_t g = (int64_t)h * kLogBins + b;
    atomicAdd(H.count + g, (unsigned long long)n);
    atomicAdd(H.sum + g, v * n);
    atomicMax(H.max + g, v);
  }
}

// one element per lane of a whole, converged wave (every lane calls it; valid
// marks the lanes with an element): small bins count in LDS; the lanes of one
// larger bin are summed across the wave and sent by one lane -- a bin every
// partition of a table falls in (1,000-row partitions: all in one or two
// bins) would otherwise take one global atomic per element on one address
__device__ __forceinline__ void int_hist_add_wave(const IntHists& H, unsigned* lds_counts, int h, int slot,
                                                  unsigned long long v, bool valid) {
  const int b = valid ? log_bin_index(v) : -1;
  if (valid && b < kSmallBins) atomicAdd(lds_counts + slot * kSmallBins + b, 1u);
  const int lane = threadIdx.x & 63;
  unsigned long long todo = __ballot(valid && b >= kSmallBins);
  while (todo) {  // wave-uniform
    const int leader = __ffsll((long long)todo) - 1;
    const int bl = __shfl(b, leader, 64);
    const bool mine = ((todo >> lane) & 1) && b == bl;
    const unsigned long long same = __ballot(mine);
    unsigned long long sum = mine ? v : 0ULL, mx = sum;
    for (int o = 32; o > 0; o >>= 1) {
      sum += __shfl_xor(sum, o, 64);
      const unsigned long long y = __shfl_xor(mx, o, 64);
      mx = y > mx ? y : mx;
    }
    if (lane == leader) {
      const int64_t g = (int64_t)h * kLogBins + bl;
      atomicAdd(H.count + g, (unsigned long long)__popcll(same));
      atomicAdd(H.sum + g, sum);
      atomicMax(H.max + g, mx);
    }
    todo &= ~same;
  }
}

__device__ __forceinline__ void flush_small(const IntHists& H, const unsigned* lds_counts, int slot, int h) {
  for (int b = threadIdx.x; b < kSmallBins; b += blockDim.x) {
    const unsigned c = lds_counts[slot * kSmallBins + b];
    if (c) atomicAdd(H.count + (int64_t)h * kLogBins + b, (unsigned long long)c);
  }
}

// x = pair key + 1 (never 0); slot = region base + high half of mix64(x) *
// region capacity, linear probing inside the region
__device__ __forceinline__ Slot* table_insert(Slot* slots, uint64_t base, uint64_t cap, uint64_t x,
                                              bool* created) {
  uint64_t h = base + __umul64hi(mix64(x), cap);
  const uint64_t end = base + cap;
  *created = false;
  for (;;) {
    // plain load first: a CAS on every probe measured 19.1 ms vs 12.3 ms
    // for k_h_rows at 1e8 rows (profiles/r01/h4_bench_hist.json)
    unsigned long long* k = &slots[h].key;
    const unsigned long long cur = *k;
    if (cur == x) return slots + h;
    if (cur == 0) {
      const unsigned long long old = atomicCAS(k, 0ULL, (unsigned long long)x);
      *created = old == 0;
      if (old == 0 || old == x) return slots + h;
    }
    h = h + 1 == end ? base : h + 1;  // region capacity > its rows: a free slot always exists
  }
}

template <int VK>
__device__ __forceinline__ double row_value(const void* value, int64_t i) {
  if (VK == PDP_VALUE_F64) return ((const double*)value)[i];
  if (VK == PDP_VALUE_I64) return (double)((const long long*)value)[i];
  return 0.0;
}

// rows per region (valid rows only); LDS histogram when the regions fit
template <bool LDS>
__global__ void __launch_bounds__(kBlock) k_h_region_count(HT t, const int64_t* __restrict__ pid,
                                                           const int64_t* __restrict__ pk, unsigned* rcnt) {
  __shared__ unsigned lh[LDS ? kRegionLdsMax : 1];
  if (LDS) {
    for (int b = threadIdx.x; b < t.R; b += blockDim.x) lh[b] = 0;
    __syncthreads();
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n; i += stride) {
    const int64_t u = pid[i], k = pk[i];
    if (u < 0 || u >= t.U || k < 0 || k >= t.P) continue;
    if (LDS) atomicAdd(lh + (k >> kRegionBits), 1u);
    else atomicAdd(rcnt + (k >> kRegionBits), 1u);
  }
  if (LDS) {
    __syncthreads();
    for (int b = threadIdx.x; b < t.R; b += blockDim.x)
      if (lh[b]) atomicAdd(rcnt + b, lh[b]);
  }
}

// region rows -> region slot capacity (1.5 per row + 64), scanned afterwards
__global__ void __launch_bounds__(kBlock) k_h_region_caps(int64_t R, unsigned* rcnt) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < R) {
    const unsigned c = rcnt[r];
    rcnt[r] = c ? c + c / 2 + 64 : 0u;
  }
}

template <int VK>
__global__ void __launch_bounds__(kBlock) k_h_rows(HT t, const int64_t* __restrict__ pid,
                                                   const int64_t* __restrict__ pk, const void* __restrict__ value,
                                                   const unsigned* __restrict__ rbase, Slot* slots,
                                                   unsigned* err) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n; i += stride) {
    const int64_t u = pid[i], k = pk[i];
    if (u < 0 || u >= t.U || k < 0 || k >= t.P) {
      atomicOr(err, 1u);
      continue;
    }
    const double v = row_value<VK>(value, i);
    bool created;
    const int64_t r = k >> kRegionBits;
    const unsigned b0 = rbase[r];
    Slot* s = table_insert(slots, b0, rbase[r + 1] - b0, (((uint64_t)u << t.pk_bits) | (uint64_t)k) + 1, &created);
    if (!created) atomicAdd(&s->cnt, 1u);
    if (VK != PDP_VALUE_NONE) atomicAdd(&s->sum, v);
  }
}

// block-wide min/max of ordered fp64 images, one atomic pair per block
__device__ __forceinline__ void block_minmax(unsigned long long mn, unsigned long long mx, unsigned long long* out) {
  __shared__ unsigned long long smn[16], smx[16];
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { smn[w] = mn; smx[w] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int j = 1; j < (int)(blockDim.x >> 6); ++j) {
      mn = smn[j] < mn ? smn[j] : mn;
      mx = smx[j] > mx ? smx[j] : mx;
    }
    if (mn != ~0ULL) atomicMin(out, mn);
    if (mx != 0ULL) atomicMax(out + 1, mx);
  }
}

// one workgroup per chunk of kPairsChunk slots; per region the chunk
// touches, the region's per-partition statistics are summed in LDS and
// flushed with contiguous atomics; per-pid statistics stay global atomics
__global__ void __launch_bounds__(kPairsBlock) k_h_pairs(HT t, const Slot* __restrict__ slots,
                                                         const unsigned* __restrict__ rbase,
                                                         unsigned long long* pidstat, unsigned long long* pkstat,
                                                         double* psum, IntHists H, unsigned long long* minmax) {
  __shared__ unsigned lds[kSmallBins];
  __shared__ unsigned long long lstat[kRegionW];
  __shared__ double lsum[kRegionW];
  __shared__ int64_t r_first;
  for (int b = threadIdx.x; b < kSmallBins; b += blockDim.x) lds[b] = 0;
  const int64_t used = rbase[t.R];
  const int64_t s0 = (int64_t)blockIdx.x * kPairsChunk;
  const int64_t s1 = s0 + kPairsChunk < used ? s0 + kPairsChunk : used;
  if (threadIdx.x == 0) {  // last region with base <= s0
    int64_t lo = 0, hi = t.R;  // rbase[lo] <= s0 < rbase[hi] (when s0 < used)
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)rbase[mid] <= s0) lo = mid;
      else hi = mid;
    }
    r_first = lo;
  }
  __syncthreads();
  unsigned long long mn = ~0ULL, mx = 0ULL;
  for (int64_t r = r_first; s0 < s1 && r < t.R && (int64_t)rbase[r] < s1; ++r) {
    const int64_t a = (int64_t)rbase[r] > s0 ? (int64_t)rbase[r] : s0;
    const int64_t e = (int64_t)rbase[r + 1] < s1 ? (int64_t)rbase[r + 1] : s1;
    if (a >= e) continue;  // empty region (uniform across the workgroup)
    for (int j = threadIdx.x; j < kRegionW; j += blockDim.x) {
      lstat[j] = 0;
      lsum[j] = 0.0;
    }
    __syncthreads();
    for (int64_t s = a + threadIdx.x; s < e; s += blockDim.x) {
      const Slot sl = slots[s];
      if (sl.key == 0) continue;
      const unsigned long long x = sl.key - 1;
      const unsigned rows = sl.cnt + 1;
      const unsigned long long inc = (1ULL << 32) | rows;
      const int j = (int)((x & t.pk_mask) & (kRegionW - 1));
      atomicAdd(pidstat + (x >> t.pk_bits), inc);
      atomicAdd(lstat + j, inc);
      if (t.has_value) atomicAdd(lsum + j, sl.sum);
      int_hist_add(H, lds, H_LINF, 0, rows);
      const unsigned long long o = ord(sl.sum);
      mn = o < mn ? o : mn;
      mx = o > mx ? o : mx;
    }
    __syncthreads();
    const int64_t p0 = r << kRegionBits;
    for (int j = threadIdx.x; j < kRegionW; j += blockDim.x) {
      const unsigned long long st = lstat[j];
      if (st) {
        atomicAdd(pkstat + p0 + j, st);
        if (t.has_value) atomicAdd(psum + p0 + j, lsum[j]);
      }
    }
    __syncthreads();
  }
  block_minmax(mn, mx, minmax);  // contains __syncthreads: every thread reaches it
  __syncthreads();
  flush_small(H, lds, 0, H_LINF);
}

constexpr int kIdsThreads = 1024;  // 16 waves per CU at one workgroup per CU (256 threads: 0.20 ms, latency-bound)
__global__ void __launch_bounds__(kIdsThreads) k_h_ids(HT t, const unsigned long long* __restrict__ pidstat,
                                                  const unsigned long long* __restrict__ pkstat,
                                                  const double* __restrict__ psum, IntHists H,
                                                  unsigned long long* minmax) {
  __shared__ unsigned lds[4 * kSmallBins];
  for (int b = threadIdx.x; b < 4 * kSmallBins; b += blockDim.x) lds[b] = 0;
  __syncthreads();
  const int64_t m = t.U > t.P ? t.U : t.P;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned long long mn = ~0ULL, mx = 0ULL;
  // the loop bound is workgroup-uniform, so every wave stays converged for
  // int_hist_add_wave; lanes past the end carry no element
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < m; i0 += stride) {
    const int64_t i = i0 + threadIdx.x;
    // the three loads together (psum not after pkstat's check)
    const unsigned long long st = i < t.U ? pidstat[i] : 0ULL;
    const bool part = t.do_parts && i < t.P;
    const unsigned long long sp = part ? pkstat[i] : 0ULL;
    const double ps = part ? psum[i] : 0.0;
    int_hist_add_wave(H, lds, H_L0, 0, st >> 32, st != 0);
    int_hist_add_wave(H, lds, H_L1, 1, st & 0xFFFFFFFFULL, st != 0);
    if (t.do_parts) {
      int_hist_add_wave(H, lds, H_COUNT, 2, sp & 0xFFFFFFFFULL, sp != 0);
      int_hist_add_wave(H, lds, H_PIDS, 3, sp >> 32, sp != 0);
      if (sp) {
        const unsigned long long o = ord(ps);
        mn = o < mn ? o : mn;
        mx = o > mx ? o : mx;
      }
    }
  }
  block_minmax(mn, mx, minmax + 2);
  __syncthreads();
  flush_small(H, lds, 0, H_L0);
  flush_small(H, lds, 1, H_L1);
  flush_small(H, lds, 2, H_COUNT);
  flush_small(H, lds, 3, H_PIDS);
}

// the lowers of k_h_lowers recomputed in registers (same roundings, so the
// same doubles): a value's bin costs no memory reads
struct LinBins {
  double mn, mx, step, delta, inv;
  int nb;
};
__device__ __forceinline__ LinBins lin_bins(const double* __restrict__ L, int nl) {
  LinBins z{0.0, 0.0, 0.0, 0.0, 0.0, nl - 1};
  if (nl < 2) return z;
  z.mn = L[0];
  z.mx = L[nl - 1];
  z.delta = __dsub_rn(z.mx, z.mn);
  z.step = __ddiv_rn(z.delta, (double)kSumBuckets);
  z.inv = z.delta > 0.0 ? (double)z.nb / z.delta : 0.0;
  return z;
}
// numpy's y = i * step + start (or (i / div) * delta + start when step == 0,
// a call-uniform case: STEP0), each operation rounded on its own: contraction
// into an FMA is off in this scope (an FMA moves values across bin edges; the
// oracle caught one).  Round 4 kept the two forms in one select, which the
// compiler evaluated both sides of: an fp64 division per lower, 2 per value
template <bool STEP0>
__device__ __forceinline__ double lin_lower(const LinBins& z, int i) {
#pragma clang fp contract(off)
  if (i == z.nb) return z.mx;
  const double y = STEP0 ? ((double)i / (double)kSumBuckets) * z.delta : (double)i * z.step;
  return y + z.mn;
}
// bisect_right(lowers, v) - 1 as float_bin, from the recomputed lowers
template <bool STEP0>
__device__ __forceinline__ int lin_bin(const LinBins& z, double v) {
  const int nb = z.nb;
  if (nb <= 1) return 0;
  // a guess; the loops make it exact.  The guess is converted only when it
  // lies in [0, nb): a subnormal range overflows inv to inf, and v == mn then
  // gives 0 * inf = NaN
  const double g = (v - z.mn) * z.inv;
  int b = g >= 0.0 && g < (double)nb ? (int)g : (g >= (double)nb ? nb - 1 : 0);
  // the guess is almost always the bin: test its two edges once, and walk
  // (the exact definition) only when it is not -- the walks unrolled ran
  // their set-up for every value, and this pass is VALU-bound
  const double lo = b > 0 ? lin_lower<STEP0>(z, b) : -__builtin_huge_val();
  const double hi = b + 1 < nb ? lin_lower<STEP0>(z, b + 1) : __builtin_huge_val();
  if (__builtin_expect(lo <= v && v < hi, 1)) return b;
#pragma nounroll
  while (b + 1 < nb && lin_lower<STEP0>(z, b + 1) <= v) ++b;
#pragma nounroll
  while (b > 0 && lin_lower<STEP0>(z, b) > v) --b;
  return b;
}
__device__ __forceinline__ int lin_bin_any(const LinBins& z, double v) {
  return z.step == 0.0 ? lin_bin<true>(z, v) : lin_bin<false>(z, v);
}
template <bool B>
struct BoolTag {
  static constexpr bool value = B;
};

// np.linspace(mn, mx, 10001) (numpy function_base.linspace): step = delta /
// div, y = i * step + start with separate roundings, y[-1] = stop; [mn, mn]
// when mn == mx; no lowers when the histogram is empty.
__global__ void __launch_bounds__(kBlock) k_h_lowers(const unsigned long long* __restrict__ minmax,
                                                     double* lowers, int* n_lowers) {
  const int f = blockIdx.y;
  const unsigned long long omn = minmax[2 * f], omx = minmax[2 * f + 1];
  const bool empty = omn == ~0ULL;
  const double mn = unord(omn), mx = unord(omx);
  double* L = lowers + (int64_t)f * kNLowers;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) n_lowers[f] = empty ? 0 : (mn == mx ? 2 : kNLowers);
  if (empty || i >= kNLowers) return;
  if (mn == mx) {
    if (i < 2) L[i] = mn;
    return;
  }
  LinBins z{mn, mx, 0.0, __dsub_rn(mx, mn), 0.0, kSumBuckets};
  z.step = __ddiv_rn(z.delta, (double)kSumBuckets);
  L[i] = z.step == 0.0 ? lin_lower<true>(z, i) : lin_lower<false>(z, i);  // the last is mx
}

// bisect_right(lowers, v) - 1, the maximum in the last bin (_bin_lower_index)
__device__ __forceinline__ int float_bin(const double* __restrict__ L, int nl, double v) {
  const int nb = nl - 1;
  if (nb <= 1) return 0;
  const double span = L[nb] - L[0];
  int b = (int)((v - L[0]) / span * (double)nb);
  b = b < 0 ? 0 : (b > nb - 1 ? nb - 1 : b);
  while (b + 1 < nb && L[b + 1] <= v) ++b;
  while (b > 0 && L[b] > v) --b;
  return b;
}

struct FloatHists {
  unsigned long long* count;  // [2][kSumBuckets]
  double* sum;
  unsigned long long* omax;   // ordered images (workspace)
};

__device__ __forceinline__ void max_filtered(unsigned long long* omax, unsigned long long o) {
  if (o > __hip_atomic_load(omax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(omax, o);
}

constexpr int kFloatBlock = 1024;
#ifndef PDP_HF_U
#define PDP_HF_U 8
#endif
constexpr int kFloatU = PDP_HF_U;  // pair sums in flight per thread

// every pair sum of the call's pair phase, in the form it left them: the pair
// buckets' list (mode 1), the privacy-id buckets' range-grouped records
// (mode 2: every bucket's row span holds its pairs, then records marked
// pk = ~0, so one flat, coalesced pass reads them all), or the pair table
template <typename Fn>
__device__ __forceinline__ void for_pair_sums(const HT& t, const Slot* __restrict__ slots,
                                              const double* __restrict__ pairsum,
                                              const unsigned* __restrict__ hb_ctl,
                                              const unsigned* __restrict__ hb_bstart,
                                              const PRec* __restrict__ hb_prec, Fn&& f) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i00 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int U = kFloatU;
  // the U loads of a round are unconditional (an index past the end is
  // clamped to the last element and its value dropped): a load under a branch
  // made the compiler wait for each before issuing the next (one in-order
  // vmcnt), U latency rounds instead of one
  if (hb_ctl[0] == 1) {
    const int64_t np = hb_ctl[1];
    for (int64_t i0 = i00; i0 < np; i0 += U * stride) {
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + u * stride;
        v[u] = pairsum[i < np ? i : np - 1];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (i0 + u * stride < np) f(v[u]);
    }
  } else if (hb_ctl[0] == 2) {
    const int64_t np = hb_bstart[t.nb];
    for (int64_t i0 = i00; i0 < np; i0 += U * stride) {
      PRec r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + u * stride;
        r[u] = hb_prec[i < np ? i : np - 1];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (i0 + u * stride < np && r[u].pk != ~0u) f(r[u].sum);
    }
  } else {
    for (int64_t i = i00; i < (int64_t)t.cap; i += stride) {
      const Slot sl = slots[i];
      if (sl.key != 0) f(sl.sum);
    }
  }
}

// the Linf-sum histogram in two passes over the pair sums, each with its bins
// privatised in LDS and flushed once per workgroup:
//   MAX = false  counts (u32) and sums (fp64), 120 KB: one workgroup per CU;
//                plus the partition-sum histogram (P elements, global atomics)
//   MAX = true   bin maxima as ordered u64 images, 80 KB; a value
//                goes to LDS only when it raises the bin's maximum
// One pass holding all three (200 KB) does not fit; the previous form kept
// only the high half of each maximum in LDS and sent every raise to a global
// atomicMax -- at ~4 raises per bin and workgroup those atomics, waited on by
// the next loads (one in-order vmcnt), took 1.0 of its 1.7 ms
// (profiles/r05/ab/ab10_hist_latency.txt); the second pass re-reads 1.6 GB.
#ifndef PDP_HF_MAXOCC
#define PDP_HF_MAXOCC 4
#endif
template <bool MAX>
__global__ void __launch_bounds__(kFloatBlock, MAX ? PDP_HF_MAXOCC : 4) k_h_float(HT t, const Slot* __restrict__ slots,
                                                         const double* __restrict__ pairsum,
                                                         const unsigned* __restrict__ hb_ctl,
                                                         const unsigned* __restrict__ hb_bstart,
                                                         const PRec* __restrict__ hb_prec,
                                                         const unsigned long long* __restrict__ pkstat,
                                                         const double* __restrict__ psum,
                                                         const double* __restrict__ lowers,
                                                         const int* __restrict__ n_lowers, FloatHists F) {
  __shared__ unsigned lcnt[MAX ? 1 : kSumBuckets];
  __shared__ double lsum[MAX ? 1 : kSumBuckets];
  __shared__ unsigned long long lmx[MAX ? kSumBuckets : 1];
  for (int b = threadIdx.x; b < kSumBuckets; b += blockDim.x) {
    if (MAX) {
      lmx[b] = 0;
    } else {
      lcnt[b] = 0;
      lsum[b] = 0.0;
    }
  }
  __syncthreads();
  const int nl0 = n_lowers[F_LINF_SUM], nl1 = n_lowers[F_PART_SUM];
  const LinBins z0 = lin_bins(lowers, nl0);
  auto bin_add = [&](auto step0, double v) {
    const int b = lin_bin<decltype(step0)::value>(z0, v);
    if (MAX) {
      const unsigned long long o = ord(v);
      if (o > lmx[b]) atomicMax(lmx + b, o);
    } else {
      atomicAdd(lcnt + b, 1u);
      atomicAdd(lsum + b, v);
    }
  };
  if (nl0 > 0 && z0.step == 0.0)  // call-uniform: one loop per lowers form
    for_pair_sums(t, slots, pairsum, hb_ctl, hb_bstart, hb_prec, [&](double v) { bin_add(BoolTag<true>{}, v); });
  else if (nl0 > 0)
    for_pair_sums(t, slots, pairsum, hb_ctl, hb_bstart, hb_prec, [&](double v) { bin_add(BoolTag<false>{}, v); });
  if (!MAX && nl1 > 0) {
    const LinBins z1 = lin_bins(lowers + kNLowers, nl1);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.P; i += stride) {
      if (pkstat[i] == 0) continue;
      const double v = psum[i];
      const int64_t g = (int64_t)F_PART_SUM * kSumBuckets + lin_bin_any(z1, v);
      atomicAdd(F.count + g, 1ULL);
      atomicAdd(F.sum + g, v);
      max_filtered(F.omax + g, ord(v));
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kSumBuckets; b += blockDim.x) {
    if (MAX) {
      const unsigned long long o = lmx[b];
      if (o) max_filtered(F.omax + b, o);
    } else {
      const unsigned c = lcnt[b];
      if (c) {
        atomicAdd(F.count + b, (unsigned long long)c);
        atomicAdd(F.sum + b, lsum[b]);
      }
    }
  }
}

// small_mask: the integer histograms whose width-1 bins hold counts only
// (pre-aggregated L0 / L1 fill theirs in k_hp_weights)
__global__ void __launch_bounds__(kBlock) k_h_final(IntHists H, FloatHists F, double* fmax_out, int small_mask) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 5 * kSmallBins && ((small_mask >> (i / kSmallBins)) & 1)) {
    const int h = i / kSmallBins, b = i % kSmallBins;
    const int64_t g = (int64_t)h * kLogBins + b;
    const unsigned long long c = H.count[g];
    H.sum[g] = c * (unsigned long long)b;
    H.max[g] = c ? (unsigned long long)b : 0ULL;
  }
  if (i < 2 * kSumBuckets) {
    const unsigned long long o = F.omax[i];
    fmax_out[i] = o ? unord(o) : 0.0;
  }
}

// min images all ones, max images zero
__global__ void k_h_init(unsigned long long* minmax) {
  if (threadIdx.x < 4) minmax[threadIdx.x] = (threadIdx.x & 1) ? 0ULL : ~0ULL;
}

// ------------------------------------------------------- bucketed pairs ----
// pair bucket of a (privacy id << pk_bits | partition) key: the high half of
// SplitMix64(key), scaled to [0, nb)
__device__ __forceinline__ unsigned hb_bucket(unsigned long long x, int64_t nb) {
  return (unsigned)(((mix64(x ^ 0x2545F4914F6CDD1DULL) >> 32) * (uint64_t)nb) >> 32);
}
// the bucket of a row's pair key under the call's keying (privacy id or pair)
__device__ __forceinline__ unsigned hb_bucket_t(const HT& t, unsigned long long x) {
  return hb_bucket(t.hb_pid ? x >> t.pk_bits : x, t.nb);
}

// exclusive scan of one u32 per thread over the workgroup (wsum: nw + 1 words)
__device__ __forceinline__ unsigned hb_block_scan(unsigned x, unsigned* wsum, unsigned* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  unsigned inc = x;
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned y = __shfl_up(inc, off, 64);
    if (lane >= off) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  if (w == 0) {
    const unsigned v = lane < nw ? wsum[lane] : 0;
    unsigned vi = v;
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned y = __shfl_up(vi, off, 64);
      if (lane >= off) vi += y;
    }
    if (lane < nw) wsum[lane] = vi - v;
    if (lane == nw - 1) wsum[nw] = vi;
  }
  __syncthreads();
  const unsigned r = wsum[w] + inc - x;
  *total = wsum[nw];
  __syncthreads();
  return r;
}

// step 1: valid rows per (tile, super-bucket); invalid keys set the error word
__global__ void __launch_bounds__(kHbThreads) k_hb_count(HT t, const int64_t* __restrict__ pid,
                                                         const int64_t* __restrict__ pk, unsigned* __restrict__ cts,
                                                         unsigned* err) {
  __shared__ unsigned h[kHbFan];
  for (int b = threadIdx.x; b < t.n_supers; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * kHbTileRows;
  const int64_t t1 = t0 + kHbTileRows < t.n ? t0 + kHbTileRows : t.n;
  bool bad = false;
  constexpr int C = 8;  // rows per thread loaded together (unconditional, clamped into the tile)
  for (int64_t i0 = t0 + threadIdx.x; i0 < t1; i0 += (int64_t)C * blockDim.x) {
    int64_t u[C], k[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int64_t i = i0 + (int64_t)c * blockDim.x;
      const int64_t ic = i < t1 ? i : t0;
      u[c] = pid[ic];
      k[c] = pk[ic];
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (i0 + (int64_t)c * blockDim.x >= t1) continue;
      if ((uint64_t)u[c] >= (uint64_t)t.U || (uint64_t)k[c] >= (uint64_t)t.P) {
        bad = true;
        continue;
      }
      atomicAdd(h + hb_bucket_t(t, ((uint64_t)u[c] << t.pk_bits) | (uint64_t)k[c]) / kHbFan, 1u);
    }
  }
  if (bad) atomicOr(err, 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < t.n_supers; b += blockDim.x) cts[(int64_t)blockIdx.x * t.n_supers + b] = h[b];
}

// step 2: per super-bucket, the tiles' counts -> offsets (in place, exclusive,
// tile order) and the super-bucket's total
__global__ void __launch_bounds__(kHbThreads) k_hb_scan_tiles(HT t, unsigned* __restrict__ cts,
                                                              unsigned* __restrict__ stotal) {
  __shared__ unsigned wsum[kHbThreads / 64 + 1];
  const int s = blockIdx.x;
  unsigned carry = 0;
  for (int64_t c = 0; c < t.n_tiles; c += blockDim.x) {  // block-uniform
    const int64_t tt = c + threadIdx.x;
    const unsigned v = tt < t.n_tiles ? cts[tt * t.n_supers + s] : 0u;
    unsigned tot;
    const unsigned ex = hb_block_scan(v, wsum, &tot);
    if (tt < t.n_tiles) cts[tt * t.n_supers + s] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) stotal[s] = carry;
}

// super-bucket totals -> bases (in place; sbase[n_supers] = valid rows)
__global__ void __launch_bounds__(kHbFan) k_hb_scan_supers(HT t, unsigned* __restrict__ sbase) {
  __shared__ unsigned wsum[kHbFan / 64 + 1];
  const unsigned v = (int)threadIdx.x < t.n_supers ? sbase[threadIdx.x] : 0u;
  unsigned tot;
  const unsigned ex = hb_block_scan(v, wsum, &tot);
  if ((int)threadIdx.x < t.n_supers) sbase[threadIdx.x] = ex;
  if (threadIdx.x == 0) sbase[t.n_supers] = tot;
}

// step 3: each tile's valid rows -> its super-buckets' regions (tile order
// within a region), as (key, value) records; LDS counting sort per stage
template <int VK>
__global__ void __launch_bounds__(kHbThreads) k_hb_l1(HT t, const int64_t* __restrict__ pid,
                                                      const int64_t* __restrict__ pk, const void* __restrict__ value,
                                                      const unsigned* __restrict__ cts,
                                                      const unsigned* __restrict__ sbase,
                                                      unsigned long long* __restrict__ okey, double* __restrict__ oval) {
  extern __shared__ unsigned long long hb_lds[];
  unsigned long long* skey = hb_lds;                       // [kHbStage]
  double* sval = (double*)(skey + kHbStage);               // [kHbStage] (VK != NONE)
  unsigned* hist = (unsigned*)(sval + (VK != PDP_VALUE_NONE ? kHbStage : 0));  // [kHbFan]
  unsigned* start = hist + kHbFan;                         // [kHbFan]
  unsigned* cur = start + kHbFan;                          // [kHbFan]: the tile's output cursor per super
  uint8_t* dest = (uint8_t*)(cur + kHbFan);                // [kHbStage]
  constexpr int N = kHbStage / kHbThreads;
  const int64_t t0 = (int64_t)blockIdx.x * kHbTileRows;
  const int64_t t1 = t0 + kHbTileRows < t.n ? t0 + kHbTileRows : t.n;
  // a stage's three columns load together (the values not after the keys'
  // check: one latency round per stage); rows past the tile load as pid -1
  // (invalid, like a bad key: no record).  Loading stage s + 1 while stage s
  // is written measured no faster (profiles/r05/ab/ab10_hist_latency.txt)
  int64_t ru[N], rk[N];
  double rv[N];
  auto load_stage = [&](int64_t c0) {
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const int64_t i = c0 + (int64_t)q * blockDim.x + threadIdx.x;
      ru[q] = -1;
      rk[q] = 0;
      rv[q] = 0.0;
      if (i >= t1) continue;
      ru[q] = pid[i];
      rk[q] = pk[i];
      if (VK == PDP_VALUE_F64) rv[q] = ((const double*)value)[i];
      if (VK == PDP_VALUE_I64) rv[q] = (double)((const long long*)value)[i];
    }
  };
  for (int b = threadIdx.x; b < t.n_supers; b += blockDim.x)
    cur[b] = sbase[b] + cts[(int64_t)blockIdx.x * t.n_supers + b];
  for (int64_t c0 = t0; c0 < t1; c0 += kHbStage) {
    for (int b = threadIdx.x; b < t.n_supers; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    load_stage(c0);
    unsigned long long x[N];
    double v[N];
    int d[N];
    unsigned rank[N];
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const int64_t u = ru[q], k = rk[q];
      d[q] = -1;
      x[q] = 0;
      v[q] = rv[q];
      if ((uint64_t)u >= (uint64_t)t.U || (uint64_t)k >= (uint64_t)t.P) continue;  // flagged by k_hb_count
      x[q] = ((uint64_t)u << t.pk_bits) | (uint64_t)k;
      d[q] = (int)(hb_bucket_t(t, x[q]) / kHbFan);
    }
#pragma unroll
    for (int q = 0; q < N; ++q) rank[q] = d[q] >= 0 ? atomicAdd(hist + d[q], 1u) : 0u;
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of hist by one wave
      const int lane = threadIdx.x;
      unsigned carry = 0;
      for (int base = 0; base < t.n_supers; base += 64) {
        const unsigned hv = base + lane < t.n_supers ? hist[base + lane] : 0u;
        unsigned incl = hv;
        for (int off = 1; off < 64; off <<= 1) {
          const unsigned up = __shfl_up(incl, off, 64);
          if (lane >= off) incl += up;
        }
        if (base + lane < t.n_supers) start[base + lane] = carry + incl - hv;
        carry += __shfl(incl, 63, 64);
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < N; ++q) {
      if (d[q] < 0) continue;
      const unsigned slot = start[d[q]] + rank[q];
      skey[slot] = x[q];
      if (VK != PDP_VALUE_NONE) sval[slot] = v[q];
      dest[slot] = (uint8_t)d[q];
    }
    __syncthreads();
    const unsigned total = t.n_supers > 0 ? start[t.n_supers - 1] + hist[t.n_supers - 1] : 0u;
    for (unsigned e = threadIdx.x; e < total; e += blockDim.x) {
      const unsigned dd = dest[e];
      const unsigned g = cur[dd] + (e - start[dd]);
      okey[g] = skey[e];
      if (VK != PDP_VALUE_NONE) oval[g] = sval[e];
    }
    __syncthreads();
    for (int b = threadIdx.x; b < t.n_supers; b += blockDim.x) cur[b] += hist[b];
  }
}

size_t hb_l1_lds(int vk) {
  return (size_t)kHbStage * (8 + (vk != PDP_VALUE_NONE ? 8 : 0) + 1) + 3 * kHbFan * 4;
}

// step 4: rows per pair bucket -- workgroup (s, k) counts windows k, k + K, ...
// of super-bucket s's region in LDS, one atomic per (workgroup, bucket)
__global__ void __launch_bounds__(kHbL2Threads) k_hb_bcount(HT t, const unsigned* __restrict__ sbase,
                                                            const unsigned long long* __restrict__ key,
                                                            unsigned* __restrict__ bcnt) {
  __shared__ unsigned h[kHbFan];
  const int s = blockIdx.x / kHbK, k = blockIdx.x % kHbK;
  for (int b = threadIdx.x; b < kHbFan; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const int64_t a = sbase[s], e = sbase[s + 1];
  for (int64_t w0 = a + (int64_t)k * kHbWin; w0 < e; w0 += (int64_t)kHbK * kHbWin) {
    const int64_t w1 = w0 + kHbWin < e ? w0 + kHbWin : e;
    constexpr int N = kHbWin / kHbL2Threads;  // a window's keys in flight at once
    unsigned long long x[N];
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const int64_t i = w0 + (int64_t)q * blockDim.x + threadIdx.x;
      x[q] = i < w1 ? key[i] : 0ULL;
    }
#pragma unroll
    for (int q = 0; q < N; ++q)
      if (w0 + (int64_t)q * blockDim.x + threadIdx.x < w1) atomicAdd(h + hb_bucket_t(t, x[q]) % kHbFan, 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kHbFan; b += blockDim.x) {
    const int64_t g = (int64_t)s * kHbFan + b;
    if (h[b] && g < t.nb) atomicAdd(bcnt + g, h[b]);
  }
}

// step 5: super-bucket windows -> pair buckets: LDS counting sort by bucket,
// one cursor atomic per (window, bucket) run
template <bool HAS_VALUE>
__global__ void __launch_bounds__(kHbL2Threads) k_hb_l2(HT t, const unsigned* __restrict__ sbase,
                                                        const unsigned long long* __restrict__ ikey,
                                                        const double* __restrict__ ival,
                                                        const unsigned* __restrict__ bstart,
                                                        unsigned* __restrict__ bcur,
                                                        unsigned long long* __restrict__ okey,
                                                        double* __restrict__ oval) {
  __shared__ unsigned long long skey[kHbWin];
  __shared__ double sval[HAS_VALUE ? kHbWin : 1];
  __shared__ uint8_t dest[kHbWin];
  __shared__ unsigned hist[kHbFan], start[kHbFan], base[kHbFan];
  constexpr int N = kHbWin / kHbL2Threads;
  const int s = blockIdx.x / kHbK, k = blockIdx.x % kHbK;
  const int64_t a = sbase[s], e = sbase[s + 1];
  for (int64_t w0 = a + (int64_t)k * kHbWin; w0 < e; w0 += (int64_t)kHbK * kHbWin) {  // block-uniform
    const int64_t w1 = w0 + kHbWin < e ? w0 + kHbWin : e;
    for (int b = threadIdx.x; b < kHbFan; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    unsigned long long x[N];
    double v[N];
    int d[N];
    unsigned rank[N];
    // all N records' loads first (unconditional: an index past the window
    // reads its first record, dropped below), then the bucket hashes -- the
    // hash inside a guarded load made each load wait for the previous one
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const int64_t i = w0 + (int64_t)q * blockDim.x + threadIdx.x;
      const int64_t ic = i < w1 ? i : w0;
      x[q] = ikey[ic];
      v[q] = HAS_VALUE ? ival[ic] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const int64_t i = w0 + (int64_t)q * blockDim.x + threadIdx.x;
      d[q] = i < w1 ? (int)(hb_bucket_t(t, x[q]) % kHbFan) : -1;
    }
#pragma unroll
    for (int q = 0; q < N; ++q) rank[q] = d[q] >= 0 ? atomicAdd(hist + d[q], 1u) : 0u;
    __syncthreads();
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      unsigned carry = 0;
      for (int b0 = 0; b0 < kHbFan; b0 += 64) {
        const unsigned hv = hist[b0 + lane];
        unsigned incl = hv;
        for (int off = 1; off < 64; off <<= 1) {
          const unsigned up = __shfl_up(incl, off, 64);
          if (lane >= off) incl += up;
        }
        start[b0 + lane] = carry + incl - hv;
        carry += __shfl(incl, 63, 64);
      }
    }
    // one cursor reservation per non-empty run of this window
    for (int b = threadIdx.x; b < kHbFan; b += blockDim.x) {
      const int64_t g = (int64_t)s * kHbFan + b;
      base[b] = (hist[b] && g < t.nb) ? bstart[g] + atomicAdd(bcur + g, hist[b]) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < N; ++q) {
      if (d[q] < 0) continue;
      const unsigned slot = start[d[q]] + rank[q];
      skey[slot] = x[q];
      if (HAS_VALUE) sval[slot] = v[q];
      dest[slot] = (uint8_t)d[q];
    }
    __syncthreads();
    const unsigned total = (unsigned)(w1 - w0);
    for (unsigned i = threadIdx.x; i < total; i += blockDim.x) {
      const unsigned dd = dest[i];
      const unsigned g = base[dd] + (i - start[dd]);
      okey[g] = skey[i];
      if (HAS_VALUE) oval[g] = sval[i];
    }
    __syncthreads();
  }
}

// step 6: one workgroup per pair bucket: its distinct pairs in an LDS hash
// table (key, rows, value sum), then per pair exactly what k_h_pairs does
// per table slot: per pid and per partition (distinct << 32 | rows) and value
// sums, the Linf histogram, the pair sums' min / max, and the pair sum into
// the compact list k_h_float bins.  More than kHbFill distinct pairs in one
// bucket: the overflow word is set and the call falls back.
template <bool HAS_VALUE>
__global__ void __launch_bounds__(kHbPairThreads) k_hb_pairs(HT t, const unsigned* __restrict__ bstart,
                                                             const unsigned long long* __restrict__ key,
                                                             const double* __restrict__ val,
                                                             unsigned long long* pidstat, unsigned long long* pkstat,
                                                             double* psum, IntHists H, unsigned long long* minmax,
                                                             double* __restrict__ pairsum, unsigned* ctl) {
  __shared__ unsigned long long tkey[kHbSlots];
  __shared__ unsigned tcnt[kHbSlots];
  __shared__ double tsum[HAS_VALUE ? kHbSlots : 1];
  __shared__ unsigned lds[kSmallBins];
  __shared__ unsigned fill, s_base;
  for (int i = threadIdx.x; i < kHbSlots; i += blockDim.x) {
    tkey[i] = ~0ULL;
    tcnt[i] = 0;
    if (HAS_VALUE) tsum[i] = 0.0;
  }
  for (int b = threadIdx.x; b < kSmallBins; b += blockDim.x) lds[b] = 0;
  if (threadIdx.x == 0) fill = 0;
  __syncthreads();
  const int64_t a = bstart[blockIdx.x], e = bstart[blockIdx.x + 1];
  bool over = false;
  for (int64_t i = a + threadIdx.x; i < e; i += blockDim.x) {
    const unsigned long long x = key[i];
    unsigned sl = (unsigned)(((mix64(x) & 0xFFFFFFFFULL) * (uint64_t)kHbSlots) >> 32);
    for (;;) {
      const unsigned long long cur = tkey[sl];
      if (cur == x) break;
      if (cur == ~0ULL) {
        if (atomicAdd(&fill, 1u) >= (unsigned)kHbFill) {  // table too full: fall back
          over = true;
          break;
        }
        const unsigned long long old = atomicCAS(tkey + sl, ~0ULL, x);
        if (old == ~0ULL) break;
        atomicSub(&fill, 1u);  // lost the slot to another key
        if (old == x) break;
      }
      sl = sl + 1 == (unsigned)kHbSlots ? 0u : sl + 1;
    }
    if (over) break;
    atomicAdd(tcnt + sl, 1u);
    if (HAS_VALUE) atomicAdd(tsum + sl, val[i]);
  }
  if (over) atomicOr(ctl + 2, 1u);
  __syncthreads();
  if (threadIdx.x == 0) {
    s_base = atomicAdd(ctl + 1, fill);  // this bucket's pair sums
    fill = 0;
  }
  __syncthreads();
  unsigned long long mn = ~0ULL, mx = 0ULL;
  for (int j = threadIdx.x; j < kHbSlots; j += blockDim.x) {
    const unsigned long long x = tkey[j];
    const unsigned rows = tcnt[j];
    if (x == ~0ULL || rows == 0) continue;
    const double sum = HAS_VALUE ? tsum[j] : 0.0;
    const unsigned long long inc = (1ULL << 32) | rows;
    atomicAdd(pidstat + (x >> t.pk_bits), inc);
    const uint64_t p = x & t.pk_mask;
    atomicAdd(pkstat + p, inc);
    if (HAS_VALUE) atomicAdd(psum + p, sum);
    int_hist_add(H, lds, H_LINF, 0, rows);
    const unsigned long long o = ord(sum);
    mn = o < mn ? o : mn;
    mx = o > mx ? o : mx;
    const unsigned long long at = (unsigned long long)s_base + atomicAdd(&fill, 1u);
    if (at < (unsigned long long)t.n) pairsum[at] = sum;  // (an overflowed call is discarded)
  }
  block_minmax(mn, mx, minmax);  // contains __syncthreads
  __syncthreads();
  flush_small(H, lds, 0, H_LINF);
}

// step 6, privacy-id buckets: one workgroup per bucket holds every row of its
// privacy ids.  Phase 1 finds the distinct pairs in an LDS table (key, rows,
// sum); each thread then keeps its <= kHbPidPer slots in registers and the
// LDS becomes a pid table (distinct partitions << 32 | rows per pid) and the
// range counters.  Per pair: its pid's counters and either (RANGES) a PRec
// in the bucket's region -- row positions [bstart[b], bstart[b] + pairs),
// grouped by partition range, run starts in pruns[b][0..R]; k_hb_prange
// then does the partition sums, the Linf bins and the pair-sum range, and
// k_h_float reads the pair sums there -- or the partition atomics, Linf bins,
// pair-sum range and list here.  No global word is touched by every
// workgroup (a returning atomic on one address per bucket serialises).  Per
// pid: one plain store of its L0 / L1 counts (no other workgroup holds that
// pid).  A table past kHbPidFill sets the overflow word; the call then
// redoes the pairs with pair-keyed buckets.
template <bool HAS_VALUE, bool RANGES>
__global__ void __launch_bounds__(kHbPidThreads) k_hb_pid_pairs(
    HT t, const unsigned* __restrict__ bstart, const unsigned long long* __restrict__ key,
    const double* __restrict__ val, unsigned long long* __restrict__ pidstat, unsigned long long* pkstat,
    double* psum, IntHists H, unsigned long long* minmax, double* __restrict__ pairsum, PRec* __restrict__ prec,
    unsigned* __restrict__ pruns, unsigned* ctl) {
  extern __shared__ unsigned long long hp_lds[];
  unsigned long long* tkey = hp_lds;                         // phase 1: [kHbPidSlots] pair keys
  double* tsum = (double*)(tkey + kHbPidSlots);              //          [kHbPidSlots] value sums
  unsigned* tcnt = (unsigned*)(tsum + kHbPidSlots);          //          [kHbPidSlots] rows
  unsigned long long* pst = hp_lds;                          // phase 2: [kHbPidSlots] pid counters
  unsigned* pkey = (unsigned*)(pst + kHbPidSlots);           //          [kHbPidSlots] pids
  unsigned* lbins = pkey + kHbPidSlots;                      //          [kSmallBins] Linf bins
  unsigned* rcnt = lbins + kSmallBins;                       //          [kHbRangeMax + 1]
  unsigned* rstart = rcnt + kHbRangeMax + 1;                 //          [kHbRangeMax + 1]
  __shared__ unsigned fill, s_base, s_over;
  const int64_t a = bstart[blockIdx.x], e = bstart[blockIdx.x + 1];
  // each thread's next kHbPidPre rows (keys and values) are loaded together,
  // the first batch before the table is cleared: one memory latency per
  // batch instead of two per row (a bucket averages 1.5 rows per thread).
  // A persistent form that loaded the next bucket's rows during this one's
  // phase 2 measured slower (1.71 vs 1.59 ms, profiles/r05/ab/ab10_hist_latency.txt)
  unsigned long long xs[kHbPidPre];
  double vs[kHbPidPre];
  auto load_rows = [&](int64_t i0) {
#pragma unroll
    for (int q = 0; q < kHbPidPre; ++q) {
      const int64_t i = i0 + (int64_t)q * blockDim.x;
      xs[q] = i < e ? key[i] : 0ULL;
      vs[q] = HAS_VALUE && i < e ? val[i] : 0.0;
    }
  };
  int64_t i0 = a + threadIdx.x;
  load_rows(i0);
  for (int i = threadIdx.x; i < kHbPidSlots; i += blockDim.x) {
    tkey[i] = ~0ULL;
    tsum[i] = 0.0;
    tcnt[i] = 0;
  }
  if (threadIdx.x == 0) {
    fill = 0;
    s_over = 0;
  }
  __syncthreads();
  // distinct pairs <= rows: only a bucket with more rows than kHbPidFill
  // counts its new slots (one LDS address for the whole workgroup)
  const bool may_over = e - a > kHbPidFill;
  for (bool over = false; i0 < e && !over; i0 += (int64_t)kHbPidPre * blockDim.x) {
#pragma unroll
    for (int q = 0; q < kHbPidPre; ++q) {
      if (over || i0 + (int64_t)q * blockDim.x >= e) break;
      const unsigned long long x = xs[q];
      unsigned sl = (unsigned)(((mix64(x) & 0xFFFFFFFFULL) * (uint64_t)kHbPidSlots) >> 32);
      for (;;) {
        const unsigned long long cur = tkey[sl];
        if (cur == x) break;
        if (cur == ~0ULL) {
          if (may_over && atomicAdd(&fill, 1u) >= (unsigned)kHbPidFill) {
            over = true;
            break;
          }
          const unsigned long long old = atomicCAS(tkey + sl, ~0ULL, x);
          if (old == ~0ULL) break;
          if (may_over) atomicSub(&fill, 1u);
          if (old == x) break;
        }
        sl = sl + 1 == (unsigned)kHbPidSlots ? 0u : sl + 1;
      }
      if (over) break;
      atomicAdd(tcnt + sl, 1u);
      if (HAS_VALUE) atomicAdd(tsum + sl, vs[q]);
    }
    if (over) s_over = 1;
    else if (i0 + (int64_t)kHbPidPre * blockDim.x < e) load_rows(i0 + (int64_t)kHbPidPre * blockDim.x);
  }
  __syncthreads();
  if (s_over) {  // workgroup-uniform: the call's results are discarded
    // k_hb_prange still reads this bucket's runs: leave them empty
    if (RANGES)
      for (int r = threadIdx.x; r <= (int)t.hb_R; r += blockDim.x) pruns[(int64_t)blockIdx.x * (t.hb_R + 1) + r] = 0;
    if (threadIdx.x == 0) atomicOr(ctl + 2, 1u);
    return;
  }
  unsigned long long kx[kHbPidPer];
  unsigned kc[kHbPidPer], rk[kHbPidPer], pp[kHbPidPer];
  double ks[kHbPidPer];
#pragma unroll
  for (int q = 0; q < kHbPidPer; ++q) {
    const int j = threadIdx.x + q * kHbPidThreads;
    kx[q] = ~0ULL;
    kc[q] = 0;
    ks[q] = 0.0;
    if (j < kHbPidSlots) {
      kx[q] = tkey[j];
      kc[q] = tcnt[j];
      if (HAS_VALUE) ks[q] = tsum[j];
    }
  }
  __syncthreads();  // the table's bytes become the pid table
  for (int i = threadIdx.x; i < kHbPidSlots; i += blockDim.x) {
    pst[i] = 0;
    pkey[i] = ~0u;
  }
  if (!RANGES)
    for (int i = threadIdx.x; i < kSmallBins; i += blockDim.x) lbins[i] = 0;
  if (RANGES)
    for (int i = threadIdx.x; i <= kHbRangeMax; i += blockDim.x) rcnt[i] = 0;
  if (threadIdx.x == 0) fill = 0;
  __syncthreads();
  unsigned long long mn = ~0ULL, mx = 0ULL;
#pragma unroll
  for (int q = 0; q < kHbPidPer; ++q) {
    rk[q] = 0;
    pp[q] = 0;
    if (kx[q] == ~0ULL) continue;
    const unsigned long long x = kx[q];
    const unsigned pid = (unsigned)(x >> t.pk_bits);  // < U <= 2^32 - 1, never the empty key
    unsigned sl = (unsigned)(((uint64_t)(pid * 0x9E3779B1u) * (uint64_t)kHbPidSlots) >> 32);
    for (;;) {  // pids <= pairs <= kHbPidFill: a free slot exists
      const unsigned cur = pkey[sl];
      if (cur == pid) break;
      if (cur == ~0u) {
        const unsigned old = atomicCAS(pkey + sl, ~0u, pid);
        if (old == ~0u || old == pid) break;
      }
      sl = sl + 1 == (unsigned)kHbPidSlots ? 0u : sl + 1;
    }
    atomicAdd(pst + sl, (1ULL << 32) | kc[q]);
    const uint64_t p = x & t.pk_mask;
    if (RANGES) {
      rk[q] = atomicAdd(rcnt + (p >> kHbRangeBits), 1u);
    } else {
      int_hist_add(H, lbins, H_LINF, 0, kc[q]);
      const unsigned long long o = ord(ks[q]);
      mn = o < mn ? o : mn;
      mx = o > mx ? o : mx;
      pp[q] = atomicAdd(&fill, 1u);
      atomicAdd(pkstat + p, (1ULL << 32) | kc[q]);
      if (HAS_VALUE) atomicAdd(psum + p, ks[q]);
    }
  }
  __syncthreads();
  const int R = (int)t.hb_R;
  if (threadIdx.x < 64) {
    if (RANGES) {  // exclusive scan of the range counts by one wave
      const int lane = threadIdx.x;
      unsigned carry = 0;
      for (int b0 = 0; b0 < R; b0 += 64) {
        const unsigned hv = b0 + lane < R ? rcnt[b0 + lane] : 0u;
        unsigned incl = hv;
        for (int off = 1; off < 64; off <<= 1) {
          const unsigned up = __shfl_up(incl, off, 64);
          if (lane >= off) incl += up;
        }
        if (b0 + lane < R) rstart[b0 + lane] = carry + incl - hv;
        carry += __shfl(incl, 63, 64);
      }
      if (lane == 0) rstart[R] = carry;
    }
    if (!RANGES && threadIdx.x == 0) s_base = atomicAdd(ctl + 1, fill);  // this bucket's pair sums
  }
  __syncthreads();
  if (RANGES)
    for (int r = threadIdx.x; r <= R; r += blockDim.x) pruns[(int64_t)blockIdx.x * (R + 1) + r] = rstart[r];
#pragma unroll
  for (int q = 0; q < kHbPidPer; ++q) {
    if (kx[q] == ~0ULL) continue;
    const uint64_t p = kx[q] & t.pk_mask;
    if (RANGES) {
      PRec rec;
      rec.pk = (unsigned)p;
      rec.rows = kc[q];
      rec.sum = ks[q];
      prec[a + rstart[p >> kHbRangeBits] + rk[q]] = rec;
    } else {
      const unsigned long long at = (unsigned long long)s_base + pp[q];
      if (at < (unsigned long long)t.n) pairsum[at] = ks[q];
    }
  }
  for (int i = threadIdx.x; i < kHbPidSlots; i += blockDim.x) {
    const unsigned pid = pkey[i];
    if (pid != ~0u) pidstat[pid] = pst[i];
  }
  if (RANGES)  // the rest of the bucket's row span: no pair (k_h_float reads the span flat)
    for (int64_t j = a + rstart[R] + threadIdx.x; j < e; j += blockDim.x) prec[j].pk = ~0u;
  if (!RANGES) {
    flush_small(H, lbins, 0, H_LINF);
    block_minmax(mn, mx, minmax);  // contains __syncthreads (workgroup-uniform branch)
  }
}

size_t hb_pid_lds() { return (size_t)kHbPidSlots * 20; }

// step 7 (privacy-id buckets with ranges): workgroup (r, g) sums the records
// of partition range r over buckets [g * per, (g + 1) * per) in LDS -- per
// partition distinct pids, rows and value sum -- and flushes each partition
// with one packed atomic (+ one for the sum); each record is one pair, so its
// rows go to the Linf bins (LDS) and its sum to the pair-sum range.  A chunk
// of 1,024 buckets' runs is flattened by a workgroup scan, so every lane
// reads a record of the same runs (contiguous within a run).
template <bool HAS_VALUE>
__global__ void __launch_bounds__(kHbRangeThreads) k_hb_prange(HT t, const unsigned* __restrict__ bstart,
                                                               const unsigned* __restrict__ pruns,
                                                               const PRec* __restrict__ prec,
                                                               unsigned long long* pkstat, double* psum, IntHists H,
                                                               unsigned long long* minmax, int64_t per) {
  __shared__ unsigned an[kHbRangeW], ar[kHbRangeW];
  __shared__ unsigned lbins[kSmallBins];
  __shared__ double as[HAS_VALUE ? kHbRangeW : 1];
  __shared__ unsigned bex[kHbRangeThreads], bbase[kHbRangeThreads];
  __shared__ unsigned wsum[kHbRangeThreads / 64 + 1];
  const int64_t r = blockIdx.x, R = t.hb_R;
  for (int p = threadIdx.x; p < kHbRangeW; p += blockDim.x) {
    an[p] = 0;
    ar[p] = 0;
    if (HAS_VALUE) as[p] = 0.0;
  }
  for (int i = threadIdx.x; i < kSmallBins; i += blockDim.x) lbins[i] = 0;
  unsigned long long mn = ~0ULL, mx = 0ULL;
  const int64_t b0 = (int64_t)blockIdx.y * per;
  const int64_t b1 = b0 + per < t.nb ? b0 + per : t.nb;
  auto add = [&](const PRec& rec) {
    const unsigned p = rec.pk & (kHbRangeW - 1);
    atomicAdd(an + p, 1u);
    atomicAdd(ar + p, rec.rows);
    if (HAS_VALUE) atomicAdd(as + p, rec.sum);
    // Linf bins: the lanes holding the first active lane's value (most
    // pairs have one row) add once, the others one by one
    const unsigned long long act = __ballot(true);
    const unsigned r0 = __shfl(rec.rows, __ffsll((long long)act) - 1, 64);
    const unsigned long long same = __ballot(rec.rows == r0);
    if (rec.rows != r0) int_hist_add(H, lbins, H_LINF, 0, rec.rows);
    else if ((int)(threadIdx.x & 63) == __ffsll((long long)same) - 1) int_hist_add_n(H, lbins, H_LINF, 0, r0, __popcll(same));
    const unsigned long long o = ord(rec.sum);
    mn = o < mn ? o : mn;
    mx = o > mx ? o : mx;
  };
#if PDP_HB_RANGE_WAVE
  // each wave takes 64 buckets' runs of range r: lane i loads bucket i's run
  // bounds (one latency round), then the wave reads kHbRangeU runs at a time,
  // one record per lane (a run averages a few dozen records), loads
  // unconditional -- no per-record search for its run
  __syncthreads();  // the LDS clears above
  const int lane = threadIdx.x & 63;
  const int64_t nwv = blockDim.x >> 6;
  for (int64_t c0 = b0 + (int64_t)(threadIdx.x >> 6) * 64; c0 < b1; c0 += nwv * 64) {  // wave-uniform
    const int64_t b = c0 + lane;
    unsigned mybase = 0, mylen = 0;
    if (b < b1) {
      const unsigned s0 = pruns[b * (R + 1) + r], s1 = pruns[b * (R + 1) + r + 1];
      const unsigned rows = bstart[b + 1] - bstart[b];
      if (s0 <= s1 && s1 <= rows) {  // a bucket's records lie inside its rows
        mybase = bstart[b] + s0;
        mylen = s1 - s0;
      }
    }
    for (int j = 0; j < 64; j += kHbRangeU) {
      unsigned bs[kHbRangeU], ln[kHbRangeU], top = 0;
#pragma unroll
      for (int u = 0; u < kHbRangeU; ++u) {
        bs[u] = __shfl(mybase, j + u, 64);
        ln[u] = __shfl(mylen, j + u, 64);
        top = ln[u] > top ? ln[u] : top;
      }
      for (unsigned k0 = 0; k0 < top; k0 += 64) {  // wave-uniform
        PRec recs[kHbRangeU];
#pragma unroll
        for (int u = 0; u < kHbRangeU; ++u) recs[u] = prec[k0 + lane < ln[u] ? bs[u] + k0 + lane : bs[u]];
#pragma unroll
        for (int u = 0; u < kHbRangeU; ++u)
          if (k0 + lane < ln[u]) add(recs[u]);
      }
    }
  }
  __syncthreads();
#else
  for (int64_t c0 = b0; c0 < b1; c0 += kHbRangeThreads) {  // workgroup-uniform
    const int64_t b = c0 + threadIdx.x;
    unsigned len = 0, base = 0;
    if (b < b1) {
      const unsigned s = pruns[b * (R + 1) + r], s1 = pruns[b * (R + 1) + r + 1];
      const unsigned rows = bstart[b + 1] - bstart[b];
      if (s <= s1 && s1 <= rows) {  // a bucket's records lie inside its rows
        base = bstart[b] + s;
        len = s1 - s;
      }
    }
    unsigned tot;
    const unsigned ex = hb_block_scan(len, wsum, &tot);  // its barriers also order the LDS clears
    bex[threadIdx.x] = ex;
    bbase[threadIdx.x] = base;
    __syncthreads();
    // kHbRangeU records per thread in flight (one memory latency per batch)
    for (unsigned f0 = threadIdx.x; f0 < tot; f0 += kHbRangeU * blockDim.x) {
      PRec recs[kHbRangeU];
#pragma unroll
      for (int u = 0; u < kHbRangeU; ++u) {
        const unsigned f = f0 + u * blockDim.x;
        if (f >= tot) break;
        int lo = 0, hi = kHbRangeThreads;  // the last run starting at or before f
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (bex[mid] <= f) lo = mid;
          else hi = mid;
        }
        recs[u] = prec[bbase[lo] + (f - bex[lo])];
      }
#pragma unroll
      for (int u = 0; u < kHbRangeU; ++u) {
        if (f0 + u * blockDim.x >= tot) break;
        add(recs[u]);
      }
    }
    __syncthreads();
  }
#endif
  block_minmax(mn, mx, minmax);  // contains __syncthreads
  __syncthreads();
  flush_small(H, lbins, 0, H_LINF);
  for (int p = threadIdx.x; p < kHbRangeW; p += blockDim.x) {
    const unsigned n = an[p];
    if (!n) continue;
    const int64_t g = r * kHbRangeW + p;
    atomicAdd(pkstat + g, ((unsigned long long)n << 32) | ar[p]);
    if (HAS_VALUE) atomicAdd(psum + g, as[p]);
  }
}

// ------------------------------------------------------ pre-aggregated input --
// compute_dataset_histograms_on_preaggregated_data (computing_histograms.py:
// 713-758): one row per (privacy id, partition) pair holding (count, sum,
// n_partitions, n_contributions), as analysis/pre_aggregation.py:19-58 emits
// them.  The pairs are given, so there is no pair table:
//   k_hp_rows     per row: Linf bin of count; per partition (rows, count sum,
//                 value sum) by atomics; min / max of the row sums; the L0 /
//                 L1 weights 1 / n_partitions summed per distinct value
//                 (values < 1000 in LDS, larger ones in an open-addressing
//                 table keyed by value)
//   k_hp_weights  per distinct value: count = round half to even of the
//                 weight sum (_compute_weighted_frequency_histogram :81-102)
//                 into its bin; the bin exists (max = value) even at count 0
//   k_hp_ids, k_h_lowers, k_hp_float, k_h_final  as for raw rows
constexpr int kWSmall = 1000;  // L0 / L1 values below this: dense LDS weight sums

struct WSlot {  // key = value * 2 + histogram + 1 (0 = empty)
  unsigned long long key;
  double w;
};

uint64_t wtab_capacity(int64_t n_rows) {
  uint64_t c = 2 * (uint64_t)n_rows;
  c = (c + 255) & ~(uint64_t)255;
  return c < kMinTable ? kMinTable : c;
}

struct PWs {
  uint64_t err, pkrows, pkcount, psum, minmax, fmax, wsmall, wtab, total;
};

PWs playout(int64_t n, int64_t P) {
  PWs w{};
  uint64_t off = 0;
  w.err = off; off = align256(off + 16);
  w.pkrows = off; off = align256(off + (uint64_t)P * 8);
  w.pkcount = off; off = align256(off + (uint64_t)P * 8);
  w.psum = off; off = align256(off + (uint64_t)P * 8);
  w.minmax = off; off = align256(off + 4 * 8);
  w.fmax = off; off = align256(off + 2 * kSumBuckets * 8);
  w.wsmall = off; off = align256(off + 2 * kWSmall * 8);
  w.wtab = off; off = align256(off + wtab_capacity(n) * sizeof(WSlot));
  w.total = off;
  return w;
}

struct PT {
  int64_t n, P;
  uint64_t cap;  // weight-table slots
  int do_parts;
};

// weight w of histogram h's value v: dense LDS sums below kWSmall, else the
// table (plain load first, CAS only on an empty slot, linear probing)
__device__ __forceinline__ void weight_add(double* lw, WSlot* tab, uint64_t cap, int h, uint64_t v, double w) {
  if (v < (uint64_t)kWSmall) {
    atomicAdd(lw + h * kWSmall + (int)v, w);
    return;
  }
  const unsigned long long x = v * 2 + (uint64_t)h + 1;
  uint64_t s = __umul64hi(mix64(x), cap);
  for (;;) {
    unsigned long long* k = &tab[s].key;
    const unsigned long long cur = *k;
    if (cur == 0) {
      const unsigned long long old = atomicCAS(k, 0ULL, x);
      if (old == 0 || old == x) break;
    } else if (cur == x) {
      break;
    }
    s = s + 1 == cap ? 0 : s + 1;  // cap >= 2 * rows > distinct values: a free slot always exists
  }
  atomicAdd(&tab[s].w, w);
}

__global__ void __launch_bounds__(kBlock) k_hp_rows(PT t, const int64_t* __restrict__ pk,
                                                    const int64_t* __restrict__ count,
                                                    const double* __restrict__ sum,
                                                    const int64_t* __restrict__ npart,
                                                    const int64_t* __restrict__ ncontr, unsigned long long* pkrows,
                                                    unsigned long long* pkcount, double* psum, IntHists H,
                                                    unsigned long long* minmax, double* wsmall, WSlot* wtab,
                                                    unsigned* err) {
  __shared__ unsigned lcnt[kSmallBins];
  __shared__ double lw[2 * kWSmall];
  for (int b = threadIdx.x; b < kSmallBins; b += blockDim.x) lcnt[b] = 0;
  for (int b = threadIdx.x; b < 2 * kWSmall; b += blockDim.x) lw[b] = 0.0;
  __syncthreads();
  constexpr int64_t kMaxV = (int64_t)1 << 62;
  unsigned long long mn = ~0ULL, mx = 0ULL;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n; i += stride) {
    const int64_t p = pk[i], c = count[i], np = npart[i], nc = ncontr[i];
    if (p < 0 || p >= t.P) {
      atomicOr(err, 1u);
      continue;
    }
    if (c < 1 || np < 1 || nc < 1 || c >= kMaxV || np >= kMaxV || nc >= kMaxV) {
      atomicOr(err, 2u);
      continue;
    }
    const double s = sum[i];
    int_hist_add(H, lcnt, H_LINF, 0, (unsigned long long)c);
    atomicAdd(pkrows + p, 1ULL);
    atomicAdd(pkcount + p, (unsigned long long)c);
    atomicAdd(psum + p, s);
    const unsigned long long o = ord(s);
    mn = o < mn ? o : mn;
    mx = o > mx ? o : mx;
    const double w = __ddiv_rn(1.0, (double)np);  // 1.0 / x[2] (:536-541, :560-565)
    weight_add(lw, wtab, t.cap, H_L0, (uint64_t)np, w);
    weight_add(lw, wtab, t.cap, H_L1, (uint64_t)nc, w);
  }
  block_minmax(mn, mx, minmax);  // contains __syncthreads: every thread reaches it
  __syncthreads();
  flush_small(H, lcnt, 0, H_LINF);
  for (int b = threadIdx.x; b < 2 * kWSmall; b += blockDim.x)
    if (lw[b] != 0.0) atomicAdd(wsmall + b, lw[b]);
}

__device__ __forceinline__ void weight_bin_add(const IntHists& H, unsigned long long key, double weight);

// int(round(sum of weights)) per distinct value (:94-97), into its bin
__global__ void __launch_bounds__(kBlock) k_hp_weights(const double* __restrict__ wsmall,
                                                       const WSlot* __restrict__ wtab, uint64_t cap, IntHists H) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 2 * kWSmall) {
    const double w = wsmall[i];
    if (w > 0.0) {  // weights are positive: the value occurs
      const int h = (int)(i / kWSmall);
      const unsigned long long v = (unsigned long long)(i % kWSmall);
      const unsigned long long f = (unsigned long long)rint(w);
      const int64_t g = (int64_t)h * kLogBins + (int64_t)v;  // width-1 bin: this value alone
      H.count[g] = f;
      H.sum[g] = f * v;
      H.max[g] = v;
    }
    return;
  }
  const int64_t j = i - 2 * kWSmall;
  if (j >= (int64_t)cap) return;
  const WSlot s = wtab[j];
  weight_bin_add(H, s.key, s.w);
}

// a weight-table entry (key = value * 2 + histogram + 1, 0 = none) into its
// logarithmic bin: int(round(weight)) elements of that value; the bin exists
// (max = value) even when the weight rounds to 0
__device__ __forceinline__ void weight_bin_add(const IntHists& H, unsigned long long key, double weight) {
  if (key == 0) return;
  const unsigned long long x = key - 1;
  const int h = (int)(x & 1);
  const unsigned long long v = x >> 1;
  const unsigned long long f = (unsigned long long)rint(weight);
  const int64_t g = (int64_t)h * kLogBins + log_bin_index(v);
  if (f) {
    atomicAdd(H.count + g, f);
    atomicAdd(H.sum + g, f * v);
  }
  atomicMax(H.max + g, v);
}

// pdp_dataset_histograms_weight_bins: an explicit (key, weight) list, e.g.
// the global weight sums a rank owns after the multi-rank exchange
__global__ void __launch_bounds__(kBlock) k_hp_weight_list(const unsigned long long* __restrict__ keys,
                                                           const double* __restrict__ weights, int64_t n,
                                                           IntHists H) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) weight_bin_add(H, keys[i], weights[i]);
}

// per partition with rows: COUNT_PER_PARTITION (sum of counts),
// PRIVACY_ID_PER_PARTITION (rows), min / max of the partition sums
__global__ void __launch_bounds__(kBlock) k_hp_ids(PT t, const unsigned long long* __restrict__ pkrows,
                                                   const unsigned long long* __restrict__ pkcount,
                                                   const double* __restrict__ psum, IntHists H,
                                                   unsigned long long* minmax) {
  __shared__ unsigned lds[2 * kSmallBins];
  for (int b = threadIdx.x; b < 2 * kSmallBins; b += blockDim.x) lds[b] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned long long mn = ~0ULL, mx = 0ULL;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.P; i += stride) {
    const unsigned long long r = pkrows[i];
    if (r == 0) continue;
    int_hist_add(H, lds, H_COUNT, 0, pkcount[i]);
    int_hist_add(H, lds, H_PIDS, 1, r);
    const unsigned long long o = ord(psum[i]);
    mn = o < mn ? o : mn;
    mx = o > mx ? o : mx;
  }
  block_minmax(mn, mx, minmax + 2);
  __syncthreads();
  flush_small(H, lds, 0, H_COUNT);
  flush_small(H, lds, 1, H_PIDS);
}

// Linf-sum histogram over the rows' sums (LDS-privatised counts and sums),
// sum-per-partition histogram over the partitions with rows
__global__ void __launch_bounds__(kFloatBlock) k_hp_float(PT t, const double* __restrict__ sum,
                                                          const unsigned long long* __restrict__ pkrows,
                                                          const double* __restrict__ psum,
                                                          const double* __restrict__ lowers,
                                                          const int* __restrict__ n_lowers, FloatHists F) {
  __shared__ unsigned lcnt[kSumBuckets];
  __shared__ double lsum[kSumBuckets];
  for (int b = threadIdx.x; b < kSumBuckets; b += blockDim.x) {
    lcnt[b] = 0;
    lsum[b] = 0.0;
  }
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int nl0 = n_lowers[F_LINF_SUM], nl1 = n_lowers[F_PART_SUM];
  if (nl0 > 0) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n; i += stride) {
      const double v = sum[i];
      const int b = float_bin(lowers, nl0, v);
      atomicAdd(lcnt + b, 1u);
      atomicAdd(lsum + b, v);
      max_filtered(F.omax + b, ord(v));
    }
  }
  if (t.do_parts && nl1 > 0) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.P; i += stride) {
      if (pkrows[i] == 0) continue;
      const double v = psum[i];
      const int64_t g = (int64_t)F_PART_SUM * kSumBuckets + float_bin(lowers + kNLowers, nl1, v);
      atomicAdd(F.count + g, 1ULL);
      atomicAdd(F.sum + g, v);
      max_filtered(F.omax + g, ord(v));
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kSumBuckets; b += blockDim.x) {
    const unsigned c = lcnt[b];
    if (c) {
      atomicAdd(F.count + b, (unsigned long long)c);
      atomicAdd(F.sum + b, lsum[b]);
    }
  }
}

#define PDP_HLAUNCH(name, st, ...)          \
  do {                                      \
    PDP_PROF_BEGIN(name, st);               \
    hipLaunchKernelGGL(__VA_ARGS__);        \
    PDP_PROF_END(st);                       \
    PDP_HIP_CHECK(hipGetLastError());       \
  } while (0)

}  // namespace
}  // namespace pdp

extern "C" {

int pdp_dataset_histograms_workspace_bytes(int64_t n_rows, int64_t n_privacy_ids, int64_t n_partitions,
                                           uint64_t* bytes) {
  if (bytes == nullptr) return pdp::set_error(PDP_E_INVALID, "NULL argument");
  if (n_rows < 0 || n_privacy_ids < 0 || n_partitions < 0)
    return pdp::set_error(PDP_E_INVALID, "sizes must be >= 0");
  *bytes = pdp::hlayout(n_rows, n_privacy_ids, n_partitions).total;
  return PDP_OK;
}

}  // extern "C"

namespace pdp {
namespace {

struct HCall {
  HWs w;
  HT t;
  char* ws;
  hipStream_t st;
  IntHists H;
  FloatHists F;
};

int hist_check(int32_t value_kind, int64_t n_rows, int64_t n_privacy_ids, int64_t n_partitions,
               const pdp_histogram_bins* out, void* workspace, uint64_t workspace_bytes, void* stream, HCall* c) {
  if (out == nullptr || out->int_count == nullptr || out->int_sum == nullptr || out->int_max == nullptr ||
      out->float_count == nullptr || out->float_sum == nullptr || out->float_max == nullptr ||
      out->float_lowers == nullptr || out->float_n_lowers == nullptr)
    return set_error(PDP_E_INVALID, "every pdp_histogram_bins output must be set");
  if (n_rows < 0 || n_privacy_ids < 0 || n_partitions < 0) return set_error(PDP_E_INVALID, "sizes must be >= 0");
  if (n_rows >= (int64_t)1 << 31) return set_error(PDP_E_UNSUPPORTED, "n_rows must be < 2^31 per shard");
  value_kind &= ~(PDP_HIST_FORCE_PAIR_TABLE | PDP_HIST_FORCE_PAIR_HASH);
  if (value_kind != PDP_VALUE_NONE && value_kind != PDP_VALUE_F64 && value_kind != PDP_VALUE_I64)
    return set_error(PDP_E_INVALID, "bad value_kind");
  if (bits_for(n_privacy_ids) + bits_for(n_partitions) > 63)
    return set_error(PDP_E_UNSUPPORTED, "pair key (privacy id bits + partition bits) exceeds 63 bits");
  c->w = hlayout(n_rows, n_privacy_ids, n_partitions);
  if (workspace == nullptr || workspace_bytes < c->w.total)
    return set_error(PDP_E_INVALID, "workspace smaller than pdp_dataset_histograms_workspace_bytes");
  c->ws = (char*)workspace;
  c->st = (hipStream_t)stream;
  HT& t = c->t;
  t.n = n_rows;
  t.U = n_privacy_ids;
  t.P = n_partitions;
  t.pk_bits = bits_for(n_partitions);
  t.cap = slots_capacity(n_rows, n_partitions);
  t.R = n_regions(n_partitions);
  t.has_value = value_kind != PDP_VALUE_NONE;
  t.do_parts = 1;
  t.pk_mask = (1ULL << t.pk_bits) - 1;
  t.nb = hb_buckets(n_rows);
  t.n_supers = (t.nb + kHbFan - 1) / kHbFan;
  t.n_tiles = (n_rows + kHbTileRows - 1) / kHbTileRows;
  c->H = IntHists{(unsigned long long*)out->int_count, (unsigned long long*)out->int_sum,
                  (unsigned long long*)out->int_max};
  c->F = FloatHists{(unsigned long long*)out->float_count, out->float_sum, (unsigned long long*)(c->ws + c->w.fmax)};
  return PDP_OK;
}

// the bucketed pairs phase (k_hb_*): pair-hash partition in two levels, then
// one LDS pair table per bucket; sets hb_ctl = {1, pairs, overflow}
int hist_pairs_bucketed(const HCall& c, const int64_t* privacy_id, const int64_t* partition, const void* value,
                        int32_t value_kind, bool pid_buckets) {
  const HWs& w = c.w;
  HT t = c.t;
  t.hb_pid = pid_buckets ? 1 : 0;
  t.hb_R = pid_buckets && w.hb_pruns ? hb_ranges(t.P) : 0;
  char* ws = c.ws;
  hipStream_t st = c.st;
  unsigned* err = (unsigned*)(ws + w.err);
  unsigned* cts = (unsigned*)(ws + w.hb_cts);
  unsigned* sbase = (unsigned*)(ws + w.hb_sbase);
  unsigned* bcnt = (unsigned*)(ws + w.hb_bcnt);
  unsigned* bcur = (unsigned*)(ws + w.hb_bcur);
  unsigned* ctl = (unsigned*)(ws + w.hb_ctl);
  // level-1 and level-2 records in the pair-table region (>= 48 bytes per row)
  unsigned long long* key1 = (unsigned long long*)(ws + w.slots);
  double* val1 = (double*)(key1 + t.n);
  unsigned long long* key2 = (unsigned long long*)(val1 + t.n);
  double* val2 = (double*)(key2 + t.n);
  const bool hv = value_kind != PDP_VALUE_NONE;
  PDP_HLAUNCH("k_hb_count", st, k_hb_count, dim3((unsigned)t.n_tiles), dim3(kHbThreads), 0, st, t, privacy_id,
              partition, cts, err);
  PDP_HLAUNCH("k_hb_scan_tiles", st, k_hb_scan_tiles, dim3((unsigned)t.n_supers), dim3(kHbThreads), 0, st, t, cts,
              sbase);
  PDP_HLAUNCH("k_hb_scan_supers", st, k_hb_scan_supers, dim3(1), dim3(kHbFan), 0, st, t, sbase);
  const size_t lds1 = hb_l1_lds(value_kind);
  const void* l1 = value_kind == PDP_VALUE_F64 ? (const void*)k_hb_l1<PDP_VALUE_F64>
                   : value_kind == PDP_VALUE_I64 ? (const void*)k_hb_l1<PDP_VALUE_I64>
                                                 : (const void*)k_hb_l1<PDP_VALUE_NONE>;
  PDP_HIP_CHECK(hipFuncSetAttribute(l1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1));
  {
    const HT tt = t;
    const unsigned* cts_c = cts;
    const unsigned* sbase_c = sbase;
    void* args[] = {(void*)&tt, (void*)&privacy_id, (void*)&partition, (void*)&value, (void*)&cts_c,
                    (void*)&sbase_c, (void*)&key1, (void*)&val1};
    PDP_PROF_BEGIN("k_hb_l1", st);
    PDP_HIP_CHECK(hipLaunchKernel(l1, dim3((unsigned)t.n_tiles), dim3(kHbThreads), args, lds1, st));
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
  }
  PDP_HIP_CHECK(hipMemsetAsync(bcnt, 0, (uint64_t)(t.nb + 1) * 4, st));
  PDP_HIP_CHECK(hipMemsetAsync(bcur, 0, (uint64_t)t.nb * 4, st));
  const unsigned g2 = (unsigned)(t.n_supers * kHbK);
  PDP_HLAUNCH("k_hb_bcount", st, k_hb_bcount, dim3(g2), dim3(kHbL2Threads), 0, st, t, (const unsigned*)sbase,
              (const unsigned long long*)key1, bcnt);
  const int rc = scan_u32(bcnt, t.nb, (unsigned*)(ws + w.hb_bchunks), st);  // -> bucket starts
  if (rc != PDP_OK) return rc;
  if (hv)
    PDP_HLAUNCH("k_hb_l2", st, k_hb_l2<true>, dim3(g2), dim3(kHbL2Threads), 0, st, t, (const unsigned*)sbase,
                (const unsigned long long*)key1, (const double*)val1, (const unsigned*)bcnt, bcur, key2, val2);
  else
    PDP_HLAUNCH("k_hb_l2", st, k_hb_l2<false>, dim3(g2), dim3(kHbL2Threads), 0, st, t, (const unsigned*)sbase,
                (const unsigned long long*)key1, (const double*)val1, (const unsigned*)bcnt, bcur, key2, val2);
  // mode: 1 = pair-sum list, 2 = privacy-id buckets' range-grouped records (+ R in word 3)
  PDP_HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)ctl, pid_buckets && t.hb_R ? 2u : 1u, 1, st));
  if (pid_buckets && t.hb_R) PDP_HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)(ctl + 3), (unsigned)t.hb_R, 1, st));
  unsigned long long* pidstat = (unsigned long long*)(ws + w.pidstat);
  unsigned long long* pkstat = (unsigned long long*)(ws + w.pkstat);
  double* psum = (double*)(ws + w.psum);
  unsigned long long* minmax = (unsigned long long*)(ws + w.minmax);
  double* pairsum = (double*)(ws + w.hb_pairsum);
  if (pid_buckets) {
    PRec* prec = (PRec*)key1;  // level-1 records are dead after level 2 (16 bytes per row)
    unsigned* pruns = t.hb_R ? (unsigned*)(ws + w.hb_pruns) : nullptr;
    const size_t lds = hb_pid_lds();
    const void* f = hv ? (t.hb_R ? (const void*)k_hb_pid_pairs<true, true> : (const void*)k_hb_pid_pairs<true, false>)
                       : (t.hb_R ? (const void*)k_hb_pid_pairs<false, true> : (const void*)k_hb_pid_pairs<false, false>);
    PDP_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    {
      const HT tt = t;
      const unsigned* bst = bcnt;
      const unsigned long long* k2 = key2;
      const double* v2 = val2;
      IntHists HH = c.H;
      void* args[] = {(void*)&tt,     (void*)&bst,    (void*)&k2,      (void*)&v2,    (void*)&pidstat,
                      (void*)&pkstat, (void*)&psum,   (void*)&HH,      (void*)&minmax, (void*)&pairsum,
                      (void*)&prec,   (void*)&pruns,  (void*)&ctl};
      PDP_PROF_BEGIN("k_hb_pid_pairs", st);
      PDP_HIP_CHECK(hipLaunchKernel(f, dim3((unsigned)t.nb), dim3(kHbPidThreads), args, lds, st));
      PDP_PROF_END(st);
      PDP_HIP_CHECK(hipGetLastError());
    }
    if (t.hb_R) {
      // ~1,024 workgroups: R ranges x G slices of the buckets
      int64_t G = 1024 / t.hb_R;
      G = G < 1 ? 1 : G;
      const int64_t per = (t.nb + G - 1) / G;
      G = (t.nb + per - 1) / per;
      const PRec* pr = prec;
      if (hv)
        PDP_HLAUNCH("k_hb_prange", st, k_hb_prange<true>, dim3((unsigned)t.hb_R, (unsigned)G), dim3(kHbRangeThreads),
                    0, st, t, (const unsigned*)bcnt, (const unsigned*)pruns, pr, pkstat, psum, c.H, minmax, per);
      else
        PDP_HLAUNCH("k_hb_prange", st, k_hb_prange<false>, dim3((unsigned)t.hb_R, (unsigned)G), dim3(kHbRangeThreads),
                    0, st, t, (const unsigned*)bcnt, (const unsigned*)pruns, pr, pkstat, psum, c.H, minmax, per);
    }
    return PDP_OK;
  }
  if (hv)
    PDP_HLAUNCH("k_hb_pairs", st, k_hb_pairs<true>, dim3((unsigned)t.nb), dim3(kHbPairThreads), 0, st, t,
                (const unsigned*)bcnt, (const unsigned long long*)key2, (const double*)val2, pidstat, pkstat, psum,
                c.H, minmax, pairsum, ctl);
  else
    PDP_HLAUNCH("k_hb_pairs", st, k_hb_pairs<false>, dim3((unsigned)t.nb), dim3(kHbPairThreads), 0, st, t,
                (const unsigned*)bcnt, (const unsigned long long*)key2, (const double*)val2, pidstat, pkstat, psum,
                c.H, minmax, pairsum, ctl);
  return PDP_OK;
}

// zero everything; k_h_rows + k_h_pairs (pair table, per-pid / per-partition
// statistics, Linf histogram, pair-sum min / max)
int hist_pairs(const HCall& c, const int64_t* privacy_id, const int64_t* partition, const void* value,
               int32_t value_kind, const pdp_histogram_bins* out) {
  const HWs& w = c.w;
  const HT& t = c.t;
  char* ws = c.ws;
  hipStream_t st = c.st;
  const bool force_table = (value_kind & PDP_HIST_FORCE_PAIR_TABLE) != 0;
  const bool force_hash = (value_kind & PDP_HIST_FORCE_PAIR_HASH) != 0;
  value_kind &= ~(PDP_HIST_FORCE_PAIR_TABLE | PDP_HIST_FORCE_PAIR_HASH);
  const bool bucketed = !force_table && hb_eligible(t.n);
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.err, 0, 16, st));
  // the pair table (slots .. region scan) only for its own path; the per-pid
  // and per-partition statistics for both
  if (!bucketed) PDP_HIP_CHECK(hipMemsetAsync(ws + w.slots, 0, w.pidstat - w.slots, st));
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.pidstat, 0, w.minmax - w.pidstat, st));  // pidstat .. psum
  PDP_HLAUNCH("k_h_init", st, k_h_init, dim3(1), dim3(64), 0, st, (unsigned long long*)(ws + w.minmax));
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.fmax, 0, 2 * kSumBuckets * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(out->int_count, 0, 5 * kLogBins * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(out->int_sum, 0, 5 * kLogBins * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(out->int_max, 0, 5 * kLogBins * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(out->float_count, 0, 2 * kSumBuckets * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(out->float_sum, 0, 2 * kSumBuckets * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(out->float_lowers, 0, 2 * kNLowers * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.hb_ctl, 0, 16, st));
  if (t.n == 0) return PDP_OK;
  if (privacy_id == nullptr || partition == nullptr || (value_kind != PDP_VALUE_NONE && value == nullptr))
    return set_error(PDP_E_INVALID, "NULL column");
  if (bucketed) {
    // privacy-id buckets first (pids < 2^32 - 1), then pair buckets, then
    // the pair table: a bucket whose distinct pairs overflow its LDS table
    // (a privacy id with thousands of partitions; crafted keys) sends the
    // whole call to the next one, from scratch
    const bool pid_ok = !force_hash && t.U <= (int64_t)0xFFFFFFFFLL;
    for (int attempt = pid_ok ? 0 : 1; attempt < 2; ++attempt) {
      const int rc = hist_pairs_bucketed(c, privacy_id, partition, value, value_kind, attempt == 0);
      if (rc != PDP_OK) return rc;
      unsigned over = 0;
      PDP_HIP_CHECK(hipMemcpyAsync(&over, ws + w.hb_ctl + 8, 4, hipMemcpyDeviceToHost, st));
      PDP_HIP_CHECK(hipStreamSynchronize(st));
      if (!over) return PDP_OK;
      PDP_HIP_CHECK(hipMemsetAsync(ws + w.hb_ctl, 0, 16, st));
      PDP_HLAUNCH("k_h_init", st, k_h_init, dim3(1), dim3(64), 0, st, (unsigned long long*)(ws + w.minmax));
      PDP_HIP_CHECK(hipMemsetAsync(out->int_count, 0, 5 * kLogBins * 8, st));
      PDP_HIP_CHECK(hipMemsetAsync(out->int_sum, 0, 5 * kLogBins * 8, st));
      PDP_HIP_CHECK(hipMemsetAsync(out->int_max, 0, 5 * kLogBins * 8, st));
      PDP_HIP_CHECK(hipMemsetAsync(ws + w.pidstat, 0, w.minmax - w.pidstat, st));  // pidstat .. psum
    }
    PDP_HIP_CHECK(hipMemsetAsync(ws + w.slots, 0, w.pidstat - w.slots, st));  // the pair table
  }
  Slot* slots = (Slot*)(ws + w.slots);
  unsigned* err = (unsigned*)(ws + w.err);
  unsigned* rbase = (unsigned*)(ws + w.rbase);
  const unsigned g = grid_for(t.n);
  if (t.R <= kRegionLdsMax)
    PDP_HLAUNCH("k_h_region_count", st, k_h_region_count<true>, dim3(grid_for(t.n, 1024)), dim3(kBlock), 0, st, t,
                privacy_id, partition, rbase);
  else
    PDP_HLAUNCH("k_h_region_count", st, k_h_region_count<false>, dim3(g), dim3(kBlock), 0, st, t, privacy_id,
                partition, rbase);
  PDP_HLAUNCH("k_h_region_caps", st, k_h_region_caps, dim3(grid_for(t.R)), dim3(kBlock), 0, st, t.R, rbase);
  {
    const int rc = scan_u32(rbase, t.R, (unsigned*)(ws + w.rchunks), st);
    if (rc != PDP_OK) return rc;
  }
  switch (value_kind) {
    case PDP_VALUE_F64:
      PDP_HLAUNCH("k_h_rows", st, k_h_rows<PDP_VALUE_F64>, dim3(g), dim3(kBlock), 0, st, t, privacy_id, partition,
                  value, rbase, slots, err);
      break;
    case PDP_VALUE_I64:
      PDP_HLAUNCH("k_h_rows", st, k_h_rows<PDP_VALUE_I64>, dim3(g), dim3(kBlock), 0, st, t, privacy_id, partition,
                  value, rbase, slots, err);
      break;
    default:
      PDP_HLAUNCH("k_h_rows", st, k_h_rows<PDP_VALUE_NONE>, dim3(g), dim3(kBlock), 0, st, t, privacy_id, partition,
                  value, rbase, slots, err);
  }
  const int64_t n_chunks = ((int64_t)t.cap + kPairsChunk - 1) / kPairsChunk;  // upper bound of the used slots
  PDP_HLAUNCH("k_h_pairs", st, k_h_pairs, dim3((unsigned)n_chunks), dim3(kPairsBlock), 0, st, t, slots, rbase,
              (unsigned long long*)(ws + w.pidstat), (unsigned long long*)(ws + w.pkstat), (double*)(ws + w.psum),
              c.H, (unsigned long long*)(ws + w.minmax));
  return PDP_OK;
}

// k_h_ids (partition part only when t.do_parts), lowers, float bins, final
int hist_finish(const HCall& c, const pdp_histogram_bins* out) {
  const HWs& w = c.w;
  const HT& t = c.t;
  char* ws = c.ws;
  hipStream_t st = c.st;
  unsigned long long* minmax = (unsigned long long*)(ws + w.minmax);
  const unsigned long long* pkstat = (const unsigned long long*)(ws + w.pkstat);
  const double* psum = (const double*)(ws + w.psum);
  const int64_t m = t.U > t.P ? t.U : t.P;
  if (m > 0)
    // at most 256 workgroups: each flushes its small bins with one global
    // atomic per bin, and 2,048 of them made those flushes most of the kernel
    PDP_HLAUNCH("k_h_ids", st, k_h_ids, dim3((unsigned)((m + kIdsThreads - 1) / kIdsThreads < 256 ? (m + kIdsThreads - 1) / kIdsThreads : 256)), dim3(kIdsThreads), 0, st, t,
                (const unsigned long long*)(ws + w.pidstat), pkstat, psum, c.H, minmax);
  PDP_HLAUNCH("k_h_lowers", st, k_h_lowers, dim3((kNLowers + kBlock - 1) / kBlock, 2), dim3(kBlock), 0, st, minmax,
              out->float_lowers, out->float_n_lowers);
  // one 1024-thread workgroup per CU (120 KB of LDS each)
  int dev = 0, cus = 256;
  PDP_HIP_CHECK(hipGetDevice(&dev));
  PDP_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int64_t mf = (int64_t)t.cap > t.P ? (int64_t)t.cap : t.P;
  int64_t gf = (mf + kFloatBlock - 1) / kFloatBlock;
  gf = gf < cus ? gf : cus;
  const Slot* fslots = (const Slot*)(ws + w.slots);
  const double* fpairsum = (const double*)(w.hb_pairsum ? ws + w.hb_pairsum : nullptr);
  const unsigned* fctl = (const unsigned*)(ws + w.hb_ctl);
  const unsigned* fbstart = (const unsigned*)(w.hb_bcnt ? ws + w.hb_bcnt : nullptr);
  const PRec* fprec = (const PRec*)(ws + w.slots);
  PDP_HLAUNCH("k_h_float", st, k_h_float<false>, dim3((unsigned)gf), dim3(kFloatBlock), 0, st, t, fslots, fpairsum,
              fctl, fbstart, fprec, pkstat, psum, out->float_lowers, out->float_n_lowers, c.F);
  PDP_HLAUNCH("k_h_float_max", st, k_h_float<true>, dim3((unsigned)gf), dim3(kFloatBlock), 0, st, t, fslots,
              fpairsum, fctl, fbstart, fprec, pkstat, psum, out->float_lowers, out->float_n_lowers, c.F);
  PDP_HLAUNCH("k_h_final", st, k_h_final, dim3((2 * kSumBuckets + kBlock - 1) / kBlock), dim3(kBlock), 0, st, c.H,
              c.F, out->float_max, 0x1F);
  return PDP_OK;
}

}  // namespace
}  // namespace pdp

extern "C" {

int pdp_dataset_histograms(const int64_t* privacy_id, const int64_t* partition, const void* value,
                           int32_t value_kind, int64_t n_rows, int64_t n_privacy_ids, int64_t n_partitions,
                           const pdp_histogram_bins* out, void* workspace, uint64_t workspace_bytes,
                           void* stream) {
  pdp::HCall c;
  int rc = pdp::hist_check(value_kind, n_rows, n_privacy_ids, n_partitions, out, workspace, workspace_bytes, stream,
                           &c);
  if (rc == PDP_OK) rc = pdp::hist_pairs(c, privacy_id, partition, value, value_kind, out);
  if (rc == PDP_OK) rc = pdp::hist_finish(c, out);
  return rc;
}

int pdp_dataset_histograms_pairs(const int64_t* privacy_id, const int64_t* partition, const void* value,
                                 int32_t value_kind, int64_t n_rows, int64_t n_privacy_ids, int64_t n_partitions,
                                 const pdp_histogram_bins* out, void* workspace, uint64_t workspace_bytes,
                                 void* stream) {
  pdp::HCall c;
  int rc = pdp::hist_check(value_kind, n_rows, n_privacy_ids, n_partitions, out, workspace, workspace_bytes, stream,
                           &c);
  return rc == PDP_OK ? pdp::hist_pairs(c, privacy_id, partition, value, value_kind, out) : rc;
}

int pdp_dataset_histograms_exchange_offsets(int64_t n_rows, int64_t n_privacy_ids, int64_t n_partitions,
                                            uint64_t* pkstat, uint64_t* psum, uint64_t* minmax) {
  if (pkstat == nullptr || psum == nullptr || minmax == nullptr) return pdp::set_error(PDP_E_INVALID, "NULL argument");
  if (n_rows < 0 || n_privacy_ids < 0 || n_partitions < 0)
    return pdp::set_error(PDP_E_INVALID, "sizes must be >= 0");
  const pdp::HWs w = pdp::hlayout(n_rows, n_privacy_ids, n_partitions);
  *pkstat = w.pkstat;
  *psum = w.psum;
  *minmax = w.minmax;
  return PDP_OK;
}

int pdp_dataset_histograms_finish(int32_t value_kind, int64_t n_rows, int64_t n_privacy_ids, int64_t n_partitions,
                                  int32_t partition_histograms, const pdp_histogram_bins* out, void* workspace,
                                  uint64_t workspace_bytes, void* stream) {
  pdp::HCall c;
  int rc = pdp::hist_check(value_kind, n_rows, n_privacy_ids, n_partitions, out, workspace, workspace_bytes, stream,
                           &c);
  if (rc != PDP_OK) return rc;
  c.t.do_parts = partition_histograms != 0;
  return pdp::hist_finish(c, out);
}

}  // extern "C"

namespace pdp {
namespace {

struct PCall {
  PWs w;
  PT t;
  char* ws;
  hipStream_t st;
  IntHists H;
  FloatHists F;
};

int pre_check(int64_t n_rows, int64_t n_partitions, const pdp_histogram_bins* out, void* workspace,
              uint64_t workspace_bytes, void* stream, PCall* c) {
  if (out == nullptr || out->int_count == nullptr || out->int_sum == nullptr || out->int_max == nullptr ||
      out->float_count == nullptr || out->float_sum == nullptr || out->float_max == nullptr ||
      out->float_lowers == nullptr || out->float_n_lowers == nullptr)
    return set_error(PDP_E_INVALID, "every pdp_histogram_bins output must be set");
  if (n_rows < 0 || n_partitions < 0) return set_error(PDP_E_INVALID, "sizes must be >= 0");
  if (n_rows >= (int64_t)1 << 31) return set_error(PDP_E_UNSUPPORTED, "n_rows must be < 2^31 per shard");
  c->w = playout(n_rows, n_partitions);
  if (workspace == nullptr || workspace_bytes < c->w.total)
    return set_error(PDP_E_INVALID, "workspace smaller than pdp_dataset_histograms_preaggregated_workspace_bytes");
  c->ws = (char*)workspace;
  c->st = (hipStream_t)stream;
  c->t = PT{n_rows, n_partitions, wtab_capacity(n_rows), 1};
  c->H = IntHists{(unsigned long long*)out->int_count, (unsigned long long*)out->int_sum,
                  (unsigned long long*)out->int_max};
  c->F = FloatHists{(unsigned long long*)out->float_count, out->float_sum, (unsigned long long*)(c->ws + c->w.fmax)};
  return PDP_OK;
}

// zero everything; k_hp_rows (Linf histogram, per-partition statistics,
// row-sum min / max, L0 / L1 weight sums)
int pre_rows(const PCall& c, const int64_t* partition, const int64_t* count, const double* sum,
             const int64_t* n_partitions_of_pid, const int64_t* n_contributions_of_pid,
             const pdp_histogram_bins* out) {
  const PWs& w = c.w;
  const PT& t = c.t;
  char* ws = c.ws;
  hipStream_t st = c.st;
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.err, 0, 16, st));
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.pkrows, 0, w.minmax - w.pkrows, st));  // pkrows .. psum
  PDP_HLAUNCH("k_h_init", st, k_h_init, dim3(1), dim3(64), 0, st, (unsigned long long*)(ws + w.minmax));
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.fmax, 0, w.total - w.fmax, st));  // fmax, weight sums, weight table
  PDP_HIP_CHECK(hipMemsetAsync(out->int_count, 0, 5 * kLogBins * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(out->int_sum, 0, 5 * kLogBins * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(out->int_max, 0, 5 * kLogBins * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(out->float_count, 0, 2 * kSumBuckets * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(out->float_sum, 0, 2 * kSumBuckets * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(out->float_lowers, 0, 2 * kNLowers * 8, st));
  if (t.n == 0) return PDP_OK;
  if (partition == nullptr || count == nullptr || sum == nullptr || n_partitions_of_pid == nullptr ||
      n_contributions_of_pid == nullptr)
    return set_error(PDP_E_INVALID, "NULL column");
  PDP_HLAUNCH("k_hp_rows", st, k_hp_rows, dim3(grid_for(t.n, 2048)), dim3(kBlock), 0, st, t, partition, count, sum,
              n_partitions_of_pid, n_contributions_of_pid, (unsigned long long*)(ws + w.pkrows),
              (unsigned long long*)(ws + w.pkcount), (double*)(ws + w.psum), c.H,
              (unsigned long long*)(ws + w.minmax), (double*)(ws + w.wsmall), (WSlot*)(ws + w.wtab),
              (unsigned*)(ws + w.err));
  return PDP_OK;
}

// weighted L0 / L1 bins, partition histograms (t.do_parts), lowers, float bins
int pre_finish(const PCall& c, const double* sum, const pdp_histogram_bins* out) {
  const PWs& w = c.w;
  const PT& t = c.t;
  char* ws = c.ws;
  hipStream_t st = c.st;
  unsigned long long* minmax = (unsigned long long*)(ws + w.minmax);
  const unsigned long long* pkrows = (const unsigned long long*)(ws + w.pkrows);
  const double* psum = (const double*)(ws + w.psum);
  const int64_t nw = 2 * kWSmall + (int64_t)t.cap;
  PDP_HLAUNCH("k_hp_weights", st, k_hp_weights, dim3((unsigned)((nw + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
              (const double*)(ws + w.wsmall), (const WSlot*)(ws + w.wtab), t.cap, c.H);
  if (t.do_parts && t.P > 0)
    PDP_HLAUNCH("k_hp_ids", st, k_hp_ids, dim3(grid_for(t.P, 2048)), dim3(kBlock), 0, st, t, pkrows,
                (const unsigned long long*)(ws + w.pkcount), psum, c.H, minmax);
  PDP_HLAUNCH("k_h_lowers", st, k_h_lowers, dim3((kNLowers + kBlock - 1) / kBlock, 2), dim3(kBlock), 0, st, minmax,
              out->float_lowers, out->float_n_lowers);
  int dev = 0, cus = 256;
  PDP_HIP_CHECK(hipGetDevice(&dev));
  PDP_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int64_t mf = t.n > t.P ? t.n : t.P;
  int64_t gf = (mf + kFloatBlock - 1) / kFloatBlock;
  gf = gf < 1 ? 1 : (gf < cus ? gf : cus);
  if (t.n > 0 && sum == nullptr) return set_error(PDP_E_INVALID, "NULL column");
  PDP_HLAUNCH("k_hp_float", st, k_hp_float, dim3((unsigned)gf), dim3(kFloatBlock), 0, st, t, sum,
              pkrows, psum, out->float_lowers, out->float_n_lowers, c.F);
  PDP_HLAUNCH("k_h_final", st, k_h_final, dim3((2 * kSumBuckets + kBlock - 1) / kBlock), dim3(kBlock), 0, st, c.H,
              c.F, out->float_max, (1 << H_LINF) | (1 << H_COUNT) | (1 << H_PIDS));
  return PDP_OK;
}

}  // namespace
}  // namespace pdp

extern "C" {

int pdp_dataset_histograms_preaggregated_workspace_bytes(int64_t n_rows, int64_t n_partitions, uint64_t* bytes) {
  if (bytes == nullptr) return pdp::set_error(PDP_E_INVALID, "NULL argument");
  if (n_rows < 0 || n_partitions < 0) return pdp::set_error(PDP_E_INVALID, "sizes must be >= 0");
  *bytes = pdp::playout(n_rows, n_partitions).total;
  return PDP_OK;
}

int pdp_dataset_histograms_preaggregated_rows(const int64_t* partition, const int64_t* count, const double* sum,
                                              const int64_t* n_partitions_of_pid,
                                              const int64_t* n_contributions_of_pid, int64_t n_rows,
                                              int64_t n_partitions, const pdp_histogram_bins* out, void* workspace,
                                              uint64_t workspace_bytes, void* stream) {
  pdp::PCall c;
  const int rc = pdp::pre_check(n_rows, n_partitions, out, workspace, workspace_bytes, stream, &c);
  return rc == PDP_OK ? pdp::pre_rows(c, partition, count, sum, n_partitions_of_pid, n_contributions_of_pid, out)
                      : rc;
}

int pdp_dataset_histograms_preaggregated_exchange_offsets(int64_t n_rows, int64_t n_partitions, uint64_t* pk_rows,
                                                          uint64_t* pk_count, uint64_t* psum, uint64_t* minmax) {
  if (pk_rows == nullptr || pk_count == nullptr || psum == nullptr || minmax == nullptr)
    return pdp::set_error(PDP_E_INVALID, "NULL argument");
  if (n_rows < 0 || n_partitions < 0) return pdp::set_error(PDP_E_INVALID, "sizes must be >= 0");
  const pdp::PWs w = pdp::playout(n_rows, n_partitions);
  *pk_rows = w.pkrows;
  *pk_count = w.pkcount;
  *psum = w.psum;
  *minmax = w.minmax;
  return PDP_OK;
}

int pdp_dataset_histograms_preaggregated_weight_offsets(int64_t n_rows, int64_t n_partitions, uint64_t* wsmall,
                                                        uint64_t* wtab, uint64_t* wtab_slots) {
  if (wsmall == nullptr || wtab == nullptr || wtab_slots == nullptr)
    return pdp::set_error(PDP_E_INVALID, "NULL argument");
  if (n_rows < 0 || n_partitions < 0) return pdp::set_error(PDP_E_INVALID, "sizes must be >= 0");
  const pdp::PWs w = pdp::playout(n_rows, n_partitions);
  *wsmall = w.wsmall;
  *wtab = w.wtab;
  *wtab_slots = pdp::wtab_capacity(n_rows);
  return PDP_OK;
}

int pdp_dataset_histograms_weight_bins(const uint64_t* keys, const double* weights, int64_t n,
                                       const pdp_histogram_bins* out, void* stream) {
  if (out == nullptr || out->int_count == nullptr || out->int_sum == nullptr || out->int_max == nullptr)
    return pdp::set_error(PDP_E_INVALID, "the integer pdp_histogram_bins outputs must be set");
  if (n < 0) return pdp::set_error(PDP_E_INVALID, "n must be >= 0");
  if (n == 0) return PDP_OK;
  if (keys == nullptr || weights == nullptr) return pdp::set_error(PDP_E_INVALID, "NULL list");
  hipStream_t st = (hipStream_t)stream;
  const pdp::IntHists H{(unsigned long long*)out->int_count, (unsigned long long*)out->int_sum,
                        (unsigned long long*)out->int_max};
  PDP_HLAUNCH("k_hp_weight_list", st, pdp::k_hp_weight_list, dim3(pdp::grid_for(n, (int64_t)1 << 30)),
              dim3(pdp::kBlock), 0, st, (const unsigned long long*)keys, weights, n, H);
  return PDP_OK;
}

int pdp_dataset_histograms_preaggregated_finish(const double* sum, int64_t n_rows, int64_t n_partitions,
                                                int32_t partition_histograms, const pdp_histogram_bins* out,
                                                void* workspace,
                                                uint64_t workspace_bytes, void* stream) {
  pdp::PCall c;
  const int rc = pdp::pre_check(n_rows, n_partitions, out, workspace, workspace_bytes, stream, &c);
  if (rc != PDP_OK) return rc;
  c.t.do_parts = partition_histograms != 0;
  return pdp::pre_finish(c, sum, out);
}

int pdp_dataset_histograms_preaggregated(const int64_t* partition, const int64_t* count, const double* sum,
                                         const int64_t* n_partitions_of_pid, const int64_t* n_contributions_of_pid,
                                         int64_t n_rows, int64_t n_partitions, const pdp_histogram_bins* out,
                                         void* workspace, uint64_t workspace_bytes, void* stream) {
  pdp::PCall c;
  int rc = pdp::pre_check(n_rows, n_partitions, out, workspace, workspace_bytes, stream, &c);
  if (rc == PDP_OK) rc = pdp::pre_rows(c, partition, count, sum, n_partitions_of_pid, n_contributions_of_pid, out);
  if (rc == PDP_OK) rc = pdp::pre_finish(c, sum, out);
  return rc;
}

}  // extern "C"
