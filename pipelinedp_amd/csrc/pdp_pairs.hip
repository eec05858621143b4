// pdp_pairs.hip — the contribution bounders WITHOUT cross-partition sampling
// (gfx950): a device hash table of (privacy_id, partition_key) pairs.
//
// Replaces, for one shard of dense columns:
//   LinfSampler.bound_contributions  (contribution_bounders.py:204-230)
//     l0 = 0, linf > 0: per (pid, pk) a uniform sample of <= linf rows;
//   NoOpSampler.bound_contributions  (:233-246)
//     l0 = 0, linf = 0: group by (pid, pk), every row;
//   SamplingPerPrivacyIdContributionBounder (:114-156)
//     max_contributions = M: per pid a uniform sample of <= M rows, then group
//     the kept rows by (pid, pk);
//   DPEngine "Wrap values into accumulators" (dp_engine.py:143-150)
//     rows_are_units: contribution_bounds_already_enforced, one accumulator
//     per row, no privacy id;
// each followed by CompoundCombiner.create_accumulator per pair and
// LocalBackend.combine_accumulators_per_key (pipeline_backend.py:555-565).
//
// Without an L0 cap the pairs of one privacy id are unbounded, so the LDS
// bucket design of pdp_bound.hip does not apply; the pairs live in an
// open-addressing table in HBM (capacity a power of two >= 2 * rows) keyed by
// (pid << pk_bits) | pk.  Sampling stays bottom-k on the same counter-based
// row keys as the bucketed path (pdp_internal.h row_key), and sketch storage is
// only given to the groups that need it (count > cap), so it is bounded by the
// row count:
//   [max_contributions]  k_pid_count -> k_pid_len + scan -> k_pid_sketch
//   k_pair_insert        insert kept rows' pairs, count rows (linf = 0: also sum)
//   [linf > 0]           k_pair_len + scan -> k_pair_rows (light pairs sum,
//                        heavy pairs keep a bottom-linf row sketch)
//   k_pair_reduce        pair accumulators -> partition accumulators
//   rows_are_units:      k_rows_units into per-partition partials, then
//                        k_add_partials into the caller's accumulators
//
// The same table also runs SamplingCrossAndPerPartitionContributionBounder
// (:62-111) when a bound is beyond the LDS / sketch designs of pdp_bound.hip
// (l0 or linf > PDP_SKETCH_MAX, or PDP_ALGO_PAIR_TABLE asked for): every row
// goes into the table first, then per privacy id the distinct pairs are
// counted (k_pid_pairs) and a privacy id with more than l0 of them keeps its
// l0 smallest pair keys (the GLOBAL path's pair_key, rand_shift = pk_bits):
// k_pid_l0 + k_pair_keep mark the kept pairs, and Linf then samples only
// their rows.
//
// A cap above PDP_SKETCH_MAX (l0, linf or max_contributions) does not use an
// atomicMin cascade of that length: the heavy group stores ALL its keys in
// the pool (its length is the group's count) and one workgroup per heavy
// group finds the cap-th smallest key by radix select (k_radix_select, 8-bit digits,
// the candidates moved to LDS once they fit) and writes it where a sketch
// keeps its maximum (pool[offset + cap - 1]), so membership is the same test
// `key <= pool[offset + cap - 1]` in both modes; Linf's kept rows of heavy
// pairs are then summed by a second pass over the rows (k_pair_rows_kept).
#include "pdp_internal.h"

namespace pdp {
namespace {

constexpr uint64_t kMinTable = 1024;

struct PT {
  int64_t n, U, P;
  int l0, linf, maxc, pk_bits;
  int sel_l0, sel_linf, sel_maxc;  // cap > PDP_SKETCH_MAX: full pools + radix select
  uint64_t seed;
  uint64_t mask;  // table capacity - 1
  uint64_t pk_mask, row_seed, pid_row_seed;
  int64_t row_offset;
  ClipParams clip;
};

uint64_t table_capacity(int64_t n_rows) {
  uint64_t c = kMinTable;
  while (c < 2 * (uint64_t)n_rows) c <<= 1;
  return c;
}

struct PWs {
  uint64_t err;
  // max_contributions: per-pid counts, sketch offsets (+ total), sketches
  uint64_t pid_cnt, pid_off, pid_pool, pid_chunks;
  // pair table
  uint64_t keys, cnt, f0, f1, f2;
  // linf > 0: per-pair sketch offsets (+ total), sketches
  uint64_t pair_off, pair_pool, pair_chunks;
  // l0 > 0: kept-pair flags; select mode: fill cursors, heavy-group lists
  uint64_t pkeep, pid_fill, pair_fill, hlist, hcount;
  // rows_are_units: per-partition partial accumulators
  uint64_t r_pc, r_cnt, r_f0, r_f1, r_f2;
  uint64_t total;
};

bool has_f0(int flags) { return flags & (PDP_ACC_SUM | PDP_SUM_PER_PARTITION); }

PWs playout(const pdp_bound_config* c) {
  PWs w{};
  uint64_t off = 0;
  const uint64_t n = (uint64_t)c->n_rows;
  w.err = off; off = align256(off + 16);
  if (c->rows_are_units) {
    const uint64_t P = (uint64_t)c->n_partitions;
    w.r_pc = off; off = align256(off + P * 8);
    w.r_cnt = off; off = align256(off + P * 8);
    if (has_f0(c->flags)) { w.r_f0 = off; off = align256(off + P * 8); }
    if (c->flags & PDP_ACC_NSUM) { w.r_f1 = off; off = align256(off + P * 8); }
    if (c->flags & PDP_ACC_NSUM2) { w.r_f2 = off; off = align256(off + P * 8); }
    w.total = off;
    return w;
  }
  w.hcount = off; off = align256(off + 16);
  w.hlist = off; off = align256(off + (n / (PDP_SKETCH_MAX + 1) + 2) * 4);
  if (c->max_contributions > 0 || c->l0 > 0) {
    // max_contributions: rows per pid; l0: distinct pairs per pid (<= rows)
    const uint64_t U = (uint64_t)c->n_privacy_ids;
    w.pid_cnt = off; off = align256(off + U * 4);
    w.pid_off = off; off = align256(off + (U + 1) * 4);
    w.pid_pool = off; off = align256(off + n * 8);
    w.pid_chunks = off; off = align256(off + (uint64_t)scan_chunk_sums_len((int64_t)U) * 4);
    w.pid_fill = off; off = align256(off + U * 4);
  }
  const uint64_t C = table_capacity(c->n_rows);
  if (c->l0 > 0) { w.pkeep = off; off = align256(off + C); }
  w.keys = off; off = align256(off + C * 8);
  w.cnt = off; off = align256(off + C * 4);
  // running sums of keep-every-row pairs (all pairs when linf = 0, the light
  // ones otherwise)
  if (c->value_kind != PDP_VALUE_NONE) {
    if (has_f0(c->flags)) { w.f0 = off; off = align256(off + C * 8); }
    if (c->flags & PDP_ACC_NSUM) { w.f1 = off; off = align256(off + C * 8); }
    if (c->flags & PDP_ACC_NSUM2) { w.f2 = off; off = align256(off + C * 8); }
  }
  if (c->linf > 0) {
    w.pair_off = off; off = align256(off + (C + 1) * 4);
    w.pair_pool = off; off = align256(off + n * 8);
    w.pair_chunks = off; off = align256(off + (uint64_t)scan_chunk_sums_len((int64_t)C) * 4);
    w.pair_fill = off; off = align256(off + C * 4);
  }
  w.total = off;
  return w;
}

PT make_pt(const pdp_bound_config* c) {
  PT t;
  t.n = c->n_rows;
  t.U = c->n_privacy_ids;
  t.P = c->n_partitions;
  t.l0 = c->l0;
  t.linf = c->linf;
  t.maxc = c->max_contributions;
  t.sel_l0 = c->l0 > PDP_SKETCH_MAX;
  t.sel_linf = c->linf > PDP_SKETCH_MAX;
  t.sel_maxc = c->max_contributions > PDP_SKETCH_MAX;
  t.seed = c->seed;
  t.pk_bits = bits_for(c->n_partitions);
  t.mask = table_capacity(c->n_rows) - 1;
  t.pk_mask = (1ULL << t.pk_bits) - 1;
  t.row_seed = derive_row_seed(c->seed);
  t.pid_row_seed = derive_row_seed(c->seed ^ 0x2545F4914F6CDD1DULL);
  t.row_offset = c->row_offset;
  t.clip = ClipParams{c->min_value, c->max_value, c->middle, c->min_sum, c->max_sum, c->flags};
  return t;
}

// A row takes part iff its keys are in range (else the error bit is set) and
// its partition is allowed (public partitions).
__device__ __forceinline__ bool row_ok(const PT& t, const int64_t* __restrict__ pid, const int64_t* __restrict__ pk,
                                       const uint8_t* __restrict__ allowed, int64_t i, int64_t* u, int64_t* k,
                                       unsigned* err) {
  *k = pk[i];
  *u = pid != nullptr ? pid[i] : 0;
  if (*u < 0 || *u >= t.U || *k < 0 || *k >= t.P) {
    if (err) atomicOr(err, 1u);
    return false;
  }
  return allowed == nullptr || allowed[*k] != 0;
}

// max_contributions: is row i among its privacy id's sampled rows?
__device__ __forceinline__ bool pid_keeps(const PT& t, const unsigned* __restrict__ pid_cnt,
                                          const unsigned* __restrict__ pid_off,
                                          const unsigned long long* __restrict__ pool, int64_t u, int64_t i) {
  if (t.maxc <= 0 || pid_cnt[u] <= (unsigned)t.maxc) return true;
  const uint64_t y = row_key(t.pid_row_seed, t.row_offset + i, (uint32_t)i);
  return y <= pool[(uint64_t)pid_off[u] + t.maxc - 1];  // the sketch holds exactly the maxc smallest keys
}

__device__ __forceinline__ uint64_t slot_hash(uint64_t x, uint64_t mask) { return mix64(x) & mask; }

__device__ __forceinline__ uint64_t table_insert(unsigned long long* keys, uint64_t mask, uint64_t x) {
  uint64_t h = slot_hash(x, mask);
  for (;;) {
    const unsigned long long cur = keys[h];
    if (cur == x) return h;
    if (cur == kEmpty) {
      const unsigned long long old = atomicCAS(keys + h, kEmpty, (unsigned long long)x);
      if (old == kEmpty || old == x) return h;
    }
    h = (h + 1) & mask;  // capacity >= 2 * rows: a free slot always exists
  }
}

__device__ __forceinline__ uint64_t table_find(const unsigned long long* keys, uint64_t mask, uint64_t x) {
  uint64_t h = slot_hash(x, mask);
  while (keys[h] != x) h = (h + 1) & mask;  // x was inserted by k_pair_insert
  return h;
}

__global__ void __launch_bounds__(kBlock) k_pid_count(PT t, const int64_t* __restrict__ pid,
                                                      const int64_t* __restrict__ pk,
                                                      const uint8_t* __restrict__ allowed, unsigned* pid_cnt,
                                                      unsigned* err) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n; i += stride) {
    int64_t u, k;
    if (row_ok(t, pid, pk, allowed, i, &u, &k, err)) atomicAdd(pid_cnt + u, 1u);
  }
}

// pool length per group: a group with more than cap members gets cap slots
// (sketch) or, in select mode, one per member, and joins the heavy list;
// keep (l0 > 0): only kept pairs take part
__global__ void __launch_bounds__(kBlock) k_sketch_len(const unsigned* __restrict__ cnt,
                                                       const unsigned long long* __restrict__ keys,
                                                       const uint8_t* __restrict__ keep, int64_t n, unsigned cap,
                                                       int select, unsigned* len, unsigned* list,
                                                       unsigned* n_list) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const bool live = (keys == nullptr || keys[i] != kEmpty) && (keep == nullptr || keep[i] != 0);
    const bool heavy = live && cnt[i] > cap;
    len[i] = heavy ? (select ? cnt[i] : cap) : 0u;
    if (heavy && select) list[atomicAdd(n_list, 1u)] = (unsigned)i;
  }
}

// Radix select: for heavy group g = list[blockIdx.x], the cap-th smallest of
// its cnt[g] distinct keys at pool[off[g]..), written to pool[off[g] + cap - 1]
// (the position a sketch's maximum has).  8-bit digits from the top; the
// candidates sharing the chosen prefix move to LDS once they fit.
constexpr int kSelBlock = 256;
constexpr int kSelLds = 4096;
__global__ void __launch_bounds__(kSelBlock) k_radix_select(const unsigned* __restrict__ list,
                                                      const unsigned* __restrict__ n_list,
                                                      const unsigned* __restrict__ off,
                                                      const unsigned* __restrict__ cnt, unsigned cap,
                                                      unsigned long long* pool) {
  __shared__ unsigned hist[256];
  __shared__ unsigned long long cand[kSelLds];
  __shared__ unsigned long long s_pre, s_mask;
  __shared__ unsigned s_k, s_match, s_ngath;
  __shared__ int s_inlds;
  if (blockIdx.x >= *n_list) return;  // grid is an upper bound on the heavy groups
  const unsigned g = list[blockIdx.x];
  unsigned long long* seg = pool + off[g];
  const unsigned m = cnt[g];
  if (threadIdx.x == 0) {
    s_pre = 0;
    s_mask = 0;
    s_k = cap;
    s_inlds = 0;
    s_ngath = 0;
  }
  __syncthreads();
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    const unsigned long long pre = s_pre, mask = s_mask;
    const bool inlds = s_inlds != 0;
    const unsigned nc = inlds ? s_ngath : m;
    for (unsigned i = threadIdx.x; i < nc; i += blockDim.x) {
      const unsigned long long x = inlds ? cand[i] : seg[i];
      if ((x & mask) == pre) atomicAdd(hist + ((x >> shift) & 255), 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned c = 0, v = 0;
      while (c + hist[v] < s_k) c += hist[v++];  // the digit holding the k-th smallest
      s_k -= c;
      s_pre = pre | ((unsigned long long)v << shift);
      s_mask = mask | (255ULL << shift);
      s_match = hist[v];
    }
    __syncthreads();
    if (!s_inlds && shift > 0 && s_match <= (unsigned)kSelLds) {  // block-uniform
      const unsigned long long p2 = s_pre, m2 = s_mask;
      for (unsigned i = threadIdx.x; i < m; i += blockDim.x) {
        const unsigned long long x = seg[i];
        if ((x & m2) == p2) cand[atomicAdd(&s_ngath, 1u)] = x;
      }
      __syncthreads();
      if (threadIdx.x == 0) s_inlds = 1;
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) seg[cap - 1] = s_pre;  // every read of seg is behind the last barrier
}

// l0 > 0: distinct pairs per privacy id
__global__ void __launch_bounds__(kBlock) k_pid_pairs(PT t, const unsigned long long* __restrict__ keys,
                                                      unsigned* pid_cnt) {
  const int64_t C = (int64_t)t.mask + 1;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < C; s += stride) {
    const uint64_t x = keys[s];
    if (x != kEmpty) atomicAdd(pid_cnt + (x >> t.pk_bits), 1u);
  }
}

__device__ __forceinline__ uint64_t slot_pair_key(const PT& t, uint64_t x) {
  return pair_key(t.seed, (int64_t)(x >> t.pk_bits), (int64_t)(x & t.pk_mask), 0, t.pk_bits);
}

// l0 > 0: pair keys of the privacy ids with more than l0 pairs: bottom-l0
// sketch, or (select mode) every pair key appended
__global__ void __launch_bounds__(kBlock) k_pid_l0(PT t, const unsigned long long* __restrict__ keys,
                                                   const unsigned* __restrict__ pid_cnt,
                                                   const unsigned* __restrict__ pid_off, unsigned* pid_fill,
                                                   unsigned long long* pool) {
  const int64_t C = (int64_t)t.mask + 1;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < C; s += stride) {
    const uint64_t x = keys[s];
    if (x == kEmpty) continue;
    const uint64_t u = x >> t.pk_bits;
    if (pid_cnt[u] <= (unsigned)t.l0) continue;
    const uint64_t y = slot_pair_key(t, x);
    if (t.sel_l0) {
      pool[(uint64_t)pid_off[u] + atomicAdd(pid_fill + u, 1u)] = y;
    } else {
      unsigned long long* sk = pool + pid_off[u];
      if (y < sk[t.l0 - 1]) sketch_insert(sk, t.l0, y);
    }
  }
}

// l0 > 0: a pair is kept iff its privacy id has <= l0 pairs or its key is
// among the l0 smallest
__global__ void __launch_bounds__(kBlock) k_pair_keep(PT t, const unsigned long long* __restrict__ keys,
                                                      const unsigned* __restrict__ pid_cnt,
                                                      const unsigned* __restrict__ pid_off,
                                                      const unsigned long long* __restrict__ pool, uint8_t* keep) {
  const int64_t C = (int64_t)t.mask + 1;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < C; s += stride) {
    const uint64_t x = keys[s];
    uint8_t k = 0;
    if (x != kEmpty) {
      const uint64_t u = x >> t.pk_bits;
      k = pid_cnt[u] <= (unsigned)t.l0 || slot_pair_key(t, x) <= pool[(uint64_t)pid_off[u] + t.l0 - 1];
    }
    keep[s] = k;
  }
}

// max_contributions, select mode: every row key of a heavy privacy id
__global__ void __launch_bounds__(kBlock) k_pid_fill(PT t, const int64_t* __restrict__ pid,
                                                     const int64_t* __restrict__ pk,
                                                     const uint8_t* __restrict__ allowed,
                                                     const unsigned* __restrict__ pid_cnt,
                                                     const unsigned* __restrict__ pid_off, unsigned* pid_fill,
                                                     unsigned long long* pool) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n; i += stride) {
    int64_t u, k;
    if (!row_ok(t, pid, pk, allowed, i, &u, &k, nullptr) || pid_cnt[u] <= (unsigned)t.maxc) continue;
    pool[(uint64_t)pid_off[u] + atomicAdd(pid_fill + u, 1u)] = row_key(t.pid_row_seed, t.row_offset + i, (uint32_t)i);
  }
}

__global__ void __launch_bounds__(kBlock) k_pid_sketch(PT t, const int64_t* __restrict__ pid,
                                                       const int64_t* __restrict__ pk,
                                                       const uint8_t* __restrict__ allowed,
                                                       const unsigned* __restrict__ pid_cnt,
                                                       const unsigned* __restrict__ pid_off,
                                                       unsigned long long* pool) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n; i += stride) {
    int64_t u, k;
    if (!row_ok(t, pid, pk, allowed, i, &u, &k, nullptr) || pid_cnt[u] <= (unsigned)t.maxc) continue;
    const uint64_t y = row_key(t.pid_row_seed, t.row_offset + i, (uint32_t)i);
    unsigned long long* s = pool + pid_off[u];
    if (y < s[t.maxc - 1]) sketch_insert(s, t.maxc, y);
  }
}

template <int VK, bool KEEP_ALL>
__global__ void __launch_bounds__(kBlock) k_pair_insert(PT t, const int64_t* __restrict__ pid,
                                                        const int64_t* __restrict__ pk,
                                                        const void* __restrict__ value,
                                                        const uint8_t* __restrict__ allowed,
                                                        const unsigned* __restrict__ pid_cnt,
                                                        const unsigned* __restrict__ pid_off,
                                                        const unsigned long long* __restrict__ pid_pool,
                                                        unsigned long long* keys, unsigned* cnt, double* f0,
                                                        double* f1, double* f2, unsigned* err) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n; i += stride) {
    int64_t u, k;
    if (!row_ok(t, pid, pk, allowed, i, &u, &k, t.maxc > 0 ? nullptr : err)) continue;
    if (!pid_keeps(t, pid_cnt, pid_off, pid_pool, u, i)) continue;
    const uint64_t slot = table_insert(keys, t.mask, ((uint64_t)u << t.pk_bits) | (uint64_t)k);
    atomicAdd(cnt + slot, 1u);
    if (KEEP_ALL) accumulate_row<VK>(value, (uint32_t)i, (int64_t)slot, f0, f1, f2, t.clip);
  }
}

// linf > 0: light pairs (<= linf rows) sum every row, heavy pairs keep the
// bottom-linf row keys in their sketch
template <int VK>
__global__ void __launch_bounds__(kBlock) k_pair_rows(PT t, const int64_t* __restrict__ pid,
                                                      const int64_t* __restrict__ pk, const void* __restrict__ value,
                                                      const uint8_t* __restrict__ allowed,
                                                      const unsigned long long* __restrict__ keys,
                                                      const unsigned* __restrict__ cnt,
                                                      const unsigned* __restrict__ pair_off,
                                                      const uint8_t* __restrict__ keep, unsigned* pair_fill,
                                                      unsigned long long* pool, double* f0, double* f1, double* f2) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n; i += stride) {
    int64_t u, k;
    if (!row_ok(t, pid, pk, allowed, i, &u, &k, nullptr)) continue;
    const uint64_t slot = table_find(keys, t.mask, ((uint64_t)u << t.pk_bits) | (uint64_t)k);
    if (keep != nullptr && keep[slot] == 0) continue;
    if (cnt[slot] <= (unsigned)t.linf) {
      accumulate_row<VK>(value, (uint32_t)i, (int64_t)slot, f0, f1, f2, t.clip);
    } else {
      const uint64_t y = row_key(t.row_seed, t.row_offset + i, (uint32_t)i);
      if (t.sel_linf) {
        pool[(uint64_t)pair_off[slot] + atomicAdd(pair_fill + slot, 1u)] = y;
      } else {
        unsigned long long* s = pool + pair_off[slot];
        if (y < s[t.linf - 1]) sketch_insert(s, t.linf, y);
      }
    }
  }
}

// select-mode Linf: the kept rows of heavy pairs (row key <= the pair's
// selected threshold) into the running sums
template <int VK>
__global__ void __launch_bounds__(kBlock) k_pair_rows_kept(PT t, const int64_t* __restrict__ pid,
                                                           const int64_t* __restrict__ pk,
                                                           const void* __restrict__ value,
                                                           const uint8_t* __restrict__ allowed,
                                                           const unsigned long long* __restrict__ keys,
                                                           const unsigned* __restrict__ cnt,
                                                           const unsigned* __restrict__ pair_off,
                                                           const uint8_t* __restrict__ keep,
                                                           const unsigned long long* __restrict__ pool, double* f0,
                                                           double* f1, double* f2) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n; i += stride) {
    int64_t u, k;
    if (!row_ok(t, pid, pk, allowed, i, &u, &k, nullptr)) continue;
    const uint64_t slot = table_find(keys, t.mask, ((uint64_t)u << t.pk_bits) | (uint64_t)k);
    if ((keep != nullptr && keep[slot] == 0) || cnt[slot] <= (unsigned)t.linf) continue;
    const uint64_t y = row_key(t.row_seed, t.row_offset + i, (uint32_t)i);
    if (y <= pool[(uint64_t)pair_off[slot] + t.linf - 1])
      accumulate_row<VK>(value, (uint32_t)i, (int64_t)slot, f0, f1, f2, t.clip);
  }
}

template <int VK, bool KEEP_ALL>
__global__ void __launch_bounds__(kBlock) k_pair_reduce(PT t, const void* __restrict__ value,
                                                        const unsigned long long* __restrict__ keys,
                                                        const unsigned* __restrict__ cnt,
                                                        const unsigned* __restrict__ pair_off,
                                                        const unsigned long long* __restrict__ pool,
                                                        const double* __restrict__ f0, const double* __restrict__ f1,
                                                        const double* __restrict__ f2,
                                                        const uint8_t* __restrict__ keep,
                                                        pdp_partition_accumulators acc) {
  const int64_t C = (int64_t)t.mask + 1;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < C; s += stride) {
    const uint64_t x = keys[s];
    if (x == kEmpty || (keep != nullptr && keep[s] == 0)) continue;
    const unsigned c = cnt[s];
    PairSums ps;
    if (!KEEP_ALL && c > (unsigned)t.linf && t.sel_linf) {  // exactly linf kept rows, summed
      ps = VK != PDP_VALUE_NONE
               ? pair_sums_from_totals((long long)t.linf, f0 ? f0[s] : 0.0, f1 ? f1[s] : 0.0, f2 ? f2[s] : 0.0,
                                       t.clip)
               : PairSums{(long long)t.linf, 0, 0.0, 0.0, 0.0};
    } else if (!KEEP_ALL && c > (unsigned)t.linf) {
      ps = pair_sums_from_rows<VK>(pool + pair_off[s], t.linf, value, t.clip);
    } else if (VK != PDP_VALUE_NONE) {
      ps = pair_sums_from_totals((long long)c, f0 ? f0[s] : 0.0, f1 ? f1[s] : 0.0, f2 ? f2[s] : 0.0, t.clip);
    } else {
      ps = PairSums{(long long)c, 0, 0.0, 0.0, 0.0};
    }
    add_pair_to_partition(acc, (int64_t)(x & t.pk_mask), ps, t.clip.flags);
  }
}

// contribution_bounds_already_enforced: create_accumulator([value]) per row
template <int VK>
__global__ void __launch_bounds__(kBlock) k_rows_units(PT t, const int64_t* __restrict__ pk,
                                                       const void* __restrict__ value,
                                                       const uint8_t* __restrict__ allowed,
                                                       pdp_partition_accumulators part, unsigned* err) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n; i += stride) {
    int64_t u, k;
    if (!row_ok(t, nullptr, pk, allowed, i, &u, &k, err)) continue;
    const unsigned long long r = (unsigned long long)i;
    const PairSums ps = pair_sums_from_rows<VK>(&r, 1, value, t.clip);
    add_pair_to_partition(part, k, ps, t.clip.flags);
  }
}

__global__ void __launch_bounds__(kBlock) k_add_partials(int64_t P, int flags, pdp_partition_accumulators part,
                                                         pdp_partition_accumulators acc) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool sum_int = flags & PDP_SUM_INT;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P; p += stride) {
    if (part.privacy_id_count[p] == 0) continue;
    acc.privacy_id_count[p] += part.privacy_id_count[p];
    if (acc.count) acc.count[p] += part.count[p];
    if (acc.sum && part.sum) {
      if (sum_int) ((long long*)acc.sum)[p] += ((const long long*)part.sum)[p];
      else ((double*)acc.sum)[p] += ((const double*)part.sum)[p];
    }
    if (acc.normalized_sum && part.normalized_sum) acc.normalized_sum[p] += part.normalized_sum[p];
    if (acc.normalized_sum_sq && part.normalized_sum_sq) acc.normalized_sum_sq[p] += part.normalized_sum_sq[p];
  }
}

pdp_partition_accumulators partials(char* ws, const PWs& w) {
  pdp_partition_accumulators a{};
  a.privacy_id_count = (int64_t*)(ws + w.r_pc);
  a.count = (int64_t*)(ws + w.r_cnt);
  a.sum = w.r_f0 ? (void*)(ws + w.r_f0) : nullptr;
  a.normalized_sum = w.r_f1 ? (double*)(ws + w.r_f1) : nullptr;
  a.normalized_sum_sq = w.r_f2 ? (double*)(ws + w.r_f2) : nullptr;
  return a;
}

template <template <int> class F, typename... A>
int dispatch_vk(int value_kind, A&&... args) {
  switch (value_kind) {
    case PDP_VALUE_NONE: return F<PDP_VALUE_NONE>::run(args...);
    case PDP_VALUE_F64: return F<PDP_VALUE_F64>::run(args...);
    default: return F<PDP_VALUE_I64>::run(args...);
  }
}

#define PDP_LAUNCH(name, st, ...)                                           \
  do {                                                                      \
    PDP_PROF_BEGIN(name, st);                                               \
    hipLaunchKernelGGL(__VA_ARGS__);                                        \
    PDP_PROF_END(st);                                                       \
    PDP_HIP_CHECK(hipGetLastError());                                       \
  } while (0)

struct BoundArgs {
  const PT* t;
  const int64_t* pid;
  const int64_t* pk;
  const void* value;
  const uint8_t* allowed;
  char* ws;
  const PWs* w;
  hipStream_t st;
};

template <int VK>
struct RunBound {
  static int run(const BoundArgs& a) {
    const PT& t = *a.t;
    const PWs& w = *a.w;
    char* ws = a.ws;
    hipStream_t st = a.st;
    unsigned* err = (unsigned*)(ws + w.err);
    const unsigned g = grid_for(t.n);
    const bool per_pid = t.maxc > 0 || t.l0 > 0;
    unsigned* pid_cnt = per_pid ? (unsigned*)(ws + w.pid_cnt) : nullptr;
    unsigned* pid_off = per_pid ? (unsigned*)(ws + w.pid_off) : nullptr;
    unsigned long long* pid_pool = per_pid ? (unsigned long long*)(ws + w.pid_pool) : nullptr;
    unsigned* pid_fill = per_pid ? (unsigned*)(ws + w.pid_fill) : nullptr;
    unsigned* hlist = (unsigned*)(ws + w.hlist);
    unsigned* hcount = (unsigned*)(ws + w.hcount);
    // heavy groups in select mode: at most n / (cap + 1) of them
    auto run_select = [&](unsigned* n_list, const unsigned* off, const unsigned* cnt, int cap,
                          unsigned long long* pool) -> int {
      const int64_t ub = t.n / ((int64_t)cap + 1) + 1;
      PDP_LAUNCH("k_radix_select", st, k_radix_select, dim3((unsigned)ub), dim3(kSelBlock), 0, st, hlist, n_list, off, cnt,
                 (unsigned)cap, pool);
      return PDP_OK;
    };
    if (t.maxc > 0) {
      PDP_LAUNCH("k_pid_count", st, k_pid_count, dim3(g), dim3(kBlock), 0, st, t, a.pid, a.pk, a.allowed, pid_cnt,
                 err);
      const unsigned gu = grid_for(t.U);
      PDP_LAUNCH("k_sketch_len", st, k_sketch_len, dim3(gu), dim3(kBlock), 0, st, pid_cnt, nullptr, nullptr, t.U,
                 (unsigned)t.maxc, t.sel_maxc, pid_off, hlist, hcount);
      int rc = scan_u32(pid_off, t.U, (unsigned*)(ws + w.pid_chunks), st);
      if (rc != PDP_OK) return rc;
      if (t.sel_maxc) {
        PDP_LAUNCH("k_pid_fill", st, k_pid_fill, dim3(g), dim3(kBlock), 0, st, t, a.pid, a.pk, a.allowed, pid_cnt,
                   pid_off, pid_fill, pid_pool);
        rc = run_select(hcount, pid_off, pid_cnt, t.maxc, pid_pool);
        if (rc != PDP_OK) return rc;
      } else {
        PDP_LAUNCH("k_pid_sketch", st, k_pid_sketch, dim3(g), dim3(kBlock), 0, st, t, a.pid, a.pk, a.allowed,
                   pid_cnt, pid_off, pid_pool);
      }
    }
    double* f0 = w.f0 ? (double*)(ws + w.f0) : nullptr;
    double* f1 = w.f1 ? (double*)(ws + w.f1) : nullptr;
    double* f2 = w.f2 ? (double*)(ws + w.f2) : nullptr;
    unsigned long long* keys = (unsigned long long*)(ws + w.keys);
    unsigned* cnt = (unsigned*)(ws + w.cnt);
    const int64_t C = (int64_t)t.mask + 1;
    const unsigned gc = grid_for(C);
    if (t.linf == 0) {
      PDP_LAUNCH("k_pair_insert", st, (k_pair_insert<VK, true>), dim3(g), dim3(kBlock), 0, st, t, a.pid, a.pk,
                 a.value, a.allowed, pid_cnt, pid_off, pid_pool, keys, cnt, f0, f1, f2, err);
    } else {
      PDP_LAUNCH("k_pair_insert", st, (k_pair_insert<VK, false>), dim3(g), dim3(kBlock), 0, st, t, a.pid, a.pk,
                 a.value, a.allowed, pid_cnt, pid_off, pid_pool, keys, cnt, f0, f1, f2, err);
    }
    uint8_t* keep = nullptr;
    if (t.l0 > 0) {  // cross-partition sampling over the table's distinct pairs
      keep = (uint8_t*)(ws + w.pkeep);
      PDP_LAUNCH("k_pid_pairs", st, k_pid_pairs, dim3(gc), dim3(kBlock), 0, st, t, keys, pid_cnt);
      const unsigned gu = grid_for(t.U);
      PDP_LAUNCH("k_sketch_len", st, k_sketch_len, dim3(gu), dim3(kBlock), 0, st, pid_cnt, nullptr, nullptr, t.U,
                 (unsigned)t.l0, t.sel_l0, pid_off, hlist, hcount + 1);
      int rc = scan_u32(pid_off, t.U, (unsigned*)(ws + w.pid_chunks), st);
      if (rc != PDP_OK) return rc;
      PDP_LAUNCH("k_pid_l0", st, k_pid_l0, dim3(gc), dim3(kBlock), 0, st, t, keys, pid_cnt, pid_off, pid_fill,
                 pid_pool);
      if (t.sel_l0) {
        rc = run_select(hcount + 1, pid_off, pid_cnt, t.l0, pid_pool);
        if (rc != PDP_OK) return rc;
      }
      PDP_LAUNCH("k_pair_keep", st, k_pair_keep, dim3(gc), dim3(kBlock), 0, st, t, keys, pid_cnt, pid_off, pid_pool,
                 keep);
    }
    if (t.linf == 0) return PDP_OK;
    unsigned* pair_off = (unsigned*)(ws + w.pair_off);
    unsigned long long* pair_pool = (unsigned long long*)(ws + w.pair_pool);
    PDP_LAUNCH("k_sketch_len", st, k_sketch_len, dim3(gc), dim3(kBlock), 0, st, cnt, keys, keep, C,
               (unsigned)t.linf, t.sel_linf, pair_off, hlist, hcount + 2);
    int rc = scan_u32(pair_off, C, (unsigned*)(ws + w.pair_chunks), st);
    if (rc != PDP_OK) return rc;
    PDP_LAUNCH("k_pair_rows", st, k_pair_rows<VK>, dim3(g), dim3(kBlock), 0, st, t, a.pid, a.pk, a.value,
               a.allowed, keys, cnt, pair_off, keep, (unsigned*)(ws + w.pair_fill), pair_pool, f0, f1, f2);
    if (t.sel_linf) {
      rc = run_select(hcount + 2, pair_off, cnt, t.linf, pair_pool);
      if (rc != PDP_OK) return rc;
      PDP_LAUNCH("k_pair_rows_kept", st, k_pair_rows_kept<VK>, dim3(g), dim3(kBlock), 0, st, t, a.pid, a.pk,
                 a.value, a.allowed, keys, cnt, pair_off, keep, pair_pool, f0, f1, f2);
    }
    return PDP_OK;
  }
};

struct ReduceArgs {
  const PT* t;
  const void* value;
  char* ws;
  const PWs* w;
  pdp_partition_accumulators acc;
  hipStream_t st;
};

template <int VK>
struct RunReduce {
  static int run(const ReduceArgs& a) {
    const PT& t = *a.t;
    const PWs& w = *a.w;
    char* ws = a.ws;
    const int64_t C = (int64_t)t.mask + 1;
    const unsigned gc = grid_for(C);
    const double* f0 = w.f0 ? (const double*)(ws + w.f0) : nullptr;
    const double* f1 = w.f1 ? (const double*)(ws + w.f1) : nullptr;
    const double* f2 = w.f2 ? (const double*)(ws + w.f2) : nullptr;
    const unsigned* pair_off = t.linf > 0 ? (const unsigned*)(ws + w.pair_off) : nullptr;
    const unsigned long long* pool = t.linf > 0 ? (const unsigned long long*)(ws + w.pair_pool) : nullptr;
    const uint8_t* keep = t.l0 > 0 ? (const uint8_t*)(ws + w.pkeep) : nullptr;
    if (t.linf == 0) {
      PDP_LAUNCH("k_pair_reduce", a.st, (k_pair_reduce<VK, true>), dim3(gc), dim3(kBlock), 0, a.st, t, a.value,
                 (const unsigned long long*)(ws + w.keys), (const unsigned*)(ws + w.cnt), pair_off, pool, f0, f1, f2,
                 keep, a.acc);
    } else {
      PDP_LAUNCH("k_pair_reduce", a.st, (k_pair_reduce<VK, false>), dim3(gc), dim3(kBlock), 0, a.st, t,
                 a.value, (const unsigned long long*)(ws + w.keys), (const unsigned*)(ws + w.cnt), pair_off, pool, f0,
                 f1, f2, keep, a.acc);
    }
    return PDP_OK;
  }
};

template <int VK>
struct RunUnits {
  static int run(const PT& t, const int64_t* pk, const void* value, const uint8_t* allowed,
                 pdp_partition_accumulators part, unsigned* err, hipStream_t st) {
    const unsigned g = grid_for(t.n);
    PDP_LAUNCH("k_rows_units", st, k_rows_units<VK>, dim3(g), dim3(kBlock), 0, st, t, pk, value, allowed, part,
               err);
    return PDP_OK;
  }
};

}  // namespace

int pairs_validate(const pdp_bound_config* c) {
  if (c->algorithm != PDP_ALGO_AUTO && c->algorithm != PDP_ALGO_PAIR_TABLE)
    return set_error(PDP_E_UNSUPPORTED,
                     "l0 = 0 / max_contributions / rows_are_units / l0 or linf > PDP_SKETCH_MAX need "
                     "PDP_ALGO_PAIR_TABLE");
  if (c->max_contributions < 0 || c->max_contributions > PDP_MAX_CONTRIBUTIONS)
    return set_error(PDP_E_UNSUPPORTED, "max_contributions out of supported range [0, PDP_MAX_CONTRIBUTIONS]");
  if (c->max_contributions > 0 && (c->l0 != 0 || c->linf != 0))
    return set_error(PDP_E_INVALID, "max_contributions excludes l0 / linf (aggregate_params.py:344-352)");
  if (c->rows_are_units && (c->l0 != 0 || c->linf != 0 || c->max_contributions != 0))
    return set_error(PDP_E_INVALID, "rows_are_units excludes every sampling bound");
  if (!c->rows_are_units && bits_for(c->n_privacy_ids) + bits_for(c->n_partitions) > 63)
    return set_error(PDP_E_UNSUPPORTED, "pair key (privacy id bits + partition bits) exceeds 63 bits");
  return PDP_OK;
}

uint64_t pairs_workspace_bytes(const pdp_bound_config* c) { return playout(c).total; }

int pairs_bound(const pdp_bound_config* c, const int64_t* pid, const int64_t* pk, const void* value,
                const uint8_t* allowed, char* ws, hipStream_t st) {
  const PWs w = playout(c);
  const PT t = make_pt(c);
  unsigned* err = (unsigned*)(ws + w.err);
  PDP_HIP_CHECK(hipMemsetAsync(err, 0, 16, st));
  if (c->rows_are_units) {
    PDP_HIP_CHECK(hipMemsetAsync(ws + w.r_pc, 0, w.total - w.r_pc, st));
    if (c->n_rows == 0) return PDP_OK;
    return dispatch_vk<RunUnits>(c->value_kind, t, pk, value, allowed, partials(ws, w), err, st);
  }
  const uint64_t C = (uint64_t)t.mask + 1;
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.hcount, 0, 16, st));
  if (c->max_contributions > 0 || c->l0 > 0) {
    PDP_HIP_CHECK(hipMemsetAsync(ws + w.pid_cnt, 0, (uint64_t)c->n_privacy_ids * 4, st));
    PDP_HIP_CHECK(hipMemsetAsync(ws + w.pid_fill, 0, (uint64_t)c->n_privacy_ids * 4, st));
    if (c->n_rows > 0) PDP_HIP_CHECK(hipMemsetAsync(ws + w.pid_pool, 0xFF, (uint64_t)c->n_rows * 8, st));
  }
  if (c->linf > 0) PDP_HIP_CHECK(hipMemsetAsync(ws + w.pair_fill, 0, C * 4, st));
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.keys, 0xFF, C * 8, st));
  PDP_HIP_CHECK(hipMemsetAsync(ws + w.cnt, 0, C * 4, st));
  for (uint64_t f : {w.f0, w.f1, w.f2})
    if (f) PDP_HIP_CHECK(hipMemsetAsync(ws + f, 0, C * 8, st));
  if (c->linf > 0 && c->n_rows > 0) PDP_HIP_CHECK(hipMemsetAsync(ws + w.pair_pool, 0xFF, (uint64_t)c->n_rows * 8, st));
  if (c->n_rows == 0) return PDP_OK;
  const BoundArgs a{&t, pid, pk, value, allowed, ws, &w, st};
  return dispatch_vk<RunBound>(c->value_kind, a);
}

int pairs_reduce(const pdp_bound_config* c, const void* value, char* ws, const pdp_partition_accumulators& acc,
                 hipStream_t st) {
  const PWs w = playout(c);
  const PT t = make_pt(c);
  if (c->rows_are_units) {
    const unsigned g = grid_for(c->n_partitions);
    PDP_LAUNCH("k_add_partials", st, k_add_partials, dim3(g), dim3(kBlock), 0, st, c->n_partitions, c->flags,
               partials(ws, w), acc);
    return PDP_OK;
  }
  if (c->n_rows == 0) return PDP_OK;
  const ReduceArgs a{&t, value, ws, &w, acc, st};
  return dispatch_vk<RunReduce>(c->value_kind, a);
}

}  // namespace pdp
