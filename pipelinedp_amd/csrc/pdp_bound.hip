// pdp_bound.hip — contribution bounding + per-partition reduction (gfx950).
//
// Replaces, for one shard of dense columns (privacy_id, partition_key, value):
//   SamplingCrossAndPerPartitionContributionBounder.bound_contributions
//     (contribution_bounders.py:72-111): "Sample per (privacy_id, partition_key)"
//     (<= linf rows) and "Sample per privacy_id" (<= l0 distinct partitions);
//   SamplingCrossPartitionContributionBounder (:168-201) when linf == 0;
//   CompoundCombiner.create_accumulator / merge_accumulators (combiners.py:749-764)
//     and LocalBackend.combine_accumulators_per_key (pipeline_backend.py:555-565).
//
// Sampling = bottom-k on counter-based keys (pdp_internal.h: pair_key, row_key),
// so the kept sets depend only on (seed, data), not on scheduling or path.
//
// Two execution paths, same results:
//
//  BUCKETED (default when the per-privacy-id state fits LDS)
//    Privacy ids are grouped in buckets of 2^bucket_bits ids (one LDS-sized
//    workgroup each) and buckets in super-buckets of 2^super_bits buckets, so
//    that every partitioning pass writes to <= 64 destinations per workgroup
//    (long coalesced runs; ~2000 direct destinations thrash L2 5x).
//    k_part_hist       per-tile histogram of bucket = pid >> bucket_bits  (8 B/row)
//    k_super_scan      per-tile write offsets of every super-bucket
//    k_gscan_*, k_scan_*   rows per bucket -> bucket starts; level-2 write
//                      cursors at every group of kL2GroupTiles tiles
//    k_scatter_l1      rows -> super-bucket order, tile runs in tile order (16 B in, 8 B out)
//    k_scatter_l2      per (tile group, super-bucket) -> bucket order, no atomics (8 B in, 8 B out)
//    k_bucket_bound    one workgroup per bucket, all sampling state in LDS:
//                      B1 bottom-l0 pair sketch per pid, B2 per-pair row count
//                      + bottom-linf row sketch, B3 gather the sampled values
//                      and merge each kept pair into the partition accumulators
//  GLOBAL (fallback for large l0 * linf)
//    k_pair_sketch / k_pair_rows / k_reduce_pairs: the same sketches in HBM,
//    updated with device-scope atomics.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "pdp_internal.h"

namespace pdp {
namespace {

constexpr int kPartThreads = 512;
// rows per thread and LDS stage of the level-1 scatter / level-2 window
constexpr int kL1Threads = 1024;
constexpr int kL1Items = 8;
constexpr int kL1Rows = kL1Threads * kL1Items;  // rows per level-1 LDS stage
constexpr int kL2Items = 16;
// level 2: two 8-wave workgroups per CU need <= 128 VGPRs (MI355X_MICROARCH.md
// register table): the kernel takes 121-123 with 16 records per thread;
// loading a stage ahead (157 VGPRs, one workgroup per CU) cost 1 ms at C3
constexpr int kL2Threads = 512;
constexpr int kL2Rows = kL2Threads * kL2Items;  // records per level-2 LDS stage
// tiles per level-2 workgroup (k_scatter_l2, k_gscan_cursors)
constexpr int kL2GroupTiles = 16;
constexpr int kScanWaves = 16;
constexpr int kScanTiles = 16;  // tiles per wave in the level-2 cursor scans; multiple of kL2GroupTiles
constexpr int kScanChunkTiles = kScanWaves * kScanTiles;
static_assert(kScanTiles % kL2GroupTiles == 0, "group starts must fall inside a wave's tiles");
constexpr int kTileRowBits = 16;
constexpr int64_t kTileRows = (int64_t)1 << kTileRowBits;
constexpr int kStagesPerTile = (int)(kTileRows / kL1Rows);  // level-1 blocks per tile
constexpr int kL2Runs = kL2GroupTiles * kStagesPerTile;  // level-1 runs per level-2 workgroup
constexpr int kUnroll = 8;
constexpr int kBucketThreads = 1024;
constexpr int64_t kLdsBudget = 124 * 1024;  // per-pid state; + range scratch + wave queues <= 160 KiB
// 512-thread bucket workgroups: per-pid state <= 56 KiB, so that with the
// range scratch (<= 4 KiB at 512 ranges), 8 wave queues (12 KiB) and the pid
// hashes two workgroups fit one CU's 160 KiB
constexpr int64_t kLdsBudget2 = 56 * 1024;
constexpr int kMinRandomBits = 24;
constexpr int64_t kMaxBuckets = 36 * 1024;  // u32 histogram in 144 KiB of LDS
constexpr int kMaxSupers = 128;   // destinations of a level-1 scatter
constexpr int64_t kSingleLevelMax = 64;      // buckets partitioned by one level
constexpr int kRangeBits = 11;                // partitions per merge range = 2048
constexpr int kRangeParts = 1 << kRangeBits;
constexpr int kMaxRanges = kBucketThreads;    // per-bucket range histogram <= one block scan
// More partitions than kMaxRanges ranges of 2^kRangeBits: the bucket kernel
// groups kept pairs by coarse ranges of 2^range_bits partitions (<= kCoarseRanges
// of them), k_split_* re-sort each coarse range's records into its
// 2^kRangeBits-partition ranges, k_fine_reduce sums them (two-level merge)
constexpr int kCoarseRanges = 256;
#ifndef PDP_RANGE_THREADS
#define PDP_RANGE_THREADS 1024
#endif
constexpr int kRangeThreads = PDP_RANGE_THREADS;  // k_range_plan workgroups
// range-reduce work item: the records of one partition range from a run of
// consecutive buckets, cut at bucket boundaries every kRangeChunk records
// (k_range_plan), so a Zipf-hot range spreads over many workgroups and a cold
// one is a single item
constexpr int64_t kRangeChunk = 8192;
constexpr unsigned kRangeDirect = 256;        // records below which a workgroup adds them directly
// k_range_reduce / k_fine_reduce workgroups: 512 threads (two per CU by their
// 68 KB of LDS: 16 waves, not 8): C3 k_range_reduce 0.275 -> 0.195 ms, C4
// k_fine_reduce 0.574 -> 0.540 (1,024: 0.212 / 0.537; profiles/r05/ab/ab12_merge_threads.txt)
constexpr int kReduceThreads = 512;
#ifndef PDP_SPLIT_THREADS
#define PDP_SPLIT_THREADS 512
#endif
constexpr int kSplitThreads = PDP_SPLIT_THREADS;  // k_split_count / k_split_scatter workgroups
constexpr size_t kRangeLds = kRangeParts * (3 * 8 + 2 * 4) + kReduceThreads * (8 + 4) + (kReduceThreads / 64 + 1) * 4;
constexpr int kQueueCap = 128;                // per-wave candidate queue (bucket kernel)
constexpr int kScanItems = 16;
constexpr int kScanChunk = kBlock * kScanItems;

constexpr int64_t kL1LocalLds = 150 * 1024;  // tile-local level 1: LDS cap (one 1,024-thread workgroup per CU)
size_t l1_stage_bytes(int key_format);       // LDS of one level-1 stage (after StageLds)
// tile-local level 1 bucket counts in LDS: u32 per bucket when they fit,
// else two u16 per word, flushed every half tile (32,768 rows: no carry) to
// counts_tm (first half) and counts_tm2 (second half)
inline int64_t l1_hist_bytes(int64_t n_buckets, bool u16) { return ((u16 ? 2 : 4) * n_buckets + 15) / 16 * 16; }
inline bool l1_hist_u16(int key_format, int64_t n_buckets) {
  return (int64_t)l1_stage_bytes(key_format) + l1_hist_bytes(n_buckets, false) > kL1LocalLds;
}

// ---- threshold sieve (Plan.sieve) ----------------------------------------
// With cross-partition sampling, a privacy id keeps the l0 pairs of smallest
// pair key, and its other pairs (usually most of its rows) contribute
// nothing.  The sieve keeps only rows whose 32-bit pair hash is below one
// global threshold t32 = sieve << 16: if a privacy id has >= l0 distinct
// pairs below it, its l0 smallest are among them, together with every row of
// those pairs (a pair's rows share its hash), so the level-1 pass writes and
// levels 2/3 read only those candidate rows.  Privacy ids with fewer than l0
// candidate pairs ("unresolved": the bucket kernel marks them in a bitmap
// and a list) are finished by a fix-up over ALL their rows: one streaming
// re-read of the privacy-id column (k_sieve_rescan, an LDS Bloom filter of
// the list in front of the exact bitmap), a scatter into bucket order and a
// second bucket-kernel launch whose pair records follow the main ones.
// Kept pairs and rows are exactly those of the unsieved path.
#ifndef PDP_SIEVE_BUFS
#define PDP_SIEVE_BUFS 2
#endif
#ifndef PDP_SIEVE_EARLY
#define PDP_SIEVE_EARLY 0
#endif
constexpr int kSieveChunkItems = 4;                            // rows per thread and chunk
constexpr int kSieveBufs = PDP_SIEVE_BUFS;  // full tiles: chunks of loads in flight (register buffers)
constexpr int kSieveItems = 12;  // stage slots per thread (records each thread handles at a flush)
// Two workgroup shapes (Plan.sieve_threads):
//  1,024 threads, a 12,288-candidate stage, 8 flush slots per tile: one
//    workgroup per CU (~150 KiB of LDS), whose flush (LDS counting sort +
//    block write) stalls the CU's loads;
//  512 threads, a 6,144-candidate stage, 16 flush slots per tile, <= 80 KiB of
//    LDS: two workgroups per CU, so one's flush overlaps the other's loads.
template <int TH>
struct SieveShape {
  static constexpr int kChunk = TH * kSieveChunkItems;  // rows filtered per chunk
  static constexpr int kCap = TH * kSieveItems;         // candidate slots of the LDS stage
  static constexpr int kSlots = TH == 1024 ? 8 : 16;    // flush blocks per tile, at most
  static constexpr int kSlotBits = TH == 1024 ? 3 : 4;
  // a tile flushes at most once per chunk, and every flush but its last holds
  // > kCap - kChunk records, so its blocks fit the kSlots level-1 slots
  static_assert((1 << kSlotBits) == kSlots, "slot bits");
  static_assert(kTileRows / kChunk <= kSlots || kTileRows / (kCap - kChunk + 1) + 1 <= kSlots,
                "sieve flushes per tile");
  static_assert(kCap <= 65535, "u16 run offsets");
};
constexpr int kSieveThreads2 = 512;
constexpr int64_t kSieveLds2 = 80 * 1024 - 256;  // two 512-thread workgroups per CU
// a tile's flush blocks lie back to back from tile * kSieveTileStride, its
// band list at tile * kBandTileStride
// (strides padded by 4 KiB measured 6 % slower at C3, profiles/r05/ab/ab1_l1_placement.txt)
// non-temporal loads (ld_nt) of the columns level 1 streams and of the band
// lists k_band_scan streams (C3 0.277 -> 0.255 ms); measured neutral or worse
// and not used: k_scatter_l1_local's key loads (C4 +0.03 ms), level 2's run
// loads and the bucket kernel's record stream (profiles/r05/ab/ab5_nt_loads.txt)
#ifndef PDP_L1_NT
#define PDP_L1_NT 1
#endif
#ifndef PDP_NT_BS
#define PDP_NT_BS 1
#endif

constexpr int64_t kSieveTileStride = kTileRows;
constexpr int64_t kBandTileStride = kTileRows;
constexpr int kSieveMaxT16 = 1 << 15;                          // t <= 1/2
// k_sieve_rescan: a 16 KiB LDS Bloom filter (a 64 KiB one limits the CU to
// two workgroups, and the rescan then streams at 3.7 instead of 6.1 TB/s:
// tools/stream_bench.hip, profiles/r03/stream_bench.txt); above
// kBloomMaxIds unresolved ids it is skipped and every row tests the bitmap
constexpr int kBloomWords = 4096;  // == 1 << kBloomBits
constexpr unsigned kBloomMaxIds = 8192;
constexpr int kRescanThreads = 512;
constexpr int kRescanBlocks = 1024;
// tile groups per level-2 workgroup with the sieve, at most: the plan takes
// as many as keep a workgroup's expected records (tiles x candidates per tile
// / super-buckets) within one LDS window (kL2Target), since a second window
// holding a few hundred records costs as much latency as a full one; and no
// more than one level-1 slot per level-2 thread
constexpr int kSieveL2Groups = 4;
constexpr double kL2Target = 7000.0;
size_t sieve_stage_bytes(int key_format, int threads);  // LDS of the sieve's level-1 stage (after StageLds)
// the side band (Plan.band): rows with t <= pair hash < t2 = 2t leave level 1
// as (privacy id << 32 | row) in a per-tile list, through a per-wave LDS queue
// written out 64 entries at a time; the fix-up reads that list instead of the
// whole privacy-id column, and only a privacy id with fewer than l0 distinct
// pairs below t2 still needs the rescan
constexpr int kBandQueue = 128;
inline int64_t sieve_band_lds(int threads) { return (threads / 64) * kBandQueue * 8; }
// LDS of a sieve workgroup: stage, bucket counts (u32, or u16 pairs), band queues
inline int64_t sieve_lds(int key_format, int threads, int64_t n_buckets, bool u16, bool band) {
  return ((int64_t)sieve_stage_bytes(key_format, threads) + 7) / 8 * 8 + l1_hist_bytes(n_buckets, u16) +
         (band ? sieve_band_lds(threads) : 0);
}

struct Plan {
  int algorithm;   // PDP_ALGO_*
  int pk_bits;
  int bucket_bits;
  int super_bits;
  int rand_shift;
  int64_t n_buckets;
  int64_t n_supers;
  int64_t n_tiles;
  int64_t lds_bytes;
  int merge;            // PDP_MERGE_* (bucketed)
  int n_ranges;         // PDP_MERGE_RANGES: ceil(P / 2^range_bits)
  int range_bits;       // partitions per merge range of the bucket kernel (kRangeBits, or coarse)
  int two_level;        // range_bits > kRangeBits: coarse ranges, then k_split_* / k_fine_*
  int64_t n_fine;       // two-level: ceil(P / 2^kRangeBits)
  int64_t fine_items;   // two-level: upper bound on the k_fine_reduce work items
  int64_t range_group;  // records per range-reduce work item (kRangeChunk)
  int64_t n_groups;     // upper bound on the range-reduce work items (+ one sentinel per range)
  int key_format;       // PDP_KEYS_WIDE / PDP_KEYS_COMPACT (bucketed)
  int l1_local;         // tile-local level 1 (k_scatter_l1_local / k_scatter_l2_local), no histogram pass
  int64_t n_stages;     // level-1 stages of kL1Rows rows
  int sieve;            // threshold sieve: t = sieve / 2^16 (0 = off); k_sieve_l1 instead of k_scatter_l1_local
  int band;             // side band: t2 = band / 2^16 (0 = off; else 2 * sieve, <= 1/2)
  int64_t n_slots1;     // level-1 blocks (stages, or sieve flush slots: n_tiles << slot_bits)
  int64_t buckets_out;  // buckets of pair records: n_buckets, x2 with the sieve (fix-up after), x3 with the band
  int l2_mult;          // tile groups per level-2 workgroup (1 without the sieve)
  int sieve_threads;    // k_sieve_l1 workgroup: 1,024 or 512 threads (SieveShape)
  int bucket_threads;   // k_bucket_bound workgroup: 1,024 or 512 threads (half-size buckets)
  int slot_bits;        // level-1 blocks per tile = 2^slot_bits (kStagesPerTile, or SieveShape::kSlots)
  int hist_u16;         // tile-local level 1 counts buckets in u16 halves (counts_tm / counts_tm2)
};

int64_t per_pid_lds(const pdp_bound_config* c) {
  const int64_t l0 = c->l0;
  const int64_t pair = 4 + (c->linf > 0 ? 8 * (int64_t)c->linf : 24);
  return l0 * 8 + l0 * pair;  // pair sketch + per-pair state
}

bool test_hooks_enabled();
Plan make_plan(const pdp_bound_config* c) {
  Plan p{};
  p.pk_bits = bits_for(c->n_partitions);
  const int64_t per_pid = per_pid_lds(c);
  // the bucket kernel's workgroup: 512 threads (on request) only where the
  // per-partition-range scan fits one thread per range
  const int64_t n_ranges_est = (c->n_partitions + kRangeParts - 1) >> kRangeBits;
  p.bucket_threads = c->bucket_threads == kBucketThreads / 2 &&
                             (n_ranges_est <= kBucketThreads / 2 || n_ranges_est > kMaxRanges)
                         ? kBucketThreads / 2
                         : kBucketThreads;
  const int64_t max_pids = (p.bucket_threads == kBucketThreads ? kLdsBudget : kLdsBudget2) / per_pid;
  int s = -1, s2 = 0;
  if (max_pids >= 16) {
    s = 0;
    while (((int64_t)2 << s) <= max_pids) ++s;          // largest 2^s <= max_pids
    if (test_hooks_enabled()) {  // test hook: smaller buckets (PIPELINEDP_AMD_BUCKET_BITS)
      const char* e = std::getenv("PIPELINEDP_AMD_BUCKET_BITS");
      if (e != nullptr && std::atoi(e) >= 4 && std::atoi(e) < s) s = std::atoi(e);
    }
    const int u_bits = bits_for(c->n_privacy_ids);
    if (s > u_bits) s = u_bits;                          // one bucket covers all pids
    const int64_t nb = (c->n_privacy_ids + ((int64_t)1 << s) - 1) >> s;
    if (nb > kSingleLevelMax) {
      // two levels: level 2's input runs are a stage's rows of one
      // super-bucket (kL1Rows / supers), its output runs a window's rows of
      // one bucket (kL2Rows / 2^s2); take the s2 whose shorter run is longest
      // (C3: 77 supers x 64 buckets, C2: 62 x 32)
      int lo = 1;
      while (((nb + ((int64_t)1 << lo) - 1) >> lo) > kMaxSupers) ++lo;
      double best = -1.0;
      for (int c = lo; c <= lo + 3 && ((int64_t)1 << c) < nb; ++c) {
        const double supers = (double)((nb + ((int64_t)1 << c) - 1) >> c);
        const double score = std::min((double)kL1Rows / supers, (double)kL2Rows / (double)((int64_t)1 << c));
        if (score > best) {
          best = score;
          s2 = c;
        }
      }
    }
    // pair keys: random bits above rand_shift = pk_bits + bucket_bits
    if (nb > kMaxBuckets || 64 - p.pk_bits - s < kMinRandomBits) s = -1;
  }
  const int auto_algo = s >= 0 ? PDP_ALGO_BUCKETED : PDP_ALGO_GLOBAL_SKETCH;
  p.algorithm = c->algorithm == PDP_ALGO_AUTO ? auto_algo : c->algorithm;
  if (p.algorithm == PDP_ALGO_BUCKETED && s < 0) p.algorithm = -1;  // infeasible
  p.bucket_bits = s < 0 ? 0 : s;
  p.super_bits = s < 0 ? 0 : s2;
  p.rand_shift = p.pk_bits + p.bucket_bits;
  p.n_buckets = (c->n_privacy_ids + ((int64_t)1 << p.bucket_bits) - 1) >> p.bucket_bits;
  p.n_supers = (p.n_buckets + ((int64_t)1 << p.super_bits) - 1) >> p.super_bits;
  p.n_tiles = (c->n_rows + kTileRows - 1) / kTileRows;
  if (p.n_tiles < 1) p.n_tiles = 1;
  p.lds_bytes = ((int64_t)1 << p.bucket_bits) * per_pid;
  p.range_bits = kRangeBits;
  p.n_fine = (c->n_partitions + kRangeParts - 1) >> kRangeBits;
  p.two_level = p.n_fine > kMaxRanges;
  if (p.two_level)
    while (((c->n_partitions + ((int64_t)1 << p.range_bits) - 1) >> p.range_bits) > kCoarseRanges) ++p.range_bits;
  p.n_ranges = (int)((c->n_partitions + ((int64_t)1 << p.range_bits) - 1) >> p.range_bits);
  const bool ranges_ok = p.n_ranges <= kMaxRanges;
  if (p.algorithm != PDP_ALGO_BUCKETED) {
    p.merge = 0;
  } else if (c->merge == PDP_MERGE_AUTO) {
    p.merge = ranges_ok ? PDP_MERGE_RANGES : PDP_MERGE_ATOMIC;
  } else {
    p.merge = c->merge;
    if (p.merge == PDP_MERGE_RANGES && !ranges_ok) p.algorithm = -1;  // infeasible
  }
  if (p.merge == PDP_MERGE_RANGES) {
    // per-bucket range histogram + cursors + block-scan scratch after the sketches
    p.lds_bytes += (2 * (int64_t)p.n_ranges + p.bucket_threads / 64 + 1) * 4;
  }
  // row records of the partition passes: u32 (sub-bucket, local pid,
  // partition) with bit 31 = dead when those fields fit (COMPACT); else the
  // level-1 u64 packed record with a tile-relative row, then COMPACT pairs
  // (PACKED); else the u64 pair key + u32 row (WIDE)
  const bool compact_ok = p.super_bits + p.bucket_bits + p.pk_bits <= 31;
  const bool packed_ok = p.bucket_bits + p.pk_bits <= 31 &&
                         p.super_bits + p.bucket_bits + p.pk_bits <= 64 - 1 - kTileRowBits;
  // PACKED level 1 with WIDE records from level 2 on (tile-local level 1 only)
  const bool packed_wide_ok = p.super_bits + p.bucket_bits + p.pk_bits <= 64 - 1 - kTileRowBits;
  // ... or with one u64 per record (PACKED64): the row above the bucket-local
  // pid and partition, all ones reserved for dead records
  const int row_bits = 64 - p.bucket_bits - p.pk_bits;
  const bool packed64_ok = packed_wide_ok && (row_bits >= 33 || c->n_rows < ((int64_t)1 << row_bits) - 2);
  p.key_format = 0;
  p.n_stages = (c->n_rows + kL1Rows - 1) / kL1Rows;
  p.l1_local = 0;
  if (p.algorithm == PDP_ALGO_BUCKETED) {
    // tile-local level 1: two levels, and the bucket counts in its LDS
    auto local_fits = [&](int fmt) {
      return p.super_bits > 0 &&
             (int64_t)l1_stage_bytes(fmt) + l1_hist_bytes(p.n_buckets, true) <= kL1LocalLds;
    };
    const int want = c->key_format;
    if (want == PDP_KEYS_AUTO) {
      // tile-local: PACKED (one u64 array at level 1, so level 2 reads each
      // run as one span), else PACKED_WIDE; else COMPACT / PACKED / WIDE
      if (packed_ok && local_fits(PDP_KEYS_PACKED))
        p.key_format = PDP_KEYS_PACKED;
      else if (!packed_ok && packed64_ok && local_fits(PDP_KEYS_PACKED64))
        p.key_format = PDP_KEYS_PACKED64;
      else if (!packed_ok && packed_wide_ok && local_fits(PDP_KEYS_PACKED_WIDE))
        p.key_format = PDP_KEYS_PACKED_WIDE;
      else
        p.key_format = compact_ok ? PDP_KEYS_COMPACT : (packed_ok ? PDP_KEYS_PACKED : PDP_KEYS_WIDE);
    } else if ((want == PDP_KEYS_COMPACT && !compact_ok) || (want == PDP_KEYS_PACKED && !packed_ok) ||
               (want == PDP_KEYS_PACKED_WIDE && !(packed_wide_ok && local_fits(PDP_KEYS_PACKED_WIDE))) ||
               (want == PDP_KEYS_PACKED64 && !(packed64_ok && local_fits(PDP_KEYS_PACKED64)))) {
      p.algorithm = -1;  // infeasible
    } else {
      p.key_format = want;
    }
    // one super-bucket (no level 2): PACKED degenerates to COMPACT, which then fits
    if (p.key_format == PDP_KEYS_PACKED && p.super_bits == 0) p.key_format = PDP_KEYS_COMPACT;
    if (p.algorithm == PDP_ALGO_BUCKETED) p.l1_local = local_fits(p.key_format) ? 1 : 0;
  }
  // threshold sieve: tile-local level 1, range merge, whole 64-pid bitmap
  // words per bucket, and the sieve's larger LDS stage must fit
  const bool sieve_ok = p.algorithm == PDP_ALGO_BUCKETED && p.l1_local && p.merge == PDP_MERGE_RANGES &&
                        p.bucket_bits >= 6 && p.key_format != PDP_KEYS_WIDE &&
                        sieve_lds(p.key_format, kL1Threads, p.n_buckets, true, false) <= kL1LocalLds &&
                        p.n_tiles * kSieveTileStride < ((int64_t)1 << 32) &&
                        c->n_privacy_ids < ((int64_t)1 << 32) - 1;  // fix-up lists hold 32-bit ids
  int t16 = 0;
  if (sieve_ok && c->sieve > 0) {
    t16 = c->sieve < kSieveMaxT16 ? c->sieve : kSieveMaxT16;
  } else if (sieve_ok && c->sieve == 0) {
    // auto: a privacy id with d distinct partitions has ~d*t candidate pairs;
    // ask for l0 + 3 sqrt(l0) + 3 of them, assuming d ~ 0.6 rows per id
    // (C3: 100 rows over Zipf(1.1) keys, t = 0.15); no sieve above t = 0.35
    const double rows_per_id = (double)c->n_rows / (double)c->n_privacy_ids;
    const double want = c->l0 + 3.0 * std::sqrt((double)c->l0) + 3.0;
    const double t = want / (0.6 * rows_per_id);
    if (t <= 0.35) t16 = (int)std::ceil(t * 65536.0);
  }
  p.sieve = t16 > 0 ? t16 : 0;
  p.band = 0;
  if (p.sieve) {
    const int t2 = 2 * p.sieve < kSieveMaxT16 ? 2 * p.sieve : kSieveMaxT16;
    const bool fits = sieve_lds(p.key_format, kL1Threads, p.n_buckets, true, true) <= kL1LocalLds;
    // auto: only below t = 1/4 -- there an id short of l0 candidate pairs,
    // and with it the 8 B/row rescan, is likely (C3: t = 0.154, ~1,600 of 1e7
    // ids; C2's t = 0.325 leaves none, and the band would only cost level 1
    // its writes: 1.43 -> 1.52 ms, profiles/r03/ab/ab4_band.txt)
    const bool want = c->sieve_band > 0 || (c->sieve_band == 0 && p.sieve <= kSieveMaxT16 / 2);
    if (t2 > p.sieve && fits && want) p.band = t2;
  }
  // the sieve's workgroup: 1,024 threads (auto), or on request two 512-thread
  // ones per CU when their LDS fits (C3: 6.86 vs 6.56 ms, level 1 3.51 vs
  // 3.44 ms and level 2 0.97 vs 0.80 ms over twice the flush blocks,
  // profiles/r04/ab/ab1_sieve_threads.txt)
  p.sieve_threads = kL1Threads;
  p.hist_u16 = p.l1_local ? (int)l1_hist_u16(p.key_format, p.n_buckets) : 0;
  if (p.sieve) {
    const bool band = p.band != 0;
    p.hist_u16 = sieve_lds(p.key_format, kL1Threads, p.n_buckets, false, band) > kL1LocalLds;
    const bool u16_2 = sieve_lds(p.key_format, kSieveThreads2, p.n_buckets, false, band) > kSieveLds2;
    const bool fits2 = sieve_lds(p.key_format, kSieveThreads2, p.n_buckets, u16_2, band) <= kSieveLds2;
    if (fits2 && c->sieve_threads == kSieveThreads2) {
      p.sieve_threads = kSieveThreads2;
      p.hist_u16 = u16_2;
    }
  }
  p.slot_bits = p.sieve_threads == kSieveThreads2 ? SieveShape<kSieveThreads2>::kSlotBits
                                                   : SieveShape<kL1Threads>::kSlotBits;
  if (!p.sieve) p.slot_bits = 3;
  static_assert(kStagesPerTile == 8, "non-sieve level-1 stages per tile = 2^3");
  p.n_slots1 = p.sieve ? p.n_tiles << p.slot_bits : p.n_stages;
  p.buckets_out = p.sieve ? (p.band ? 3 : 2) * p.n_buckets : p.n_buckets;
  p.l2_mult = 1;
  if (p.sieve) {
    // expected records of one (group of kL2GroupTiles tiles, super-bucket)
    const double per_group = (double)kL2GroupTiles * (double)kTileRows * ((double)p.sieve / 65536.0) /
                             (double)(p.n_supers > 0 ? p.n_supers : 1);
    int m = (int)(kL2Target / (per_group > 1.0 ? per_group : 1.0));
    const int m_max = kL2Threads / (kL2GroupTiles << p.slot_bits);  // one slot per level-2 thread
    const int cap = kSieveL2Groups < m_max ? kSieveL2Groups : m_max;
    p.l2_mult = m < 1 ? 1 : (m > cap ? cap : m);
  }
  if (p.algorithm == PDP_ALGO_BUCKETED) {  // candidate queues (key + row) per wave + pid hashes
    p.lds_bytes = ((p.lds_bytes + 7) & ~(int64_t)7) + (p.bucket_threads / 64) * kQueueCap * 12;
    p.lds_bytes += ((int64_t)8 << p.bucket_bits);  // {pid hash, sketch-maximum high half} per pid
  }
  if (p.merge == PDP_MERGE_RANGES) {
    // range r yields ceil(records_r / C) items + 1 sentinel, and a bucket
    // emits at most l0 * 2^bucket_bits records in all
    const int64_t recs = p.buckets_out * ((int64_t)c->l0 << p.bucket_bits);
    p.range_group = kRangeChunk;
    p.n_groups = recs / kRangeChunk + 2 * (int64_t)p.n_ranges + 1;
    p.fine_items = p.two_level ? recs / kRangeChunk + p.n_fine + 1 : 0;
  } else {
    p.n_ranges = 0;
    p.range_group = 0;
    p.n_groups = 0;
    p.two_level = 0;
    p.fine_items = 0;
  }
  return p;
}

struct Ws {
  // common
  uint64_t err;
  // global path
  uint64_t sketch, cnt, rows, fsum, nsum, nsum2;
  // bucketed path
  uint64_t counts_tm, counts, chunk_sums, super_base, super_tm, super_off, keys1, rows1, keys2, rows2;
  uint64_t csum, gcur;  // level-2 cursor scans: per tile chunk, per tile group (x n_buckets)
  uint64_t cand_key, cand_idx;  // bucket kernel: B1's candidate list (record-local key, row)
  uint64_t soff;                // tile-local level 1: per stage, super-bucket run starts (u16)
  uint64_t counts_tm2;          // tile-local level 1, u16 counts: second half-tile bucket counts
  // threshold sieve: flush-block starts (u32 per slot), unresolved privacy
  // ids (bitmap + list), {unresolved count, fix-up rows}, fix-up rows per
  // bucket (-> starts) and their write cursors; the fix-up row list itself
  // reuses keys1 (dead after level 2), its bucket-ordered records keys2/rows2
  uint64_t sbase, unres_bits, unres_list, sctl, fix_cnt, fix_cur;
  // the fix-up's (id << 32 | row) list: the level-1 region (keys1, and rows1
  // right after it for COMPACT records), dead after level 2; fix_cap entries
  // (>= n_rows: every list holds distinct rows)
  uint64_t fix_rec, fix_cap;
  // side band: per-tile (pid << 32 | row) lists and their lengths; the ids
  // still unresolved after the band fix-up (bitmap, list, {count, rows}) and
  // their rescan's per-bucket counts / cursors
  uint64_t band, band_cnt, unres2_bits, unres2_list, sctl2, fix_cnt2, fix_cur2;
  uint64_t fix_blist;  // fix-up bucket launches: {count, buckets holding fix-up rows...}
  uint64_t tile_over;  // tile-local level 1: per tile, the bucket holding all 65,536 of its rows (else ~0)
  // bucketed PDP_MERGE_RANGES: pair records per bucket block, grouped by range
  uint64_t runs, rec_key, rec_f0, rec_f1, rec_f2;
  uint64_t rr_items, rr_count;  // range-reduce work items (uint4) and their count
  // two-level merge: fine-range totals / starts (+ scan scratch), write cursors,
  // the records re-sorted by fine range, fine work items and their count
  uint64_t fine_total, fine_chunks, fine_cur, stg_key, stg_f0, stg_f1, stg_f2, fine_items, fine_count;
  uint64_t item_hist;  // two-level: per coarse work item, its records per fine range (k_split_count)
  uint64_t total;
};

// row stride of the per-tile bucket counts in buckets (KP.cstride): whole
// 16-byte rows of u16 pairs (tile-local level 1) or u32 counts, so
// k_gscan_sums reads eight or four buckets per lane
inline int64_t counts_stride(int64_t n_buckets) { return (n_buckets + 7) & ~(int64_t)7; }

Ws layout(const pdp_bound_config* c, const Plan& p) {
  Ws w{};
  uint64_t off = 0;
  w.err = off;
  off = align256(off + 16);
  if (p.algorithm == PDP_ALGO_GLOBAL_SKETCH) {
    const uint64_t slots = (uint64_t)c->n_privacy_ids * (uint64_t)c->l0;
    w.sketch = off; off = align256(off + slots * 8);
    w.cnt = off; off = align256(off + slots * 4);
    if (c->linf > 0) {
      w.rows = off; off = align256(off + slots * (uint64_t)c->linf * 8);
    } else {
      w.fsum = off; off = align256(off + slots * 8);  // double or int64
      w.nsum = off; off = align256(off + slots * 8);
      w.nsum2 = off; off = align256(off + slots * 8);
    }
  } else {
    const uint64_t n_counts = (uint64_t)counts_stride(p.n_buckets) * (uint64_t)p.n_tiles;
    const uint64_t n_chunks = ((uint64_t)p.n_buckets + kScanChunk - 1) / kScanChunk;
    const uint64_t n = (uint64_t)c->n_rows;
    w.counts_tm = off; off = align256(off + n_counts * 4);
    const bool u16 = p.hist_u16 != 0;
    if (p.l1_local && u16) { w.counts_tm2 = off; off = align256(off + n_counts * 4); }
    w.tile_over = off; off = align256(off + (uint64_t)p.n_tiles * 4);
    w.counts = off; off = align256(off + ((uint64_t)p.n_buckets + 1) * 4);  // bucket starts
    w.chunk_sums = off; off = align256(off + (n_chunks + 1) * 4);
    const uint64_t n_sc = ((uint64_t)p.n_tiles + kScanChunkTiles - 1) / kScanChunkTiles;
    const uint64_t n_grp = ((uint64_t)p.n_tiles + kL2GroupTiles - 1) / kL2GroupTiles;
    w.csum = off; off = align256(off + n_sc * (uint64_t)p.n_buckets * 4);
    w.gcur = off; off = align256(off + n_grp * (uint64_t)p.n_buckets * 4);
    w.super_base = off; off = align256(off + (uint64_t)(p.n_supers + 1) * 4);
    w.super_tm = off; off = align256(off + (uint64_t)p.n_tiles * p.n_supers * 4);
    w.super_off = off; off = align256(off + (uint64_t)p.n_tiles * p.n_supers * 4);
    const bool packed = (p.key_format == PDP_KEYS_PACKED || p.key_format == PDP_KEYS_PACKED_WIDE ||
                         p.key_format == PDP_KEYS_PACKED64) && p.super_bits > 0;
    const uint64_t kb1 = p.key_format == PDP_KEYS_COMPACT ? 4 : 8;  // level-1 key
    const uint64_t kb2 = (p.key_format == PDP_KEYS_WIDE || p.key_format == PDP_KEYS_PACKED_WIDE ||
                          p.key_format == PDP_KEYS_PACKED64) ? 8 : 4;  // level-2 key
    const bool rows2 = p.key_format != PDP_KEYS_PACKED64;  // PACKED64: the row rides in the key
    // level-1 records: stage blocks, or the sieve's per-tile flush blocks
    const uint64_t n1 = p.sieve ? (uint64_t)p.n_tiles * kSieveTileStride
                                : (p.l1_local ? (uint64_t)p.n_stages * kL1Rows : n);
    w.keys1 = off; off = align256(off + n1 * (packed ? 8 : kb1));
    if (!packed) { w.rows1 = off; off = align256(off + n1 * 4); }
    if (p.sieve) {  // the fix-up list reuses [keys1, end of rows1), at least 8 B per row
      if (off - w.keys1 < 8 * n) off = w.keys1 + align256(8 * n);
      w.fix_rec = w.keys1;
      w.fix_cap = (off - w.keys1) / 8;
    }
    if (p.l1_local) { w.soff = off; off = align256(off + (uint64_t)p.n_slots1 * (p.n_supers + 1) * 2); }
    if (p.sieve) {
      const uint64_t ids = (uint64_t)p.n_buckets << p.bucket_bits;
      w.sbase = off; off = align256(off + (uint64_t)p.n_slots1 * 4);
      w.unres_bits = off; off = align256(off + ids / 8);
      w.unres_list = off; off = align256(off + ids * 4);
      w.sctl = off; off = align256(off + 16);
      w.fix_cnt = off; off = align256(off + ((uint64_t)p.n_buckets + 1) * 4);
      w.fix_cur = off; off = align256(off + (uint64_t)p.n_buckets * 4);
      w.fix_blist = off; off = align256(off + ((uint64_t)p.n_buckets + 1) * 4);
      if (p.band) {  // the band lists; the second fix-up's unresolved ids and counts
        w.band = off; off = align256(off + (uint64_t)p.n_tiles * kBandTileStride * 8);
        w.band_cnt = off; off = align256(off + (uint64_t)p.n_tiles * 4);
        w.unres2_bits = off; off = align256(off + ids / 8);
        w.unres2_list = off; off = align256(off + ids * 4);
        w.sctl2 = w.sctl + 8;  // {count, rows} beside sctl's: pdp_bound_stats_async reads both with one copy
        w.fix_cnt2 = off; off = align256(off + ((uint64_t)p.n_buckets + 1) * 4);
        w.fix_cur2 = off; off = align256(off + (uint64_t)p.n_buckets * 4);
      }
    }
    if (p.super_bits > 0) {
      w.keys2 = off; off = align256(off + n * kb2);
      if (rows2) { w.rows2 = off; off = align256(off + n * 4); }
      else w.rows2 = w.keys2;  // unused
    } else {
      w.keys2 = w.keys1;
      w.rows2 = w.rows1;
    }
    w.cand_key = off; off = align256(off + n * kb2);
    w.cand_idx = off; off = align256(off + n * 4);
    if (p.merge == PDP_MERGE_RANGES) {
      const uint64_t recs = (uint64_t)p.buckets_out * ((uint64_t)c->l0 << p.bucket_bits);
      w.runs = off; off = align256(off + (uint64_t)p.buckets_out * (p.n_ranges + 1) * 4);
      w.rec_key = off; off = align256(off + recs * 8);
      if (c->flags & (PDP_ACC_SUM | PDP_SUM_PER_PARTITION)) { w.rec_f0 = off; off = align256(off + recs * 8); }
      if (c->flags & PDP_ACC_NSUM) { w.rec_f1 = off; off = align256(off + recs * 8); }
      if (c->flags & PDP_ACC_NSUM2) { w.rec_f2 = off; off = align256(off + recs * 8); }
      w.rr_items = off; off = align256(off + (uint64_t)p.n_groups * 16);
      w.rr_count = off; off = align256(off + 16);
      if (p.two_level) {  // fine-range counts, starts, cursors; records re-sorted by fine range
        const uint64_t nf = (uint64_t)p.n_fine;
        w.fine_total = off; off = align256(off + (nf + 1) * 4);
        w.fine_chunks = off; off = align256(off + (uint64_t)scan_chunk_sums_len((int64_t)nf) * 4);
        w.fine_cur = off; off = align256(off + nf * 4);
        w.stg_key = off; off = align256(off + recs * 8);
        if (w.rec_f0) { w.stg_f0 = off; off = align256(off + recs * 8); }
        if (w.rec_f1) { w.stg_f1 = off; off = align256(off + recs * 8); }
        if (w.rec_f2) { w.stg_f2 = off; off = align256(off + recs * 8); }
        w.fine_items = off; off = align256(off + (uint64_t)p.fine_items * 16);
        w.fine_count = off; off = align256(off + 16);
        const uint64_t F = (uint64_t)1 << (p.range_bits - kRangeBits);
        w.item_hist = off; off = align256(off + (uint64_t)p.n_groups * F * 4);
      }
    }
  }
  w.total = off;
  return w;
}

// PDP_DEBUG_CORRUPT_RECORDS deliberately corrupts the level-2 records: only
// accepted when the process asked for test hooks
bool test_hooks_enabled() {
  const char* v = std::getenv("PIPELINEDP_AMD_TEST_HOOKS");
  return v != nullptr && v[0] == '1';
}

int validate(const pdp_bound_config* c) {
  if (c == nullptr) return set_error(PDP_E_INVALID, "config is NULL");
  if (c->n_rows < 0 || c->n_rows >= ((int64_t)1 << 32))
    return set_error(PDP_E_INVALID, "n_rows must be in [0, 2^32)");
  if (c->n_privacy_ids < 1 || c->n_privacy_ids >= ((int64_t)1 << 40))
    return set_error(PDP_E_INVALID, "n_privacy_ids must be in [1, 2^40)");
  if (c->n_partitions < 1 || c->n_partitions >= ((int64_t)1 << 32))
    return set_error(PDP_E_INVALID, "n_partitions must be in [1, 2^32)");
  if (c->l0 < 0 || c->l0 > PDP_MAX_L0)
    return set_error(PDP_E_UNSUPPORTED, "l0 out of supported range [0, PDP_MAX_L0]");
  if (c->linf < 0 || c->linf > PDP_MAX_LINF)
    return set_error(PDP_E_UNSUPPORTED, "linf out of supported range [0, PDP_MAX_LINF]");
  if (c->max_contributions < 0 || c->max_contributions > PDP_MAX_CONTRIBUTIONS)
    return set_error(PDP_E_UNSUPPORTED, "max_contributions out of supported range [0, PDP_MAX_CONTRIBUTIONS]");
  if (c->value_kind < PDP_VALUE_NONE || c->value_kind > PDP_VALUE_I64)
    return set_error(PDP_E_INVALID, "bad value_kind");
  if (c->value_kind != PDP_VALUE_I64 && (c->flags & PDP_SUM_INT))
    return set_error(PDP_E_INVALID, "PDP_SUM_INT requires int64 values");
  if (c->algorithm < PDP_ALGO_AUTO || c->algorithm > PDP_ALGO_PAIR_TABLE)
    return set_error(PDP_E_INVALID, "bad algorithm");
  if (c->merge < PDP_MERGE_AUTO || c->merge > PDP_MERGE_RANGES)
    return set_error(PDP_E_INVALID, "bad merge");
  if (c->key_format < PDP_KEYS_AUTO || c->key_format > PDP_KEYS_PACKED64)
    return set_error(PDP_E_INVALID, "bad key_format");
  if (c->sieve_threads != 0 && c->sieve_threads != kSieveThreads2 && c->sieve_threads != kL1Threads)
    return set_error(PDP_E_INVALID, "sieve_threads must be 0, 512 or 1024");
  if (c->bucket_threads != 0 && c->bucket_threads != kBucketThreads / 2 && c->bucket_threads != kBucketThreads)
    return set_error(PDP_E_INVALID, "bucket_threads must be 0, 512 or 1024");
  if ((c->flags & PDP_DEBUG_CORRUPT_RECORDS) && !test_hooks_enabled())
    return set_error(PDP_E_INVALID, "PDP_DEBUG_CORRUPT_RECORDS is a test hook: set PIPELINEDP_AMD_TEST_HOOKS=1");
  if (pairs_mode(c)) return pairs_validate(c);
  if (make_plan(c).algorithm < 0)
    return set_error(PDP_E_UNSUPPORTED, "bucketed algorithm / range merge / compact keys infeasible for this l0/linf/U/P");
  return PDP_OK;
}


struct KP {  // kernel parameters
  int64_t n, U, P;
  int l0, linf;
  int pk_bits, bucket_bits, super_bits, rand_shift;
  int64_t n_buckets, n_supers, n_tiles;
  int n_ranges;
  int range_bits;
  int64_t n_fine_ranges;  // two-level merge: ceil(P / 2^kRangeBits)
  int keys_vec;  // privacy_id / partition_key columns are 16-byte aligned
  uint64_t pk_mask, seed, row_seed;
  int64_t row_offset;
  int64_t cstride;  // row stride of counts_tm / counts_tm2 in buckets: n_buckets rounded up to 8
  ClipParams clip;
  int64_t n_slots1;     // level-1 blocks read by level 2 (Plan.n_slots1)
  int l2_group_mult;    // tile groups per level-2 workgroup
  uint32_t sieve_t32;   // threshold sieve: candidate rows have pair_hash < sieve_t32 (0 = off)
  int sieve_mark;       // bucket kernel: mark privacy ids with < l0 candidate pairs unresolved
  uint32_t band_t32;    // side band: level 1 lists rows with sieve_t32 <= pair_hash < band_t32 (0 = off)
  int sieve_emit;       // bucket kernel (main launch, band on): unresolved ids' candidate rows -> fix_rec
  int slot_bits;        // level-1 blocks per tile = 2^slot_bits (Plan.slot_bits)
  int64_t fix_cap;      // sieve: entries the fix-up row list (fix_rec, Ws.fix_rec) holds
  int row_shift;        // PACKED64 level-2 records: the row's first bit (pk_bits + bucket_bits)
};

KP make_kp(const pdp_bound_config* c, const Plan& p) {
  KP k;
  k.n = c->n_rows;
  k.U = c->n_privacy_ids;
  k.P = c->n_partitions;
  k.l0 = c->l0;
  k.linf = c->linf;
  k.pk_bits = p.pk_bits;
  k.bucket_bits = p.bucket_bits;
  k.super_bits = p.super_bits;
  k.rand_shift = p.rand_shift;
  k.n_buckets = p.n_buckets;
  k.n_supers = p.n_supers;
  k.n_tiles = p.n_tiles;
  k.n_ranges = p.n_ranges;
  k.range_bits = p.range_bits;
  k.n_fine_ranges = p.n_fine;
  k.keys_vec = 0;
  k.n_slots1 = p.n_slots1;
  k.l2_group_mult = p.l2_mult;
  k.sieve_t32 = (uint32_t)p.sieve << 16;
  k.sieve_mark = p.sieve != 0;
  k.band_t32 = (uint32_t)p.band << 16;
  k.sieve_emit = p.band != 0;
  k.slot_bits = p.slot_bits;
  k.fix_cap = 0;  // set from the layout (Ws.fix_cap) where the fix-up runs
  k.row_shift = p.pk_bits + p.bucket_bits;
  k.pk_mask = (1ULL << p.pk_bits) - 1;
  k.seed = c->seed;
  k.row_seed = derive_row_seed(c->seed);
  k.row_offset = c->row_offset;
  k.cstride = counts_stride(p.n_buckets);
  k.clip = ClipParams{c->min_value, c->max_value, c->middle, c->min_sum, c->max_sum, c->flags};
  return k;
}

// ============================================================ GLOBAL path ==
__global__ void __launch_bounds__(kBlock) k_pair_sketch(KP kp, const int64_t* __restrict__ pid,
                                                        const int64_t* __restrict__ pk,
                                                        const uint8_t* __restrict__ allowed,
                                                        unsigned long long* sketch, unsigned int* err) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < kp.n; i += stride) {
    const int64_t u = pid[i];
    const int64_t k = pk[i];
    if (u < 0 || u >= kp.U || k < 0 || k >= kp.P) {
      atomicOr(err, 1u);
      continue;
    }
    if (allowed != nullptr && allowed[k] == 0) continue;
    const uint64_t x = pair_key(kp.seed, u, k, 0, kp.rand_shift);
    unsigned long long* s = sketch + u * kp.l0;
    if (x >= s[kp.l0 - 1]) continue;  // values only decrease: a stale read is safe
    sketch_insert(s, kp.l0, x);
  }
}

template <int VALUE_KIND, bool KEEP_ALL_ROWS>
__global__ void __launch_bounds__(kBlock) k_pair_rows(KP kp, const int64_t* __restrict__ pid,
                                                      const int64_t* __restrict__ pk,
                                                      const void* __restrict__ value,
                                                      const uint8_t* __restrict__ allowed,
                                                      const unsigned long long* __restrict__ sketch,
                                                      unsigned int* pair_cnt, unsigned long long* pair_rows,
                                                      double* pair_fsum, double* pair_nsum,
                                                      double* pair_nsum2) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < kp.n; i += stride) {
    const int64_t u = pid[i];
    const int64_t k = pk[i];
    if (u < 0 || u >= kp.U || k < 0 || k >= kp.P) continue;
    if (allowed != nullptr && allowed[k] == 0) continue;
    const uint64_t x = pair_key(kp.seed, u, k, 0, kp.rand_shift);
    const unsigned long long* s = sketch + u * kp.l0;
    if (x > s[kp.l0 - 1]) continue;
    const int j = sketch_find(s, kp.l0, x);
    if (j < 0) continue;
    const int64_t slot = u * kp.l0 + j;
    atomicAdd(pair_cnt + slot, 1u);
    if (!KEEP_ALL_ROWS) {
      const uint64_t y = row_key(kp.row_seed, kp.row_offset + i, (uint32_t)i);
      unsigned long long* r = pair_rows + slot * kp.linf;
      if (y < r[kp.linf - 1]) sketch_insert(r, kp.linf, y);
    } else {
      accumulate_row<VALUE_KIND>(value, (uint32_t)i, slot, pair_fsum, pair_nsum, pair_nsum2, kp.clip);
    }
  }
}

template <int VALUE_KIND, bool KEEP_ALL_ROWS>
__global__ void __launch_bounds__(kBlock) k_reduce_pairs(KP kp, const void* __restrict__ value,
                                                         const unsigned long long* __restrict__ sketch,
                                                         const unsigned int* __restrict__ pair_cnt,
                                                         const unsigned long long* __restrict__ pair_rows,
                                                         const double* __restrict__ pair_fsum,
                                                         const double* __restrict__ pair_nsum,
                                                         const double* __restrict__ pair_nsum2,
                                                         pdp_partition_accumulators acc) {
  const int64_t n_slots = kp.U * kp.l0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_slots; s += stride) {
    const uint64_t x = sketch[s];
    if (x == kEmpty) continue;
    const int64_t p = (int64_t)(x & kp.pk_mask);
    const unsigned int c = pair_cnt[s];
    if (c == 0) continue;
    PairSums ps;
    if (!KEEP_ALL_ROWS) {
      const long long m = c < (unsigned)kp.linf ? (long long)c : (long long)kp.linf;
      ps = pair_sums_from_rows<VALUE_KIND>(pair_rows + s * kp.linf, m, value, kp.clip);
    } else if (VALUE_KIND != PDP_VALUE_NONE) {
      ps = pair_sums_from_totals((long long)c, pair_fsum[s], pair_nsum[s], pair_nsum2[s], kp.clip);
    } else {
      ps = PairSums{(long long)c, 0, 0.0, 0.0, 0.0};
    }
    add_pair_to_partition(acc, p, ps, kp.clip.flags);
  }
}

// ========================================================== BUCKETED path ==
// A key whose random part is all ones is "dead" (non-public or invalid
// partition): it keeps its pid bits so it stays in its bucket, and is skipped.
__device__ __forceinline__ bool dead_key(uint64_t x, int rand_shift) {
  return (x | ((1ULL << rand_shift) - 1)) == kEmpty;
}

__global__ void __launch_bounds__(kPartThreads) k_part_hist(KP kp, const int64_t* __restrict__ pid,
                                                            unsigned* __restrict__ counts_tm,
                                                            unsigned* __restrict__ super_tm, unsigned* err) {
  extern __shared__ unsigned hist[];
  for (int64_t b = threadIdx.x; b < kp.n_buckets; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * kTileRows;
  const int64_t t1 = t0 + kTileRows < kp.n ? t0 + kTileRows : kp.n;
  for (int64_t i0 = t0 + 2 * (int64_t)threadIdx.x; i0 < t1; i0 += (int64_t)blockDim.x * kUnroll) {
    int64_t u[kUnroll];  // two consecutive rows per 16-byte load
#pragma unroll
    for (int k = 0; k < kUnroll; k += 2) {
      const int64_t i = i0 + (int64_t)k * blockDim.x;
      if (kp.keys_vec && i + 1 < t1) {
        const longlong2 a = *reinterpret_cast<const longlong2*>(pid + i);
        u[k] = a.x;
        u[k + 1] = a.y;
      } else {
        u[k] = i < t1 ? pid[i] : INT64_MIN;
        u[k + 1] = i + 1 < t1 ? pid[i + 1] : INT64_MIN;
      }
    }
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
      if (u[k] == INT64_MIN) continue;
      if (u[k] < 0 || u[k] >= kp.U) {
        atomicOr(err, 1u);
        continue;
      }
      atomicAdd(hist + (u[k] >> kp.bucket_bits), 1u);
    }
  }
  __syncthreads();
  unsigned* row = counts_tm + (int64_t)blockIdx.x * kp.cstride;  // tile-major: coalesced
  for (int64_t b = threadIdx.x; b < kp.n_buckets; b += blockDim.x) row[b] = hist[b];
  // this tile's rows per super-bucket (the level-1 scatter's destinations)
  const int64_t nsub = (int64_t)1 << kp.super_bits;
  for (int64_t B = threadIdx.x; B < kp.n_supers; B += blockDim.x) {
    unsigned v = 0;
    const int64_t b1 = (B + 1) * nsub < kp.n_buckets ? (B + 1) * nsub : kp.n_buckets;
    for (int64_t b = B * nsub; b < b1; ++b) v += hist[b];
    super_tm[(int64_t)blockIdx.x * kp.n_supers + B] = v;
  }
}


// Level-2 cursors.  Level 2 runs one workgroup per (group of kL2GroupTiles
// tiles, super-bucket): its records are the runs of those tiles in the
// super-bucket's region, and the rows of bucket b from tiles < t start at
// start[b] + sum over t' < t of counts_tm[t'][b].  These exclusive column
// scans of the tile histogram, taken at group boundaries, are computed in
// three passes over chunks of kScanWaves * kScanTiles tiles (one wave per
// kScanTiles tiles, one lane per bucket): chunk sums, a scan over chunks
// (which also gives the bucket totals), and the cursors at group starts.
// Level 2 then needs no atomics and writes every bucket's rows in tile order.

// counts_tm2 (nullable): the tile-local level 1's second half-tile counts
__device__ __forceinline__ unsigned tile_count(const unsigned* __restrict__ counts_tm,
                                               const unsigned* __restrict__ counts_tm2, int64_t i) {
  return counts_tm[i] + (counts_tm2 != nullptr ? counts_tm2[i] : 0u);
}

__device__ __forceinline__ unsigned tile_slab_sum(const unsigned* __restrict__ counts_tm,
                                                  const unsigned* __restrict__ counts_tm2, int64_t n_tiles,
                                                  int64_t n_buckets, int64_t cstride, int64_t b, int64_t t0) {
  unsigned v = 0;
#pragma unroll
  for (int j = 0; j < kScanTiles; ++j) {
    const int64_t t = t0 + j;
    if (t < n_tiles && b < n_buckets) v += tile_count(counts_tm, counts_tm2, t * cstride + b);
  }
  return v;
}

// csum[chunk][b] = rows of bucket b in the chunk's tiles; gsum (nullable):
// gsum[g][b] = rows of bucket b in the kL2GroupTiles tiles of group g.
// PACKED16: the count rows are u16 pairs (tile-local level 1,
// flush_counts16: cstride / 2 words per row, tile_over adds 65,536 back),
// eight buckets per lane; else u32 rows of cstride, four per lane.  16-byte
// loads, a wave's kScanTiles rows in flight together (C3: 149 MB of counts)
template <bool PACKED16>
__global__ void __launch_bounds__(64 * kScanWaves) k_gscan_sums(const unsigned* __restrict__ counts_tm,
                                                                 const unsigned* __restrict__ counts_tm2,
                                                                 const unsigned* __restrict__ tile_over,
                                                                 int64_t n_tiles, int64_t n_buckets, int64_t cstride,
                                                                 unsigned* __restrict__ csum,
                                                                 unsigned* __restrict__ gsum) {
  static_assert(kScanTiles % kL2GroupTiles == 0, "group sums end inside a wave's tiles");
  constexpr int V = PACKED16 ? 8 : 4;  // buckets per lane
  __shared__ unsigned part[kScanWaves][V][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b0 = ((int64_t)blockIdx.x * 64 + lane) * V;
  const int64_t t0 = (int64_t)blockIdx.y * kScanChunkTiles + (int64_t)w * kScanTiles;
  const int64_t row = PACKED16 ? cstride / 2 : cstride;  // u32 words per row
  const int64_t col = PACKED16 ? b0 / 2 : b0;
  const bool in = b0 < n_buckets;  // then the 16-byte load stays inside the row
  uint4 x[kScanTiles];
  // PACKED16 halves: each u16 of a half tile is <= 2^15 (32,768 rows), so the
  // sum of two can be exactly 2^16 (a bucket holding every row of the tile).
  // The halves are added lane by lane; a lane's carry (bit k of the tile's
  // byte: bucket b0 + k) goes to cy and is added back as 65,536 below
  unsigned cy[kScanTiles / 4];
#pragma unroll
  for (int j = 0; j < kScanTiles / 4; ++j) cy[j] = 0u;
  // (loading all kScanTiles tiles' words before the adds measured slower,
  // 0.084 -> 0.099 ms at C3: the register peak costs occupancy;
  // profiles/r06/ab/ab21_*)
#pragma unroll
  for (int j = 0; j < kScanTiles; ++j) {
    const int64_t t = t0 + j;
    x[j] = make_uint4(0u, 0u, 0u, 0u);
    if (in && t < n_tiles) {
      x[j] = *reinterpret_cast<const uint4*>(counts_tm + t * row + col);
      if (counts_tm2 != nullptr) {
        const uint4 y = *reinterpret_cast<const uint4*>(counts_tm2 + t * row + col);
        if constexpr (PACKED16) {
          const unsigned a[4] = {x[j].x, x[j].y, x[j].z, x[j].w}, b[4] = {y.x, y.y, y.z, y.w};
          unsigned s[4], c = 0u;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const unsigned lo = (a[k] & 0xFFFFu) + (b[k] & 0xFFFFu), hi = (a[k] >> 16) + (b[k] >> 16);
            s[k] = (lo & 0xFFFFu) | (hi << 16);
            c |= ((lo >> 16) | ((hi >> 16) << 1)) << (2 * k);
          }
          x[j] = make_uint4(s[0], s[1], s[2], s[3]);
          cy[j / 4] |= c << (8 * (j % 4));
        } else {
          x[j] = make_uint4(x[j].x + y.x, x[j].y + y.y, x[j].z + y.z, x[j].w + y.w);
        }
      }
    }
  }
  unsigned v[V], gv[V];
#pragma unroll
  for (int k = 0; k < V; ++k) v[k] = gv[k] = 0u;
#pragma unroll
  for (int j = 0; j < kScanTiles; ++j) {
    const unsigned e[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
#pragma unroll
    for (int k = 0; k < V; ++k)
      gv[k] += PACKED16 ? ((e[k / 2] >> (16 * (k & 1))) & 0xFFFFu) + (((cy[j / 4] >> (8 * (j % 4) + k)) & 1u) << 16)
                        : e[k];
    if (PACKED16 && tile_over != nullptr && in && t0 + j < n_tiles) {
      const unsigned o = tile_over[t0 + j];  // the bucket with all 65,536 rows, or ~0
#pragma unroll
      for (int k = 0; k < V; ++k) gv[k] += (o == (unsigned)(b0 + k)) ? 65536u : 0u;
    }
    if ((j + 1) % kL2GroupTiles == 0) {
      if (gsum != nullptr && in && t0 + j + 1 - kL2GroupTiles < n_tiles) {
        unsigned* g = gsum + ((t0 + j + 1) / kL2GroupTiles - 1) * n_buckets + b0;
#pragma unroll
        for (int k = 0; k < V; ++k)
          if (b0 + k < n_buckets) g[k] = gv[k];
      }
#pragma unroll
      for (int k = 0; k < V; ++k) {
        v[k] += gv[k];
        gv[k] = 0u;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < V; ++k) part[w][k][lane] = v[k];
  __syncthreads();
  if (w == 0 && in) {
    unsigned* c = csum + (int64_t)blockIdx.y * n_buckets + b0;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      unsigned sum = 0;
      for (int q = 0; q < kScanWaves; ++q) sum += part[q][k][lane];
      if (b0 + k < n_buckets) c[k] = sum;
    }
  }
}

// per bucket: exclusive scan of the chunk sums in place, total -> total[b]
__global__ void __launch_bounds__(kBlock) k_gscan_chunks(unsigned* __restrict__ csum, int64_t n_chunks,
                                                         int64_t n_buckets, unsigned* __restrict__ total) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_buckets) return;
  unsigned run = 0;
  constexpr int B = 16;  // loads in flight per thread (the in-place stores would serialise them)
  for (int64_t c0 = 0; c0 < n_chunks; c0 += B) {
    unsigned v[B];
#pragma unroll
    for (int j = 0; j < B; ++j) v[j] = c0 + j < n_chunks ? csum[(c0 + j) * n_buckets + b] : 0u;
#pragma unroll
    for (int j = 0; j < B; ++j) {
      if (c0 + j < n_chunks) csum[(c0 + j) * n_buckets + b] = run;
      run += v[j];
    }
  }
  total[b] = run;
}

// gcur[g][b] in place: the group sums of k_gscan_sums -> rows of bucket b in
// tiles < g * kL2GroupTiles (cpre: k_gscan_chunks' exclusive chunk sums)
__global__ void __launch_bounds__(kBlock) k_gscan_groups(const unsigned* __restrict__ cpre, int64_t n_tiles,
                                                         int64_t n_buckets, unsigned* __restrict__ gcur) {
  const int64_t n_sc = (n_tiles + kScanChunkTiles - 1) / kScanChunkTiles;
  const int64_t n_grp = (n_tiles + kL2GroupTiles - 1) / kL2GroupTiles;
  constexpr int kGroups = kScanChunkTiles / kL2GroupTiles;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_sc * n_buckets) return;
  const int64_t c = i / n_buckets, b = i % n_buckets;
  unsigned run = cpre[i];
  unsigned v[kGroups];  // all loads first (the in-place stores would serialise them)
#pragma unroll
  for (int k = 0; k < kGroups; ++k) {
    const int64_t g = c * kGroups + k;
    v[k] = g < n_grp ? gcur[g * n_buckets + b] : 0u;
  }
#pragma unroll
  for (int k = 0; k < kGroups; ++k) {
    const int64_t g = c * kGroups + k;
    if (g < n_grp) gcur[g * n_buckets + b] = run;
    run += v[k];
  }
}

// gcur[g][b] = rows of bucket b in tiles < g * kL2GroupTiles
__global__ void __launch_bounds__(64 * kScanWaves) k_gscan_cursors(const unsigned* __restrict__ counts_tm,
                                                                    const unsigned* __restrict__ counts_tm2,
                                                                    int64_t n_tiles, int64_t n_buckets,
                                                                    int64_t cstride,
                                                                    const unsigned* __restrict__ cpre,
                                                                    unsigned* __restrict__ gcur) {
  __shared__ unsigned part[kScanWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = (int64_t)blockIdx.x * 64 + lane;
  const int64_t t0 = (int64_t)blockIdx.y * kScanChunkTiles + (int64_t)w * kScanTiles;
  part[w][lane] = tile_slab_sum(counts_tm, counts_tm2, n_tiles, n_buckets, cstride, b, t0);
  __syncthreads();
  if (b >= n_buckets || t0 >= n_tiles) return;
  unsigned run = cpre[(int64_t)blockIdx.y * n_buckets + b];
  for (int k = 0; k < w; ++k) run += part[k][lane];
  for (int j = 0; j < kScanTiles; ++j) {
    const int64_t t = t0 + j;
    if (t >= n_tiles) break;
    if (t % kL2GroupTiles == 0) gcur[(t / kL2GroupTiles) * n_buckets + b] = run;
    run += tile_count(counts_tm, counts_tm2, t * cstride + b);
  }
}

// super_base[B] = start of super-bucket B
__global__ void __launch_bounds__(kBlock) k_super_bases(KP kp, const unsigned* __restrict__ counts,
                                                        unsigned* __restrict__ super_base) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= kp.n_supers) {
    const int64_t b = i << kp.super_bits;
    super_base[i] = counts[b < kp.n_buckets ? b : kp.n_buckets];
  }
}

// LDS-staged multi-destination write: the rows of one sub-chunk (ITEMS per
// thread) are counting-sorted by destination in LDS and each destination's
// run is then written contiguously at gcur[dest] (coalesced, long runs).
constexpr int kMaxDest = 1024;

// row record key of the partition passes: u64 record (PDP_KEYS_WIDE: dead bit
// 63, bucket-within-super and local pid, partition; expand_key gives its pair key) or u32
// compact record (PDP_KEYS_COMPACT, and PDP_KEYS_PACKED from level 2 on)
template <bool COMPACT>
using RecKey = typename std::conditional<COMPACT, uint32_t, unsigned long long>::type;
// level-1 record key per format (PACKED: the u64 packed record, no row array)
template <int FMT>
using L1Key = typename std::conditional<FMT == PDP_KEYS_COMPACT, uint32_t, unsigned long long>::type;
template <int FMT>
constexpr bool kPackedL1 =
    FMT == PDP_KEYS_PACKED || FMT == PDP_KEYS_PACKED_WIDE || FMT == PDP_KEYS_PACKED64;  // no level-1 row array
// level-2 (bucket-order) record key per format
template <int FMT>
using L2Key = RecKey<FMT != PDP_KEYS_WIDE && FMT != PDP_KEYS_PACKED_WIDE && FMT != PDP_KEYS_PACKED64>;
// level-2 records of the bucket kernel: u32 key + u32 row (COMPACT, and
// PACKED from level 2 on), u64 key + u32 row (WIDE, PACKED_WIDE), one u64
// with the row in its high bits (PACKED64; all ones = dead)
constexpr int kRecCompact = 0, kRecWide = 1, kRecP64 = 2;
template <int FMT>
constexpr int kRecOf = FMT == PDP_KEYS_PACKED64 ? kRecP64
                                                 : ((FMT == PDP_KEYS_WIDE || FMT == PDP_KEYS_PACKED_WIDE) ? kRecWide
                                                                                                          : kRecCompact);
inline int rec_of(int key_format) {
  return key_format == PDP_KEYS_PACKED64 ? kRecP64
                                         : ((key_format == PDP_KEYS_WIDE || key_format == PDP_KEYS_PACKED_WIDE)
                                                ? kRecWide : kRecCompact);
}

// MAXD destinations per stage; the small form (<= 256 destinations, u8 tags)
// fits four workgroups per CU with compact keys instead of three.  ROWS:
// the stage carries a u32 row array beside the keys.
template <typename K, int MAXD, bool ROWS, int N, int THREADS = kPartThreads>
struct StageLds {
  using D = typename std::conditional<(MAXD <= 256), uint8_t, unsigned short>::type;
  unsigned hist[MAXD];
  unsigned start[MAXD];
  unsigned gcur[MAXD];
  K keys[THREADS * N];
  unsigned rows[ROWS ? THREADS * N : 1];
  D dest[THREADS * N];
};
constexpr int kSmallDest = 256;  // u8 tags; 39.9 KB with compact keys: four workgroups per CU

size_t l1_stage_bytes(int key_format) {
  switch (key_format) {
    case PDP_KEYS_COMPACT: return sizeof(StageLds<L1Key<PDP_KEYS_COMPACT>, kSmallDest, true, kL1Items, kL1Threads>);
    case PDP_KEYS_PACKED:
    case PDP_KEYS_PACKED_WIDE:
    case PDP_KEYS_PACKED64: return sizeof(StageLds<L1Key<PDP_KEYS_PACKED>, kSmallDest, false, kL1Items, kL1Threads>);
    default: return sizeof(StageLds<L1Key<PDP_KEYS_WIDE>, kSmallDest, true, kL1Items, kL1Threads>);
  }
}

template <int TH>
size_t sieve_stage_bytes_t(int key_format) {
  switch (key_format) {
    case PDP_KEYS_COMPACT: return sizeof(StageLds<L1Key<PDP_KEYS_COMPACT>, kSmallDest, true, kSieveItems, TH>);
    case PDP_KEYS_PACKED:
    case PDP_KEYS_PACKED_WIDE:
    case PDP_KEYS_PACKED64: return sizeof(StageLds<L1Key<PDP_KEYS_PACKED>, kSmallDest, false, kSieveItems, TH>);
    default: return sizeof(StageLds<L1Key<PDP_KEYS_WIDE>, kSmallDest, true, kSieveItems, TH>);
  }
}
size_t sieve_stage_bytes(int key_format, int threads) {
  return threads == kSieveThreads2 ? sieve_stage_bytes_t<kSieveThreads2>(key_format)
                                   : sieve_stage_bytes_t<kL1Threads>(key_format);
}

// phase 1: histogram + local rank (dest < 0 = drop the row)
template <typename K, int MAXD, bool ROWS, int N, int TH>
__device__ __forceinline__ void stage_count(StageLds<K, MAXD, ROWS, N, TH>& s, int ndest, const int (&d)[N],
                                            unsigned (&rank)[N]) {
  for (int t = threadIdx.x; t < ndest; t += blockDim.x) s.hist[t] = 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < N; ++q) rank[q] = d[q] >= 0 ? atomicAdd(s.hist + d[q], 1u) : 0;
  __syncthreads();
  if (threadIdx.x < 64) {  // exclusive scan of hist by one wave
    const int lane = threadIdx.x;
    unsigned carry = 0;
    for (int base = 0; base < ndest; base += 64) {
      const unsigned v = base + lane < ndest ? s.hist[base + lane] : 0;
      unsigned incl = v;
      for (int off = 1; off < 64; off <<= 1) {
        const unsigned up = __shfl_up(incl, off, 64);
        if (lane >= off) incl += up;
      }
      if (base + lane < ndest) s.start[base + lane] = carry + incl - v;
      carry += __shfl(incl, 63, 64);
    }
  }
  __syncthreads();
}

// phase 2: place into the LDS stage, then write every run at gcur[dest]
template <typename K, int MAXD, bool ROWS, int N, int TH>
__device__ __forceinline__ void stage_write(StageLds<K, MAXD, ROWS, N, TH>& s, int ndest, const int (&d)[N],
                                            const unsigned (&rank)[N], const K (&x)[N],
                                            const unsigned (&r)[N], K* __restrict__ out_keys,
                                            unsigned* __restrict__ out_rows) {
#pragma unroll
  for (int q = 0; q < N; ++q) {
    if (d[q] < 0) continue;
    const unsigned slot = s.start[d[q]] + rank[q];
    s.keys[slot] = x[q];
    if (ROWS) s.rows[slot] = r[q];
    s.dest[slot] = (typename StageLds<K, MAXD, ROWS, N, TH>::D)d[q];
  }
  __syncthreads();
  const unsigned total = s.start[ndest - 1] + s.hist[ndest - 1];
  for (unsigned k = threadIdx.x; k < total; k += blockDim.x) {
    const unsigned dd = s.dest[k];
    const unsigned g = s.gcur[dd] + (k - s.start[dd]);
    out_keys[g] = s.keys[k];
    if (ROWS) out_rows[g] = s.rows[k];
  }
  __syncthreads();
}

// Compact row record: bit 31 = dead (non-public / invalid partition: skipped,
// but kept in its bucket), bits [pk_bits, pk_bits + bucket_bits + super_bits)
// = the pid's bucket-within-super and bucket-local bits, [0, pk_bits) = pk.
__device__ __forceinline__ uint32_t compact_key(const KP& kp, int64_t u, int64_t k, bool dead) {
  const uint32_t mid = (uint32_t)((uint64_t)u & ((1ULL << (kp.bucket_bits + kp.super_bits)) - 1));
  return dead ? (0x80000000u | (mid << kp.pk_bits)) : ((mid << kp.pk_bits) | (uint32_t)k);
}

// Packed level-1 record (PDP_KEYS_PACKED): bit 63 = dead, bits [47, 63) = the
// row's index within its 65,536-row tile, [pk_bits, pk_bits + bucket_bits +
// super_bits) = bucket-within-super and bucket-local pid, [0, pk_bits) = pk.
// The tile is not stored: level 2 recovers it from the record's position in
// its super-bucket region (the tiles' runs there are in tile order).
constexpr int kPackedRowShift = 63 - kTileRowBits;
__device__ __forceinline__ uint64_t packed_key(const KP& kp, int64_t u, int64_t k, uint32_t tile_row, bool dead) {
  const uint64_t mid = (uint64_t)u & ((1ULL << (kp.bucket_bits + kp.super_bits)) - 1);
  return (dead ? (1ULL << 63) : 0ULL) | ((uint64_t)tile_row << kPackedRowShift) | (mid << kp.pk_bits) |
         (dead ? 0ULL : (uint64_t)k);
}

// The pair key of a row record (dead records -> kEmpty, skipped): random
// bits from rand_shift = pk_bits + bucket_bits up, the bucket-local pid, the
// partition -- pair_key(seed, pid, pk, local << pk_bits, rand_shift).  hpid[]
// holds pid_hash of the bucket's 2^bucket_bits privacy ids (LDS).  COMPACT
// records are u32 (bit 31 dead), WIDE records u64 (bit 63 dead); both keep
// the bucket-within-super bits above the local pid, which the key drops.
__device__ __forceinline__ uint64_t expand_key(const KP& kp, const uint2* hpid, uint32_t v) {
  // COMPACT records have rand_shift = pk_bits + bucket_bits <= 31, so the
  // pair key is the 32-bit pair hash above the record's (local pid,
  // partition) bits -- the bucket-within-super bits above them dropped -- and
  // pair_key_from's all-ones guard cannot fire
  if (v >> 31) return kEmpty;
  const uint32_t local = (v >> kp.pk_bits) & ((1u << kp.bucket_bits) - 1);
  return ((uint64_t)pair_hash_from(hpid[local].x, kp.seed, (int64_t)(v & (uint32_t)kp.pk_mask)) << 32) |
         (v & ((1u << kp.rand_shift) - 1));
}
__device__ __forceinline__ uint64_t expand_key(const KP& kp, const uint2* hpid, unsigned long long v) {
  if (v >> 63) return kEmpty;
  const uint64_t local = (v >> kp.pk_bits) & ((1ULL << kp.bucket_bits) - 1);
  return pair_key_from(hpid[local].x, kp.seed, (int64_t)(v & kp.pk_mask), local << kp.pk_bits, kp.rand_shift);
}

// B1's candidate test in one LDS read: hpid[local] = {pid hash, high 32 bits
// of the pid's sketch maximum (or above it: the maximum only decreases)}; a
// record whose key's high half exceeds that cannot be at or below the
// maximum.  Returns the pair key of a candidate, kEmpty otherwise.
__device__ __forceinline__ uint64_t b1_candidate(const KP& kp, const uint2* hpid, uint32_t v) {
  if (v >> 31) return kEmpty;
  const uint32_t local = (v >> kp.pk_bits) & ((1u << kp.bucket_bits) - 1);
  const uint2 e = hpid[local];
  const uint32_t h = pair_hash_from(e.x, kp.seed, (int64_t)(v & (uint32_t)kp.pk_mask));
  return h <= e.y ? (((uint64_t)h << 32) | (v & ((1u << kp.rand_shift) - 1))) : kEmpty;
}
__device__ __forceinline__ uint64_t b1_candidate(const KP& kp, const uint2* hpid, unsigned long long v) {
  const uint64_t x = expand_key(kp, hpid, v);
  if (x == kEmpty) return kEmpty;
  const uint32_t local = (uint32_t)((v >> kp.pk_bits) & ((1ULL << kp.bucket_bits) - 1));
  return (uint32_t)(x >> 32) <= hpid[local].y ? x : kEmpty;
}

// Level 1: tile rows -> super-bucket regions (<= 64 destinations per tile).
template <int FMT>
__global__ void __launch_bounds__(kL1Threads)  k_scatter_l1(KP kp, const int64_t* __restrict__ pid,
                                                             const int64_t* __restrict__ pk,
                                                             const uint8_t* __restrict__ allowed,
                                                             const unsigned* __restrict__ super_off,
                                                             const unsigned* __restrict__ super_base,
                                                             L1Key<FMT>* __restrict__ keys1,
                                                             unsigned* __restrict__ rows1, unsigned* err) {
  using K = L1Key<FMT>;
  constexpr bool ROWS = FMT != PDP_KEYS_PACKED;
  extern __shared__ unsigned long long stage_raw[];
  static_assert(kMaxSupers <= kSmallDest, "level-1 destinations must fit the small stage");
  using SL = StageLds<K, kSmallDest, ROWS, kL1Items, kL1Threads>;
  SL& s = *reinterpret_cast<SL*>(stage_raw);
  const int64_t t = blockIdx.x;
  const int nd = (int)kp.n_supers;
  // this tile's first row in each super-bucket region (k_super_scan)
  for (int B = threadIdx.x; B < nd; B += blockDim.x) s.gcur[B] = super_base[B] + super_off[t * nd + B];
  __syncthreads();
  const int64_t t0 = t * kTileRows;
  const int64_t t1 = t0 + kTileRows < kp.n ? t0 + kTileRows : kp.n;
  const int mid_bits = kp.bucket_bits + kp.super_bits;
  const uint64_t mid_mask = (1ULL << mid_bits) - 1;
  // two consecutive rows per 16-byte load (tiles and chunks start even)
  auto load = [&](int64_t c0, int64_t (&u)[kL1Items], int64_t (&k)[kL1Items]) {
#pragma unroll
    for (int q = 0; q < kL1Items; q += 2) {
      const int64_t i = c0 + 2 * ((int64_t)threadIdx.x + (int64_t)(q / 2) * blockDim.x);
      if (kp.keys_vec && i + 1 < t1) {
        const longlong2 a = *reinterpret_cast<const longlong2*>(pid + i);
        const longlong2 c = *reinterpret_cast<const longlong2*>(pk + i);
        u[q] = a.x;
        u[q + 1] = a.y;
        k[q] = c.x;
        k[q + 1] = c.y;
      } else {
        u[q] = i < t1 ? pid[i] : -1;
        k[q] = i < t1 ? pk[i] : 0;
        u[q + 1] = i + 1 < t1 ? pid[i + 1] : -1;
        k[q + 1] = i + 1 < t1 ? pk[i + 1] : 0;
      }
    }
  };
  int64_t u[kL1Items], k[kL1Items];
  if (t0 < t1) load(t0, u, k);
  for (int64_t c0 = t0; c0 < t1; c0 += kL1Rows) {
    int d[kL1Items];
    K x[kL1Items];
    unsigned r[kL1Items];
#pragma unroll
    for (int q = 0; q < kL1Items; ++q) {
      r[q] = (unsigned)(c0 + 2 * ((int64_t)threadIdx.x + (int64_t)(q / 2) * blockDim.x) + (q & 1));
      if (u[q] < 0 || u[q] >= kp.U) {  // flagged by k_part_hist, not counted
        d[q] = -1;
        x[q] = 0;
        continue;
      }
      d[q] = (int)(u[q] >> mid_bits);
      bool is_dead = false;
      if (k[q] < 0 || k[q] >= kp.P) {
        atomicOr(err, 1u);
        is_dead = true;
      } else if (allowed != nullptr && allowed[k[q]] == 0) {
        is_dead = true;
      }
      if constexpr (FMT == PDP_KEYS_COMPACT) {
        x[q] = (K)compact_key(kp, u[q], k[q], is_dead);
      } else if constexpr (FMT == PDP_KEYS_PACKED) {
        x[q] = (K)packed_key(kp, u[q], k[q], (uint32_t)(r[q] - (unsigned)t0), is_dead);
      } else {  // WIDE: u64 (dead bit 63 | bucket-within-super and local pid | partition)
        const uint64_t midv = ((uint64_t)u[q] & mid_mask) << kp.pk_bits;
        x[q] = (K)(is_dead ? ((1ULL << 63) | midv) : (midv | (uint64_t)k[q]));
      }
    }
    unsigned rank[kL1Items];
    stage_count(s, nd, d, rank);
    stage_write(s, nd, d, rank, x, r, keys1, rows1);
    for (int B = threadIdx.x; B < nd; B += blockDim.x) s.gcur[B] += s.hist[B];
    __syncthreads();
    if (c0 + kL1Rows < t1) load(c0 + kL1Rows, u, k);
  }
}

// Level 2: one workgroup per (group g of kL2GroupTiles tiles, super-bucket
// B) moves the runs of those tiles in B's region -- in tile order, so one
// contiguous range -- into B's 2^super_bits bucket regions, kL2Rows records
// per LDS stage.  Every bucket's write cursor starts at start[b] + gcur[g][b]
// (k_gscan_cursors) and advances in LDS: no atomics, each bucket's rows land
// in tile order, and consecutive stages of a workgroup append to the same
// runs (their partial cache lines meet in the same L2).  PACKED input: the
// u64 packed records are unpacked into COMPACT (key, row) pairs, the row =
// tile * 65,536 + tile row, the tile found among the group's run starts.
template <int FMT, int MAXD>
__global__ void __launch_bounds__(kL2Threads)  k_scatter_l2(KP kp, const unsigned* __restrict__ super_base,
                                                             const unsigned* __restrict__ super_off,
                                                             const unsigned* __restrict__ bucket_start,
                                                             const unsigned* __restrict__ gcur,
                                                             const L1Key<FMT>* __restrict__ keys1,
                                                             const unsigned* __restrict__ rows1,
                                                             L2Key<FMT>* __restrict__ keys2,
                                                             unsigned* __restrict__ rows2) {
  using KI = L1Key<FMT>;
  using KO = L2Key<FMT>;
  constexpr bool PACKED = FMT == PDP_KEYS_PACKED;
  constexpr int R = 16 / sizeof(KI);  // records per 16-byte key load
  extern __shared__ unsigned long long stage_raw[];
  using SL = StageLds<KO, MAXD, true, kL2Items, kL2Threads>;
  SL& s = *reinterpret_cast<SL*>(stage_raw);
  __shared__ unsigned toff[kL2GroupTiles + 1];  // run starts of the group's tiles, relative to B's region
  const int64_t g = blockIdx.x;
  const int B = blockIdx.y;
  const int64_t T0 = g * kL2GroupTiles;
  const int J = (int)(kp.n_tiles - T0 < kL2GroupTiles ? kp.n_tiles - T0 : kL2GroupTiles);
  const int64_t sb = super_base[B];
  if (threadIdx.x <= J) {
    const int64_t t = T0 + threadIdx.x;
    toff[threadIdx.x] = t < kp.n_tiles ? super_off[t * kp.n_supers + B] : (unsigned)(super_base[B + 1] - sb);
  }
  const int nsub = 1 << kp.super_bits;
  const int64_t s_first = (int64_t)B << kp.super_bits;
  for (int t = threadIdx.x; t < nsub; t += blockDim.x) {
    const int64_t b = s_first + t;
    s.gcur[t] = b < kp.n_buckets ? bucket_start[b] + gcur[g * kp.n_buckets + b] : 0u;
  }
  __syncthreads();
  const int64_t lo = sb + toff[0], hi = sb + toff[J];
  if (lo >= hi) return;  // block-uniform
  const int bb = kp.bucket_bits;
  const uint32_t local_mask = (1u << bb) - 1;
  // PACKED: tile of the record at absolute index i; a thread's records come
  // in increasing order, so the cursor only moves forward
  int jcur = 0;
  auto tile_of = [&](int64_t i) -> int64_t {
    const int64_t o = i - sb;
    while (jcur + 1 < J && (int64_t)toff[jcur + 1] <= o) ++jcur;
    return T0 + jcur;
  };
  auto unpack = [&](uint64_t v, int64_t i, KO* key, unsigned* row, int* dest) {
    const uint32_t mid = (uint32_t)((v >> kp.pk_bits) & ((1ULL << (bb + kp.super_bits)) - 1));
    *dest = (int)(mid >> bb);
    const uint32_t lpk = ((mid & local_mask) << kp.pk_bits);
    *key = (KO)((v >> 63) ? (0x80000000u | lpk) : (lpk | (uint32_t)(v & kp.pk_mask)));
    const uint32_t trow = (uint32_t)((v >> kPackedRowShift) & (kTileRows - 1));
    *row = (unsigned)(tile_of(i) * kTileRows + trow);
  };
  const int sub_shift = kp.pk_bits + kp.bucket_bits;
  const uint64_t sub_mask = (uint64_t)nsub - 1;
  for (int64_t base = lo & ~(int64_t)(R - 1); base < hi; base += kL2Rows) {
    const int64_t r0 = base > lo ? base : lo;
    const int64_t r1 = base + kL2Rows < hi ? base + kL2Rows : hi;
    KO x[kL2Items];
    unsigned r[kL2Items];
    int d[kL2Items];
#pragma unroll
    for (int q = 0; q < kL2Items; q += R) {  // R records per 16-byte key load
      const int64_t i = base + R * ((int64_t)threadIdx.x + (int64_t)(q / R) * blockDim.x);
      if (i >= r0 && i + R - 1 < r1) {
        if constexpr (PACKED) {
          const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(keys1 + i);
          unpack(a.x, i, &x[q], &r[q], &d[q]);
          unpack(a.y, i + 1, &x[q + 1], &r[q + 1], &d[q + 1]);
        } else if constexpr (R == 4) {
          const uint4 a = *reinterpret_cast<const uint4*>(keys1 + i);
          const uint4 c = *reinterpret_cast<const uint4*>(rows1 + i);
          x[q] = a.x; x[q + 1] = a.y; x[q + 2] = a.z; x[q + 3] = a.w;
          r[q] = c.x; r[q + 1] = c.y; r[q + 2] = c.z; r[q + 3] = c.w;
        } else {
          const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(keys1 + i);
          const uint2 c = *reinterpret_cast<const uint2*>(rows1 + i);
          x[q] = a.x; x[q + 1] = a.y;
          r[q] = c.x; r[q + 1] = c.y;
        }
        if constexpr (!PACKED) {
#pragma unroll
          for (int e = 0; e < R; ++e) d[q + e] = (int)((x[q + e] >> sub_shift) & sub_mask);
        }
      } else {
#pragma unroll
        for (int e = 0; e < R; ++e) {
          const bool ok = i + e >= r0 && i + e < r1;
          if constexpr (PACKED) {
            if (ok) unpack(keys1[i + e], i + e, &x[q + e], &r[q + e], &d[q + e]);
            else { x[q + e] = 0; r[q + e] = 0; d[q + e] = -1; }
          } else {
            x[q + e] = ok ? keys1[i + e] : 0;
            r[q + e] = ok ? rows1[i + e] : 0;
            d[q + e] = ok ? (int)((x[q + e] >> sub_shift) & sub_mask) : -1;
          }
        }
      }
    }
    unsigned rank[kL2Items];
    stage_count(s, nsub, d, rank);
    stage_write(s, nsub, d, rank, x, r, keys2, rows2);
    for (int t = threadIdx.x; t < nsub; t += blockDim.x) s.gcur[t] += s.hist[t];
    __syncthreads();
  }
}

// exclusive block-wide scan of one u32 per thread; wsum = LDS[blockDim/64]
__device__ __forceinline__ unsigned block_excl_scan(unsigned x, unsigned* wsum, unsigned* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  unsigned inc = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned y = __shfl_up(inc, off, 64);
    if (lane >= off) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  if (w == 0) {
    const unsigned v = lane < nw ? wsum[lane] : 0;
    unsigned vi = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned y = __shfl_up(vi, off, 64);
      if (lane >= off) vi += y;
    }
    if (lane < nw) wsum[lane] = vi - v;
    if (lane == nw - 1) wsum[nw] = vi;
  }
  __syncthreads();
  *total = wsum[nw];
  return wsum[w] + inc - x;
}

// super_off[t][B] = rows of super-bucket B in tiles < t (exclusive scan over
// tiles, one workgroup per super-bucket): the level-1 scatter's per-tile
// write offsets, read as one contiguous row per tile
__global__ void __launch_bounds__(kBlock) k_super_scan(KP kp, const unsigned* __restrict__ super_tm,
                                                       unsigned* __restrict__ super_off) {
  __shared__ unsigned wsum[kBlock / 64 + 1];
  const int64_t B = blockIdx.x;
  unsigned carry = 0;
  for (int64_t t0 = 0; t0 < kp.n_tiles; t0 += blockDim.x) {
    const int64_t t = t0 + threadIdx.x;
    const unsigned x = t < kp.n_tiles ? super_tm[t * kp.n_supers + B] : 0u;
    unsigned total;
    const unsigned ex = block_excl_scan(x, wsum, &total);
    if (t < kp.n_tiles) super_off[t * kp.n_supers + B] = carry + ex;
    carry += total;
    __syncthreads();  // wsum is reused by the next chunk
  }
}

// ------------------------------------------------ tile-local level 1 / 2 --
// Plan.l1_local: level 1 needs no histogram pass before it.  Each 4,096-row
// stage is counting-sorted by super-bucket in LDS and written whole to its
// own block keys1[stage * kL1Rows, + rows kept) -- one contiguous span per
// stage -- with soff[stage][B] (u16, n_supers + 1 entries) = where
// super-bucket B's run starts in that block.  The tile's rows per bucket
// (counts_tm, the level-2 cursor input) are counted in LDS on the way, so the
// privacy-id column is read once (k_part_hist + k_super_scan are not run).
static_assert(kTileRows % kL1Rows == 0, "a tile is a whole number of level-1 stages");
static_assert(kL2Runs * kSieveL2Groups <= kL2Threads, "one level-1 slot per thread in the run scan");
static_assert(kSieveTileStride == kTileRows && kBandTileStride >= kTileRows, "level 2 recovers a run's tile from its position");

// the LDS stage block [0, total) -> dst, 16 bytes per lane
template <typename K>
__device__ __forceinline__ void copy_block(K* __restrict__ dst, const K* src, unsigned total) {
  constexpr unsigned V = 16 / sizeof(K);
  using VT = typename std::conditional<V == 4, uint4, ulonglong2>::type;
  const unsigned nv = total / V;
  for (unsigned k = threadIdx.x; k < nv; k += blockDim.x)
    reinterpret_cast<VT*>(dst)[k] = reinterpret_cast<const VT*>(src)[k];
  for (unsigned k = nv * V + threadIdx.x; k < total; k += blockDim.x) dst[k] = src[k];
}

// The tile-local level 1's bucket counts leave LDS as u16 pairs per u32
// word (rows of kp.cstride / 2 words; bucket 2w in the low half): half the
// bytes of u32 counts for level 1 to write and k_gscan_sums to read.  The
// LDS counts are u32 per bucket, or (U16) already u16 pairs of a half tile
// (<= 2^15 each; two halves can add up to 2^16, which k_gscan_sums adds lane
// by lane with the carry kept apart).  A u32 count of 65,536 -- every row of the tile in one
// bucket -- is stored as 0 with the bucket in tile_over[t], which the scan
// adds back (tile_over is all ones otherwise; the caller sets it so).
template <bool U16>
__device__ __forceinline__ void flush_counts16(unsigned* __restrict__ bh, int64_t n_buckets,
                                               unsigned* __restrict__ dst, unsigned* __restrict__ over, int th) {
  const int64_t n_pairs = (n_buckets + 1) / 2;
  for (int64_t w = threadIdx.x; w < n_pairs; w += th) {
    if constexpr (U16) {
      dst[w] = bh[w];
      bh[w] = 0;
    } else {
      const unsigned v0 = bh[2 * w], v1 = 2 * w + 1 < n_buckets ? bh[2 * w + 1] : 0u;
      bh[2 * w] = 0;
      if (2 * w + 1 < n_buckets) bh[2 * w + 1] = 0;
      dst[w] = (v0 & 0xFFFFu) | (v1 << 16);
      if (v0 > 0xFFFFu) *over = (unsigned)(2 * w);
      if (v1 > 0xFFFFu) *over = (unsigned)(2 * w + 1);
    }
  }
}

template <int FMT, bool U16>
__global__ void __launch_bounds__(kL1Threads)  k_scatter_l1_local(KP kp, const int64_t* __restrict__ pid,
                                                                   const int64_t* __restrict__ pk,
                                                                   const uint8_t* __restrict__ allowed,
                                                                   unsigned* __restrict__ counts_tm,
                                                                   unsigned* __restrict__ counts_tm2,
                                                                   uint16_t* __restrict__ soff,
                                                                   L1Key<FMT>* __restrict__ keys1,
                                                                   unsigned* __restrict__ rows1, unsigned* err,
                                                                   unsigned* __restrict__ tile_over) {
  using K = L1Key<FMT>;
  constexpr bool ROWS = !kPackedL1<FMT>;
  extern __shared__ unsigned long long stage_raw[];
  using SL = StageLds<K, kSmallDest, ROWS, kL1Items, kL1Threads>;
  SL& s = *reinterpret_cast<SL*>(stage_raw);
  // rows per bucket: u32 each, or (U16) two u16 per word, flushed every half
  // tile so that no count carries into its neighbour
  unsigned* bh = reinterpret_cast<unsigned*>(stage_raw + (sizeof(SL) + 7) / 8);
  const int64_t n_words = U16 ? (kp.n_buckets + 1) / 2 : kp.n_buckets;
  for (int64_t b = threadIdx.x; b < n_words; b += blockDim.x) bh[b] = 0;
  __syncthreads();
  const int64_t t = blockIdx.x;
  auto flush = [&](unsigned* __restrict__ dst) {  // after a barrier; leaves bh zeroed
    flush_counts16<U16>(bh, kp.n_buckets, dst, tile_over + t, blockDim.x);
  };
  const int nd = (int)kp.n_supers;
  const int64_t t0 = t * kTileRows;
  const int64_t t1 = t0 + kTileRows < kp.n ? t0 + kTileRows : kp.n;
  const int mid_bits = kp.bucket_bits + kp.super_bits;
  const uint64_t mid_mask = (1ULL << mid_bits) - 1;
  auto load = [&](int64_t c0, int64_t (&u)[kL1Items], int64_t (&k)[kL1Items]) {
#pragma unroll
    for (int q = 0; q < kL1Items; q += 2) {
      const int64_t i = c0 + 2 * ((int64_t)threadIdx.x + (int64_t)(q / 2) * blockDim.x);
      if (kp.keys_vec && i + 1 < t1) {
        const longlong2 a = *reinterpret_cast<const longlong2*>(pid + i);
        const longlong2 c = *reinterpret_cast<const longlong2*>(pk + i);
        u[q] = a.x;
        u[q + 1] = a.y;
        k[q] = c.x;
        k[q + 1] = c.y;
      } else {
        u[q] = i < t1 ? pid[i] : 0;
        k[q] = i < t1 ? pk[i] : 0;
        u[q + 1] = i + 1 < t1 ? pid[i + 1] : 0;
        k[q + 1] = i + 1 < t1 ? pk[i + 1] : 0;
      }
    }
  };
  int64_t u[kL1Items], k[kL1Items];
  // U16: the tile's counts in two halves (counts_tm, counts_tm2)
  const bool split = U16 && t1 - t0 > (kStagesPerTile / 2 - 1) * kL1Rows;
  if (t0 < t1) load(t0, u, k);
  for (int64_t c0 = t0; c0 < t1; c0 += kL1Rows) {
    const int64_t st = c0 / kL1Rows;  // global stage index
    int d[kL1Items];
    K x[kL1Items];
    unsigned r[kL1Items];
#pragma unroll
    for (int q = 0; q < kL1Items; ++q) {
      const int64_t i = c0 + 2 * ((int64_t)threadIdx.x + (int64_t)(q / 2) * blockDim.x) + (q & 1);
      r[q] = (unsigned)i;
      d[q] = -1;
      x[q] = 0;
      if (i >= t1) continue;
      if (u[q] < 0 || u[q] >= kp.U) {  // invalid privacy id: flagged, not counted
        atomicOr(err, 1u);
        continue;
      }
      const int64_t bkt = u[q] >> kp.bucket_bits;
      if constexpr (U16) atomicAdd(bh + (bkt >> 1), 1u << (16 * (bkt & 1)));
      else atomicAdd(bh + bkt, 1u);
      d[q] = (int)(u[q] >> mid_bits);
      bool is_dead = false;
      if (k[q] < 0 || k[q] >= kp.P) {
        atomicOr(err, 1u);
        is_dead = true;
      } else if (allowed != nullptr && allowed[k[q]] == 0) {
        is_dead = true;
      }
      if constexpr (FMT == PDP_KEYS_COMPACT) {
        x[q] = (K)compact_key(kp, u[q], k[q], is_dead);
      } else if constexpr (kPackedL1<FMT>) {
        x[q] = (K)packed_key(kp, u[q], k[q], (uint32_t)(i - t0), is_dead);
      } else {
        const uint64_t midv = ((uint64_t)u[q] & mid_mask) << kp.pk_bits;
        x[q] = (K)(is_dead ? ((1ULL << 63) | midv) : (midv | (uint64_t)k[q]));
      }
    }
    unsigned rank[kL1Items];
    stage_count(s, nd, d, rank);
#pragma unroll
    for (int q = 0; q < kL1Items; ++q) {
      if (d[q] < 0) continue;
      const unsigned slot = s.start[d[q]] + rank[q];
      s.keys[slot] = x[q];
      if (ROWS) s.rows[slot] = r[q];
    }
    __syncthreads();
    const unsigned total = s.start[nd - 1] + s.hist[nd - 1];
    copy_block(keys1 + st * kL1Rows, s.keys, total);
    if (ROWS) copy_block(rows1 + st * kL1Rows, s.rows, total);
    for (int B = threadIdx.x; B <= nd; B += blockDim.x)
      soff[st * (nd + 1) + B] = (uint16_t)(B < nd ? s.start[B] : total);
    __syncthreads();
    if (c0 + kL1Rows < t1) load(c0 + kL1Rows, u, k);
    if (split && c0 - t0 == (kStagesPerTile / 2 - 1) * kL1Rows) {  // first half tile done
      flush(counts_tm + t * (kp.cstride / 2));
      __syncthreads();
    }
  }
  __syncthreads();
  // tile-major rows: coalesced.  Counts of a half tile never exceed 2^15
  if (split) {
    flush(counts_tm2 + t * (kp.cstride / 2));
  } else {
    flush(counts_tm + t * (kp.cstride / 2));
    if constexpr (U16)
      for (int64_t w = threadIdx.x; w < kp.cstride / 2; w += blockDim.x) counts_tm2[t * (kp.cstride / 2) + w] = 0;
  }
}

// Threshold-sieve level 1 (Plan.sieve): one 1,024-thread workgroup per
// 65,536-row tile filters the tile in chunks of kSieveChunk rows.  A row is a
// candidate when it is live (valid keys, public partition) and its pair hash
// is below kp.sieve_t32; candidates' level-1 records are appended to an LDS
// stage (wave-compacted: one LDS atomic per wave and chunk).  When the stage
// cannot take another chunk, or the tile ends, it is counting-sorted by
// super-bucket and written as one block right after the tile's previous
// blocks (keys1 + tile * kSieveTileStride + sbase[slot]) with its run
// offsets in soff[slot], as k_scatter_l1_local writes a stage;
// the tile's unused slots get empty runs.  Rows with invalid keys set the
// error word; dead rows (non-public partitions) are simply dropped.  The
// tile's candidate counts per bucket feed the level-2 cursors as before.
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifdef PDP_PHASE_CLOCK
__device__ unsigned g_phase_l1, g_phase_l2, g_phase_bk;  // profiling builds: prints so far per kernel
#endif
// BAND: rows with sieve_t32 <= pair hash < band_t32 also go, as (privacy id
// << 32 | row), to this tile's band list band[t * 65,536 ...], through a
// per-wave LDS queue flushed 64 entries (512 contiguous bytes) at a time;
// band_cnt[t] = the list's length
template <int FMT, bool U16, bool BAND, int TH>
__global__ void __launch_bounds__(TH, TH == kL1Threads ? 1 : 4) k_sieve_l1(KP kp, const int64_t* __restrict__ pid,
                                                         const int64_t* __restrict__ pk,
                                                         const uint8_t* __restrict__ allowed,
                                                         unsigned* __restrict__ counts_tm,
                                                         unsigned* __restrict__ counts_tm2,
                                                         uint16_t* __restrict__ soff, unsigned* __restrict__ sbase,
                                                         L1Key<FMT>* __restrict__ keys1,
                                                         unsigned* __restrict__ rows1, unsigned* err,
                                                         unsigned long long* __restrict__ band,
                                                         unsigned* __restrict__ band_cnt,
                                                         unsigned* __restrict__ tile_over) {
  using K = L1Key<FMT>;
  using SS = SieveShape<TH>;
  constexpr bool ROWS = !kPackedL1<FMT>;
  constexpr int Q = kSieveChunkItems;
  constexpr int kSieveChunk = SS::kChunk;
  constexpr int kSieveCap = SS::kCap;
  extern __shared__ unsigned long long stage_raw[];
  using SL = StageLds<K, kSmallDest, ROWS, kSieveItems, TH>;
  SL& s = *reinterpret_cast<SL*>(stage_raw);
  unsigned* bh = reinterpret_cast<unsigned*>(stage_raw + (sizeof(SL) + 7) / 8);
  // BAND: the per-wave queues after the bucket counts (l1_hist_bytes)
  unsigned long long* const bq =
      stage_raw + (sizeof(SL) + 7) / 8 + (((U16 ? 2 : 4) * kp.n_buckets + 15) / 16 * 16) / 8;
  __shared__ unsigned fill, bfill;
  const int64_t n_words = U16 ? (kp.n_buckets + 1) / 2 : kp.n_buckets;
  for (int64_t b = threadIdx.x; b < n_words; b += TH) bh[b] = 0;
  for (int B = threadIdx.x; B < (int)kp.n_supers; B += TH) s.hist[B] = 0;
  if (threadIdx.x == 0) {
    fill = 0;
    bfill = 0;
  }
  __syncthreads();
  // persistent: workgroup g takes tiles g, g + G, ... (G = gridDim.x, about
  // one per CU), so a tile's last chunks prefetch the next tile's first ones
  // and no tile starts with its loads' latency exposed
  const int nd = (int)kp.n_supers;
  int64_t t = 0, t0 = 0, t1 = 0, next_t0 = -1;  // the tile; the next one's first row (-1: none)
  auto flush_counts = [&](unsigned* __restrict__ dst) {  // after a barrier; leaves bh zeroed
    flush_counts16<U16>(bh, kp.n_buckets, dst, tile_over + t, TH);
  };
  const int mid_bits = kp.bucket_bits + kp.super_bits;
  const uint32_t t32 = kp.sieve_t32;
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ULL << lane) - 1;
  K* blk = nullptr;
  unsigned* rblk = nullptr;
  unsigned long long* band_tile = nullptr;
  unsigned long long* const wq = bq + (threadIdx.x >> 6) * kBandQueue;
  int qn = 0;            // wave-uniform: entries waiting in this wave's band queue
  unsigned written = 0;  // block-uniform: this tile's records already written
  int slot = 0;
  bool split = false;    // U16: the tile's counts in two halves (counts_tm, counts_tm2)
  auto begin_tile = [&](int64_t tt) {
    t = tt;
    t0 = tt * kTileRows;
    t1 = t0 + kTileRows < kp.n ? t0 + kTileRows : kp.n;
    blk = keys1 + tt * kSieveTileStride;
    rblk = ROWS ? rows1 + tt * kSieveTileStride : nullptr;
    band_tile = BAND ? band + tt * kBandTileStride : nullptr;
    written = 0;
    slot = 0;
    split = U16 && t1 - t0 > kTileRows / 2 - kSieveChunk;
  };
  // the stage's `total` records -> counting sort by super-bucket -> block
#ifdef PDP_PHASE_CLOCK
  unsigned long long fl_ticks = 0, t_start = wall_clock64();
#endif
  auto flush = [&](unsigned total) {
#ifdef PDP_PHASE_CLOCK
    const unsigned long long f0 = wall_clock64();
#endif
    // the stage's runs per super-bucket were counted as its records were
    // appended (s.hist; the tile's bucket counts too), so the flush is a
    // one-wave scan and one pass that places each record through an LDS
    // cursor per run: little work while the CU's loads are stalled
    if (threadIdx.x < 64) {
      unsigned carry = 0;
      for (int base = 0; base < nd; base += 64) {
        const unsigned v = base + lane < nd ? s.hist[base + lane] : 0;
        unsigned incl = v;
        for (int off = 1; off < 64; off <<= 1) {
          const unsigned up = __shfl_up(incl, off, 64);
          if (lane >= off) incl += up;
        }
        if (base + lane < nd) {
          s.start[base + lane] = written + carry + incl - v;
          s.gcur[base + lane] = carry + incl - v;  // stage-relative cursor
        }
        carry += __shfl(incl, 63, 64);
      }
    }
    __syncthreads();
    for (int B = threadIdx.x; B < nd; B += TH) s.hist[B] = 0;  // the next stage's counts (not read below)
    // every record straight to its run: the block (<= kSieveCap records) is
    // written whole by this workgroup, so its partial lines merge in L2
#pragma unroll
    for (int j = 0; j < kSieveItems; ++j) {
      const unsigned e = threadIdx.x + (unsigned)j * TH;
      if (e >= total) continue;
      const unsigned pos = written + atomicAdd(s.gcur + s.dest[e], 1u);
      blk[pos] = s.keys[e];
      if (ROWS) rblk[pos] = s.rows[e];
    }
    const int64_t sl = t * SS::kSlots + slot;
    for (int B = threadIdx.x; B <= nd; B += TH)
      soff[sl * (nd + 1) + B] = (uint16_t)(B < nd ? s.start[B] - written : total);
    if (threadIdx.x == 0) {
      sbase[sl] = written;
      fill = 0;
    }
    written += total;
    ++slot;
    __syncthreads();
#ifdef PDP_PHASE_CLOCK
    fl_ticks += wall_clock64() - f0;
#endif
  };
  bool bad = false;  // a key outside [0, U) x [0, P): flagged once per thread at the end
  // end of a tile: the band queues' rest and the list length, the unused
  // flush slots, the bucket counts; leaves the LDS state zeroed for the next
  auto end_tile = [&]() {
    if constexpr (BAND) {
      wave_lds_fence();
      if (qn > 0) {
        unsigned bb = 0;
        if (lane == 0) bb = atomicAdd(&bfill, (unsigned)qn);
        bb = __shfl(bb, 0, 64);
        if (lane < qn) band_tile[bb + lane] = wq[lane];
        qn = 0;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        band_cnt[t] = bfill;
        bfill = 0;
      }
    }
#ifdef PDP_PHASE_CLOCK
    if (threadIdx.x == 0 && blockIdx.x % 97 == 5 && atomicAdd(&g_phase_l1, 1u) < 40u)
      printf("l1 tile %d slots %d records %u total %llu flush %llu (10 ns)\n", (int)t, slot, written,
             wall_clock64() - t_start, fl_ticks);
    t_start = wall_clock64();
    fl_ticks = 0;
#endif
    for (int j = slot; j < SS::kSlots; ++j) {
      const int64_t sl = t * SS::kSlots + j;
      for (int B = threadIdx.x; B <= nd; B += TH) soff[sl * (nd + 1) + B] = 0;
      if (threadIdx.x == 0) sbase[sl] = written;
    }
    __syncthreads();
    if (split) {
      flush_counts(counts_tm2 + t * (kp.cstride / 2));
    } else {
      flush_counts(counts_tm + t * (kp.cstride / 2));
      if constexpr (U16)
        for (int64_t w = threadIdx.x; w < kp.cstride / 2; w += TH) counts_tm2[t * (kp.cstride / 2) + w] = 0;
    }
    __syncthreads();
  };
  // FULL (a whole tile of 16-byte aligned columns): every load is an
  // unconditional 16-byte load and the prefetch address is clamped into the
  // tile, so no branch surrounds a load and the compiler keeps two chunks of
  // loads in flight (a guarded load per row made it wait for every load);
  // otherwise guarded 8-byte loads (the last tile, unaligned columns)
  auto run = [&](auto full_tag) {
    constexpr bool FULL = decltype(full_tag)::value;
    auto load = [&](int64_t c0, int64_t (&u)[Q], int64_t (&k)[Q]) {
#pragma unroll
      for (int q = 0; q < Q; q += 2) {
        const int64_t i = c0 + 2 * ((int64_t)threadIdx.x + (int64_t)(q / 2) * TH);
        if constexpr (FULL) {
          const longlong2 a = ld_maybe_nt<PDP_L1_NT>(reinterpret_cast<const longlong2*>(pid + i));
          const longlong2 c = ld_maybe_nt<PDP_L1_NT>(reinterpret_cast<const longlong2*>(pk + i));
          u[q] = a.x;
          u[q + 1] = a.y;
          k[q] = c.x;
          k[q + 1] = c.y;
        } else {
          u[q] = i < t1 ? pid[i] : 0;
          k[q] = i < t1 ? pk[i] : 0;
          u[q + 1] = i + 1 < t1 ? pid[i + 1] : 0;
          k[q + 1] = i + 1 < t1 ? pk[i + 1] : 0;
        }
      }
    };
    // one chunk: its keys narrowed to 32 bits and range-checked (sieve plans
    // have U < 2^32 - 1 and P < 2^32), which frees the load registers, so the
    // loads of the chunk two ahead go out before the hashing; then filter,
    // append / flush -- two chunks of loads in flight almost all the time
    auto body = [&](int64_t c0, int64_t (&u)[Q], int64_t (&k)[Q]) {
      const bool more = c0 + kSieveChunk < t1;  // block-uniform
      bool cand[Q], bnd[Q], ok[Q];
      uint32_t ul[Q], kl[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int64_t i = c0 + 2 * ((int64_t)threadIdx.x + (int64_t)(q / 2) * TH) + (q & 1);
        const bool valid = FULL || i < t1;
        const bool in_range = (uint64_t)u[q] < (uint64_t)kp.U && (uint64_t)k[q] < (uint64_t)kp.P;
        bad |= valid & !in_range;
        ok[q] = valid & in_range;
        ul[q] = (uint32_t)u[q];
        kl[q] = (uint32_t)k[q];
      }
      if (allowed != nullptr) {  // block-uniform; the mask bytes gathered and used before the prefetch
        uint8_t pub[Q];          // (one in-order vmcnt: a later use would wait for the prefetch too)
#pragma unroll
        for (int q = 0; q < Q; ++q) pub[q] = allowed[ok[q] ? kl[q] : 0u];
#pragma unroll
        for (int q = 0; q < Q; ++q) ok[q] = ok[q] & (pub[q] != 0);  // a non-public partition's rows are dropped
      }
      // two buffers: the next loads go out now; three or more: after the
      // append / flush below, so that a flush runs with the other buffers'
      // loads in flight and this one's registers free (the register peak)
      constexpr bool kEarly = !FULL || kSieveBufs < 3 || PDP_SIEVE_EARLY;
      auto prefetch = [&]() {
        if constexpr (FULL) {  // past the tile: the next tile's chunk, else clamped (no branch)
          const int64_t ahead = c0 + kSieveBufs * kSieveChunk;
          const int64_t cp = ahead < t1 ? ahead : (next_t0 >= 0 ? next_t0 + (ahead - t1) : t1 - kSieveChunk);
          load(cp, u, k);
        } else {
          if (c0 + 2 * kSieveChunk < t1) load(c0 + 2 * kSieveChunk, u, k);
        }
      };
      if constexpr (kEarly) prefetch();
      int d[Q];
      K x[Q];
      const uint32_t mid_mask = (uint32_t)(((uint64_t)1 << mid_bits) - 1);
      const uint32_t row0 = (uint32_t)(c0 - t0) + 2u * threadIdx.x;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        // every term evaluated (no short circuit: no branch); the pair hash
        // of an id below 2^32 (pid_hash's high word is zero)
        const uint32_t h = pair_hash_from((ul[q] ^ (uint32_t)kp.seed) * 0x9E3779B1U, kp.seed, (int64_t)kl[q]);
        bnd[q] = BAND && (ok[q] & (h >= t32) & (h < kp.band_t32));
        cand[q] = ok[q] & (h < t32);
        d[q] = mid_bits < 32 ? (int)(ul[q] >> mid_bits) : 0;
        const uint32_t mid = ul[q] & mid_mask;
        if constexpr (FMT == PDP_KEYS_COMPACT) {
          x[q] = (K)((mid << kp.pk_bits) | kl[q]);
        } else {  // PACKED / PACKED_WIDE: (row within the tile | mid | partition)
          const uint32_t tile_row = row0 + (uint32_t)((q / 2) * 2 * TH) + (uint32_t)(q & 1);
          x[q] = (K)(((uint64_t)tile_row << kPackedRowShift) | ((uint64_t)mid << kp.pk_bits) | (uint64_t)kl[q]);
        }
        // a band row is no candidate: its key slot carries its privacy id
        if constexpr (BAND) x[q] = bnd[q] ? (K)ul[q] : x[q];
      }
      // append this wave's candidates at one reserved range of the stage
      unsigned long long m[Q];
      unsigned nw = 0;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        m[q] = __ballot(cand[q]);
        nw += (unsigned)__popcll(m[q]);
      }
      unsigned base = 0;
      if (lane == 0 && nw) base = atomicAdd(&fill, nw);
      base = __shfl(base, 0, 64);
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (cand[q]) {
          const unsigned pos = base + (unsigned)__popcll(m[q] & below);
          s.keys[pos] = x[q];
          s.dest[pos] = (typename SL::D)d[q];
          if (ROWS) s.rows[pos] = (unsigned)(c0 + 2 * ((int64_t)threadIdx.x + (int64_t)(q / 2) * TH) + (q & 1));
          // the stage's run lengths and the tile's bucket counts (bucket = id >> bucket_bits)
          atomicAdd(s.hist + d[q], 1u);
          const unsigned bkt = ul[q] >> kp.bucket_bits;
          if constexpr (U16) atomicAdd(bh + (bkt >> 1), 1u << (16 * (bkt & 1)));
          else atomicAdd(bh + bkt, 1u);
        }
        base += (unsigned)__popcll(m[q]);
      }
      if constexpr (BAND) {  // band rows -> the wave's queue; 64 of them out at once
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const unsigned long long mb = __ballot(bnd[q]);
          if (mb == 0) continue;  // wave-uniform
          const int64_t i = c0 + 2 * ((int64_t)threadIdx.x + (int64_t)(q / 2) * TH) + (q & 1);
          if (bnd[q]) wq[qn + __popcll(mb & below)] = ((unsigned long long)(uint32_t)x[q] << 32) | (uint32_t)i;
          qn += __popcll(mb);
          if (qn >= 64) {
            wave_lds_fence();
            const unsigned long long e = wq[lane];
            unsigned bb = 0;
            if (lane == 0) bb = atomicAdd(&bfill, 64u);
            bb = __shfl(bb, 0, 64);
            band_tile[bb + lane] = e;
            const unsigned long long rest = lane + 64 < qn ? wq[lane + 64] : 0ULL;
            wave_lds_fence();
            if (lane + 64 < qn) wq[lane] = rest;
            qn -= 64;
            wave_lds_fence();
          }
        }
      }
      __syncthreads();
      const unsigned f = fill;
      if (f > 0 && (f > (unsigned)(kSieveCap - kSieveChunk) || !more)) flush(f);  // block-uniform
      else __syncthreads();  // every thread has read `fill` before the next chunk's appends
      if constexpr (!kEarly) prefetch();
      if (split && c0 - t0 == kTileRows / 2 - kSieveChunk) {  // first half tile counted
        flush_counts(counts_tm + t * (kp.cstride / 2));
        __syncthreads();
      }
    };
    if constexpr (FULL) {  // a fixed trip count: the same loads are pending on every path
      constexpr int kChunks = (int)(kTileRows / kSieveChunk);
      // the ring of kSieveBufs register buffers turns a whole number of times
      // per tile, so the chunks prefetched across the tile boundary land in
      // the buffers the next tile reads them from
      static_assert(kChunks % kSieveBufs == 0, "whole ring turns per tile");
      int64_t ub[kSieveBufs][Q], kb[kSieveBufs][Q];
      const int64_t n_full = kp.n / kTileRows;  // tiles of kTileRows rows (16-byte aligned columns)
      // (workgroup g takes tiles g, g + G, ...: contiguous tile ranges per
      // workgroup measured 5 % slower, profiles/r05/ab/ab1_l1_placement.txt)
      const int64_t tile_lo = blockIdx.x, tile_hi = n_full, tile_step = gridDim.x;
      if (tile_lo >= tile_hi) return;  // block-uniform
#pragma unroll
      for (int b = 0; b < kSieveBufs; ++b) load(tile_lo * kTileRows + (int64_t)b * kSieveChunk, ub[b], kb[b]);
      for (int64_t tt = tile_lo; tt < tile_hi; tt += tile_step) {
        begin_tile(tt);
        next_t0 = tt + tile_step < tile_hi ? (tt + tile_step) * kTileRows : -1;
        for (int j = 0; j < kChunks; j += kSieveBufs) {
#pragma unroll
          for (int b = 0; b < kSieveBufs; ++b) body(t0 + (int64_t)(j + b) * kSieveChunk, ub[b], kb[b]);
        }
        end_tile();
      }
    } else {  // the last tile, unaligned columns: two chunks in flight
      int64_t ua[Q], ka[Q], ub[Q], kb[Q];
      if (t0 < t1) load(t0, ua, ka);
      if (t0 + kSieveChunk < t1) load(t0 + kSieveChunk, ub, kb);
      for (int64_t c0 = t0; c0 < t1; c0 += 2 * kSieveChunk) {
        body(c0, ua, ka);
        if (c0 + kSieveChunk < t1) body(c0 + kSieveChunk, ub, kb);  // block-uniform
      }
    }
  };
  if (kp.keys_vec) run(std::true_type{});
  // the rest: a partial last tile, or every tile when the columns are unaligned
  for (int64_t tt = (kp.keys_vec ? kp.n / kTileRows : 0) + blockIdx.x; tt < kp.n_tiles; tt += gridDim.x) {
    begin_tile(tt);
    next_t0 = -1;
    run(std::false_type{});
    end_tile();
  }
  if (bad) atomicOr(err, 1u);
}

// Level 2 over tile-local level-1 blocks: workgroup (group g of kL2GroupTiles
// tiles, super-bucket B) takes B's run from each of the group's stages
// (kL2Runs runs: keys1[st * kL1Rows + soff[st][B], + soff[st][B + 1])),
// concatenated in stage order, kL2Rows records per LDS window.  Per window an
// LDS map (the run of every record, in the stage's destination-tag array
// before the counting sort reuses it) lets each thread address its own
// records, so all of a thread's loads go out together.  Cursors as in
// k_scatter_l2; PACKED rows are (stage >> slot_bits) * 65,536 + tile row.
// level-2 key of a packed level-1 record w (bit 63 dead): COMPACT u32
// (bit 31 dead | local pid | partition) or, PACKED_WIDE, the same fields in a u64
template <typename KO>
__device__ __forceinline__ KO unpacked_key(const KP& kp, uint32_t local, uint64_t w) {
  if constexpr (sizeof(KO) == 4) {
    const uint32_t lpk = local << kp.pk_bits;
    return (KO)((w >> 63) ? (0x80000000u | lpk) : (lpk | (uint32_t)(w & kp.pk_mask)));
  } else {
    const uint64_t lpk = (uint64_t)local << kp.pk_bits;
    return (KO)((w >> 63) ? ((1ULL << 63) | lpk) : (lpk | (w & kp.pk_mask)));
  }
}

// tile-local level 2 records per thread: half for 8-byte level-2 keys with a
// row array (WIDE / PACKED_WIDE), so their LDS windows and registers leave
// room for two workgroups per CU; PACKED64 carries no row array
template <int FMT>
constexpr int l2_items() { return sizeof(L2Key<FMT>) == 8 && FMT != PDP_KEYS_PACKED64 ? kL2Items / 2 : kL2Items; }
template <int FMT>
constexpr bool kL2RowArray = FMT != PDP_KEYS_PACKED64;  // level 2 writes a row array

template <int FMT, int MAXD>
__global__ void __launch_bounds__(kL2Threads, 4) k_scatter_l2_local(KP kp, const uint16_t* __restrict__ soff,
                                                                   const unsigned* __restrict__ sbase,
                                                                   const unsigned* __restrict__ bucket_start,
                                                                   const unsigned* __restrict__ gcur,
                                                                   const L1Key<FMT>* __restrict__ keys1,
                                                                   const unsigned* __restrict__ rows1,
                                                                   L2Key<FMT>* __restrict__ keys2,
                                                                   unsigned* __restrict__ rows2) {
  using KI = L1Key<FMT>;
  using KO = L2Key<FMT>;
  constexpr int NI = l2_items<FMT>();  // records per thread and window
  constexpr int NR = kL2Threads * NI;
  constexpr bool PACKED = kPackedL1<FMT>;  // PACKED / PACKED_WIDE level-1 records
  constexpr bool ROWS1 = !PACKED;
  extern __shared__ unsigned long long stage_raw[];
  using SL = StageLds<KO, MAXD, kL2RowArray<FMT>, NI, kL2Threads>;
  using D = typename SL::D;
  SL& s = *reinterpret_cast<SL*>(stage_raw);
#ifdef PDP_PHASE_CLOCK
  unsigned long long c0 = wall_clock64(), c_tab = 0, c_ld = 0, c_sort = 0, c_wr = 0, cw = 0;
  int n_win = 0;
#endif
  // the workgroup's non-empty runs, in slot order
  // (a run's tile is rsrc / kTileRows: every level-1 block of tile t starts at
  // or after t * kTileRows, inside its tile's region -- and keeping the LDS of
  // a PACKED workgroup at <= 80 KiB lets two of them share a CU)
  __shared__ unsigned rbeg[kL2Threads + 1];  // start of each run in the concatenation
  __shared__ unsigned rsrc[kL2Threads];      // its first record in keys1
  __shared__ unsigned wsum[kL2Threads / 64 + 1], wsum2[kL2Threads / 64 + 1];
  // XCD-aware order: a group's workgroups (all super-buckets) run one after
  // another on one XCD (blocks are placed round-robin, linear id % 8), so the
  // cache lines that two neighbouring runs of a stage block share are read
  // from that XCD's L2
  // a workgroup takes kp.l2_group_mult tile groups (up to 4 with the sieve, whose
  // blocks hold a fraction of the rows; <= kL2Threads slots, one per thread)
  const int nd = (int)kp.n_supers;
  const int M = kp.l2_group_mult;
  const int64_t n_grp = (kp.n_tiles + (int64_t)kL2GroupTiles * M - 1) / ((int64_t)kL2GroupTiles * M);
  const int64_t lin = blockIdx.x, kx = lin >> 3;
  const int64_t g = (kx / nd) * 8 + (lin & 7);
  const int B = (int)(kx % nd);
  if (g >= n_grp) return;  // block-uniform
  const int64_t runs = ((int64_t)kL2GroupTiles << kp.slot_bits) * M;  // level-1 slots of the workgroup
  const int64_t S0 = g * runs;
  const int64_t n_all = kp.n_slots1 - S0 < runs ? kp.n_slots1 - S0 : runs;
  // this workgroup's bucket write cursors: loaded first, so that their
  // latency overlaps the run table's loads below (thread t < 2^super_bits)
  const int nsub = 1 << kp.super_bits;
  const int64_t s_first = (int64_t)B << kp.super_bits;
  unsigned cur0 = 0;
  if ((int)threadIdx.x < nsub && s_first + threadIdx.x < kp.n_buckets)
    cur0 = bucket_start[s_first + threadIdx.x] + gcur[g * M * kp.n_buckets + s_first + threadIdx.x];
  unsigned len = 0, src = 0;
  if ((int64_t)threadIdx.x < n_all) {
    // block sl starts at sl * kL1Rows, or (sieve, sbase != NULL) at its
    // tile's region + sbase[sl]
    const int64_t sl = S0 + threadIdx.x;
    const uint16_t* o = soff + sl * (nd + 1) + B;
    len = (unsigned)o[1] - (unsigned)o[0];
    src = (sbase != nullptr ? (unsigned)((sl >> kp.slot_bits) * kSieveTileStride) + sbase[sl]
                            : (unsigned)(sl * kL1Rows)) + o[0];
  }
  unsigned total, nnz;
  const unsigned ex = block_excl_scan(len, wsum, &total);
  const unsigned idx = block_excl_scan(len > 0 ? 1u : 0u, wsum2, &nnz);
  if (len > 0) {
    rbeg[idx] = ex;
    rsrc[idx] = src;
  }
  if (threadIdx.x == 0) rbeg[nnz] = total;
  const int nr = (int)nnz;
  if ((int)threadIdx.x < nsub) s.gcur[threadIdx.x] = cur0;
  for (int t = threadIdx.x + blockDim.x; t < nsub; t += blockDim.x) {
    const int64_t b = s_first + t;
    s.gcur[t] = b < kp.n_buckets ? bucket_start[b] + gcur[g * M * kp.n_buckets + b] : 0u;
  }
  __syncthreads();
  if (total == 0) return;  // block-uniform
#ifdef PDP_PHASE_CLOCK
  c_tab = wall_clock64() - c0;
#endif
  const int bb = kp.bucket_bits;
  const uint32_t local_mask = (1u << bb) - 1;
  const int sub_shift = kp.pk_bits + kp.bucket_bits;
  const uint64_t sub_mask = (uint64_t)nsub - 1;
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  int j0 = 0;  // first run overlapping the window (block-uniform)
  for (unsigned base = 0, wend = 0; base < total; base = wend) {
    while (rbeg[j0 + 1] <= base) ++j0;
    wend = base + NR < total ? base + NR : total;
    // at most 256 runs per window (u8 run tags): a cap only tiny runs reach
    if (j0 + 256 < nr && rbeg[j0 + 256] < wend) wend = rbeg[j0 + 256];
    for (int j = j0 + (int)(threadIdx.x >> 6); j < nr && rbeg[j] < wend; j += nw) {
      const unsigned a = rbeg[j] > base ? rbeg[j] : base;
      const unsigned e = rbeg[j + 1] < wend ? rbeg[j + 1] : wend;
      for (unsigned v = a + lane; v < e; v += 64) s.dest[v - base] = (D)(j - j0);
    }
    __syncthreads();
    // records in two halves of loads in flight (register budget of two
    // workgroups per CU), unpacked into the counting sort's items
    KO x[NI];
    unsigned r[NI];
    int d[NI];
    constexpr int H = NI / 2;  // (all NI in one round spills 21-33 VGPRs: level 2 +37 %, profiles/r05/ab/ab9)
#pragma unroll
    for (int h = 0; h < NI; h += H) {
      KI raw[H];
      unsigned rr[H];  // PACKED: the record's tile's first row; else its row
      bool live[H];
#pragma unroll
      for (int q = 0; q < H; ++q) {
        const unsigned v = base + threadIdx.x + (unsigned)(h + q) * blockDim.x;
        live[q] = v < wend;
        if constexpr (ROWS1) {
          // key and row loads unconditional (a dead slot reads record 0), so
          // all H pairs go out together: under the branch each pair waited
          // for the previous one (COMPACT / WIDE)
          const int j = j0 + (int)s.dest[live[q] ? v - base : 0u];
          const unsigned i = live[q] ? rsrc[j] + (v - rbeg[j]) : 0u;
          raw[q] = keys1[i];
          rr[q] = rows1[i];
        } else if (live[q]) {
          const int j = j0 + (int)s.dest[v - base];
          const unsigned i = rsrc[j] + (v - rbeg[j]);
          raw[q] = keys1[i];
          rr[q] = rsrc[j] & ~(unsigned)(kTileRows - 1);  // first row of the run's tile
        }
      }
#pragma unroll
      for (int q = 0; q < H; ++q) {
        d[h + q] = -1;
        x[h + q] = 0;
        r[h + q] = 0;
        if (!live[q]) continue;
        if constexpr (PACKED) {
          const uint64_t v = raw[q];
          const uint32_t mid = (uint32_t)((v >> kp.pk_bits) & ((1ULL << (bb + kp.super_bits)) - 1));
          d[h + q] = (int)(mid >> bb);
          r[h + q] = rr[q] + (uint32_t)((v >> kPackedRowShift) & (kTileRows - 1));
          if constexpr (FMT == PDP_KEYS_PACKED64)  // (row | local pid | partition), all ones if dead
            x[h + q] = (KO)((v >> 63) ? ~0ULL
                                      : (((uint64_t)r[h + q] << kp.row_shift) |
                                         ((uint64_t)(mid & local_mask) << kp.pk_bits) | (v & kp.pk_mask)));
          else
            x[h + q] = unpacked_key<KO>(kp, mid & local_mask, v);
        } else {
          x[h + q] = (KO)raw[q];
          r[h + q] = rr[q];
          d[h + q] = (int)((raw[q] >> sub_shift) & sub_mask);
        }
      }
    }
    __syncthreads();  // the destination tags are rewritten by the counting sort
#ifdef PDP_PHASE_CLOCK
    const unsigned long long ca = wall_clock64();
#endif
    unsigned rank[NI];
    stage_count(s, nsub, d, rank);
#ifdef PDP_PHASE_CLOCK
    const unsigned long long cb = wall_clock64();
#endif
    stage_write(s, nsub, d, rank, x, r, keys2, rows2);
    for (int t = threadIdx.x; t < nsub; t += blockDim.x) s.gcur[t] += s.hist[t];
    __syncthreads();
#ifdef PDP_PHASE_CLOCK
    const unsigned long long cc = wall_clock64();
    c_ld += ca - (cw ? cw : c0 + c_tab);
    c_sort += cb - ca;
    c_wr += cc - cb;
    cw = cc;
    ++n_win;
#endif
  }
#ifdef PDP_PHASE_CLOCK
  if (threadIdx.x == 0 && blockIdx.x % 4001 == 77 && atomicAdd(&g_phase_l2, 1u) < 40u)
    printf("l2 wg %d runs %d records %u windows %d table %llu load %llu sort %llu write %llu total %llu (10 ns)\n",
           (int)blockIdx.x, nr, total, n_win, c_tab, c_ld, c_sort, c_wr, wall_clock64() - c0);
#endif
}

// Per-wave LDS queue of candidate rows (capacity 2 waves' worth): rows that
// pass a cheap per-row test are compacted here and the expensive per-candidate
// work then runs on full wavefronts instead of on the few lanes of each
// load that happen to hold a candidate.
struct WaveQueue {
  unsigned long long* key;  // [kQueueCap]
  unsigned* row;            // [kQueueCap]
};

// Streams the rows [begin, end) of one bucket: conv(record) gives the row's
// pair key, pred(key) selects candidates, work(key, row) handles each
// candidate on compacted wavefronts.  R = 16 / sizeof(K) rows per lane per
// 16-byte key load (and 4·R-byte row load when ROWS), KU loads in flight per
// lane; every wave runs the same trip count so the queue stays convergent.
// RM: what a candidate carries beside its key -- kRowNone, kRowLoad (rows[i],
// a 16-byte load per R records beside the keys) or kRowIndex (the record's
// position i in `keys`, for candidate lists).
// kRowFromKey: the row is the record's bits from row_shift up (PACKED64).
constexpr int kRowNone = 0, kRowLoad = 1, kRowIndex = 2, kRowFromKey = 3;
template <int KU, int RM, typename K, typename CV, typename P, typename W>
__device__ __forceinline__ void stream_bucket(const K* __restrict__ keys, const unsigned* __restrict__ rows,
                                              int64_t begin, int64_t end, WaveQueue q, CV&& conv, P&& pred,
                                              W&& work, int row_shift = 0) {
  constexpr bool ROWS = RM != kRowNone;
  constexpr bool LOADR = RM == kRowLoad;
  constexpr int R = 16 / sizeof(K);
  using KV = typename std::conditional<R == 4, uint4, ulonglong2>::type;
  using RV = typename std::conditional<R == 4, uint4, uint2>::type;
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ULL << lane) - 1;
  int n = 0;  // wave-uniform queue length
  auto push_p = [&](uint64_t x, uint32_t r, bool p) {
    const unsigned long long m = __ballot(p);
    if (p) {
      const int pos = n + __popcll(m & below);
      q.key[pos] = x;
      if (ROWS) q.row[pos] = r;
    }
    n += __popcll(m);
    if (n >= 64) {
      wave_lds_fence();
      const uint64_t wx = q.key[lane];
      const uint32_t wr = ROWS ? q.row[lane] : 0u;
      n -= 64;
      uint64_t mx = 0;
      uint32_t mr = 0;
      if (lane < n) {
        mx = q.key[64 + lane];
        if (ROWS) mr = q.row[64 + lane];
      }
      wave_lds_fence();
      if (lane < n) {
        q.key[lane] = mx;
        if (ROWS) q.row[lane] = mr;
      }
      work(wx, wr);
    }
  };
  auto push = [&](uint64_t x, uint32_t r) { push_p(x, r, pred(x)); };
  int64_t a0 = (begin + R - 1) & ~(int64_t)(R - 1);
  if (a0 > end) a0 = end;
  const int64_t a1 = a0 + ((end - a0) & ~(int64_t)(R - 1));
  {  // unaligned head rows [begin, a0) on lanes 0..R-2, tail rows [a1, end) on lanes R..2R-2 of wave 0
    uint64_t x = kEmpty;
    uint32_t r = 0;
    const int t = threadIdx.x;
    if (t < R - 1 && begin + t < a0) {
      x = conv(keys[begin + t]);
      if (LOADR) r = rows[begin + t];
      if (RM == kRowIndex) r = (uint32_t)(begin + t);
      if (RM == kRowFromKey) r = (uint32_t)((uint64_t)keys[begin + t] >> row_shift);
    }
    if (t >= R && t < 2 * R - 1 && a1 + (t - R) < end) {
      x = conv(keys[a1 + (t - R)]);
      if (LOADR) r = rows[a1 + (t - R)];
      if (RM == kRowIndex) r = (uint32_t)(a1 + (t - R));
      if (RM == kRowFromKey) r = (uint32_t)((uint64_t)keys[a1 + (t - R)] >> row_shift);
    }
    push(x, r);
  }
  const int64_t np = (a1 - a0) / R;
  const KV* kv = reinterpret_cast<const KV*>(keys + a0);
  const RV* rv = reinterpret_cast<const RV*>(rows + a0);
  const int64_t step = (int64_t)blockDim.x * KU;
  auto load = [&](int64_t g0, KV (&kx)[KU], RV (&rx)[KU]) {
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int64_t g = g0 + (int64_t)u * blockDim.x + threadIdx.x;
      if (g < np) {
        kx[u] = kv[g];
        if (LOADR) rx[u] = rv[g];
      } else {
        if constexpr (R == 4) kx[u] = make_uint4(~0u, ~0u, ~0u, ~0u);  // dead records
        else kx[u] = make_ulonglong2(kEmpty, kEmpty);
      }
    }
  };
  KV kx[KU];
  RV rx[KU];
  if (np > 0) load(0, kx, rx);
  for (int64_t g0 = 0; g0 < np; g0 += step) {
    // the row carried by component e of this lane's load u
    auto rowv = [&](int u, int e) -> uint32_t {
      if constexpr (RM == kRowIndex) {
        return (uint32_t)(a0 + (g0 + (int64_t)u * blockDim.x + threadIdx.x) * R + e);
      } else if constexpr (RM == kRowLoad) {
        if constexpr (R == 4) return e == 0 ? rx[u].x : (e == 1 ? rx[u].y : (e == 2 ? rx[u].z : rx[u].w));
        else return e == 0 ? rx[u].x : rx[u].y;
      } else if constexpr (RM == kRowFromKey) {
        static_assert(R == 2, "row-in-key records are 8 bytes");
        return (uint32_t)((uint64_t)(e == 0 ? kx[u].x : kx[u].y) >> row_shift);
      } else {
        return 0u;
      }
    };
    // software pipeline: the next batch's loads are in flight while this
    // batch runs through the queue (LDS work only, no vector memory)
    KV nk[KU];
    RV nr[KU];
    const bool more = g0 + step < np;  // block-uniform
    if (more) load(g0 + step, nk, nr);
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      if constexpr (R == 4) {
        push(conv(kx[u].x), rowv(u, 0));
        push(conv(kx[u].y), rowv(u, 1));
        push(conv(kx[u].z), rowv(u, 2));
        push(conv(kx[u].w), rowv(u, 3));
      } else {
        push(conv(kx[u].x), rowv(u, 0));
        push(conv(kx[u].y), rowv(u, 1));
      }
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        kx[u] = nk[u];
        if (LOADR) rx[u] = nr[u];
      }
    }
  }
  if (n > 0) {  // partial wave
    wave_lds_fence();
    if (lane < n) work((uint64_t)q.key[lane], ROWS ? q.row[lane] : 0u);
  }
}

// blockIdx -> work index with each XCD (blockIdx % 8) owning one contiguous
// block: XCD x gets q + (x < rem) indices starting at x * q + min(x, rem).
// A bijection on [0, G) for any G; a speed hint only.
__device__ __forceinline__ int64_t xcd_major(int64_t id, int64_t G) {
  const int64_t q = G >> 3, rem = G & 7, x = id & 7, j = id >> 3;
  return x * q + (x < rem ? x : rem) + j;
}

struct PairRecords {  // PDP_MERGE_RANGES output of the bucket kernel
  unsigned* runs;                // [n_ranges + 1][run_stride] run starts within the bucket block (range-major)
  int64_t run_stride;            // buckets_out: one column per output bucket
  unsigned long long* key;       // (partition << 32) | count
  double* f0;                    // sum (int64 bits with PDP_SUM_INT)
  double* f1;                    // normalized sum
  double* f2;                    // normalized sum of squares
};

// PDP_PHASE_CLOCK (profiling builds only, tools/build_variants.sh): thread 0
// of a few buckets prints the wall-clock time (10 ns ticks) of each phase of
// k_bucket_bound; results are unchanged (the r02 ablation builds that skipped
// phases left the merge reading unwritten records)
#ifdef PDP_PHASE_CLOCK
#define PDP_PHASE(k)                             \
  do {                                           \
    __syncthreads();                             \
    if (threadIdx.x == 0) ph[k] = wall_clock64(); \
  } while (0)
#else
#define PDP_PHASE(k) \
  do {               \
  } while (0)
#endif

template <int VALUE_KIND, bool KEEP_ALL_ROWS, bool RANGES, int REC>
__global__ void __launch_bounds__(kBucketThreads) k_bucket_bound(KP kp, const RecKey<REC == kRecCompact>* __restrict__ keys,
                                                                 const unsigned* __restrict__ rowidx,
                                                                 const unsigned* __restrict__ offsets,
                                                                 const void* __restrict__ value,
                                                                 pdp_partition_accumulators acc, PairRecords rec,
                                                                 RecKey<REC == kRecCompact>* __restrict__ cand_key,
                                                                 unsigned* __restrict__ cand_idx,
                                                                 unsigned* __restrict__ unres_bits,
                                                                 unsigned* __restrict__ unres_list,
                                                                 unsigned* __restrict__ sctl, unsigned* __restrict__ err,
                                                                 unsigned long long* __restrict__ fix_rec,
                                                                 const unsigned* __restrict__ unres_prev,
                                                                 const unsigned* __restrict__ blist) {
  constexpr bool COMPACT = REC == kRecCompact;
  extern __shared__ unsigned long long smem[];
  __shared__ unsigned ccount;
  const int64_t S = (int64_t)1 << kp.bucket_bits;
  const int l0 = kp.l0;
  auto body = [&](const int64_t b) {
#ifdef PDP_PHASE_CLOCK
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};
  if (threadIdx.x == 0) ph[0] = wall_clock64();
#endif
  // threshold sieve: a privacy id of this bucket with fewer than l0
  // candidate pairs (its sketch not full; `sketch` = false: every id) may
  // have kept pairs among rows this launch did not see; mark it in the
  // bitmap (a wave covers 64 ids = one u64 word; the bucket's ids are whole
  // words) and list it.  unres_prev (the band's fix-up launch): only ids the
  // main launch left unresolved can be.
  auto mark = [&](bool sketch) {
    const int lane = threadIdx.x & 63;
    const int64_t id0 = b << kp.bucket_bits;
    for (int64_t p0 = (int64_t)(threadIdx.x >> 6) * 64; p0 < S; p0 += blockDim.x) {
      const int64_t id = id0 + p0 + lane;
      bool un = id < kp.U;
      if (sketch) un = un && smem[(int64_t)(l0 - 1) * S + p0 + lane] == kEmpty;  // sk is smem's first array
      if (unres_prev != nullptr) un = un && ((unres_prev[id >> 5] >> (id & 31)) & 1u);
      const unsigned long long m = __ballot(un);
      if (lane == 0) reinterpret_cast<uint2*>(unres_bits)[(id0 + p0) >> 6] = make_uint2((unsigned)m, (unsigned)(m >> 32));
      if (m) {
        unsigned base = 0;
        if (lane == 0) base = atomicAdd(sctl, (unsigned)__popcll(m));
        base = __shfl(base, 0, 64);
        if (un) unres_list[base + __popcll(m & ((1ULL << lane) - 1))] = (unsigned)id;
      }
    }
  };
  // an empty bucket of a fix-up launch (most of them: only unresolved
  // privacy ids have rows there) writes its empty runs and stops -- in the
  // band's fix-up launch after marking its previously unresolved ids (none
  // of their pairs is below t2); the main launch's empty buckets still mark
  // their privacy ids unresolved
  if ((!kp.sieve_mark || unres_prev != nullptr) && offsets[b] == offsets[b + 1]) {  // block-uniform
    if (RANGES) {
      for (int t = threadIdx.x; t <= kp.n_ranges; t += blockDim.x) rec.runs[t * rec.run_stride + b] = 0;
    }
    if (kp.sieve_mark) mark(false);
    return;
  }
  const int64_t n_slots = S * l0;
  // LDS state is structure-of-arrays: entry j of privacy id p at [j * S + p]
  // (row-sketch entry t of slot s at [t * S*l0 + s]), so a wave's lanes, which
  // touch random privacy ids, spread over the LDS banks
  unsigned long long* sk = smem;                      // [l0][S] pair sketch per pid
  unsigned long long* rsk = sk + n_slots;             // bounded: [linf][S*l0] row sketches
  double* tot = (double*)(sk + n_slots);              // keep-all: [3][S*l0] pair sums
  unsigned* cnt = KEEP_ALL_ROWS ? (unsigned*)(tot + 3 * n_slots) : (unsigned*)(rsk + n_slots * kp.linf);
  unsigned* rh = cnt + n_slots;          // RANGES: [n_ranges] kept pairs per partition range
  unsigned* rcur = rh + kp.n_ranges;     //         [n_ranges] write cursors
  unsigned* wsum = rcur + kp.n_ranges;   //         block-scan scratch
  const int n_waves = (int)(blockDim.x >> 6);  // 16 or 8 (Plan.bucket_threads)
  unsigned* tail = RANGES ? wsum + n_waves + 1 : rh;
  // derived from smem by offset (not through an integer round trip) so the
  // compiler keeps the LDS address space and emits ds_* rather than flat_*
  unsigned long long* qbase = smem + (((const char*)tail - (const char*)smem) + 7) / 8;
  const int wave = threadIdx.x >> 6;
  const WaveQueue wq{qbase + wave * kQueueCap,
                     (unsigned*)(qbase + n_waves * kQueueCap) + wave * kQueueCap};
  // per privacy id of the bucket, after the queues: {pid_hash (expand_key),
  // high half of its sketch maximum (b1_candidate)}
  uint2* hpid = (uint2*)((unsigned*)(qbase + n_waves * kQueueCap) + n_waves * kQueueCap);
  for (int64_t t = threadIdx.x; t < S; t += blockDim.x)
    hpid[t] = make_uint2(pid_hash(kp.seed, (b << kp.bucket_bits) | t), 0xFFFFFFFFu);
  for (int64_t t = threadIdx.x; t < n_slots; t += blockDim.x) {
    sk[t] = kEmpty;
    cnt[t] = 0;
  }
  if (RANGES)
    for (int t = threadIdx.x; t < kp.n_ranges; t += blockDim.x) rh[t] = 0;
  if (!KEEP_ALL_ROWS) {
    for (int64_t t = threadIdx.x; t < n_slots * kp.linf; t += blockDim.x) rsk[t] = kEmpty;
  } else {
    for (int64_t t = threadIdx.x; t < 3 * n_slots; t += blockDim.x) tot[t] = 0.0;
  }
  __syncthreads();
  const int64_t begin = offsets[b];
  const int64_t end = offsets[b + 1];  // offsets has n_buckets + 1 entries
  const uint64_t bmask = (uint64_t)S - 1;
  // PACKED64 records (row | local pid | partition; all ones dead) and their
  // candidate-list form (local pid | partition)
  auto expand64 = [&](unsigned long long v) -> uint64_t {
    if (v == ~0ULL) return kEmpty;
    const uint64_t local = (v >> kp.pk_bits) & ((1ULL << kp.bucket_bits) - 1);
    return pair_key_from(hpid[local].x, kp.seed, (int64_t)(v & kp.pk_mask), local << kp.pk_bits, kp.rand_shift);
  };
  auto conv = [&](RecKey<COMPACT> v) -> uint64_t {
    if constexpr (REC == kRecP64) return expand64(v);
    else return expand_key(kp, hpid, v);
  };
  // B1: bottom-l0 distinct pair keys per privacy id; candidates are keys at or
  // below their sketch's current maximum.  A pair kept in the end entered the
  // sketch at its first row and never left it (the maximum only decreases),
  // so every one of its rows is a candidate here: the candidates still in
  // their sketch after the insert are appended to a per-bucket list
  // (record-local key + row) and B2 reads only that list.
  if (threadIdx.x == 0) ccount = 0;
  __syncthreads();
  PDP_PHASE(1);
  const uint64_t lbits = ((uint64_t)1 << (kp.pk_bits + kp.bucket_bits)) - 1;  // local pid | partition
  // (each record's row index rides along, loaded with its key: B2 then needs
  // no dependent gather of it)
  stream_bucket<COMPACT ? 4 : kUnroll, REC == kRecP64 ? kRowFromKey : kRowLoad>(
      keys, rowidx, begin, end, wq,
      // the candidate test rides on the pid-hash read (b1_candidate)
      [&](RecKey<COMPACT> v) -> uint64_t {
        if constexpr (REC == kRecP64) {
          const uint64_t x = expand64(v);
          if (x == kEmpty) return kEmpty;
          return (uint32_t)(x >> 32) <= hpid[(v >> kp.pk_bits) & ((1ULL << kp.bucket_bits) - 1)].y ? x : kEmpty;
        } else {
          return b1_candidate(kp, hpid, v);
        }
      },
      [&](uint64_t x) { return x != kEmpty; },
      [&](uint64_t x, uint32_t i)  {  // i: the record's row
        const int64_t pl = (int64_t)((x >> kp.pk_bits) & bmask);
        unsigned long long* s = sk + pl;
        if (x < s[(l0 - 1) * S]) sketch_insert_strided(s, l0, S, x);
        const unsigned long long smax = s[(l0 - 1) * S];
        // a maximum read after this insert: never below the current one
        hpid[pl].y = (uint32_t)(smax >> 32);
        const bool keep = x <= smax;
        const unsigned long long active = __ballot(true);
        const unsigned long long m = __ballot(keep);
        const int leader = __ffsll((long long)active) - 1;
        unsigned base = 0;
        if ((int)(threadIdx.x & 63) == leader && m) base = atomicAdd(&ccount, (unsigned)__popcll(m));
        base = __shfl(base, leader, 64);
        if (keep) {
          const int64_t o = begin + base + __popcll(m & ((1ULL << (threadIdx.x & 63)) - 1));
          cand_key[o] = (RecKey<COMPACT>)(x & lbits);
          cand_idx[o] = i;
        }
      },
      kp.row_shift);
  __syncthreads();
  if (kp.sieve_mark) mark(true);  // emits nothing for its unresolved ids (B2 skips them): the fix-up's
  PDP_PHASE(2);
  // B2: rows of kept pairs, from B1's candidate list (key + row)
  const int flags = kp.clip.flags;
  stream_bucket<COMPACT ? 1 : kUnroll / 2, kRowLoad>(
      cand_key, cand_idx, begin, begin + ccount, wq, conv,
      [&](uint64_t x) {
        // (dead keys: also the padding lanes' kEmpty, whose bits name no pid)
        if (dead_key(x, kp.rand_shift)) return false;
        const unsigned long long smax = sk[(l0 - 1) * S + (int64_t)((x >> kp.pk_bits) & bmask)];
        // band: an unresolved id's candidate rows (every one of its records
        // is on the list; the sieve dropped the dead ones) go to the fix-up
        if (kp.sieve_emit && smax == kEmpty) return true;
        return x <= smax && !(kp.sieve_mark && smax == kEmpty);  // sieve: unresolved ids are the fix-up's
      },
      [&](uint64_t x, uint32_t ci)  {
      const int64_t pl = (x >> kp.pk_bits) & bmask;
      if (kp.sieve_emit) {  // block-uniform: the main launch with the band
        const bool un = sk[(l0 - 1) * S + pl] == kEmpty && ci < (uint64_t)kp.n;
        const unsigned long long mu = __ballot(un);
        if (mu) {  // wave-uniform
          const int lead = __ffsll((long long)mu) - 1;
          const int lane = threadIdx.x & 63;
          unsigned base = 0;
          if (lane == lead) base = atomicAdd(sctl + 1, (unsigned)__popcll(mu));
          base = __shfl(base, lead, 64);
          const int64_t at = (int64_t)base + __popcll(mu & ((1ULL << lane) - 1));
          if (un && at < kp.fix_cap)
            fix_rec[at] = ((unsigned long long)(uint32_t)((b << kp.bucket_bits) | pl) << 32) | (unsigned long long)ci;
        }
        if (sk[(l0 - 1) * S + pl] == kEmpty) return;
      }
      const int j = sketch_find_strided(sk + pl, l0, S, x);
      if (j < 0) return;
      const uint32_t r = ci;  // the candidate's row (B1 carried it)
      if (r >= (uint64_t)kp.n) {  // malformed record: flagged, never dereferenced
        atomicOr(err, 1u);
        return;
      }
      const int64_t slot = j * S + pl;  // entry j of pid pl (structure of arrays)
      atomicAdd(cnt + slot, 1u);
      if (!KEEP_ALL_ROWS) {
        const uint64_t y = row_key(kp.row_seed, kp.row_offset + r, r);
        unsigned long long* rs = rsk + slot;
        if (y < rs[(kp.linf - 1) * n_slots]) sketch_insert_strided(rs, kp.linf, n_slots, y);
      } else if (VALUE_KIND != PDP_VALUE_NONE) {
        double v;
        long long iv;
        load_value<VALUE_KIND>(value, r, &v, &iv);
        if (flags & PDP_SUM_PER_PARTITION) {
          if (flags & PDP_SUM_INT) atomicAdd((unsigned long long*)(tot + slot), (unsigned long long)iv);
          else atomicAdd(tot + slot, v);
        } else if (flags & PDP_ACC_SUM) {
          if (flags & PDP_SUM_INT)
            atomicAdd((unsigned long long*)(tot + slot),
                      (unsigned long long)clamp_ll(iv, (long long)kp.clip.lo, (long long)kp.clip.hi));
          else atomicAdd(tot + slot, fmin(fmax(v, kp.clip.lo), kp.clip.hi));
        }
        if (flags & (PDP_ACC_NSUM | PDP_ACC_NSUM2)) {
          const double c = fmin(fmax(v, kp.clip.lo), kp.clip.hi) - kp.clip.mid;
          if (flags & PDP_ACC_NSUM) atomicAdd(tot + n_slots + slot, c);
          if (flags & PDP_ACC_NSUM2) atomicAdd(tot + 2 * n_slots + slot, c * c);
        }
      }
  });
  __syncthreads();
  PDP_PHASE(3);
  // B2.5: the kept rows' values replace their row keys in the row sketches
  // (B3 then reads LDS only; same rows, same order, so the sums are
  // unchanged), all of a thread's gathers in flight together.  The first
  // batch (entries 0 and 1 of the thread's first G slots: all of them at C3,
  // C2 and C4) is issued before B3a's LDS histogram, scan and run-table
  // stores, which then run under the gathers' latency
  constexpr int G = 4;
  constexpr int T0 = 2;  // row-sketch entries of the pre-issued batch (C2 / C4: Linf = 2)
  constexpr bool B25 = !KEEP_ALL_ROWS && VALUE_KIND != PDP_VALUE_NONE;
  long long bits0[T0][G];
  bool live0[T0][G];
  if constexpr (B25) {
    uint32_t rr[T0][G];
#pragma unroll
    for (int t = 0; t < T0; ++t)
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int64_t slot = (int64_t)threadIdx.x + (int64_t)u * blockDim.x;
        live0[t][u] = t < kp.linf && slot < n_slots && sk[slot] != kEmpty && (unsigned)t < cnt[slot];
        rr[t][u] = live0[t][u] ? (uint32_t)rsk[t * n_slots + slot] : 0u;
      }
#pragma unroll
    for (int t = 0; t < T0; ++t)
#pragma unroll
      for (int u = 0; u < G; ++u) bits0[t][u] = live0[t][u] ? ((const long long*)value)[rr[t][u]] : 0;
  }
  PDP_PHASE(4);
  const void* const b3_value = B25 ? nullptr : value;
  if (RANGES) {
    // B3a: kept pairs per partition range -> this bucket's run starts
    for (int64_t slot = threadIdx.x; slot < n_slots; slot += blockDim.x) {
      const uint64_t x = sk[slot];
      if (x == kEmpty || cnt[slot] == 0 || (int64_t)(x & kp.pk_mask) >= kp.P) continue;
      atomicAdd(rh + ((x & kp.pk_mask) >> kp.range_bits), 1u);
    }
    __syncthreads();
    const unsigned h = threadIdx.x < kp.n_ranges ? rh[threadIdx.x] : 0u;  // n_ranges <= blockDim
    unsigned total;
    const unsigned ex = block_excl_scan(h, wsum, &total);
    if (threadIdx.x < kp.n_ranges) {
      rec.runs[threadIdx.x * rec.run_stride + b] = ex;
      rcur[threadIdx.x] = ex;
    }
    if (threadIdx.x == 0) rec.runs[kp.n_ranges * rec.run_stride + b] = total;
    __syncthreads();
  }
  if constexpr (B25) {
#pragma unroll
    for (int t = 0; t < T0; ++t)
#pragma unroll
      for (int u = 0; u < G; ++u)
        if (live0[t][u]) rsk[t * n_slots + (int64_t)threadIdx.x + (int64_t)u * blockDim.x] = (unsigned long long)bits0[t][u];
    // the rest (more slots than G per thread, or Linf > T0), G at a time
    for (int t = 0; t < kp.linf; ++t) {
      for (int64_t s0 = threadIdx.x + (t < T0 ? (int64_t)G * blockDim.x : 0); s0 < n_slots;
           s0 += (int64_t)G * blockDim.x) {
        uint32_t rr[G];
        bool live[G];
#pragma unroll
        for (int u = 0; u < G; ++u) {
          const int64_t slot = s0 + (int64_t)u * blockDim.x;
          live[u] = slot < n_slots && sk[slot] != kEmpty && (unsigned)t < cnt[slot];
          rr[u] = live[u] ? (uint32_t)rsk[t * n_slots + slot] : 0u;
        }
        long long bits[G];
#pragma unroll
        for (int u = 0; u < G; ++u)
          bits[u] = live[u] ? ((const long long*)value)[rr[u]] : 0;
#pragma unroll
        for (int u = 0; u < G; ++u)
          if (live[u]) rsk[t * n_slots + s0 + (int64_t)u * blockDim.x] = (unsigned long long)bits[u];
      }
    }
    __syncthreads();
  }
  // B3: merge every kept pair into its partition (RANGES: emit a pair record)
  for (int64_t slot = threadIdx.x; slot < n_slots; slot += blockDim.x) {
    const uint64_t x = sk[slot];
    if (x == kEmpty) continue;
    const int64_t p = (int64_t)(x & kp.pk_mask);
    const unsigned c = cnt[slot];
    if (c == 0) continue;
    if (p >= kp.P) {  // malformed record (pk_mask spans up to 2^pk_bits > P): flagged, skipped
      atomicOr(err, 1u);
      continue;
    }
    PairSums ps;
    if (!KEEP_ALL_ROWS) {
      const long long m = c < (unsigned)kp.linf ? (long long)c : (long long)kp.linf;
      ps = pair_sums_from_rows<VALUE_KIND>(rsk + slot, m, b3_value, kp.clip, n_slots);
    } else if (VALUE_KIND != PDP_VALUE_NONE) {
      ps = pair_sums_from_totals((long long)c, tot[slot], tot[n_slots + slot], tot[2 * n_slots + slot], kp.clip);
    } else {
      ps = PairSums{(long long)c, 0, 0.0, 0.0, 0.0};
    }
    if (RANGES) {
      const int64_t i = b * n_slots + atomicAdd(rcur + (p >> kp.range_bits), 1u);
      rec.key[i] = ((unsigned long long)p << 32) | (unsigned long long)(uint32_t)ps.count;
      if (flags & (PDP_ACC_SUM | PDP_SUM_PER_PARTITION))
        rec.f0[i] = (flags & PDP_SUM_INT) ? __longlong_as_double(ps.isum) : ps.fsum;
      if (flags & PDP_ACC_NSUM) rec.f1[i] = ps.nsum;
      if (flags & PDP_ACC_NSUM2) rec.f2[i] = ps.nsum2;
    } else {
      add_pair_to_partition(acc, p, ps, flags);
    }
  }
#ifdef PDP_PHASE_CLOCK
  PDP_PHASE(5);
  if (threadIdx.x == 0 && blockIdx.x % 997 == 11 && atomicAdd(&g_phase_bk, 1u) < 40u)
    printf("phase bucket %d records %u cand %u init %llu b1 %llu b2 %llu b25 %llu b3 %llu (10 ns)\n", (int)b,
           (unsigned)(end - begin), ccount, ph[1] - ph[0], ph[2] - ph[1], ph[3] - ph[2], ph[4] - ph[3],
           ph[5] - ph[4]);
#endif
  };
  if (blist == nullptr) {
    // XCD-aware bucket order: workgroups are dispatched round-robin over the
    // 8 XCDs (blockIdx % 8), so XCD x takes one contiguous block of buckets
    // and its writes to the range-major run table (and the records) share L2
    // lines
    body(xcd_major(blockIdx.x, gridDim.x));
  } else {
    // a fix-up launch over the buckets that hold fix-up rows only (blist[0]
    // of them, listed from blist[1]; k_fix_buckets did the empty ones'
    // work): a persistent loop, one bucket at a time
    const unsigned nb = blist[0];
    for (unsigned i = blockIdx.x; i < nb; i += gridDim.x) {
      body((int64_t)blist[1 + i]);
      __syncthreads();  // the LDS state is the next bucket's
    }
  }
}

// ------------------------------------------------ threshold-sieve fix-up --
// Bloom filter of the unresolved privacy ids (k_sieve_rescan): one
// multiplicative hash per id, its top 12 bits the LDS word, two bit
// positions from its low 10 bits (one full-rate-cheap test per row: the
// rescan streams 8 B per row and must stay memory-bound)
constexpr int kBloomBits = 12;
static_assert(kBloomWords == 1 << kBloomBits, "Bloom filter size");
__device__ __forceinline__ uint32_t bloom_hash(uint32_t id) { return id * 0x9E3779B1u; }
__device__ __forceinline__ unsigned bloom_word(uint32_t h) { return h >> (32 - kBloomBits); }
__device__ __forceinline__ unsigned bloom_bits(uint32_t h) { return (1u << (h & 31)) | (1u << ((h >> 5) & 31)); }

// Fix-up step 1: the rows that may belong to an unresolved privacy id.  One
// streaming read of the privacy-id column (8 B per row); a row is tested
// against an LDS Bloom filter of the unresolved list (one word, two bits;
// each workgroup builds its own), and the positives -- with the filter's
// false positives, ~1e-3 of the rows -- are appended to fix_rec as
// (privacy id << 32 | row).  The test touches LDS only, and positives wait in
// a per-wave LDS queue that goes out 64 entries at a time, so the stream's
// loads (the next iteration's in flight while this one is tested) are never
// drained by a dependent global access.  k_fix_filter then keeps the exact
// ones.  Without the filter (more than kBloomMaxIds unresolved ids) every
// in-range row is tested against the bitmap here.  No unresolved id: no work.
constexpr int kRescanQueue = 128;  // per-wave queue: < 64 waiting + one batch of <= 64
template <bool BLOOM>
__device__ __forceinline__ bool rescan_maybe(const KP& kp, int64_t u, const unsigned* bloom,
                                             const unsigned* __restrict__ unres_bits) {
  if constexpr (BLOOM) {  // LDS only, no short circuit: the reads of a batch go out together
    const uint32_t h = bloom_hash((uint32_t)u);
    const unsigned bits = bloom_bits(h);
    return ((uint64_t)u < (uint64_t)kp.U) & ((bloom[bloom_word(h)] & bits) == bits);
  } else {
    return (uint64_t)u < (uint64_t)kp.U && ((unres_bits[u >> 5] >> (u & 31)) & 1u);  // invalid ids: flagged by level 1
  }
}

template <bool VEC>
__global__ void __launch_bounds__(kRescanThreads) k_sieve_rescan(KP kp, const int64_t* __restrict__ pid,
                                                                 const unsigned* __restrict__ unres_bits,
                                                                 const unsigned* __restrict__ unres_list,
                                                                 unsigned* __restrict__ sctl,
                                                                 unsigned long long* __restrict__ fix_rec) {
  __shared__ unsigned bloom[kBloomWords];
  __shared__ unsigned long long queue[kRescanThreads / 64][kRescanQueue];
  const unsigned n_unres = sctl[0];
  if (n_unres == 0) return;  // grid-uniform
  const bool use_bloom = n_unres <= kBloomMaxIds;  // grid-uniform
  for (int i = threadIdx.x; i < kBloomWords; i += blockDim.x) bloom[i] = 0;
  __syncthreads();
  for (unsigned i = threadIdx.x; use_bloom && i < n_unres; i += blockDim.x) {
    const uint32_t h = bloom_hash(unres_list[i]);
    atomicOr(bloom + bloom_word(h), bloom_bits(h));
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ULL << lane) - 1;
  unsigned long long* const wq = queue[threadIdx.x >> 6];
  int qn = 0;  // wave-uniform queue length
  // the wave's positives (`pos` on the active lanes) into its queue; 64 out
  auto enqueue = [&](bool pos, int64_t u, int64_t i) {
    const unsigned long long m = __ballot(pos);
    if (m == 0) return;  // wave-uniform
    if (pos) wq[qn + __popcll(m & below)] = ((unsigned long long)u << 32) | (unsigned long long)(uint32_t)i;
    qn += __popcll(m);
    if (qn >= 64) {
      wave_lds_fence();
      const unsigned long long e = wq[lane];
      unsigned base = 0;
      if (lane == 0) base = atomicAdd(sctl + 1, 64u);
      base = __shfl(base, 0, 64);
      if (base + lane < kp.fix_cap) fix_rec[base + lane] = e;
      const unsigned long long rest = lane + 64 < qn ? wq[lane + 64] : 0ULL;
      wave_lds_fence();
      if (lane + 64 < qn) wq[lane] = rest;
      qn -= 64;
      wave_lds_fence();
    }
  };
  constexpr int KU = 8;  // 16-byte loads (two rows) per lane and iteration
  const int64_t per_iter = (int64_t)blockDim.x * KU;  // row pairs per block iteration
  const int64_t n_iters = VEC ? (kp.n / 2) / per_iter : 0;
  const longlong2* __restrict__ pv = reinterpret_cast<const longlong2*>(pid);
  auto run = [&](auto bloom_tag) {
    constexpr bool BLOOM = decltype(bloom_tag)::value;
    int64_t it = blockIdx.x;
    if (it < n_iters) {
      longlong2 cur[KU], nxt[KU];
#pragma unroll
      for (int v = 0; v < KU; ++v) cur[v] = pv[it * per_iter + (int64_t)v * blockDim.x + threadIdx.x];
      for (; it < n_iters; it += gridDim.x) {  // block-uniform trips
        const int64_t nx = it + gridDim.x < n_iters ? it + gridDim.x : it;  // in range: no branch around the loads
#pragma unroll
        for (int v = 0; v < KU; ++v) nxt[v] = pv[nx * per_iter + (int64_t)v * blockDim.x + threadIdx.x];
        unsigned maybe = 0;
#pragma unroll
        for (int v = 0; v < KU; ++v) {
          maybe |= (unsigned)rescan_maybe<BLOOM>(kp, cur[v].x, bloom, unres_bits) << (2 * v);
          maybe |= (unsigned)rescan_maybe<BLOOM>(kp, cur[v].y, bloom, unres_bits) << (2 * v + 1);
        }
        if (__ballot(maybe != 0) != 0) {  // wave-uniform, ~1 in 2 wave iterations at C3
#pragma unroll
          for (int v = 0; v < KU; ++v) {
            const int64_t i = 2 * (it * per_iter + (int64_t)v * blockDim.x + threadIdx.x);
            enqueue((maybe >> (2 * v)) & 1u, cur[v].x, i);
            enqueue((maybe >> (2 * v + 1)) & 1u, cur[v].y, i + 1);
          }
        }
#pragma unroll
        for (int v = 0; v < KU; ++v) cur[v] = nxt[v];
      }
    }
    // the rows no full iteration covered (all of them without VEC): every lane
    // of a wave runs the same trip count, so the queue stays wave-uniform
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t i0 = 2 * n_iters * per_iter + (int64_t)blockIdx.x * blockDim.x;
    for (int64_t w0 = i0 + (int64_t)(threadIdx.x & ~63); w0 < kp.n; w0 += stride) {  // w0: the wave's first row
      const int64_t i = w0 + lane;
      const int64_t u = i < kp.n ? pid[i] : -1;
      enqueue(i < kp.n && rescan_maybe<BLOOM>(kp, u, bloom, unres_bits), u, i);
    }
  };
  if (use_bloom) run(std::true_type{});
  else run(std::false_type{});
  // the rest of the queue
  wave_lds_fence();
  if (qn > 0) {
    unsigned base = 0;
    if (lane == 0) base = atomicAdd(sctl + 1, (unsigned)qn);
    base = __shfl(base, 0, 64);
    if (lane < qn && base + lane < kp.fix_cap) fix_rec[base + lane] = wq[lane];
  }
}

// Fix-up step 1, side band: the tiles' band lists (privacy id << 32 | row,
// written by k_sieve_l1<BAND>) instead of the whole privacy-id column, with
// the same Bloom filter, per-wave queues and output (fix_rec, sctl[1]) as
// k_sieve_rescan; the unresolved ids' candidate rows are already on fix_rec
// (the main bucket launch put them there).  Every lane of a wave runs the
// same trips (band_cnt[t] is block-uniform), so the queues stay wave-uniform.
__global__ void __launch_bounds__(kRescanThreads) k_band_scan(KP kp, const unsigned long long* __restrict__ band,
                                                              const unsigned* __restrict__ band_cnt,
                                                              const unsigned* __restrict__ unres_bits,
                                                              const unsigned* __restrict__ unres_list,
                                                              unsigned* __restrict__ sctl,
                                                              unsigned long long* __restrict__ fix_rec) {
  __shared__ unsigned bloom[kBloomWords];
  __shared__ unsigned long long queue[kRescanThreads / 64][kRescanQueue];
  const unsigned n_unres = sctl[0];
  if (n_unres == 0) return;  // grid-uniform
  const bool use_bloom = n_unres <= kBloomMaxIds;  // grid-uniform
  for (int i = threadIdx.x; i < kBloomWords; i += blockDim.x) bloom[i] = 0;
  __syncthreads();
  for (unsigned i = threadIdx.x; use_bloom && i < n_unres; i += blockDim.x) {
    const uint32_t h = bloom_hash(unres_list[i]);
    atomicOr(bloom + bloom_word(h), bloom_bits(h));
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ULL << lane) - 1;
  unsigned long long* const wq = queue[threadIdx.x >> 6];
  int qn = 0;
  auto enqueue = [&](bool pos, unsigned long long e) {
    const unsigned long long m = __ballot(pos);
    if (m == 0) return;  // wave-uniform
    if (pos) wq[qn + __popcll(m & below)] = e;
    qn += __popcll(m);
    if (qn >= 64) {
      wave_lds_fence();
      const unsigned long long x = wq[lane];
      unsigned base = 0;
      if (lane == 0) base = atomicAdd(sctl + 1, 64u);
      base = __shfl(base, 0, 64);
      if (base + lane < kp.fix_cap) fix_rec[base + lane] = x;
      const unsigned long long rest = lane + 64 < qn ? wq[lane + 64] : 0ULL;
      wave_lds_fence();
      if (lane + 64 < qn) wq[lane] = rest;
      qn -= 64;
      wave_lds_fence();
    }
  };
  // entries per lane and trip, loaded together (8: at an N = 8 rank's share a
  // block sees ~2 tiles, so its trips are latency rounds, not a stream)
  constexpr int KU = 8;
  const int64_t w0 = (int64_t)(threadIdx.x >> 6) * 64 * KU;
  auto run = [&](auto bloom_tag) {
    constexpr bool BLOOM = decltype(bloom_tag)::value;
    for (int64_t t = blockIdx.x; t < kp.n_tiles; t += gridDim.x) {
      const unsigned long long* __restrict__ bt = band + t * kBandTileStride;
      unsigned cnt = band_cnt[t];
      cnt = cnt <= (unsigned)kTileRows ? cnt : (unsigned)kTileRows;
      for (int64_t j0 = w0; j0 < cnt; j0 += (int64_t)blockDim.x * KU) {  // wave-uniform trips
        unsigned long long e[KU];
#pragma unroll
        for (int v = 0; v < KU; ++v) {
          const int64_t j = j0 + v * 64 + lane;
          e[v] = j < cnt ? ld_maybe_nt<PDP_NT_BS>(bt + j) : ~0ULL;
        }
#pragma unroll
        for (int v = 0; v < KU; ++v) {
          const int64_t u = e[v] == ~0ULL ? -1 : (int64_t)(e[v] >> 32);
          enqueue(u >= 0 && rescan_maybe<BLOOM>(kp, u, bloom, unres_bits), e[v]);
        }
      }
    }
  };
  if (use_bloom) run(std::true_type{});
  else run(std::false_type{});
  wave_lds_fence();
  if (qn > 0) {
    unsigned base = 0;
    if (lane == 0) base = atomicAdd(sctl + 1, (unsigned)qn);
    base = __shfl(base, 0, 64);
    if (lane < qn && base + lane < kp.fix_cap) fix_rec[base + lane] = wq[lane];
  }
}

// Fix-up step 1b: the exact test of every listed row (the bitmap of the
// unresolved ids); a false positive's entry becomes ~0 (skipped by
// k_fix_scatter), a true one is counted for its bucket.
__global__ void __launch_bounds__(kBlock) k_fix_filter(KP kp, const unsigned* __restrict__ unres_bits,
                                                       const unsigned* __restrict__ sctl,
                                                       unsigned long long* __restrict__ fix_rec,
                                                       unsigned* __restrict__ fix_cnt, unsigned* err,
                                                       unsigned* __restrict__ blist) {
  // a list longer than its region cannot happen (each list holds distinct
  // rows); were it to, error bit 1 says so instead of reading past the region
  const int64_t listed = sctl[1];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (listed > kp.fix_cap) atomicOr(err, 2u);
    blist[0] = 0;  // k_fix_buckets' count (the previous fix-up launch is done with it)
  }
  const int64_t total = listed < kp.fix_cap ? listed : kp.fix_cap;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t u = fix_rec[i] >> 32;
    if ((unres_bits[u >> 5] >> (u & 31)) & 1u) atomicAdd(fix_cnt + (u >> kp.bucket_bits), 1u);
    else fix_rec[i] = ~0ULL;
  }
}

// Fix-up step 2: the listed rows -> bucket order (fix_start = exclusive scan
// of the per-bucket counts; a slot per row from the bucket's cursor), as the
// bucket kernel's records: (bucket-local pid << pk_bits | partition), dead
// bit for a non-public or invalid partition, and the row.
template <int REC>
__global__ void __launch_bounds__(kBlock) k_fix_scatter(KP kp, const int64_t* __restrict__ pk,
                                                        const uint8_t* __restrict__ allowed,
                                                        const unsigned long long* __restrict__ fix_rec,
                                                        const unsigned* __restrict__ sctl,
                                                        const unsigned* __restrict__ fix_start,
                                                        unsigned* __restrict__ fix_cur,
                                                        RecKey<REC == kRecCompact>* __restrict__ keys,
                                                        unsigned* __restrict__ rows) {
  const int64_t total = (int64_t)sctl[1] < kp.fix_cap ? (int64_t)sctl[1] : kp.fix_cap;
  const uint64_t lmask = ((uint64_t)1 << kp.bucket_bits) - 1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t e = fix_rec[i];
    if (e == ~0ULL) continue;  // a Bloom false positive (k_fix_filter)
    const uint64_t u = e >> 32;
    const uint32_t r = (uint32_t)e;
    const int64_t k = pk[r];
    const bool dead = k < 0 || k >= kp.P || (allowed != nullptr && allowed[k] == 0);
    const uint64_t lpk = (u & lmask) << kp.pk_bits;
    const int64_t b = (int64_t)(u >> kp.bucket_bits);
    const unsigned pos = fix_start[b] + atomicAdd(fix_cur + b, 1u);
    if constexpr (REC == kRecCompact)
      keys[pos] = (uint32_t)(dead ? (0x80000000ull | lpk) : (lpk | (uint64_t)k));
    else if constexpr (REC == kRecWide)
      keys[pos] = dead ? ((1ull << 63) | lpk) : (lpk | (uint64_t)k);
    else  // PACKED64: the row in the key, all ones if dead
      keys[pos] = dead ? ~0ull : (((uint64_t)r << kp.row_shift) | lpk | (uint64_t)k);
    if constexpr (REC != kRecP64) rows[pos] = r;
  }
}

// Fix-up step 3a: the buckets a fix-up bucket launch must run.  Only buckets
// holding fix-up rows are listed (blist[1 + i], blist[0] of them): their
// count is at most the unresolved ids', a small fraction of the buckets.  An
// empty bucket's launch work is done here instead: its run-table column
// (range-major, `runs` already offset to the launch's record segment) gets
// empty runs and, in the band's fix-up (prev != NULL), the ids the main
// launch left unresolved stay unresolved -- none of their pairs lies below t2
// -- so they are copied to the second bitmap and list (what k_bucket_bound's
// mark(false) does for an empty bucket).  blist[0] is zeroed by the caller.
// Grid (buckets / kBlock, kFixRunRows): blockIdx.y = 0 lists and marks,
// every y writes its share of the run-table rows (consecutive threads:
// consecutive columns of one row)
constexpr int kFixRunRows = 16;
__global__ void __launch_bounds__(kBlock) k_fix_buckets(KP kp, const unsigned* __restrict__ fix_start,
                                                        unsigned* __restrict__ runs, int64_t run_stride,
                                                        unsigned* __restrict__ blist,
                                                        const unsigned* __restrict__ prev,
                                                        unsigned* __restrict__ bits2,
                                                        unsigned* __restrict__ list2,
                                                        unsigned* __restrict__ sctl2) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= kp.n_buckets) return;
  const bool empty = fix_start[b + 1] == fix_start[b];
  if (runs != nullptr && empty)
    for (int r = blockIdx.y; r <= kp.n_ranges; r += gridDim.y) runs[(int64_t)r * run_stride + b] = 0;
  if (blockIdx.y != 0) return;
  if (!empty) {
    blist[1 + atomicAdd(blist, 1u)] = (unsigned)b;
    return;
  }
  if (prev == nullptr) return;
  const int64_t id0 = b << kp.bucket_bits;  // bucket_bits >= 6: whole u64 words
  for (int64_t w = 0; w < ((int64_t)1 << kp.bucket_bits) / 64; ++w) {
    const int64_t i0 = id0 + 64 * w;
    const uint2 pw = reinterpret_cast<const uint2*>(prev)[i0 >> 6];
    unsigned long long m = (unsigned long long)pw.x | ((unsigned long long)pw.y << 32);
    if (i0 + 64 > kp.U) m &= kp.U > i0 ? (1ULL << (kp.U - i0)) - 1 : 0ULL;  // ids >= U are no ids
    reinterpret_cast<uint2*>(bits2)[i0 >> 6] = make_uint2((unsigned)m, (unsigned)(m >> 32));
    if (m == 0) continue;
    unsigned at = atomicAdd(sctl2, (unsigned)__popcll(m));
    for (; m; m &= m - 1) list2[at++] = (unsigned)(i0 + __ffsll((long long)m) - 1);
  }
}

// PDP_MERGE_RANGES work items.  Range r's records, taken bucket-major, are cut
// into items at bucket boundaries: a new item starts after the bucket that
// holds record position k * kRangeChunk (k >= 1), so every item holds about
// kRangeChunk records or one bucket's run, a Zipf-hot range spreads over many
// workgroups and a cold range is one item.  Range r appends its K_r =
// ceil(total_r / C) items plus a sentinel at a base taken with one atomicAdd
// (ranges land in any order); entry k + 1 holds item k's end.  Entry:
// {r | sentinel << 31, first bucket, first record position within the range}.
// last_ids (the band's second fix-up): its id count; 0 leaves the last
// `last_buckets` buckets (that launch's record segment) empty, so they are
// not read
__global__ void __launch_bounds__(kRangeThreads) k_range_plan(KP kp, const unsigned* __restrict__ runs,
                                                              uint4* __restrict__ items,
                                                              unsigned* __restrict__ n_items,
                                                              const unsigned* __restrict__ last_ids,
                                                              int64_t last_buckets) {
  __shared__ unsigned wsum[kRangeThreads / 64 + 1];
  __shared__ unsigned s_base;
  const int r = blockIdx.x;
  const int64_t stride = kp.n_buckets;  // range-major: row r is contiguous over buckets
  const int64_t n_buckets = last_ids != nullptr && *last_ids == 0u ? kp.n_buckets - last_buckets : kp.n_buckets;
  auto len_of = [&](int64_t b) -> unsigned {
    if (b >= n_buckets) return 0u;
    const unsigned* run = runs + r * stride + b;
    return run[stride] - run[0];
  };
  unsigned total = 0;
  for (int64_t c = 0; c < n_buckets; c += blockDim.x) {
    unsigned t;
    block_excl_scan(len_of(c + threadIdx.x), wsum, &t);
    total += t;
    __syncthreads();
  }
  if (total == 0) return;  // block-uniform: no items
  const unsigned C = (unsigned)kRangeChunk;
  const unsigned K = (total + C - 1) / C;
  if (threadIdx.x == 0) s_base = atomicAdd(n_items, K + 1);
  __syncthreads();
  const unsigned base = s_base;
  if (threadIdx.x == 0) items[base] = make_uint4((unsigned)r, 0u, 0u, 0u);
  if (threadIdx.x == 0 && total % C != 0)
    items[base + K] = make_uint4((unsigned)r | 0x80000000u, (unsigned)n_buckets, total, 0u);
  unsigned carry = 0;
  for (int64_t c = 0; c < n_buckets; c += blockDim.x) {
    const int64_t b = c + threadIdx.x;
    const unsigned len = len_of(b);
    unsigned t;
    const unsigned ex = carry + block_excl_scan(len, wsum, &t);
    if (len > 0) {
      // items k >= 1 with k * C in (ex, ex + len] start after this bucket
      const unsigned e = ex + len;
      for (unsigned k = ex / C + 1; k * C <= e; ++k)
        items[base + k] = make_uint4((unsigned)r | (k == K ? 0x80000000u : 0u), (unsigned)(b + 1), e, 0u);
    }
    carry += t;
    __syncthreads();
  }
}

// PDP_MERGE_RANGES: one workgroup per work item (k_range_plan) sums its
// records of partitions [r*2^11, (r+1)*2^11) in LDS, then adds the partial
// sums with coalesced device atomics (an item of few records adds them
// directly).
// workgroup -> work item: i * p mod n for the prime p = 2^31 - 1 > n (a
// bijection on [0, n)), so the many items of a Zipf-hot range, which k_range_plan
// lists together, run spread over the launch instead of side by side (their
// device atomics go to the same partitions)
__device__ __forceinline__ unsigned item_order(unsigned i, unsigned n) {
  return (unsigned)(((uint64_t)i * 2147483647ull) % (uint64_t)n);
}

__global__ void __launch_bounds__(kReduceThreads) k_range_reduce(KP kp, PairRecords rec, const uint4* __restrict__ items,
                                                               const unsigned* __restrict__ n_items,
                                                               pdp_partition_accumulators acc, unsigned* err) {
  extern __shared__ unsigned long long smem[];
  double* s0 = (double*)smem;               // [kRangeParts] sum
  double* s1 = s0 + kRangeParts;            // normalized sum
  double* s2 = s1 + kRangeParts;            // normalized sum of squares
  unsigned long long* start = (unsigned long long*)(s2 + kRangeParts);  // [kReduceThreads]
  unsigned* pc = (unsigned*)(start + kReduceThreads);  // [kRangeParts] kept pairs
  unsigned* cn = pc + kRangeParts;                    // [kRangeParts] row count
  unsigned* pre = cn + kRangeParts;                   // [kReduceThreads] run prefix
  unsigned* wsum = pre + kReduceThreads;              // block-scan scratch
  const unsigned n_it = *n_items;
  if (blockIdx.x >= n_it) return;  // grid is an upper bound on the item count
  const unsigned iw = item_order(blockIdx.x, n_it);
  const uint4 it = items[iw];
  if (it.x >> 31) return;  // sentinel
  const uint4 nx = items[iw + 1];
  const int r = (int)it.x;
  const int64_t b_lo = it.y, b_hi = nx.y;
  const unsigned item_total = nx.z - it.z;
  if (item_total == 0) return;
  const int flags = kp.clip.flags;
  const bool f0 = flags & (PDP_ACC_SUM | PDP_SUM_PER_PARTITION), f1 = flags & PDP_ACC_NSUM,
             f2 = flags & PDP_ACC_NSUM2, sum_int = flags & PDP_SUM_INT;
  const int64_t p0 = (int64_t)r << kRangeBits;
  const int64_t n_slots = (int64_t)kp.l0 << kp.bucket_bits;
  const bool direct = item_total < kRangeDirect;  // few records: straight into the accumulators
  if (!direct) {
    for (int t = threadIdx.x; t < kRangeParts; t += blockDim.x) {
      pc[t] = 0;
      cn[t] = 0;
      s0[t] = 0.0;
      s1[t] = 0.0;
      s2[t] = 0.0;
    }
  }
  // buckets in batches of one per thread: run starts, block scan, then the
  // batch's records, RR per thread in flight (their run lookups and loads
  // issued before the atomics)
  constexpr int RR = 4;
  for (int64_t bb = b_lo; bb < b_hi; bb += blockDim.x) {
    int64_t nb = b_hi - bb;
    if (nb > blockDim.x) nb = blockDim.x;
    unsigned len = 0;
    if (threadIdx.x < nb) {
      const int64_t b = bb + threadIdx.x;
      const unsigned* run = rec.runs + r * rec.run_stride + b;
      const unsigned s = run[0];
      len = run[rec.run_stride] - s;
      start[threadIdx.x] = (unsigned long long)(b * n_slots + s);
    }
    unsigned total;
    const unsigned ex = block_excl_scan(len, wsum, &total);
    pre[threadIdx.x] = ex;
    __syncthreads();
    for (unsigned i0 = threadIdx.x; i0 < total; i0 += RR * blockDim.x) {
      uint64_t idx[RR];
      bool ok[RR];
#pragma unroll
      for (int u = 0; u < RR; ++u) {
        const unsigned i = i0 + u * blockDim.x;
        ok[u] = i < total;
        int lo = 0, hi = (int)nb - 1;  // last run with pre <= i
        while (ok[u] && lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (pre[mid] <= i) lo = mid;
          else hi = mid - 1;
        }
        idx[u] = ok[u] ? start[lo] + (i - pre[lo]) : 0;
      }
      unsigned long long key[RR];
      double v0[RR], v1[RR], v2[RR];
#pragma unroll
      for (int u = 0; u < RR; ++u) {
        key[u] = ok[u] ? rec.key[idx[u]] : 0ull;
        v0[u] = (ok[u] && f0) ? rec.f0[idx[u]] : 0.0;
        v1[u] = (ok[u] && f1) ? rec.f1[idx[u]] : 0.0;
        v2[u] = (ok[u] && f2) ? rec.f2[idx[u]] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < RR; ++u) {
        if (!ok[u]) continue;
        // a record outside this item's range (malformed workspace): flagged, skipped
        if ((int64_t)(key[u] >> 32) >= kp.P || (key[u] >> 32) - (uint64_t)p0 >= (uint64_t)kRangeParts) {
          atomicOr(err, 1u);
          continue;
        }
        if (direct) {
          const int64_t p = (int64_t)(key[u] >> 32);
          atomicAdd((unsigned long long*)(acc.privacy_id_count + p), 1ull);
          if (acc.count) atomicAdd((unsigned long long*)(acc.count + p), (unsigned long long)(uint32_t)key[u]);
          if (f0) {
            if (sum_int) atomicAdd((unsigned long long*)acc.sum + p, (unsigned long long)__double_as_longlong(v0[u]));
            else unsafeAtomicAdd((double*)acc.sum + p, v0[u]);
          }
          if (f1) unsafeAtomicAdd(acc.normalized_sum + p, v1[u]);
          if (f2) unsafeAtomicAdd(acc.normalized_sum_sq + p, v2[u]);
          continue;
        }
        const int lp = (int)((key[u] >> 32) - (uint64_t)p0);
        atomicAdd(pc + lp, 1u);
        atomicAdd(cn + lp, (unsigned)key[u]);
        if (f0) {
          if (sum_int) atomicAdd((unsigned long long*)(s0 + lp), (unsigned long long)__double_as_longlong(v0[u]));
          else atomicAdd(s0 + lp, v0[u]);
        }
        if (f1) atomicAdd(s1 + lp, v1[u]);
        if (f2) atomicAdd(s2 + lp, v2[u]);
      }
    }
    __syncthreads();  // pre / start / wsum are reused by the next batch
  }
  if (direct) return;
  int64_t plen = kp.P - p0;
  if (plen > kRangeParts) plen = kRangeParts;
  for (int t = threadIdx.x; t < plen; t += blockDim.x) {
    if (pc[t] == 0) continue;
    const int64_t p = p0 + t;
    atomicAdd((unsigned long long*)(acc.privacy_id_count + p), (unsigned long long)pc[t]);
    if (acc.count) atomicAdd((unsigned long long*)(acc.count + p), (unsigned long long)cn[t]);
    if (f0) {
      if (sum_int) atomicAdd((unsigned long long*)acc.sum + p, (unsigned long long)__double_as_longlong(s0[t]));
      else unsafeAtomicAdd((double*)acc.sum + p, s0[t]);
    }
    if (f1) unsafeAtomicAdd(acc.normalized_sum + p, s1[t]);
    if (f2) unsafeAtomicAdd(acc.normalized_sum_sq + p, s2[t]);
  }
}

// ----------------------------------------------------- two-level merge --
// Records of coarse range r (work item from k_range_plan, buckets [b_lo,
// b_hi)) in batches of one bucket per thread; visit(idx, ok) for RR records
// per thread at a time (ok = a real record), then `after()` once per round.
template <typename V, typename A>
__device__ __forceinline__ void item_rounds(const KP& kp, const PairRecords& rec, int r, int64_t b_lo, int64_t b_hi,
                                            unsigned long long* start, unsigned* pre, unsigned* wsum, V&& visit,
                                            A&& after) {
  constexpr int RR = 4;
  const int64_t n_slots = (int64_t)kp.l0 << kp.bucket_bits;
  for (int64_t bb = b_lo; bb < b_hi; bb += blockDim.x) {
    int64_t nb = b_hi - bb;
    if (nb > blockDim.x) nb = blockDim.x;
    unsigned len = 0;
    if (threadIdx.x < nb) {
      const int64_t b = bb + threadIdx.x;
      const unsigned* run = rec.runs + r * rec.run_stride + b;
      const unsigned s0 = run[0];
      len = run[rec.run_stride] - s0;
      start[threadIdx.x] = (unsigned long long)(b * n_slots + s0);
    }
    unsigned total;
    const unsigned ex = block_excl_scan(len, wsum, &total);
    pre[threadIdx.x] = ex;
    __syncthreads();
    for (unsigned i0 = 0; i0 < total; i0 += RR * blockDim.x) {  // block-uniform trip count
      uint64_t idx[RR];
      bool ok[RR];
#pragma unroll
      for (int u = 0; u < RR; ++u) {
        const unsigned i = i0 + threadIdx.x + u * blockDim.x;
        ok[u] = i < total;
        int lo = 0, hi = (int)nb - 1;  // last run with pre <= i
        while (ok[u] && lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (pre[mid] <= i) lo = mid;
          else hi = mid - 1;
        }
        idx[u] = ok[u] ? start[lo] + (i - pre[lo]) : 0;
      }
      visit(idx, ok);
      after();
    }
    __syncthreads();  // pre / start / wsum are reused by the next batch
  }
}

#ifndef PDP_SPLIT_STAGED
#define PDP_SPLIT_STAGED 1
#endif
constexpr int kFinePerCoarseMax = 1 << 13;  // 2^(range_bits - kRangeBits) <= 2^13 (P < 2^32, 256 coarse ranges)

// fine-range totals: per item an LDS histogram of its records' fine ranges,
// added to fine_total with one atomic per touched fine range
__global__ void __launch_bounds__(kSplitThreads) k_split_count(KP kp, PairRecords rec, const uint4* __restrict__ items,
                                                              const unsigned* __restrict__ n_items,
                                                              unsigned* __restrict__ fine_total,
                                                              unsigned* __restrict__ item_hist) {
  __shared__ unsigned long long start[kSplitThreads];
  __shared__ unsigned pre[kSplitThreads], wsum[kSplitThreads / 64 + 1];
  __shared__ unsigned lh[kFinePerCoarseMax];
  if (blockIdx.x >= *n_items) return;
  const uint4 it = items[blockIdx.x];
  if (it.x >> 31) return;  // sentinel
  const uint4 nx = items[blockIdx.x + 1];
  if (nx.z == it.z) return;  // empty item
  const int r = (int)it.x;
  const int F = 1 << (kp.range_bits - kRangeBits);
  const int64_t f0 = (int64_t)r << (kp.range_bits - kRangeBits);
  for (int t = threadIdx.x; t < F; t += blockDim.x) lh[t] = 0;
  __syncthreads();
  item_rounds(kp, rec, r, it.y, nx.y, start, pre, wsum,
              [&](const uint64_t (&idx)[4], const bool (&ok)[4]) {
                // the four loads unconditional (idx = 0 where !ok), so they
                // go out together: under the `ok` branch each waited for the last
                unsigned long long kk[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) kk[u] = rec.key[idx[u]];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  if (!ok[u]) continue;
                  const uint64_t f = (kk[u] >> (32 + kRangeBits)) - (uint64_t)f0;
                  if (f < (uint64_t)F) atomicAdd(lh + (int)f, 1u);  // else malformed: k_split_scatter skips it too
                }
              },
              [] {});
  __syncthreads();
  // the item's histogram for k_split_scatter, which then reserves its slots
  // once per fine range instead of once per round
  for (int t = threadIdx.x; t < F; t += blockDim.x) {
    const bool in = f0 + t < kp.n_fine_ranges;
    item_hist[(int64_t)blockIdx.x * F + t] = in ? lh[t] : 0u;
    if (lh[t] && in) atomicAdd(fine_total + f0 + t, lh[t]);
  }
}

// records of an item -> the fine-range-sorted arrays: the item reserves its
// slots of every fine range once (its histogram from k_split_count, one
// device atomic per touched fine range), then each record takes the next slot
// of its fine range from an LDS cursor (a returning LDS atomic) -- no
// barriers between the batches, so their loads overlap
__global__ void __launch_bounds__(kSplitThreads) k_split_scatter(KP kp, PairRecords rec, PairRecords stg,
                                                                const uint4* __restrict__ items,
                                                                const unsigned* __restrict__ n_items,
                                                                unsigned* __restrict__ fine_cur,
                                                                const unsigned* __restrict__ item_hist) {
  __shared__ unsigned long long start[kSplitThreads];
  __shared__ unsigned pre[kSplitThreads], wsum[kSplitThreads / 64 + 1];
  __shared__ unsigned lcur[kFinePerCoarseMax];
  if (blockIdx.x >= *n_items) return;
  const uint4 it = items[blockIdx.x];
  if (it.x >> 31) return;
  const uint4 nx = items[blockIdx.x + 1];
  if (nx.z == it.z) return;
  const int r = (int)it.x;
  const int F = 1 << (kp.range_bits - kRangeBits);
  const int64_t f0 = (int64_t)r << (kp.range_bits - kRangeBits);
  for (int t = threadIdx.x; t < F; t += blockDim.x) {
    const unsigned c = item_hist[(int64_t)blockIdx.x * F + t];
    lcur[t] = c ? atomicAdd(fine_cur + f0 + t, c) : 0u;
  }
  __syncthreads();
  item_rounds(kp, rec, r, it.y, nx.y, start, pre, wsum,
              [&](const uint64_t (&idx)[4], const bool (&ok)[4]) {
                unsigned long long key[4];
                double v0[4], v1[4], v2[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  key[u] = ok[u] ? rec.key[idx[u]] : 0ull;
                  v0[u] = (ok[u] && stg.f0) ? rec.f0[idx[u]] : 0.0;
                  v1[u] = (ok[u] && stg.f1) ? rec.f1[idx[u]] : 0.0;
                  v2[u] = (ok[u] && stg.f2) ? rec.f2[idx[u]] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  const uint64_t fu = (key[u] >> (32 + kRangeBits)) - (uint64_t)f0;
                  // a malformed record is skipped, as k_split_count leaves it uncounted
                  if (!ok[u] || fu >= (uint64_t)F || f0 + (int64_t)fu >= kp.n_fine_ranges) continue;
                  const uint64_t o = atomicAdd(lcur + (int)fu, 1u);
                  stg.key[o] = key[u];
                  if (stg.f0) stg.f0[o] = v0[u];
                  if (stg.f1) stg.f1[o] = v1[u];
                  if (stg.f2) stg.f2[o] = v2[u];
                }
              },
              [] {});
}

// k_split_scatter for coarse ranges of <= kSplitStageFan fine ranges (C4 /
// C5: 32): each round's records are counting-sorted by fine range in LDS
// first, so a fine range's records leave as one contiguous run (~32 per
// round) instead of one scattered 8-byte store per record and array
constexpr int kSplitStageFan = 256;
constexpr int kSplitStageRows = 4 * kSplitThreads;  // item_rounds' RR records per thread
__global__ void __launch_bounds__(kSplitThreads) k_split_scatter_staged(KP kp, PairRecords rec, PairRecords stg,
                                                                       const uint4* __restrict__ items,
                                                                       const unsigned* __restrict__ n_items,
                                                                       unsigned* __restrict__ fine_cur,
                                                                       const unsigned* __restrict__ item_hist) {
  __shared__ unsigned long long start[kSplitThreads];
  __shared__ unsigned pre[kSplitThreads], wsum[kSplitThreads / 64 + 1];
  __shared__ unsigned lcur[kSplitStageFan], hist[kSplitStageFan], hstart[kSplitStageFan], gbase[kSplitStageFan];
  __shared__ unsigned long long skey[kSplitStageRows];
  __shared__ double sf0[kSplitStageRows], sf1[kSplitStageRows], sf2[kSplitStageRows];
  __shared__ uint8_t sdest[kSplitStageRows];
  if (blockIdx.x >= *n_items) return;
  const uint4 it = items[blockIdx.x];
  if (it.x >> 31) return;
  const uint4 nx = items[blockIdx.x + 1];
  if (nx.z == it.z) return;
  const int r = (int)it.x;
  const int F = 1 << (kp.range_bits - kRangeBits);  // <= kSplitStageFan (host-checked)
  const int64_t f0 = (int64_t)r << (kp.range_bits - kRangeBits);
  for (int t = threadIdx.x; t < F; t += blockDim.x) {
    const unsigned c = item_hist[(int64_t)blockIdx.x * F + t];
    lcur[t] = c ? atomicAdd(fine_cur + f0 + t, c) : 0u;
    hist[t] = 0;
  }
  __syncthreads();
  item_rounds(kp, rec, r, it.y, nx.y, start, pre, wsum,
              [&](const uint64_t (&idx)[4], const bool (&ok)[4]) {
                unsigned long long key[4];
                double v0[4], v1[4], v2[4];
                int fu[4];
                unsigned rk[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  key[u] = ok[u] ? rec.key[idx[u]] : 0ull;
                  v0[u] = (ok[u] && stg.f0) ? rec.f0[idx[u]] : 0.0;
                  v1[u] = (ok[u] && stg.f1) ? rec.f1[idx[u]] : 0.0;
                  v2[u] = (ok[u] && stg.f2) ? rec.f2[idx[u]] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  const uint64_t f = (key[u] >> (32 + kRangeBits)) - (uint64_t)f0;
                  // a malformed record is skipped, as k_split_count leaves it uncounted
                  fu[u] = ok[u] && f < (uint64_t)F && f0 + (int64_t)f < kp.n_fine_ranges ? (int)f : -1;
                  rk[u] = fu[u] >= 0 ? atomicAdd(hist + fu[u], 1u) : 0u;
                }
                __syncthreads();
                if (threadIdx.x < 64) {  // run starts in the stage; the runs' output positions
                  const int lane = threadIdx.x;
                  unsigned carry = 0;
                  for (int b0 = 0; b0 < F; b0 += 64) {
                    const unsigned hv = b0 + lane < F ? hist[b0 + lane] : 0u;
                    unsigned incl = hv;
                    for (int o = 1; o < 64; o <<= 1) {
                      const unsigned up = __shfl_up(incl, o, 64);
                      if (lane >= o) incl += up;
                    }
                    if (b0 + lane < F) {
                      hstart[b0 + lane] = carry + incl - hv;
                      gbase[b0 + lane] = lcur[b0 + lane];
                      lcur[b0 + lane] += hv;
                    }
                    carry += __shfl(incl, 63, 64);
                  }
                }
                __syncthreads();
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  if (fu[u] < 0) continue;
                  const unsigned sl = hstart[fu[u]] + rk[u];
                  skey[sl] = key[u];
                  sf0[sl] = v0[u];
                  sf1[sl] = v1[u];
                  sf2[sl] = v2[u];
                  sdest[sl] = (uint8_t)fu[u];
                }
                __syncthreads();
                const unsigned n = hstart[F - 1] + hist[F - 1];
                for (unsigned i = threadIdx.x; i < n; i += blockDim.x) {
                  const int f = sdest[i];
                  const uint64_t o = (uint64_t)gbase[f] + (i - hstart[f]);
                  stg.key[o] = skey[i];
                  if (stg.f0) stg.f0[o] = sf0[i];
                  if (stg.f1) stg.f1[o] = sf1[i];
                  if (stg.f2) stg.f2[o] = sf2[i];
                }
                __syncthreads();
                for (int t = threadIdx.x; t < F; t += blockDim.x) hist[t] = 0;
                __syncthreads();
              },
              [] {});
}

// fine work items: fine range f's records [start_f, start_f+1) in chunks of
// kRangeChunk, appended at a base taken with one atomic (any order)
__global__ void __launch_bounds__(kBlock) k_fine_plan(KP kp, const unsigned* __restrict__ fine_start,
                                                      uint4* __restrict__ items, unsigned* __restrict__ n_items) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= kp.n_fine_ranges) return;
  const unsigned s0 = fine_start[f], s1 = fine_start[f + 1];
  if (s1 <= s0) return;
  const unsigned C = (unsigned)kRangeChunk;
  const unsigned k = (s1 - s0 + C - 1) / C;
  const unsigned base = atomicAdd(n_items, k);
  for (unsigned j = 0; j < k; ++j) {
    const unsigned a = s0 + j * C;
    items[base + j] = make_uint4((unsigned)f, a, (s1 - a < C ? s1 - a : C), 0u);
  }
}

// one workgroup per fine item: contiguous records of one 2^kRangeBits range,
// summed in LDS (or added directly when few), then coalesced atomics
__global__ void __launch_bounds__(kReduceThreads) k_fine_reduce(KP kp, PairRecords stg, const uint4* __restrict__ items,
                                                              const unsigned* __restrict__ n_items,
                                                              pdp_partition_accumulators acc, unsigned* err) {
  extern __shared__ unsigned long long smem[];
  double* s0 = (double*)smem;
  double* s1 = s0 + kRangeParts;
  double* s2 = s1 + kRangeParts;
  unsigned* pc = (unsigned*)(s2 + kRangeParts);
  unsigned* cn = pc + kRangeParts;
  if (blockIdx.x >= *n_items) return;
  const uint4 it = items[blockIdx.x];
  const int64_t p0 = (int64_t)it.x << kRangeBits;
  const uint64_t a = it.y;
  const unsigned len = it.z;
  const int flags = kp.clip.flags;
  const bool f0 = flags & (PDP_ACC_SUM | PDP_SUM_PER_PARTITION), f1 = flags & PDP_ACC_NSUM,
             f2 = flags & PDP_ACC_NSUM2, sum_int = flags & PDP_SUM_INT;
  const bool direct = len < kRangeDirect;
  if (!direct) {
    for (int t = threadIdx.x; t < kRangeParts; t += blockDim.x) {
      pc[t] = 0;
      cn[t] = 0;
      s0[t] = 0.0;
      s1[t] = 0.0;
      s2[t] = 0.0;
    }
    __syncthreads();
  }
  // RB records per thread loaded together, then summed
  constexpr int RB = 4;
  for (unsigned i0 = threadIdx.x; i0 < len; i0 += RB * blockDim.x) {
    unsigned long long kk[RB];
    double w0[RB], w1[RB], w2[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const unsigned i = i0 + u * blockDim.x;
      const uint64_t o = a + (i < len ? i : 0u);
      kk[u] = i < len ? stg.key[o] : ~0ull;
      w0[u] = (i < len && f0) ? stg.f0[o] : 0.0;
      w1[u] = (i < len && f1) ? stg.f1[o] : 0.0;
      w2[u] = (i < len && f2) ? stg.f2[o] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      if (i0 + u * blockDim.x >= len) continue;
      const unsigned long long key = kk[u];
      if ((int64_t)(key >> 32) >= kp.P || (key >> 32) - (uint64_t)p0 >= (uint64_t)kRangeParts) {  // malformed
        atomicOr(err, 1u);
        continue;
      }
      const double v0 = w0[u], v1 = w1[u], v2 = w2[u];
      if (direct) {
        const int64_t p = (int64_t)(key >> 32);
        atomicAdd((unsigned long long*)(acc.privacy_id_count + p), 1ull);
        if (acc.count) atomicAdd((unsigned long long*)(acc.count + p), (unsigned long long)(uint32_t)key);
        if (f0) {
          if (sum_int) atomicAdd((unsigned long long*)acc.sum + p, (unsigned long long)__double_as_longlong(v0));
          else unsafeAtomicAdd((double*)acc.sum + p, v0);
        }
        if (f1) unsafeAtomicAdd(acc.normalized_sum + p, v1);
        if (f2) unsafeAtomicAdd(acc.normalized_sum_sq + p, v2);
        continue;
      }
      const int lp = (int)((key >> 32) - (uint64_t)p0);
      atomicAdd(pc + lp, 1u);
      atomicAdd(cn + lp, (unsigned)key);
      if (f0) {
        if (sum_int) atomicAdd((unsigned long long*)(s0 + lp), (unsigned long long)__double_as_longlong(v0));
        else atomicAdd(s0 + lp, v0);
      }
      if (f1) atomicAdd(s1 + lp, v1);
      if (f2) atomicAdd(s2 + lp, v2);
    }
  }
  if (direct) return;
  __syncthreads();
  int64_t plen = kp.P - p0;
  if (plen > kRangeParts) plen = kRangeParts;
  for (int t = threadIdx.x; t < plen; t += blockDim.x) {
    if (pc[t] == 0) continue;
    const int64_t p = p0 + t;
    atomicAdd((unsigned long long*)(acc.privacy_id_count + p), (unsigned long long)pc[t]);
    if (acc.count) atomicAdd((unsigned long long*)(acc.count + p), (unsigned long long)cn[t]);
    if (f0) {
      if (sum_int) atomicAdd((unsigned long long*)acc.sum + p, (unsigned long long)__double_as_longlong(s0[t]));
      else unsafeAtomicAdd((double*)acc.sum + p, s0[t]);
    }
    if (f1) unsafeAtomicAdd(acc.normalized_sum + p, s1[t]);
    if (f2) unsafeAtomicAdd(acc.normalized_sum_sq + p, s2[t]);
  }
}
constexpr size_t kFineLds = kRangeParts * (3 * 8 + 2 * 4);

// exclusive scan of u32 counts[0..n) in place, total -> counts[n]
__global__ void __launch_bounds__(kBlock) k_scan_chunks(const unsigned* __restrict__ v, int64_t n,
                                                        unsigned* __restrict__ chunk_sums) {
  __shared__ unsigned red[kBlock / 64];
  const int64_t base = (int64_t)blockIdx.x * kScanChunk + (int64_t)threadIdx.x * kScanItems;
  unsigned s = 0;
#pragma unroll
  for (int t = 0; t < kScanItems; ++t)
    if (base + t < n) s += v[base + t];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += red[w];
    chunk_sums[blockIdx.x] = t;
  }
}

__global__ void __launch_bounds__(kBlock) k_scan_top(unsigned* chunk_sums, int64_t n_chunks) {
  __shared__ unsigned part[kBlock];
  __shared__ unsigned carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < n_chunks; base += kBlock) {
    const int64_t i = base + threadIdx.x;
    const unsigned x = i < n_chunks ? chunk_sums[i] : 0;
    part[threadIdx.x] = x;
    __syncthreads();
    for (int off = 1; off < kBlock; off <<= 1) {
      const unsigned t = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < n_chunks) chunk_sums[i] = carry + part[threadIdx.x] - x;
    __syncthreads();
    if (threadIdx.x == kBlock - 1) carry += part[kBlock - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) chunk_sums[n_chunks] = carry;
}

__global__ void __launch_bounds__(kBlock) k_scan_apply(unsigned* v, int64_t n,
                                                       const unsigned* __restrict__ chunk_sums,
                                                       int64_t n_chunks) {
  __shared__ unsigned part[kBlock];
  const int64_t base = (int64_t)blockIdx.x * kScanChunk + (int64_t)threadIdx.x * kScanItems;
  unsigned loc[kScanItems];
  unsigned s = 0;
#pragma unroll
  for (int t = 0; t < kScanItems; ++t) {
    loc[t] = base + t < n ? v[base + t] : 0;
    s += loc[t];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < kBlock; off <<= 1) {
    const unsigned t = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += t;
    __syncthreads();
  }
  unsigned run = chunk_sums[blockIdx.x] + part[threadIdx.x] - s;
#pragma unroll
  for (int t = 0; t < kScanItems; ++t) {
    if (base + t < n) v[base + t] = run;
    run += loc[t];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) v[n] = chunk_sums[n_chunks];
}

// the same scan in one launch for n <= kScanSmallMax (bucket offsets: C2 1,954
// and C3 4,928 entries), 16 consecutive entries per thread
constexpr int kScanSmallThreads = 1024;
constexpr int64_t kScanSmallMax = (int64_t)kScanSmallThreads * kScanItems;
__global__ void __launch_bounds__(kScanSmallThreads) k_scan_small(unsigned* v, int64_t n) {
  __shared__ unsigned wsum[kScanSmallThreads / 64 + 1];
  const int64_t base = (int64_t)threadIdx.x * kScanItems;
  unsigned loc[kScanItems];
  unsigned s = 0;
#pragma unroll
  for (int t = 0; t < kScanItems; ++t) {
    loc[t] = base + t < n ? v[base + t] : 0u;
    s += loc[t];
  }
  unsigned total;
  unsigned run = block_excl_scan(s, wsum, &total);
#pragma unroll
  for (int t = 0; t < kScanItems; ++t) {
    if (base + t < n) v[base + t] = run;
    run += loc[t];
  }
  if (threadIdx.x == 0) v[n] = total;
}

}  // namespace

int64_t scan_chunk_sums_len(int64_t n) { return (n + kScanChunk - 1) / kScanChunk + 1; }

int scan_u32(unsigned* v, int64_t n, unsigned* chunk_sums, hipStream_t st) {
  const int64_t n_chunks = (n + kScanChunk - 1) / kScanChunk;
  if (n_chunks == 0) return set_error(PDP_E_INVALID, "scan of an empty array");
  if (n <= kScanSmallMax) {
    PDP_PROF_BEGIN("k_scan_small", st);
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(kScanSmallThreads), 0, st, v, n);
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
    return PDP_OK;
  }
  PDP_PROF_BEGIN("k_scan_chunks", st);
  hipLaunchKernelGGL(k_scan_chunks, dim3((unsigned)n_chunks), dim3(kBlock), 0, st, v, n, chunk_sums);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  PDP_PROF_BEGIN("k_scan_top", st);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kBlock), 0, st, chunk_sums, n_chunks);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  PDP_PROF_BEGIN("k_scan_apply", st);
  hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)n_chunks), dim3(kBlock), 0, st, v, n, chunk_sums, n_chunks);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

namespace {

// ---------------------------------------------------------- launchers --
template <int VK, bool KA>
int launch_global_rows(const KP& kp, hipStream_t st, const int64_t* pid, const int64_t* pk, const void* value,
                       const uint8_t* allowed, char* ws, const Ws& w) {
  PDP_PROF_BEGIN("k_pair_rows", st);
  hipLaunchKernelGGL((k_pair_rows<VK, KA>), dim3(grid_for(kp.n)), dim3(kBlock), 0, st, kp, pid, pk, value,
                     allowed, (const unsigned long long*)(ws + w.sketch), (unsigned*)(ws + w.cnt),
                     KA ? nullptr : (unsigned long long*)(ws + w.rows), KA ? (double*)(ws + w.fsum) : nullptr,
                     KA ? (double*)(ws + w.nsum) : nullptr, KA ? (double*)(ws + w.nsum2) : nullptr);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

template <int VK, bool KA>
int launch_global_reduce(const KP& kp, hipStream_t st, const void* value, const char* ws, const Ws& w,
                         const pdp_partition_accumulators& acc) {
  PDP_PROF_BEGIN("k_reduce_pairs", st);
  hipLaunchKernelGGL((k_reduce_pairs<VK, KA>), dim3(grid_for(kp.U * kp.l0)), dim3(kBlock), 0, st, kp, value,
                     (const unsigned long long*)(ws + w.sketch), (const unsigned*)(ws + w.cnt),
                     KA ? nullptr : (const unsigned long long*)(ws + w.rows),
                     KA ? (const double*)(ws + w.fsum) : nullptr, KA ? (const double*)(ws + w.nsum) : nullptr,
                     KA ? (const double*)(ws + w.nsum2) : nullptr, acc);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

// where a bucket launch marks unresolved ids (the main launch: the first
// bitmap / list / counters; the band's fix-up launch: the second ones, only
// ids in `prev`), and where the main launch with the band sends their rows
struct Marks {
  unsigned* bits;
  unsigned* list;
  unsigned* sctl;
  const unsigned* prev;
  unsigned long long* fix_rec;
};

int64_t device_cus();  // compute units of the current device

template <int VK, bool KA>
int launch_bucket_kernel(const KP& kp, const Plan& p, hipStream_t st, const void* keys, const unsigned* rows,
                         const unsigned* offsets, const void* value, const pdp_partition_accumulators& acc,
                         PairRecords rec, char* ws, const Ws& w, const char* name, const Marks& mk,
                         const unsigned* blist = nullptr) {
  const bool ranges = p.merge == PDP_MERGE_RANGES;
  // PACKED: COMPACT records from level 2 on; PACKED_WIDE: WIDE ones; PACKED64: its own
  const int kind = rec_of(p.key_format);
  const void* kern =
      kind == kRecCompact ? (ranges ? (const void*)k_bucket_bound<VK, KA, true, kRecCompact>
                                   : (const void*)k_bucket_bound<VK, KA, false, kRecCompact>)
      : kind == kRecWide  ? (ranges ? (const void*)k_bucket_bound<VK, KA, true, kRecWide>
                                   : (const void*)k_bucket_bound<VK, KA, false, kRecWide>)
                         : (ranges ? (const void*)k_bucket_bound<VK, KA, true, kRecP64>
                                   : (const void*)k_bucket_bound<VK, KA, false, kRecP64>);
  PDP_HIP_CHECK(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds_bytes));
  void* cand_key = ws + w.cand_key;
  unsigned* cand_idx = (unsigned*)(ws + w.cand_idx);
  unsigned* unres_bits = mk.bits;
  unsigned* unres_list = mk.list;
  unsigned* sctl = mk.sctl;
  unsigned* err = (unsigned*)(ws + w.err);
  unsigned long long* fix_rec = mk.fix_rec;
  const unsigned* prev = mk.prev;
  void* args[] = {(void*)&kp,       (void*)&keys,       (void*)&rows,       (void*)&offsets,
                  (void*)&value,    (void*)&acc,        (void*)&rec,        (void*)&cand_key,
                  (void*)&cand_idx, (void*)&unres_bits, (void*)&unres_list, (void*)&sctl,
                  (void*)&err,      (void*)&fix_rec,    (void*)&prev,       (void*)&blist};
  // a listed launch (fix-ups): a persistent grid of one workgroup per CU (the
  // bucket LDS allows no more) looping over the listed buckets
  const int64_t grid = blist != nullptr ? std::min<int64_t>(p.n_buckets, device_cus()) : p.n_buckets;
  PDP_PROF_BEGIN(name, st);
  PDP_HIP_CHECK(hipLaunchKernel(kern, dim3((unsigned)grid), dim3((unsigned)p.bucket_threads), args,
                                (size_t)p.lds_bytes, st));
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

PairRecords pair_records(char* ws, const Ws& w, const Plan& p) {
  PairRecords rec{};
  if (w.runs) {
    rec.runs = (unsigned*)(ws + w.runs);
    rec.run_stride = p.buckets_out;
    rec.key = (unsigned long long*)(ws + w.rec_key);
    rec.f0 = w.rec_f0 ? (double*)(ws + w.rec_f0) : nullptr;
    rec.f1 = w.rec_f1 ? (double*)(ws + w.rec_f1) : nullptr;
    rec.f2 = w.rec_f2 ? (double*)(ws + w.rec_f2) : nullptr;
  }
  return rec;
}

// Sampling (every bucket kernel): the main launch over the level-2 records;
// with the sieve, the fix-up of the unresolved privacy ids (their rows
// gathered, scattered into bucket order, a second launch whose pair records
// follow the main ones: buckets [n_buckets, 2 n_buckets) of `rec`).  The
// rows come from a rescan of the privacy-id column, or with the band from
// the band lists plus the candidate rows the main launch sent; the band's
// fix-up launch marks the ids still short of l0 pairs, whose rows a rescan
// then gathers for a third launch (buckets [2 n_buckets, 3 n_buckets)).
// Every step past the main launch reads its counts on the device, so an
// empty fix-up costs a few near-empty launches and no host round trip.
template <int VK, bool KA>
int launch_buckets(const KP& kp, const Plan& p, hipStream_t st, const int64_t* pid, const int64_t* pk,
                   const uint8_t* allowed, const void* value, const pdp_partition_accumulators& acc, char* ws,
                   const Ws& w) {
  const PairRecords rec = pair_records(ws, w, p);
  unsigned long long* fix_rec = (unsigned long long*)(ws + w.fix_rec);  // level-1 blocks are dead
  Marks m1{w.unres_bits ? (unsigned*)(ws + w.unres_bits) : nullptr,
           w.unres_list ? (unsigned*)(ws + w.unres_list) : nullptr, w.sctl ? (unsigned*)(ws + w.sctl) : nullptr,
           nullptr, p.band ? fix_rec : nullptr};
  int rc = launch_bucket_kernel<VK, KA>(kp, p, st, ws + w.keys2, (const unsigned*)(ws + w.rows2),
                                        (const unsigned*)(ws + w.counts), value, acc, rec, ws, w, "k_bucket_bound", m1);
  if (rc != PDP_OK || !p.sieve) return rc;
  const int kind = rec_of(p.key_format);
  const int64_t n_slots = (int64_t)kp.l0 << kp.bucket_bits;
  // one fix-up: rows listed in fix_rec (sctl[1] of them) -> exact test ->
  // bucket order -> a bucket launch over them into record segment `seg`
  auto fixup = [&](unsigned* bits, unsigned* sctl, unsigned* fix_cnt, unsigned* fix_cur, int seg, const Marks& mk,
                   int mark, const char* name) -> int {
    PDP_PROF_BEGIN("k_fix_filter", st);
    unsigned* blist = (unsigned*)(ws + w.fix_blist);
    hipLaunchKernelGGL(k_fix_filter, dim3(grid_for(kp.n, 1024)), dim3(kBlock), 0, st, kp, (const unsigned*)bits,
                       (const unsigned*)sctl, fix_rec, fix_cnt, (unsigned*)(ws + w.err), blist);
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
    int r = scan_u32(fix_cnt, p.n_buckets, (unsigned*)(ws + w.chunk_sums), st);  // -> starts
    if (r != PDP_OK) return r;
    const unsigned fix_grid = grid_for(kp.n, 2048);
    PDP_PROF_BEGIN("k_fix_scatter", st);
    if (kind == kRecCompact)
      hipLaunchKernelGGL(k_fix_scatter<kRecCompact>, dim3(fix_grid), dim3(kBlock), 0, st, kp, pk, allowed,
                         (const unsigned long long*)fix_rec, (const unsigned*)sctl, (const unsigned*)fix_cnt, fix_cur,
                         (uint32_t*)(ws + w.keys2), (unsigned*)(ws + w.rows2));
    else if (kind == kRecWide)
      hipLaunchKernelGGL(k_fix_scatter<kRecWide>, dim3(fix_grid), dim3(kBlock), 0, st, kp, pk, allowed,
                         (const unsigned long long*)fix_rec, (const unsigned*)sctl, (const unsigned*)fix_cnt, fix_cur,
                         (unsigned long long*)(ws + w.keys2), (unsigned*)(ws + w.rows2));
    else
      hipLaunchKernelGGL(k_fix_scatter<kRecP64>, dim3(fix_grid), dim3(kBlock), 0, st, kp, pk, allowed,
                         (const unsigned long long*)fix_rec, (const unsigned*)sctl, (const unsigned*)fix_cnt, fix_cur,
                         (unsigned long long*)(ws + w.keys2), (unsigned*)(ws + w.rows2));
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
    KP kf = kp;
    kf.sieve_mark = mark;
    kf.sieve_emit = 0;
    PairRecords fr = rec;
    fr.runs += seg * p.n_buckets;  // column offset (range-major table)
    fr.key += seg * p.n_buckets * n_slots;
    if (fr.f0) fr.f0 += seg * p.n_buckets * n_slots;
    if (fr.f1) fr.f1 += seg * p.n_buckets * n_slots;
    if (fr.f2) fr.f2 += seg * p.n_buckets * n_slots;
    // fix-up buckets hold only unresolved ids' rows and most are empty: the
    // buckets with rows are listed (k_fix_buckets, which also writes the
    // empty ones' runs and marks) and run on 512 threads (the kernel sizes its
    // queues from blockDim)
    PDP_PROF_BEGIN("k_fix_buckets", st);
    hipLaunchKernelGGL(k_fix_buckets, dim3(grid_for(p.n_buckets), kFixRunRows), dim3(kBlock), 0, st, kf,
                       (const unsigned*)fix_cnt,
                       p.merge == PDP_MERGE_RANGES ? fr.runs : nullptr, fr.run_stride, blist,
                       mark ? mk.prev : nullptr, mk.bits, mk.list, mk.sctl);
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
    Plan pf = p;
    if (p.merge != PDP_MERGE_RANGES || p.n_ranges <= kBucketThreads / 2) pf.bucket_threads = kBucketThreads / 2;
    return launch_bucket_kernel<VK, KA>(kf, pf, st, ws + w.keys2, (const unsigned*)(ws + w.rows2),
                                        (const unsigned*)fix_cnt, value, acc, fr, ws, w, name, mk, blist);
  };
  auto rescan = [&](const unsigned* bits, const unsigned* list, unsigned* sctl) {
    PDP_PROF_BEGIN("k_sieve_rescan", st);
    if (kp.keys_vec)
      hipLaunchKernelGGL(k_sieve_rescan<true>, dim3(kRescanBlocks), dim3(kRescanThreads), 0, st, kp, pid, bits, list,
                         sctl, fix_rec);
    else
      hipLaunchKernelGGL(k_sieve_rescan<false>, dim3(kRescanBlocks), dim3(kRescanThreads), 0, st, kp, pid, bits, list,
                         sctl, fix_rec);
    PDP_PROF_END(st);
  };
  unsigned* sctl = (unsigned*)(ws + w.sctl);
  unsigned* fix_cnt = (unsigned*)(ws + w.fix_cnt);
  unsigned* fix_cur = (unsigned*)(ws + w.fix_cur);
  const Marks none{m1.bits, m1.list, m1.sctl, nullptr, nullptr};
  if (!p.band) {
    rescan(m1.bits, m1.list, sctl);
    PDP_HIP_CHECK(hipGetLastError());
    return fixup(m1.bits, sctl, fix_cnt, fix_cur, 1, none, 0, "k_bucket_fix");
  }
  // the band: its lists (Bloom filter unless too many ids) -> fix-up launch
  // that marks the ids still unresolved -> their rescan -> a third launch
  PDP_PROF_BEGIN("k_band_scan", st);
  hipLaunchKernelGGL(k_band_scan, dim3(kRescanBlocks), dim3(kRescanThreads), 0, st, kp,
                       (const unsigned long long*)(ws + w.band), (const unsigned*)(ws + w.band_cnt),
                       (const unsigned*)m1.bits, (const unsigned*)m1.list, sctl, fix_rec);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  unsigned* sctl2 = (unsigned*)(ws + w.sctl2);
  const Marks m2{(unsigned*)(ws + w.unres2_bits), (unsigned*)(ws + w.unres2_list), sctl2, m1.bits, nullptr};
  rc = fixup(m1.bits, sctl, fix_cnt, fix_cur, 1, m2, 1, "k_bucket_fix");
  if (rc != PDP_OK) return rc;
  rescan(m2.bits, m2.list, sctl2);
  PDP_HIP_CHECK(hipGetLastError());
  return fixup(m2.bits, sctl2, (unsigned*)(ws + w.fix_cnt2), (unsigned*)(ws + w.fix_cur2), 2, m2, 0, "k_bucket_fix2");
}

// PDP_MERGE_RANGES: the pair records of every bucket (p.buckets_out of them)
// summed per partition
int launch_merge(const KP& kp0, const Plan& p, hipStream_t st, char* ws, const Ws& w,
                 const pdp_partition_accumulators& acc) {
  KP kp = kp0;
  kp.n_buckets = p.buckets_out;
  const PairRecords rec = pair_records(ws, w, p);
  unsigned* err = (unsigned*)(ws + w.err);
  {
    PDP_HIP_CHECK(hipFuncSetAttribute((const void*)k_range_reduce, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kRangeLds));
    uint4* items = (uint4*)(ws + w.rr_items);
    unsigned* n_items = (unsigned*)(ws + w.rr_count);
    PDP_HIP_CHECK(hipMemsetAsync(n_items, 0, 4, st));
    PDP_PROF_BEGIN("k_range_plan", st);
    const unsigned* last_ids = p.band ? (const unsigned*)(ws + w.sctl2) : nullptr;
    hipLaunchKernelGGL(k_range_plan, dim3((unsigned)p.n_ranges), dim3(kRangeThreads), 0, st, kp,
                       (const unsigned*)rec.runs, items, n_items, last_ids, (int64_t)p.n_buckets);
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
    if (!p.two_level) {
      PDP_PROF_BEGIN("k_range_reduce", st);
      hipLaunchKernelGGL(k_range_reduce, dim3((unsigned)p.n_groups), dim3(kReduceThreads), kRangeLds, st, kp, rec,
                         (const uint4*)items, (const unsigned*)n_items, acc, err);
      PDP_PROF_END(st);
      PDP_HIP_CHECK(hipGetLastError());
      return PDP_OK;
    }
    // two-level: coarse items -> fine-range totals -> starts -> records
    // re-sorted by fine range -> fine items -> LDS sums
    unsigned* fine_total = (unsigned*)(ws + w.fine_total);
    unsigned* fine_cur = (unsigned*)(ws + w.fine_cur);
    PairRecords stg{};
    stg.key = (unsigned long long*)(ws + w.stg_key);
    stg.f0 = w.stg_f0 ? (double*)(ws + w.stg_f0) : nullptr;
    stg.f1 = w.stg_f1 ? (double*)(ws + w.stg_f1) : nullptr;
    stg.f2 = w.stg_f2 ? (double*)(ws + w.stg_f2) : nullptr;
    PDP_HIP_CHECK(hipMemsetAsync(fine_total, 0, (uint64_t)(p.n_fine + 1) * 4, st));
    PDP_PROF_BEGIN("k_split_count", st);
    unsigned* item_hist = (unsigned*)(ws + w.item_hist);
    hipLaunchKernelGGL(k_split_count, dim3((unsigned)p.n_groups), dim3(kSplitThreads), 0, st, kp, rec,
                       (const uint4*)items, (const unsigned*)n_items, fine_total, item_hist);
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
    const int rc = scan_u32(fine_total, p.n_fine, (unsigned*)(ws + w.fine_chunks), st);
    if (rc != PDP_OK) return rc;
    PDP_HIP_CHECK(hipMemcpyAsync(fine_cur, fine_total, (uint64_t)p.n_fine * 4, hipMemcpyDeviceToDevice, st));
    PDP_PROF_BEGIN("k_split_scatter", st);
    if ((1 << (kp.range_bits - kRangeBits)) <= kSplitStageFan && PDP_SPLIT_STAGED)
      hipLaunchKernelGGL(k_split_scatter_staged, dim3((unsigned)p.n_groups), dim3(kSplitThreads), 0, st, kp, rec, stg,
                         (const uint4*)items, (const unsigned*)n_items, fine_cur, (const unsigned*)item_hist);
    else
      hipLaunchKernelGGL(k_split_scatter, dim3((unsigned)p.n_groups), dim3(kSplitThreads), 0, st, kp, rec, stg,
                         (const uint4*)items, (const unsigned*)n_items, fine_cur, (const unsigned*)item_hist);
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
    uint4* fitems = (uint4*)(ws + w.fine_items);
    unsigned* n_fitems = (unsigned*)(ws + w.fine_count);
    PDP_HIP_CHECK(hipMemsetAsync(n_fitems, 0, 4, st));
    PDP_PROF_BEGIN("k_fine_plan", st);
    hipLaunchKernelGGL(k_fine_plan, dim3(grid_for(p.n_fine, 1 << 20)), dim3(kBlock), 0, st, kp,
                       (const unsigned*)fine_total, fitems, n_fitems);
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
    PDP_HIP_CHECK(hipFuncSetAttribute((const void*)k_fine_reduce, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kFineLds));
    PDP_PROF_BEGIN("k_fine_reduce", st);
    hipLaunchKernelGGL(k_fine_reduce, dim3((unsigned)p.fine_items), dim3(kReduceThreads), kFineLds, st, kp, stg,
                       (const uint4*)fitems, (const unsigned*)n_fitems, acc, err);
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
  }
  return PDP_OK;
}

template <int FMT>
int launch_scatter(const KP& kp, const Plan& p, hipStream_t st, const int64_t* pid, const int64_t* pk,
                   const uint8_t* allowed, const unsigned* super_off, const unsigned* super_base,
                   const unsigned* bucket_start, const unsigned* gcur, char* ws, const Ws& w, unsigned* err) {
  using K1 = L1Key<FMT>;
  using K2 = L2Key<FMT>;
  constexpr bool ROWS1 = FMT != PDP_KEYS_PACKED;
  const size_t lds = sizeof(StageLds<K1, kSmallDest, ROWS1, kL1Items, kL1Threads>);
  PDP_HIP_CHECK(hipFuncSetAttribute((const void*)k_scatter_l1<FMT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
  PDP_PROF_BEGIN("k_scatter_l1", st);
  hipLaunchKernelGGL(k_scatter_l1<FMT>, dim3((unsigned)p.n_tiles), dim3(kL1Threads), lds, st, kp, pid, pk,
                     allowed, super_off, super_base, (K1*)(ws + w.keys1), ROWS1 ? (unsigned*)(ws + w.rows1) : nullptr,
                     err);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  if (p.super_bits > 0) {
    const int64_t n_grp = (p.n_tiles + kL2GroupTiles - 1) / kL2GroupTiles;
    const bool small = ((int64_t)1 << p.super_bits) <= kSmallDest;
    const void* l2 = small ? (const void*)k_scatter_l2<FMT, kSmallDest> : (const void*)k_scatter_l2<FMT, kMaxDest>;
    const size_t lds2 =
        small ? sizeof(StageLds<K2, kSmallDest, true, kL2Items, kL2Threads>)
              : sizeof(StageLds<K2, kMaxDest, true, kL2Items, kL2Threads>);
    PDP_HIP_CHECK(hipFuncSetAttribute(l2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2));
    const K1* keys1 = (const K1*)(ws + w.keys1);
    const unsigned* rows1 = ROWS1 ? (const unsigned*)(ws + w.rows1) : nullptr;
    K2* keys2 = (K2*)(ws + w.keys2);
    unsigned* rows2 = (unsigned*)(ws + w.rows2);
    void* args[] = {(void*)&kp, (void*)&super_base, (void*)&super_off, (void*)&bucket_start, (void*)&gcur,
                    (void*)&keys1, (void*)&rows1, (void*)&keys2, (void*)&rows2};
    PDP_PROF_BEGIN("k_scatter_l2", st);
    PDP_HIP_CHECK(hipLaunchKernel(l2, dim3((unsigned)n_grp, (unsigned)p.n_supers), dim3(kL2Threads), args, lds2, st));
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
  }
  return PDP_OK;
}

// compute units of the current device (cached per device)
int64_t device_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

// The small control regions a bounding call starts from (error word, the
// tiles' overflow marks, the fix-ups' counters and cursors), set by ONE
// launch instead of a memset each (C3: eight fills of 16 B - 20 KB, ~4 us
// apiece on the stream)
constexpr int kMaxFills = 10;
struct Fills {
  unsigned* p[kMaxFills];
  int64_t n[kMaxFills];  // u32 words
  unsigned v[kMaxFills];
  int k;
};
__global__ void __launch_bounds__(kBlock) k_fill(Fills f) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int j = 0; j < f.k; ++j)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < f.n[j]; i += stride) f.p[j][i] = f.v[j];
}

int launch_fills(const Fills& f, hipStream_t st) {
  int64_t most = 0;
  for (int j = 0; j < f.k; ++j) most = std::max(most, f.n[j]);
  if (most == 0) return PDP_OK;
  PDP_PROF_BEGIN("k_fill", st);
  hipLaunchKernelGGL(k_fill, dim3((unsigned)std::min<int64_t>((most + kBlock - 1) / kBlock, 256)), dim3(kBlock), 0, st, f);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

// tile-local level 1 -> level-2 cursors and bucket starts -> tile-local level 2
template <int FMT>
int launch_local(const KP& kp, const Plan& p, hipStream_t st, const int64_t* pid, const int64_t* pk,
                 const uint8_t* allowed, char* ws, const Ws& w, unsigned* err) {
  using K1 = L1Key<FMT>;
  using K2 = L2Key<FMT>;
  constexpr bool ROWS1 = !kPackedL1<FMT>;
  unsigned* counts_tm = (unsigned*)(ws + w.counts_tm);
  const bool u16 = p.hist_u16 != 0;
  unsigned* counts_tm2 = u16 ? (unsigned*)(ws + w.counts_tm2) : nullptr;
  unsigned* counts = (unsigned*)(ws + w.counts);
  uint16_t* soff = (uint16_t*)(ws + w.soff);
  unsigned* tile_over = (unsigned*)(ws + w.tile_over);  // all ones (k_fill) unless a tile's rows are all one bucket's
  unsigned* sbase = p.sieve ? (unsigned*)(ws + w.sbase) : nullptr;
  K1* keys1 = (K1*)(ws + w.keys1);
  unsigned* rows1 = ROWS1 ? (unsigned*)(ws + w.rows1) : nullptr;
  if constexpr (FMT != PDP_KEYS_WIDE) {
    if (p.sieve) {
      const int th = p.sieve_threads;
      const size_t lds1 = (size_t)sieve_lds(FMT, th, p.n_buckets, u16, p.band != 0);
      auto pick = [&](auto th_tag) -> const void* {
        constexpr int TH = decltype(th_tag)::value;
        return p.band ? (u16 ? (const void*)k_sieve_l1<FMT, true, true, TH> : (const void*)k_sieve_l1<FMT, false, true, TH>)
                      : (u16 ? (const void*)k_sieve_l1<FMT, true, false, TH> : (const void*)k_sieve_l1<FMT, false, false, TH>);
      };
      const void* l1 = th == kSieveThreads2 ? pick(std::integral_constant<int, kSieveThreads2>{})
                                            : pick(std::integral_constant<int, kL1Threads>{});
      PDP_HIP_CHECK(hipFuncSetAttribute(l1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1));
      unsigned long long* band = p.band ? (unsigned long long*)(ws + w.band) : nullptr;
      unsigned* band_cnt = p.band ? (unsigned*)(ws + w.band_cnt) : nullptr;
      void* args1[] = {(void*)&kp,   (void*)&pid,   (void*)&pk,    (void*)&allowed, (void*)&counts_tm,
                       (void*)&counts_tm2, (void*)&soff, (void*)&sbase, (void*)&keys1, (void*)&rows1, (void*)&err,
                       (void*)&band, (void*)&band_cnt, (void*)&tile_over};
      PDP_PROF_BEGIN("k_sieve_l1", st);
      // persistent: as many workgroups as fit at once (one per CU at 1,024
      // threads, two at 512), each looping over its tiles
      const int64_t per_cu = th == kSieveThreads2 ? 2 : 1;
      int64_t grid1 = std::min<int64_t>(p.n_tiles, per_cu * device_cus());
      // test hook: fewer workgroups, so that each loops over several tiles
      // (the cross-tile prefetch and the per-tile LDS reset) at test sizes
      if (test_hooks_enabled()) {
        const char* g = std::getenv("PIPELINEDP_AMD_L1_GRID");
        const long long v = g != nullptr ? std::atoll(g) : 0;
        if (v > 0 && v < grid1) grid1 = v;
      }
      PDP_HIP_CHECK(hipLaunchKernel(l1, dim3((unsigned)grid1), dim3(th), args1, lds1, st));
      PDP_PROF_END(st);
      PDP_HIP_CHECK(hipGetLastError());
    }
  }
  if ((kp.clip.flags & PDP_PROBE_LEVEL1) && p.sieve) return PDP_OK;  // placement probe: level 1 only
  if (test_hooks_enabled() && std::getenv("PIPELINEDP_AMD_STOP_AFTER_L1") != nullptr && p.sieve) return PDP_OK;
  if (!p.sieve) {
    const size_t lds1 = (l1_stage_bytes(FMT) + 7) / 8 * 8 + (size_t)l1_hist_bytes(p.n_buckets, u16);
    const void* l1 = u16 ? (const void*)k_scatter_l1_local<FMT, true> : (const void*)k_scatter_l1_local<FMT, false>;
    PDP_HIP_CHECK(hipFuncSetAttribute(l1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1));
    void* args1[] = {(void*)&kp,         (void*)&pid,  (void*)&pk,    (void*)&allowed, (void*)&counts_tm,
                     (void*)&counts_tm2, (void*)&soff, (void*)&keys1, (void*)&rows1,   (void*)&err,
                     (void*)&tile_over};
    PDP_PROF_BEGIN("k_scatter_l1", st);
    // (one workgroup per tile: a persistent form with the next stage's loads
    // issued early measured the same at C5, 3.04 vs 3.06 ms -- the 2:1
    // read/write mix, not load latency, bounds it; profiles/r04/ab/ab3_l1_local.txt)
    PDP_HIP_CHECK(hipLaunchKernel(l1, dim3((unsigned)p.n_tiles), dim3(kL1Threads), args1, lds1, st));
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
    if (kp.clip.flags & PDP_PROBE_LEVEL1) return PDP_OK;  // placement probe: level 1 only
  }
  const int64_t n_bblk8 = (p.n_buckets + 511) / 512;  // k_gscan_sums<true>: eight buckets per lane
  const int64_t n_sc = (p.n_tiles + kScanChunkTiles - 1) / kScanChunkTiles;
  unsigned* csum = (unsigned*)(ws + w.csum);
  unsigned* gcur = (unsigned*)(ws + w.gcur);
  PDP_PROF_BEGIN("k_gscan_sums", st);
  hipLaunchKernelGGL(k_gscan_sums<true>, dim3((unsigned)n_bblk8, (unsigned)n_sc), dim3(64 * kScanWaves), 0, st,
                     (const unsigned*)counts_tm, (const unsigned*)counts_tm2, (const unsigned*)tile_over, p.n_tiles,
                     p.n_buckets, kp.cstride, csum, gcur);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  PDP_PROF_BEGIN("k_gscan_chunks", st);
  hipLaunchKernelGGL(k_gscan_chunks, dim3(grid_for(p.n_buckets)), dim3(kBlock), 0, st, csum, n_sc, p.n_buckets,
                     counts);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  // level-2 cursors from the group sums (one pass over counts_tm in all)
  PDP_PROF_BEGIN("k_gscan_groups", st);
  hipLaunchKernelGGL(k_gscan_groups, dim3(grid_for(n_sc * p.n_buckets, (int64_t)1 << 30)), dim3(kBlock), 0, st,
                     (const unsigned*)csum, p.n_tiles, p.n_buckets, gcur);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  const int rc = scan_u32(counts, p.n_buckets, (unsigned*)(ws + w.chunk_sums), st);
  if (rc != PDP_OK) return rc;
  const int64_t n_grp = (p.n_tiles + kL2GroupTiles - 1) / kL2GroupTiles;
  const bool small = ((int64_t)1 << p.super_bits) <= kSmallDest;
  const void* l2 = small ? (const void*)k_scatter_l2_local<FMT, kSmallDest>
                         : (const void*)k_scatter_l2_local<FMT, kMaxDest>;
  const size_t lds2 = small ? sizeof(StageLds<K2, kSmallDest, kL2RowArray<FMT>, l2_items<FMT>(), kL2Threads>)
                            : sizeof(StageLds<K2, kMaxDest, kL2RowArray<FMT>, l2_items<FMT>(), kL2Threads>);
  PDP_HIP_CHECK(hipFuncSetAttribute(l2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2));
  const uint16_t* soff_c = soff;
  const unsigned* sbase_c = sbase;
  const unsigned* counts_c = counts;
  const unsigned* gcur_c = gcur;
  const K1* keys1_c = keys1;
  const unsigned* rows1_c = rows1;
  K2* keys2 = (K2*)(ws + w.keys2);
  unsigned* rows2 = (unsigned*)(ws + w.rows2);
  void* args[] = {(void*)&kp,       (void*)&soff_c,  (void*)&sbase_c, (void*)&counts_c, (void*)&gcur_c,
                  (void*)&keys1_c, (void*)&rows1_c, (void*)&keys2,   (void*)&rows2};
  PDP_PROF_BEGIN("k_scatter_l2", st);
  const int64_t n_mgrp = (n_grp + kp.l2_group_mult - 1) / kp.l2_group_mult;  // tile groups per workgroup
  const int64_t n_blk = (n_mgrp + 7) / 8 * 8 * p.n_supers;  // k_scatter_l2_local maps ids to (group, super)
  PDP_HIP_CHECK(hipLaunchKernel(l2, dim3((unsigned)n_blk), dim3(kL2Threads), args, lds2, st));
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

// PDP_DEBUG_CORRUPT_RECORDS (tests only): every level-2 record of bucket 0
// gets the all-ones partition (>= P when P is not a power of two) and every
// record of bucket 1 an out-of-range row, as a malformed workspace would
// carry; the bucket kernel must flag them in the error word, not fault
template <int REC>
__global__ void __launch_bounds__(kBlock) k_debug_corrupt(KP kp, const unsigned* __restrict__ starts,
                                                          RecKey<REC == kRecCompact>* __restrict__ keys,
                                                          unsigned* __restrict__ rows) {
  const int64_t nb = kp.n_buckets < 2 ? kp.n_buckets : 2;
  for (int64_t i = (int64_t)starts[0] + blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)starts[nb];
       i += (int64_t)gridDim.x * blockDim.x) {
    if (i < (int64_t)starts[1]) {
      if (REC != kRecP64 || keys[i] != ~0ull) keys[i] = keys[i] | (RecKey<REC == kRecCompact>)kp.pk_mask;
    } else if constexpr (REC == kRecP64) {  // row field all ones but one: >= n_rows (the plan keeps rows below)
      const uint64_t low = (1ull << kp.row_shift) - 1;
      if (keys[i] != ~0ull) keys[i] = (keys[i] & low) | (((~0ull >> kp.row_shift) - 1) << kp.row_shift);
    } else {
      rows[i] = 0xFFFFFFF0u;
    }
  }
}

int launch_debug_corrupt(const KP& kp, const Plan& p, hipStream_t st, char* ws, const Ws& w) {
  const int rec = rec_of(p.key_format);
  const unsigned* starts = (const unsigned*)(ws + w.counts);
  if (rec == kRecCompact)
    hipLaunchKernelGGL(k_debug_corrupt<kRecCompact>, dim3(64), dim3(kBlock), 0, st, kp, starts,
                       (uint32_t*)(ws + w.keys2), (unsigned*)(ws + w.rows2));
  else if (rec == kRecP64)
    hipLaunchKernelGGL(k_debug_corrupt<kRecP64>, dim3(64), dim3(kBlock), 0, st, kp, starts,
                       (unsigned long long*)(ws + w.keys2), (unsigned*)(ws + w.rows2));
  else
    hipLaunchKernelGGL(k_debug_corrupt<kRecWide>, dim3(64), dim3(kBlock), 0, st, kp, starts,
                       (unsigned long long*)(ws + w.keys2), (unsigned*)(ws + w.rows2));
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}

// histogram pass over the privacy ids -> global offsets -> level 1 -> level 2
// (plans whose tile-local level 1 does not fit)
int launch_offsets(const KP& kp, const Plan& p, hipStream_t st, const int64_t* privacy_id,
                   const int64_t* partition_key, const uint8_t* pk_allowed, char* ws, const Ws& w, unsigned* err) {
  unsigned* counts = (unsigned*)(ws + w.counts);
  unsigned* counts_tm = (unsigned*)(ws + w.counts_tm);
  unsigned* chunk_sums = (unsigned*)(ws + w.chunk_sums);
  const size_t hist_lds = (size_t)p.n_buckets * 4;
  PDP_HIP_CHECK(hipFuncSetAttribute((const void*)k_part_hist, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)hist_lds));
  PDP_PROF_BEGIN("k_part_hist", st);
  unsigned* super_tm = (unsigned*)(ws + w.super_tm);
  unsigned* super_off = (unsigned*)(ws + w.super_off);
  hipLaunchKernelGGL(k_part_hist, dim3((unsigned)p.n_tiles), dim3(kPartThreads), hist_lds, st, kp, privacy_id,
                     counts_tm, super_tm, err);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  PDP_PROF_BEGIN("k_super_scan", st);
  hipLaunchKernelGGL(k_super_scan, dim3((unsigned)p.n_supers), dim3(kBlock), 0, st, kp, super_tm, super_off);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  // rows per bucket (and, with two levels, the level-2 cursors at tile-group starts)
  const int64_t n_bblk = (p.n_buckets + 63) / 64;
  const int64_t n_bblk4 = (p.n_buckets + 255) / 256;
  const int64_t n_sc = (p.n_tiles + kScanChunkTiles - 1) / kScanChunkTiles;
  unsigned* csum = (unsigned*)(ws + w.csum);
  unsigned* gcur = (unsigned*)(ws + w.gcur);
  PDP_PROF_BEGIN("k_gscan_sums", st);
  hipLaunchKernelGGL(k_gscan_sums<false>, dim3((unsigned)n_bblk4, (unsigned)n_sc), dim3(64 * kScanWaves), 0, st,
                     (const unsigned*)counts_tm, (const unsigned*)nullptr, (const unsigned*)nullptr, p.n_tiles,
                     p.n_buckets, kp.cstride, csum, (unsigned*)nullptr);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  PDP_PROF_BEGIN("k_gscan_chunks", st);
  hipLaunchKernelGGL(k_gscan_chunks, dim3(grid_for(p.n_buckets)), dim3(kBlock), 0, st, csum, n_sc, p.n_buckets,
                     counts);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  if (p.super_bits > 0) {
    PDP_PROF_BEGIN("k_gscan_cursors", st);
    hipLaunchKernelGGL(k_gscan_cursors, dim3((unsigned)n_bblk, (unsigned)n_sc), dim3(64 * kScanWaves), 0, st,
                       counts_tm, (const unsigned*)nullptr, p.n_tiles, p.n_buckets, kp.cstride, (const unsigned*)csum,
                       gcur);
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
  }
  const int rc = scan_u32(counts, p.n_buckets, chunk_sums, st);
  if (rc != PDP_OK) return rc;
  unsigned* super_base = (unsigned*)(ws + w.super_base);
  PDP_PROF_BEGIN("k_super_bases", st);
  hipLaunchKernelGGL(k_super_bases, dim3(grid_for(p.n_supers + 1)), dim3(kBlock), 0, st, kp, counts, super_base);
  PDP_PROF_END(st);
  PDP_HIP_CHECK(hipGetLastError());
  if (p.key_format == PDP_KEYS_COMPACT)
    return launch_scatter<PDP_KEYS_COMPACT>(kp, p, st, privacy_id, partition_key, pk_allowed, super_off, super_base,
                                            counts, gcur, ws, w, err);
  if (p.key_format == PDP_KEYS_PACKED)
    return launch_scatter<PDP_KEYS_PACKED>(kp, p, st, privacy_id, partition_key, pk_allowed, super_off, super_base,
                                           counts, gcur, ws, w, err);
  return launch_scatter<PDP_KEYS_WIDE>(kp, p, st, privacy_id, partition_key, pk_allowed, super_off, super_base,
                                       counts, gcur, ws, w, err);
}

template <template <int, bool> class F, typename... A>
int dispatch(int value_kind, bool keep_all, A&&... args) {
  switch (value_kind) {
    case PDP_VALUE_NONE:
      return keep_all ? F<PDP_VALUE_NONE, true>::run(args...) : F<PDP_VALUE_NONE, false>::run(args...);
    case PDP_VALUE_F64:
      return keep_all ? F<PDP_VALUE_F64, true>::run(args...) : F<PDP_VALUE_F64, false>::run(args...);
    default:
      return keep_all ? F<PDP_VALUE_I64, true>::run(args...) : F<PDP_VALUE_I64, false>::run(args...);
  }
}

template <int VK, bool KA>
struct GlobalRows {
  template <typename... A>
  static int run(A&&... a) { return launch_global_rows<VK, KA>(a...); }
};
template <int VK, bool KA>
struct GlobalReduce {
  template <typename... A>
  static int run(A&&... a) { return launch_global_reduce<VK, KA>(a...); }
};
template <int VK, bool KA>
struct Buckets {
  template <typename... A>
  static int run(A&&... a) { return launch_buckets<VK, KA>(a...); }
};

int check_ws(const pdp_bound_config* cfg, const void* workspace, uint64_t workspace_bytes, Plan* p, Ws* w) {
  const int rc = validate(cfg);
  if (rc != PDP_OK) return rc;
  if (pairs_mode(cfg)) {
    if (workspace == nullptr || workspace_bytes < pairs_workspace_bytes(cfg))
      return set_error(PDP_E_WORKSPACE, "workspace too small (see pdp_bound_workspace_bytes)");
    return PDP_OK;
  }
  *p = make_plan(cfg);
  *w = layout(cfg, *p);
  if (workspace == nullptr || workspace_bytes < w->total)
    return set_error(PDP_E_WORKSPACE, "workspace too small (see pdp_bound_workspace_bytes)");
  return PDP_OK;
}

}  // namespace
}  // namespace pdp

using namespace pdp;

extern "C" {

int pdp_bound_plan(const pdp_bound_config* cfg, pdp_bound_plan_info* info) {
  const int rc = validate(cfg);
  if (rc != PDP_OK) return rc;
  if (info == nullptr) return set_error(PDP_E_INVALID, "info is NULL");
  if (pairs_mode(cfg)) {
    *info = pdp_bound_plan_info{};
    info->algorithm = PDP_ALGO_PAIR_TABLE;
    info->pk_bits = bits_for(cfg->n_partitions);
    return PDP_OK;
  }
  const Plan p = make_plan(cfg);
  info->algorithm = p.algorithm;
  info->bucket_bits = p.bucket_bits;
  info->rand_shift = p.rand_shift;
  info->pk_bits = p.pk_bits;
  info->n_buckets = p.algorithm == PDP_ALGO_BUCKETED ? p.n_buckets : 0;
  info->n_tiles = p.n_tiles;
  info->lds_bytes = p.algorithm == PDP_ALGO_BUCKETED ? p.lds_bytes : 0;
  info->merge = p.merge;
  info->n_ranges = p.n_ranges;
  info->range_group = p.range_group;
  info->key_format = p.key_format;
  info->sieve = p.sieve;
  info->band = p.band;
  info->sieve_threads = p.sieve ? p.sieve_threads : 0;
  info->bucket_threads = p.bucket_threads;
  info->hist_u16 = p.algorithm == PDP_ALGO_BUCKETED && p.l1_local ? p.hist_u16 : 0;
  info->reserved = 0;
  return PDP_OK;
}

int pdp_bound_workspace_bytes(const pdp_bound_config* cfg, uint64_t* bytes) {
  const int rc = validate(cfg);
  if (rc != PDP_OK) return rc;
  if (bytes == nullptr) return set_error(PDP_E_INVALID, "bytes is NULL");
  *bytes = pairs_mode(cfg) ? pairs_workspace_bytes(cfg) : layout(cfg, make_plan(cfg)).total;
  return PDP_OK;
}

int pdp_bound_contributions(const pdp_bound_config* cfg, const int64_t* privacy_id, const int64_t* partition_key,
                            const void* value, const uint8_t* pk_allowed, void* workspace,
                            uint64_t workspace_bytes, void* stream) {
  Plan p;
  Ws w;
  int rc = check_ws(cfg, workspace, workspace_bytes, &p, &w);
  if (rc != PDP_OK) return rc;
  if (cfg->n_rows > 0 && (partition_key == nullptr || (privacy_id == nullptr && !cfg->rows_are_units)))
    return set_error(PDP_E_INVALID, "key columns are NULL");
  if (cfg->value_kind != PDP_VALUE_NONE && cfg->n_rows > 0 && value == nullptr)
    return set_error(PDP_E_INVALID, "value column is NULL");
  if (cfg->value_kind == PDP_VALUE_NONE &&
      (cfg->flags & (PDP_ACC_SUM | PDP_ACC_NSUM | PDP_ACC_NSUM2 | PDP_SUM_PER_PARTITION)))
    return set_error(PDP_E_INVALID, "value sums requested without a value column");
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  if (pairs_mode(cfg)) return pairs_bound(cfg, privacy_id, partition_key, value, pk_allowed, ws, st);
  KP kp = make_kp(cfg, p);
  kp.keys_vec = ((((uintptr_t)privacy_id) | ((uintptr_t)partition_key)) & 15) == 0;
  kp.fix_cap = (int64_t)w.fix_cap;
  // test hook: a smaller fix-up list region, so that the guard of its writes
  // and error bit 1 can be exercised (the real region cannot overflow)
  if (test_hooks_enabled()) {
    const char* fc = std::getenv("PIPELINEDP_AMD_FIX_CAP");
    const long long v = fc != nullptr ? std::atoll(fc) : 0;
    if (v > 0 && v < kp.fix_cap) kp.fix_cap = v;
  }
  unsigned* err = (unsigned*)(ws + w.err);
  if (p.algorithm != PDP_ALGO_BUCKETED || cfg->n_rows == 0) PDP_HIP_CHECK(hipMemsetAsync(err, 0, 16, st));
  if (p.algorithm == PDP_ALGO_GLOBAL_SKETCH) {
    const uint64_t slots = (uint64_t)cfg->n_privacy_ids * (uint64_t)cfg->l0;
    PDP_HIP_CHECK(hipMemsetAsync(ws + w.sketch, 0xFF, slots * 8, st));
    PDP_HIP_CHECK(hipMemsetAsync(ws + w.cnt, 0, slots * 4, st));
    if (cfg->linf > 0) PDP_HIP_CHECK(hipMemsetAsync(ws + w.rows, 0xFF, slots * (uint64_t)cfg->linf * 8, st));
    else PDP_HIP_CHECK(hipMemsetAsync(ws + w.fsum, 0, w.total - w.fsum, st));
    if (cfg->n_rows == 0) return PDP_OK;
    PDP_PROF_BEGIN("k_pair_sketch", st);
    hipLaunchKernelGGL(k_pair_sketch, dim3(grid_for(cfg->n_rows)), dim3(kBlock), 0, st, kp, privacy_id,
                       partition_key, pk_allowed, (unsigned long long*)(ws + w.sketch), err);
    PDP_PROF_END(st);
    PDP_HIP_CHECK(hipGetLastError());
    return dispatch<GlobalRows>(cfg->value_kind, cfg->linf == 0, kp, st, privacy_id, partition_key, value,
                                pk_allowed, ws, w);
  }
  // bucketed: histogram -> transpose -> scan -> cursors -> scatter (1 or 2 levels)
  unsigned* counts = (unsigned*)(ws + w.counts);  // rows per bucket -> bucket starts
  if (cfg->n_rows == 0) {
    PDP_HIP_CHECK(hipMemsetAsync(counts, 0, (p.n_buckets + 1) * 4, st));
    return PDP_OK;
  }
  {  // the control regions: one k_fill launch
    Fills f{};
    auto add = [&](uint64_t off, int64_t words, unsigned v) {
      f.p[f.k] = (unsigned*)(ws + off);
      f.n[f.k] = words;
      f.v[f.k] = v;
      ++f.k;
    };
    add(w.err, 4, 0u);
    if (p.l1_local) add(w.tile_over, p.n_tiles, ~0u);
    if (p.merge == PDP_MERGE_RANGES && p.sieve) {
      add(w.sctl, 4, 0u);
      add(w.fix_cnt, p.n_buckets + 1, 0u);
      add(w.fix_cur, p.n_buckets, 0u);
    }
    if (p.merge == PDP_MERGE_RANGES && p.band) {
      add(w.fix_cnt2, p.n_buckets + 1, 0u);
      add(w.fix_cur2, p.n_buckets, 0u);
    }
    const int rcf = launch_fills(f, st);
    if (rcf != PDP_OK) return rcf;
  }
  int rc2 = PDP_OK;
  if (p.l1_local) {
    if (p.key_format == PDP_KEYS_COMPACT)
      rc2 = launch_local<PDP_KEYS_COMPACT>(kp, p, st, privacy_id, partition_key, pk_allowed, ws, w, err);
    else if (p.key_format == PDP_KEYS_PACKED)
      rc2 = launch_local<PDP_KEYS_PACKED>(kp, p, st, privacy_id, partition_key, pk_allowed, ws, w, err);
    else if (p.key_format == PDP_KEYS_PACKED_WIDE)
      rc2 = launch_local<PDP_KEYS_PACKED_WIDE>(kp, p, st, privacy_id, partition_key, pk_allowed, ws, w, err);
    else if (p.key_format == PDP_KEYS_PACKED64)
      rc2 = launch_local<PDP_KEYS_PACKED64>(kp, p, st, privacy_id, partition_key, pk_allowed, ws, w, err);
    else
      rc2 = launch_local<PDP_KEYS_WIDE>(kp, p, st, privacy_id, partition_key, pk_allowed, ws, w, err);
  } else {
    rc2 = launch_offsets(kp, p, st, privacy_id, partition_key, pk_allowed, ws, w, err);
  }
  if (rc2 != PDP_OK) return rc2;
  if (cfg->flags & PDP_PROBE_LEVEL1) return PDP_OK;  // placement probe: level 1 only
  // test hook (tools/l1_probe.py): level 1 alone, timed by the profiler;
  // nothing downstream reads what it wrote
  if (test_hooks_enabled() && std::getenv("PIPELINEDP_AMD_STOP_AFTER_L1") != nullptr) return PDP_OK;
  // PDP_MERGE_ATOMIC: the bucket kernel adds into the accumulators, so it
  // runs in pdp_reduce_partitions; PDP_MERGE_RANGES: all sampling runs here
  if (p.merge != PDP_MERGE_RANGES) return PDP_OK;
  if (cfg->flags & PDP_DEBUG_CORRUPT_RECORDS) {
    rc2 = launch_debug_corrupt(kp, p, st, ws, w);
    if (rc2 != PDP_OK) return rc2;
  }
  const pdp_partition_accumulators none{};
  return dispatch<Buckets>(cfg->value_kind, cfg->linf == 0, kp, p, st, privacy_id, partition_key, pk_allowed, value,
                           none, ws, w);
}

int pdp_bound_stats_read(const pdp_bound_config* cfg, const void* workspace, uint64_t workspace_bytes,
                         pdp_bound_stats* out, void* stream) {
  if (out == nullptr) return set_error(PDP_E_INVALID, "out is NULL");
  Plan p;
  Ws w;
  const int rc = check_ws(cfg, workspace, workspace_bytes, &p, &w);
  if (rc != PDP_OK) return rc;
  *out = pdp_bound_stats{};
  hipStream_t st = (hipStream_t)stream;
  const char* ws = (const char*)workspace;
  PDP_HIP_CHECK(hipMemcpyAsync(&out->error_flags, ws + w.err, 4, hipMemcpyDeviceToHost, st));
  unsigned rows = 0, ctl[2] = {0, 0};
  const bool bucketed = !pairs_mode(cfg) && p.algorithm == PDP_ALGO_BUCKETED && cfg->n_rows > 0;
  if (bucketed) PDP_HIP_CHECK(hipMemcpyAsync(&rows, ws + w.counts + (uint64_t)p.n_buckets * 4, 4, hipMemcpyDeviceToHost, st));
  if (bucketed && p.sieve) PDP_HIP_CHECK(hipMemcpyAsync(ctl, ws + w.sctl, 8, hipMemcpyDeviceToHost, st));
  unsigned ctl2[2] = {0, 0};
  std::vector<unsigned> bc;
  if (bucketed && p.band) {
    PDP_HIP_CHECK(hipMemcpyAsync(ctl2, ws + w.sctl2, 8, hipMemcpyDeviceToHost, st));
    bc.resize((size_t)p.n_tiles);
    PDP_HIP_CHECK(hipMemcpyAsync(bc.data(), ws + w.band_cnt, (size_t)p.n_tiles * 4, hipMemcpyDeviceToHost, st));
  }
  PDP_HIP_CHECK(hipStreamSynchronize(st));
  out->rows_partitioned = rows;
  out->unresolved_ids = ctl[0];
  out->fixup_rows = ctl[1];
  out->sieve = bucketed ? p.sieve : 0;
  out->band = bucketed ? p.band : 0;
  for (unsigned v : bc) out->band_rows += v;
  out->unresolved2_ids = ctl2[0];
  out->fixup2_rows = ctl2[1];
  return PDP_OK;
}

int pdp_bound_stats_async(const pdp_bound_config* cfg, const void* workspace, uint64_t workspace_bytes,
                          uint32_t* out, void* stream) {
  if (out == nullptr) return set_error(PDP_E_INVALID, "out is NULL");
  Plan p;
  Ws w;
  const int rc = check_ws(cfg, workspace, workspace_bytes, &p, &w);
  if (rc != PDP_OK) return rc;
  hipStream_t st = (hipStream_t)stream;
  const char* ws = (const char*)workspace;
  const bool bucketed = !pairs_mode(cfg) && p.algorithm == PDP_ALGO_BUCKETED && cfg->n_rows > 0;
  if (!(bucketed && p.sieve)) out[0] = out[1] = 0;
  if (!(bucketed && p.band)) out[2] = out[3] = 0;
  // sctl2 = sctl + 8 bytes (layout): one copy of both counter pairs
  if (bucketed && p.sieve) PDP_HIP_CHECK(hipMemcpyAsync(out, ws + w.sctl, p.band ? 16 : 8, hipMemcpyDeviceToHost, st));
  return PDP_OK;
}

int pdp_reduce_partitions(const pdp_bound_config* cfg, const void* value, void* workspace,
                          uint64_t workspace_bytes, const pdp_partition_accumulators* acc, void* stream) {
  Plan p;
  Ws w;
  int rc = check_ws(cfg, workspace, workspace_bytes, &p, &w);
  if (rc != PDP_OK) return rc;
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
  if (cfg->value_kind != PDP_VALUE_NONE && cfg->n_rows > 0 && value == nullptr)
    return set_error(PDP_E_INVALID, "value column is NULL");
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  if (pairs_mode(cfg)) return pairs_reduce(cfg, value, ws, *acc, st);
  const KP kp = make_kp(cfg, p);
  if (p.algorithm == PDP_ALGO_GLOBAL_SKETCH)
    return dispatch<GlobalReduce>(cfg->value_kind, cfg->linf == 0, kp, st, value, ws, w, *acc);
  if (cfg->n_rows == 0) return PDP_OK;
  if (p.merge == PDP_MERGE_RANGES) return launch_merge(kp, p, st, ws, w, *acc);
  if (cfg->flags & PDP_DEBUG_CORRUPT_RECORDS) {
    rc = launch_debug_corrupt(kp, p, st, ws, w);
    if (rc != PDP_OK) return rc;
  }
  // PDP_MERGE_ATOMIC (never sieved: the key columns are not needed here)
  return dispatch<Buckets>(cfg->value_kind, cfg->linf == 0, kp, p, st, (const int64_t*)nullptr,
                           (const int64_t*)nullptr, (const uint8_t*)nullptr, value, *acc, ws, w);
}

}  // extern "C"
