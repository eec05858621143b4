/*
 * pipelinedp_amd.h — C ABI of the MI355X (gfx950) DPEngine.aggregate hot path.
 *
 * The reference (lagodiuk/PipelineDP 0.2.2rc2) is pure Python and has no C ABI;
 * every entry point below replaces one stage of the reference's LocalBackend
 * execution of DPEngine._aggregate (pipeline_dp/dp_engine.py:109-187).  The
 * citation above each function names the reference code it replaces.
 *
 * Conventions
 *  - Every function returns 0 on success and a negative PDP_E_* code on
 *    failure; pdp_last_error() returns a thread-local message.  No C++
 *    exception crosses this boundary.
 *  - All array arguments are DEVICE pointers owned by the caller (allocated by
 *    hipMalloc or by torch-ROCm).  `stream` is a hipStream_t passed as void*;
 *    NULL means the legacy default stream.  Nothing here synchronises the
 *    stream or allocates memory, so the sequence can be captured in a hipGraph.
 *  - Keys are dense: privacy ids in [0, n_privacy_ids), partition keys in
 *    [0, n_partitions).  The Python host layer dictionary-encodes other keys.
 */
#ifndef PIPELINEDP_AMD_H_
#define PIPELINEDP_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PDP_ABI_VERSION 14

/* error codes */
#define PDP_OK 0
#define PDP_E_INVALID (-1)   /* bad argument / shape */
#define PDP_E_HIP (-2)       /* a HIP runtime call failed */
#define PDP_E_WORKSPACE (-3) /* workspace too small */
#define PDP_E_UNSUPPORTED (-4)

/* value column kinds */
#define PDP_VALUE_NONE 0
#define PDP_VALUE_F64 1
#define PDP_VALUE_I64 2

/* accumulator flags (pdp_bound_config.flags) */
#define PDP_ACC_SUM 0x1            /* SumCombiner: sum of clipped values */
#define PDP_ACC_NSUM 0x2           /* Mean/Variance: sum of (clip(v) - middle) */
#define PDP_ACC_NSUM2 0x4          /* Variance: sum of (clip(v) - middle)^2 */
#define PDP_SUM_PER_PARTITION 0x8  /* SumCombiner bounds_per_partition: clip(sum_pair) */
#define PDP_SUM_INT 0x10           /* SUM accumulator is int64 (int values, int bounds) */
#define PDP_PROBE_LEVEL1 0x20000000 /* placement probe: pdp_bound_contributions runs the partition pass's
                                      level 1 only (its output is not a bounding result); the API layer
                                      times it on candidate workspaces (executor.py, placement probe) */
#define PDP_DEBUG_CORRUPT_RECORDS 0x40000000 /* tests only: overwrite the level-2 records of buckets 0
                                                and 1 with an out-of-range partition / row before the
                                                bucket kernel, which must flag them in the error word
                                                (pdp_bound_error_flags) instead of reading out of bounds;
                                                rejected (PDP_E_INVALID) unless the environment has
                                                PIPELINEDP_AMD_TEST_HOOKS=1 */

/* One shard's contribution-bounding configuration. */
typedef struct pdp_bound_config {
  int64_t n_rows;        /* rows in this shard (< 2^32) */
  int64_t n_privacy_ids; /* U: privacy ids are dense in [0, U) */
  int64_t n_partitions;  /* P: partition keys are dense in [0, P) (< 2^32) */
  int32_t l0;            /* max_partitions_contributed (1..PDP_MAX_L0); 0 = no
                            cross-partition bounding (LinfSampler / NoOpSampler) */
  int32_t linf;          /* max_contributions_per_partition (1..PDP_MAX_LINF); 0 = keep all rows */
  int32_t value_kind;    /* PDP_VALUE_* */
  int32_t flags;         /* PDP_ACC_* | PDP_SUM_* */
  double min_value;      /* per-value clipping bounds (SUM/MEAN/VARIANCE) */
  double max_value;
  double middle;         /* min_value + (max_value - min_value) / 2 */
  double min_sum;        /* per-partition SUM bounds (PDP_SUM_PER_PARTITION) */
  double max_sum;
  int64_t row_offset;    /* global index of this shard's row 0 (row priorities) */
  uint64_t seed;         /* sampling seed */
  int32_t algorithm;     /* PDP_ALGO_*; every algorithm keeps the same samples */
  int32_t merge;         /* PDP_MERGE_*: how BUCKETED merges kept pairs per partition */
  int32_t max_contributions; /* > 0: SamplingPerPrivacyIdContributionBounder — keep a
                                uniform sample of <= this many rows per privacy id
                                (1..PDP_MAX_CONTRIBUTIONS); needs l0 = linf = 0 */
  int32_t rows_are_units;    /* != 0: contribution_bounds_already_enforced — every row is
                                its own accumulator; privacy_id may be NULL */
  int32_t key_format;        /* PDP_KEYS_*: row record format of the BUCKETED partition passes */
  int32_t sieve;             /* BUCKETED threshold sieve (identical results): 0 = auto, < 0 = off,
                                1..32768 = keep rows whose 32-bit pair hash is below sieve * 2^16
                                (candidate fraction t = sieve / 2^16 <= 1/2) through the partition
                                passes; privacy ids with < l0 candidate pairs are finished from a
                                side band or a re-read of the privacy-id column */
  int32_t sieve_band;        /* with the sieve, the side band: level 1 also lists the rows whose pair
                                hash is in [t, 2t), and the fix-up reads that list; only ids with
                                < l0 pairs below 2t re-read the privacy-id column.  0 = auto (on
                                for t <= 1/4), > 0 = on, < 0 = off (identical results) */
  int32_t sieve_threads;     /* the sieve's level-1 workgroup (identical results): 0 = auto (1024),
                                1024, or 512 (two per CU, when its LDS fits) */
  int32_t bucket_threads;    /* the bucket kernel's workgroup (identical results): 0 = auto (1024),
                                1024, or 512 (buckets of half as many privacy ids, whose LDS lets two
                                workgroups share a CU; needs <= 512 partition ranges) */
} pdp_bound_config;

/* bounds up to int32; above 256 (l0, linf) the pair-table algorithm runs, and
 * a cap above 256 is applied by radix select instead of a sorted sketch */
#define PDP_MAX_L0 2147483647
#define PDP_MAX_LINF 2147483647
#define PDP_MAX_CONTRIBUTIONS 2147483647

/* bounding algorithms (identical results, different data movement) */
#define PDP_ALGO_AUTO 0
#define PDP_ALGO_GLOBAL_SKETCH 1 /* per-pid / per-pair sketches in HBM, device atomics */
#define PDP_ALGO_BUCKETED 2      /* rows partitioned by pid bucket, sketches in LDS */
#define PDP_ALGO_PAIR_TABLE 3    /* device hash table of (pid, pk) pairs: the bounders
                                    without cross-partition sampling (l0 = 0,
                                    max_contributions, rows_are_units), and any bounder
                                    with l0 or linf > 256 (L0 over the table's distinct
                                    pairs, the GLOBAL path's pair keys); chosen by AUTO */

/* row records moved by the BUCKETED partition passes (identical results) */
#define PDP_KEYS_AUTO 0
#define PDP_KEYS_WIDE 1    /* u64 record (bit 63 dead | bucket-within-super and bucket-local
                              pid | partition) + u32 row: 12 B per row and pass; any
                              partition count (pair keys are rebuilt in the bucket kernel) */
#define PDP_KEYS_COMPACT 2 /* u32 (bucket-local pid, partition) + u32 row: 8 B per row and pass;
                              needs super/bucket/partition bits <= 31 (AUTO picks it then) */
#define PDP_KEYS_PACKED 3  /* level 1: one u64 (row within its 65,536-row tile | bucket-local pid |
                              partition), the tile known from the stage block it was read from;
                              level 2 on: the COMPACT pair.  8 B per row and pass: needs bucket +
                              partition bits <= 31 and super + bucket + partition bits <= 47
                              (AUTO's first choice with the tile-local level 1) */
#define PDP_KEYS_PACKED64 5 /* level 1 PACKED (8 B), level 2 on one u64 per record (row << (bucket + partition
                              bits) | bucket-local pid << partition bits | partition; all ones = dead): 8 B
                              per record and pass with no row array, where the bucket + partition bits
                              exceed 31 (C4/C5: P = 1e7) but rows < 2^(64 - bucket - partition bits) - 2 and
                              super + bucket + partition bits <= 47; tile-local level 1 only (AUTO picks it
                              there before PACKED_WIDE) */
#define PDP_KEYS_PACKED_WIDE 4 /* level 1 PACKED (8 B), level 2 on WIDE (u64 key + u32 row):
                              partition counts whose bucket + partition bits exceed 31 (C4/C5:
                              P = 1e7) with super + bucket + partition bits <= 47; tile-local
                              level 1 only (AUTO picks it there before WIDE) */

/* per-partition merge of the kept pairs (BUCKETED; identical sums up to fp
 * summation order) */
#define PDP_MERGE_AUTO 0
#define PDP_MERGE_ATOMIC 1 /* one device atomic per kept pair and field */
#define PDP_MERGE_RANGES 2 /* pair records grouped by partition range, LDS reduction */

typedef struct pdp_bound_plan_info {
  int32_t algorithm;   /* resolved PDP_ALGO_* */
  int32_t bucket_bits; /* privacy ids per bucket = 2^bucket_bits */
  int32_t rand_shift;  /* pair sampling key: random bits [rand_shift, 64) */
  int32_t pk_bits;     /* partition bits [0, pk_bits) */
  int64_t n_buckets;
  int64_t n_tiles;
  int64_t lds_bytes;   /* per bucket workgroup */
  int32_t merge;       /* resolved PDP_MERGE_* (0 for GLOBAL_SKETCH) */
  int32_t n_ranges;    /* PDP_MERGE_RANGES: partition ranges of 2^11 keys */
  int64_t range_group; /* PDP_MERGE_RANGES: records per range-reduce work item */
  int32_t key_format;  /* resolved PDP_KEYS_* (BUCKETED) */
  int32_t sieve;       /* resolved threshold sieve, t = sieve / 2^16 (0 = off) */
  int32_t band;        /* resolved side band, t2 = band / 2^16 (0 = off) */
  int32_t sieve_threads; /* resolved sieve level-1 workgroup size (0 without the sieve) */
  int32_t bucket_threads; /* resolved bucket-kernel workgroup size (BUCKETED) */
  int32_t hist_u16;    /* tile-local level 1 keeps its per-tile bucket counts as u16 halves */
  int32_t reserved;
} pdp_bound_plan_info;

/* Resolves the execution plan for `cfg` (no device work). */
int pdp_bound_plan(const pdp_bound_config* cfg, pdp_bound_plan_info* info);

/* Per-partition accumulators, dense arrays of length n_partitions.  They are
 * the columnar form of CompoundCombiner's accumulator (combiners.py:749-764):
 * row_count, then the children's accumulators. */
typedef struct pdp_partition_accumulators {
  int64_t* privacy_id_count; /* kept (privacy_id, partition) pairs = row_count */
  int64_t* count;            /* CountCombiner / Mean / Variance count */
  void* sum;                 /* SumCombiner: double, or int64 with PDP_SUM_INT */
  double* normalized_sum;    /* Mean/Variance: sum(clip(v) - middle) */
  double* normalized_sum_sq; /* Variance: sum((clip(v) - middle)^2) */
} pdp_partition_accumulators;

int pdp_abi_version(void);
const char* pdp_last_error(void);

/* Bytes of device workspace pdp_bound_contributions needs for `cfg`. */
int pdp_bound_workspace_bytes(const pdp_bound_config* cfg, uint64_t* bytes);

/* Contribution bounding: per privacy id keep at most l0 distinct partitions,
 * per (privacy id, partition) keep at most linf rows, both uniform samples
 * without replacement drawn with counter-based hash priorities.
 * Replaces SamplingCrossAndPerPartitionContributionBounder.bound_contributions
 * (contribution_bounders.py:72-111) and, with linf = 0,
 * SamplingCrossPartitionContributionBounder (contribution_bounders.py:168-201),
 * i.e. LocalBackend.sample_fixed_per_key (pipeline_backend.py:531-547) twice.
 * With l0 = 0: LinfSampler (linf > 0, :204-230) or NoOpSampler (linf = 0,
 * :233-246); with max_contributions: SamplingPerPrivacyIdContributionBounder
 * (:114-156); with rows_are_units: DPEngine's contribution_bounds_already_enforced
 * branch ("Wrap values into accumulators", dp_engine.py:143-150).
 * `pk_allowed` (nullable, u8[n_partitions]) drops rows of non-public
 * partitions first (DPEngine._drop_partitions, dp_engine.py:290-296).
 * The workspace is fully (re)initialised on `stream` by this call.  With
 * PDP_MERGE_RANGES (the default) the whole sampling runs here and leaves
 * per-pair records in the workspace; with PDP_MERGE_ATOMIC the per-bucket
 * sampling runs in pdp_reduce_partitions. */
int pdp_bound_contributions(const pdp_bound_config* cfg, const int64_t* privacy_id,
                            const int64_t* partition_key, const void* value,
                            const uint8_t* pk_allowed, void* workspace,
                            uint64_t workspace_bytes, void* stream);

/* Per-pair accumulators (CompoundCombiner.create_accumulator on the sampled
 * values, combiners.py:749-753) merged per partition key
 * (LocalBackend.combine_accumulators_per_key, pipeline_backend.py:555-565).
 * Must follow pdp_bound_contributions on the same workspace and stream
 * (BUCKETED + PDP_MERGE_ATOMIC: the per-bucket sampling itself runs here).
 * `acc` arrays are ADDED to (zero them first, or chain shards). */
int pdp_reduce_partitions(const pdp_bound_config* cfg, const void* value,
                          void* workspace, uint64_t workspace_bytes,
                          const pdp_partition_accumulators* acc, void* stream);

/* Noise of one additive mechanism, the granularity-snapped secure samplers of
 * Google's differential-privacy library that PyDP wraps (python-dp ~=1.1.5rc4,
 * numerical_mechanisms.LaplaceMechanism / GaussianMechanism, called at
 * dp_computations.py:439-440, 489-491; restated, not vendored):
 *   out = round_to_multiple(x, granularity) + granularity * k,
 * k a two-sided geometric sample P(k) ~ exp(-lambda |k|) (Laplace, found by an
 * integer bisection whose every step is a Bernoulli with the exact conditional
 * mass), or a centred Binomial(n, 1/2) sample drawn by geometric-proposal
 * rejection (Gaussian).  Outputs lie on the power-of-two grid, so their low
 * bits carry no information about x (the floating-point attack of Mironov
 * 2012 on textbook samplers).  The host computes every field
 * (pipelinedp_amd/dp_computations.py: laplace_noise_params /
 * gaussian_noise_params); granularity = 0 means no noise. */
#define PDP_NOISE_LAPLACE 0
#define PDP_NOISE_GAUSSIAN 1

typedef struct pdp_noise_params {
  int32_t kind;        /* PDP_NOISE_* */
  int32_t reserved;
  double scale;        /* Laplace b = sensitivity / eps, Gaussian sigma (reporting) */
  double granularity;  /* output grid, a power of two; 0 = no noise */
  double lambda;       /* Laplace: granularity * eps / (sensitivity + granularity) */
  int64_t step;        /* Gaussian: round(sqrt(2) * sqrt_n + 1), sqrt_n = 2 sigma / granularity */
  double n;            /* Gaussian: sqrt_n^2 (binomial trials) */
  double bound;        /* Gaussian: sqrt_n * sqrt(log(n) / 2), |m| above it has probability 0 */
  double coef;         /* Gaussian: sqrt(2 / pi) / sqrt_n */
  double corr;         /* Gaussian: 1 - 0.4 * (2 log n)^1.5 / sqrt_n */
} pdp_noise_params;

/* partition selection strategies */
#define PDP_SELECT_ALL_NONEMPTY 0 /* keep every partition with row_count > 0 */
#define PDP_SELECT_TRUNCATED_GEOMETRIC 1
#define PDP_SELECT_LAPLACE_THRESHOLDING 2
#define PDP_SELECT_GAUSSIAN_THRESHOLDING 3
#define PDP_SELECT_PUBLIC 4       /* keep partitions with public_mask[p] != 0 */

typedef struct pdp_select_config {
  int64_t n_partitions;          /* length of the slice */
  int64_t partition_offset;      /* global index of slice element 0 (RNG counter) */
  int32_t strategy;              /* PDP_SELECT_* */
  int32_t max_rows_per_privacy_id; /* n = ceil(row_count / this), dp_engine.py:346-353 */
  int32_t pre_threshold;         /* 0 = none */
  int32_t keep_table_len;        /* truncated geometric: keep_prob[0..len-1] */
  const double* keep_prob;       /* device; prob of keep for n; n >= len uses [len-1] */
  pdp_noise_params noise;        /* thresholding strategies: the secure mechanism */
  double threshold;              /* thresholding strategies */
  const uint8_t* public_mask;    /* PDP_SELECT_PUBLIC */
  uint64_t seed;
} pdp_select_config;

/* Private partition selection (dp_engine.py:315-371 → PyDP
 * create_partition_strategy(...).should_keep / noised_value_if_should_keep,
 * partition_selection.py:29-44).  Writes keep[p] in {0,1}; if `noised_count`
 * is non-NULL the thresholding strategies also write the noised
 * privacy-unit count (PostAggregationThresholdingCombiner, combiners.py:353-357). */
int pdp_select_partitions(const pdp_select_config* cfg, const int64_t* row_count,
                          uint8_t* keep, double* noised_count, void* stream);

/* Stream compaction of keep flags into ascending partition indices.
 * `out_count` (device int64[1]) receives the number kept.  Workspace bytes:
 * pdp_compact_workspace_bytes. */
int pdp_compact_workspace_bytes(int64_t n, uint64_t* bytes);
int pdp_compact(const uint8_t* keep, int64_t n, int64_t* out_index, int64_t* out_count,
                void* workspace, uint64_t workspace_bytes, void* stream);

/* metric operations (one per combiner in CompoundCombiner order) */
#define PDP_OP_COUNT 1            /* CountCombiner.compute_metrics, combiners.py:262-263 */
#define PDP_OP_SUM 2              /* SumCombiner, combiners.py:416-417 */
#define PDP_OP_PRIVACY_ID_COUNT 3 /* PrivacyIdCountCombiner, combiners.py:304-305 */
#define PDP_OP_MEAN 4             /* MeanCombiner + MeanMechanism, dp_computations.py:562-568 */
#define PDP_OP_VARIANCE 5         /* VarianceCombiner + compute_dp_var, dp_computations.py:306-365 */
#define PDP_OP_THRESHOLDED_PID 6  /* PostAggregationThresholdingCombiner: copy noised_count */

typedef struct pdp_metric_op {
  int32_t kind;        /* PDP_OP_* */
  int32_t degenerate;  /* VARIANCE: min_value == max_value */
  int32_t out_col[4];  /* output column for each produced metric, -1 = not produced.
                          COUNT/SUM/PID: [0]; MEAN: mean,count,sum;
                          VARIANCE: variance,count,sum,mean */
  pdp_noise_params noise[3]; /* per mechanism: COUNT/SUM/PID: [0]; MEAN: count,nsum;
                                VARIANCE: count,nsum,nsum2 */
  double middle;       /* MEAN/VARIANCE: middle of [min_value, max_value] */
  double min_value;    /* VARIANCE: for min_value == max_value shortcut */
  double sq_min_value; /* VARIANCE: lower end of the squares interval */
} pdp_metric_op;

#define PDP_MAX_OPS 8

/* Noise + compute_metrics for the kept partitions (CompoundCombiner.
 * compute_metrics, combiners.py:766-788).  For each i < n_kept with
 * p = index[i]: out[col * out_stride + i] = metric value (double).
 * `n_kept_dev` (device int64[1], nullable) bounds i on device when n_kept is
 * only known on device; pass n_kept = capacity then. */
int pdp_noise_metrics(const pdp_metric_op* ops, int32_t n_ops, const int64_t* index,
                      int64_t n_kept, const int64_t* n_kept_dev, int64_t partition_offset,
                      const pdp_partition_accumulators* acc, int32_t sum_is_int,
                      const double* noised_count, double* out, int64_t out_stride,
                      uint64_t seed, void* stream);

/* DPEngine.add_dp_noise (dp_engine.py:551-607): out[i] = the secure
 * mechanism `noise` applied to (double)values[i], the `lambda value:
 * create_mechanism().add_noise(float(value))` of its "Add noise" map_values
 * stage (dp_engine.py:595-599) over a column.  values: n int64
 * (PDP_VALUE_I64) or fp64 (PDP_VALUE_F64); `noise` (host pointer): Laplace
 * (l1 = l0*linf, dp_computations.py:430-477) or Gaussian (:480-537).
 * Element i draws from the Philox4x32-10 streams (seed, index_offset + i), so
 * shards of one column noised with their global offsets equal the unsharded
 * result.  values and out: device, 16-byte aligned; out may alias values when
 * both are fp64. */
int pdp_add_noise(const void* values, int32_t value_kind, int64_t n, const pdp_noise_params* noise,
                  uint64_t seed, int64_t index_offset, double* out, void* stream);

/* Device error word: the bounding kernels set bit 0 when a key is outside
 * [0, n_privacy_ids) x [0, n_partitions) (the row is skipped, never read out
 * of bounds), bit 1 if the sieve's fix-up row list would outgrow its
 * workspace region (cannot happen: each list holds distinct rows; checked
 * rather than assumed).  Reads it from the workspace of pdp_bound_contributions
 * (synchronises `stream`). */
int pdp_bound_error_flags(const void* workspace, uint32_t* flags, void* stream);

/* The same error word, copied to `flags` by a copy enqueued on `stream`
 * (nothing synchronises; `flags` should be pinned host memory, valid until the
 * stream has passed the copy).  The library's API layer reads it once the
 * aggregate's result is materialised, so the key check costs no pipeline
 * drain between bounding and the merge. */
int pdp_bound_error_flags_async(const void* workspace, uint32_t* flags, void* stream);

/* What the last pdp_bound_contributions (BUCKETED) moved, read from its
 * workspace (synchronises `stream`): rows that entered the partition passes
 * (every live row, or the sieve's candidates), privacy ids the sieve left
 * unresolved and the rows of those ids its fix-up gathered (from the side
 * band's list and the candidates, or the re-read), the band's rows, the ids
 * the band left unresolved and their re-read rows.  Diagnostics for
 * the measurement (bench.py's algorithmic bytes); zeros for other
 * algorithms. */
typedef struct pdp_bound_stats {
  int64_t rows_partitioned;
  int64_t unresolved_ids;
  int64_t fixup_rows;
  int32_t sieve;        /* resolved sieve (pdp_bound_plan_info.sieve) */
  uint32_t error_flags; /* pdp_bound_error_flags */
  int64_t band_rows;    /* side band: rows level 1 listed (t <= pair hash < t2) */
  int64_t unresolved2_ids; /* side band: ids still unresolved after it (< l0 pairs below t2) */
  int64_t fixup2_rows;  /* their rows, from the re-read of the privacy-id column */
  int32_t band;         /* resolved side band (pdp_bound_plan_info.band) */
  int32_t reserved;
} pdp_bound_stats;

int pdp_bound_stats_read(const pdp_bound_config* cfg, const void* workspace, uint64_t workspace_bytes,
                         pdp_bound_stats* out, void* stream);

/* The sieve's fix-up counters of the last pdp_bound_contributions, copied
 * to out[0..3] = {unresolved ids, fix-up rows, ids the side band left
 * unresolved, their re-read rows} by copies enqueued on `stream` (nothing
 * synchronises; `out` should be pinned host memory, valid until the stream
 * has passed the copies).  Entries a plan has no counter for (no sieve, no
 * band) are set to 0 before returning.  The library's own plan choice uses
 * it: a table whose fix-up needed the whole-column re-read for many ids runs
 * unsieved on the next call (pipelinedp_amd/executor.py, plan feedback). */
int pdp_bound_stats_async(const pdp_bound_config* cfg, const void* workspace, uint64_t workspace_bytes,
                          uint32_t* out, void* stream);

/* Dataset histograms: compute_dataset_histograms
 * (pipeline_dp/dataset_histograms/computing_histograms.py:456-513) over one
 * shard of dense columns privacy_id in [0, n_privacy_ids), partition in
 * [0, n_partitions) and an optional value column (PDP_VALUE_NONE: sums 0).
 * Integer histograms (logarithmic bins, _to_bin_lower_upper_logarithmic
 * :28-47) are indexed densely: index b < 1000 is the bin [b, b + 1); index
 * b >= 1000 is lower = q * 10^e with e = (b - 1000) / 900 + 1,
 * q = (b - 1000) % 900 + 100, upper = lower + 10^e.  Their order in the
 * int_* arrays: L0, L1, LINF, COUNT_PER_PARTITION, PRIVACY_ID_PER_PARTITION
 * (HistogramType, histograms.py:60-76).  Float histograms (LINF_SUM,
 * SUM_PER_PARTITION) have PDP_HIST_SUM_BUCKETS bins over np.linspace(min,
 * max, PDP_HIST_SUM_BUCKETS + 1) (_min_max_lowers :346-370); bin i is
 * [lowers[i], lowers[i + 1]]; float_n_lowers is PDP_HIST_SUM_BUCKETS + 1, 2
 * when min == max (one bin [min, min]), 0 when empty.  A bin with count 0 is
 * absent from the reference's histogram.  All outputs are device arrays the
 * library zeroes and fills on `stream`; out-of-range keys set the error word
 * that pdp_bound_error_flags reads from this workspace.  n_rows < 2^31.
 * Up to ~1e8 rows the (privacy id, partition) pairs are found by hashing rows
 * into buckets, one LDS table per bucket: first by privacy id (every pid's
 * statistics complete in one workgroup), and if a bucket's distinct pairs do
 * not fit (privacy ids with thousands of partitions) by (pid, pk) pair; the
 * call reads one word back after each attempt (it synchronizes `stream`) and
 * redoes the pairs on an HBM pair table if both overflowed (never for hashed
 * real data).  Larger shards use the HBM pair table directly.  value_kind |
 * PDP_HIST_FORCE_PAIR_TABLE (tests) forces the pair table, value_kind |
 * PDP_HIST_FORCE_PAIR_HASH (tests) skips the privacy-id buckets. */
#define PDP_HIST_FORCE_PAIR_TABLE 0x100
#define PDP_HIST_FORCE_PAIR_HASH 0x200
#define PDP_HIST_LOG_BINS 16384
#define PDP_HIST_SUM_BUCKETS 10000
#define PDP_HIST_N_INT 5
#define PDP_HIST_N_FLOAT 2

typedef struct pdp_histogram_bins {
  int64_t* int_count;      /* [PDP_HIST_N_INT][PDP_HIST_LOG_BINS] */
  int64_t* int_sum;        /* [PDP_HIST_N_INT][PDP_HIST_LOG_BINS] */
  int64_t* int_max;        /* [PDP_HIST_N_INT][PDP_HIST_LOG_BINS] */
  int64_t* float_count;    /* [PDP_HIST_N_FLOAT][PDP_HIST_SUM_BUCKETS] */
  double* float_sum;       /* [PDP_HIST_N_FLOAT][PDP_HIST_SUM_BUCKETS] */
  double* float_max;       /* [PDP_HIST_N_FLOAT][PDP_HIST_SUM_BUCKETS] */
  double* float_lowers;    /* [PDP_HIST_N_FLOAT][PDP_HIST_SUM_BUCKETS + 1] */
  int32_t* float_n_lowers; /* [PDP_HIST_N_FLOAT] */
} pdp_histogram_bins;

int pdp_dataset_histograms_workspace_bytes(int64_t n_rows, int64_t n_privacy_ids, int64_t n_partitions,
                                           uint64_t* bytes);
int pdp_dataset_histograms(const int64_t* privacy_id, const int64_t* partition, const void* value,
                           int32_t value_kind, int64_t n_rows, int64_t n_privacy_ids, int64_t n_partitions,
                           const pdp_histogram_bins* out, void* workspace, uint64_t workspace_bytes,
                           void* stream);

/* The same computation in two phases, for rows sharded by privacy id over
 * ranks (pipelinedp_amd.executor.dataset_histograms with torch.distributed).
 * _pairs zeroes `out` and builds the pair table, the per-pid and
 * per-partition statistics and the Linf histogram.  Between the phases the
 * caller reduces across ranks, at the byte offsets that _exchange_offsets
 * gives into the workspace: the per-partition counters (uint64[n_partitions],
 * sum), the per-partition value sums (double[n_partitions], sum), and the
 * pair-sum minimum / maximum (two order-preserving uint64 words at
 * minmax + 0 / + 8: min / max as unsigned integers).  _finish then builds
 * the remaining histograms; partition_histograms = 0 skips the three
 * per-partition histograms (so that one rank owns them).  The bins of all
 * ranks are then merged: counts and sums added, maxima by maximum (only
 * over bins with a count), lowers taken from any rank (pair histogram) or
 * from the rank with partition_histograms = 1. */
int pdp_dataset_histograms_pairs(const int64_t* privacy_id, const int64_t* partition, const void* value,
                                 int32_t value_kind, int64_t n_rows, int64_t n_privacy_ids, int64_t n_partitions,
                                 const pdp_histogram_bins* out, void* workspace, uint64_t workspace_bytes,
                                 void* stream);
int pdp_dataset_histograms_exchange_offsets(int64_t n_rows, int64_t n_privacy_ids, int64_t n_partitions,
                                            uint64_t* pkstat, uint64_t* psum, uint64_t* minmax);
int pdp_dataset_histograms_finish(int32_t value_kind, int64_t n_rows, int64_t n_privacy_ids, int64_t n_partitions,
                                  int32_t partition_histograms, const pdp_histogram_bins* out, void* workspace,
                                  uint64_t workspace_bytes, void* stream);

/* Dataset histograms of pre-aggregated rows:
 * compute_dataset_histograms_on_preaggregated_data
 * (pipeline_dp/dataset_histograms/computing_histograms.py:713-758).  One row
 * per (privacy id, partition) pair, as analysis/pre_aggregation.py:19-58
 * emits them: partition in [0, n_partitions), count (rows of the pair, >= 1),
 * sum (their value sum), n_partitions_of_pid and n_contributions_of_pid (the
 * pair's privacy id's distinct partitions and rows, >= 1); all < 2^62.  The
 * bins are those of pdp_dataset_histograms, except L0 / L1, which weigh every
 * row by 1 / n_partitions_of_pid and count, per distinct value v of
 * n_partitions_of_pid (L0) or n_contributions_of_pid (L1), the weight sum
 * rounded half to even (_compute_weighted_frequency_histogram :81-102): such a
 * bin can hold count 0 with max v, and it is present in the reference's
 * histogram (present bins: count > 0 or max > 0).  Error word bit 0: partition
 * out of range; bit 1: count / n_partitions / n_contributions outside
 * [1, 2^62).  n_rows < 2^31.  The two-phase form mirrors
 * pdp_dataset_histograms_pairs / _finish for rows of one privacy id on one
 * rank: between _rows and _finish the caller sums pk_rows and pk_count
 * (uint64[n_partitions]) and psum (double[n_partitions]) over ranks and takes
 * min / max of the two minmax words, at the offsets _exchange_offsets gives.
 * The L0 / L1 weight sums must be global before they are rounded: between
 * _rows and _finish the caller sums the dense weights (double[2][1000] at
 * _weight_offsets' wsmall: values below 1000) over ranks and keeps them on one
 * rank (zeros elsewhere), takes every live entry of the weight table
 * ({uint64 key, double weight}[wtab_slots] at wtab, key 0 = empty) out of it
 * (zeroing the table), sums the entries per key over ranks, and after _finish
 * adds each key's global sum once with pdp_dataset_histograms_weight_bins. */
int pdp_dataset_histograms_preaggregated_workspace_bytes(int64_t n_rows, int64_t n_partitions, uint64_t* bytes);
int pdp_dataset_histograms_preaggregated(const int64_t* partition, const int64_t* count, const double* sum,
                                         const int64_t* n_partitions_of_pid, const int64_t* n_contributions_of_pid,
                                         int64_t n_rows, int64_t n_partitions, const pdp_histogram_bins* out,
                                         void* workspace, uint64_t workspace_bytes, void* stream);
int pdp_dataset_histograms_preaggregated_rows(const int64_t* partition, const int64_t* count, const double* sum,
                                              const int64_t* n_partitions_of_pid,
                                              const int64_t* n_contributions_of_pid, int64_t n_rows,
                                              int64_t n_partitions, const pdp_histogram_bins* out, void* workspace,
                                              uint64_t workspace_bytes, void* stream);
int pdp_dataset_histograms_preaggregated_exchange_offsets(int64_t n_rows, int64_t n_partitions, uint64_t* pk_rows,
                                                          uint64_t* pk_count, uint64_t* psum, uint64_t* minmax);
int pdp_dataset_histograms_preaggregated_weight_offsets(int64_t n_rows, int64_t n_partitions, uint64_t* wsmall,
                                                        uint64_t* wtab, uint64_t* wtab_slots);
int pdp_dataset_histograms_preaggregated_finish(const double* sum, int64_t n_rows, int64_t n_partitions,
                                                int32_t partition_histograms, const pdp_histogram_bins* out,
                                                void* workspace, uint64_t workspace_bytes, void* stream);
/* Adds n weight-table entries (keys as in the table above: value * 2 +
 * histogram + 1, histogram 0 = L0, 1 = L1; key 0 skipped) to the integer bins:
 * int(round(weight)) elements of the value, half to even; the bin's max is the
 * value even at count 0.  Device arrays; asynchronous on `stream`. */
int pdp_dataset_histograms_weight_bins(const uint64_t* keys, const double* weights, int64_t n,
                                       const pdp_histogram_bins* out, void* stream);

/* Multi-GPU sharding check (ColumnarBackend privacy_id_sharding="verify"):
 * counts the ids whose owner rank is not `rank`, where owner(id) =
 * mix(id) mod world with mix(z) = (z ^ (z >> 31)) * 0x9E3779B97F4A7C15, then
 * z ^ (z >> 29) (int64, arithmetic shifts, wrapping multiply; the value
 * taken non-negative mod world) — pipelinedp_amd.parallel.owner_of.  When no
 * rank holds an id it does not own, no id can be on two ranks, so the
 * library skips the exchange of distinct ids (contribution_bounders.py:62-111
 * bounds per privacy id over the whole dataset).  ids: device int64[n];
 * *mismatches: device uint32, overwritten (a saturating count: 2^32 - 1 at most, never wraps to 0). */
int pdp_owner_mismatches(const int64_t* ids, int64_t n, int32_t world, int32_t rank, uint32_t* mismatches,
                         void* stream);

/* Kernel profiler: when enabled, every kernel launch of this library is
 * bracketed by HIP events recorded on its launch stream.  enable(1) clears
 * previous records; report() synchronises on them and returns, per kernel
 * name (first-launch order), the summed milliseconds and the launch count.
 * `names` is max_entries * PDP_PROF_NAME_LEN bytes. */
#define PDP_PROF_NAME_LEN 64
int pdp_profiler_enable(int enable);
int pdp_profiler_report(int32_t max_entries, char* names, double* total_ms, int64_t* calls,
                        int32_t* n_entries);

#ifdef __cplusplus
}
#endif

#endif /* PIPELINEDP_AMD_H_ */
