/*
 * skyline_hip.h — C ABI of libskyline_hip.so, the MI355X-native engine behind the
 * reference's Flink skyline operators (Asterinos1/Flink-Skyline-QoS).
 *
 * Plain C types only (JNI / Panama-FFM / ctypes friendly).  Every entry point
 * returns an int status: SKY_OK (0) or a negative SKY_E_* code; the message of
 * the last failure on the calling thread is in sky_last_error().  No C++
 * exception crosses this boundary.
 *
 * Threading: calls on one handle must not run concurrently (Flink's mailbox
 * model gives one thread per operator subtask); distinct handles may be used
 * from distinct threads.  Each entry point binds its context's device.
 *
 * Buffers: `*_dev` entry points take device pointers (HBM-resident inputs and
 * outputs, for callers that already hold device memory); the others take
 * caller-owned host buffers that are only read/written during the call.
 *
 * Reference interfaces replaced (paths relative to /root/reference/java/org.main/):
 *   sky_partition_keys   <- PartitioningLogic.SkylinePartitioner.getKey
 *                           (FlinkSkyline.java:675; Dim :707-712, Grid :774-789, Angle :827-875)
 *   sky_part_*           <- SkylineLocalProcessor keyed state + processBuffer BNL
 *                           (FlinkSkyline.java:214-445; BNL :417-444; snapshot :387-392)
 *   sky_global_merge     <- GlobalSkylineAggregator.processElement merge (FlinkSkyline.java:515-569)
 *   sky_global_stats     <- optimality integers (FlinkSkyline.java:593-608)
 *   sky_query[_dev]      <- the whole keyBy -> local -> global path for a trigger that arrives
 *                           after the last tuple (FlinkSkyline.java:138-174)
 *   dominance            <- ServiceTuple.dominates (ServiceTuple.java:67-77)
 *   sky_parse_csv[_dev]  <- ServiceTuple.fromString (ServiceTuple.java:89-104) mapped over the raw
 *                           Kafka values + .filter(Objects::nonNull) (FlinkSkyline.java:103-104)
 *                           + Long.parseLong(point.id) (FlinkSkyline.java:276)
 *   sky_format_csv_dev   <- the producers' "id,v1,...,vD" payload (python/unified_producer.py:174)
 */
#ifndef SKYLINE_HIP_H
#define SKYLINE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define SKY_OK          0
#define SKY_E_ARG      -1   /* invalid argument (null pointer, dims out of range, ...) */
#define SKY_E_HIP      -2   /* HIP runtime failure (message in sky_last_error) */
#define SKY_E_CAPACITY -3   /* output buffer too small; *n_out holds the required count */
#define SKY_E_NAN      -4   /* a value is NaN: the reference BNL result is order-dependent for NaN */
#define SKY_E_NOMEM    -5   /* device allocation failed */
#define SKY_E_NOLIB    -6   /* no HIP device / code object for gfx950 */
#define SKY_E_RETRY    -7   /* multi-GPU step: some rank's planned local phase missed, run the step again */

/* partitioners (FlinkSkyline.java:112-134, flag --algo) */
#define SKY_ALGO_DIM    0   /* "mr-dim"   */
#define SKY_ALGO_GRID   1   /* "mr-grid"  */
#define SKY_ALGO_ANGLE  2   /* "mr-angle" (the reference default) */

/* query semantics */
#define SKY_SEM_REFERENCE 0 /* only keys 0..P-1 are queried (FlinkSkyline.java:152-154): MR-Grid
                               tuples with key >= P never reach the global merge */
#define SKY_SEM_COMPLETE  1 /* every key in [0, 2^D) of MR-Grid is queried (D <= 8) */

/* synthetic streams (restating python/unified_producer.py:50-123 with a counter RNG) */
#define SKY_DIST_UNIFORM    0
#define SKY_DIST_CORRELATED 1
#define SKY_DIST_ANTI       2   /* reference anti-correlated formula */
#define SKY_DIST_STD_ANTI   3   /* Borzsonyi-style anti-correlated band (extension, labelled) */
#define SKY_DIST_MIXED      4   /* 65536-tuple blocks cycling 0,1,2 (extension for config C5) */

#define SKY_MAX_DIMS       16
#define SKY_MAX_PARTITIONS 256

typedef struct sky_ctx sky_ctx;
typedef struct sky_part sky_part;
typedef struct sky_stream sky_stream;

/* ---- context ------------------------------------------------------------ */
/* devices/ndev: HIP device ordinals; one process drives one device (ndev == 1),
 * multi-GPU runs one process per GPU (see the sky_dist_* step).
 * dims in [1,16]; num_partitions P in [1,256] (= 2 x Flink parallelism, :76);
 * domain_max = --domain (default 1000.0, :71). */
int sky_ctx_create(const int *devices, int ndev, int dims, int num_partitions, int algo,
                   double domain_max, sky_ctx **out);
int sky_ctx_destroy(sky_ctx *ctx);
int sky_ctx_set_semantics(sky_ctx *ctx, int semantics);
/* MR-Grid dominance filter (FlinkSkyline.java:716-733, commented out in the reference, with
 * its `processedData` hook at :107): on = drop every tuple whose values are all >= maxVal/2
 * before keyBy (its key becomes -1).  Such a tuple is dominated whenever the stream holds a
 * tuple with every value < maxVal/2, so the skyline is unchanged then.  Off by default. */
int sky_ctx_set_grid_filter(sky_ctx *ctx, int on);
/* Use a caller-owned hipStream_t (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL returns to the context's own stream. */
int sky_ctx_set_stream(sky_ctx *ctx, void *hip_stream);
int sky_ctx_sync(sky_ctx *ctx);
/* the shape a handle was created with (any pointer may be NULL): FFI shims size arrays by it */
int sky_ctx_info(sky_ctx *ctx, int32_t *dims, int32_t *num_partitions, int32_t *algo);
int sky_part_info(sky_part *part, int32_t *key, int32_t *dims);
int sky_stream_info(sky_stream *s, int32_t *dims);
/* One-time warm-up: a small device-generated query down each pipeline branch, so that no later
 * query pays for first kernel launches / first allocations inside its latency.  Optional; call
 * once after sky_ctx_create (e.g. in the operator's open()), never on a timed path. */
int sky_ctx_warmup(sky_ctx *ctx);
/* cross-stream ordering for *_dev callers that produce / consume the device buffers on
 * their own HIP stream (e.g. a framework's current stream): wait_stream makes the
 * context's later work wait for everything already enqueued on `hip_stream`;
 * signal_stream makes `hip_stream`'s later work wait for everything already enqueued
 * on the context.  GPU-side only (events), no host synchronisation. */
int sky_ctx_wait_stream(sky_ctx *ctx, void *hip_stream);
int sky_ctx_signal_stream(sky_ctx *ctx, void *hip_stream);
const char *sky_last_error(void);
const char *sky_version(void);
/* HIP devices this process sees (*n_out = 0 without a GPU, not an error), and the device a
 * Flink subtask's context goes on: subtask % ndev.  The reference runs `parallelism` subtasks
 * over 2p keys (FlinkSkyline.java:66,76,138); HipSkylineOperators creates each subtask's
 * context on sky_device_for_subtask(getIndexOfThisSubtask(), sky_device_count()). */
int sky_device_count(int32_t *n_out);
int sky_device_for_subtask(int32_t subtask, int32_t ndev, int32_t *dev_out);

/* ---- partitioners --------------------------------------------------------- */
/* keys_out[i] = getKey(tuple i), bit-exact with Java (fdlibm atan2, no FMA);
 * MR-Grid keys are the unclamped mask in [0, 2^D). values: n x dims row-major. */
int sky_partition_keys(sky_ctx *ctx, const double *values, int64_t n, int32_t *keys_out);
int sky_partition_keys_dev(sky_ctx *ctx, const double *d_values, int64_t n, int32_t *d_keys_out);

/* ---- local operator state (one per Flink key) ----------------------------- */
int sky_part_open(sky_ctx *ctx, int32_t key, sky_part **out);
int sky_part_close(sky_part *part);
/* S <- SKY(S u batch)  (processBuffer, FlinkSkyline.java:417-444); duplicates kept.
 * Asynchronous: the batch is copied before the call returns and applied on the device without
 * a host read; size / snapshot wait for every earlier insert.  A batch holding a NaN is
 * rejected before anything is launched (SKY_E_NAN) and the state is unchanged. */
int sky_part_insert(sky_part *part, const int64_t *ids, const double *values, int64_t n);
/* the same for the batches of several keys (parts of ONE context) in one launch set: the
 * full buffers of a subtask's keys flushed together.  A NaN anywhere rejects the whole call. */
int sky_parts_insert(int nparts, sky_part *const *parts, const int64_t *const *ids,
                     const double *const *values, const int64_t *counts);
int sky_part_size(sky_part *part, int64_t *n_out);
/* copy of the current local skyline (ids + values), order = ascending insertion order;
 * SKY_E_CAPACITY with *n_out set if cap is too small */
int sky_part_snapshot(sky_part *part, int64_t *ids_out, double *values_out, int64_t cap,
                      int64_t *n_out);
/* the local skyline as the state holds it: T tuples (ids_out[i], rep_out[i] = index of its
 * vector) in insertion order, and R distinct vectors (reps_out: R x dims row-major, and
 * rep_count_out[r] = tuples on vector r).  What LocalProcessor.processQuery ships to the
 * aggregator: on the reference streams key 0's 4.4M skyline tuples are ONE vector, so the
 * message is its ids and rep indices (12 bytes per tuple) instead of 8 + 8 dims.
 * sky_part_sizes gives T and R; SKY_E_CAPACITY with both counts set if a cap is too small. */
int sky_part_sizes(sky_part *part, int64_t *n_tuples, int64_t *n_reps);
int sky_part_snapshot_reps(sky_part *part, int64_t *ids_out, int32_t *rep_out, int64_t cap,
                           double *reps_out, int32_t *rep_count_out, int64_t rep_cap,
                           int64_t *n_out, int64_t *nrep_out);

/* ---- global merge ---------------------------------------------------------- */
/* G = SKY(u_k list_k) for the nparts local skylines; origin_out[j] = part_ids[k] of
 * the list that supplied ids_out[j].  Output order: list order, then position. */
int sky_global_merge(sky_ctx *ctx, int nparts, const int32_t *part_ids,
                     const int64_t *const *ids, const double *const *values,
                     const int64_t *counts, int64_t *ids_out, int32_t *origin_out,
                     int64_t cap, int64_t *n_out);
/* the same merge over the keys' device-resident states (no snapshot through host memory): the
 * result, its order (part order, then insertion order), origin_out (= part_ids[k], or k when
 * part_ids is NULL) and sky_global_stats equal sky_global_merge over the parts' snapshots.
 * For an aggregator co-located with the local processors (one process drives the device). */
int sky_parts_global_merge(sky_ctx *ctx, int nparts, sky_part *const *parts, const int32_t *part_ids,
                           int64_t *ids_out, int32_t *origin_out, int64_t cap, int64_t *n_out);
/* sky_global_merge over lists shipped as sky_part_snapshot_reps output (list g: counts[g]
 * tuples ids[g] / rep_idx[g], nreps[g] vectors reps[g] with rep_counts[g] tuples each): same
 * result, order, origins and sky_global_stats as sky_global_merge over the expanded lists.
 * A rep index outside [0, nreps[g]) is SKY_E_ARG. */
int sky_global_merge_reps(sky_ctx *ctx, int nlists, const int32_t *part_ids, const int64_t *const *ids,
                          const int32_t *const *rep_idx, const int64_t *counts, const double *const *reps,
                          const int32_t *const *rep_counts, const int64_t *nreps, int64_t *ids_out,
                          int32_t *origin_out, int64_t cap, int64_t *n_out);
/* integers behind the optimality metric of the last merge / query:
 * local_sizes[k] = |L_k|, survivors[k] = |G n L_k| for k < K
 * (K = P, or max(P, 2^D) for MR-Grid with SKY_SEM_COMPLETE). */
int sky_global_stats(sky_ctx *ctx, int64_t *local_sizes, int64_t *survivors, int32_t *k_out);
/* records job-wide integers (e.g. integers a caller merged itself) so that sky_global_stats
 * returns them until the next query (sky_dist_finish records the all-reduced shares itself) */
int sky_global_stats_set(sky_ctx *ctx, int32_t k, const int64_t *local_sizes, const int64_t *survivors);

/* ---- fused whole-stream query --------------------------------------------- */
/* keyBy -> per-key local skylines -> global merge, the trigger arriving after
 * the last tuple.  ids_out/origin_out: the global skyline in stream order.
 * On any error (e.g. SKY_E_NAN found at the final verification of a planned query) the
 * output buffers hold unspecified data; only *n_out of a SKY_E_CAPACITY return is defined. */
int sky_query(sky_ctx *ctx, const int64_t *ids, const double *values, int64_t n,
              int64_t *ids_out, int32_t *origin_out, int64_t cap, int64_t *n_out);
int sky_query_dev(sky_ctx *ctx, const int64_t *d_ids, const double *d_values, int64_t n,
                  int64_t *d_ids_out, int32_t *d_origin_out, int64_t cap, int64_t *n_out);

/* ---- continuous queries over a stream ---- */
/* A device-resident stream state behind the operators' continuous queries.
 * window == 0: the reference's landmark window (every tuple since the start counts,
 *   FlinkSkyline.java:265-316 state + :417-444 BNL).  Only the tuples of the last
 *   query's local skylines stay resident (SKY(L_k ∪ new) = SKY(all of key k)), plus
 *   the tuples appended since; each query re-runs keys -> local -> global over them.
 * window == W > 0: count-based sliding window over the last W appended tuples
 *   (an extension: the reference has no window; expiry needs the non-skyline
 *   tuples, so all W stay resident and each query runs over the window).
 * Results (ids in arrival order, origin keys) and sky_global_stats match a whole-
 * stream sky_query over the same tuples (landmark) / the window's tuples (sliding). */
int sky_stream_create(sky_ctx *ctx, int64_t window, sky_stream **out);
int sky_stream_destroy(sky_stream *s);
int sky_stream_append(sky_stream *s, const int64_t *ids, const double *values, int64_t n);
int sky_stream_append_dev(sky_stream *s, const int64_t *d_ids, const double *d_values, int64_t n);
/* pre-sizes the device state for up to `tuples` resident tuples plus one appended batch (the
 * resident buffers, the query's working buffers, the host-view output), so that no trigger
 * pays a device allocation (each regrowth synchronises the device).  Optional; call before
 * the stream starts (e.g. in the operator's open()), never on a timed path. */
int sky_stream_reserve(sky_stream *s, int64_t tuples);
/* resident tuples and tuples appended since creation */
int sky_stream_size(sky_stream *s, int64_t *resident, int64_t *appended);
/* the rows the next query runs over: a landmark stream holds its local-skyline tuples as
 * distinct vectors (rep + tuple count, tuples as (id, rep) in arrival order), so this is the
 * distinct local-skyline vectors plus the tuples appended since the last query; a sliding
 * window: its resident tuples */
int sky_stream_vectors(sky_stream *s, int64_t *vectors);
int sky_stream_query(sky_stream *s, int64_t *ids_out, int32_t *origin_out, int64_t cap, int64_t *n_out);
int sky_stream_query_dev(sky_stream *s, int64_t *d_ids_out, int32_t *d_origin_out, int64_t cap,
                         int64_t *n_out);
/* The reference's query result is its integers (skyline_size, |L_k|, survivors_k:
 * FlinkSkyline.java:593-608, the JSON of :631-648).  sky_stream_query_async returns as soon as
 * they are known (*n_out, sky_global_stats) and leaves the copy of the ids / origins into
 * ids_out / origin_out in flight on a copy stream of its own, where it overlaps the next
 * appends (give page-locked host memory for an asynchronous copy).  The host arrays are valid
 * after sky_stream_wait (every later query and sky_stream_destroy wait too); *copy_ms
 * (optional): the copy's device time, from the end of the query's kernels to the last byte in
 * host memory. */
int sky_stream_query_async(sky_stream *s, int64_t *ids_out, int32_t *origin_out, int64_t cap, int64_t *n_out);
int sky_stream_wait(sky_stream *s, double *copy_ms);

/* ---- multi-GPU step with one host read (one process per GPU) --------------------
 * The reference scales out by Flink's keyBy shuffle and one global reducer per query
 * (FlinkSkyline.java:138, :171-174, GlobalSkylineAggregator :515-569).  Here every rank owns
 * a shard of the stream (SKY(u SKY(shard_r)) = SKY(u shard_r) for any split) and exchanges a
 * FIXED-SIZE block, so the caller's collectives (RCCL over xGMI, device-resident buffers) need
 * no host-side sizes and one step reads the device back exactly once:
 *   sky_dist_export_dev  local skylines of this rank's shard -> d_block (this rank's block)
 *   caller               all-gather the blocks of every rank into d_blocks (rank order)
 *   sky_dist_merge_dev   this rank's own vectors against the union; this rank's global-skyline
 *                        ids (stream order) -> d_ids_out / d_origin_out (positions < out_cap);
 *                        this rank's share of |L_k| / survivors_k -> d_stats
 *                        (int64[SKY_DIST_STATS_WORDS(K)]: [0, K) |L_k|, [K, 2K) survivors_k,
 *                        [2K] route misses, [2K+1] merge errors -- the last two are verdict
 *                        words, summed so that every rank sees every rank's)
 *   caller               all-reduce (sum) d_stats over the ranks
 *   sky_dist_finish      the one host read: every rank's verdict (from the gathered headers, so
 *                        every rank returns the same code), *n_out = this rank's output count;
 *                        sky_global_stats then returns the job-wide |L_k| / survivors_k.
 * Block: int64[SKY_DIST_BLOCK_WORDS(cap, dims)]: a header row (count, verdict, shard tuples,
 * dims) and up to cap rows of (dims value bits as f64, partition key, multiplicity).
 * sky_dist_finish returns, on every rank alike:
 *   SKY_E_NAN       some shard holds a NaN;
 *   SKY_E_HIP       a look-back ran out of its spin bound on some rank (export or merge);
 *   SKY_E_RETRY     some rank's planned local phase missed, or some rank's union outgrew the
 *                   pair-kernel route it chose from the previous step's sizes: call
 *                   sky_dist_export_dev again (the next attempt takes the sized route);
 *   SKY_E_CAPACITY  with *need_cap > cap: some rank exported more than cap vectors: call
 *                   sky_dist_reblock_dev with a cap >= *need_cap (every rank), then all-gather,
 *                   merge and finish again (no local re-run);
 * and on this rank only SKY_E_CAPACITY with *need_cap == 0 when *n_out > out_cap (out_cap >=
 * the shard's tuple count never overflows).  Output buffers hold unspecified data on error. */
#define SKY_DIST_BLOCK_WORDS(cap, dims) (((int64_t)(cap) + 1) * ((int64_t)(dims) + 2))
#define SKY_DIST_STATS_WORDS(K) (2 * (int64_t)(K) + 2)
int sky_dist_export_dev(sky_ctx *ctx, const int64_t *d_ids, const double *d_values, int64_t n, int64_t *d_block,
                        int64_t cap);
int sky_dist_reblock_dev(sky_ctx *ctx, int64_t *d_block, int64_t cap);
int sky_dist_merge_dev(sky_ctx *ctx, const int64_t *d_blocks, int32_t world, int32_t rank, int64_t cap,
                       int64_t *d_ids_out, int32_t *d_origin_out, int64_t out_cap, int64_t *d_stats);
int sky_dist_finish(sky_ctx *ctx, const int64_t *d_stats_sum, int64_t out_cap, int64_t *n_out, int64_t *need_cap);

/* ---- bulk CSV ingest ------------------------------------------------------ */
/* Decodes '\n'-separated records "id,v1,...,vD" (a non-empty unterminated tail is one
 * more record) exactly as the reference's ingest does per Kafka value: String.split(",")
 * (trailing empty fields dropped), Double.parseDouble on each value (trim, NaN, Infinity,
 * hex, decimal with exponent, one f/F/d/D suffix; correctly rounded), Long.parseLong on
 * the id.  Accepted records are written in record order (ids_out[i], values_out[i*dims..]);
 * the others are dropped and counted per cause in counts_out[4]:
 *   [0] records, [SKY_CSV_MALFORMED] fromString returned null (the reference filters it),
 *   [SKY_CSV_BAD_ID] the id is not a Java long (the reference task would fail),
 *   [SKY_CSV_ARITY]  a well-formed record whose value count is not the context's dims.
 * *n_out = accepted records; SKY_E_CAPACITY (with *n_out set) if cap is too small.
 * d_status_out (optional, one byte per record) receives each record's SKY_CSV_* code. */
#define SKY_CSV_OK        0
#define SKY_CSV_MALFORMED 1
#define SKY_CSV_BAD_ID    2
#define SKY_CSV_ARITY     3
int sky_parse_csv_dev(sky_ctx *ctx, const char *d_text, int64_t nbytes, int64_t *d_ids_out,
                      double *d_values_out, int64_t cap, int64_t *n_out, int64_t *counts_out,
                      uint8_t *d_status_out);
int sky_parse_csv(sky_ctx *ctx, const char *text, int64_t nbytes, int64_t *ids_out, double *values_out,
                  int64_t cap, int64_t *n_out, int64_t *counts_out);
/* formats a device-resident stream as the producers' CSV payload ("%d" for integral
 * values |v| < 2^53, records "id,v1,...,vD\n"); call with cap = 0 to size d_text. */
int sky_format_csv_dev(sky_ctx *ctx, const int64_t *d_ids, const double *d_values, int64_t n,
                       char *d_text, int64_t cap, int64_t *nbytes_out);

/* ---- utilities ------------------------------------------------------------- */
int sky_synth_dev(sky_ctx *ctx, int dist, int dmin, int dmax, uint64_t seed, int64_t id0,
                  int64_t n, double *d_values, int64_t *d_ids);
int sky_synth(int dist, int dims, int dmin, int dmax, uint64_t seed, int64_t id0, int64_t n,
              double *values, int64_t *ids);   /* host copy of the generator (no device) */
/* device memory helpers for callers without a HIP runtime binding of their own */
int sky_dev_alloc(sky_ctx *ctx, int64_t bytes, void **d_out);
int sky_dev_free(sky_ctx *ctx, void *d_ptr);
int sky_memcpy_h2d(sky_ctx *ctx, void *d_dst, const void *h_src, int64_t bytes);
int sky_memcpy_d2h(sky_ctx *ctx, void *h_dst, const void *d_src, int64_t bytes);

/* profiling: HIP-event timings (ms) of the last query, per phase, and the
 * dominant streaming kernel's accumulated time / launch count since reset */
#define SKY_PHASES 8
/* on: 0 off; 1 HIP-event timers around the timed kernels only (light: usable inside a timed
 * region); 2 also the per-phase events of sky_profile_phases */
int sky_profile_enable(sky_ctx *ctx, int on);
/* counters_out: n, candidates, reps (slots on the small-set route), global reps, output size,
 * SFS rounds, pair tests, and [7] = bit0 f64 compares, bit1 score ties, bit2 packed u16,
 * bit3 the planned (device-sized, no mid-query host read) route served the query, bit4 a
 * planned attempt missed and the query re-ran synchronised, bit5 the planned route's tail ran
 * as one workgroup (k_tiny_tail), bits 8.. bounding-box tiles */
int sky_profile_phases(sky_ctx *ctx, double *ms_out /* SKY_PHASES */, int64_t *counters_out /* 8 */);
int sky_profile_kernel(sky_ctx *ctx, const char *name, double *total_ms, int64_t *launches,
                       int64_t *units);
/* algorithmic dominance work of the last query, in pair tests over distinct vectors
 * (SURVEY.md §8d): W = sum_k [s_k(s_k-1)/2 + (n_k - s_k)] + s_G(s_G-1)/2, with n_k / s_k
 * the distinct vectors / distinct local-skyline vectors of partition k and s_G the
 * distinct union of the local skylines; D compares per pair test */
int sky_profile_dominance(sky_ctx *ctx, int64_t *work_out);
int sky_profile_reset(sky_ctx *ctx);
/* host synchronisations (device read-backs) the context has made since it was created */
int sky_profile_host_syncs(sky_ctx *ctx, int64_t *n_out);
/* the pipeline's device radix sort (k_radix.hip: onesweep LSD, 8-bit digits over the varying
 * key bits) run alone on n (u64 key, u32 value) pairs in place, for the sort-phase HBM
 * roofline at scale; *passes_out = digit passes, *ms_out = HIP-event time of the sort */
int sky_profile_sort_dev(sky_ctx *ctx, uint64_t *d_keys, uint32_t *d_vals, int64_t n, int32_t *passes_out,
                         double *ms_out);
/* the small-set route's dense all-pairs kernel (k_brute16_pairs for integer rows, k_brute_pairs
 * f32 / f64 otherwise: every row against every row, ServiceTuple.dominates over the pairs of
 * FlinkSkyline.java:424-441) run alone on n device rows (n x dims f64) with the given partition
 * keys, for the dense dominance roofline: d_fates_out[i] bit0 = some row of i's partition
 * dominates row i, bit1 = some row does; *kind_out = 0 packed u16, 1 f32, 2 f64 compares;
 * *ms_out = HIP-event time of the pair kernel */
int sky_profile_pairs_dev(sky_ctx *ctx, const double *d_values, const int32_t *d_keys, int64_t n,
                          uint32_t *d_fates_out, int32_t *kind_out, double *ms_out);

#ifdef __cplusplus
}
#endif
#endif /* SKYLINE_HIP_H */
