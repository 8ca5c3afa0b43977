// sky_internal.h — host-side declarations shared by the kernel translation units
// and the engine.  Nothing here is part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <algorithm>
#include <utility>
#include <vector>
#include "sky_common.h"
#include "sky_device.h"

#define SKY_DISPATCH_D(D, BODY)                                                    \
    switch (D) {                                                                   \
        case 1: { constexpr int DD = 1; BODY; } break;                             \
        case 2: { constexpr int DD = 2; BODY; } break;                             \
        case 3: { constexpr int DD = 3; BODY; } break;                             \
        case 4: { constexpr int DD = 4; BODY; } break;                             \
        case 5: { constexpr int DD = 5; BODY; } break;                             \
        case 6: { constexpr int DD = 6; BODY; } break;                             \
        case 7: { constexpr int DD = 7; BODY; } break;                             \
        case 8: { constexpr int DD = 8; BODY; } break;                             \
        case 9: { constexpr int DD = 9; BODY; } break;                             \
        case 10: { constexpr int DD = 10; BODY; } break;                           \
        case 11: { constexpr int DD = 11; BODY; } break;                           \
        case 12: { constexpr int DD = 12; BODY; } break;                           \
        case 13: { constexpr int DD = 13; BODY; } break;                           \
        case 14: { constexpr int DD = 14; BODY; } break;                           \
        case 15: { constexpr int DD = 15; BODY; } break;                           \
        case 16: { constexpr int DD = 16; BODY; } break;                           \
        default: break;                                                            \
    }

namespace sky {

// ---- k_scan.hip ----
size_t scan_scratch_words(size_t n);
// d_n (optional): the item count on the device, n its bound
void scan_excl_u32(const uint32_t *in, uint32_t *out, size_t n, uint32_t *d_total, uint32_t *scratch,
                   hipStream_t st, const uint32_t *d_n = nullptr);
// the same in ONE launch above one workgroup's size (decoupled look-back over the earlier tiles
// in blockIdx order, instead of reduce + partials + tiles): lb holds scan_lb_words(n) u64 words,
// zeroed when allocated; epoch in [1, 2^30), larger than every earlier launch's on the same words
// (their words then read as not yet published); a look-back past its spin bound sets *err = 1
size_t scan_lb_words(size_t n);
void scan_excl_u32_lb(const uint32_t *in, uint32_t *out, size_t n, uint32_t *d_total, unsigned long long *lb,
                      uint32_t epoch, uint32_t *err, hipStream_t st);

// ---- k_radix.hip ----
size_t radix_scratch_words(size_t m);
int radix_last_passes();   // digit passes of this thread's last radix_sort_pairs
// err: device word, kFlagRadixSpin is OR-ed in if a look-back spin ran out (never
// expected; the caller checks it at its next synchronisation)
// launch_err (optional): a failed launch of the scratch fill (the kernels' own launch
// errors stay sticky for the caller's next hipGetLastError)
bool radix_sort_pairs(uint64_t *keys, uint32_t *vals, uint64_t *keys_alt, uint32_t *vals_alt, uint32_t m,
                      uint64_t key_or, uint64_t key_and, uint32_t *scratch, uint32_t *err, hipStream_t st,
                      hipError_t *launch_err = nullptr);
void radix_debug_check(const uint64_t *orig, const uint64_t *skey, const uint32_t *perm, uint32_t m, uint32_t *seen,
                       uint32_t *bad, hipStream_t st);
void radix_key_orand(const uint64_t *keys, uint32_t m, unsigned long long *d_orand, hipStream_t st);

// ---- k_partition.hip ----
struct FilterArgs {
    const double *vals;           // n x D row-major f64 (the boundary format)
    uint32_t n;
    KeyParams kp;
    const int32_t *given_keys;    // partition key per tuple (nullptr: computed by kp.algo)
    int single;                   // 1: every tuple is partition 0 (merge / part state)
    const double *pruners;        // [Kp][M][D]
    const int32_t *npr;           // [Kp]
    int M, Kp;
    uint16_t *status;             // [n]
    // candidate slots (unordered append): f64 rows, sort keys, source index, slot per tuple
    double *crow;                 // [n + Kp*M][pad(D)]
    uint64_t *sortkey;
    uint32_t *slot_src;
    uint32_t *m_total;
    unsigned long long *orand;        // device {OR, AND} (deferred tuples add atomically)
    uint32_t *dup_cnt;            // [Kp*M]
    uint32_t *flags;              // kFlag*
    uint32_t *defer_list;         // [n] MR-Angle tuples whose key needs the exact path
    uint32_t *defer_cnt;
    uint32_t slot_cap;            // slots allocated: appends past it are counted, not written
    uint32_t *tile_hist;          // [tiles][Kp*M] duplicates per tile (nullptr: not kept; Kp*M <= kHistMaxKM)
    int dbg;                      // SKY_FILTER_DBG (measurement only, results invalid): 1 = loads + status only, 2 = loads only, 4 = no global atomics
    // status planes (nullptr: every status word is stored): per tile 32 (item, wave) pairs of
    // 64-bit words, B = duplicate of the designated group dom_kj (k * M + j), E = the status
    // word is stored (candidates, other duplicate groups, deferred keys); else dropped
    uint64_t *planes = nullptr;
    int32_t dom_kj = -1;
    // the pruner pick inside the filter (k_pick_pruners' work, redone by every workgroup from
    // the sample minima; workgroup 0 also writes pruners / npr for the later kernels):
    // pick_gmin non-null replaces reading pruners / npr
    const unsigned long long *pick_gmin = nullptr;
    uint32_t pick_S = 0;
    uint32_t pick_tag = 0;            // this query's sample-minima tag (k_sample_min)
    double *pruners_w = nullptr;
    int32_t *npr_w = nullptr;
};
void launch_filter_deferred(int D, const FilterArgs &a, hipStream_t st);
void launch_keys(int D, const double *vals, uint32_t n, const KeyParams &kp, int32_t *keys, hipStream_t st);
// pruners: per partition up to M (<= 64) distinct, mutually non-dominated sample tuples
// (pick = false: only the sample minima; the filter picks them itself, FilterArgs.pick_gmin).
// The minima words are tagged, (tag << 48) | order-key(c) << 16 | sample id (S <= 65536): a
// word of an earlier query (a larger tag) loses to any of this one and reads as empty, so the
// words need no fill between queries (the caller fills them all-ones when the buffer is new and
// when its 16-bit query count wraps).  pre: the query's other fills, done by the sample pass's
// threads before their samples (one launch less; nullptr: the caller launched them)
struct FillRanges;
void launch_select_pruners(int D, const double *vals, uint32_t n, uint32_t S, const KeyParams &kp,
                           const int32_t *given_keys, int single, int Kp, int M, unsigned long long *gmin,
                           double *pruners, int32_t *npr, hipStream_t st, bool pick, uint32_t tag,
                           const FillRanges *pre);
void launch_filter(int D, const FilterArgs &a, hipStream_t st);

struct AppendArgs {
    const double *pruners;        // [Kp][M][D]
    const uint32_t *dup_cnt;      // [Kp*M]
    int Kp, M;
    const uint32_t *m_total;      // device: number of compacted candidates
    uint32_t *nps_total;          // device out: number of pruner slots
    int32_t *entries;             // [nps] -> k*M+j
    int32_t *pruner_slot;         // [Kp*M] -> slot or -1
    void *rows;                   // f64 slot rows
    uint64_t *sortkey;
    uint32_t *slot_src;
    uint32_t *flags;
    unsigned long long *orand;
    uint32_t slot_cap;
    uint32_t *mt_total = nullptr;  // device out (optional): min(m + nps, slot_cap)
};
void launch_append_pruners(int D, const AppendArgs &a, hipStream_t st);
struct FateArgs {
    uint32_t mt;                          // slots (candidates + appended pruner slots)
    const uint32_t *slot_rep, *slot_src;
    const uint8_t *alive_l, *alive_g;     // per representative
    int KM, M, K;
    const int32_t *pruner_slot;
    uint16_t *status;                     // candidates' words rewritten: kCodeFate0 + fate
    uint8_t *pruner_fate;
    const uint32_t *dup_cnt;              // stats only
    unsigned long long *lsz, *surv;       // [kStatShards][K] stat shards, or nullptr: no stats
    uint32_t *tile_cand;                  // [tiles] zeroed: += candidates in G per tile (nullptr: not counted)
    const uint32_t *d_mt = nullptr;       // device slot count (mt is then its bound)
    // the brute route's k_brute_finish folded in: fates from the pair pass's domination bits per
    // slot (every slot its own representative), and the finish's outputs written here -- alive_l /
    // alive_g / slot_rep per slot, per-partition slot / local-skyline counts (zeroed); nullptr: the
    // finish ran and the fates come from alive_l / alive_g / slot_rep
    const uint32_t *domf = nullptr;
    const uint64_t *key = nullptr;        // slot sort keys (partition in bits 63..56)
    int gmerge = 0;
    uint8_t *alive_l_w = nullptr, *alive_g_w = nullptr;
    uint32_t *slot_rep_w = nullptr, *segalive = nullptr, *segn = nullptr;
};
void launch_fate_tables(const FateArgs &a, hipStream_t st);

// candidate prefilter (second-level pruners drawn from the candidates, k_partition.hip)
struct CandArgs {
    uint32_t mt;                  // slots
    const double *rows;           // [mt][pad(D)] f64 slot rows
    const uint64_t *key;          // [mt] sort keys (partition in bits 63..56)
    const uint32_t *src;          // [mt] slot sources
    int Kp, M2;                   // Kp * M2 <= 2048, M2 <= 64
    unsigned long long *cmin;     // [Kp*M2], all-ones on entry
    double *pr2;                  // [Kp][M2][D]
    int32_t *npr2;                // [Kp]
    uint32_t *live;               // [mt] out
    const uint32_t *d_mt = nullptr;   // device slot count (mt is then its bound)
    // the fused pass (k_cand_fused: pick + live test + scan + ordered compaction in one launch)
    double *rows2 = nullptr;
    uint64_t *key2 = nullptr;
    uint32_t *src2 = nullptr;
    uint32_t *d_live = nullptr;           // out: surviving slots
    int32_t *pruner_slot = nullptr;       // remapped in place (appended pruner slots)
    const int32_t *entries = nullptr;     // pruner slot entry -> k * M + j
    int KM = 0;                           // pruner_slot entries (k * M + j)
    unsigned long long *lb = nullptr;     // [cand_fused_tiles(mt)] look-back words, zeroed
    uint32_t *ticket = nullptr;           // zeroed
    uint32_t *err = nullptr;              // kFlagRadixSpin if a look-back ran out of spins
    bool picked = false;                  // k_cand_pick first (pr2 / npr2), then one slot per thread
};
void launch_cand_prefilter(int D, const CandArgs &a, hipStream_t st);
// the criterion minima alone (k_cand_min), for the fused pass after it
void launch_cand_min(int D, const CandArgs &a, hipStream_t st);
// the fused pass: false (nothing launched) when its pruner image does not fit LDS -- the caller
// then runs k_cand_pick / k_cand_filter / the scan / k_cand_compact
bool cand_fused_fits(int D, int Kp, int M2);
// (four slots per thread, or one after k_cand_pick)
inline uint32_t cand_fused_tiles(uint32_t mt, bool picked) {
    const uint32_t per = picked ? kThreads : 4 * kThreads;
    return (mt + per - 1) / per;
}
void launch_cand_fused(int D, const CandArgs &a, hipStream_t st);
void launch_cand_compact(int D, const CandArgs &a, const uint32_t *pos, double *rows2, uint64_t *key2, uint32_t *src2,
                         int32_t *pruner_slot, int KM, hipStream_t st);

struct RepArgs {
    uint32_t mt;                  // sorted slots
    const uint32_t *perm;         // sorted position -> slot
    const uint64_t *skey;         // sorted keys
    const void *rows;             // [mt][DP] by slot
    void *rows_sorted;            // [mt][DP] by sorted position
    uint32_t *runflag, *runscan, *run_first, *repof, *repflag, *repscan;
    void *rep_rows;               // [mr][DP]
    uint64_t *rep_key;            // [mr]
    uint32_t *rep_of_sorted;      // [mt]
    uint32_t *slot_rep;           // [mt]
};
void launch_gather_runs(int D, bool f64, const RepArgs &a, hipStream_t st);
void launch_run_first(const RepArgs &a, hipStream_t st);
void launch_rep_of(int D, bool f64, const RepArgs &a, hipStream_t st);
void launch_build_reps(int D, bool f64, const RepArgs &a, hipStream_t st);
void launch_seg_bounds(const uint64_t *rep_key, uint32_t mt, const uint32_t *d_mr, uint32_t *seg_begin,
                       uint32_t *seg_end, hipStream_t st);
void launch_rep_mult(uint32_t mt, const uint32_t *perm, const uint32_t *slot_src, const uint32_t *rep_of_sorted,
                     const int64_t *given_w, const uint32_t *dup_cnt, const int32_t *pr_entries,
                     unsigned long long *mult, hipStream_t st);

struct OutArgs {
    const uint16_t *status;
    uint32_t n;
    const uint8_t *pruner_fate;   // [Kp*M]
    int M, KM;
    const int32_t *given_origin;  // per tuple origin (nullptr: partition key)
    const int64_t *given_w;       // per tuple weight (nullptr: 1)
    int K;                        // stats slots
    unsigned long long *lsz, *surv;   // [K]
    uint32_t *out_cnt;            // [tiles]
    const uint32_t *out_off;      // [tiles] (write pass)
    const int64_t *ids;           // nullptr: ids are the tuple index
    const double *vals;           // for rows_out
    int D;
    int64_t *ids_out;
    int32_t *origin_out;
    double *rows_out;
    uint8_t *row_flags;           // optional per tuple: bit0 inL, bit1 inG
    int64_t out_cap = INT64_MAX;  // write pass: output positions >= out_cap are not written
    int select_local;             // output tuples in L instead of G
    const uint64_t *planes = nullptr;   // the filter's status planes (k_out_write only)
    int32_t dom_kj = -1;
    const uint32_t *skip_flags = nullptr;   // write pass: nothing is written if this word has a tail miss / guard bit
    bool sparse_ids = false;                 // write pass: ids loaded after the selection, by selected lanes only
    // write pass: the brute route's final read folded in (k_stat_reduce + k_gather_words): K more
    // workgroups past the tiles reduce one stat key each, one more copies the other words, all into
    // host-mapped memory in tiny_pin_layout (ep_pin nullptr: no epilogue)
    uint32_t *ep_pin = nullptr;
    uint32_t ep_off[5] = {};
    const unsigned long long *ep_lsz = nullptr, *ep_surv = nullptr;   // [kStatShards][K]
    unsigned long long *ep_statk = nullptr;                          // [2K]
    const uint32_t *ep_totals = nullptr, *ep_segalive = nullptr, *ep_segn = nullptr, *ep_flags = nullptr,
                   *ep_dup = nullptr;
    int ep_Kp = 0;
};
void launch_out_count(const OutArgs &a, hipStream_t st);
// per-tile counts of the global level from the filter's duplicate histograms + k_fate_tables'
// candidate counts (replaces the count pass for unit weights / slot stats)
constexpr int kHistMaxKM = 256;
void launch_out_hist_count(const uint32_t *hist, const uint32_t *tile_cand, const uint8_t *pruner_fate, int KM,
                           uint32_t ntiles, uint32_t *out_cnt, hipStream_t st);
// the same counts + their exclusive scan (out_off, *d_total) in one launch: lb holds
// out_hist_scan_blocks(ntiles) look-back words, zeroed when allocated; epoch != the last launch's
uint32_t out_hist_scan_blocks(uint32_t ntiles);
struct Pipe;
int out_hist_scan_words(Pipe &p, uint32_t tiles, hipStream_t st);   // engine.hip: sizes / zeroes the words
void launch_out_hist_scan(const uint32_t *hist, const uint32_t *tile_cand, const uint8_t *pruner_fate, int KM,
                          uint32_t ntiles, uint32_t *out_cnt, uint32_t *out_off, uint32_t *d_total,
                          unsigned long long *lb, uint32_t epoch, uint32_t *err, hipStream_t st);
void launch_out_write(const OutArgs &a, hipStream_t st);
// count + prefix + write in one pass (decoupled look-back over tiles): lb [tiles] u64 and
// *ticket zeroed by the caller; *d_total = selected tuples; writes positions < cap only
void launch_out_fused(const OutArgs &a, unsigned long long *lb, uint32_t *ticket, uint32_t *d_total, uint32_t *err,
                      int64_t cap, hipStream_t st);

// ---- k_sfs.hip ----
struct SfsSeg { uint32_t begin, count; };
struct SfsTile { uint32_t seg, start, count, out; };
void launch_block_sky(int D, bool f64, bool full, bool ties, int B, int TB, const void *rows, const uint64_t *key,
                      const uint32_t *act, const SfsSeg *segs, const uint32_t *seg_list, uint32_t nseg_work,
                      uint8_t *alive, uint8_t *xkeep, hipStream_t st);
void launch_filter_rest(int D, bool f64, bool full, int B, int TB, const void *rows, const uint32_t *act,
                        const SfsTile *tiles, uint32_t ntiles, const SfsSeg *segs, const uint8_t *xkeep,
                        uint32_t *keep, hipStream_t st);
void launch_act_compact(const uint32_t *act_old, const uint32_t *keep, const uint32_t *keep_scan,
                        const SfsTile *tiles, uint32_t ntiles, uint32_t *act_new, uint32_t *segcnt,
                        hipStream_t st);
void launch_iota(uint32_t *a, uint32_t n, hipStream_t st);
void launch_nan_any(const double *v, size_t count, uint32_t *flag, hipStream_t st);
// up to kFillMax byte ranges (4-byte aligned starts, < 4 GiB each): the kernel argument of
// one k_fill_multi / k_gather_words launch
constexpr int kFillMax = 16;
struct FillRanges {
    uint8_t *p[kFillMax] = {};
    uint32_t bytes[kFillMax] = {};
    uint32_t val[kFillMax] = {};
    int n = 0;
};
// any number of fills: batched kFillMax per k_fill_multi launch; ranges of 4 GiB or more are
// split, unaligned ranges go through hipMemsetAsync.  Never aborts.
struct FillSet : FillRanges {
    std::vector<FillRanges> full;                 // batches already complete
    std::vector<std::pair<std::pair<void *, size_t>, int>> plain;   // unaligned: hipMemsetAsync
    void add(void *ptr, size_t nbytes, int value = 0);
    hipError_t launch(hipStream_t st);
    // the pending ranges as ONE kernel argument for another kernel to fill (cleared here, nothing
    // launched); false (nothing taken) when they need more than one batch or a hipMemsetAsync
    bool take(FillRanges &out);
};
// a kernel's grid-wide share of k_fill_multi's work (every thread of the grid calls it)
__device__ inline void fill_ranges_grid(const FillRanges &f) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, T = gridDim.x * blockDim.x;
#pragma unroll
    for (int j = 0; j < kFillMax; j++) {           // (compile-time indices into the argument)
        if (j >= f.n) break;
        uint8_t *p = f.p[j];
        const uint32_t bytes = f.bytes[j], val = f.val[j];
        const uint32_t words = bytes >> 2, w4 = val * 0x01010101u;
        uint32_t *p4 = reinterpret_cast<uint32_t *>(p);
        for (uint32_t q = t; q < words; q += T) p4[q] = w4;
        if (t < (bytes & 3u)) p[words * 4 + t] = (uint8_t)val;
    }
}

// ranges g.p[j] (g.bytes[j] bytes, 4-aligned) copied to pinned_dst + g.val[j] in one launch
hipError_t launch_gather_words(const FillRanges &g, void *pinned_dst, hipStream_t st);
void launch_global_keys(const uint64_t *rep_key, const uint8_t *alive_l, const uint32_t *alive_scan, uint32_t mr,
                        uint64_t *gkey, uint32_t *gval, unsigned long long *orand, hipStream_t st);
void launch_sfs_small(int D, bool f64, bool full, bool ties, int B, const void *rows, const uint64_t *key,
                      const SfsSeg *segs, const uint32_t *seg_list, uint32_t nwork, uint8_t *alive, void *conf,
                      hipStream_t st);
void launch_gather_rows(int D, bool f64, const void *src, const uint32_t *idx, uint32_t m, void *dst,
                        hipStream_t st);
void launch_scatter_alive(const uint32_t *gval, const uint8_t *galive, uint32_t mg, uint8_t *alive_g,
                          hipStream_t st);
void launch_stat_reduce(const unsigned long long *lsz, const unsigned long long *surv, int K, unsigned long long *out,
                        hipStream_t st);
// both skyline levels of a small rep set in one launch (alive_l, alive_g, segalive counts)
// the largest slot count the brute pass takes (SKY_BRUTE_MAX, default 32768; engine.hip)
uint32_t brute_max();
// over f64 candidate slots (rows [mr][pad(D)], sort keys): domf / segalive / segn zeroed by
// the caller; writes alive_l / alive_g / slot_rep (identity) per slot
// f32: compare in f32 (every candidate value exactly an f32), else f64; u16: every candidate
// value an integer in [0, 65535]: packed u16 compares (k_brute16_pairs)
// d_mr (optional): the slot count on the device, mr its bound
// the pair kernel of launch_brute_fates alone (domf zeroed by the caller)
void launch_brute_pairs(int D, bool f32, bool u16, const void *rows, const uint64_t *key, uint32_t mr, uint32_t *domf,
                        hipStream_t st, const uint32_t *d_mr = nullptr);
// rows n x D (f64, row-major) + partition keys -> slot rows (f64, padded) + sort keys as the
// filter writes them; *flags |= kFlagNotF32 / kFlagNotU16 / kFlagScoreTies
void launch_prof_slots(int D, const double *vals, const int32_t *keys, uint32_t n, double *rows, uint64_t *key,
                       uint32_t *flags, hipStream_t st);
void launch_brute_fates(int D, bool f32, bool u16, const void *rows, const uint64_t *key, uint32_t mr, bool gmerge,
                        uint32_t *domf, uint8_t *alive_l, uint8_t *alive_g, uint32_t *segalive, uint32_t *segn,
                        uint32_t *slot_rep, hipStream_t st, const uint32_t *d_mr = nullptr);
void launch_seg_alive(const uint64_t *rep_key, const uint8_t *alive, uint32_t mr, uint32_t *cnt, hipStream_t st);
void launch_flag_u8_to_u32(const uint8_t *in, uint32_t n, uint32_t *out, hipStream_t st);

// ---- k_dom16.hip (integer-valued rows packed as u16 pairs) ----
struct DomItem { uint32_t seg, y0, ny, x0, nx, flags; };
constexpr uint32_t kDomDiag = 1u;             // x and y ranges overlap: only x before y
constexpr uint32_t kDomRest = 2u;             // x from xbuf[seg] (X'), count from xcnt[seg]
int dom16_ppt();                              // y rows per lane (work item = 64 * ppt y rows)
uint32_t dom16_tx();                          // x rows per work item: SKY_DOM_TX, 0 = adaptive
constexpr uint32_t kDomTx = 512u;             // largest adaptive x rows per work item
int dom16_words(int D);
void launch_pack16(int D, const float *rows, uint32_t m, const uint32_t *idx, uint32_t *out, hipStream_t st);
constexpr int kDomTriPPT = 1;                 // tri tiles: 64 y per wave (latency-bound, many waves)
void launch_dom16(int W, int ppt, bool diag, const uint32_t *rows, const uint32_t *xbuf, const uint32_t *xcnt, const DomItem *items,
                  uint32_t nitems, uint32_t xcap, uint32_t *dead, hipStream_t st);
void launch_xcompact16(int W, const uint32_t *rows, const uint32_t *idx, const SfsSeg *xseg, uint32_t nslots,
                       uint32_t xcap, uint32_t *dead, uint32_t *xbuf, uint32_t *xcnt, uint8_t *alive, hipStream_t st);
void launch_keep16(const uint32_t *dead, uint32_t n, uint32_t *keep, hipStream_t st);
void launch_move16(int W, const uint32_t *keep, const uint32_t *scan, uint32_t n, const uint32_t *idx,
                   const uint32_t *rows, uint32_t *idx_out, uint32_t *rows_out, hipStream_t st);
void launch_gather_u32(const uint32_t *src, const uint32_t *at, uint32_t n, uint32_t *out, hipStream_t st);

// ---- k_mbr.hip (both skyline levels of a large rep set, bounding-box pruned all-pairs) ----
constexpr int kMbrLptHead = 64;   // head words of MbrArgs::lpt: [0, 32) bucket counts, [32] ticket,
                                  // [33] work items, [36..37] total cost (u64)
constexpr int kMbrSplitMax = 64;  // work items per y tile at most (its reachable groups split between them)
constexpr int kMbrSubMax = 8;     // sub-box corners per 64-row tile (k_mbr.hip mbr_subs)
// work items <= ytiles + max(ytiles, 4096) (k_mbr_order's split rule); 2 words per item
inline size_t mbr_items_max(size_t ytiles) { return ytiles + std::max<size_t>(ytiles, 4096); }
inline size_t mbr_lpt_words(size_t ytiles) { return kMbrLptHead + ytiles + 2 * mbr_items_max(ytiles); }
struct MbrArgs {
    int D = 0;
    int fmt = 0;                  // 0: packed u16 rows (dom16 layout), 1: f32 rows, 2: f64 rows
    const void *rows = nullptr;   // [mr][mbr_row_words] by rep
    const uint64_t *rep_key = nullptr;   // partition in bits 63..56
    uint32_t mr = 0;
    bool gmerge = false;          // the global level (alive_g) too
    bool full = false;            // complete dominance test (rows may repeat a vector)
    int row_min = 24;
    int dbg = 0;                  // SKY_MBR_DBG (measurement only): 1 skip the pair tests, 2 also the lane tests
    uint32_t *mm = nullptr;       // [2D]: {0xffffffff} x D, {0} x D on entry
    uint64_t *code = nullptr, *code_alt = nullptr;   // [mr]
    uint32_t *idx = nullptr, *idx_alt = nullptr;     // [mr]
    uint32_t *radix_scratch = nullptr, *err = nullptr;
    uint32_t *trows = nullptr;    // [ntiles*64][NW]
    uint32_t *tpart = nullptr;    // [mr]
    uint32_t *tmin = nullptr, *tmax = nullptr;       // [NW][ntiles]
    uint32_t *tprange = nullptr;  // [ntiles]
    uint32_t *tsub = nullptr;     // [ntiles][S][NW] (room for kMbrSubMax): min corners of the sub-boxes
    uint32_t *gmin = nullptr;     // [NW][ngroups]: min corners of the groups of 64 tiles
    uint32_t *gprange = nullptr;  // [ngroups]: their partition ranges
    uint32_t *domf = nullptr;     // [mr], zeroed by the caller
    unsigned long long *pairs = nullptr;             // executed pair tests (optional, zeroed)
    // the pair pass's work queue (k_mbr_cost / k_mbr_order, mbr_lpt_words): [kMbrLptHead] head
    // words zeroed by the caller, a cost word per y tile, then the work items (y tile, part |
    // parts << 16), heaviest first
    uint32_t *lpt = nullptr;
    uint8_t *alive_l = nullptr, *alive_g = nullptr;  // [mr] by rep
    // measurement builds only (SKY_MBR_DBG & 8): per work item of the pair pass {start, end,
    // tested tiles, pair tests} (s_memrealtime ticks, 100 MHz)
    unsigned long long *trace = nullptr;
};
// the multi-GPU merge: own rows (y, a contiguous range of the union) against the whole union
// (x), FULL test, both levels; x.gmin / x.gprange needed, y's group buffers unused
struct MbrUnionArgs {
    MbrArgs x, y;                 // rows / rep_key / mr and the tile buffers of each set; y.domf zeroed
    const int64_t *ymult = nullptr;
    int K = 0;
    uint8_t *flags = nullptr;     // per own row: inL | inG << 1
    unsigned long long *lsz = nullptr, *surv = nullptr;   // [K] this rank's shares
};
hipError_t launch_mbr_union(const MbrUnionArgs &a, hipStream_t st);
int mbr_row_words(int D, int fmt);
size_t mbr_tiles(uint32_t mr);
size_t mbr_groups(uint32_t mr);
hipError_t launch_mbr(const MbrArgs &a, hipStream_t st);

// ---- k_part.hip (per-key operator state, incremental) ----
// one part's share of a batched insert (device memory, uploaded with the batch)
struct PartDesc {
    const double *bvals;          // [nb][D] this part's batch
    const int64_t *bids;          // [nb]
    uint32_t nb;
    uint32_t rb;                  // bound of the state's rep count (launch sizes; the device count decides)
    uint32_t *dom_b, *eq_s, *eq_b, *kpos, *fpos;   // [nb] work (dom_b, eq_* initialised by k_parts_prune)
    uint32_t *dom_s;              // [rb] work (zeroed by k_parts_prune)
    uint32_t *eqp;                // [nb] pruner class of the tuple (~0: none), written by k_parts_prune
    uint32_t *uidx;               // [nb] the undecided tuples (batch indices), written by k_parts_prune
    uint32_t *meta;               // [kPartMeta] |U|, pruner index / first index per class, killed, ticket
    double *sl_v;                 // [slices][kPartPruners] per slice: criterion minima (k_parts_crit)
    uint32_t *sl_i;               // [slices][kPartPruners] ... and their indices
    uint32_t *sl_k;               // [2][slices] per slice: kept tuples, new reps (k_parts_count)
    double *rrows;                // state: reps [R][D], alive, tuples per rep
    uint8_t *ralive;
    uint32_t *rcnt;
    int64_t *tids;                // state: tuples (id, rep) in insertion order
    uint32_t *trep;
    uint32_t *dcnt;               // device counts: R, T, dead (u64 lo, hi)
    uint32_t *mirror;             // host-mapped seqlock mirror of the counts (nullptr: none)
    uint32_t seq;                 // this insert's sequence number (the mirror's tag)
};
struct PartItem {
    uint32_t part;
    uint32_t mode;                // 0: batch vs batch, 1: batch vs state reps, 2: state reps vs batch
    uint32_t y0, x0;              // 256 y rows from y0, kPartChunk x rows from x0
};
// one key's tuples in sky_parts_global_merge: ids / rep of its T alive tuples (insertion
// order), where they start in the concatenation (toff) and its reps (roff), the output origin
struct PgmList {
    const int64_t *tids;
    const uint32_t *trep;
    uint32_t toff, roff;
    int32_t part_id;
    uint32_t nrep;                // reps of the list (bound of its trep entries)
};
void launch_pgm_prep(uint32_t R, const uint32_t *rcnt, int32_t k, int32_t *origin, int64_t *w, hipStream_t st);
void launch_pgm_flags(uint32_t n, const int64_t *surv_idx, uint8_t *flag, hipStream_t st);
void launch_pgm_tuples(const PgmList *lists, int nl, uint32_t ttot, const uint8_t *flag, uint32_t *tsel,
                       uint32_t *tpos, uint32_t *d_total, uint32_t *scratch, int64_t *ids_out, int32_t *org_out,
                       uint32_t *err, hipStream_t st);
constexpr uint32_t kPartItemY = 256, kPartItemX = 256;
constexpr int kPartPruners = 4;   // batch pruners per insert (k_parts_crit / k_parts_classify)
constexpr int kPartMeta = 16;     // words of PartDesc::meta
constexpr uint32_t kPartSlice = 1024;   // batch tuples per workgroup of the insert kernels
void launch_parts_insert(int D, const PartDesc *descs, int nparts, uint32_t max_slices, const PartItem *items,
                         uint32_t nitems, hipStream_t st);
void launch_part_rkeep(uint32_t R, const uint8_t *ralive, uint32_t *keep, hipStream_t st);
void launch_part_rmove(int D, uint32_t R, const uint32_t *keep, const uint32_t *pos, const double *rows,
                       const uint32_t *cnt, double *rows2, uint32_t *cnt2, uint8_t *alive2, hipStream_t st);
void launch_part_tkeep(uint32_t T, const uint32_t *trep, const uint8_t *ralive, uint32_t *keep, hipStream_t st);
void launch_part_tmove(uint32_t T, const uint32_t *keep, const uint32_t *pos, const uint32_t *rpos, const int64_t *ids,
                       const uint32_t *trep, int64_t *ids2, uint32_t *trep2, hipStream_t st);
void launch_part_rows_out(int D, uint32_t T, const uint32_t *trep, const double *rrows, double *out, hipStream_t st);

// ---- k_dist.hip (multi-GPU step, device-sized) ----
// verdict bits of a rank's block header (sky_dist_finish reads them for every rank)
constexpr uint32_t kDistNaN = 1u;       // a tuple value is NaN: every rank returns SKY_E_NAN
constexpr uint32_t kDistReplan = 2u;    // the planned local phase missed an assumption: re-run the step
constexpr uint32_t kDistError = 4u;     // a look-back exceeded its spin bound (internal error)
struct PlanCheck {                      // pipe_finish's planned-route checks, as kernel arguments
    int planned = 0;
    uint32_t cap = 0;                   // candidate slots allocated
    uint32_t bound[4] = {};             // slots entering round r / the brute pass
    int rounds = 0;
    uint32_t brute_max = 0;
    int k_u16 = 0, k_f32 = 0;           // the brute pass's compare type
};
void launch_plan_verdict(const uint32_t *totals, const uint32_t *flags, const PlanCheck &pc, uint32_t *verdict,
                         hipStream_t st);
void launch_dist_flags(const uint8_t *alive, uint32_t n, const uint32_t *d_n, uint32_t *out, hipStream_t st);
// the slot-mode export tail (verdict, flags, scan, rows, header) in one workgroup, for up to
// dist_export_one_max() units; pos has n_units + 1 entries
uint32_t dist_export_one_max();
void launch_dist_export_one(int D, const uint32_t *tot, const uint32_t *flags, const PlanCheck &pc, uint32_t *verdict,
                            const uint8_t *alive, uint32_t n_units, const uint32_t *d_n, uint32_t *flag, uint32_t *pos,
                            uint32_t *d_count, const double *rows, const uint64_t *key, const uint32_t *slot_src,
                            const uint32_t *dup_cnt, const int32_t *pr_entries, int64_t *block, uint32_t cap,
                            uint32_t n_tuples, hipStream_t st);
void launch_dist_rows(int D, bool f64, const void *rows, const uint64_t *key, const uint32_t *flag, const uint32_t *pos,
                      uint32_t n, const uint32_t *slot_src, const uint32_t *dup_cnt, const int32_t *pr_entries,
                      const unsigned long long *mult, int64_t *block, uint32_t cap, hipStream_t st);
void launch_dist_header(const uint32_t *d_count, const uint32_t *verdict, uint32_t n, int D, int64_t *block,
                        hipStream_t st);
void launch_dist_summary(const int64_t *blocks, int world, int rank, uint32_t cap, int D, unsigned long long *sum,
                         hipStream_t st);
void launch_dist_compact(int D, const int64_t *blocks, int world, uint32_t cap, unsigned long long *sum, double *urows,
                         uint64_t *ukey, int64_t *umult, hipStream_t st);
void launch_dist_pack(int D, const double *rows, uint32_t m, int fmt, uint32_t *out, hipStream_t st);
void launch_dist_union_fate(int D, const int64_t *blocks, int world, int rank, uint32_t cap, int K, uint8_t *flags,
                            uint32_t *dom, unsigned long long *lsz, unsigned long long *surv, unsigned long long *sum,
                            unsigned long long limit, unsigned long long *miss, hipStream_t st);
void launch_dist_merge_err(const uint32_t *flags, unsigned long long *statk, int err_word, int words, int64_t *out,
                           hipStream_t st);
void launch_dist_alive_g(const uint32_t *flag, const uint32_t *pos, uint32_t n, const uint8_t *own_flags, uint32_t cap,
                         uint8_t *alive_g, hipStream_t st);

// ---- k_synth.hip ----
void launch_synth(int dist, int D, int dmin, int dmax, uint64_t seed, int64_t id0, int64_t n, double *vals,
                  int64_t *ids, hipStream_t st);
void synth_host(int dist, int D, int dmin, int dmax, uint64_t seed, int64_t id0, int64_t n, double *vals,
                int64_t *ids);

// ---- k_csv.hip ----
int64_t csv_chunks(int64_t nbytes);
void launch_csv_nl_count(const uint8_t *text, int64_t nbytes, uint32_t *blk_cnt, uint32_t *cnt1k,
                         unsigned long long *ncomma, hipStream_t st);
// positions of the newlines that end groups of R records: line_g[g] = end of group g
void launch_csv_nl_groups(const uint8_t *text, int64_t nbytes, const uint32_t *blk_off, const uint32_t *cnt1k,
                          int64_t nl, int R, int64_t *line_g, hipStream_t st);
void launch_csv_parse(const uint8_t *text, int64_t nbytes, const int64_t *line_g, int64_t nl, int64_t nrec, int D,
                      int64_t *ids, double *vals, uint8_t *status, unsigned long long *counts, uint32_t *spill,
                      longlong3 *slow, unsigned long long *slow_n, unsigned long long slow_cap, int R,
                      hipStream_t st);
// line_g: group boundaries for groups of 256 (kCsvThreads) records
void launch_csv_parse_exact(const uint8_t *text, int64_t nbytes, const int64_t *line_g, int64_t nl, int64_t nrec,
                            int D, int64_t *ids, double *vals, uint8_t *status, unsigned long long *counts,
                            hipStream_t st);
int csv_records_per_block(int64_t nbytes, int64_t nrec, int64_t nfields, int D);
void launch_csv_keep(const uint8_t *status, int64_t n, uint32_t *keep, hipStream_t st);
void launch_csv_compact(const uint8_t *status, const uint32_t *pos, int64_t n, int D, const int64_t *ids_in,
                        const double *vals_in, int64_t *ids_out, double *vals_out, hipStream_t st);
void launch_csv_fmt_len(const int64_t *ids, const double *vals, int64_t n, int D, uint32_t *len,
                        unsigned long long *tot_err, hipStream_t st);
void launch_csv_fmt_write(const int64_t *ids, const double *vals, int64_t n, int D, const uint32_t *off,
                          uint8_t *text, hipStream_t st);

}  // namespace sky

namespace sky {

// ---- the small planned route's tail in ONE workgroup (k_partition.hip k_tiny_tail) ----
// Everything between the filter and the output write pass of a planned query whose candidate
// slot rows are few (bound[0] rows of f64 <= kTinyCandBytes: the prefilter passes read them from
// one CU) and whose last query ended with <= 3/4 of tiny_brute_rows(D) slots:
// append the duplicated pruners, the prefilter rounds, the brute pair pass (exact f64 tests),
// the fate tables, the per-tile output counts + their scan and the stats -- one launch instead
// of ~12 dependent launches of 2-6 us each, its phases' data kept in LDS.  If the final slots
// exceed tiny_brute_rows(D) the kernel raises kFlagTinyMiss and writes no fate: the host re-runs the
// query on the synchronised route.
constexpr size_t kTinyCandBytes = 512 * 1024;
constexpr uint32_t kTinyTiles = 4096;
// LDS arena of the tail (bytes): the prefilter phase (minima, weights, second-level pruners) and
// the brute / fate phase (final rows + partition + fate per slot, then per-partition stats and
// counts, per-tile counts, pruner fates) reuse it; the final slots it holds follow from D
constexpr size_t kTinyArena = 56 * 1024;
constexpr size_t kTinyFixed = (size_t)kMaxK * 24 + (size_t)kTinyTiles * 4 + 2 * kHistMaxKM + 16 + 8;
constexpr uint32_t tiny_brute_rows(int D) {     // per final slot: the row, partition, fate, source
    return (kTinyArena - kTinyFixed) / (D * 8 + 12) < 512 ? (uint32_t)((kTinyArena - kTinyFixed) / (D * 8 + 12)) : 512u;
}
constexpr int kTinyThreads = 1024;
constexpr int kTinyM2 = 16;             // second-level pruners per partition in the tail (compile-time)
constexpr uint32_t kTinyForce = 192;      // a plan without rounds: the tail runs one above this many slots
constexpr uint32_t kFlagTinyMiss = 64u;
// an index of the one-workgroup tail fell outside the capacity the host passed for its array: the
// access was skipped and the run is invalid (SKY_E_HIP; the product build's device guard)
constexpr uint32_t kFlagTinyOob = 128u;
struct TinyArgs {
    AppendArgs ap;                        // rows / sortkey / slot_src: the filter's slots
    int rounds = 0, M2 = 0;
    uint32_t bound[4] = {};               // plan bounds (slots entering round r; [rounds]: the brute)
    double *pr2 = nullptr;                // [Kp*M2][D] second-level pruners (scratch)
    const unsigned long long *cmin0 = nullptr;   // round 0's criterion minima from k_cand_min (or nullptr)
    uint32_t *live = nullptr, *livepos = nullptr;        // [bound0] scratch
    double *rows_r[3] = {};               // the rounds' compaction targets (f64 slot rows)
    uint64_t *key_r[3] = {};
    uint32_t *src_r[3] = {};
    // [10] slots, [11 + r] survivors of round r, [14] the final slots, [3] output total
    uint32_t *totals = nullptr;
    bool gmerge = false;
    uint8_t *alive_l = nullptr, *alive_g = nullptr;
    uint32_t *segalive = nullptr, *segn = nullptr, *slot_rep = nullptr;
    // fate tables (FateArgs semantics, slot stats), output counts
    uint16_t *status = nullptr;
    uint8_t *pruner_fate = nullptr;
    int K = 1;
    const uint32_t *tile_hist = nullptr;
    uint32_t ntiles = 0;
    uint32_t *out_cnt = nullptr, *out_off = nullptr;
    unsigned long long *statk = nullptr;  // [2K]: |L_k|, survivors_k
    // measurement builds (SKY_TINY_CHK): every global index checked against its buffer's
    // capacity, an out-of-range access skipped and reported as a bit of *chk.  cap: slots,
    // live, rows_r[0..2] (slots), final slots, status words, Kp*M
    uint32_t *chk = nullptr;
    uint32_t cap[8] = {};
    unsigned long long *clk = nullptr;    // (SKY_TINY_CLK) s_memrealtime at the phase ends, [10]
    int dbg = 0;                          // (SKY_TINY_DBG, measurement only, results invalid): 1 no atomics, 2 no criteria
    // the final read's words written straight into the host-mapped buffer (no gather launch):
    // totals at word 0, then (word offsets) statk, segalive, segn, flags, dup_cnt -- the layout of
    // pipe_finish's read list (tiny_pin_layout)
    uint32_t *pin = nullptr;
    uint32_t pin_off[5] = {};
};
// word offsets of statk / segalive / segn / flags / dup_cnt after the 16 totals words, each range
// rounded up to 16 bytes as sync_read lays them out; returns the bytes in all
inline size_t tiny_pin_layout(int K, int Kp, int KM, uint32_t off[5]) {
    const size_t sz[6] = {64, (size_t)K * 16, (size_t)Kp * 4, (size_t)Kp * 4, 4, (size_t)KM * 4};
    size_t o = 0;
    for (int i = 0; i < 6; i++) {
        if (i) off[i - 1] = (uint32_t)(o / 4);
        o += (sz[i] + 15) & ~size_t(15);
    }
    return o;
}
void launch_tiny_tail(int D, const TinyArgs &a, hipStream_t st);
// the tail's LDS arena holds both phases' data for this shape (host check before the launch)
bool tiny_fits(int D, int Kp, int M2, int KM, int K, uint32_t tiles);

}  // namespace sky
