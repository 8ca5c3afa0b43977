// engine.h — host-side orchestration of the gfx950 skyline pipeline.
#pragma once
#include <hip/hip_runtime.h>
#include <string>
#include <vector>
#include "sky_internal.h"

namespace sky {

void set_error(const std::string &msg);

// grow-only device buffer
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    DevBuf(DevBuf &&o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr; o.cap = 0; }
    DevBuf &operator=(DevBuf &&o) noexcept {
        if (this != &o) {
            release();
            p = o.p;
            cap = o.cap;
            o.p = nullptr;
            o.cap = 0;
        }
        return *this;
    }
    int ensure(size_t bytes);
    void release();
    template <typename T> T *as() const { return reinterpret_cast<T *>(p); }
    ~DevBuf() { release(); }
};

struct PipeIn {
    const double *vals = nullptr;   // device, n x D f64
    uint32_t n = 0;
    const int64_t *ids = nullptr;   // device ids (nullptr: tuple index)
    const int32_t *keys = nullptr;  // given partition keys (nullptr: computed)
    const int32_t *origin = nullptr;// given origin tags for stats / output (nullptr: partition key)
    const int64_t *weights = nullptr;
    bool single = false;            // one partition (global merge of lists, local state insert)
    bool global = true;             // run the global merge after the local skylines
    bool fate = true;               // per-tuple fate pass (stats, output counts)
    bool planes_ok = false;         // the output comes from this run's own write pass only (no later
                                    // recount over the status words): the filter may store status planes
    bool dist = false;              // multi-GPU export (sky_dist_export_dev): local skylines only, the
                                    // small-set / planned routes allowed, the run's checks deferred to a
                                    // device verdict (no host read at the end of the run)
    int K = 1;                      // stats slots
    // optional: the global skyline's stream-ordered ids / origins, written by the run itself
    // (single-pass output) when the stats come from the slots; pipe_output then only checks
    int64_t *out_ids = nullptr;
    int32_t *out_org = nullptr;
    int64_t out_cap = 0;
    // optional: per tuple its fate (bit 0 in L_k, bit 1 in G), written by the run's count pass when
    // it has one (given origins / weights: the landmark stream's state update), else left untouched
    uint8_t *row_flags = nullptr;
};

struct PhaseTimer;

// One pipeline instance = its own workspace (a context owns two so that the
// multi-GPU import can run on the union while the local shard's state is kept).
struct Pipe {
    // per tuple / per tile
    DevBuf status, out_cnt, out_off;
    // pruners
    DevBuf pmin, pruners, npr, dup_cnt, pr_entries, pruner_slot;
    uint32_t pmin_epoch = 0;          // queries since pmin was filled all-ones (its words' tags)
    const void *pmin_at = nullptr;    // ... and the buffer that fill was for (address and capacity:
    size_t pmin_cap = 0;              //     a regrown buffer may come back at the same address)
    // candidates (slot order) and sort
    DevBuf rows, sortkey, slot_src, perm, key_alt, val_alt, rows_sorted;
    DevBuf runflag, runscan, run_first, repof, repflag, repscan, rep_rows, rep_key, rep_of_sorted, slot_rep;
    DevBuf alive_l, alive_g, alive_u32, alive_scan, mult;
    // SFS
    DevBuf act, act2, keep, keep_scan, conf_rows, nconf, segs, seg_list, tiles, seg_begin, seg_end, segcnt;
    DevBuf conf_small, seg_small, pruner_fate, defer, xkeep;
    // global
    DevBuf gkey, gval, gkey_alt, gval_alt, grows, galive, gact_dummy;
    // integer-valued fast path (k_dom16.hip): packed u16 rows, round layouts, X' buffers
    DevBuf r16, r16g, r16a, r16b, i16a, i16b, dead16, keep16, scan16, xbuf16, xcnt16, xseg16, items16, at16, atv16;
    DevBuf scratch, flags, totals, orand, lsz, surv, statk, segalive;
    // candidate prefilter (second-level pruners) and its compaction targets
    DevBuf cmin, pr2, npr2, live, livepos, rows2, sortkey2, slot_src2, rows3, sortkey3, slot_src3;
    // bounding-box pruned all-pairs pass over large rep sets (k_mbr.hip)
    DevBuf mbr_mm, mbr_code, mbr_code2, mbr_idx, mbr_idx2, mbr_rows, mbr_part, mbr_min, mbr_max, mbr_pr, mbr_sub, mbr_domf,
        mbr_pairs, mbr_gmin, mbr_gpr, mbr_lpt;
    bool used_mbr = false;
    size_t slot_hint = 0;       // candidate slots the next run allocates (grown on overflow)
    int64_t slot_reruns = 0;    // runs repeated because the slots overflowed
    int64_t mbr_tiles = 0;
    // the candidate slots after the filter (rows / sortkey / slot_src) or, after the
    // prefilter's compaction, its *2 buffers: downstream stages read these (no swap, so
    // the stream-sized buffers keep their capacity across queries)
    DevBuf *s_rows = &rows, *s_key = &sortkey, *s_src = &slot_src;
    // single-pass output: look-back words per tile; what the last run wrote
    DevBuf lbuf;
    DevBuf tile_hist, tile_cand;      // per-tile duplicate histograms / surviving candidates (output counts)
    bool hist_count = false;
    bool row_flags_done = false;      // the last run's count pass wrote PipeIn::row_flags
    // status planes (k_filter): B / E words per tile instead of a status word per tuple; the
    // designated duplicate group (B) is the largest group of the last run with the same shape
    DevBuf planes;
    bool planes_on = false;
    int32_t dom_kj = -1, dom_km = 0;
    // the small-set route of the last query (prefilter rounds + brute pair pass), replayed by
    // the next with device-sized launches (bounds from this query's counts)
    struct Plan {
        static constexpr int kMaxRounds = 3;
        bool valid = false;
        int rounds = 0;
        uint32_t bound[kMaxRounds + 1] = {};   // slots entering round r; bound[rounds]: the brute pass
        bool f64 = false, ints = false;
        int D = 0, Kp = 0, M = 0;
        bool single = false, global = false;
        bool tiny = false;                     // its final slots were few: the one-workgroup tail
    } plan;
    int64_t plan_runs = 0, plan_misses = 0;
    // candidate prefilter learning: when its first round cut fewer than 3 % of the slots (large
    // anti-correlated skylines: the second-level pruners dominate almost nothing) the next queries
    // skip it -- it is exact, so the result does not change -- and every 16th query probes again
    bool pf_skip = false;
    uint32_t pf_since_probe = 0, pf_mt = 0;    // pf_mt: the slot count the skip was learned on
    int64_t pf_skipped = 0;
    bool last_planned = false, last_plan_miss = false;   // the last query's route (counters[7] bits 3, 4)
    bool last_tiny = false;                              // ... its tail in one workgroup (bit 5)
    int64_t tiny_runs = 0;
    uint32_t tiny_block = 0;                             // plans learned without trying the tail (after a miss)
    DevBuf cand_lb;                                      // the fused prefilter pass's look-back words
    DevBuf dbg_clk;                                      // measurement builds: the tail's phase clocks
    bool fused = false;
    const int64_t *fused_ids = nullptr;
    const int32_t *fused_org = nullptr;
    // multi-GPU step (sky_dist_*): what the export left for the merge
    DevBuf dverd;                         // u64 words: [0] the run's verdict, [8..15] the merge's summary
    DevBuf dist_flag, dist_pos, dist_own; // per unit: alive (u32), export position; per own row: fates
    DevBuf dist_dom;                      // per own row: dominated bits of the wide pair pass (u32, kept zero)
    DevBuf out_lb;                        // k_out_hist_scan's look-back words (zeroed when allocated)
    uint32_t out_epoch = 0;               // ... and the epoch its last launch tagged them with
    bool dist_slots = false;              // units = candidate slots (small-set route) or representatives
    uint32_t dist_n = 0;                  // units (their bound on the planned route)
    const uint32_t *dist_d_n = nullptr;   // the unit count on the device (planned route)
    PlanCheck dist_pc;
    bool dist_verdict_pending = false;    // the verdict is computed by the one-workgroup export tail
    int64_t host_syncs = 0;               // host synchronisations (read-backs) of this pipeline
    // host-visible pinned staging
    void *pin = nullptr;
    size_t pin_cap = 0;

    // results of the last run
    uint32_t n = 0, m = 0, nps = 0, mt = 0, mr = 0, mg = 0, nout = 0, mt_pre = 0;
    uint32_t n_prev = 0, nout_prev = 0;   // the last completed run's tuples / output (the write pass's form)
    int M = 1, Kp = 1, K = 1;
    bool f64 = false, ties = false, u16 = false, ints = false;   // ints: every candidate value an integer in [0, 65535]
    std::vector<uint32_t> h_dup;
    std::vector<int32_t> h_entries;
    std::vector<unsigned long long> h_lsz, h_surv;
    int64_t sfs_rounds = 0, sfs_pairs_upper = 0;
    // algorithmic dominance work of the last run: distinct vectors per
    // partition n_k, distinct local-skyline vectors s_k, W = pair tests
    std::vector<uint32_t> h_seg_n, h_seg_s;
    int64_t dom_w = 0;

    // pinned bump buffer for small host->device uploads (segment tables, tile lists):
    // asynchronous, no implicit synchronisation of the stream
    void *up = nullptr;
    size_t up_cap = 0, up_used = 0;

    ~Pipe();
    int pinned(size_t bytes);
    int upload(void *dst, const void *src, size_t bytes, hipStream_t st);
};

struct Ctx;
int pipe_run(Ctx &c, Pipe &p, const PipeIn &in, PhaseTimer *tm);
// pre-size the tuple-count-proportional buffers of a run over n tuples
int pipe_reserve(Ctx &c, Pipe &p, uint32_t n);
// SKY_MBR_LPT=0 turns the bounding-box pass's cost-ordered work queue off (A/B knob)
// read device ranges into host memory in one synchronisation (one gather launch when they are small)
// prewritten: a kernel of the run already wrote the words into p.pin (this layout); only the
// synchronisation and the unpacking remain
int sync_read(Pipe &p, hipStream_t st, const std::vector<std::pair<const void *, size_t>> &srcs,
              std::vector<void *> dsts, bool prewritten = false);
// the designated duplicate group of the next run's status planes, from p.h_dup
void pick_dom_group(Pipe &p, int KM);
// stream-ordered output of the tuples selected by the last run
int pipe_output(Ctx &c, Pipe &p, const PipeIn &in, bool select_local, int64_t *d_ids_out, int32_t *d_origin_out,
                double *d_rows_out, int64_t cap, int64_t *n_out, uint8_t *d_row_flags);

}  // namespace sky
