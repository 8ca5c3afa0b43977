// ctx.h — the object behind an sky_ctx* handle.
#pragma once
#include <hip/hip_runtime.h>
#include <cstring>
#include <map>
#include <string>
#include <vector>
#include "engine.h"

namespace sky {

// HIP-event timings of the pipeline phases of one query (profiling only)
struct PhaseTimer {
    hipEvent_t ev[SKY_PHASES + 1] = {};
    bool marked[SKY_PHASES + 1] = {};
    bool ok = false;
    void init() {
        ok = true;
        for (auto &e : ev)
            if (hipEventCreate(&e) != hipSuccess) ok = false;
    }
    void reset() {
        for (bool &m : marked) m = false;
    }
    void mark(int i, hipStream_t st) {
        if (ok && i >= 0 && i <= SKY_PHASES) {
            hipEventRecord(ev[i], st);
            marked[i] = true;
        }
    }
    void destroy() {
        for (auto &e : ev)
            if (e) hipEventDestroy(e);
    }
};

// accumulated HIP-event time of one kernel family on the launching stream
struct KTime {
    double ms = 0;
    int64_t launches = 0, units = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    std::vector<int64_t> pending_units;
};

struct Ctx {
    int dev = 0, D = 2, P = 8, algo = SKY_ALGO_ANGLE, sem = SKY_SEM_REFERENCE, grid_filter = 0;
    double domain = 1000.0;
    hipStream_t own = nullptr, st = nullptr;
    Pipe main, aux;
    std::vector<int64_t> lsz, surv;
    int K_last = 0;
    int profile = 0;            // 0 off, 1 kernel timers (HIP events per timed kernel), 2 + phase events
    int warm_mode = 0;          // sky_ctx_warmup: 1 force the bounding-box pass, 2 force the SFS path
    PhaseTimer pt;
    double phase_ms[SKY_PHASES] = {};
    int64_t counters[8] = {};
    int64_t dom_w = 0;          // algorithmic dominance pair tests of the last query
    std::map<std::string, KTime> kt;
    std::vector<hipEvent_t> event_pool;
    // staging for the host-buffer entry points
    DevBuf h_vals, h_ids, h_keys, h_out_ids, h_out_org, h_origin, h_flags;
    // multi-GPU phase-1 state (the shard stays caller-owned)
    PipeIn shard;
    bool shard_valid = false;
    // the one-read multi-GPU step (sky_dist_*): 0 none, 1 exported, 2 exported with a NaN (the
    // block carries the verdict, the merge only completes the collective pattern), 3 merged
    int dist_state = 0;
    int64_t dist_cap = 0;
    int64_t dist_hist_pairs = -1;   // |own| x |union| of the last merge (-1: none yet)
    int dist_last_route = 0;        // 0: one pair kernel over the blocks, 1: the bounding-box pass
    int dist_world = 0;
    bool dist_merged = false;
    int64_t host_syncs = 0;     // entry-point level host synchronisations (pipelines count their own)
    DevBuf dist_sum;            // the merge's summary of every block header (u64 words)
    DevBuf dist_union, dist_ukey, dist_umult, dist_uflags;   // the compacted union (bounding-box path)
    // bulk CSV ingest workspace (k_csv.hip)
    DevBuf csv_blk, csv_scr, csv_lines, csv_status, csv_counts, csv_ids, csv_vals, csv_keep, csv_pos, csv_text, csv_slow,
        csv_spans;
    DevBuf prof_k, prof_v, prof_scr;   // sky_profile_sort_dev workspace
    // batched per-key inserts (sky_parts_insert): the call's upload (descriptors, work items,
    // ids, rows) and work arrays on the device; pinned staging slots, each reusable once its
    // event (the upload) has completed
    // the upload goes out on a copy stream into one of two device buffers, so that a call's
    // upload overlaps the previous call's kernels; part_done[b]: the kernels that read buffer b
    DevBuf part_batch[2], part_work;
    // sky_parts_global_merge work buffers
    DevBuf pgm_w, pgm_flag, pgm_tsel, pgm_tpos, pgm_scr, pgm_lists, pgm_surv, pgm_sorg, pgm_ids, pgm_org, pgm_up, pgm_err;
    hipStream_t part_copy_st = nullptr;
    hipEvent_t part_done[2] = {nullptr, nullptr};
    bool part_done_rec[2] = {false, false};
    int part_buf_next = 0;
    struct Staging {
        void *h = nullptr;
        size_t cap = 0;
        hipEvent_t ev = nullptr;
        bool used = false;
    };
    Staging part_stage[4];
    int part_stage_next = 0;
    ~Ctx() {
        for (Staging &s : part_stage) {
            if (s.h) (void)hipHostFree(s.h);
            if (s.ev) (void)hipEventDestroy(s.ev);
        }
        for (hipEvent_t &e : part_done)
            if (e) (void)hipEventDestroy(e);
        if (part_copy_st) {
            (void)hipStreamSynchronize(part_copy_st);
            (void)hipStreamDestroy(part_copy_st);
        }
    }

    int Kq() const {
        if (algo == SKY_ALGO_GRID && sem == SKY_SEM_COMPLETE) return std::max(P, 1 << D);
        return P;
    }
    KeyParams kp() const {
        KeyParams k{};
        k.algo = algo;
        k.P = P;
        k.K = Kq();
        k.dim_width = domain / (double)P;
        k.grid_mid = domain / 2.0;
        k.margin = angle_margin(P);
        k.ang_scale = D >= 2 ? (float)((2.0 / 3.141592653589793) / (double)(D - 1) * (double)P) : 0.0f;
        k.ang_lo = (float)k.margin;
        k.ang_hi = (float)(1.0 - k.margin);
        // special-case keys: avg = c / (D-1), key = clamp(d2i(avg * P)) (AnglePartitioner,
        // FlinkSkyline.java:760-780), c = 0..2(D-1) <= 30; keys < P <= 256 fit a byte
        uint64_t sp[4] = {0, 0, 0, 0};
        for (int c = 0; D >= 2 && c <= 2 * (D - 1); c++) {
            const double avg = (double)c / (double)(D - 1);
            const double t = avg * (double)P;
            int32_t key = t != t ? 0 : t >= 2147483647.0 ? 2147483647 : t <= -2147483648.0 ? INT32_MIN : (int32_t)t;
            key = key > P - 1 ? P - 1 : (key < 0 ? 0 : key);
            sp[c / 8] |= (uint64_t)(uint32_t)key << ((c % 8) * 8);
        }
        k.ang_special0 = sp[0];
        k.ang_special1 = sp[1];
        k.ang_special2 = sp[2];
        k.ang_special3 = sp[3];
        k.grid_filter = algo == SKY_ALGO_GRID ? grid_filter : 0;
        return k;
    }
    hipEvent_t take_event() {
        if (!event_pool.empty()) {
            hipEvent_t e = event_pool.back();
            event_pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        hipEventCreate(&e);
        return e;
    }
    // level 1 (light, usable inside a timed region): only the single kernels a measurement
    // reads back; every timed pair is two event records on the stream (≈ 10 µs of gap each
    // between short kernels), so the small-phase timers run at level 2 only
    static bool ktimer_light(const char *name) {
        static const char *const names[] = {"filter", "mbr", "dom", "csv_count", "csv_lines", "csv_parse",
                                            "union_fate"};
        for (const char *n : names)
            if (!strcmp(n, name)) return true;
        return false;
    }
    void ktimer_begin(const char *name, hipStream_t s) {
        if (!profile || (profile < 2 && !ktimer_light(name))) return;
        KTime &k = kt[name];
        hipEvent_t a = take_event(), b = take_event();
        hipEventRecord(a, s);
        k.pending.push_back({a, b});
        k.pending_units.push_back(0);
    }
    void ktimer_end(const char *name, hipStream_t s, int64_t units) {
        if (!profile || (profile < 2 && !ktimer_light(name))) return;
        KTime &k = kt[name];
        if (k.pending.empty()) return;
        hipEventRecord(k.pending.back().second, s);
        k.pending_units.back() = units;
    }
    void ktimer_collect() {
        for (auto &kv : kt) {
            KTime &k = kv.second;
            for (size_t i = 0; i < k.pending.size(); i++) {
                float ms = 0;
                hipEventSynchronize(k.pending[i].second);
                if (hipEventElapsedTime(&ms, k.pending[i].first, k.pending[i].second) == hipSuccess) {
                    k.ms += ms;
                    k.launches++;
                    k.units += k.pending_units[i];
                }
                event_pool.push_back(k.pending[i].first);
                event_pool.push_back(k.pending[i].second);
            }
            k.pending.clear();
            k.pending_units.clear();
        }
    }
};

}  // namespace sky

struct sky_ctx : sky::Ctx {};

// one Flink key's local skyline (SkylineLocalProcessor.localSkylineState, FlinkSkyline.java:243-248)
// as distinct vectors + the tuples on them (k_part.hip): an insert costs O(|B| (|B| + R)) pair
// tests and no host read.  The counts live on the device; the host keeps bounds for launch
// sizes and capacities, tightened from the commit kernel's host-mapped mirror.
constexpr uint32_t kPartRing = 4096;       // inserts whose cumulative tuple counts the host keeps
struct sky_part {
    sky_ctx *ctx = nullptr;
    int32_t key = 0;
    // distinct vectors: rows f64 [R][D], alive flag, tuples per rep; tuples: id, rep (insertion order)
    sky::DevBuf rrows, ralive, rcnt, tids, trep;
    size_t Rcap = 0, Tcap = 0;              // capacities (elements)
    sky::DevBuf dcnt;                       // device counts: R, T, dead (u64)
    uint32_t *mirror = nullptr;             // host-mapped seqlock mirror: begin, R, T, dead lo, hi, end
    uint32_t *mirror_dev = nullptr;         // its device address
    uint32_t seq = 0;                       // inserts issued (the mirror's tags)
    uint64_t issued = 0;                    // tuples issued
    uint64_t cum[kPartRing] = {};           // tuples issued up to and including insert s (s % kPartRing)
    uint32_t seq_known = 0;                 // the counts below are those after insert seq_known
    uint64_t R_known = 0, T_known = 0, dead_known = 0, cum_known = 0;
    std::vector<sky::DevBuf> grave;         // replaced state buffers, freed at the next synchronisation
    // compaction targets and read-out staging
    sky::DevBuf rrows2, ralive2, rcnt2, tids2, trep2, rk, rp, tk, tp, out_rows, scratch, words;
    void *pin = nullptr;                    // pinned read-back words
    ~sky_part() {
        if (pin) (void)hipHostFree(pin);
        if (mirror) (void)hipHostFree(mirror);
    }
};

struct sky_stream_landmark;     // stream.hip: the landmark window's distinct-vector state
struct sky_stream {
    sky_ctx *ctx = nullptr;
    int64_t window = 0;         // 0: landmark
    sky_stream_landmark *lm = nullptr;
    sky::DevBuf ids[2], rows[2];   // sliding window: a ring of two buffers
    int cur = 0;
    int64_t off = 0, n = 0;     // resident tuples (sliding window: [off, off + n) of buffer `cur`)
    int64_t cap = 0;            // capacity (tuples) of both ring buffers
    int64_t appended = 0;
    sky::DevBuf out_ids, out_org, nanflag;
    void *nan_host = nullptr;   // pinned word: the append's NaN admission flag
    // sky_stream_query_async: the result copy to host memory on its own stream (overlaps the
    // next appends on the context's stream); ev_ready / ev_done bracket it
    hipStream_t cst = nullptr;
    hipEvent_t ev_ready = nullptr, ev_done = nullptr;
    bool copy_pending = false;
    sky_stream() = default;
    sky_stream(const sky_stream &) = delete;
    sky_stream &operator=(const sky_stream &) = delete;
    ~sky_stream();
};
