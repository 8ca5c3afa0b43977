// engine.hip — host orchestration of one skyline query on one MI355X.
//
//   sample + pruners -> k_filter (HBM stream) -> scan -> k_compact<T>
//   -> radix sort (partition | score | hash) -> duplicate collapse
//   -> segmented SFS (local skylines L_k) -> SFS over the union of the L_k (G)
//   -> per-tuple fate pass (|L_k|, survivors_k, stream-ordered ids)
//
// Host synchronisations happen only where the host must size the next launch
// (candidate count, representative count, per-round SFS segment counts).
#include "engine.h"
#include "sky_tail.h"
#include "knobs.h"
#include "ctx.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace sky {

size_t mbr_group_slots(uint32_t mr);   // k_mbr.hip: gmin / gprange entries (groups + super-groups)

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) {                                                           \
            set_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " #expr);   \
            return SKY_E_HIP;                                                             \
        }                                                                                 \
    } while (0)
#define SKY_TRY(expr)            \
    do {                         \
        int r_ = (expr);         \
        if (r_ != SKY_OK) return r_; \
    } while (0)

int DevBuf::ensure(size_t bytes) {
    if (bytes <= cap && p) return SKY_OK;
    // a buffer that has to grow again gets 1.5x headroom, a first one 1/8: query-to-query size
    // changes (candidate counts, rep counts) then reallocate rarely (each hipFree synchronises the
    // device and landed inside a query's latency: the learned prefilter skip grew every rep-sized
    // buffer by 0.3 % in the first skipping query, +4.6 ms at std-anti 8D 2M)
    const bool regrow = cap != 0;
    release();
    size_t want = std::max<size_t>(bytes, 256);
    want = regrow ? std::max(want, bytes + bytes / 2) : want + want / 8;
    want = (want + 4095) & ~size_t(4095);
    static const bool trace_alloc = SKY_MEASURE_ENV("SKY_TRACE_ALLOC") != nullptr;   // measurement only
    auto t0 = std::chrono::steady_clock::now();
    const hipError_t me = hipMalloc(&p, want);
    if (trace_alloc)
        fprintf(stderr, "[sky] hipMalloc %zu bytes: %.3f ms\n", want,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    if (me != hipSuccess) {
        p = nullptr;
        cap = 0;
        (void)hipGetLastError();
        set_error("hipMalloc of " + std::to_string(want) + " bytes failed");
        return SKY_E_NOMEM;
    }
    cap = want;
    return SKY_OK;
}

void DevBuf::release() {
    static const bool trace_alloc = SKY_MEASURE_ENV("SKY_TRACE_ALLOC") != nullptr;   // measurement only
    if (p) {
        auto t0 = std::chrono::steady_clock::now();
        (void)hipFree(p);
        if (trace_alloc)
            fprintf(stderr, "[sky] hipFree %zu bytes: %.3f ms\n", cap,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    p = nullptr;
    cap = 0;
}

Pipe::~Pipe() {
    if (pin) (void)hipHostFree(pin);
    if (up) (void)hipHostFree(up);
}

int Pipe::upload(void *dst, const void *src, size_t bytes, hipStream_t st) {
    if (!bytes) return SKY_OK;
    const size_t need = (bytes + 255) & ~size_t(255);
    if (up_used + need > up_cap) {
        // wrap: every earlier upload must have been consumed before the area is reused
        host_syncs++;
        if (hipStreamSynchronize(st) != hipSuccess) {
            set_error("stream synchronisation failed");
            return SKY_E_HIP;
        }
        up_used = 0;
        if (need > up_cap) {
            if (up) (void)hipHostFree(up);
            up = nullptr;
            up_cap = std::max<size_t>(need, size_t(4) << 20);
            if (hipHostMalloc(&up, up_cap, hipHostMallocDefault) != hipSuccess) {
                up = nullptr;
                up_cap = 0;
                set_error("hipHostMalloc failed");
                return SKY_E_NOMEM;
            }
        }
    }
    char *slot = (char *)up + up_used;
    memcpy(slot, src, bytes);
    up_used += need;
    if (hipMemcpyAsync(dst, slot, bytes, hipMemcpyHostToDevice, st) != hipSuccess) {
        set_error("upload failed");
        return SKY_E_HIP;
    }
    return SKY_OK;
}

int Pipe::pinned(size_t bytes) {
    if (bytes <= pin_cap && pin) return SKY_OK;
    if (pin) (void)hipHostFree(pin);
    pin = nullptr;
    size_t want = std::max<size_t>(bytes, 1 << 16);
    if (hipHostMalloc(&pin, want, hipHostMallocDefault) != hipSuccess) {
        pin = nullptr;
        pin_cap = 0;
        set_error("hipHostMalloc failed");
        return SKY_E_NOMEM;
    }
    pin_cap = want;
    return SKY_OK;
}

// SKY_DEBUG=1: synchronise and check after every stage, naming the stage
static int debug_level() {
    static int lvl = [] {
        const char *e = SKY_MEASURE_ENV("SKY_DEBUG");
        return e ? atoi(e) : 0;
    }();
    return lvl;
}
// SKY_SFS16=0 forces the generic f32/f64 SFS (read per query: the tests compare the
// two paths in one process)
static bool sfs16_disabled() {
    const char *e = SKY_ENV("SKY_SFS16");
    return e && atoi(e) == 0;
}
// SKY_PREFILTER=0 skips the candidate prefilter (A/B knob; read per query)
static bool prefilter_disabled() {
    const char *e = SKY_ENV("SKY_PREFILTER");
    return e && atoi(e) == 0;
}
static int prefilter_m2() {   // second-level pruners per partition (SKY_PREFILTER_M2, default 16)
    static const int m = [] {
        const char *e = SKY_MEASURE_ENV("SKY_PREFILTER_M2");
        const int v = e ? atoi(e) : 16;
        return v < 1 ? 1 : (v > 64 ? 64 : v);
    }();
    return m;
}
constexpr uint32_t kPrefilterMin = 4096;
// candidate slots of a first run (SKY_SLOT_MIN overrides: tests force the overflow re-run)
static size_t slot_min() {
    const char *e = SKY_ENV("SKY_SLOT_MIN");
    return e ? (size_t)std::max(1, atoi(e)) : (size_t(1) << 20);
}
constexpr uint32_t kPrefilterProbe = 16;  // a skipped prefilter is probed again every 16 queries
constexpr uint32_t kTinyBlock = 16;       // plans learned without the one-workgroup tail after it missed
constexpr uint32_t kPickInFilterMax = 16u << 20;   // tuples up to which the filter picks its own pruners
constexpr uint32_t kTailTilesMax = 1024;        // tiles up to which the brute route's counts run as k_tail_counts
constexpr int kPrefilterRounds = 3;   // fewer slots: the SFS runs in one small pass anyway
static bool fused_disabled() {   // SKY_FUSED_OUT=0: count pass + scan + write pass (A/B knob)
    const char *e = SKY_ENV("SKY_FUSED_OUT");
    return e && atoi(e) == 0;
}
static bool fused_onepass() {   // SKY_FUSED_OUT=2: the one-pass look-back output kernel
    const char *e = SKY_ENV("SKY_FUSED_OUT");
    return e && atoi(e) == 2;
}
static bool hist_disabled() {   // SKY_HIST_COUNT=0: the status-word count pass (A/B knob)
    const char *e = SKY_MEASURE_ENV("SKY_HIST_COUNT");
    return e && e[0] == '0';
}
// SKY_PLANES=0: the filter stores every status word (A/B knob, read per query)
static bool planes_disabled() {
    const char *e = SKY_MEASURE_ENV("SKY_PLANES");
    return e && e[0] == '0';
}
// SKY_PLAN=0: every query takes the host-synchronised route (A/B knob, read per query)
static bool plan_disabled() {
    const char *e = SKY_ENV("SKY_PLAN");
    return e && e[0] == '0';
}
// a device-sized launch's bound for a count the last query saw
static uint32_t plan_bound(uint32_t x) { return x + x / 4 + 1024u; }
// SKY_MBR=0 keeps the round-based SFS for large rep sets (A/B knob, read per query);
// SKY_MBR_MIN: smallest rep count for the bounding-box pruned all-pairs pass
static bool mbr_disabled() {
    const char *e = SKY_ENV("SKY_MBR");
    return e && atoi(e) == 0;
}
static uint32_t mbr_min() {
    const char *e = SKY_ENV("SKY_MBR_MIN");
    return e ? (uint32_t)atoi(e) : 16384u;
}
// Up to 32768 slots the brute pair pass (one 64 x 64 block pair per workgroup, no sort or
// dedup) beats the sorted bounding-box route, whose 64-row y tiles leave a small rep set at a
// few hundred waves on 1024 SIMDs (C5 sliding window: 21-25k reps took 0.6-0.85 ms there).
uint32_t brute_max() {
    static const uint32_t v = [] {
        const char *e = SKY_MEASURE_ENV("SKY_BRUTE_MAX");
        const long x = e ? atol(e) : 32768;
        return (uint32_t)std::min<long>(std::max<long>(x, 64), 1 << 20);
    }();
    return v;
}
static bool brute_disabled() {
    const char *e = SKY_ENV("SKY_BRUTE");
    return e && atoi(e) == 0;
}
// SKY_BRUTE16=0: the small-set pair pass compares f32 even for integer rows (A/B knob)
static bool cand_fused_disabled() {   // SKY_CAND_FUSED=0: pick / filter / scan / compact launches (A/B knob)
    const char *e = SKY_ENV("SKY_CAND_FUSED");
    return e && e[0] == '0';
}
// the fused prefilter pass's look-back words of each planned round: [tiles][u64] + a ticket word
// the fused pass after one k_cand_pick, one slot per thread (default), or redoing the pick in every
// workgroup with four slots per thread (SKY_CAND_FUSED=1, A/B knob): the per-workgroup pick measured
// slower at every size tried -- C4's 241k slots 46 vs 27 us, C2's 40k 28.5 vs 24.6, a 1M 6D trigger's
// 29.7 vs 23.1 (with k_cand_min)
static bool cand_picked(uint32_t) {
    const char *e = SKY_ENV("SKY_CAND_FUSED");
    return !(e && e[0] == '1');
}
static size_t cand_lb_bytes(uint32_t bound) { return (size_t)cand_fused_tiles(bound, cand_picked(bound)) * 8 + 64; }
static bool tail_counts_disabled() {   // SKY_TAIL_COUNTS=0: hist counts / scan / stat reduce / gather launches (A/B knob)
    const char *e = SKY_ENV("SKY_TAIL_COUNTS");
    return e && e[0] == '0';
}
static bool epilogue_disabled() {   // SKY_OUT_EPILOGUE=0: k_stat_reduce + k_gather_words launches (A/B knob)
    const char *e = SKY_ENV("SKY_OUT_EPILOGUE");
    return e && e[0] == '0';
}
static bool sparse_out_disabled() {   // SKY_SPARSE_OUT=0: the write pass always loads every id first (A/B knob)
    const char *e = SKY_ENV("SKY_SPARSE_OUT");
    return e && e[0] == '0';
}
static bool fill_embed_disabled() {   // SKY_FILL_EMBED=0: the query's fills as their own launch (A/B knob)
    const char *e = SKY_ENV("SKY_FILL_EMBED");
    return e && e[0] == '0';
}
static bool finish_fold_disabled() {   // SKY_FINISH_FOLD=0: k_brute_finish as its own launch (A/B knob)
    const char *e = SKY_ENV("SKY_FINISH_FOLD");
    return e && e[0] == '0';
}
static bool tiny_disabled() {    // SKY_TINY=0: the planned tail as one launch per stage (A/B knob)
    const char *e = SKY_ENV("SKY_TINY");
    return e && e[0] == '0';
}
static bool brute16_disabled() {
    const char *e = SKY_ENV("SKY_BRUTE16");
    return e && atoi(e) == 0;
}
// SKY_GATHER=0 reads counters back by one hipMemcpyAsync per range (A/B knob)
static bool gather_disabled() {
    const char *e = SKY_ENV("SKY_GATHER");
    return e && atoi(e) == 0;
}
static int stage_check(hipStream_t st, const char *where) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && debug_level()) {
        e = hipStreamSynchronize(st);
        if (e == hipSuccess) e = hipGetLastError();
    }
    if (e != hipSuccess) {
        set_error(std::string("HIP error ") + hipGetErrorString(e) + " in stage " + where);
        return SKY_E_HIP;
    }
    return SKY_OK;
}
#define STAGE(st, name) SKY_TRY(stage_check(st, name))

static int choose_B(bool f64, int D) {
    const int DP = f64 ? padded_dims<double>(D) : padded_dims<float>(D);
    const int rowb = DP * (f64 ? 8 : 4);
    int lim = 49152 / rowb;
    int B = 1024;
    while (B > lim) B >>= 1;
    return B < 64 ? 64 : B;
}

static size_t row_bytes(bool f64, int D) {
    return f64 ? padded_dims<double>(D) * 8 : padded_dims<float>(D) * 4;
}

// ---- segmented blocked SFS -------------------------------------------------------
// Several small host arrays (work lists, segment tables) staged into ONE device
// buffer by one upload: one copy dispatch instead of one per array.
struct UpBlob {
    std::vector<char> h;
    size_t put(const void *src, size_t bytes) {
        const size_t off = (h.size() + 255) & ~size_t(255);
        h.resize(off + bytes);
        if (bytes) memcpy(h.data() + off, src, bytes);
        return off;
    }
    int send(Pipe &p, DevBuf &dst, hipStream_t st) {
        SKY_TRY(dst.ensure(std::max<size_t>(h.size(), 256)));
        return p.upload(dst.p, h.data(), h.size(), st);
    }
};

static int sfs_run(Ctx &c, Pipe &p, const void *rows, const uint64_t *key, uint32_t nrep,
                   std::vector<uint32_t> begin, std::vector<uint32_t> cnt, bool full, uint8_t *alive) {
    hipStream_t st = c.st;
    const int D = c.D;
    const uint32_t nseg = (uint32_t)begin.size();
    const int B = choose_B(p.f64, D);
    const size_t rb = row_bytes(p.f64, D);
    constexpr uint32_t kTileP = 1024;   // 256 threads x PPT(4)
    SKY_TRY(p.act.ensure((size_t)nrep * 4));
    SKY_TRY(p.act2.ensure((size_t)nrep * 4));
    SKY_TRY(p.keep.ensure((size_t)nrep * 4));
    SKY_TRY(p.keep_scan.ensure((size_t)nrep * 4));
    // large partitions: rounds of BB candidates; X streamed through LDS in tiles of TB rows
    const int TB = std::min(512, B);
    const int BB = 4096;
    SKY_TRY(p.xkeep.ensure((size_t)nseg * BB));
    SKY_TRY(p.segs.ensure((size_t)nseg * sizeof(SfsSeg)));
    SKY_TRY(p.seg_list.ensure((size_t)nseg * 4));
    SKY_TRY(p.segcnt.ensure((size_t)nseg * 4));
    SKY_TRY(p.scratch.ensure(scan_scratch_words(nrep + 1) * 4 + 64));
    SKY_TRY(p.totals.ensure(64));
    std::vector<SfsSeg> hsegs(nseg);
    std::vector<uint32_t> work;
    std::vector<SfsTile> tiles;
    // small partitions: the whole SFS in one workgroup each, one launch, no host sync
    {
        constexpr uint32_t kSmallSeg = 2048;
        std::vector<uint32_t> small;
        for (uint32_t k = 0; k < nseg; k++) {
            hsegs[k] = SfsSeg{begin[k], cnt[k]};
            if (cnt[k] && cnt[k] <= kSmallSeg) small.push_back(k);
        }
        if (debug_level() >= 2) {
            fprintf(stderr, "[sky] sfs nrep=%u nseg=%u small=%zu full=%d:", nrep, nseg, small.size(), (int)full);
            for (uint32_t k = 0; k < nseg; k++) fprintf(stderr, " %u", cnt[k]);
            fprintf(stderr, "\n");
        }
        if (!small.empty()) {
            SKY_TRY(p.conf_small.ensure((size_t)nrep * rb));
            UpBlob ub;
            const size_t o_segs = ub.put(hsegs.data(), nseg * sizeof(SfsSeg));
            const size_t o_small = ub.put(small.data(), small.size() * 4);
            SKY_TRY(ub.send(p, p.seg_small, st));
            c.ktimer_begin("sfs_small", st);
            launch_sfs_small(D, p.f64, full, p.ties, std::min(512, B / 2), rows, key,
                             (const SfsSeg *)(p.seg_small.as<char>() + o_segs),
                             (const uint32_t *)(p.seg_small.as<char>() + o_small), (uint32_t)small.size(), alive,
                             p.conf_small.p, st);
            c.ktimer_end("sfs_small", st, 0);
            STAGE(st, "sfs_small");
            for (uint32_t k : small) cnt[k] = 0;
            p.sfs_rounds++;
        }
    }
    bool any_big = false;
    for (uint32_t k = 0; k < nseg; k++) any_big |= cnt[k] != 0;
    if (!any_big) return SKY_OK;
    launch_iota(p.act.as<uint32_t>(), nrep, st);
    for (;;) {
        work.clear();
        for (uint32_t k = 0; k < nseg; k++) {
            hsegs[k] = SfsSeg{begin[k], cnt[k]};
            if (cnt[k]) work.push_back(k);
        }
        if (work.empty()) break;
        p.sfs_rounds++;
        if (debug_level() >= 2) {
            fprintf(stderr, "[sky] sfs round %lld full=%d segs:", (long long)p.sfs_rounds, (int)full);
            for (uint32_t k : work) fprintf(stderr, " %u:%u", k, cnt[k]);
            fprintf(stderr, "\n");
        }
        SKY_TRY(p.upload(p.segs.p, hsegs.data(), nseg * sizeof(SfsSeg), st));
        SKY_TRY(p.upload(p.seg_list.p, work.data(), work.size() * 4, st));
        c.ktimer_begin("block_sky", st);
        launch_block_sky(D, p.f64, full, p.ties, BB, TB, rows, key, p.act.as<uint32_t>(), p.segs.as<SfsSeg>(),
                         p.seg_list.as<uint32_t>(), (uint32_t)work.size(), alive, p.xkeep.as<uint8_t>(), st);
        c.ktimer_end("block_sky", st, 0);
        STAGE(st, "block_sky");
        tiles.clear();
        uint32_t out = 0;
        for (uint32_t k : work) {
            const uint32_t xk = std::min<uint32_t>(BB, cnt[k]);
            const uint32_t rem = cnt[k] - xk;
            for (uint32_t off = 0; off < rem; off += kTileP) {
                const uint32_t cn = std::min<uint32_t>(kTileP, rem - off);
                tiles.push_back(SfsTile{k, begin[k] + xk + off, cn, out});
                out += cn;
            }
            p.sfs_pairs_upper += (int64_t)rem * xk + (int64_t)xk * (xk - 1) / 2;
        }
        if (out == 0) break;
        SKY_TRY(p.tiles.ensure(tiles.size() * sizeof(SfsTile)));
        SKY_TRY(p.upload(p.tiles.p, tiles.data(), tiles.size() * sizeof(SfsTile), st));
        c.ktimer_begin("sfs_filter", st);
        launch_filter_rest(D, p.f64, full, BB, TB, rows, p.act.as<uint32_t>(), p.tiles.as<SfsTile>(),
                           (uint32_t)tiles.size(), p.segs.as<SfsSeg>(), p.xkeep.as<uint8_t>(), p.keep.as<uint32_t>(),
                           st);
        c.ktimer_end("sfs_filter", st, out);
        STAGE(st, "sfs_filter");
        scan_excl_u32(p.keep.as<uint32_t>(), p.keep_scan.as<uint32_t>(), out, nullptr, p.scratch.as<uint32_t>(), st);
        HIP_TRY(hipMemsetAsync(p.segcnt.p, 0, nseg * 4, st));
        launch_act_compact(p.act.as<uint32_t>(), p.keep.as<uint32_t>(), p.keep_scan.as<uint32_t>(),
                           p.tiles.as<SfsTile>(), (uint32_t)tiles.size(), p.act2.as<uint32_t>(),
                           p.segcnt.as<uint32_t>(), st);
        STAGE(st, "act_compact");
        SKY_TRY(p.pinned(nseg * 4));
        HIP_TRY(hipMemcpyAsync(p.pin, p.segcnt.p, nseg * 4, hipMemcpyDeviceToHost, st));
        p.host_syncs++;
        HIP_TRY(hipStreamSynchronize(st));
        p.up_used = 0;
        const uint32_t *sc = (const uint32_t *)p.pin;
        uint32_t run = 0;
        for (uint32_t k = 0; k < nseg; k++) {
            begin[k] = run;
            cnt[k] = sc[k];
            run += sc[k];
        }
        std::swap(p.act, p.act2);
    }
    return SKY_OK;
}

// ---- segmented SFS for integer-valued rows (k_dom16.hip) ---------------------------
// rows16: packed rows by position; segments [begin[k], begin[k]+cnt[k]) sorted by a
// strictly monotone score.  alive[position of round 0] = 1 for skyline members.
static int sfs_run16(Ctx &c, Pipe &p, const uint32_t *rows16, uint32_t nrep, std::vector<uint32_t> begin,
                     std::vector<uint32_t> cnt, uint8_t *alive, int W) {
    hipStream_t st = c.st;
    const uint32_t nseg = (uint32_t)begin.size();
    if (nrep == 0 || nseg == 0) return SKY_OK;
    // X per round: start small (few-skyline streams die in the first round's rest
    // filter); double while most of the rest survives a round (large skylines)
    constexpr uint32_t kBmax = 16384u;
    uint32_t B = 2048u;
    uint64_t rest_before = 0;
    const size_t rowb = (size_t)W * 4;
    SKY_TRY(p.dead16.ensure((size_t)nrep * 4));
    SKY_TRY(p.keep16.ensure(((size_t)nrep + 1) * 4));
    SKY_TRY(p.scan16.ensure(((size_t)nrep + 1) * 4));
    SKY_TRY(p.r16a.ensure((size_t)nrep * rowb));
    SKY_TRY(p.r16b.ensure((size_t)nrep * rowb));
    SKY_TRY(p.i16a.ensure((size_t)nrep * 4));
    SKY_TRY(p.i16b.ensure((size_t)nrep * 4));
    SKY_TRY(p.xbuf16.ensure((size_t)nseg * kBmax * rowb));
    SKY_TRY(p.xcnt16.ensure((size_t)nseg * 4));
    SKY_TRY(p.xseg16.ensure((size_t)nseg * sizeof(SfsSeg)));
    SKY_TRY(p.at16.ensure((size_t)nseg * 8));
    SKY_TRY(p.atv16.ensure((size_t)nseg * 8));
    SKY_TRY(p.scratch.ensure(scan_scratch_words(nrep + 1) * 4 + 64));
    const uint32_t *cur_rows = rows16;
    const uint32_t *cur_idx = nullptr;                     // round 0: identity
    uint32_t npos = 0;
    for (uint32_t k = 0; k < nseg; k++) npos = std::max(npos, begin[k] + cnt[k]);
    int flip = 0;
    std::vector<uint32_t> work;
    std::vector<SfsSeg> xseg;
    std::vector<DomItem> tri, tdiag, rest;
    const int ppt = dom16_ppt();
    const uint32_t Ty = 64u * (uint32_t)ppt;              // y rows per rest work item
    const uint32_t Tt = 64u * (uint32_t)kDomTriPPT;       // y rows per tri work item
    const uint32_t Tx_env = dom16_tx();                   // x rows per work item (0: adaptive)
    std::vector<uint32_t> at;
    for (;;) {
        work.clear();
        for (uint32_t k = 0; k < nseg; k++)
            if (cnt[k]) work.push_back(k);
        if (work.empty()) break;
        p.sfs_rounds++;
        if (debug_level() >= 2) {
            fprintf(stderr, "[sky] sfs16 round %lld B=%u segs:", (long long)p.sfs_rounds, B);
            for (uint32_t k : work) fprintf(stderr, " %u:%u", k, cnt[k]);
            fprintf(stderr, "\n");
        }
        xseg.clear();
        tri.clear();
        tdiag.clear();
        rest.clear();
        bool more = false;
        uint32_t maxch = 0;
        rest_before = 0;
        for (uint32_t k : work) rest_before += cnt[k] - std::min(B, cnt[k]);
        // x rows per item: a round with few items is latency-bound (one wave scans its
        // x rows serially), so halve the chunk until ~8k items fill the machine
        uint32_t Tx = Tx_env ? Tx_env : kDomTx;
        if (!Tx_env) {
            auto items_at = [&](uint32_t tx) {
                uint64_t c = 0;
                for (uint32_t k : work) {
                    const uint32_t xk = std::min(B, cnt[k]);
                    c += (uint64_t)((xk + tx - 1) / tx) * ((xk + Tt - 1) / Tt / 2 + 1 + (cnt[k] - xk + Ty - 1) / Ty);
                }
                return c;
            };
            while (Tx > 64 && items_at(Tx) < 8192) Tx /= 2;
        }
        for (uint32_t s = 0; s < (uint32_t)work.size(); s++) {
            const uint32_t k = work[s], b = begin[k], xk = std::min(B, cnt[k]);
            xseg.push_back(SfsSeg{b, xk});
            more |= cnt[k] > xk;
            maxch = std::max(maxch, (xk + Tx - 1) / Tx);
        }
        // items ordered by x chunk, so the first chunks (most dominating rows) run first
        for (uint32_t cx = 0; cx < maxch; cx++)
            for (uint32_t s = 0; s < (uint32_t)work.size(); s++) {
                const uint32_t k = work[s], b = begin[k], xk = std::min(B, cnt[k]);
                if (cx * Tx >= xk) continue;
                const uint32_t x0 = b + cx * Tx, nx = std::min(Tx, xk - cx * Tx);
                for (uint32_t y = 0; y < xk; y += Tt) {
                    const uint32_t y0 = b + y, ny = std::min(Tt, xk - y);
                    if (x0 >= y0 + ny) continue;                 // every x after every y
                    if (x0 + nx > y0) tdiag.push_back(DomItem{s, y0, ny, x0, nx, kDomDiag});
                    else tri.push_back(DomItem{s, y0, ny, x0, nx, 0u});
                    p.sfs_pairs_upper += (int64_t)ny * nx;
                }
                for (uint32_t y = xk; y < cnt[k]; y += Ty) {
                    const uint32_t ny = std::min(Ty, cnt[k] - y);
                    rest.push_back(DomItem{s, b + y, ny, cx * Tx, nx, kDomRest});
                    p.sfs_pairs_upper += (int64_t)ny * nx;
                }
            }
        {
            FillSet fill;
            fill.add(p.dead16.p, (size_t)npos * 4);
            HIP_TRY(fill.launch(st));
        }
        // each list is ordered by x chunk; the chunk-0 items go in a launch of their own
        // so that later chunks start after the most dominating rows have marked their y
        auto first_chunk_end = [&](const std::vector<DomItem> &v, bool rest_list) {
            size_t c = 0;
            for (; c < v.size(); c++) {
                const uint32_t off = rest_list ? v[c].x0 : v[c].x0 - xseg[v[c].seg].begin;
                if (off >= kDomTx) break;
            }
            return c;
        };
        const size_t nt = tri.size(), nd = tdiag.size(), nr = rest.size();
        const size_t nt0 = first_chunk_end(tri, false), nd0 = first_chunk_end(tdiag, false);
        const size_t nr0 = first_chunk_end(rest, true);
        // the three item lists (contiguous) and the x segments: one upload
        UpBlob ub;
        const size_t o_items = ub.put(tri.data(), nt * sizeof(DomItem));
        ub.h.resize(o_items + (nt + nd + nr) * sizeof(DomItem));
        if (nd) memcpy(ub.h.data() + o_items + nt * sizeof(DomItem), tdiag.data(), nd * sizeof(DomItem));
        if (nr) memcpy(ub.h.data() + o_items + (nt + nd) * sizeof(DomItem), rest.data(), nr * sizeof(DomItem));
        const size_t o_xseg = ub.put(xseg.data(), xseg.size() * sizeof(SfsSeg));
        SKY_TRY(ub.send(p, p.items16, st));
        DomItem *di = (DomItem *)(p.items16.as<char>() + o_items);
        const SfsSeg *xsegd = (const SfsSeg *)(p.items16.as<char>() + o_xseg);
        c.ktimer_begin("dom", st);
        // tri: the chunk-0 tiles (plain, diagonal), then the later chunks
        uint32_t *dd = p.dead16.as<uint32_t>();
        const int tp = kDomTriPPT;
        launch_dom16(W, tp, false, cur_rows, nullptr, nullptr, di, (uint32_t)nt0, 0, dd, st);
        launch_dom16(W, tp, true, cur_rows, nullptr, nullptr, di + nt, (uint32_t)nd0, 0, dd, st);
        launch_dom16(W, tp, false, cur_rows, nullptr, nullptr, di + nt0, (uint32_t)(nt - nt0), 0, dd, st);
        launch_dom16(W, tp, true, cur_rows, nullptr, nullptr, di + nt + nd0, (uint32_t)(nd - nd0), 0, dd, st);
        launch_xcompact16(W, cur_rows, cur_idx, xsegd, (uint32_t)work.size(), B,
                          p.dead16.as<uint32_t>(), p.xbuf16.as<uint32_t>(), p.xcnt16.as<uint32_t>(), alive, st);
        DomItem *dr = di + nt + nd;
        launch_dom16(W, ppt, false, cur_rows, p.xbuf16.as<uint32_t>(), p.xcnt16.as<uint32_t>(), dr, (uint32_t)nr0, B,
                     p.dead16.as<uint32_t>(), st);
        launch_dom16(W, ppt, false, cur_rows, p.xbuf16.as<uint32_t>(), p.xcnt16.as<uint32_t>(), dr + nr0,
                     (uint32_t)(nr - nr0), B, p.dead16.as<uint32_t>(), st);
        c.ktimer_end("dom", st, 0);
        STAGE(st, "dom16");
        if (!more) break;
        // next layout: the live rest of every segment, segments kept in order
        launch_keep16(p.dead16.as<uint32_t>(), npos, p.keep16.as<uint32_t>(), st);
        scan_excl_u32(p.keep16.as<uint32_t>(), p.scan16.as<uint32_t>(), npos, p.scan16.as<uint32_t>() + npos,
                      p.scratch.as<uint32_t>(), st);
        uint32_t *nrows = flip ? p.r16a.as<uint32_t>() : p.r16b.as<uint32_t>();
        uint32_t *nidx = flip ? p.i16a.as<uint32_t>() : p.i16b.as<uint32_t>();
        launch_move16(W, p.keep16.as<uint32_t>(), p.scan16.as<uint32_t>(), npos, cur_idx, cur_rows, nidx, nrows, st);
        at.clear();
        for (uint32_t k : work) { at.push_back(begin[k]); at.push_back(begin[k] + cnt[k]); }
        SKY_TRY(p.upload(p.at16.p, at.data(), at.size() * 4, st));
        launch_gather_u32(p.scan16.as<uint32_t>(), p.at16.as<uint32_t>(), (uint32_t)at.size(), p.atv16.as<uint32_t>(),
                          st);
        STAGE(st, "dom16_next");
        std::vector<uint32_t> atv(at.size());
        SKY_TRY(sync_read(p, st, {{p.atv16.p, at.size() * 4}}, {atv.data()}));
        std::fill(cnt.begin(), cnt.end(), 0u);
        npos = 0;
        uint64_t rest_after = 0;
        for (size_t s = 0; s < work.size(); s++) {
            begin[work[s]] = atv[2 * s];
            cnt[work[s]] = atv[2 * s + 1] - atv[2 * s];
            npos = std::max(npos, atv[2 * s + 1]);
            rest_after += cnt[work[s]];
        }
        if (rest_after * 2 > rest_before) B = std::min(kBmax, B * 2);
        cur_rows = nrows;
        cur_idx = nidx;
        flip ^= 1;
    }
    return SKY_OK;
}

int sync_read(Pipe &p, hipStream_t st, const std::vector<std::pair<const void *, size_t>> &srcs,
              std::vector<void *> dsts, bool prewritten) {
    p.host_syncs++;
    if (prewritten) {                   // a kernel of the run wrote the words into p.pin itself
        HIP_TRY(hipStreamSynchronize(st));
        p.up_used = 0;
        size_t off = 0;
        for (size_t i = 0; i < srcs.size(); i++) {
            if (srcs[i].second) memcpy(dsts[i], (char *)p.pin + off, srcs[i].second);
            off += (srcs[i].second + 15) & ~size_t(15);
        }
        return SKY_OK;
    }
    size_t tot = 0;
    for (auto &s : srcs) tot += (s.second + 15) & ~size_t(15);
    SKY_TRY(p.pinned(tot));
    // small word-aligned ranges: one gather launch writing into the host-mapped buffer
    FillSet g;
    bool batched = srcs.size() <= (size_t)kFillMax && tot <= (64u << 10) && !gather_disabled();
    size_t off = 0;
    for (auto &s : srcs) {
        batched &= ((uintptr_t)s.first & 3u) == 0 && (s.second & 3u) == 0;
        if (batched && s.second) {
            g.p[g.n] = (uint8_t *)s.first;
            g.bytes[g.n] = (uint32_t)s.second;
            g.val[g.n] = (uint32_t)off;
            g.n++;
        }
        off += (s.second + 15) & ~size_t(15);
    }
    if (batched) {
        if (g.n) HIP_TRY(launch_gather_words(g, p.pin, st));
    } else {
        off = 0;
        for (auto &s : srcs) {
            if (s.second) HIP_TRY(hipMemcpyAsync((char *)p.pin + off, s.first, s.second, hipMemcpyDeviceToHost, st));
            off += (s.second + 15) & ~size_t(15);
        }
    }
    HIP_TRY(hipStreamSynchronize(st));
    p.up_used = 0;
    off = 0;
    for (size_t i = 0; i < srcs.size(); i++) {
        if (srcs[i].second) memcpy(dsts[i], (char *)p.pin + off, srcs[i].second);
        off += (srcs[i].second + 15) & ~size_t(15);
    }
    return SKY_OK;
}


#ifdef SKY_MEASURE
// SKY_MBR_DBG & 8 (measurement builds): how the pair pass's work items spread over time --
// duration percentiles, the share of the pass the longest items cover, and the number of items
// in flight per twentieth of the pass (the occupancy the pass actually reaches)
static void mbr_trace_report(const unsigned long long *d, size_t n, hipStream_t st) {
    std::vector<unsigned long long> h(n * 4);
    if (hipMemcpyAsync(h.data(), d, n * 32, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess || !n)
        return;
    {   // the items that ran (the buffer holds room for the most items the split can make)
        size_t m = 0;
        for (size_t i = 0; i < n; i++)
            if (h[4 * i + 1]) {
                for (int q = 0; q < 4; q++) h[4 * m + q] = h[4 * i + q];
                m++;
            }
        n = m;
        if (!n) return;
    }
    unsigned long long t0 = ~0ull, t1 = 0, tt = 0, tp = 0;
    std::vector<double> dur(n);
    for (size_t i = 0; i < n; i++) {
        t0 = std::min(t0, h[4 * i]);
        t1 = std::max(t1, h[4 * i + 1]);
        dur[i] = (double)(h[4 * i + 1] - h[4 * i]) * 0.01;   // us (100 MHz)
        tt += h[4 * i + 2];
        tp += h[4 * i + 3];
    }
    const double span = (double)(t1 - t0) * 0.01;
    std::vector<double> sd(dur);
    std::sort(sd.begin(), sd.end());
    double busy = 0;
    for (double x : dur) busy += x;
    auto pct = [&](double q) { return sd[std::min(n - 1, (size_t)(q * (double)(n - 1)))]; };
    fprintf(stderr, "[mbr-trace] items %zu span %.1f us, item us p50 %.1f p90 %.1f p99 %.1f max %.1f, mean in flight %.0f, "
            "tested tiles %llu pair tests %llu\n", n, span, pct(0.5), pct(0.9), pct(0.99), sd[n - 1], busy / span,
            tt, tp);
    const int B = 20;
    std::vector<double> occ(B, 0.0);
    for (size_t i = 0; i < n; i++) {
        const double a = (double)(h[4 * i] - t0) * 0.01, b = (double)(h[4 * i + 1] - t0) * 0.01;
        for (int k = 0; k < B; k++) {
            const double lo = span * k / B, hi = span * (k + 1) / B;
            const double ov = std::min(b, hi) - std::max(a, lo);
            if (ov > 0) occ[k] += ov / (hi - lo);
        }
    }
    fprintf(stderr, "[mbr-trace] in flight per 5%% of the span:");
    for (int k = 0; k < B; k++) fprintf(stderr, " %.0f", occ[k]);
    fprintf(stderr, "\n");
}
#endif

// both skyline levels of the rep set in one bounding-box pruned all-pairs pass (k_mbr.hip)
static int mbr_run(Ctx &c, Pipe &p, const PipeIn &in, uint32_t mr, bool gmerge) {
    hipStream_t st = c.st;
    const int D = c.D;
    const int fmt = p.u16 ? 0 : (p.f64 ? 2 : 1);
    const int NW = mbr_row_words(D, fmt);
    const size_t ntiles = mbr_tiles(mr);
    const void *rows = p.rep_rows.p;
    if (fmt == 0) {
        SKY_TRY(p.r16.ensure((size_t)mr * NW * 4));
        launch_pack16(D, p.rep_rows.as<float>(), mr, nullptr, p.r16.as<uint32_t>(), st);
        rows = p.r16.p;
    }
    SKY_TRY(p.mbr_mm.ensure((size_t)D * 8));
    SKY_TRY(p.mbr_code.ensure((size_t)mr * 8));
    SKY_TRY(p.mbr_code2.ensure((size_t)mr * 8));
    SKY_TRY(p.mbr_idx.ensure((size_t)mr * 4));
    SKY_TRY(p.mbr_idx2.ensure((size_t)mr * 4));
    SKY_TRY(p.mbr_rows.ensure(ntiles * 64 * NW * 4));
    SKY_TRY(p.mbr_part.ensure((size_t)mr * 4));
    SKY_TRY(p.mbr_min.ensure(ntiles * NW * 4));
    SKY_TRY(p.mbr_max.ensure(ntiles * NW * 4));
    SKY_TRY(p.mbr_pr.ensure(ntiles * 4));
    SKY_TRY(p.mbr_sub.ensure(ntiles * kMbrSubMax * NW * 4));
    SKY_TRY(p.mbr_gmin.ensure(mbr_group_slots(mr) * NW * 4));
    SKY_TRY(p.mbr_gpr.ensure(mbr_group_slots(mr) * 4));
    SKY_TRY(p.mbr_domf.ensure((size_t)mr * 4));
    SKY_TRY(p.mbr_pairs.ensure(128));
    SKY_TRY(p.mbr_lpt.ensure(mbr_lpt_words(ntiles) * 4));
    SKY_TRY(p.scratch.ensure(std::max(radix_scratch_words(mr), scan_scratch_words(mr + 1)) * 4 + 64));
    FillSet fill;
    fill.add(p.mbr_lpt.p, kMbrLptHead * 4, 0);
    fill.add(p.mbr_mm.p, (size_t)D * 4, 0xff);
    fill.add(p.mbr_mm.as<uint32_t>() + D, (size_t)D * 4, 0);
    fill.add(p.mbr_pairs.p, 128, 0);
    fill.add(p.mbr_domf.p, (size_t)mr * 4, 0);
    HIP_TRY(fill.launch(st));
    MbrArgs a;
    a.D = D;
    a.fmt = fmt;
    a.rows = rows;
    a.rep_key = p.rep_key.as<uint64_t>();
    a.mr = mr;
    a.gmerge = gmerge;
    a.full = fmt != 0 || in.keys != nullptr;   // ±0 twins (f32/f64) or vectors repeated across given keys
    {
        const char *e = SKY_MEASURE_ENV("SKY_MBR_DBG");
        a.dbg = e ? atoi(e) : 0;
    }
    a.mm = p.mbr_mm.as<uint32_t>();
    a.code = p.mbr_code.as<uint64_t>();
    a.code_alt = p.mbr_code2.as<uint64_t>();
    a.idx = p.mbr_idx.as<uint32_t>();
    a.idx_alt = p.mbr_idx2.as<uint32_t>();
    a.radix_scratch = p.scratch.as<uint32_t>();
    a.err = p.flags.as<uint32_t>();
    a.trows = p.mbr_rows.as<uint32_t>();
    a.tpart = p.mbr_part.as<uint32_t>();
    a.tmin = p.mbr_min.as<uint32_t>();
    a.tmax = p.mbr_max.as<uint32_t>();
    a.tprange = p.mbr_pr.as<uint32_t>();
    a.tsub = p.mbr_sub.as<uint32_t>();
    a.gmin = p.mbr_gmin.as<uint32_t>();
    a.gprange = p.mbr_gpr.as<uint32_t>();
    a.domf = p.mbr_domf.as<uint32_t>();
    a.pairs = p.mbr_pairs.as<unsigned long long>();
    a.lpt = p.mbr_lpt.as<uint32_t>();
    a.alive_l = p.alive_l.as<uint8_t>();
    a.alive_g = p.alive_g.as<uint8_t>();
#ifdef SKY_MEASURE
    DevBuf trace;
    const size_t nitems = mbr_items_max(mbr_tiles(mr));
    if (a.dbg & 8) {
        SKY_TRY(trace.ensure(nitems * 32));
        HIP_TRY(hipMemsetAsync(trace.p, 0, nitems * 32, st));
        a.trace = trace.as<unsigned long long>();
    }
#endif
    c.ktimer_begin("mbr", st);
    HIP_TRY(launch_mbr(a, st));
    c.ktimer_end("mbr", st, mr);
#ifdef SKY_MEASURE
    if (a.dbg & 8) mbr_trace_report(trace.as<unsigned long long>(), nitems, st);
#endif
    STAGE(st, "mbr");
    p.used_mbr = true;
    p.sfs_rounds++;
    return SKY_OK;
}

// The fate tables, the per-tuple fate / output pass and the final read of a run.  mt: the
// slots; on the planned route (pr) their bound, the count itself on the device (pr->d_cnt),
// and the final read verifies the route's assumptions (kPlanMiss: run it again, synchronised).
constexpr int kPlanMiss = -1000;
struct PlanRun {
    size_t cap = 0, cap_full = 0;     // slots allocated / needed at most
    const uint32_t *d_cnt = nullptr;  // slots entering the brute pass (device)
    bool k_u16 = false, k_f32 = false;   // the brute pass's compare type
    bool tiny = false;                    // k_tiny_tail ran the tail (fates, counts, scan, stats)
    const uint32_t *domf = nullptr;       // k_brute_finish left to k_fate_tables: the pass's bits
    bool gmerge = false;
};
// the next run's designated duplicate group (status planes): the largest group of this run
void pick_dom_group(Pipe &p, int KM) {
    uint32_t best = 0;
    int32_t kj = -1;
    for (int q = 0; q < KM && q < (int)p.h_dup.size(); q++)
        if (p.h_dup[q] > best) {
            best = p.h_dup[q];
            kj = q;
        }
    p.dom_kj = kj;
    p.dom_km = KM;
}

// The end of a multi-GPU export run (in.dist): nothing is read back.  The route's checks (the
// planned route's assumptions, NaN, a look-back's spin bound) become a device verdict that the
// export writes into its block header; the fates of this shard's units follow the union merge.
static int dist_finish_run(Ctx &c, Pipe &p, PhaseTimer *tm, bool brute, uint32_t mt, const PlanRun *pr) {
    hipStream_t st = c.st;
    SKY_TRY(p.dverd.ensure(128));
    PlanCheck pc{};
    if (pr) {
        pc.planned = 1;
        pc.cap = (uint32_t)pr->cap;
        pc.rounds = p.plan.rounds;
        for (int r = 0; r <= p.plan.rounds && r < 4; r++) pc.bound[r] = p.plan.bound[r];
        pc.brute_max = brute_max();
        pc.k_u16 = pr->k_u16 ? 1 : 0;
        pc.k_f32 = pr->k_f32 ? 1 : 0;
    }
    // a slot-mode export of few units computes the verdict in its one-workgroup tail (dist_write_block)
    p.dist_verdict_pending = brute && mt > 0 && mt <= dist_export_one_max();
    if (!p.dist_verdict_pending)
        launch_plan_verdict(p.totals.as<uint32_t>(), p.flags.as<uint32_t>(), pc, p.dverd.as<uint32_t>(), st);
    p.dist_pc = pc;
    p.dist_slots = brute;
    p.dist_n = brute ? mt : p.mr;
    p.dist_d_n = brute && pr ? pr->d_cnt : nullptr;
    if (brute) p.mr = p.mt = mt;        // slots (on the planned route: their bound)
    p.mg = 0;
    p.nout = 0;
    if (tm) {
        tm->mark(7, st);
        tm->mark(8, st);
    }
    return stage_check(st, "dist export");
}

// k_out_hist_scan's look-back words: zeroed when (re)allocated; every launch tags them with a new
// epoch, so they need no zeroing per query
int out_hist_scan_words(Pipe &p, uint32_t tiles, hipStream_t st) {
    const size_t bytes = (size_t)std::max<uint32_t>(out_hist_scan_blocks(tiles), 1) * 8;
    const void *before = p.out_lb.p;
    const size_t cap_before = p.out_lb.cap;
    SKY_TRY(p.out_lb.ensure(bytes));
    if (p.out_lb.p != before || p.out_lb.cap != cap_before) {
        HIP_TRY(hipMemsetAsync(p.out_lb.p, 0, p.out_lb.cap, st));
        p.out_epoch = 0;
    }
    return SKY_OK;
}

static int pipe_finish(Ctx &c, Pipe &p, const PipeIn &in, PhaseTimer *tm, FillSet &fill, bool brute, uint32_t mt,
                       uint32_t tiles, const PlanRun *pr) {
    hipStream_t st = c.st;
    if (in.dist) return dist_finish_run(c, p, tm, brute, mt, pr);
    const uint32_t n = in.n;
    const int KM = p.Kp * p.M;
    // stats: summed over slots (unit weights, computed origins) or, for given origins /
    // weights, over tuples in the count pass
    const bool slot_stats = in.fate && !in.origin && !in.weights;
    FateArgs fta{};
    fta.mt = mt;
    fta.d_mt = pr ? pr->d_cnt : nullptr;
    fta.slot_rep = p.slot_rep.as<uint32_t>();
    fta.slot_src = p.s_src->as<uint32_t>();
    fta.alive_l = p.alive_l.as<uint8_t>();
    fta.alive_g = p.alive_g.as<uint8_t>();
    fta.KM = KM;
    fta.M = p.M;
    fta.K = p.K;
    fta.pruner_slot = p.pruner_slot.as<int32_t>();
    fta.status = p.status.as<uint16_t>();
    fta.pruner_fate = p.pruner_fate.as<uint8_t>();
    fta.dup_cnt = p.dup_cnt.as<uint32_t>();
    fta.lsz = slot_stats ? p.lsz.as<unsigned long long>() : nullptr;
    fta.surv = slot_stats ? p.surv.as<unsigned long long>() : nullptr;
    fta.tile_cand = p.hist_count ? p.tile_cand.as<uint32_t>() : nullptr;
    if (pr && pr->domf) {                       // the brute pass's finish, folded in
        fta.domf = pr->domf;
        fta.key = p.s_key->as<uint64_t>();
        fta.gmerge = pr->gmerge ? 1 : 0;
        fta.alive_l_w = p.alive_l.as<uint8_t>();
        fta.alive_g_w = p.alive_g.as<uint8_t>();
        fta.slot_rep_w = p.slot_rep.as<uint32_t>();
        fta.segalive = p.segalive.as<uint32_t>();
        fta.segn = p.seg_begin.as<uint32_t>();
    }
    const bool tiny = pr && pr->tiny;
    if (!tiny) launch_fate_tables(fta, st);
    if (tm) tm->mark(7, st);
    if (!in.fate) {                  // multi-GPU export: the shard's fates come after the union
        p.nout = 0;
        if (tm) tm->mark(8, st);
        return SKY_OK;
    }

    // ---- per-tuple fate: stats + output counts
    SKY_TRY(p.out_cnt.ensure((size_t)tiles * 4));
    SKY_TRY(p.out_off.ensure((size_t)tiles * 4));
    // the tile scan below needs its scratch even when no tuple was a candidate (mt == 0:
    // every tuple in an unqueried MR-Grid cell or removed by the grid filter)
    SKY_TRY(p.scratch.ensure(scan_scratch_words(tiles + 1) * 4 + 64));
    OutArgs oa{};
    oa.status = p.status.as<uint16_t>();
    oa.n = n;
    oa.pruner_fate = p.pruner_fate.as<uint8_t>();
    oa.M = p.M;
    oa.KM = p.Kp * p.M;
    oa.given_origin = in.origin;
    oa.given_w = in.weights;
    oa.K = p.K;
    oa.lsz = slot_stats ? nullptr : p.lsz.as<unsigned long long>();
    oa.surv = slot_stats ? nullptr : p.surv.as<unsigned long long>();
    oa.out_cnt = p.out_cnt.as<uint32_t>();
    oa.select_local = 0;
    p.fused = slot_stats && (in.out_ids || in.out_org) && !fused_disabled();
    // the brute route's counts, scan, stats and final read in one workgroup (k_tail_counts)
    // (up to kTailTilesMax tiles: one workgroup's pass over C2's 4883 tiles took 20 us, slower than
    // the four launches it replaces; C1-sized runs take the one-workgroup tail anyway)
    const bool tailk = !tiny && brute && p.fused && !fused_onepass() && p.hist_count && slot_stats &&
                       tiles <= kTailTilesMax && (p.segalive.p && p.seg_begin.p) && !tail_counts_disabled();
    // the brute route's stat reduce and final read as the write pass's epilogue workgroups
    const bool ep = !tiny && !tailk && brute && p.fused && !fused_onepass() && slot_stats && p.segalive.p &&
                    p.seg_begin.p && p.K <= 65536 && !epilogue_disabled();
    p.fused_ids = in.out_ids;
    p.fused_org = in.out_org;
    c.ktimer_begin("out", st);
    if (p.fused && fused_onepass()) {
        // count + prefix + write in one pass (decoupled look-back; A/B knob SKY_FUSED_OUT=2)
        SKY_TRY(p.lbuf.ensure((size_t)tiles * 8 + 64));
        fill.add(p.lbuf.p, (size_t)tiles * 8);
        fill.add(p.totals.as<uint32_t>() + 9, 4);          // ticket
        HIP_TRY(fill.launch(st));
        oa.ids = in.ids;
        oa.ids_out = in.out_ids;
        oa.origin_out = in.out_org;
        oa.given_origin = nullptr;
        c.ktimer_begin("outw", st);
        launch_out_fused(oa, p.lbuf.as<unsigned long long>(), p.totals.as<uint32_t>() + 9,
                         p.totals.as<uint32_t>() + 3, p.flags.as<uint32_t>(), in.out_cap, st);
        c.ktimer_end("outw", st, n);
    } else if (p.fused) {
        // count pass -> tile scan -> write pass, chained on the device (no host read in
        // between; positions >= out_cap are not written, the final read reports the total)
        // (the one-workgroup tail wrote the counts, their offsets and the total; on the brute route
        // k_tail_counts writes them, the stats and the final read in one launch)
        if (tailk) {
            SKY_TRY(p.statk.ensure((size_t)p.K * 16));
            TailArgs ta{};
            ta.tile_hist = p.tile_hist.as<uint32_t>();
            ta.tile_cand = p.tile_cand.as<uint32_t>();
            ta.pruner_fate = p.pruner_fate.as<uint8_t>();
            ta.KM = KM;
            ta.K = p.K;
            ta.Kp = p.Kp;
            ta.ntiles = tiles;
            ta.out_cnt = p.out_cnt.as<uint32_t>();
            ta.out_off = p.out_off.as<uint32_t>();
            ta.totals = p.totals.as<uint32_t>();
            ta.lsz = p.lsz.as<unsigned long long>();
            ta.surv = p.surv.as<unsigned long long>();
            ta.statk = p.statk.as<unsigned long long>();
            ta.segalive = p.segalive.as<uint32_t>();
            ta.segn = p.seg_begin.as<uint32_t>();
            ta.flags = p.flags.as<uint32_t>();
            ta.dup_cnt = p.dup_cnt.as<uint32_t>();
            SKY_TRY(p.pinned(tiny_pin_layout(p.K, p.Kp, KM, ta.pin_off)));
            ta.pin = reinterpret_cast<uint32_t *>(p.pin);
            c.ktimer_begin("outc", st);
            launch_tail_counts(ta, st);
            c.ktimer_end("outc", st, n);
        } else if (!tiny) {
            c.ktimer_begin("outc", st);
            if (p.hist_count) {             // counts + scan in one launch
                SKY_TRY(out_hist_scan_words(p, tiles, st));
                launch_out_hist_scan(p.tile_hist.as<uint32_t>(), p.tile_cand.as<uint32_t>(), p.pruner_fate.as<uint8_t>(),
                                     KM, tiles, p.out_cnt.as<uint32_t>(), p.out_off.as<uint32_t>(),
                                     p.totals.as<uint32_t>() + 3, p.out_lb.as<unsigned long long>(), ++p.out_epoch,
                                     p.flags.as<uint32_t>(), st);
            } else {
                launch_out_count(oa, st);
                scan_excl_u32(p.out_cnt.as<uint32_t>(), p.out_off.as<uint32_t>(), tiles, p.totals.as<uint32_t>() + 3,
                              p.scratch.as<uint32_t>(), st);
            }
            c.ktimer_end("outc", st, n);
        }
        OutArgs ow = oa;
        ow.out_off = p.out_off.as<uint32_t>();
        ow.ids = in.ids;
        ow.ids_out = in.out_ids;
        ow.origin_out = in.out_org;
        ow.out_cap = in.out_cap;
        ow.planes = p.planes_on ? p.planes.as<uint64_t>() : nullptr;
        ow.dom_kj = p.dom_kj;
        ow.skip_flags = tiny ? p.flags.as<uint32_t>() : nullptr;
        // a shape whose last run selected < 1/32 of its tuples: ids loaded by the selected lanes only
        ow.sparse_ids = p.n_prev == n && (uint64_t)p.nout_prev * 32 < n && !sparse_out_disabled();
        if (ep) {
            SKY_TRY(p.statk.ensure((size_t)p.K * 16));
            SKY_TRY(p.pinned(tiny_pin_layout(p.K, p.Kp, KM, ow.ep_off)));
            ow.ep_pin = reinterpret_cast<uint32_t *>(p.pin);
            ow.ep_lsz = p.lsz.as<unsigned long long>();
            ow.ep_surv = p.surv.as<unsigned long long>();
            ow.ep_statk = p.statk.as<unsigned long long>();
            ow.ep_totals = p.totals.as<uint32_t>();
            ow.ep_segalive = p.segalive.as<uint32_t>();
            ow.ep_segn = p.seg_begin.as<uint32_t>();
            ow.ep_flags = p.flags.as<uint32_t>();
            ow.ep_dup = p.dup_cnt.as<uint32_t>();
            ow.ep_Kp = p.Kp;
        }
        c.ktimer_begin("outw", st);
        launch_out_write(ow, st);
        c.ktimer_end("outw", st, n);
    } else {
        c.ktimer_begin("outc", st);
        oa.row_flags = in.row_flags;           // (the same pass: no second one over the status words)
        launch_out_count(oa, st);
        oa.row_flags = nullptr;
        c.ktimer_end("outc", st, n);
        scan_excl_u32(p.out_cnt.as<uint32_t>(), p.out_off.as<uint32_t>(), tiles, p.totals.as<uint32_t>() + 3,
                      p.scratch.as<uint32_t>(), st);
    }
    p.row_flags_done = in.row_flags && !p.fused && in.fate;
    c.ktimer_end("out", st, n);
    STAGE(st, "fate");
    uint32_t nout = 0;
    SKY_TRY(p.statk.ensure((size_t)p.K * 16));
    if (!tiny && !tailk && !ep)
        launch_stat_reduce(p.lsz.as<unsigned long long>(), p.surv.as<unsigned long long>(), p.K,
                           p.statk.as<unsigned long long>(), st);
    std::vector<unsigned long long> sk2((size_t)p.K * 2);
    const bool have_seg = mt && (brute || !p.h_seg_n.empty());
    p.h_seg_s.assign(have_seg ? p.Kp : 0, 0u);
    if (brute) {
        uint32_t flags2 = 0, tot[16] = {};
        p.h_seg_n.assign(p.Kp, 0u);
        p.h_dup.assign(KM, 0u);
        // (the one-workgroup tail wrote these words into p.pin in this layout: tiny_pin_layout)
        SKY_TRY(sync_read(p, st, {{p.totals.p, 64}, {p.statk.p, (size_t)p.K * 16},
                                  {p.segalive.p, (size_t)p.Kp * 4}, {p.seg_begin.p, (size_t)p.Kp * 4},
                                  {p.flags.p, 4}, {p.dup_cnt.p, (size_t)KM * 4}},
                          {tot, sk2.data(), p.h_seg_s.data(), p.h_seg_n.data(), &flags2, p.h_dup.data()},
                          tiny || tailk || ep));
        nout = tot[3];
#ifdef SKY_MEASURE
        if (SKY_MEASURE_ENV("SKY_FILTER_COUNT")) {   // k_filter's stores (tools/: the write itemisation)
            uint32_t fw[16] = {};
            HIP_TRY(hipMemcpy(fw, p.flags.p, 64, hipMemcpyDeviceToHost));
            fprintf(stderr, "[filter-count] n %u candidates %u deferred %u status_stored %u planes %d hist %d dom_kj %d\n",
                    n, tot[0], tot[6], fw[8], p.planes_on ? 1 : 0, p.hist_count ? 1 : 0, p.dom_kj);
        }
#endif
        if (flags2 & kFlagRadixSpin) {
            set_error("a look-back (output) exceeded its spin bound");
            return SKY_E_HIP;
        }
        if (flags2 & kFlagTinyOob) {
            set_error("the one-workgroup tail computed an index past a buffer's capacity (device guard): no result");
            return SKY_E_HIP;
        }
        if (pr) {
            // the planned route's assumptions: no NaN, no slot overflow, every count within
            // the bound its launches were sized for, the small-set size, the compare type
            if (flags2 & kFlagNaN) {
                set_error("a tuple value is NaN: the reference BNL result is order-dependent for NaN; rejected");
                return SKY_E_NAN;
            }
            if (flags2 & kFlagTinyMiss) {     // the final slots outgrew the one-workgroup tail
                p.plan.tiny = false;
                p.tiny_block = kTinyBlock;
                return kPlanMiss;
            }
            const uint32_t m = tot[0], nps = tot[5];
            if ((size_t)m + nps > pr->cap) {
                p.slot_hint = std::min(pr->cap_full, ((size_t)m + nps) * 5 / 4 + (size_t)KM);
                p.slot_reruns++;
                return kPlanMiss;
            }
            bool ok = tot[10] <= p.plan.bound[0];
            for (int r = 0; r < p.plan.rounds; r++) ok &= tot[11 + r] <= p.plan.bound[r + 1];
            const uint32_t fin = pr->tiny ? tot[14] : (p.plan.rounds ? tot[10 + p.plan.rounds] : tot[10]);
            ok &= fin <= brute_max();
            const bool f64 = (flags2 & kFlagNotF32) != 0, ints = !f64 && (flags2 & kFlagNotU16) == 0;
            ok &= pr->k_u16 ? ints : (pr->k_f32 ? !f64 : true);
            if (!ok && debug_level() >= 1)
                fprintf(stderr, "[sky] plan miss: slots %u/%u rounds %d live %u/%u fin %u tiny %d u16 %d/%d f32 %d/%d\n",
                        tot[10], p.plan.bound[0], p.plan.rounds, p.plan.rounds ? tot[11] : 0u,
                        p.plan.rounds ? p.plan.bound[1] : 0u, fin, (int)pr->tiny, (int)pr->k_u16, (int)ints,
                        (int)pr->k_f32, (int)!f64);
            if (!ok) return kPlanMiss;
            p.m = m;
            p.nps = nps;
            p.mt_pre = tot[10];
            p.mt = fin;
            p.plan.tiny = fin <= tiny_brute_rows(c.D) * 3 / 4;
            p.f64 = f64;
            p.ints = ints;
            p.ties = (flags2 & kFlagScoreTies) != 0;
            p.u16 = p.ints && !p.ties && !sfs16_disabled();
            mt = fin;
        }
        p.mr = mt;                            // brute mode: slots (duplicates not collapsed)
        uint32_t alive_sum = 0;
        for (int k = 0; k < p.Kp; k++) alive_sum += p.h_seg_s[k];
        p.mg = in.global && !in.single ? alive_sum : 0;
    } else {
        uint32_t flags3 = 0;
        unsigned long long mbr_pairs[5] = {0, 0, 0, 0, 0};
        p.h_dup.assign(KM, 0u);
        SKY_TRY(sync_read(p, st, {{p.totals.as<uint32_t>() + 3, 4}, {p.statk.p, (size_t)p.K * 16},
                                  {p.segalive.p, have_seg ? (size_t)p.Kp * 4 : 0}, {p.flags.p, 4},
                                  {p.mbr_pairs.p, p.used_mbr ? 40u : 0u}, {p.dup_cnt.p, (size_t)KM * 4}},
                          {&nout, sk2.data(), p.h_seg_s.data(), &flags3, mbr_pairs, p.h_dup.data()}));
        if (p.used_mbr) {
            p.sfs_pairs_upper = (int64_t)mbr_pairs[0];  // pair tests the pruned pass executed
            p.mbr_tiles = (int64_t)mbr_pairs[1];        // (y tile, x tile) pairs it tested
            if (mbr_pairs[3])                             // SKY_MBR_DBG bit 4: the scan's funnel
                fprintf(stderr, "[mbr] reps %u groups %llu box %llu pre %llu tested %llu pairs %llu\n", p.mr,
                        mbr_pairs[2], mbr_pairs[3], mbr_pairs[4], mbr_pairs[1], mbr_pairs[0]);
#ifdef SKY_MEASURE
            {
                unsigned long long tk[6] = {};
                HIP_TRY(hipMemcpy(tk, p.mbr_pairs.as<unsigned long long>() + 8, 48, hipMemcpyDeviceToHost));
                if (tk[0] | tk[1] | tk[2] | tk[3] | tk[4] | tk[5])   // SKY_MBR_DBG bit 16: region clocks
                    fprintf(stderr, "[mbr-clock] setup %llu scans %llu pretest %llu loads %llu subbox %llu rows %llu\n",
                            tk[0], tk[1], tk[2], tk[3], tk[4], tk[5]);
            }
#endif
            uint32_t alive_sum = 0;
            for (int k = 0; k < p.Kp; k++) alive_sum += p.h_seg_s[k];
            p.mg = in.global && !in.single ? alive_sum : 0;
        }
        if (flags3 & kFlagRadixSpin) {
            set_error("a look-back (radix sort / output) exceeded its spin bound");
            return SKY_E_HIP;
        }
        if (flags3 & kFlagMbrQueue) {
            set_error("the bounding-box pass's work items outgrew their queue (k_mbr_order): no pass ran");
            return SKY_E_HIP;
        }
    }
    pick_dom_group(p, KM);
    p.dom_w = 0;
    if (have_seg) {
        int64_t sg = 0;
        for (int k = 0; k < p.Kp; k++) {
            const int64_t nk = p.h_seg_n[k], sk = p.h_seg_s[k];
            p.dom_w += sk * (sk - 1) / 2 + (nk - sk);
            sg += sk;
        }
        if (in.global && !in.single) p.dom_w += sg * (sg - 1) / 2;
    }
    for (int k = 0; k < p.K; k++) {
        p.h_lsz[k] = sk2[k];
        p.h_surv[k] = sk2[(size_t)p.K + k];
    }
    p.nout = nout;
    p.n_prev = n;
    p.nout_prev = nout;
    if (debug_level() >= 3) {
        fprintf(stderr, "[sky] run n=%u m=%u nps=%u mr=%u mg=%u nout=%u u16=%d seg_n:", n, p.m, p.nps, p.mr, p.mg,
                nout, (int)p.u16);
        for (uint32_t x : p.h_seg_n) fprintf(stderr, " %u", x);
        fprintf(stderr, " seg_s:");
        for (uint32_t x : p.h_seg_s) fprintf(stderr, " %u", x);
        fprintf(stderr, "\n");
    }
    if (tm) tm->mark(8, st);
    return SKY_OK;
}


// The planned route's zero / all-ones initialisations, added to the run's first fill launch:
// the criterion minima of every prefilter round (a slice each), the brute pass's domination
// bits (its bound) and per-partition counts.
static int plan_prepare(Pipe &p, int D, bool tiny, FillSet &fill) {
    const Pipe::Plan &pl = p.plan;
    const int M2 = std::min(prefilter_m2(), 2048 / p.Kp);
    const size_t KM2 = (size_t)p.Kp * M2;
    uint32_t fin = pl.bound[0];
    for (int r = 0; r < pl.rounds; r++) fin = std::min(pl.bound[r + 1], fin);
    if (pl.rounds && tiny) {            // round 0's minima: k_cand_min on the whole GPU before the tail
        SKY_TRY(p.cmin.ensure(KM2 * 8));
        fill.add(p.cmin.p, KM2 * 8, 0xff);
    }
    if (pl.rounds && !tiny) {           // (the one-workgroup tail keeps its minima in LDS)
        SKY_TRY(p.cmin.ensure(KM2 * pl.rounds * 8));
        fill.add(p.cmin.p, KM2 * pl.rounds * 8, 0xff);
        if (cand_fused_fits(D, p.Kp, M2) && !cand_fused_disabled()) {   // the fused pass's look-back words
            size_t lb = 0;
            uint32_t b = pl.bound[0];
            for (int r = 0; r < pl.rounds; r++) {
                lb += cand_lb_bytes(b);
                b = std::min(pl.bound[r + 1], b);
            }
            SKY_TRY(p.cand_lb.ensure(lb));
            fill.add(p.cand_lb.p, lb);
        }
    }
    SKY_TRY(p.segalive.ensure((size_t)p.Kp * 4));
    SKY_TRY(p.seg_begin.ensure((size_t)p.Kp * 4));
    fill.add(p.segalive.p, (size_t)p.Kp * 4);
    fill.add(p.seg_begin.p, (size_t)p.Kp * 4);
    if (!tiny) {
        SKY_TRY(p.keep.ensure((size_t)std::max<uint32_t>(fin, 1) * 4));
        fill.add(p.keep.p, (size_t)std::max<uint32_t>(fin, 1) * 4);
    }
    return SKY_OK;
}

// the planned route's final read; a miss re-runs the query on the synchronised route
static int plan_finish(Ctx &c, Pipe &p, const PipeIn &in, PhaseTimer *tm, FillSet &fill, uint32_t bound,
                       uint32_t tiles, const PlanRun &pr) {
    const int r = pipe_finish(c, p, in, tm, fill, true, bound, tiles, &pr);
    if (r != kPlanMiss) {
        p.last_planned = r == SKY_OK;
        p.last_tiny = pr.tiny && r == SKY_OK;
        return r;
    }
    p.plan.valid = false;                      // re-run on the synchronised route (learns a new plan)
    p.plan_misses++;
    const int r2 = pipe_run(c, p, in, tm);
    p.last_plan_miss = true;
    return r2;
}

// The planned route's tail in ONE launch (k_tiny_tail, sky_internal.h): the pruner slots, the
// prefilter rounds, the brute pass, the fate tables, the output counts + offsets and the stats;
// pipe_finish then runs only the output write pass and the final read.
static int pipe_run_tiny(Ctx &c, Pipe &p, const PipeIn &in, PhaseTimer *tm, size_t cap, size_t cap_full,
                         uint32_t tiles, FillSet &fill, const AppendArgs &ap) {
    hipStream_t st = c.st;
    const int D = c.D;
    const Pipe::Plan pl = p.plan;
    const int KM = p.Kp * p.M;
    const size_t rb64 = row_bytes(true, D);
    TinyArgs ta{};
    ta.ap = ap;
    ta.rounds = pl.rounds;
    ta.M2 = std::min(prefilter_m2(), 2048 / p.Kp);
    uint32_t bound = pl.bound[0];
    ta.bound[0] = bound;
    SKY_TRY(p.live.ensure((size_t)std::max<uint32_t>(bound, 1) * 4));
    SKY_TRY(p.livepos.ensure((size_t)std::max<uint32_t>(bound, 1) * 4));
    ta.live = p.live.as<uint32_t>();
    ta.livepos = p.livepos.as<uint32_t>();
    p.s_rows = &p.rows;
    p.s_key = &p.sortkey;
    p.s_src = &p.slot_src;
    // survivors of round r: at most its input bound (a plan without rounds: the round the tail
    // runs itself above kTinyForce slots, bound = the slots' bound)
    const int nr = std::max(pl.rounds, 1);
    for (int r = 0; r < nr; r++) {
        DevBuf *dr = r & 1 ? &p.rows3 : &p.rows2, *dk = r & 1 ? &p.sortkey3 : &p.sortkey2,
               *ds = r & 1 ? &p.slot_src3 : &p.slot_src2;
        SKY_TRY(dr->ensure((size_t)bound * rb64));
        SKY_TRY(dk->ensure((size_t)bound * 8));
        SKY_TRY(ds->ensure((size_t)bound * 4));
        ta.rows_r[r] = dr->as<double>();
        ta.key_r[r] = dk->as<uint64_t>();
        ta.src_r[r] = ds->as<uint32_t>();
        if (r < pl.rounds) {                   // (after a tail-chosen round the final slots' arrays
            p.s_rows = dr;                     // are known on the device only; nothing reads them)
            p.s_key = dk;
            p.s_src = ds;
            bound = std::min(pl.bound[r + 1], bound);
        }
        ta.bound[r + 1] = bound;
    }
    SKY_TRY(p.slot_rep.ensure((size_t)std::max<uint32_t>(bound, 1) * 4));
    SKY_TRY(p.alive_l.ensure(std::max<uint32_t>(bound, 1)));
    SKY_TRY(p.alive_g.ensure(std::max<uint32_t>(bound, 1)));
    SKY_TRY(p.pruner_fate.ensure(std::max<size_t>(KM, 1)));
    SKY_TRY(p.out_cnt.ensure((size_t)tiles * 4));
    SKY_TRY(p.out_off.ensure((size_t)tiles * 4));
    SKY_TRY(p.statk.ensure((size_t)p.K * 16));
    ta.totals = p.totals.as<uint32_t>();
    ta.gmerge = in.global && !in.single;
    ta.alive_l = p.alive_l.as<uint8_t>();
    ta.alive_g = p.alive_g.as<uint8_t>();
    ta.segalive = p.segalive.as<uint32_t>();   // zeroed by plan_prepare
    ta.segn = p.seg_begin.as<uint32_t>();
    ta.slot_rep = p.slot_rep.as<uint32_t>();
    ta.status = p.status.as<uint16_t>();
    ta.pruner_fate = p.pruner_fate.as<uint8_t>();
    ta.K = p.K;
    ta.tile_hist = p.tile_hist.as<uint32_t>();
    ta.ntiles = tiles;
    ta.out_cnt = p.out_cnt.as<uint32_t>();
    ta.out_off = p.out_off.as<uint32_t>();
    ta.statk = p.statk.as<unsigned long long>();
    SKY_TRY(p.pinned(tiny_pin_layout(p.K, p.Kp, KM, ta.pin_off)));   // the final read, written by the tail
    ta.pin = reinterpret_cast<uint32_t *>(p.pin);
    // the capacities every global index of the tail is checked against on the device (an index
    // past one skips its access and raises kFlagTinyOob: SKY_E_HIP, not a fault)
    ta.cap[0] = (uint32_t)std::min<size_t>(cap, 0xffffffffu);
    ta.cap[1] = (uint32_t)(p.live.cap / 4);
    ta.cap[2] = (uint32_t)(p.rows2.cap / rb64);
    ta.cap[3] = (uint32_t)(p.rows3.cap / rb64);
    ta.cap[4] = (uint32_t)(p.rows2.cap / rb64);
    ta.cap[5] = (uint32_t)p.alive_l.cap;
    ta.cap[6] = (uint32_t)(p.status.cap / 2);
    ta.cap[7] = (uint32_t)(p.pr_entries.cap / 4);
#ifdef SKY_MEASURE
    {   // SKY_TINY_CAP=i:c (measurement builds): capacity i forced to c -- the guard's test
        const char *e = SKY_MEASURE_ENV("SKY_TINY_CAP");
        if (e) {
            const int i = atoi(e);
            const char *c2 = strchr(e, ':');
            if (i >= 0 && i < 8 && c2) ta.cap[i] = (uint32_t)strtoul(c2 + 1, nullptr, 10);
        }
    }
    static const bool tchk = SKY_MEASURE_ENV("SKY_TINY_CHK") != nullptr;
    if (tchk) {                                 // bounds-checked tail: every global index vs its capacity
        {
            const hipError_t e0 = hipStreamSynchronize(st);   // the launches before the tail
            fprintf(stderr, "[tiny-chk] before the tail: %s\n", hipGetErrorString(e0));
            if (e0 != hipSuccess) return SKY_E_HIP;
        }
        fprintf(stderr, "[tiny-chk] ptrs pr %p dup %p ent %p ps %p rows %p key %p src %p orand %p live %p lp %p "
                        "r0 %p k0 %p s0 %p tot %p al %p ag %p sa %p sn %p rep %p st %p pf %p th %p oc %p oo %p sk %p\n",
                (void *)ta.ap.pruners, (void *)ta.ap.dup_cnt, (void *)ta.ap.entries, (void *)ta.ap.pruner_slot,
                ta.ap.rows, (void *)ta.ap.sortkey, (void *)ta.ap.slot_src, (void *)ta.ap.orand, (void *)ta.live,
                (void *)ta.livepos, (void *)ta.rows_r[0], (void *)ta.key_r[0], (void *)ta.src_r[0], (void *)ta.totals,
                (void *)ta.alive_l, (void *)ta.alive_g, (void *)ta.segalive, (void *)ta.segn, (void *)ta.slot_rep,
                (void *)ta.status, (void *)ta.pruner_fate, (void *)ta.tile_hist, (void *)ta.out_cnt,
                (void *)ta.out_off, (void *)ta.statk);
        fprintf(stderr, "[tiny-chk] Kp %d M %d M2 %d K %d ntiles %u slot_cap %u D %d\n", ta.ap.Kp, ta.ap.M, ta.M2, ta.K,
                ta.ntiles, ta.ap.slot_cap, D);
        ta.chk = p.flags.as<uint32_t>() + 13;
    }
#endif
#ifdef SKY_MEASURE
    static const bool tclk = SKY_MEASURE_ENV("SKY_TINY_CLK") != nullptr;
    {
        const char *e = SKY_MEASURE_ENV("SKY_TINY_DBG");
        ta.dbg = e ? atoi(e) : 0;
    }
    if (tclk) {
        SKY_TRY(p.dbg_clk.ensure(128));
        HIP_TRY(hipMemsetAsync(p.dbg_clk.p, 0, 128, st));
        ta.clk = p.dbg_clk.as<unsigned long long>();
    }
#endif
    if (pl.rounds) {                    // round 0's criterion minima over the candidate slots
        CandArgs ca{};
        ca.mt = pl.bound[0];
        ca.d_mt = p.totals.as<uint32_t>();     // the filter's candidates (the pruner slots follow them)
        ca.rows = p.rows.as<double>();
        ca.key = p.sortkey.as<uint64_t>();
        ca.Kp = p.Kp;
        ca.M2 = ta.M2;
        ca.cmin = p.cmin.as<unsigned long long>();   // filled by plan_prepare
        launch_cand_min(D, ca, st);
        ta.cmin0 = ca.cmin;
    }
    c.ktimer_begin("tiny", st);
    launch_tiny_tail(D, ta, st);
#ifdef SKY_MEASURE
    if (tclk) {
        unsigned long long t[10] = {};
        HIP_TRY(hipMemcpyAsync(t, ta.clk, 80, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        fprintf(stderr, "[tiny-clk] us:");
        for (int i = 1; i < 10; i++) fprintf(stderr, " %d:%.2f", i, t[i] && t[i - 1] ? (t[i] - t[i - 1]) / 100.0 : -1.0);
        fprintf(stderr, " total %.2f\n", t[9] && t[0] ? (t[9] - t[0]) / 100.0 : -1.0);
    }
#endif
    c.ktimer_end("tiny", st, bound);
#ifdef SKY_MEASURE
    if (tchk) {
        uint32_t w = 0;
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMemcpy(&w, ta.chk, 4, hipMemcpyDeviceToHost));
        fprintf(stderr, "[tiny-chk] bits 0x%x caps %u %u %u %u %u %u %u %u bounds %u %u rounds %d\n", w, ta.cap[0],
                ta.cap[1], ta.cap[2], ta.cap[3], ta.cap[4], ta.cap[5], ta.cap[6], ta.cap[7], ta.bound[0], ta.bound[1],
                ta.rounds);
    }
#endif
    STAGE(st, "tiny tail");
    p.plan_runs++;
    p.tiny_runs++;
    p.f64 = pl.f64;
    p.ints = pl.ints;
    if (tm) {
        tm->mark(3, st);
        tm->mark(4, st);
        tm->mark(5, st);
        tm->mark(6, st);
    }
    PlanRun pr;
    pr.cap = cap;
    pr.cap_full = cap_full;
    pr.d_cnt = p.totals.as<uint32_t>() + 14;
    pr.tiny = true;                            // exact f64 tests: no compare-type assumption
    return plan_finish(c, p, in, tm, fill, bound, tiles, pr);
}

// The planned route (see pipe_run): the prefilter rounds and the brute pass of the last
// query's small-set route, every launch sized by the plan's bounds and reading its count
// from the device; no host synchronisation before pipe_finish's final read.
static int pipe_run_planned(Ctx &c, Pipe &p, const PipeIn &in, PhaseTimer *tm, size_t cap, size_t cap_full,
                            uint32_t tiles, FillSet &fill, const AppendArgs *tiny_ap) {
    hipStream_t st = c.st;
    const int D = c.D;
    const Pipe::Plan pl = p.plan;
    const int KM = p.Kp * p.M;
    const size_t rb64 = row_bytes(true, D);
    p.plan_runs++;
    if (tm) tm->mark(3, st);
    p.f64 = pl.f64;
    p.ints = pl.ints;
    p.s_rows = &p.rows;
    p.s_key = &p.sortkey;
    p.s_src = &p.slot_src;
    const uint32_t *d_cnt = p.totals.as<uint32_t>() + 10;   // min(m + nps, cap), by k_append_pruners
    uint32_t bound = pl.bound[0];
    if (tiny_ap) return pipe_run_tiny(c, p, in, tm, cap, cap_full, tiles, fill, *tiny_ap);
    size_t lb_off = 0;                         // this round's look-back words (fused prefilter pass)
    for (int round = 0; round < pl.rounds; round++) {
        const int M2 = std::min(prefilter_m2(), 2048 / p.Kp);
        const int KM2 = p.Kp * M2;
        DevBuf *dr = round & 1 ? &p.rows3 : &p.rows2, *dk = round & 1 ? &p.sortkey3 : &p.sortkey2,
               *ds = round & 1 ? &p.slot_src3 : &p.slot_src2;
        SKY_TRY(p.pr2.ensure((size_t)KM2 * D * 8));
        SKY_TRY(p.npr2.ensure((size_t)p.Kp * 4));
        SKY_TRY(p.live.ensure((size_t)bound * 4));
        SKY_TRY(p.livepos.ensure((size_t)(bound + 1) * 4));
        SKY_TRY(dr->ensure((size_t)bound * rb64));
        SKY_TRY(dk->ensure((size_t)bound * 8));
        SKY_TRY(ds->ensure((size_t)bound * 4));
        SKY_TRY(p.scratch.ensure(scan_scratch_words(bound + 1) * 4 + 64));
        CandArgs ca{};
        ca.mt = bound;
        ca.d_mt = d_cnt;
        ca.rows = p.s_rows->as<double>();
        ca.key = p.s_key->as<uint64_t>();
        ca.src = p.s_src->as<uint32_t>();
        ca.Kp = p.Kp;
        ca.M2 = M2;
        ca.cmin = p.cmin.as<unsigned long long>() + (size_t)round * KM2;   // filled by plan_prepare
        ca.pr2 = p.pr2.as<double>();
        ca.npr2 = p.npr2.as<int32_t>();
        ca.live = p.live.as<uint32_t>();
        uint32_t *d_live = p.totals.as<uint32_t>() + 11 + round;
        c.ktimer_begin("prefilter", st);
        if (cand_fused_fits(D, p.Kp, M2) && !cand_fused_disabled()) {   // (plan_prepare zeroed its words)
            ca.rows2 = dr->as<double>();
            ca.key2 = dk->as<uint64_t>();
            ca.src2 = ds->as<uint32_t>();
            ca.d_live = d_live;
            ca.pruner_slot = p.pruner_slot.as<int32_t>();
            ca.entries = p.pr_entries.as<int32_t>();
            ca.KM = KM;
            ca.lb = reinterpret_cast<unsigned long long *>(p.cand_lb.as<char>() + lb_off);
            ca.picked = cand_picked(bound);
            ca.ticket = reinterpret_cast<uint32_t *>(p.cand_lb.as<char>() + lb_off +
                                                     (size_t)cand_fused_tiles(bound, ca.picked) * 8);
            ca.err = p.flags.as<uint32_t>();
            launch_cand_min(D, ca, st);
            launch_cand_fused(D, ca, st);
            lb_off += cand_lb_bytes(bound);
        } else {
            launch_cand_prefilter(D, ca, st);
            scan_excl_u32(ca.live, p.livepos.as<uint32_t>(), bound, d_live, p.scratch.as<uint32_t>(), st, d_cnt);
            launch_cand_compact(D, ca, p.livepos.as<uint32_t>(), dr->as<double>(), dk->as<uint64_t>(),
                                ds->as<uint32_t>(), p.pruner_slot.as<int32_t>(), KM, st);
        }
        c.ktimer_end("prefilter", st, bound);
        STAGE(st, "prefilter");
        p.s_rows = dr;
        p.s_key = dk;
        p.s_src = ds;
        // the next stage reads at most min(count, its bound) <= this bound compacted slots
        d_cnt = d_live;
        bound = std::min(pl.bound[round + 1], bound);
    }
    if (tm) tm->mark(4, st);
    if (tm) tm->mark(5, st);
    SKY_TRY(p.slot_rep.ensure((size_t)std::max<uint32_t>(bound, 1) * 4));
    SKY_TRY(p.alive_l.ensure(std::max<uint32_t>(bound, 1)));
    SKY_TRY(p.alive_g.ensure(std::max<uint32_t>(bound, 1)));
    SKY_TRY(p.pruner_fate.ensure(std::max<size_t>(KM, 1)));
    PlanRun pr;                                // segalive / seg_begin / keep: filled by plan_prepare
    pr.cap = cap;
    pr.cap_full = cap_full;
    pr.d_cnt = d_cnt;
    pr.k_u16 = p.ints && !brute16_disabled();
    pr.k_f32 = !p.f64;
    c.ktimer_begin("brute", st);
    // the finish (alive flags, per-partition counts) runs inside k_fate_tables unless this run
    // writes no fates (multi-GPU export; SKY_FINISH_FOLD=0: the separate k_brute_finish, A/B knob)
    const bool fold = !in.dist && in.fate && !finish_fold_disabled();
    if (fold) {
        launch_brute_pairs(D, pr.k_f32, pr.k_u16, p.s_rows->p, p.s_key->as<uint64_t>(), bound, p.keep.as<uint32_t>(), st,
                           d_cnt);
        pr.domf = p.keep.as<uint32_t>();
        pr.gmerge = in.global && !in.single;
    } else {
        launch_brute_fates(D, pr.k_f32, pr.k_u16, p.s_rows->p, p.s_key->as<uint64_t>(), bound, in.global && !in.single,
                           p.keep.as<uint32_t>(), p.alive_l.as<uint8_t>(), p.alive_g.as<uint8_t>(),
                           p.segalive.as<uint32_t>(), p.seg_begin.as<uint32_t>(), p.slot_rep.as<uint32_t>(), st, d_cnt);
    }
    c.ktimer_end("brute", st, (int64_t)bound * bound);
    STAGE(st, "brute");
    if (tm) tm->mark(6, st);
    return plan_finish(c, p, in, tm, fill, bound, tiles, pr);
}

// every buffer of a whole-stream run whose size follows the tuple count, sized for n tuples
// (sky_stream_reserve: a continuous query's resident set grows trigger by trigger, and each
// regrowth's hipFree synchronises the device inside that trigger's latency)
int pipe_reserve(Ctx &c, Pipe &p, uint32_t n) {
    const uint32_t tiles = (n + kTile - 1) / kTile;
    const int Kp = c.Kq();
    const int M = std::max(1, std::min(8, 49152 / (Kp * c.D * 8)));
    SKY_TRY(p.status.ensure((size_t)tiles * kTile * 2));
    SKY_TRY(p.planes.ensure((size_t)tiles * 32 * 16));
    if (Kp * M <= kHistMaxKM) SKY_TRY(p.tile_hist.ensure((size_t)tiles * Kp * M * 4));
    SKY_TRY(p.tile_cand.ensure((size_t)tiles * 4));
    SKY_TRY(p.defer.ensure((size_t)n * 4));
    SKY_TRY(p.out_cnt.ensure((size_t)tiles * 4));
    SKY_TRY(p.out_off.ensure((size_t)tiles * 4));
    SKY_TRY(p.scratch.ensure(scan_scratch_words(tiles + 1) * 4 + 64));
    return SKY_OK;
}

int pipe_run(Ctx &c, Pipe &p, const PipeIn &in, PhaseTimer *tm) {
    hipStream_t st = c.st;
    const int D = c.D;
    const uint32_t n = in.n;
    p.n = n;
    p.K = in.K;
    p.last_planned = p.last_plan_miss = p.last_tiny = false;
    p.row_flags_done = false;
    p.Kp = in.single ? 1 : c.Kq();
    p.M = std::max(1, std::min(8, 49152 / (p.Kp * D * 8)));
    p.m = p.nps = p.mt = p.mr = p.mg = p.nout = 0;
    p.fused = false;
    p.used_mbr = false;
    p.mbr_tiles = 0;
    p.sfs_rounds = p.sfs_pairs_upper = 0;
    p.h_seg_n.clear();
    p.h_seg_s.clear();
    p.h_lsz.assign(p.K, 0);
    p.h_surv.assign(p.K, 0);
    const uint32_t tiles = (n + kTile - 1) / kTile;
    const size_t stat_bytes = (size_t)kStatShards * p.K * 8;
    SKY_TRY(p.lsz.ensure(stat_bytes));
    SKY_TRY(p.surv.ensure(stat_bytes));
    SKY_TRY(p.totals.ensure(64));
    SKY_TRY(p.flags.ensure(64));
    FillSet fill;
    fill.add(p.lsz.p, stat_bytes);
    fill.add(p.surv.p, stat_bytes);
    if (n == 0) {
        HIP_TRY(fill.launch(st));
        return SKY_OK;
    }
    KeyParams kp = c.kp();
    kp.K = p.Kp;
    if (tm) tm->mark(0, st);

    // ---- pruners from a strided sample
    // buffers of the HBM stream (below) first: its counters are zeroed by the same
    // launch that initialises the pruner sample
    const int KM = p.Kp * p.M;
    const size_t rb64 = row_bytes(true, D);
    // candidate slots: sized by the last runs' need (at least 1M), not by n (f64 rows of n + KM
    // slots were 6.4 GB at 100M tuples for 241k candidates); a run that overflows the slots
    // (counted on the device, writes past the capacity dropped) is re-run with room for all
    const size_t cap_full = (size_t)n + KM;
    const size_t cap = std::min(cap_full, std::max(p.slot_hint, std::min(cap_full, slot_min())));
    SKY_TRY(p.status.ensure((size_t)tiles * kTile * 2));         // whole tiles: see load_status8
    SKY_TRY(p.rows.ensure(cap * rb64));
    SKY_TRY(p.sortkey.ensure(cap * 8));
    SKY_TRY(p.slot_src.ensure(cap * 4));
    SKY_TRY(p.dup_cnt.ensure((size_t)KM * 4));
    SKY_TRY(p.pr_entries.ensure((size_t)KM * 4));
    SKY_TRY(p.pruner_slot.ensure((size_t)KM * 4));
    SKY_TRY(p.orand.ensure(16));
    fill.add(p.dup_cnt.p, (size_t)KM * 4);      // with lsz / surv: one launch for the query's counters
    fill.add(p.flags.p, 64);
    fill.add(p.totals.p, 64);
    fill.add(p.orand.p, 8, 0);
    fill.add(p.orand.as<char>() + 8, 8, 0xff);
    const uint32_t S = std::min<uint32_t>(n, 65536);
    SKY_TRY(p.pmin.ensure((size_t)p.Kp * p.M * 8));
    SKY_TRY(p.pruners.ensure((size_t)p.Kp * p.M * D * 8));
    SKY_TRY(p.npr.ensure((size_t)p.Kp * 4));
    // the sample minima are tagged per query (launch_select_pruners): all-ones only for a new buffer
    // and when the 16-bit query count wraps
    const bool pmin_reset = p.pmin.p != p.pmin_at || p.pmin.cap != p.pmin_cap || ((p.pmin_epoch + 1) & 0xffffu) == 0;
    if (pmin_reset) {
        fill.add(p.pmin.p, p.pmin.cap, 0xff);     // (the whole buffer: no word of an earlier use survives)
        p.pmin_at = p.pmin.p;
        p.pmin_cap = p.pmin.cap;
        p.pmin_epoch = 0;
#ifdef SKY_MEASURE
        if (const char *e = SKY_MEASURE_ENV("SKY_PMIN_EPOCH0")) p.pmin_epoch = (uint32_t)atoi(e) & 0xffffu;   // the wrap's test
#endif
    }
    p.pmin_epoch++;
    const uint32_t ptag = 0xffffu - (p.pmin_epoch & 0xffffu);
    // output counts from per-tile duplicate histograms (unit weights, stats over slots, the
    // single-pass output's buffers): the filter keeps them, the fate pass counts candidates
    p.hist_count = ((in.fate && (in.out_ids || in.out_org)) || in.dist) && !in.origin && !in.weights &&
                   !fused_disabled() && !fused_onepass() && KM <= kHistMaxKM && !hist_disabled();
    // the planned route: the last query's small-set route (prefilter rounds, then the brute
    // pair pass) replayed with device-sized launches and no host synchronisation until the
    // final read, which verifies every assumption (counts within the bounds, the row type);
    // a miss re-runs the query on the synchronised route.  Results are identical either way
    // (the prefilter is exact, so its round count does not change the skyline).
    const bool planned = p.plan.valid && !plan_disabled() && c.warm_mode == 0 && (in.fate || in.dist) &&
                         !brute_disabled() &&
                         p.plan.D == D && p.plan.Kp == p.Kp && p.plan.M == p.M && p.plan.single == in.single &&
                         p.plan.global == in.global && (p.plan.rounds == 0 || !prefilter_disabled()) &&
                         cap >= p.plan.bound[0];
    if (p.hist_count) {
        SKY_TRY(p.tile_hist.ensure((size_t)tiles * KM * 4));
        SKY_TRY(p.tile_cand.ensure((size_t)tiles * 4));
        fill.add(p.tile_cand.p, (size_t)tiles * 4);
    }
    // status planes: only when this run's own write pass (k_out_write, hist counts) makes the
    // output, so nothing reads the status words of dropped / designated-group tuples
    p.planes_on = p.hist_count && (in.planes_ok || in.dist) && !planes_disabled();
    if (p.planes_on) SKY_TRY(p.planes.ensure((size_t)tiles * 32 * 16));
    if (p.dom_km != KM) p.dom_kj = -1;
    // the planned route's counters and flags go out with this launch too: one criterion-minima
    // slice per prefilter round, the brute pass's domination bits and partition counts
    // the planned route's tail in one workgroup (k_tiny_tail): the last query's final slots
    // few, its first bound small, the output from the duplicate histograms, the shape within
    // the kernel's LDS arena (SKY_TINY=0: the launch-per-stage tail, A/B knob)
    // (a plan without prefilter rounds also tries it: the tail runs a round of its own, which may
    // cut the slots to what it holds; not for kTinyBlock queries after such a try missed)
    const bool tiny_try = p.plan.tiny || (p.plan.rounds == 0 && p.tiny_block == 0);
    if (planned && p.tiny_block) p.tiny_block--;
    const bool tiny = planned && tiny_try && !in.dist && p.hist_count &&
                      (size_t)p.plan.bound[0] * rb64 <= kTinyCandBytes &&
                      !tiny_disabled() &&
                      tiny_fits(D, p.Kp, std::min(prefilter_m2(), 2048 / p.Kp), KM, in.K, tiles);
    if (debug_level() >= 2 && p.plan.valid)
        fprintf(stderr, "[sky] plan: planned %d tiny %d (plan.tiny %d hist %d bound0 %u rounds %d fits %d)\n",
                (int)planned, (int)tiny, (int)p.plan.tiny, (int)p.hist_count, p.plan.bound[0], p.plan.rounds,
                (int)tiny_fits(D, p.Kp, std::min(prefilter_m2(), 2048 / p.Kp), KM, in.K, tiles));
    if (planned) SKY_TRY(plan_prepare(p, D, tiny, fill));
    // the fills go with the sample pass (one launch less) unless pmin itself is among them
    FillRanges pre{};
    const bool pre_taken = !pmin_reset && !fill_embed_disabled() && fill.take(pre);
    if (!pre_taken) HIP_TRY(fill.launch(st));
    // small streams: the sample minima only, the filter's workgroups pick the pruners from them (one
    // dependent launch less, where launches are the query's cost); large ones keep k_pick_pruners
    // (every filter workgroup's prologue would wait on two more dependent loads)
    const bool pick_in_filter = n <= kPickInFilterMax;
    launch_select_pruners(D, in.vals, n, S, kp, in.keys, in.single, p.Kp, p.M, p.pmin.as<unsigned long long>(),
                          p.pruners.as<double>(), p.npr.as<int32_t>(), st, !pick_in_filter, ptag,
                          pre_taken ? &pre : nullptr);
    STAGE(st, "pruners");
    if (tm) tm->mark(1, st);

    // ---- the HBM stream: keys + pruner test + status, candidates appended to slots
    //      (f64 rows + sort keys); the row type (f32/f64), the OR/AND of the sort keys
    //      and the slot count are read back in ONE synchronisation
    FilterArgs fa{};
    fa.vals = in.vals;
    fa.n = n;
    fa.kp = kp;
    fa.given_keys = in.keys;
    fa.single = in.single;
    fa.pruners = p.pruners.as<double>();
    fa.npr = p.npr.as<int32_t>();
    fa.M = p.M;
    fa.Kp = p.Kp;
    fa.status = p.status.as<uint16_t>();
    fa.crow = p.rows.as<double>();
    fa.sortkey = p.sortkey.as<uint64_t>();
    fa.slot_src = p.slot_src.as<uint32_t>();
    fa.m_total = p.totals.as<uint32_t>();
    fa.orand = p.orand.as<unsigned long long>();
    fa.dup_cnt = p.dup_cnt.as<uint32_t>();
    fa.flags = p.flags.as<uint32_t>();
    fa.slot_cap = (uint32_t)cap;
    fa.tile_hist = p.hist_count ? p.tile_hist.as<uint32_t>() : nullptr;
    fa.planes = p.planes_on ? p.planes.as<uint64_t>() : nullptr;
    fa.dom_kj = p.dom_kj;
    fa.pick_gmin = pick_in_filter ? p.pmin.as<unsigned long long>() : nullptr;
    fa.pick_S = S;
    fa.pick_tag = ptag;
    fa.pruners_w = p.pruners.as<double>();
    fa.npr_w = p.npr.as<int32_t>();
    {
        static const int fdbg = [] { const char *e = SKY_MEASURE_ENV("SKY_FILTER_DBG"); return e ? atoi(e) : 0; }();
        fa.dbg = fdbg;
    }
    const bool angle_keys = !in.single && !in.keys && c.algo == SKY_ALGO_ANGLE;
    if (angle_keys) {
        SKY_TRY(p.defer.ensure((size_t)n * 4));
        fa.defer_list = p.defer.as<uint32_t>();
        fa.defer_cnt = p.totals.as<uint32_t>() + 6;
    }
    c.ktimer_begin("filter", st);
    launch_filter(D, fa, st);
    c.ktimer_end("filter", st, n);
    if (angle_keys) {
        FilterArgs fd = fa;                    // the pruners are in place by now (filter workgroup 0)
        fd.pick_gmin = nullptr;
        launch_filter_deferred(D, fd, st);
    }
    STAGE(st, "filter");
    if (tm) tm->mark(2, st);

    // ---- one slot per duplicated pruner (device-side, no host round trip)
    AppendArgs aa{};
    aa.pruners = p.pruners.as<double>();
    aa.dup_cnt = p.dup_cnt.as<uint32_t>();
    aa.Kp = p.Kp;
    aa.M = p.M;
    aa.m_total = p.totals.as<uint32_t>();
    aa.nps_total = p.totals.as<uint32_t>() + 5;
    aa.entries = p.pr_entries.as<int32_t>();
    aa.pruner_slot = p.pruner_slot.as<int32_t>();
    aa.rows = p.rows.p;
    aa.sortkey = p.sortkey.as<uint64_t>();
    aa.slot_src = p.slot_src.as<uint32_t>();
    aa.flags = p.flags.as<uint32_t>();
    aa.orand = p.orand.as<unsigned long long>();
    aa.slot_cap = (uint32_t)cap;
    aa.mt_total = p.totals.as<uint32_t>() + 10;
    if (!tiny) launch_append_pruners(D, aa, st);
    STAGE(st, "compact");
    if (planned) return pipe_run_planned(c, p, in, tm, cap, cap_full, tiles, fill, tiny ? &aa : nullptr);
    uint32_t m = 0, nps = 0, flags = 0;
    unsigned long long orand[2] = {0ull, 0ull};
    SKY_TRY(sync_read(p, st, {{p.totals.p, 4}, {p.totals.as<uint32_t>() + 5, 4}, {p.flags.p, 4}, {p.orand.p, 16}},
                      {&m, &nps, &flags, orand}));
    if (tm) tm->mark(3, st);
    if (flags & kFlagNaN) {
        set_error("a tuple value is NaN: the reference BNL result is order-dependent for NaN; rejected");
        return SKY_E_NAN;
    }
    if ((size_t)m + nps > cap) {                 // slots overflowed: again, with room for every candidate
        p.slot_hint = std::min(cap_full, ((size_t)m + nps) * 5 / 4 + (size_t)KM);
        p.slot_reruns++;
        return pipe_run(c, p, in, tm);
    }
    p.slot_hint = std::max(p.slot_hint, std::min(cap_full, 2 * ((size_t)m + nps)));
    p.m = m;
    p.nps = nps;
    p.f64 = (flags & kFlagNotF32) != 0;
    p.ties = (flags & kFlagScoreTies) != 0;
    p.ints = !p.f64 && (flags & kFlagNotU16) == 0;
    p.u16 = p.ints && !p.ties && !sfs16_disabled();
    p.mt = m + nps;
    p.mt_pre = p.mt;
    p.s_rows = &p.rows;
    p.s_key = &p.sortkey;
    p.s_src = &p.slot_src;
    // ---- candidate prefilter: second-level pruners drawn from the candidates drop the
    //      candidates they dominate before the sort (worth it once the candidates
    //      outnumber what one small-SFS workgroup per partition handles)
    // rounds: a round's survivors draw new pruners; another round runs only while the
    // survivors are still too many for the brute path and the last round cut them by > 30 %
    int plan_rounds = 0;
    uint32_t plan_live[kPrefilterRounds] = {};
    // (probed again every kPrefilterProbe queries, and as soon as the slot count moved more than
    // 1/16 from the one it was learned on: a sliding window's candidates change under it)
    const bool pf_moved = p.mt > p.pf_mt + p.pf_mt / 16 || p.mt + p.pf_mt / 16 < p.pf_mt;
    const bool pf_probe = !p.pf_skip || pf_moved || ++p.pf_since_probe >= kPrefilterProbe;
    if (!pf_probe && p.mt >= kPrefilterMin) p.pf_skipped++;
    for (int round = 0; round < kPrefilterRounds && p.mt >= kPrefilterMin && !prefilter_disabled() && pf_probe;
         round++) {
        const uint32_t mt0 = p.mt;
        const int M2 = std::min(prefilter_m2(), 2048 / p.Kp);
        const int KM2 = p.Kp * M2;
        const int KM = p.Kp * p.M;
        DevBuf *dr = round & 1 ? &p.rows3 : &p.rows2, *dk = round & 1 ? &p.sortkey3 : &p.sortkey2,
               *ds = round & 1 ? &p.slot_src3 : &p.slot_src2;
        SKY_TRY(p.cmin.ensure((size_t)KM2 * 8));
        SKY_TRY(p.pr2.ensure((size_t)KM2 * D * 8));
        SKY_TRY(p.npr2.ensure((size_t)p.Kp * 4));
        SKY_TRY(p.live.ensure((size_t)mt0 * 4));
        SKY_TRY(p.livepos.ensure((size_t)(mt0 + 1) * 4));
        SKY_TRY(dr->ensure((size_t)mt0 * rb64));
        SKY_TRY(dk->ensure((size_t)mt0 * 8));
        SKY_TRY(ds->ensure((size_t)mt0 * 4));
        SKY_TRY(p.scratch.ensure(scan_scratch_words(mt0 + 1) * 4 + 64));
        const bool fused = cand_fused_fits(D, p.Kp, M2) && !cand_fused_disabled();
        if (fused) {
            SKY_TRY(p.cand_lb.ensure(cand_lb_bytes(mt0)));
            fill.add(p.cand_lb.p, cand_lb_bytes(mt0));
        }
        fill.add(p.cmin.p, (size_t)KM2 * 8, 0xff);
        HIP_TRY(fill.launch(st));
        CandArgs ca{};
        ca.mt = mt0;
        ca.rows = p.s_rows->as<double>();
        ca.key = p.s_key->as<uint64_t>();
        ca.src = p.s_src->as<uint32_t>();
        ca.Kp = p.Kp;
        ca.M2 = M2;
        ca.cmin = p.cmin.as<unsigned long long>();
        ca.pr2 = p.pr2.as<double>();
        ca.npr2 = p.npr2.as<int32_t>();
        ca.live = p.live.as<uint32_t>();
        c.ktimer_begin("prefilter", st);
        if (fused) {
            ca.rows2 = dr->as<double>();
            ca.key2 = dk->as<uint64_t>();
            ca.src2 = ds->as<uint32_t>();
            ca.d_live = p.totals.as<uint32_t>() + 8;
            ca.pruner_slot = p.pruner_slot.as<int32_t>();
            ca.entries = p.pr_entries.as<int32_t>();
            ca.KM = KM;
            ca.lb = p.cand_lb.as<unsigned long long>();
            ca.picked = cand_picked(mt0);
            ca.ticket = reinterpret_cast<uint32_t *>(p.cand_lb.as<char>() + (size_t)cand_fused_tiles(mt0, ca.picked) * 8);
            ca.err = p.flags.as<uint32_t>();
            launch_cand_min(D, ca, st);
            launch_cand_fused(D, ca, st);
        } else {
            launch_cand_prefilter(D, ca, st);
            scan_excl_u32(ca.live, p.livepos.as<uint32_t>(), mt0, p.totals.as<uint32_t>() + 8, p.scratch.as<uint32_t>(),
                          st);
            launch_cand_compact(D, ca, p.livepos.as<uint32_t>(), dr->as<double>(), dk->as<uint64_t>(),
                                ds->as<uint32_t>(), p.pruner_slot.as<int32_t>(), KM, st);
        }
        c.ktimer_end("prefilter", st, mt0);
        STAGE(st, "prefilter");
        uint32_t live_n = 0;
        SKY_TRY(sync_read(p, st, {{p.totals.as<uint32_t>() + 8, 4}}, {&live_n}));
        p.s_rows = dr;
        p.s_key = dk;
        p.s_src = ds;
        p.mt = live_n;
        plan_live[plan_rounds++] = live_n;
        if (debug_level() >= 3)
            fprintf(stderr, "[sky] prefilter round %d: %u -> %u slots (M2=%d)\n", round, mt0, live_n, M2);
        if (round == 0) {                          // learn whether the next queries should run it
            p.pf_skip = (uint64_t)live_n * 100 > (uint64_t)mt0 * 97 && live_n > brute_max();
            p.pf_mt = mt0;
            p.pf_since_probe = 0;
        }
        if (live_n <= brute_max() || (uint64_t)live_n * 10 > (uint64_t)mt0 * 7) break;
    }
    const uint32_t mt = p.mt;
    // small candidate sets (typical after the prefilter): both skyline levels by one
    // brute-force launch instead of the round-based SFS (SKY_BRUTE=0: A/B knob)
    const bool brute = (in.fate || in.dist) && mt > 0 && mt <= brute_max() && !brute_disabled() && c.warm_mode == 0;
    // the route for the next queries' planned replay: this one's, if it was the small-set one
    p.plan.valid = brute && plan_rounds <= Pipe::Plan::kMaxRounds;
    if (p.plan.valid) {
        p.plan.rounds = plan_rounds;
        p.plan.bound[0] = plan_bound(p.mt_pre);
        for (int r = 0; r < plan_rounds; r++) p.plan.bound[r + 1] = plan_bound(plan_live[r]);
        p.plan.f64 = p.f64;
        p.plan.ints = p.ints;
        p.plan.D = D;
        p.plan.Kp = p.Kp;
        p.plan.M = p.M;
        p.plan.single = in.single;
        p.plan.global = in.global;
        p.plan.tiny = mt <= tiny_brute_rows(D) * 3 / 4;   // the final slots fit the one-workgroup tail
    }
    const size_t rb = row_bytes(p.f64, D);
    SKY_TRY(p.slot_rep.ensure(std::max<size_t>(mt, 1) * 4));
    SKY_TRY(p.alive_l.ensure(std::max<size_t>(mt, 1)));
    SKY_TRY(p.alive_g.ensure(std::max<size_t>(mt, 1)));
    SKY_TRY(p.pruner_fate.ensure(std::max<size_t>(KM, 1)));
    uint32_t mr = 0;
    if (mt && !brute) {
        // ---- sort the candidates by (partition, score, hash)
        SKY_TRY(p.perm.ensure((size_t)mt * 4));
        SKY_TRY(p.key_alt.ensure((size_t)mt * 8));
        SKY_TRY(p.val_alt.ensure((size_t)mt * 4));
        SKY_TRY(p.scratch.ensure(std::max(radix_scratch_words(mt), scan_scratch_words(mt + 1)) * 4 + 64));
        if (debug_level() >= 4) {
            SKY_TRY(p.segalive.ensure(64));
            radix_key_orand(p.s_key->as<uint64_t>(), mt, p.segalive.as<unsigned long long>(), st);
            unsigned long long chk[2] = {0, 0};
            SKY_TRY(sync_read(p, st, {{p.segalive.p, 16}}, {chk}));
            fprintf(stderr, "[sky] orand filter %016llx %016llx recomputed %016llx %016llx\n", orand[0], orand[1],
                    chk[0], chk[1]);
        }
        launch_iota(p.perm.as<uint32_t>(), mt, st);
        hipError_t lerr = hipSuccess;
        const bool alt = radix_sort_pairs(p.s_key->as<uint64_t>(), p.perm.as<uint32_t>(), p.key_alt.as<uint64_t>(),
                                          p.val_alt.as<uint32_t>(), mt, orand[0], orand[1],
                                          p.scratch.as<uint32_t>(), p.flags.as<uint32_t>(), st, &lerr);
        HIP_TRY(lerr);
        STAGE(st, "sort");
        const uint64_t *skey = alt ? p.key_alt.as<uint64_t>() : p.s_key->as<uint64_t>();
        const uint32_t *perm = alt ? p.val_alt.as<uint32_t>() : p.perm.as<uint32_t>();
        if (debug_level() >= 4 && alt) {
            SKY_TRY(p.runflag.ensure((size_t)mt * 4));
            HIP_TRY(hipMemsetAsync(p.totals.as<uint32_t>() + 7, 0, 4, st));
            radix_debug_check(p.s_key->as<uint64_t>(), skey, perm, mt, p.runflag.as<uint32_t>(),
                              p.totals.as<uint32_t>() + 7, st);
            uint32_t bad = 0;
            SKY_TRY(sync_read(p, st, {{p.totals.as<uint32_t>() + 7, 4}}, {&bad}));
            fprintf(stderr, "[sky] sort check m=%u bad=%u\n", mt, bad);
        }
        if (tm) tm->mark(4, st);

        // ---- collapse exact duplicates: one representative per distinct vector
        SKY_TRY(p.rows_sorted.ensure((size_t)mt * rb));
        for (DevBuf *b : {&p.runflag, &p.runscan, &p.run_first, &p.repof, &p.repflag, &p.repscan, &p.rep_of_sorted})
            SKY_TRY(b->ensure((size_t)mt * 4));
        SKY_TRY(p.rep_rows.ensure((size_t)mt * rb));
        SKY_TRY(p.rep_key.ensure((size_t)mt * 8));
        RepArgs ra{};
        ra.mt = mt;
        ra.perm = perm;
        ra.skey = skey;
        ra.rows = p.s_rows->p;
        ra.rows_sorted = p.rows_sorted.p;
        ra.runflag = p.runflag.as<uint32_t>();
        ra.runscan = p.runscan.as<uint32_t>();
        ra.run_first = p.run_first.as<uint32_t>();
        ra.repof = p.repof.as<uint32_t>();
        ra.repflag = p.repflag.as<uint32_t>();
        ra.repscan = p.repscan.as<uint32_t>();
        ra.rep_rows = p.rep_rows.p;
        ra.rep_key = p.rep_key.as<uint64_t>();
        ra.rep_of_sorted = p.rep_of_sorted.as<uint32_t>();
        ra.slot_rep = p.slot_rep.as<uint32_t>();
        launch_gather_runs(D, p.f64, ra, st);
        scan_excl_u32(ra.runflag, ra.runscan, mt, nullptr, p.scratch.as<uint32_t>(), st);
        launch_run_first(ra, st);
        launch_rep_of(D, p.f64, ra, st);
        scan_excl_u32(ra.repflag, ra.repscan, mt, p.totals.as<uint32_t>() + 1, p.scratch.as<uint32_t>(), st);
        launch_build_reps(D, p.f64, ra, st);
        SKY_TRY(p.seg_begin.ensure((size_t)p.Kp * 4));
        SKY_TRY(p.seg_end.ensure((size_t)p.Kp * 4));
        fill.add(p.seg_begin.p, (size_t)p.Kp * 4);
        fill.add(p.seg_end.p, (size_t)p.Kp * 4);
        HIP_TRY(fill.launch(st));
        launch_seg_bounds(p.rep_key.as<uint64_t>(), mt, p.totals.as<uint32_t>() + 1, p.seg_begin.as<uint32_t>(),
                          p.seg_end.as<uint32_t>(), st);
        STAGE(st, "dedup");
        std::vector<uint32_t> sb(p.Kp), se(p.Kp);
        uint32_t flags2 = 0;
        SKY_TRY(sync_read(p, st, {{p.totals.as<uint32_t>() + 1, 4}, {p.seg_begin.p, (size_t)p.Kp * 4},
                                  {p.seg_end.p, (size_t)p.Kp * 4}, {p.flags.p, 4}},
                          {&mr, sb.data(), se.data(), &flags2}));
        if (flags2 & kFlagRadixSpin) {
            set_error("radix sort look-back exceeded its spin bound");
            return SKY_E_HIP;
        }
        p.mr = mr;
        for (int k = 0; k < p.Kp; k++) se[k] -= sb[k];
        if (tm) tm->mark(5, st);

        // ---- local skylines
        // the flags and counters of the SFS / global phases, zeroed in one launch
        const bool gmerge = in.global && !in.single;
        SKY_TRY(p.segalive.ensure((size_t)p.Kp * 4));
        fill.add(p.alive_l.p, mr);
        fill.add(p.segalive.p, (size_t)p.Kp * 4);
        if (gmerge) {
            fill.add(p.alive_g.p, mr);
            fill.add(p.orand.p, 8, 0);
            fill.add(p.orand.as<char>() + 8, 8, 0xff);
        }
        HIP_TRY(fill.launch(st));
        const int W16 = dom16_words(D);
        const bool use_mbr = c.warm_mode == 1 || (c.warm_mode == 0 && mr >= mbr_min() && !mbr_disabled());
        if (use_mbr) {
            SKY_TRY(mbr_run(c, p, in, mr, gmerge));
        } else if (p.u16) {
            SKY_TRY(p.r16.ensure((size_t)std::max<uint32_t>(mr, 1) * W16 * 4));
            launch_pack16(D, p.rep_rows.as<float>(), mr, nullptr, p.r16.as<uint32_t>(), st);
            SKY_TRY(sfs_run16(c, p, p.r16.as<uint32_t>(), mr, sb, se, p.alive_l.as<uint8_t>(), W16));
        } else {
            SKY_TRY(sfs_run(c, p, p.rep_rows.p, p.rep_key.as<uint64_t>(), mr, sb, se, false,
                            p.alive_l.as<uint8_t>()));
        }
        launch_seg_alive(p.rep_key.as<uint64_t>(), p.alive_l.as<uint8_t>(), mr, p.segalive.as<uint32_t>(), st);
        p.h_seg_n.assign(se.begin(), se.end());
        if (tm) tm->mark(6, st);

        // ---- global merge over the union of the local skylines (the all-pairs pass did both)
        if (use_mbr) {
        } else if (gmerge) {
            SKY_TRY(p.alive_u32.ensure((size_t)mr * 4));
            SKY_TRY(p.alive_scan.ensure((size_t)mr * 4));
            SKY_TRY(p.gkey.ensure((size_t)mr * 8));
            SKY_TRY(p.gval.ensure((size_t)mr * 4));
            launch_flag_u8_to_u32(p.alive_l.as<uint8_t>(), mr, p.alive_u32.as<uint32_t>(), st);
            scan_excl_u32(p.alive_u32.as<uint32_t>(), p.alive_scan.as<uint32_t>(), mr, p.totals.as<uint32_t>() + 2,
                          p.scratch.as<uint32_t>(), st);
            launch_global_keys(p.rep_key.as<uint64_t>(), p.alive_l.as<uint8_t>(), p.alive_scan.as<uint32_t>(), mr,
                               p.gkey.as<uint64_t>(), p.gval.as<uint32_t>(), p.orand.as<unsigned long long>(), st);
            uint32_t mg = 0;
            SKY_TRY(sync_read(p, st, {{p.totals.as<uint32_t>() + 2, 4}, {p.orand.p, 16}}, {&mg, orand}));
            p.mg = mg;
            if (mg) {
                SKY_TRY(p.gkey_alt.ensure((size_t)mg * 8));
                SKY_TRY(p.gval_alt.ensure((size_t)mg * 4));
                SKY_TRY(p.grows.ensure((size_t)mg * rb));
                SKY_TRY(p.galive.ensure((size_t)mg));
                hipError_t glerr = hipSuccess;
                const bool galt = radix_sort_pairs(p.gkey.as<uint64_t>(), p.gval.as<uint32_t>(),
                                                   p.gkey_alt.as<uint64_t>(), p.gval_alt.as<uint32_t>(), mg,
                                                   orand[0], orand[1], p.scratch.as<uint32_t>(),
                                                   p.flags.as<uint32_t>(), st, &glerr);
                HIP_TRY(glerr);
                const uint64_t *gk = galt ? p.gkey_alt.as<uint64_t>() : p.gkey.as<uint64_t>();
                const uint32_t *gv = galt ? p.gval_alt.as<uint32_t>() : p.gval.as<uint32_t>();
                FillSet gfill;
                gfill.add(p.galive.p, mg);
                HIP_TRY(gfill.launch(st));
                // computed keys: a vector has one partition, so the union of the
                // partitions' representatives is duplicate-free and the distinct-row
                // test applies; given keys (lists of a merge) may repeat a vector
                if (p.u16 && !in.keys && mg > 2048) {     // small unions: one k_sfs_small launch
                    SKY_TRY(p.r16g.ensure((size_t)mg * W16 * 4));
                    launch_pack16(D, p.rep_rows.as<float>(), mg, gv, p.r16g.as<uint32_t>(), st);
                    SKY_TRY(sfs_run16(c, p, p.r16g.as<uint32_t>(), mg, {0u}, {mg}, p.galive.as<uint8_t>(), W16));
                } else {
                    launch_gather_rows(D, p.f64, p.rep_rows.p, gv, mg, p.grows.p, st);
                    SKY_TRY(sfs_run(c, p, p.grows.p, gk, mg, {0u}, {mg}, true, p.galive.as<uint8_t>()));
                }
                launch_scatter_alive(gv, p.galive.as<uint8_t>(), mg, p.alive_g.as<uint8_t>(), st);
                STAGE(st, "global");
            }
        } else {
            HIP_TRY(hipMemcpyAsync(p.alive_g.p, p.alive_l.p, mr, hipMemcpyDeviceToDevice, st));
        }
    } else if (brute) {
        // ---- small slot set (typical after the prefilter): both skyline levels straight over
        //      the candidate slots, duplicates included (equal vectors never dominate each other),
        //      in one pair launch: no sort, no duplicate collapse, no SFS rounds, no host round
        //      trip (the per-partition counts come back with the final read)
        if (tm) tm->mark(4, st);
        if (tm) tm->mark(5, st);
        SKY_TRY(p.segalive.ensure((size_t)p.Kp * 4));
        SKY_TRY(p.seg_begin.ensure((size_t)p.Kp * 4));
        SKY_TRY(p.keep.ensure((size_t)mt * 4));              // per-slot domination bits
        SKY_TRY(p.slot_rep.ensure((size_t)mt * 4));
        fill.add(p.segalive.p, (size_t)p.Kp * 4);
        fill.add(p.seg_begin.p, (size_t)p.Kp * 4);
        fill.add(p.keep.p, (size_t)mt * 4);
        HIP_TRY(fill.launch(st));
        c.ktimer_begin("brute", st);
        launch_brute_fates(D, !p.f64, p.ints && !brute16_disabled(), p.s_rows->p, p.s_key->as<uint64_t>(), mt, in.global && !in.single,
                           p.keep.as<uint32_t>(), p.alive_l.as<uint8_t>(), p.alive_g.as<uint8_t>(),
                           p.segalive.as<uint32_t>(), p.seg_begin.as<uint32_t>(), p.slot_rep.as<uint32_t>(), st);
        c.ktimer_end("brute", st, (int64_t)mt * mt);
        STAGE(st, "brute");
        if (tm) tm->mark(6, st);
    }
    return pipe_finish(c, p, in, tm, fill, brute, mt, tiles, nullptr);
}

int pipe_output(Ctx &c, Pipe &p, const PipeIn &in, bool select_local, int64_t *d_ids_out, int32_t *d_origin_out,
                double *d_rows_out, int64_t cap, int64_t *n_out, uint8_t *d_row_flags) {
    // the run's count pass selected G (global runs) or L (single-partition runs); the local
    // skyline of a global run needs its own count + scan (stats untouched)
    const bool writes = d_ids_out || d_origin_out || d_rows_out || d_row_flags;
    const bool fused_done = p.fused && !select_local && !d_rows_out && !d_row_flags && d_ids_out == p.fused_ids &&
                            d_origin_out == p.fused_org;
    // the local skyline of a global run, or other buffers than the single-pass output wrote:
    // a count pass + scan of its own (stats untouched)
    const bool recount = p.n > 0 && ((select_local && in.global) || (p.fused && writes && !fused_done));
    if (p.planes_on && p.n > 0 && (recount || d_rows_out || d_row_flags || select_local)) {
        set_error("internal: the run stored status planes, not status words; this output needs the words");
        return SKY_E_HIP;
    }
    uint32_t nsel = p.nout;
    OutArgs oa{};
    oa.status = p.status.as<uint16_t>();
    oa.n = p.n;
    oa.pruner_fate = p.pruner_fate.as<uint8_t>();
    oa.M = p.M;
    oa.KM = p.Kp * p.M;
    oa.given_origin = in.origin;
    oa.given_w = in.weights;
    oa.K = p.K;
    oa.out_cnt = p.out_cnt.as<uint32_t>();
    oa.out_off = p.out_off.as<uint32_t>();
    oa.ids = in.ids;
    oa.vals = in.vals;
    oa.D = c.D;
    oa.ids_out = d_ids_out;
    oa.origin_out = d_origin_out;
    oa.rows_out = d_rows_out;
    oa.select_local = 0;
    if (recount) {
        const uint32_t tiles = (p.n + kTile - 1) / kTile;
        oa.select_local = select_local ? 1 : 0;
        oa.lsz = nullptr;
        oa.surv = nullptr;
        oa.row_flags = nullptr;
        launch_out_count(oa, c.st);
        scan_excl_u32(p.out_cnt.as<uint32_t>(), p.out_off.as<uint32_t>(), tiles, p.totals.as<uint32_t>() + 3,
                      p.scratch.as<uint32_t>(), c.st);
        SKY_TRY(sync_read(p, c.st, {{p.totals.as<uint32_t>() + 3, 4}}, {&nsel}));
    }
    if (n_out) *n_out = nsel;
    if ((int64_t)nsel > cap && (d_ids_out || d_origin_out || d_rows_out)) {
        set_error("output capacity " + std::to_string(cap) + " < skyline size " + std::to_string(nsel));
        return SKY_E_CAPACITY;
    }
    if (p.n == 0) return SKY_OK;
    if (fused_done) return SKY_OK;          // the run's single-pass output already wrote them
    if (d_row_flags) {
        oa.row_flags = d_row_flags;
        oa.lsz = nullptr;
        oa.surv = nullptr;
        launch_out_count(oa, c.st);
        oa.row_flags = nullptr;
    }
    if (d_ids_out || d_origin_out || d_rows_out) {
        c.ktimer_begin("out", c.st);
        c.ktimer_begin("outw", c.st);
        launch_out_write(oa, c.st);
        c.ktimer_end("outw", c.st, p.n);
        c.ktimer_end("out", c.st, 0);
    }
    return SKY_OK;
}

}  // namespace sky
