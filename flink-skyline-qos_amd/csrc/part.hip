// part.hip — the per-key operator state behind SkylineLocalProcessor (sky_part_*,
// sky_parts_insert), FlinkSkyline.java:214-445.
//
// processBuffer (:417-444) sets S <- SKY(S u B) for every 5000-tuple buffer B of a key.  An
// insert here is asynchronous: the batches of one call (one or several keys) are staged into
// pinned memory (the NaN check rides along), uploaded with their descriptors and work items in
// ONE copy, and applied by k_parts_pairs + k_parts_commit (k_part.hip) with device-side counts.
// No host read: launch sizes and capacities come from host bounds (the last counts the commit
// kernel mirrored into host memory, plus every tuple issued since).  The host synchronises only
// when it must see the state: sky_part_size / sky_part_snapshot / compaction / close.
#include "abi_common.h"
#include "knobs.h"
#include "stage_pool.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace {

constexpr size_t kAlign = 256;
inline size_t align_up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

// ---- the staging pool: a call's batches copied into pinned memory (and checked for NaN) by the
// caller plus a few persistent threads
struct StageChunk {
    const int64_t *ids;
    const double *vals;
    int64_t *ids_dst;
    double *vals_dst;
    size_t n;                 // tuples
    int part;
    bool nan;
};
constexpr size_t kStageChunkTuples = 2048;

// copy + NaN check on the bits (NaN <=> |bits| > +inf's bits; the wrapping subtraction sets bit
// 63 exactly then): a loop the compiler vectorises
void stage_one(StageChunk &k, int D) {
    memcpy(k.ids_dst, k.ids, k.n * 8);
    const uint64_t *src = reinterpret_cast<const uint64_t *>(k.vals);
    uint64_t *dst = reinterpret_cast<uint64_t *>(k.vals_dst);
    uint64_t acc = 0;
    const size_t nq = k.n * (size_t)D;
    for (size_t q = 0; q < nq; q++) {
        const uint64_t u = src[q];
        dst[q] = u;
        acc |= 0x7ff0000000000000ull - (u & 0x7fffffffffffffffull);
    }
    k.nan = (acc >> 63) != 0;
}

StagePool &stage_pool() {
    // the caller + 3 workers (SKY_STAGE_THREADS in a measurement build)
    static StagePool pool([] {
        const char *e = SKY_MEASURE_ENV("SKY_STAGE_THREADS");
        return e ? atoi(e) : 4;
    }());
    return pool;
}

void stage_chunks(std::vector<StageChunk> &ch, int D) {
    size_t bytes = 0;
    for (const StageChunk &k : ch) bytes += k.n * (8 + 8 * (size_t)D);
    if (bytes < (256u << 10)) {                              // small: not worth a wake-up
        for (StageChunk &k : ch) stage_one(k, D);
        return;
    }
    stage_pool().run(ch.size(), [&](size_t i) { stage_one(ch[i], D); });
}

// the newest consistent counts the commit kernel mirrored (seqlock: end, data, begin)
void refresh_known(sky_part *p) {
    if (!p->mirror || p->seq_known == p->seq) return;
    volatile const uint32_t *m = p->mirror;
    const uint32_t e = m[5];
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    const uint32_t R = m[1], T = m[2], dlo = m[3], dhi = m[4];
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    const uint32_t b = m[0];
    if (b != e || e == p->seq_known || e == 0) return;
    if ((int32_t)(e - p->seq_known) < 0 || p->seq - e >= kPartRing) return;   // stale, or the ring moved on
    p->seq_known = e;
    p->R_known = R;
    p->T_known = T;
    p->dead_known = ((uint64_t)dhi << 32) | dlo;
    p->cum_known = p->cum[e % kPartRing];
}

inline uint64_t bound_R(const sky_part *p) { return p->R_known + (p->issued - p->cum_known); }
inline uint64_t bound_T(const sky_part *p) { return p->T_known + (p->issued - p->cum_known); }

// wait for the part's work, then its exact counts
int part_sync(sky_part *p) {
    sky_ctx *c = p->ctx;
    c->host_syncs++;
    HIP_TRY(hipStreamSynchronize(c->st));
    p->grave.clear();
    if (!p->pin && hipHostMalloc(&p->pin, 256, hipHostMallocDefault) != hipSuccess) {
        p->pin = nullptr;
        set_error("hipHostMalloc failed");
        return SKY_E_NOMEM;
    }
    if (!p->dcnt.p) {
        memset(p->pin, 0, 16);
    } else {
        HIP_TRY(hipMemcpy(p->pin, p->dcnt.p, 16, hipMemcpyDeviceToHost));
    }
    const uint32_t *h = (const uint32_t *)p->pin;
    p->R_known = h[0];
    p->T_known = h[1];
    p->dead_known = ((uint64_t)h[3] << 32) | h[2];
    p->seq_known = p->seq;
    p->cum_known = p->issued;
    return SKY_OK;
}

// grow a state buffer keeping its first `used` bytes, stream-ordered (the old buffer waits in
// the grave until the next synchronisation)
int grow_async(sky_part *p, DevBuf &b, size_t need, size_t used) {
    if (need <= b.cap && b.p) return SKY_OK;
    DevBuf nb;
    SKY_TRY(nb.ensure(std::max(need, b.cap * 2)));
    if (used && b.p) HIP_TRY(hipMemcpyAsync(nb.p, b.p, std::min(used, b.cap), hipMemcpyDeviceToDevice, p->ctx->st));
    if (b.p) p->grave.push_back(std::move(b));
    b = std::move(nb);
    return SKY_OK;
}

// drop the dead reps and their tuples (order kept); after part_sync
int part_compact(sky_part *p) {
    sky_ctx *c = p->ctx;
    hipStream_t st = c->st;
    const int D = c->D;
    const uint32_t R = (uint32_t)p->R_known, T = (uint32_t)p->T_known;
    SKY_TRY(p->rk.ensure((size_t)R * 4 + 4));
    SKY_TRY(p->rp.ensure((size_t)R * 4 + 4));
    SKY_TRY(p->tk.ensure((size_t)T * 4 + 4));
    SKY_TRY(p->tp.ensure((size_t)T * 4 + 4));
    SKY_TRY(p->rrows2.ensure(std::max<size_t>(p->rrows.cap, 256)));
    SKY_TRY(p->ralive2.ensure(std::max<size_t>(p->ralive.cap, 256)));
    SKY_TRY(p->rcnt2.ensure(std::max<size_t>(p->rcnt.cap, 256)));
    SKY_TRY(p->tids2.ensure(std::max<size_t>(p->tids.cap, 256)));
    SKY_TRY(p->trep2.ensure(std::max<size_t>(p->trep.cap, 256)));
    SKY_TRY(p->scratch.ensure(scan_scratch_words((size_t)std::max(R, T) + 1) * 4 + 64));
    SKY_TRY(p->words.ensure(256));
    uint32_t *w = p->words.as<uint32_t>();
    launch_part_rkeep(R, p->ralive.as<uint8_t>(), p->rk.as<uint32_t>(), st);
    scan_excl_u32(p->rk.as<uint32_t>(), p->rp.as<uint32_t>(), R, w + 8, p->scratch.as<uint32_t>(), st);
    launch_part_rmove(D, R, p->rk.as<uint32_t>(), p->rp.as<uint32_t>(), p->rrows.as<double>(), p->rcnt.as<uint32_t>(),
                      p->rrows2.as<double>(), p->rcnt2.as<uint32_t>(), p->ralive2.as<uint8_t>(), st);
    launch_part_tkeep(T, p->trep.as<uint32_t>(), p->ralive.as<uint8_t>(), p->tk.as<uint32_t>(), st);
    scan_excl_u32(p->tk.as<uint32_t>(), p->tp.as<uint32_t>(), T, w + 9, p->scratch.as<uint32_t>(), st);
    launch_part_tmove(T, p->tk.as<uint32_t>(), p->tp.as<uint32_t>(), p->rp.as<uint32_t>(), p->tids.as<int64_t>(),
                      p->trep.as<uint32_t>(), p->tids2.as<int64_t>(), p->trep2.as<uint32_t>(), st);
    HIP_TRY(hipGetLastError());
    uint32_t h[2] = {0, 0};
    c->host_syncs++;
    HIP_TRY(hipMemcpyAsync(p->pin, w + 8, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    memcpy(h, p->pin, 8);
    std::swap(p->rrows, p->rrows2);
    std::swap(p->ralive, p->ralive2);
    std::swap(p->rcnt, p->rcnt2);
    std::swap(p->tids, p->tids2);
    std::swap(p->trep, p->trep2);
    p->Rcap = std::min({p->rcnt.cap / 4, p->ralive.cap, p->rrows.cap / ((size_t)D * 8)});
    p->Tcap = std::min(p->trep.cap / 4, p->tids.cap / 8);
    const uint32_t cnt[4] = {h[0], h[1], 0u, 0u};
    memcpy(p->pin, cnt, 16);
    HIP_TRY(hipMemcpy(p->dcnt.p, p->pin, 16, hipMemcpyHostToDevice));
    p->R_known = h[0];
    p->T_known = h[1];
    p->dead_known = 0;
    return SKY_OK;
}

Ctx::Staging *take_stage(sky_ctx *c, size_t bytes) {
    Ctx::Staging &s = c->part_stage[c->part_stage_next];
    c->part_stage_next = (c->part_stage_next + 1) % 4;
    if (s.used && s.ev) (void)hipEventSynchronize(s.ev);   // its upload has left (normally long ago)
    s.used = false;
    if (!s.ev && hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) {
        s.ev = nullptr;
        return nullptr;
    }
    if (s.cap < bytes) {
        if (s.h) (void)hipHostFree(s.h);
        s.h = nullptr;
        s.cap = std::max(bytes, (size_t)4 << 20);
        if (hipHostMalloc(&s.h, s.cap, hipHostMallocDefault) != hipSuccess) {
            s.h = nullptr;
            s.cap = 0;
            return nullptr;
        }
    }
    return &s;
}

// SKY_PART_HOSTPROF=1 (measurement only): host time of the insert calls split into the bounds /
// work items, the staging copy, and the copy + launches; printed at process exit
struct HostProf {
    double pre = 0, wait = 0, stage = 0, launch = 0;
    uint64_t calls = 0;
    bool on = SKY_MEASURE_ENV("SKY_PART_HOSTPROF") != nullptr;
    ~HostProf() {
        if (on && calls)
            fprintf(stderr, "[part] %llu calls, host us/call: bounds+items %.2f slot wait %.2f staging %.2f "
                    "copy+launch %.2f\n", (unsigned long long)calls, pre / calls, wait / calls, stage / calls,
                    launch / calls);
    }
};
HostProf g_hprof;
inline double us_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count();
}

int parts_insert(int np_all, sky_part *const *parts_all, const int64_t *const *ids_all,
                 const double *const *values_all, const int64_t *counts_all) {
    sky_ctx *c = parts_all[0]->ctx;
    hipStream_t st = c->st;
    const int D = c->D;
    // the parts with a batch
    std::vector<sky_part *> parts;
    std::vector<const int64_t *> ids;
    std::vector<const double *> values;
    std::vector<int64_t> counts;
    uint64_t ntot = 0;
    for (int g = 0; g < np_all; g++) {
        if (counts_all[g] == 0) continue;
        parts.push_back(parts_all[g]);
        ids.push_back(ids_all[g]);
        values.push_back(values_all[g]);
        counts.push_back(counts_all[g]);
        ntot += (uint64_t)counts_all[g];
    }
    const int np = (int)parts.size();
    const auto t_pre = std::chrono::steady_clock::now();
    if (ntot == 0) return SKY_OK;
    ARG_CHECK(ntot < 0x7fffffffull, "too many tuples in one call");
    // ---- bounds, compaction, capacity (per part; no host read unless compaction is due)
    std::vector<uint64_t> rb(np), tb(np);
    uint64_t rbtot = 0;
    for (int g = 0; g < np; g++) {
        sky_part *p = parts[g];
        refresh_known(p);
        if (p->dead_known >= 4096 && p->dead_known * 2 > p->T_known) {   // more than half the tuples dead
            SKY_TRY(part_sync(p));
            if (p->dead_known) SKY_TRY(part_compact(p));
        }
        const uint64_t nb = (uint64_t)counts[g];
        rb[g] = bound_R(p);
        tb[g] = bound_T(p);
        ARG_CHECK(rb[g] + nb < 0xffffffffull && tb[g] + nb < 0xffffffffull, "partition state too large");
        if (!p->dcnt.p) {
            SKY_TRY(p->dcnt.ensure(64));
            HIP_TRY(hipMemsetAsync(p->dcnt.p, 0, 16, st));
        }
        if (!p->mirror) {
            void *m = nullptr, *dm = nullptr;
            if (hipHostMalloc(&m, 64, hipHostMallocCoherent) == hipSuccess) {
                memset(m, 0, 64);
                if (hipHostGetDevicePointer(&dm, m, 0) == hipSuccess) {
                    p->mirror = (uint32_t *)m;
                    p->mirror_dev = (uint32_t *)dm;
                } else {
                    (void)hipHostFree(m);
                }
            }
        }
        const size_t Rn = (size_t)(rb[g] + nb), Tn = (size_t)(tb[g] + nb);
        if (Rn > p->Rcap) {
            const size_t want = std::max(Rn, p->Rcap * 2);
            SKY_TRY(grow_async(p, p->rrows, want * D * 8, (size_t)rb[g] * D * 8));
            SKY_TRY(grow_async(p, p->ralive, want, (size_t)rb[g]));
            SKY_TRY(grow_async(p, p->rcnt, want * 4, (size_t)rb[g] * 4));
            p->Rcap = want;
        }
        if (Tn > p->Tcap) {
            const size_t want = std::max(Tn, p->Tcap * 2);
            SKY_TRY(grow_async(p, p->tids, want * 8, (size_t)tb[g] * 8));
            SKY_TRY(grow_async(p, p->trep, want * 4, (size_t)tb[g] * 4));
            p->Tcap = want;
        }
        rbtot += rb[g];
    }
    // ---- work items: batch vs batch, batch vs state, state vs batch (over the undecided tuples
    //      k_parts_prune leaves; their count lives on the device, the batch size bounds it)
    std::vector<PartItem> items;
    for (int g = 0; g < np; g++) {
        const uint32_t nb = (uint32_t)counts[g];
        for (uint32_t y = 0; y < nb; y += kPartItemY) {
            for (uint32_t x = 0; x < nb; x += kPartItemX) items.push_back(PartItem{(uint32_t)g, 0u, y, x});
            for (uint64_t x = 0; x < rb[g]; x += kPartItemX) items.push_back(PartItem{(uint32_t)g, 1u, y, (uint32_t)x});
        }
        for (uint64_t y = 0; y < rb[g]; y += kPartItemY)
            for (uint32_t x = 0; x < nb; x += kPartItemX) items.push_back(PartItem{(uint32_t)g, 2u, (uint32_t)y, x});
    }
    // ---- the upload: descriptors, items, ids, rows (one pinned staging slot, one copy)
    const size_t o_desc = 0, o_items = align_up((size_t)np * sizeof(PartDesc));
    const size_t o_ids = o_items + align_up(items.size() * sizeof(PartItem));
    const size_t o_vals = o_ids + align_up((size_t)ntot * 8);
    const size_t up_bytes = o_vals + (size_t)ntot * D * 8;
    if (g_hprof.on) g_hprof.pre += us_since(t_pre);
    const auto t_wait = std::chrono::steady_clock::now();
    Ctx::Staging *sg = take_stage(c, up_bytes);
    if (g_hprof.on) g_hprof.wait += us_since(t_wait);
    const auto t_stage = std::chrono::steady_clock::now();
    if (!sg) {
        set_error("pinned staging allocation failed");
        return SKY_E_NOMEM;
    }
    char *h = (char *)sg->h;
    bool nan = false;
    int nan_part = -1;
    {
        // staged and checked in one pass, in chunks spread over the staging pool (the caller and
        // SKY_STAGE_THREADS - 1 persistent threads): one thread copies ~10 GB/s, and a call's
        // 0.8 MB was most of the host side of the operator path
        std::vector<StageChunk> ch;
        uint64_t off = 0;
        for (int g = 0; g < np; g++) {
            const size_t nb = (size_t)counts[g];
            for (size_t t0 = 0; t0 < nb; t0 += kStageChunkTuples) {
                const size_t t1 = std::min(nb, t0 + kStageChunkTuples);
                ch.push_back(StageChunk{ids[g] + t0, values[g] + t0 * D, (int64_t *)(h + o_ids) + off + t0,
                                        (double *)(h + o_vals) + (off + t0) * D, t1 - t0, g, false});
            }
            off += nb;
        }
        stage_chunks(ch, D);
        if (g_hprof.on) g_hprof.stage += us_since(t_stage);
        for (const StageChunk &k : ch)
            if (k.nan && (!nan || k.part < nan_part)) {
                nan = true;
                nan_part = k.part;
            }
    }
    if (nan) {   // the whole call is rejected before any launch: the states never see the batch
        set_error("a tuple value is NaN (batch of key " + std::to_string(parts[nan_part]->key) +
                  "): the reference BNL result is order-dependent for NaN; batch rejected");
        return SKY_E_NAN;
    }
    const auto t_launch = std::chrono::steady_clock::now();
    // double-buffered upload target: this call's copy may run while the previous call's kernels
    // still read the other buffer; a buffer is overwritten only after the kernels that read it
    if (!c->part_copy_st) {
        HIP_TRY(hipStreamCreateWithFlags(&c->part_copy_st, hipStreamNonBlocking));
        for (hipEvent_t &e : c->part_done) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    const int bsel = c->part_buf_next;
    c->part_buf_next ^= 1;
    DevBuf &pbuf = c->part_batch[bsel];
    if (up_bytes > pbuf.cap && c->part_done_rec[bsel]) HIP_TRY(hipEventSynchronize(c->part_done[bsel]));
    SKY_TRY(pbuf.ensure(up_bytes));
    // work arrays: dom_b | eq_s | eq_b | kpos | fpos | eqp | uidx (per tuple), meta (per part),
    // dom_s (per bounded rep)
    const size_t w_nb = (size_t)ntot * 4;
    // per-slice words: criterion minima (f64 + index per criterion), kept / new-rep counts
    uint64_t sltot = 0;
    uint32_t max_sl = 0;
    for (int g = 0; g < np; g++) {
        const uint32_t ns = (uint32_t)(((uint64_t)counts[g] + kPartSlice - 1) / kPartSlice);
        sltot += ns;
        max_sl = std::max(max_sl, ns);
    }
    const size_t sl_bytes = (size_t)sltot * (kPartPruners * 12 + 8);
    SKY_TRY(c->part_work.ensure(7 * w_nb + (size_t)np * kPartMeta * 4 + sl_bytes + 16 +
                                (size_t)std::max<uint64_t>(rbtot, 1) * 4 + 64));
    char *dev = pbuf.as<char>();
    uint32_t *w = c->part_work.as<uint32_t>();
    uint32_t *w_dom_b = w, *w_eq_s = w + ntot, *w_eq_b = w + 2 * ntot, *w_kpos = w + 3 * ntot, *w_fpos = w + 4 * ntot;
    uint32_t *w_eqp = w + 5 * ntot, *w_uidx = w + 6 * ntot, *w_meta = w + 7 * ntot;
    // the f64 slice minima 8-byte aligned
    double *w_slv = reinterpret_cast<double *>(
        (reinterpret_cast<uintptr_t>(w_meta + (size_t)np * kPartMeta) + 7) & ~uintptr_t(7));
    uint32_t *w_sli = reinterpret_cast<uint32_t *>(w_slv + (size_t)sltot * kPartPruners);
    uint32_t *w_slk = w_sli + (size_t)sltot * kPartPruners;
    uint32_t *w_dom_s = w_slk + 2 * (size_t)sltot;
    {
        PartDesc *ds = (PartDesc *)(h + o_desc);
        uint64_t off = 0, roff = 0, sloff = 0;
        for (int g = 0; g < np; g++) {
            sky_part *p = parts[g];
            PartDesc d{};
            const uint32_t nb = (uint32_t)counts[g];
            d.bvals = (const double *)(dev + o_vals) + off * D;
            d.bids = (const int64_t *)(dev + o_ids) + off;
            d.nb = nb;
            d.rb = (uint32_t)rb[g];
            d.dom_b = w_dom_b + off;
            d.eq_s = w_eq_s + off;
            d.eq_b = w_eq_b + off;
            d.kpos = w_kpos + off;
            d.fpos = w_fpos + off;
            d.dom_s = w_dom_s + roff;
            d.eqp = w_eqp + off;
            d.uidx = w_uidx + off;
            d.meta = w_meta + (size_t)g * kPartMeta;
            d.sl_v = w_slv + (size_t)sloff * kPartPruners;
            d.sl_i = w_sli + (size_t)sloff * kPartPruners;
            d.sl_k = w_slk + 2 * (size_t)sloff;
            sloff += ((uint64_t)nb + kPartSlice - 1) / kPartSlice;
            d.rrows = p->rrows.as<double>();
            d.ralive = p->ralive.as<uint8_t>();
            d.rcnt = p->rcnt.as<uint32_t>();
            d.tids = p->tids.as<int64_t>();
            d.trep = p->trep.as<uint32_t>();
            d.dcnt = p->dcnt.as<uint32_t>();
            d.mirror = p->mirror_dev;
            p->seq++;
            p->issued += nb;
            p->cum[p->seq % kPartRing] = p->issued;
            d.seq = p->seq;
            ds[g] = d;
            off += nb;
            roff += rb[g];
        }
        if (!items.empty()) memcpy(h + o_items, items.data(), items.size() * sizeof(PartItem));
    }
    if (c->part_done_rec[bsel]) HIP_TRY(hipStreamWaitEvent(c->part_copy_st, c->part_done[bsel], 0));
    HIP_TRY(hipMemcpyAsync(dev, h, up_bytes, hipMemcpyHostToDevice, c->part_copy_st));
    HIP_TRY(hipEventRecord(sg->ev, c->part_copy_st));
    sg->used = true;
    HIP_TRY(hipStreamWaitEvent(st, sg->ev, 0));      // the kernels wait for their upload
    // (the work arrays are initialised by k_parts_prune: no fill launch)
    launch_parts_insert(D, (const PartDesc *)(dev + o_desc), np, max_sl, (const PartItem *)(dev + o_items),
                        (uint32_t)items.size(), st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->part_done[bsel], st));
    c->part_done_rec[bsel] = true;
    if (g_hprof.on) {
        g_hprof.launch += us_since(t_launch);
        g_hprof.calls++;
    }
    return SKY_OK;
}

// GlobalSkylineAggregator (FlinkSkyline.java:515-569) over lists held as distinct vectors: list g
// has R[g] reps (rows already concatenated into c->h_vals, weights = tuples on each rep in
// c->pgm_w, origins in c->h_origin) and T[g] tuples (id, rep index) at src[g].  The alive reps
// run through the single-partition pipeline, the surviving reps are flagged, and every list's
// tuples whose rep survives are written in list order, then insertion order: the result, its
// order, the origins and sky_global_stats equal sky_global_merge over the expanded lists.
struct PgmSrc {
    const int64_t *tids;
    const uint32_t *trep;
};
int pgm_core(sky_ctx *c, int nparts, const uint32_t *R, const uint32_t *T, const PgmSrc *src, const int32_t *part_ids,
             int64_t *ids_out, int32_t *origin_out, int64_t cap, int64_t *n_out) {
    hipStream_t st = c->st;
    uint64_t rtot = 0, ttot = 0;
    for (int g = 0; g < nparts; g++) {
        rtot += R[g];
        ttot += T[g];
    }
    const size_t rr = (size_t)std::max<uint64_t>(rtot, 1), tt = (size_t)std::max<uint64_t>(ttot, 1);
    SKY_TRY(c->pgm_surv.ensure(rr * 8));
    SKY_TRY(c->pgm_sorg.ensure(rr * 4));
    SKY_TRY(c->pgm_flag.ensure(rr));
    PipeIn in;
    in.vals = c->h_vals.as<double>();
    in.n = (uint32_t)rtot;
    in.ids = nullptr;                           // the rep's index in the concatenation
    in.origin = c->h_origin.as<int32_t>();
    in.weights = c->pgm_w.as<int64_t>();
    in.single = true;
    in.global = false;
    in.K = std::max(nparts, 1);
    c->shard_valid = false;
    SKY_TRY(pipe_run(*c, c->main, in, nullptr));
    // GlobalSkylineAggregator: localSkylineSizes[k] = incoming list size (:544); survivors by
    // originPartition (:593-596), weighted by the tuples on each rep
    c->K_last = nparts;
    c->lsz.assign(nparts, 0);
    c->surv.assign(nparts, 0);
    uint64_t gtot = 0;
    for (int g = 0; g < nparts; g++) {
        c->lsz[g] = T[g];
        c->surv[g] = (int64_t)c->main.h_lsz[g];
        gtot += (uint64_t)c->main.h_lsz[g];
    }
    if (n_out) *n_out = (int64_t)gtot;
    if ((int64_t)gtot > cap && (ids_out || origin_out)) {
        set_error("output capacity too small");
        return SKY_E_CAPACITY;
    }
    const uint32_t greps = (uint32_t)c->main.nout;
    int64_t gr = 0;
    SKY_TRY(pipe_output(*c, c->main, in, false, c->pgm_surv.as<int64_t>(), c->pgm_sorg.as<int32_t>(), nullptr,
                        (int64_t)rr, &gr, nullptr));
    HIP_TRY(hipMemsetAsync(c->pgm_flag.p, 0, rr, st));
    launch_pgm_flags(greps, c->pgm_surv.as<int64_t>(), c->pgm_flag.as<uint8_t>(), st);
    // every list's tuples whose rep survives, list order then insertion order
    std::vector<PgmList> lists((size_t)std::max(nparts, 1));
    uint64_t toff = 0, roff = 0;
    for (int g = 0; g < nparts; g++) {
        PgmList &L = lists[g];
        L.tids = src[g].tids;
        L.trep = src[g].trep;
        L.toff = (uint32_t)toff;
        L.roff = (uint32_t)roff;
        L.part_id = part_ids ? part_ids[g] : g;
        L.nrep = R[g];
        toff += T[g];
        roff += R[g];
    }
    SKY_TRY(c->pgm_lists.ensure(lists.size() * sizeof(PgmList)));
    SKY_TRY(c->pgm_tsel.ensure(tt * 4));
    SKY_TRY(c->pgm_tpos.ensure(tt * 4 + 64));
    SKY_TRY(c->pgm_scr.ensure(scan_scratch_words(tt) * 4 + 64));
    SKY_TRY(c->pgm_ids.ensure((size_t)std::max<uint64_t>(gtot, 1) * 8));
    SKY_TRY(c->pgm_org.ensure((size_t)std::max<uint64_t>(gtot, 1) * 4));
    SKY_TRY(c->pgm_err.ensure(64));
    HIP_TRY(hipMemsetAsync(c->pgm_err.p, 0, 4, st));
    HIP_TRY(hipMemcpyAsync(c->pgm_lists.p, lists.data(), lists.size() * sizeof(PgmList), hipMemcpyHostToDevice, st));
    launch_pgm_tuples(c->pgm_lists.as<PgmList>(), nparts, (uint32_t)ttot, c->pgm_flag.as<uint8_t>(),
                      c->pgm_tsel.as<uint32_t>(), c->pgm_tpos.as<uint32_t>(), c->pgm_tpos.as<uint32_t>() + tt,
                      c->pgm_scr.as<uint32_t>(), c->pgm_ids.as<int64_t>(), c->pgm_org.as<int32_t>(),
                      c->pgm_err.as<uint32_t>(), st);
    HIP_TRY(hipGetLastError());
    uint32_t herr = 0;
    if (gtot && ids_out) HIP_TRY(hipMemcpyAsync(ids_out, c->pgm_ids.p, gtot * 8, hipMemcpyDeviceToHost, st));
    if (gtot && origin_out) HIP_TRY(hipMemcpyAsync(origin_out, c->pgm_org.p, gtot * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&herr, c->pgm_err.p, 4, hipMemcpyDeviceToHost, st));
    c->host_syncs++;
    HIP_TRY(hipStreamSynchronize(st));
    if (herr) {
        set_error("a tuple's rep index is not below its list's rep count");
        return SKY_E_ARG;
    }
    return SKY_OK;
}

}  // namespace

extern "C" {

int sky_part_open(sky_ctx *c, int32_t key, sky_part **out) {
    GUARD_BEGIN
    ARG_CHECK(c && out, "null argument");
    sky_part *p = new sky_part();
    p->ctx = c;
    p->key = key;
    *out = p;
    return SKY_OK;
    GUARD_END
}

int sky_part_close(sky_part *p) {
    if (!p) return SKY_OK;
    hipSetDevice(p->ctx->dev);
    hipStreamSynchronize(p->ctx->st);
    delete p;
    return SKY_OK;
}

int sky_part_size(sky_part *p, int64_t *n_out) {
    GUARD_BEGIN
    ARG_CHECK(p && n_out, "null argument");
    SKY_TRY(bind(p->ctx));
    SKY_TRY(part_sync(p));
    *n_out = (int64_t)(p->T_known - p->dead_known);
    return SKY_OK;
    GUARD_END
}

// SkylineLocalProcessor.processBuffer (FlinkSkyline.java:417-444) for one key
int sky_part_insert(sky_part *p, const int64_t *ids, const double *values, int64_t n) {
    GUARD_BEGIN
    ARG_CHECK(p && (n == 0 || (ids && values)), "null argument");
    ARG_CHECK(n >= 0 && n < (int64_t)0x7fffffffLL, "n out of range");
    if (n == 0) return SKY_OK;
    SKY_TRY(bind(p->ctx));
    return parts_insert(1, &p, &ids, &values, &n);
    GUARD_END
}

// processBuffer for the full buffers of several keys of one context in one launch set
int sky_parts_insert(int nparts, sky_part *const *parts, const int64_t *const *ids, const double *const *values,
                     const int64_t *counts) {
    GUARD_BEGIN
    ARG_CHECK(nparts >= 0 && nparts <= 65536, "nparts out of range");
    if (nparts == 0) return SKY_OK;
    ARG_CHECK(parts && ids && values && counts, "null argument");
    for (int g = 0; g < nparts; g++) {
        ARG_CHECK(parts[g] && parts[g]->ctx == parts[0]->ctx, "every part must belong to one context");
        ARG_CHECK(counts[g] >= 0 && counts[g] < (int64_t)0x7fffffffLL, "count out of range");
        ARG_CHECK(counts[g] == 0 || (ids[g] && values[g]), "null batch");
        for (int h = 0; h < g; h++) ARG_CHECK(parts[h] != parts[g], "a part appears twice in one call");
    }
    SKY_TRY(bind(parts[0]->ctx));
    return parts_insert(nparts, parts, ids, values, counts);
    GUARD_END
}

// GlobalSkylineAggregator over the keys' device-resident states (co-located aggregator): the
// same result and stats as sky_global_merge over the parts' snapshots, without moving the local
// skylines through host memory (see skyline_hip.h)
int sky_parts_global_merge(sky_ctx *c, int nparts, sky_part *const *parts, const int32_t *part_ids,
                           int64_t *ids_out, int32_t *origin_out, int64_t cap, int64_t *n_out) {
    GUARD_BEGIN
    ARG_CHECK(c && nparts >= 0 && nparts <= SKY_MAX_PARTITIONS, "bad nparts (<= 256 parts)");
    ARG_CHECK(nparts == 0 || parts, "null parts");
    for (int g = 0; g < nparts; g++) {
        ARG_CHECK(parts[g] && parts[g]->ctx == c, "every part must belong to this context");
        for (int h = 0; h < g; h++) ARG_CHECK(parts[h] != parts[g], "a part appears twice");
    }
    SKY_TRY(bind(c));
    hipStream_t st = c->st;
    const int D = c->D;
    // exact counts; dead reps and their tuples dropped (insertion order kept)
    std::vector<uint32_t> R(nparts), T(nparts);
    std::vector<PgmSrc> src(nparts);
    uint64_t rtot = 0, ttot = 0;
    for (int g = 0; g < nparts; g++) {
        sky_part *p = parts[g];
        SKY_TRY(part_sync(p));
        if (p->dead_known) SKY_TRY(part_compact(p));
        R[g] = (uint32_t)p->R_known;
        T[g] = (uint32_t)p->T_known;
        src[g] = PgmSrc{p->tids.as<int64_t>(), p->trep.as<uint32_t>()};
        rtot += R[g];
        ttot += T[g];
    }
    ARG_CHECK(rtot < 0x7fffffffull && ttot < 0x7fffffffull, "too many tuples");
    const size_t rr = (size_t)std::max<uint64_t>(rtot, 1);
    SKY_TRY(c->h_vals.ensure(rr * D * 8));
    SKY_TRY(c->h_origin.ensure(rr * 4));
    SKY_TRY(c->pgm_w.ensure(rr * 8));
    // the alive reps of every part as one single-partition run (origin = list, weight = tuples)
    uint64_t off = 0;
    for (int g = 0; g < nparts; g++) {
        if (!R[g]) continue;
        HIP_TRY(hipMemcpyAsync(c->h_vals.as<double>() + off * D, parts[g]->rrows.p, (size_t)R[g] * D * 8,
                               hipMemcpyDeviceToDevice, st));
        launch_pgm_prep(R[g], parts[g]->rcnt.as<uint32_t>(), g, c->h_origin.as<int32_t>() + off,
                        c->pgm_w.as<int64_t>() + off, st);
        off += R[g];
    }
    HIP_TRY(hipGetLastError());
    return pgm_core(c, nparts, R.data(), T.data(), src.data(), part_ids, ids_out, origin_out, cap, n_out);
    GUARD_END
}

// GlobalSkylineAggregator over local skylines shipped as distinct vectors (sky_part_snapshot_reps):
// the aggregator of a job whose local processors run elsewhere (see skyline_hip.h)
int sky_global_merge_reps(sky_ctx *c, int nlists, const int32_t *part_ids, const int64_t *const *ids,
                          const int32_t *const *rep_idx, const int64_t *counts, const double *const *reps,
                          const int32_t *const *rep_counts, const int64_t *nreps, int64_t *ids_out,
                          int32_t *origin_out, int64_t cap, int64_t *n_out) {
    GUARD_BEGIN
    ARG_CHECK(c && nlists >= 0 && nlists <= SKY_MAX_PARTITIONS, "bad nlists (<= 256 lists)");
    ARG_CHECK(nlists == 0 || (ids && rep_idx && counts && reps && rep_counts && nreps), "null argument");
    uint64_t rtot = 0, ttot = 0;
    for (int g = 0; g < nlists; g++) {
        ARG_CHECK(counts[g] >= 0 && nreps[g] >= 0, "negative count");
        ARG_CHECK(counts[g] == 0 || (ids[g] && rep_idx[g]), "null tuple list");
        ARG_CHECK(nreps[g] == 0 || (reps[g] && rep_counts[g]), "null rep list");
        ARG_CHECK(counts[g] == 0 || nreps[g] > 0, "tuples without reps");
        rtot += (uint64_t)nreps[g];
        ttot += (uint64_t)counts[g];
    }
    ARG_CHECK(rtot < 0x7fffffffull && ttot < 0x7fffffffull, "too many tuples");
    SKY_TRY(bind(c));
    hipStream_t st = c->st;
    const int D = c->D;
    const size_t rr = (size_t)std::max<uint64_t>(rtot, 1), tt = (size_t)std::max<uint64_t>(ttot, 1);
    SKY_TRY(c->h_vals.ensure(rr * D * 8));
    SKY_TRY(c->h_origin.ensure(rr * 4));
    SKY_TRY(c->pgm_w.ensure(rr * 8));
    // the lists' tuples: ids [tt] then rep indices [tt] (weights and origins built here)
    SKY_TRY(c->pgm_up.ensure(tt * 12 + 256));
    std::vector<int64_t> w((size_t)rtot);
    std::vector<int32_t> org((size_t)rtot);
    std::vector<uint32_t> R(nlists), T(nlists);
    std::vector<PgmSrc> src(nlists);
    uint64_t roff = 0, toff = 0;
    for (int g = 0; g < nlists; g++) {
        R[g] = (uint32_t)nreps[g];
        T[g] = (uint32_t)counts[g];
        // the reps' tuple counts are the pipeline's weights (|L_k| = counts[g], survivors_k = the
        // weight of the surviving reps): each >= 1 and together exactly the list's tuples, or
        // sky_global_stats could report survivors above the local size
        int64_t wsum = 0;
        for (uint32_t r = 0; r < R[g]; r++) {
            ARG_CHECK(rep_counts[g][r] >= 1, "rep_counts: a distinct vector must carry at least one tuple");
            wsum += rep_counts[g][r];
            w[roff + r] = rep_counts[g][r];
            org[roff + r] = g;
        }
        ARG_CHECK(wsum == counts[g], "rep_counts of a list must sum to its tuple count");
        if (R[g]) HIP_TRY(hipMemcpyAsync(c->h_vals.as<double>() + roff * D, reps[g], (size_t)R[g] * D * 8,
                                         hipMemcpyHostToDevice, st));
        int64_t *d_ids = c->pgm_up.as<int64_t>() + toff;
        uint32_t *d_rep = reinterpret_cast<uint32_t *>(c->pgm_up.as<int64_t>() + tt) + toff;
        if (T[g]) {
            HIP_TRY(hipMemcpyAsync(d_ids, ids[g], (size_t)T[g] * 8, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(d_rep, rep_idx[g], (size_t)T[g] * 4, hipMemcpyHostToDevice, st));
        }
        src[g] = PgmSrc{d_ids, d_rep};
        roff += R[g];
        toff += T[g];
    }
    if (rtot) {
        HIP_TRY(hipMemcpyAsync(c->pgm_w.p, w.data(), (size_t)rtot * 8, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(c->h_origin.p, org.data(), (size_t)rtot * 4, hipMemcpyHostToDevice, st));
    }
    return pgm_core(c, nlists, R.data(), T.data(), src.data(), part_ids, ids_out, origin_out, cap, n_out);
    GUARD_END
}

// exact tuple and distinct-vector counts of a part (after its pending work)
int sky_part_sizes(sky_part *p, int64_t *n_tuples, int64_t *n_reps) {
    GUARD_BEGIN
    ARG_CHECK(p && n_tuples && n_reps, "null argument");
    SKY_TRY(bind(p->ctx));
    SKY_TRY(part_sync(p));
    if (p->dead_known) SKY_TRY(part_compact(p));
    *n_tuples = (int64_t)p->T_known;
    *n_reps = (int64_t)p->R_known;
    return SKY_OK;
    GUARD_END
}

// the state as distinct vectors: tuples (id, rep index) in insertion order, reps (values, tuples
// on each) -- what a local processor ships to an aggregator elsewhere (sky_global_merge_reps)
int sky_part_snapshot_reps(sky_part *p, int64_t *ids_out, int32_t *rep_out, int64_t cap, double *reps_out,
                           int32_t *rep_count_out, int64_t rep_cap, int64_t *n_out, int64_t *nrep_out) {
    GUARD_BEGIN
    ARG_CHECK(p, "null part");
    sky_ctx *c = p->ctx;
    SKY_TRY(bind(c));
    SKY_TRY(part_sync(p));
    if (p->dead_known) SKY_TRY(part_compact(p));
    const int64_t T = (int64_t)p->T_known, R = (int64_t)p->R_known;
    if (n_out) *n_out = T;
    if (nrep_out) *nrep_out = R;
    if (T > cap || R > rep_cap) {
        set_error("snapshot capacity too small");
        return SKY_E_CAPACITY;
    }
    if (T && ids_out) HIP_TRY(hipMemcpyAsync(ids_out, p->tids.p, (size_t)T * 8, hipMemcpyDeviceToHost, c->st));
    if (T && rep_out) HIP_TRY(hipMemcpyAsync(rep_out, p->trep.p, (size_t)T * 4, hipMemcpyDeviceToHost, c->st));
    if (R && reps_out)
        HIP_TRY(hipMemcpyAsync(reps_out, p->rrows.p, (size_t)R * c->D * 8, hipMemcpyDeviceToHost, c->st));
    if (R && rep_count_out)
        HIP_TRY(hipMemcpyAsync(rep_count_out, p->rcnt.p, (size_t)R * 4, hipMemcpyDeviceToHost, c->st));
    c->host_syncs++;
    HIP_TRY(hipStreamSynchronize(c->st));
    return SKY_OK;
    GUARD_END
}

int sky_part_snapshot(sky_part *p, int64_t *ids_out, double *values_out, int64_t cap, int64_t *n_out) {
    GUARD_BEGIN
    ARG_CHECK(p, "null part");
    sky_ctx *c = p->ctx;
    SKY_TRY(bind(c));
    SKY_TRY(part_sync(p));
    const int64_t live = (int64_t)(p->T_known - p->dead_known);
    if (n_out) *n_out = live;
    if (live > cap) {
        set_error("snapshot capacity too small");
        return SKY_E_CAPACITY;
    }
    if (live == 0) return SKY_OK;
    if (p->dead_known) SKY_TRY(part_compact(p));
    const int D = c->D;
    const size_t T = (size_t)p->T_known;
    if (ids_out) HIP_TRY(hipMemcpyAsync(ids_out, p->tids.p, T * 8, hipMemcpyDeviceToHost, c->st));
    if (values_out) {
        SKY_TRY(p->out_rows.ensure(T * D * 8));
        launch_part_rows_out(D, (uint32_t)T, p->trep.as<uint32_t>(), p->rrows.as<double>(), p->out_rows.as<double>(),
                             c->st);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(values_out, p->out_rows.p, T * D * 8, hipMemcpyDeviceToHost, c->st));
    }
    c->host_syncs++;
    HIP_TRY(hipStreamSynchronize(c->st));
    return SKY_OK;
    GUARD_END
}

}  // extern "C"
