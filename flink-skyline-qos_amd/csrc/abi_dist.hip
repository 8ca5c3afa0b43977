// abi_dist.hip — the multi-GPU step with one host read (include/skyline_hip.h, "multi-GPU").
//
// The reference scales out by Flink's keyBy shuffle to P keys and one reducer per query
// (FlinkSkyline.java:138, :171-174; GlobalSkylineAggregator :515-569).  Here each rank (one
// process per GPU) owns a shard of the stream; SKY(u SKY(shard_r)) = SKY(u shard_r) makes the
// split exact.  One step:
//   sky_dist_export_dev  the shard's local skylines (the planned small-set route replays with
//                        device-sized launches) -> this rank's block: its distinct local-skyline
//                        vectors with key and multiplicity, plus a header whose verdict carries
//                        the run's checks (planned-route assumptions, NaN)
//   caller: RCCL all-gather of the fixed-size blocks (no host-side sizes needed)
//   sky_dist_merge_dev   own vectors against the union (small: one pair kernel straight over the
//                        blocks; large: the bounding-box pass, own tiles vs union tiles), the
//                        shard's per-tuple fates and stream-ordered output, this rank's share of
//                        |L_k| / survivors_k into the caller's int64 buffer
//   caller: RCCL all-reduce (sum) of the shares
//   sky_dist_finish      the step's one host read: every rank's verdict and count (all ranks
//                        reach the same decision from the same gathered headers), the output
//                        count, the summed integers behind the optimality (:593-608)
#include "abi_common.h"
#include "knobs.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace sky {
size_t mbr_group_slots(uint32_t mr);   // k_mbr.hip: gmin / gprange entries (groups + super-groups)
uint32_t dist_export_one_max();        // k_dist.hip
bool dist_summary_fused(int world);    // k_dist.hip: the pair pass computes k_dist_summary's words
}

namespace {

// pair tests below which the own-vs-union fates run as one pair kernel over the blocks
// (SKY_DIST_BRUTE_PAIRS overrides, read per call: tests force the bounding-box route)
uint64_t dist_brute_pairs() {
    const char *e = SKY_ENV("SKY_DIST_BRUTE_PAIRS");
    return e ? strtoull(e, nullptr, 10) : (1ull << 28);
}

// the wide pair pass's per-own-row bits: zeroed when (re)allocated, cleared by its finish kernel
int dist_dom_ready(Pipe &p, int64_t cap, hipStream_t st) {
    const size_t bytes = (size_t)std::max<int64_t>(cap, 1) * 4;
    const void *before = p.dist_dom.p;
    const size_t cap_before = p.dist_dom.cap;
    SKY_TRY(p.dist_dom.ensure(bytes));
    if (p.dist_dom.p != before || p.dist_dom.cap != cap_before) HIP_TRY(hipMemsetAsync(p.dist_dom.p, 0, p.dist_dom.cap, st));
    return SKY_OK;
}

int dist_write_block(sky_ctx *c, int64_t *d_block, int64_t cap) {
    Pipe &p = c->main;
    hipStream_t st = c->st;
    const int D = c->D;
    const uint32_t units = p.dist_n;
    SKY_TRY(p.dist_flag.ensure((size_t)std::max<uint32_t>(units, 1) * 4));
    SKY_TRY(p.dist_pos.ensure(((size_t)units + 1) * 4));
    SKY_TRY(p.scratch.ensure(scan_scratch_words((size_t)units + 1) * 4 + 64));
    uint32_t *d_count = p.totals.as<uint32_t>() + 4;
    if (units && p.dist_slots && units <= dist_export_one_max()) {
        // verdict, flags, scan, rows and header in one workgroup
        launch_dist_export_one(D, p.totals.as<uint32_t>(), p.flags.as<uint32_t>(), p.dist_pc, p.dverd.as<uint32_t>(),
                               p.alive_l.as<uint8_t>(), units, p.dist_d_n, p.dist_flag.as<uint32_t>(),
                               p.dist_pos.as<uint32_t>(), d_count, p.s_rows->as<double>(), p.s_key->as<uint64_t>(),
                               p.s_src->as<uint32_t>(), p.dup_cnt.as<uint32_t>(), p.pr_entries.as<int32_t>(), d_block,
                               (uint32_t)cap, p.n, st);
        HIP_TRY(hipGetLastError());
        return SKY_OK;
    }
    if (p.dist_verdict_pending)
        launch_plan_verdict(p.totals.as<uint32_t>(), p.flags.as<uint32_t>(), p.dist_pc, p.dverd.as<uint32_t>(), st);
    if (units) {
        launch_dist_flags(p.alive_l.as<uint8_t>(), units, p.dist_d_n, p.dist_flag.as<uint32_t>(), st);
        scan_excl_u32(p.dist_flag.as<uint32_t>(), p.dist_pos.as<uint32_t>(), units, d_count, p.scratch.as<uint32_t>(),
                      st);
        if (p.dist_slots) {
            launch_dist_rows(D, true, p.s_rows->p, p.s_key->as<uint64_t>(), p.dist_flag.as<uint32_t>(),
                             p.dist_pos.as<uint32_t>(), units, p.s_src->as<uint32_t>(), p.dup_cnt.as<uint32_t>(),
                             p.pr_entries.as<int32_t>(), nullptr, d_block, (uint32_t)cap, st);
        } else {
            // representatives: multiplicity = tuples of every slot collapsed into the rep
            SKY_TRY(p.mult.ensure((size_t)units * 8));
            SKY_TRY(p.perm.ensure((size_t)std::max<uint32_t>(p.mt, 1) * 4));
            HIP_TRY(hipMemsetAsync(p.mult.p, 0, (size_t)units * 8, st));
            launch_iota(p.perm.as<uint32_t>(), p.mt, st);
            launch_rep_mult(p.mt, p.perm.as<uint32_t>(), p.s_src->as<uint32_t>(), p.slot_rep.as<uint32_t>(), nullptr,
                            p.dup_cnt.as<uint32_t>(), p.pr_entries.as<int32_t>(), p.mult.as<unsigned long long>(), st);
            launch_dist_rows(D, p.f64, p.rep_rows.p, p.rep_key.as<uint64_t>(), p.dist_flag.as<uint32_t>(),
                             p.dist_pos.as<uint32_t>(), units, nullptr, nullptr, nullptr,
                             p.mult.as<unsigned long long>(), d_block, (uint32_t)cap, st);
        }
    } else {
        HIP_TRY(hipMemsetAsync(d_count, 0, 4, st));
    }
    launch_dist_header(d_count, p.dverd.as<uint32_t>(), p.n, D, d_block, st);
    HIP_TRY(hipGetLastError());
    return SKY_OK;
}

// a NaN found on the synchronised route: the block carries the verdict (every rank returns
// SKY_E_NAN from sky_dist_finish; the collectives in between still run everywhere)
int dist_nan_block(sky_ctx *c, int64_t *d_block) {
    Pipe &p = c->main;
    SKY_TRY(p.dverd.ensure(128));
    FillSet f;
    f.add(p.dverd.p, 4, 0);
    f.add(p.totals.as<uint32_t>() + 4, 4, 0);
    HIP_TRY(f.launch(c->st));
    launch_plan_verdict(p.totals.as<uint32_t>(), p.flags.as<uint32_t>(), PlanCheck{}, p.dverd.as<uint32_t>(), c->st);
    launch_dist_header(p.totals.as<uint32_t>() + 4, p.dverd.as<uint32_t>(), p.n, c->D, d_block, c->st);
    HIP_TRY(hipGetLastError());
    return SKY_OK;
}

// own vectors against a large union: the bounding-box pass (k_mbr.hip) over the compacted union
// as x tiles and this rank's own rows as y tiles.  Reads the union's size and row type back
// first (the large-union route's one extra host synchronisation).
int dist_union_mbr(sky_ctx *c, const int64_t *d_blocks, int world, int rank, int64_t cap, int K,
                   unsigned long long *lsz, unsigned long long *surv, uint64_t *own_out, uint64_t *union_out) {
    Pipe &p = c->aux;      // the union's workspace; main keeps the shard
    hipStream_t st = c->st;
    const int D = c->D;
    unsigned long long *sum = c->dist_sum.as<unsigned long long>();
    const uint64_t tot_bound = (uint64_t)world * (uint64_t)cap;
    const int DP = padded_dims<double>(D);
    SKY_TRY(c->dist_union.ensure((size_t)std::max<uint64_t>(tot_bound, 1) * DP * 8));
    SKY_TRY(c->dist_ukey.ensure((size_t)std::max<uint64_t>(tot_bound, 1) * 8));
    SKY_TRY(c->dist_umult.ensure((size_t)std::max<uint64_t>(tot_bound, 1) * 8));
    launch_dist_compact(D, d_blocks, world, (uint32_t)cap, sum, c->dist_union.as<double>(),
                        c->dist_ukey.as<uint64_t>(), c->dist_umult.as<int64_t>(), st);
    unsigned long long h[16] = {};
    SKY_TRY(sync_read(p, st, {{sum, 128}}, {h}));
    const uint32_t n_union = (uint32_t)h[3], n_own = (uint32_t)h[4], own_off = (uint32_t)h[6];
    *own_out = h[8];
    *union_out = h[7];
    if (!n_own || h[0] > (unsigned long long)cap) return SKY_OK;   // overflow: sky_dist_finish re-runs
    if ((uint64_t)n_own * n_union <= dist_brute_pairs()) {
        SKY_TRY(dist_dom_ready(c->main, cap, st));
        launch_dist_union_fate(D, d_blocks, world, rank, (uint32_t)cap, K, c->main.dist_own.as<uint8_t>(),
                               c->main.dist_dom.as<uint32_t>(), lsz, surv, sum, ~0ull, nullptr, st);
        return SKY_OK;
    }
    const uint32_t fl = (uint32_t)h[5];
    const int fmt = (fl & kFlagNotF32) ? 2 : ((fl & kFlagNotU16) ? 1 : 0);
    const int NW = mbr_row_words(D, fmt);
    const void *rows = c->dist_union.p;
    if (fmt != 2) {
        SKY_TRY(p.r16.ensure((size_t)n_union * NW * 4));
        launch_dist_pack(D, c->dist_union.as<double>(), n_union, fmt, p.r16.as<uint32_t>(), st);
        rows = p.r16.p;
    }
    const size_t xt = mbr_tiles(n_union), yt = mbr_tiles(n_own);
    SKY_TRY(p.mbr_mm.ensure((size_t)D * 16));
    SKY_TRY(p.mbr_code.ensure((size_t)(n_union + n_own) * 8));
    SKY_TRY(p.mbr_code2.ensure((size_t)(n_union + n_own) * 8));
    SKY_TRY(p.mbr_idx.ensure((size_t)(n_union + n_own) * 4));
    SKY_TRY(p.mbr_idx2.ensure((size_t)(n_union + n_own) * 4));
    SKY_TRY(p.mbr_rows.ensure((xt + yt) * 64 * NW * 4));
    SKY_TRY(p.mbr_part.ensure((size_t)(n_union + n_own) * 4));
    SKY_TRY(p.mbr_min.ensure((xt + yt) * NW * 4));
    SKY_TRY(p.mbr_max.ensure((xt + yt) * NW * 4));
    SKY_TRY(p.mbr_pr.ensure((xt + yt) * 4));
    SKY_TRY(p.mbr_sub.ensure((xt + yt) * kMbrSubMax * NW * 4));
    SKY_TRY(p.mbr_gmin.ensure(mbr_group_slots(n_union) * NW * 4));
    SKY_TRY(p.mbr_gpr.ensure(mbr_group_slots(n_union) * 4));
    SKY_TRY(p.mbr_domf.ensure((size_t)n_own * 4));
    SKY_TRY(p.mbr_pairs.ensure(128));
    SKY_TRY(p.mbr_lpt.ensure(mbr_lpt_words(yt) * 4));
    // one radix scratch for both sorts (they run one after the other on the stream)
    SKY_TRY(p.scratch.ensure(radix_scratch_words(std::max(n_union, n_own)) * 4 + 64));
    FillSet fill;
    fill.add(p.mbr_mm.p, (size_t)D * 4, 0xff);
    fill.add(p.mbr_mm.as<uint32_t>() + D, (size_t)D * 4, 0);
    fill.add(p.mbr_mm.as<uint32_t>() + 2 * D, (size_t)D * 4, 0xff);
    fill.add(p.mbr_mm.as<uint32_t>() + 3 * D, (size_t)D * 4, 0);
    fill.add(p.mbr_pairs.p, 128, 0);
    fill.add(p.mbr_lpt.p, kMbrLptHead * 4, 0);
    fill.add(p.mbr_domf.p, (size_t)n_own * 4, 0);
    HIP_TRY(fill.launch(st));
    MbrUnionArgs a;
    auto set = [&](MbrArgs &s, const void *r, const uint64_t *key, uint32_t m, size_t t0, size_t rowoff, int mmoff,
                   uint32_t *scr) {
        s.D = D;
        s.fmt = fmt;
        s.rows = r;
        s.rep_key = key;
        s.mr = m;
        s.full = true;
        s.gmerge = true;
        s.mm = p.mbr_mm.as<uint32_t>() + mmoff;
        s.code = p.mbr_code.as<uint64_t>() + rowoff;
        s.code_alt = p.mbr_code2.as<uint64_t>() + rowoff;
        s.idx = p.mbr_idx.as<uint32_t>() + rowoff;
        s.idx_alt = p.mbr_idx2.as<uint32_t>() + rowoff;
        s.radix_scratch = scr;
        s.err = c->main.flags.as<uint32_t>();   // a look-back's spin bound: checked by sky_dist_finish
        s.trows = p.mbr_rows.as<uint32_t>() + t0 * 64 * NW;
        s.tpart = p.mbr_part.as<uint32_t>() + rowoff;
        s.tmin = p.mbr_min.as<uint32_t>() + t0 * NW;
        s.tmax = p.mbr_max.as<uint32_t>() + t0 * NW;
        s.tprange = p.mbr_pr.as<uint32_t>() + t0;
        s.tsub = p.mbr_sub.as<uint32_t>() + t0 * kMbrSubMax * NW;
        s.pairs = p.mbr_pairs.as<unsigned long long>();
    };
    const size_t rb = (size_t)NW * 4;
    set(a.x, rows, c->dist_ukey.as<uint64_t>(), n_union, 0, 0, 0, p.scratch.as<uint32_t>());
    a.x.gmin = p.mbr_gmin.as<uint32_t>();
    a.x.gprange = p.mbr_gpr.as<uint32_t>();
    set(a.y, (const char *)rows + (size_t)own_off * rb, c->dist_ukey.as<uint64_t>() + own_off, n_own, xt, n_union,
        2 * D, p.scratch.as<uint32_t>());
    a.y.domf = p.mbr_domf.as<uint32_t>();
    a.y.lpt = p.mbr_lpt.as<uint32_t>();
    a.ymult = c->dist_umult.as<int64_t>() + own_off;
    a.K = K;
    a.flags = c->main.dist_own.as<uint8_t>();
    a.lsz = lsz;
    a.surv = surv;
#ifdef SKY_MEASURE
    {
        const char *e = SKY_MEASURE_ENV("SKY_MBR_DBG");
        a.x.dbg = e ? atoi(e) : 0;
    }
#endif
    c->ktimer_begin("union_fate", st);
    HIP_TRY(launch_mbr_union(a, st));
    c->ktimer_end("union_fate", st, (int64_t)n_own * n_union);
#ifdef SKY_MEASURE
    if (a.x.dbg & 4) {        // the scan's funnel (measurement builds): as engine.hip prints it for a query
        unsigned long long f[5] = {};
        HIP_TRY(hipMemcpyAsync(f, p.mbr_pairs.p, 40, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        fprintf(stderr, "[mbr-union] own %u union %u groups %llu box %llu pre %llu tested %llu pairs %llu\n", n_own,
                n_union, f[2], f[3], f[4], f[1], f[0]);
    }
#endif
    return SKY_OK;
}

}  // namespace

extern "C" {

int sky_dist_export_dev(sky_ctx *c, const int64_t *d_ids, const double *d_values, int64_t n, int64_t *d_block,
                        int64_t cap) {
    GUARD_BEGIN
    ARG_CHECK(c && d_block && (n == 0 || d_values), "null argument");
    ARG_CHECK(n >= 0 && n < (int64_t)0x7fffffffLL, "n out of range");
    ARG_CHECK(cap >= 0 && cap < (int64_t)0x7fffffffLL, "cap out of range");
    SKY_TRY(bind(c));
    c->shard_valid = false;
    c->dist_state = 0;
    if (c->profile >= 2) {
        if (!c->pt.ok) c->pt.init();
        c->pt.reset();
    }
    PipeIn in;
    in.vals = d_values;
    in.n = (uint32_t)n;
    in.ids = d_ids;
    in.global = false;
    in.fate = false;
    in.dist = true;
    in.K = c->Kq();
    Pipe &p = c->main;
    SKY_TRY(p.dverd.ensure(128));
    if (n == 0) {                       // an empty shard still takes part in the collectives
        SKY_TRY(pipe_run(*c, p, in, nullptr));
        p.dist_n = 0;
        p.dist_d_n = nullptr;
        p.dist_slots = false;
        p.dist_verdict_pending = false;
        HIP_TRY(hipMemsetAsync(p.dverd.p, 0, 4, c->st));
    } else {
        const int r = pipe_run(*c, p, in, c->profile >= 2 ? &c->pt : nullptr);
        if (r == SKY_E_NAN) {
            SKY_TRY(dist_nan_block(c, d_block));
            c->dist_state = 2;
            c->dist_cap = cap;
            return SKY_OK;
        }
        SKY_TRY(r);
    }
    c->shard = in;
    c->shard_valid = true;
    SKY_TRY(dist_write_block(c, d_block, cap));
    c->dist_state = 1;
    c->dist_cap = cap;
    return SKY_OK;
    GUARD_END
}

int sky_dist_reblock_dev(sky_ctx *c, int64_t *d_block, int64_t cap) {
    GUARD_BEGIN
    ARG_CHECK(c && d_block, "null argument");
    ARG_CHECK(c->dist_state != 0, "call sky_dist_export_dev first");
    ARG_CHECK(cap >= 0 && cap < (int64_t)0x7fffffffLL, "cap out of range");
    SKY_TRY(bind(c));
    if (c->dist_state == 2) SKY_TRY(dist_nan_block(c, d_block));
    else SKY_TRY(dist_write_block(c, d_block, cap));
    if (c->dist_state == 3) c->dist_state = 1;
    c->dist_cap = cap;
    return SKY_OK;
    GUARD_END
}

int sky_dist_merge_dev(sky_ctx *c, const int64_t *d_blocks, int32_t world, int32_t rank, int64_t cap,
                       int64_t *d_ids_out, int32_t *d_origin_out, int64_t out_cap, int64_t *d_stats) {
    GUARD_BEGIN
    ARG_CHECK(c && d_blocks && d_stats, "null argument");
    ARG_CHECK(c->dist_state != 0, "call sky_dist_export_dev first");
    ARG_CHECK(world >= 1 && world <= 4096 && rank >= 0 && rank < world, "bad world / rank");
    ARG_CHECK(cap == c->dist_cap, "cap differs from the one this rank's block was written with");
    ARG_CHECK(out_cap >= 0, "out_cap out of range");
    SKY_TRY(bind(c));
    hipStream_t st = c->st;
    Pipe &p = c->main;
    const int D = c->D;
    const int K = c->Kq();
    SKY_TRY(c->dist_sum.ensure((size_t)(16 + world) * 8));   // [0..15] summary, [16..] offsets
    SKY_TRY(p.statk.ensure((size_t)SKY_DIST_STATS_WORDS(K) * 8));
    SKY_TRY(p.dist_own.ensure((size_t)std::max<int64_t>(cap, 1)));
    unsigned long long *sum = c->dist_sum.as<unsigned long long>();
    unsigned long long *lsz = p.statk.as<unsigned long long>(), *surv = lsz + K;
    unsigned long long *w_miss = lsz + 2 * K, *w_err = lsz + 2 * K + 1;   // summed over the ranks
    const uint32_t tiles = (p.n + kTile - 1) / kTile;
    FillSet fill;
    fill.add(p.statk.p, (size_t)SKY_DIST_STATS_WORDS(K) * 8);
    fill.add(c->dist_sum.p, 128);
    if (p.hist_count && c->dist_state == 1 && tiles) fill.add(p.tile_cand.p, (size_t)tiles * 4);
    HIP_TRY(fill.launch(st));
    const uint64_t bp0 = dist_brute_pairs();
    const bool brute_route = c->dist_state == 1 && p.n && c->dist_hist_pairs >= 0 &&
                             (uint64_t)c->dist_hist_pairs <= bp0;
    // the pair-kernel route computes the summary words itself (one launch less)
    if (!(brute_route && dist_summary_fused(world))) launch_dist_summary(d_blocks, world, rank, (uint32_t)cap, D, sum, st);
    if (c->dist_state == 2 || p.n == 0)        // NaN (finish reports it) or an empty shard: no fates
        HIP_TRY(hipMemsetAsync(p.totals.as<uint32_t>() + 3, 0, 4, st));
    if (c->dist_state == 1 && p.n) {
        // ---- own vectors against the union: one pair kernel over the blocks while the last
        //      step's |own| x |union| was small, else (and on the first step) the sized route
        //      (the capacity only grows: if cap x world x cap could exceed the route's bound, the
        //      kernel checks this step's sizes on the device and, when they are too large, writes
        //      no fate and raises the route-miss word: every rank returns SKY_E_RETRY, this one
        //      then takes the sized route)
        const uint64_t bp = bp0;
        const bool brute = brute_route;
        if (brute) {
            const unsigned __int128 worst = (unsigned __int128)(uint64_t)cap * (uint64_t)cap * (uint64_t)world;
            const unsigned long long limit = worst <= bp ? ~0ull : (unsigned long long)bp;
            c->ktimer_begin("union_fate", st);
            SKY_TRY(dist_dom_ready(p, cap, st));
            launch_dist_union_fate(D, d_blocks, world, rank, (uint32_t)cap, K, p.dist_own.as<uint8_t>(),
                                   p.dist_dom.as<uint32_t>(), lsz, surv, sum, limit, w_miss, st);
            c->ktimer_end("union_fate", st, 0);
            c->dist_last_route = 0;
        } else {
            uint64_t no = 0, nu = 0;
            SKY_TRY(dist_union_mbr(c, d_blocks, world, rank, cap, K, lsz, surv, &no, &nu));
            c->dist_last_route = (no * nu <= dist_brute_pairs()) ? 0 : 1;
        }
        HIP_TRY(hipGetLastError());
        // ---- the shard's units: global level from the own-vector fates
        const uint32_t units = p.dist_n;
        launch_dist_alive_g(p.dist_flag.as<uint32_t>(), p.dist_pos.as<uint32_t>(), units, p.dist_own.as<uint8_t>(),
                            (uint32_t)cap, p.alive_g.as<uint8_t>(), st);
        // ---- per-tuple fates, output counts, stream-ordered output
        const int KM = p.Kp * p.M;
        FateArgs fta{};
        fta.mt = p.mt;
        fta.d_mt = p.dist_slots ? p.dist_d_n : nullptr;
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
        fta.lsz = nullptr;
        fta.surv = nullptr;
        fta.tile_cand = p.hist_count ? p.tile_cand.as<uint32_t>() : nullptr;
        launch_fate_tables(fta, st);
        SKY_TRY(p.out_cnt.ensure((size_t)std::max<uint32_t>(tiles, 1) * 4));
        SKY_TRY(p.out_off.ensure((size_t)std::max<uint32_t>(tiles, 1) * 4));
        SKY_TRY(p.scratch.ensure(scan_scratch_words(tiles + 1) * 4 + 64));
        OutArgs oa{};
        oa.status = p.status.as<uint16_t>();
        oa.n = p.n;
        oa.pruner_fate = p.pruner_fate.as<uint8_t>();
        oa.M = p.M;
        oa.KM = KM;
        oa.K = p.K;
        oa.out_cnt = p.out_cnt.as<uint32_t>();
        c->ktimer_begin("out", st);
        if (p.hist_count) {                   // counts + scan in one launch
            SKY_TRY(out_hist_scan_words(p, tiles, st));
            launch_out_hist_scan(p.tile_hist.as<uint32_t>(), p.tile_cand.as<uint32_t>(), p.pruner_fate.as<uint8_t>(), KM,
                                 tiles, p.out_cnt.as<uint32_t>(), p.out_off.as<uint32_t>(), p.totals.as<uint32_t>() + 3,
                                 p.out_lb.as<unsigned long long>(), ++p.out_epoch, p.flags.as<uint32_t>(), st);
        } else {
            launch_out_count(oa, st);
            scan_excl_u32(p.out_cnt.as<uint32_t>(), p.out_off.as<uint32_t>(), tiles, p.totals.as<uint32_t>() + 3,
                          p.scratch.as<uint32_t>(), st);
        }
        if (d_ids_out || d_origin_out) {
            OutArgs ow = oa;
            ow.out_off = p.out_off.as<uint32_t>();
            ow.ids = c->shard.ids;
            ow.ids_out = d_ids_out;
            ow.origin_out = d_origin_out;
            ow.out_cap = out_cap;
            ow.planes = p.planes_on ? p.planes.as<uint64_t>() : nullptr;
            ow.dom_kj = p.dom_kj;
            launch_out_write(ow, st);
        }
        c->ktimer_end("out", st, p.n);
    }
    // merge-time errors (the union pass's look-backs) into the summed words, then this rank's
    // shares for the caller's all-reduce
    launch_dist_merge_err(p.flags.as<uint32_t>(), lsz, (int)(w_err - lsz), (int)SKY_DIST_STATS_WORDS(K), d_stats, st);
    HIP_TRY(hipGetLastError());
    c->dist_world = world;
    c->dist_merged = true;
    return SKY_OK;
    GUARD_END
}

int sky_dist_finish(sky_ctx *c, const int64_t *d_stats_sum, int64_t out_cap, int64_t *n_out, int64_t *need_cap) {
    GUARD_BEGIN
    ARG_CHECK(c && d_stats_sum, "null argument");
    ARG_CHECK(c->dist_state != 0 && c->dist_merged, "call sky_dist_merge_dev first");
    SKY_TRY(bind(c));
    Pipe &p = c->main;
    const int K = c->Kq();
    if (n_out) *n_out = 0;
    if (need_cap) *need_cap = 0;
    unsigned long long sum[16] = {};
    uint32_t tot[16] = {}, flags = 0;
    std::vector<int64_t> st((size_t)SKY_DIST_STATS_WORDS(K));
    const int KM = p.Kp * p.M;
    p.h_dup.assign(KM, 0u);
    SKY_TRY(sync_read(p, c->st,
                      {{c->dist_sum.p, 128}, {p.totals.p, 64}, {p.flags.p, 4}, {d_stats_sum, (size_t)SKY_DIST_STATS_WORDS(K) * 8},
                       {p.dup_cnt.p, p.n ? (size_t)KM * 4 : 0}},
                      {sum, tot, &flags, st.data(), p.h_dup.data()}));
    if (p.n) pick_dom_group(p, KM);
    c->dist_merged = false;
    // the next merge's route: |own| x |union| as exported (a capped exchange holds fewer rows)
    c->dist_hist_pairs = (int64_t)(sum[8] * sum[7]);
    const uint32_t own = (uint32_t)sum[2], any = (uint32_t)sum[1];
    // this rank's route: what the planned run found (the synchronised route set these already)
    if (p.last_planned && !(own & kDistReplan)) {
        p.m = tot[0];
        p.nps = tot[5];
        p.mt_pre = tot[10];
        p.mt = p.dist_pc.rounds ? tot[10 + p.dist_pc.rounds] : tot[10];
        p.mr = p.mt;
        p.f64 = (flags & kFlagNotF32) != 0;
        p.ints = !p.f64 && (flags & kFlagNotU16) == 0;
        p.ties = (flags & kFlagScoreTies) != 0;
    }
    if (own & kDistReplan) {                  // the next export runs the synchronised route
        p.plan.valid = false;
        p.plan_misses++;
        p.last_plan_miss = true;
        const size_t KM = (size_t)p.Kp * p.M;
        if ((size_t)tot[0] + tot[5] > p.dist_pc.cap)
            p.slot_hint = std::min<size_t>((size_t)p.n + KM, ((size_t)tot[0] + tot[5]) * 5 / 4 + KM);
    }
    // every code below comes from data identical on every rank (the gathered headers, the
    // all-reduced words), so every rank returns the same one
    const int64_t route_miss = st[2 * K], merge_err = st[2 * K + 1];
    if ((any & kDistError) || merge_err > 0) {
        set_error("a look-back exceeded its spin bound, or the bounding-box pass's work queue overflowed, on some rank");
        return SKY_E_HIP;
    }
    if (any & kDistNaN) {
        set_error("a tuple value is NaN (on some rank): the reference BNL result is order-dependent for NaN; rejected");
        return SKY_E_NAN;
    }
    if (any & kDistReplan) {
        set_error("a rank's planned local phase missed its assumptions: run the step again");
        return SKY_E_RETRY;
    }
    if (route_miss > 0 && (int64_t)sum[0] <= c->dist_cap) {
        set_error("a rank's union was too large for the pair-kernel route it took from the last step: run the step "
                  "again");
        return SKY_E_RETRY;
    }
    if ((int64_t)sum[0] > c->dist_cap) {
        if (need_cap) *need_cap = (int64_t)sum[0];
        set_error("exchange capacity " + std::to_string(c->dist_cap) + " < exported vectors " + std::to_string(sum[0]));
        return SKY_E_CAPACITY;
    }
    const int64_t g = p.n ? tot[3] : 0;
    if (n_out) *n_out = g;
    c->K_last = K;
    c->lsz.assign(st.begin(), st.begin() + K);
    c->surv.assign(st.begin() + K, st.begin() + 2 * K);
    c->counters[0] = p.n;
    c->counters[1] = p.m;
    c->counters[2] = p.mr;
    c->counters[3] = (int64_t)sum[4];       // own exported vectors
    c->counters[4] = g;
    c->counters[5] = (int64_t)sum[3];       // union vectors
    c->counters[6] = c->dist_last_route;
    c->counters[7] = (p.f64 ? 1 : 0) | (p.ties ? 2 : 0) | (p.u16 ? 4 : 0) | (p.last_planned ? 8 : 0) |
                     (p.last_plan_miss ? 16 : 0) | (p.last_tiny ? 32 : 0);
    if (g > out_cap) {
        set_error("output capacity " + std::to_string(out_cap) + " < this rank's skyline share " + std::to_string(g));
        return SKY_E_CAPACITY;
    }
    c->dist_state = 3;
    finish_profile(c);
    return SKY_OK;
    GUARD_END
}

int sky_profile_host_syncs(sky_ctx *c, int64_t *n_out) {
    ARG_CHECK(c && n_out, "null argument");
    *n_out = c->host_syncs + c->main.host_syncs + c->aux.host_syncs;
    return SKY_OK;
}

}  // extern "C"
