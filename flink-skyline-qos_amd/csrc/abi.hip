// abi.hip — extern "C" entry points of libskyline_hip.so (include/skyline_hip.h).
// Status codes only; no exception crosses the boundary.
#include "abi_common.h"
#include "knobs.h"

#include <cstring>
#include <new>
#include <string>

namespace sky {
static thread_local std::string g_err;
void set_error(const std::string &m) { g_err = m; }
}  // namespace sky

using namespace sky;


extern "C" {

const char *sky_last_error(void) { return g_err.c_str(); }
const char *sky_version(void) { return "skyline_hip 0.1 (gfx950)"; }

// devices this process sees (0 without a GPU: no error), for the operators' subtask -> device map
int sky_device_count(int32_t *n_out) {
    ARG_CHECK(n_out != nullptr, "null argument");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) {
        (void)hipGetLastError();
        count = 0;
    }
    *n_out = count;
    return SKY_OK;
}

// the device of a subtask: subtasks round-robin over the node's GPUs (a TaskManager per node
// runs subtasks 0..parallelism-1 of an operator; each keeps its context on one GPU)
int sky_device_for_subtask(int32_t subtask, int32_t ndev, int32_t *dev_out) {
    ARG_CHECK(dev_out != nullptr, "null argument");
    ARG_CHECK(subtask >= 0 && ndev >= 1, "subtask must be >= 0 and ndev >= 1");
    *dev_out = subtask % ndev;
    return SKY_OK;
}

int sky_ctx_create(const int *devices, int ndev, int dims, int num_partitions, int algo, double domain_max,
                   sky_ctx **out) {
    GUARD_BEGIN
    ARG_CHECK(out != nullptr, "out is null");
    *out = nullptr;
    ARG_CHECK(dims >= 1 && dims <= SKY_MAX_DIMS, "dims must be in [1,16]");
    ARG_CHECK(num_partitions >= 1 && num_partitions <= SKY_MAX_PARTITIONS, "num_partitions must be in [1,256]");
    ARG_CHECK(algo >= SKY_ALGO_DIM && algo <= SKY_ALGO_ANGLE, "algo must be 0 (dim), 1 (grid) or 2 (angle)");
    ARG_CHECK(ndev >= 0 && ndev <= 1, "one device per context (run one process per GPU)");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        (void)hipGetLastError();
        set_error("no HIP device visible");
        return SKY_E_NOLIB;
    }
    const int dev = (ndev == 1 && devices) ? devices[0] : 0;
    ARG_CHECK(dev >= 0 && dev < count, "device ordinal out of range");
    sky_ctx *c = new sky_ctx();
    c->dev = dev;
    c->D = dims;
    c->P = num_partitions;
    c->algo = algo;
    c->domain = domain_max;
    if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        delete c;
        set_error("could not bind the HIP device / create a stream");
        return SKY_E_HIP;
    }
    c->st = c->own;
    *out = c;
    return SKY_OK;
    GUARD_END
}

int sky_ctx_destroy(sky_ctx *c) {
    if (!c) return SKY_OK;
    hipSetDevice(c->dev);
    hipStreamSynchronize(c->st);
    c->ktimer_collect();
    for (hipEvent_t e : c->event_pool) hipEventDestroy(e);
    if (c->pt.ok) c->pt.destroy();
    if (c->own) hipStreamDestroy(c->own);
    delete c;
    return SKY_OK;
}

int sky_ctx_set_semantics(sky_ctx *c, int sem) {
    ARG_CHECK(c, "ctx is null");
    ARG_CHECK(sem == SKY_SEM_REFERENCE || sem == SKY_SEM_COMPLETE, "semantics must be 0 or 1");
    ARG_CHECK(!(sem == SKY_SEM_COMPLETE && c->algo == SKY_ALGO_GRID && c->D > 8),
              "complete MR-Grid semantics needs 2^dims <= 256 keys");
    c->sem = sem;
    return SKY_OK;
}

int sky_ctx_set_stream(sky_ctx *c, void *s) {
    ARG_CHECK(c, "ctx is null");
    c->st = s ? (hipStream_t)s : c->own;
    return SKY_OK;
}

int sky_ctx_set_grid_filter(sky_ctx *c, int on) {
    ARG_CHECK(c, "ctx is null");
    c->grid_filter = on ? 1 : 0;
    return SKY_OK;
}

int sky_ctx_wait_stream(sky_ctx *c, void *s) {
    ARG_CHECK(c, "ctx is null");
    SKY_TRY(bind(c));
    if ((hipStream_t)s == c->st) return SKY_OK;
    hipEvent_t e = c->take_event();
    HIP_TRY(hipEventRecord(e, (hipStream_t)s));
    HIP_TRY(hipStreamWaitEvent(c->st, e, 0));
    c->event_pool.push_back(e);   // re-recording later does not affect the enqueued wait
    return SKY_OK;
}
int sky_ctx_signal_stream(sky_ctx *c, void *s) {
    ARG_CHECK(c, "ctx is null");
    SKY_TRY(bind(c));
    if ((hipStream_t)s == c->st) return SKY_OK;
    hipEvent_t e = c->take_event();
    HIP_TRY(hipEventRecord(e, c->st));
    HIP_TRY(hipStreamWaitEvent((hipStream_t)s, e, 0));
    c->event_pool.push_back(e);
    return SKY_OK;
}

int sky_ctx_info(sky_ctx *c, int32_t *dims, int32_t *num_partitions, int32_t *algo) {
    ARG_CHECK(c, "ctx is null");
    if (dims) *dims = c->D;
    if (num_partitions) *num_partitions = c->P;
    if (algo) *algo = c->algo;
    return SKY_OK;
}
int sky_part_info(sky_part *p, int32_t *key, int32_t *dims) {
    ARG_CHECK(p && p->ctx, "part is null");
    if (key) *key = p->key;
    if (dims) *dims = p->ctx->D;
    return SKY_OK;
}
int sky_stream_info(sky_stream *s, int32_t *dims) {
    ARG_CHECK(s && s->ctx, "stream is null");
    if (dims) *dims = s->ctx->D;
    return SKY_OK;
}

int sky_ctx_sync(sky_ctx *c) {
    ARG_CHECK(c, "ctx is null");
    SKY_TRY(bind(c));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SKY_OK;
}

// One-time warm-up (off any timed path): a small device-generated query down each pipeline
// branch — the bounding-box pass (forced), the brute pass, the sort path — so that the first
// real query that takes a branch does not pay for its kernels' first launch (code-object
// loading) and first allocations inside its latency (C5: a 20-30 ms first-use spike).
int sky_ctx_warmup(sky_ctx *c) {
    GUARD_BEGIN
    ARG_CHECK(c, "ctx is null");
    SKY_TRY(bind(c));
    const int D = c->D;
    const int64_t n = 40000;
    DevBuf v, ids, oi, oo;
    SKY_TRY(v.ensure((size_t)n * D * 8));
    SKY_TRY(ids.ensure((size_t)n * 8));
    SKY_TRY(oi.ensure((size_t)n * 8));
    SKY_TRY(oo.ensure((size_t)n * 4));
    for (int pass = 0; pass < 3; pass++) {
        // std-anti: many distinct candidates (bounding-box pass, then the SFS sort path);
        // the reference formula: few candidates (brute pass)
        launch_synth(pass == 2 ? 2 : 3, D, 0, 1000, 99 + pass, 0, n, v.as<double>(), ids.as<int64_t>(), c->st);
        HIP_TRY(hipGetLastError());
        PipeIn in;
        in.vals = v.as<double>();
        in.ids = ids.as<int64_t>();
        in.n = (uint32_t)n;
        in.global = true;
        in.K = c->Kq();
        in.out_ids = oi.as<int64_t>();
        in.out_org = oo.as<int32_t>();
        in.out_cap = n;
        c->shard_valid = false;
        c->warm_mode = pass == 0 ? 1 : (pass == 1 ? 2 : 0);   // 1: force the box pass, 2: force SFS
        const int rc = pipe_run(*c, c->main, in, nullptr);
        c->warm_mode = 0;
        if (rc != SKY_OK) return rc;
        int64_t g = 0;
        SKY_TRY(pipe_output(*c, c->main, in, false, in.out_ids, in.out_org, nullptr, n, &g, nullptr));
    }
    HIP_TRY(hipStreamSynchronize(c->st));
    return SKY_OK;
    GUARD_END
}

int sky_partition_keys_dev(sky_ctx *c, const double *d_values, int64_t n, int32_t *d_keys_out) {
    GUARD_BEGIN
    ARG_CHECK(c && (n == 0 || (d_values && d_keys_out)), "null argument");
    ARG_CHECK(n >= 0 && n < (int64_t)0xffffffffLL, "n out of range");
    SKY_TRY(bind(c));
    launch_keys(c->D, d_values, (uint32_t)n, c->kp(), d_keys_out, c->st);
    HIP_TRY(hipGetLastError());
    return SKY_OK;
    GUARD_END
}

int sky_partition_keys(sky_ctx *c, const double *values, int64_t n, int32_t *keys_out) {
    GUARD_BEGIN
    ARG_CHECK(c && (n == 0 || (values && keys_out)), "null argument");
    ARG_CHECK(n >= 0 && n < (int64_t)0xffffffffLL, "n out of range");
    if (n == 0) return SKY_OK;
    SKY_TRY(bind(c));
    SKY_TRY(c->h_vals.ensure((size_t)n * c->D * 8));
    SKY_TRY(c->h_keys.ensure((size_t)n * 4));
    HIP_TRY(hipMemcpyAsync(c->h_vals.p, values, (size_t)n * c->D * 8, hipMemcpyHostToDevice, c->st));
    launch_keys(c->D, c->h_vals.as<double>(), (uint32_t)n, c->kp(), c->h_keys.as<int32_t>(), c->st);
    HIP_TRY(hipMemcpyAsync(keys_out, c->h_keys.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SKY_OK;
    GUARD_END
}

// ---- fused query -------------------------------------------------------------
int sky_query_dev(sky_ctx *c, const int64_t *d_ids, const double *d_values, int64_t n, int64_t *d_ids_out,
                  int32_t *d_origin_out, int64_t cap, int64_t *n_out) {
    GUARD_BEGIN
    ARG_CHECK(c && (n == 0 || d_values), "null argument");
    ARG_CHECK(n >= 0 && n < (int64_t)0x7fffffffLL, "n out of range");
    SKY_TRY(bind(c));
    if (c->profile >= 2) {
        if (!c->pt.ok) c->pt.init();
        c->pt.reset();
    }
    PipeIn in;
    in.vals = d_values;
    in.n = (uint32_t)n;
    in.ids = d_ids;
    in.global = true;
    in.K = c->Kq();
    in.out_ids = d_ids_out;
    in.out_org = d_origin_out;
    in.out_cap = cap;
    in.planes_ok = true;            // the run's own write pass makes the output
    c->shard_valid = false;
    int r = pipe_run(*c, c->main, in, c->profile >= 2 ? &c->pt : nullptr);
    if (r == SKY_OK) {
        store_stats(c, c->main);
        r = pipe_output(*c, c->main, in, false, d_ids_out, d_origin_out, nullptr, cap, n_out, nullptr);
    }
    HIP_TRY(hipGetLastError());
    finish_profile(c);
    return r;
    GUARD_END
}

int sky_query(sky_ctx *c, const int64_t *ids, const double *values, int64_t n, int64_t *ids_out, int32_t *origin_out,
              int64_t cap, int64_t *n_out) {
    GUARD_BEGIN
    ARG_CHECK(c && (n == 0 || values), "null argument");
    ARG_CHECK(n >= 0 && n < (int64_t)0x7fffffffLL, "n out of range");
    SKY_TRY(bind(c));
    const size_t nn = (size_t)std::max<int64_t>(n, 1);
    SKY_TRY(c->h_vals.ensure(nn * c->D * 8));
    SKY_TRY(c->h_ids.ensure(nn * 8));
    if (n) HIP_TRY(hipMemcpyAsync(c->h_vals.p, values, (size_t)n * c->D * 8, hipMemcpyHostToDevice, c->st));
    if (n && ids) HIP_TRY(hipMemcpyAsync(c->h_ids.p, ids, (size_t)n * 8, hipMemcpyHostToDevice, c->st));
    PipeIn in;
    in.vals = c->h_vals.as<double>();
    in.n = (uint32_t)n;
    in.ids = ids ? c->h_ids.as<int64_t>() : nullptr;
    in.global = true;
    in.K = c->Kq();
    SKY_TRY(c->h_out_ids.ensure(nn * 8));
    SKY_TRY(c->h_out_org.ensure(nn * 4));
    in.out_ids = c->h_out_ids.as<int64_t>();
    in.out_org = c->h_out_org.as<int32_t>();
    in.out_cap = n;
    in.planes_ok = true;
    c->shard_valid = false;
    if (c->profile >= 2) {
        if (!c->pt.ok) c->pt.init();
        c->pt.reset();
    }
    SKY_TRY(pipe_run(*c, c->main, in, c->profile >= 2 ? &c->pt : nullptr));
    store_stats(c, c->main);
    const int64_t g = c->main.nout;
    if (n_out) *n_out = g;
    if (g > cap && (ids_out || origin_out)) {
        set_error("output capacity too small");
        return SKY_E_CAPACITY;
    }
    SKY_TRY(pipe_output(*c, c->main, in, false, c->h_out_ids.as<int64_t>(), c->h_out_org.as<int32_t>(), nullptr,
                        n, nullptr, nullptr));
    if (g && ids_out) HIP_TRY(hipMemcpyAsync(ids_out, c->h_out_ids.p, (size_t)g * 8, hipMemcpyDeviceToHost, c->st));
    if (g && origin_out)
        HIP_TRY(hipMemcpyAsync(origin_out, c->h_out_org.p, (size_t)g * 4, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    finish_profile(c);
    return SKY_OK;
    GUARD_END
}

int sky_global_stats_set(sky_ctx *c, int32_t k, const int64_t *local_sizes, const int64_t *survivors) {
    GUARD_BEGIN
    ARG_CHECK(c && k >= 0 && k <= 65536 && (k == 0 || (local_sizes && survivors)), "bad arguments");
    c->K_last = k;
    c->lsz.assign(local_sizes, local_sizes + k);
    c->surv.assign(survivors, survivors + k);
    return SKY_OK;
    GUARD_END
}

int sky_global_stats(sky_ctx *c, int64_t *local_sizes, int64_t *survivors, int32_t *k_out) {
    ARG_CHECK(c, "ctx is null");
    if (k_out) *k_out = c->K_last;
    for (int k = 0; k < c->K_last; k++) {
        if (local_sizes) local_sizes[k] = c->lsz[k];
        if (survivors) survivors[k] = c->surv[k];
    }
    return SKY_OK;
}

// ---- global merge of host lists -------------------------------------------------
int sky_global_merge(sky_ctx *c, int nparts, const int32_t *part_ids, const int64_t *const *ids,
                     const double *const *values, const int64_t *counts, int64_t *ids_out, int32_t *origin_out,
                     int64_t cap, int64_t *n_out) {
    GUARD_BEGIN
    ARG_CHECK(c && nparts >= 0 && nparts <= SKY_MAX_PARTITIONS, "bad nparts (<= 256 lists)");
    ARG_CHECK(nparts == 0 || (counts && values), "null argument");
    SKY_TRY(bind(c));
    int64_t n = 0;
    for (int k = 0; k < nparts; k++) {
        ARG_CHECK(counts[k] >= 0, "negative count");
        ARG_CHECK(counts[k] == 0 || values[k], "null values list");
        n += counts[k];
    }
    ARG_CHECK(n < (int64_t)0x7fffffffLL, "too many tuples");
    const size_t nn = (size_t)std::max<int64_t>(n, 1);
    SKY_TRY(c->h_vals.ensure(nn * c->D * 8));
    SKY_TRY(c->h_ids.ensure(nn * 8));
    SKY_TRY(c->h_origin.ensure(nn * 4));
    std::vector<int32_t> org((size_t)n);
    int64_t off = 0;
    for (int k = 0; k < nparts; k++) {
        if (counts[k] == 0) continue;
        HIP_TRY(hipMemcpyAsync(c->h_vals.as<double>() + off * c->D, values[k], (size_t)counts[k] * c->D * 8,
                               hipMemcpyHostToDevice, c->st));
        if (ids && ids[k]) {
            HIP_TRY(hipMemcpyAsync(c->h_ids.as<int64_t>() + off, ids[k], (size_t)counts[k] * 8, hipMemcpyHostToDevice,
                                   c->st));
        } else {
            std::vector<int64_t> seq((size_t)counts[k]);
            for (int64_t j = 0; j < counts[k]; j++) seq[j] = j;
            HIP_TRY(hipMemcpy(c->h_ids.as<int64_t>() + off, seq.data(), (size_t)counts[k] * 8, hipMemcpyHostToDevice));
        }
        for (int64_t j = 0; j < counts[k]; j++) org[off + j] = k;
        off += counts[k];
    }
    if (n) HIP_TRY(hipMemcpyAsync(c->h_origin.p, org.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->st));
    PipeIn in;
    in.vals = c->h_vals.as<double>();
    in.n = (uint32_t)n;
    in.ids = c->h_ids.as<int64_t>();
    in.origin = c->h_origin.as<int32_t>();
    in.single = true;
    in.global = false;
    in.K = std::max(nparts, 1);
    c->shard_valid = false;
    SKY_TRY(pipe_run(*c, c->main, in, nullptr));
    // GlobalSkylineAggregator: localSkylineSizes[k] = incoming list size (:544);
    // survivors by originPartition (:593-596)
    c->K_last = nparts;
    c->lsz.assign(nparts, 0);
    c->surv.assign(nparts, 0);
    for (int k = 0; k < nparts; k++) {
        c->lsz[k] = counts[k];
        c->surv[k] = (int64_t)c->main.h_lsz[k];
    }
    const int64_t g = c->main.nout;
    if (n_out) *n_out = g;
    if (g > cap && (ids_out || origin_out)) {
        set_error("output capacity too small");
        return SKY_E_CAPACITY;
    }
    SKY_TRY(c->h_out_ids.ensure((size_t)std::max<int64_t>(g, 1) * 8));
    SKY_TRY(c->h_out_org.ensure((size_t)std::max<int64_t>(g, 1) * 4));
    SKY_TRY(pipe_output(*c, c->main, in, false, c->h_out_ids.as<int64_t>(), c->h_out_org.as<int32_t>(), nullptr, g,
                        nullptr, nullptr));
    std::vector<int32_t> o((size_t)std::max<int64_t>(g, 1));
    if (g && ids_out) HIP_TRY(hipMemcpyAsync(ids_out, c->h_out_ids.p, (size_t)g * 8, hipMemcpyDeviceToHost, c->st));
    if (g) HIP_TRY(hipMemcpyAsync(o.data(), c->h_out_org.p, (size_t)g * 4, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    if (origin_out)
        for (int64_t j = 0; j < g; j++) origin_out[j] = part_ids ? part_ids[o[j]] : o[j];
    return SKY_OK;
    GUARD_END
}

// ---- utilities ------------------------------------------------------------------------
int sky_synth_dev(sky_ctx *c, int dist, int dmin, int dmax, uint64_t seed, int64_t id0, int64_t n, double *d_values,
                  int64_t *d_ids) {
    GUARD_BEGIN
    ARG_CHECK(c && (n == 0 || d_values), "null argument");
    ARG_CHECK(dist >= 0 && dist <= 4 && dmax >= dmin, "bad distribution arguments");
    SKY_TRY(bind(c));
    launch_synth(dist, c->D, dmin, dmax, seed, id0, n, d_values, d_ids, c->st);
    HIP_TRY(hipGetLastError());
    return SKY_OK;
    GUARD_END
}

int sky_synth(int dist, int dims, int dmin, int dmax, uint64_t seed, int64_t id0, int64_t n, double *values,
              int64_t *ids) {
    ARG_CHECK(dims >= 1 && dims <= SKY_MAX_DIMS && (n == 0 || values), "bad arguments");
    ARG_CHECK(dist >= 0 && dist <= 4 && dmax >= dmin, "bad distribution arguments");
    synth_host(dist, dims, dmin, dmax, seed, id0, n, values, ids);
    return SKY_OK;
}

int sky_dev_alloc(sky_ctx *c, int64_t bytes, void **d_out) {
    ARG_CHECK(c && d_out && bytes >= 0, "bad arguments");
    SKY_TRY(bind(c));
    HIP_TRY(hipMalloc(d_out, (size_t)std::max<int64_t>(bytes, 1)));
    return SKY_OK;
}
int sky_dev_free(sky_ctx *c, void *d) {
    ARG_CHECK(c, "ctx is null");
    SKY_TRY(bind(c));
    if (d) HIP_TRY(hipFree(d));
    return SKY_OK;
}
int sky_memcpy_h2d(sky_ctx *c, void *d_dst, const void *h_src, int64_t bytes) {
    ARG_CHECK(c && bytes >= 0, "bad arguments");
    SKY_TRY(bind(c));
    if (bytes) HIP_TRY(hipMemcpyAsync(d_dst, h_src, (size_t)bytes, hipMemcpyHostToDevice, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SKY_OK;
}
int sky_memcpy_d2h(sky_ctx *c, void *h_dst, const void *d_src, int64_t bytes) {
    ARG_CHECK(c && bytes >= 0, "bad arguments");
    SKY_TRY(bind(c));
    if (bytes) HIP_TRY(hipMemcpyAsync(h_dst, d_src, (size_t)bytes, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SKY_OK;
}

int sky_profile_enable(sky_ctx *c, int on) {
    ARG_CHECK(c, "ctx is null");
    c->profile = on < 0 ? 0 : (on > 2 ? 2 : on);
    return SKY_OK;
}
int sky_profile_phases(sky_ctx *c, double *ms_out, int64_t *counters_out) {
    ARG_CHECK(c, "ctx is null");
    for (int i = 0; i < SKY_PHASES; i++)
        if (ms_out) ms_out[i] = c->phase_ms[i];
    for (int i = 0; i < 8; i++)
        if (counters_out) counters_out[i] = c->counters[i];
    return SKY_OK;
}
int sky_profile_kernel(sky_ctx *c, const char *name, double *total_ms, int64_t *launches, int64_t *units) {
    ARG_CHECK(c && name, "null argument");
    c->ktimer_collect();
    auto it = c->kt.find(name);
    if (total_ms) *total_ms = it == c->kt.end() ? 0.0 : it->second.ms;
    if (launches) *launches = it == c->kt.end() ? 0 : it->second.launches;
    if (units) *units = it == c->kt.end() ? 0 : it->second.units;
    return SKY_OK;
}
int sky_profile_dominance(sky_ctx *c, int64_t *work_out) {
    ARG_CHECK(c && work_out, "null argument");
    *work_out = c->dom_w;
    return SKY_OK;
}
int sky_profile_reset(sky_ctx *c) {
    ARG_CHECK(c, "ctx is null");
    c->ktimer_collect();
    c->kt.clear();
    for (double &x : c->phase_ms) x = 0;
    return SKY_OK;
}

}  // extern "C"

// ---- bulk CSV ingest (k_csv.hip) ---------------------------------------------
namespace sky {
int csv_chunk_bytes(int64_t nbytes, int64_t nrec, int64_t nfields, int D, int *tail);
int64_t csv_count_blocks(int64_t nbytes);
int64_t csv_chunk_count(int64_t nbytes, int chunk);
void launch_csv_parse_chunks(const uint8_t *text, int64_t nbytes, int chunk, int tail, const uint32_t *blk_off,
                             const uint32_t *cnt1k, int D,
                             int64_t *ids, double *vals, uint8_t *status, unsigned long long *counts, uint32_t *spill,
                             longlong4 *spans, longlong3 *slow, unsigned long long *slow_n,
                             unsigned long long slow_cap, hipStream_t st);
}
// Parse route (knob read per call; every CSV test runs both).  Default: R records per parse
// workgroup, the group boundaries found from the count pass's prefixes (k_csv_group_pos, ~1 KB of
// text per group).  SKY_CSV_CHUNKS=1: byte chunks, each workgroup finds its records itself.  On the
// C4 text (100M records): decode 4.27 ms for groups (count 0.78 + group ends 0.25 + parse 3.04)
// against 4.77 ms for chunks (count 0.74 + parse 3.82) (profiles/r04_csv_parse_ab.txt).  Texts of
// very short records (chunks under 512 bytes) take the group route either way.
static bool csv_chunk_mode() {
    const char *e = SKY_ENV("SKY_CSV_CHUNKS");
    return e && e[0] == '1';
}
// ServiceTuple.fromString (ServiceTuple.java:89-104) + filter(nonNull) (FlinkSkyline.java:103)
// + Long.parseLong(id) (FlinkSkyline.java:276), over a whole device-resident buffer of records.
int sky_parse_csv_dev(sky_ctx *c, const char *d_text, int64_t nbytes, int64_t *d_ids_out, double *d_values_out,
                      int64_t cap, int64_t *n_out, int64_t *counts_out, uint8_t *d_status_out) {
    GUARD_BEGIN
    ARG_CHECK(c && n_out && (nbytes == 0 || d_text), "null argument");
    ARG_CHECK(nbytes >= 0 && nbytes < ((int64_t)1 << 40), "nbytes out of range");
    ARG_CHECK(cap >= 0, "cap out of range");
    SKY_TRY(bind(c));
    const uint8_t *text = reinterpret_cast<const uint8_t *>(d_text);
    const int64_t nb = csv_chunks(nbytes), nbc = csv_count_blocks(nbytes);   // 4 KB passes, 1 KB counts
    const int D = c->D;
    SKY_TRY(c->csv_blk.ensure((size_t)(nb + 1) * 8 + 32 + (size_t)nbc * 4));
    SKY_TRY(c->csv_scr.ensure(scan_scratch_words((size_t)std::max<int64_t>(nb, 1)) * 4));
    SKY_TRY(c->csv_counts.ensure(64 + 256 * 8));
    uint32_t *blk = c->csv_blk.as<uint32_t>(), *blk_off = blk + (nb + 1), *d_nl = blk_off + (nb + 1);
    uint32_t *cnt1k = reinterpret_cast<uint32_t *>(((uintptr_t)(d_nl + 4) + 15) & ~(uintptr_t)15);   // 16-byte stores
    uint32_t h_nl = 0;
    uint8_t last = '\n';
    unsigned long long *d_cnt = c->csv_counts.as<unsigned long long>();
    unsigned long long h_commas = 0;
    std::vector<unsigned long long> h_shards(256, 0);
    // exact-conversion queue (SKY_CSV_SLOW_CAP: tests force the re-parse-everything path)
    static const unsigned long long slow_cap = [] {
        const char *e = SKY_ENV("SKY_CSV_SLOW_CAP");
        return e ? (unsigned long long)std::max(1, atoi(e)) : (1ull << 20);
    }();
    SKY_TRY(c->csv_slow.ensure(slow_cap * sizeof(longlong3)));
    unsigned long long h_cnt[5] = {};
    int64_t nrec = 0;
    bool direct = false;
    int64_t *pid = d_ids_out;
    double *pval = d_values_out;
    if (nb) {
        HIP_TRY(hipMemsetAsync(d_cnt + 8, 0, 256 * 8, c->st));
        c->ktimer_begin("csv_count", c->st);
        launch_csv_nl_count(text, nbytes, blk, cnt1k, d_cnt + 8, c->st);
        scan_excl_u32(blk, blk_off, (size_t)nb, d_nl, c->csv_scr.as<uint32_t>(), c->st);
        c->ktimer_end("csv_count", c->st, nbytes);
        HIP_TRY(hipMemcpyAsync(h_shards.data(), d_cnt + 8, 256 * 8, hipMemcpyDeviceToHost, c->st));
        HIP_TRY(hipMemcpyAsync(&h_nl, d_nl, 4, hipMemcpyDeviceToHost, c->st));
        HIP_TRY(hipMemcpyAsync(&last, text + nbytes - 1, 1, hipMemcpyDeviceToHost, c->st));
        HIP_TRY(hipStreamSynchronize(c->st));
    }
    for (unsigned long long x : h_shards) h_commas += x;
    const int64_t nl = h_nl;
    nrec = nl + (nbytes > 0 && last != '\n' ? 1 : 0);
    const size_t nr1 = (size_t)std::max<int64_t>(nrec, 1);
    // group boundaries only (R records per parse workgroup; R >= 8, and the exact path's groups of
    // 256 need fewer): 8 bytes per group instead of per record
    const int R = csv_records_per_block(nbytes, nrec, (int64_t)h_commas + nrec, D);
    SKY_TRY(c->csv_status.ensure(nr1));
    // byte chunks (SKY_CSV_CHUNKS=1): each parse workgroup finds its records itself and takes the
    // index of its first one from the count pass's prefix, so no group pass
    int ctail = 0;
    const int chunk =
        csv_chunk_mode() ? csv_chunk_bytes(nbytes, nrec, (int64_t)h_commas + nrec, D, &ctail) : 0;
    if (chunk == 0) {
        SKY_TRY(c->csv_lines.ensure((size_t)(std::max<int64_t>(nl, 1) / R + 2) * 8));
        c->ktimer_begin("csv_lines", c->st);
        if (nl) launch_csv_nl_groups(text, nbytes, blk_off, cnt1k, nl, R, c->csv_lines.as<int64_t>(), c->st);
        c->ktimer_end("csv_lines", c->st, nbytes);
    }
    direct = cap >= nrec && d_ids_out && d_values_out;
    if (!direct) {
        SKY_TRY(c->csv_ids.ensure(nr1 * 8));
        SKY_TRY(c->csv_vals.ensure(nr1 * D * 8));
        pid = c->csv_ids.as<int64_t>();
        pval = c->csv_vals.as<double>();
    }
    HIP_TRY(hipMemsetAsync(d_cnt, 0, 40, c->st));   // [1..3] rejected per cause, [4] queued exact conversions
    if (chunk > 0) {
        SKY_TRY(c->csv_keep.ensure(16));                                   // [0]: listed spans
        SKY_TRY(c->csv_spans.ensure((size_t)csv_chunk_count(nbytes, chunk) * sizeof(longlong4)));
        HIP_TRY(hipMemsetAsync(c->csv_keep.p, 0, 4, c->st));
        c->ktimer_begin("csv_parse", c->st);
        launch_csv_parse_chunks(text, nbytes, chunk, ctail, blk_off, cnt1k, D, pid, pval, c->csv_status.as<uint8_t>(), d_cnt,
                                c->csv_keep.as<uint32_t>(), c->csv_spans.as<longlong4>(), c->csv_slow.as<longlong3>(),
                                d_cnt + 4, slow_cap, c->st);
        c->ktimer_end("csv_parse", c->st, nrec);
    } else {
        SKY_TRY(c->csv_keep.ensure((size_t)((nrec + R - 1) / R + 1) * 4));   // spill list of k_csv_fields
        HIP_TRY(hipMemsetAsync(c->csv_keep.p, 0, 4, c->st));
        c->ktimer_begin("csv_parse", c->st);
        launch_csv_parse(text, nbytes, c->csv_lines.as<int64_t>(), nl, nrec, D, pid, pval, c->csv_status.as<uint8_t>(),
                         d_cnt, c->csv_keep.as<uint32_t>(), c->csv_slow.as<longlong3>(), d_cnt + 4, slow_cap, R, c->st);
        c->ktimer_end("csv_parse", c->st, nrec);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(h_cnt, d_cnt, 40, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    if (h_cnt[4] > slow_cap) {   // more exact conversions than the queue holds: re-parse every record exactly
        HIP_TRY(hipMemsetAsync(d_cnt, 0, 40, c->st));
        SKY_TRY(c->csv_lines.ensure((size_t)(std::max<int64_t>(nl, 1) / 256 + 2) * 8));   // unsized on the chunk path
        if (nl) launch_csv_nl_groups(text, nbytes, blk_off, cnt1k, nl, 256, c->csv_lines.as<int64_t>(), c->st);
        launch_csv_parse_exact(text, nbytes, c->csv_lines.as<int64_t>(), nl, nrec, D, pid, pval,
                               c->csv_status.as<uint8_t>(), d_cnt, c->st);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(h_cnt, d_cnt, 40, hipMemcpyDeviceToHost, c->st));
        HIP_TRY(hipStreamSynchronize(c->st));
    }
    const int64_t nbad = (int64_t)(h_cnt[1] + h_cnt[2] + h_cnt[3]);
    const int64_t nacc = nrec - nbad;
    if (counts_out) {
        counts_out[0] = nrec;
        for (int k = 1; k < 4; k++) counts_out[k] = (int64_t)h_cnt[k];
    }
    *n_out = nacc;
    if (d_status_out && nrec)
        HIP_TRY(hipMemcpyAsync(d_status_out, c->csv_status.p, (size_t)nrec, hipMemcpyDeviceToDevice, c->st));
    if (nacc > cap) {
        HIP_TRY(hipStreamSynchronize(c->st));
        set_error("output capacity too small for the accepted records");
        return SKY_E_CAPACITY;
    }
    ARG_CHECK(nacc == 0 || (d_ids_out && d_values_out), "null output buffers");
    if (nbad > 0 || !direct) {
        if (direct) {   // rows were parsed in place: move them aside, then compact back
            SKY_TRY(c->csv_ids.ensure(nr1 * 8));
            SKY_TRY(c->csv_vals.ensure(nr1 * D * 8));
            HIP_TRY(hipMemcpyAsync(c->csv_ids.p, d_ids_out, (size_t)nrec * 8, hipMemcpyDeviceToDevice, c->st));
            HIP_TRY(hipMemcpyAsync(c->csv_vals.p, d_values_out, (size_t)nrec * D * 8, hipMemcpyDeviceToDevice,
                                   c->st));
        }
        SKY_TRY(c->csv_keep.ensure(nr1 * 4));
        SKY_TRY(c->csv_pos.ensure(nr1 * 4 + 16));
        SKY_TRY(c->csv_scr.ensure(scan_scratch_words(nr1) * 4));
        launch_csv_keep(c->csv_status.as<uint8_t>(), nrec, c->csv_keep.as<uint32_t>(), c->st);
        scan_excl_u32(c->csv_keep.as<uint32_t>(), c->csv_pos.as<uint32_t>(), (size_t)nrec,
                      c->csv_pos.as<uint32_t>() + nr1, c->csv_scr.as<uint32_t>(), c->st);
        launch_csv_compact(c->csv_status.as<uint8_t>(), c->csv_pos.as<uint32_t>(), nrec, D, c->csv_ids.as<int64_t>(),
                           c->csv_vals.as<double>(), d_ids_out, d_values_out, c->st);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->st));
    if (c->profile) c->ktimer_collect();
    return SKY_OK;
    GUARD_END
}

int sky_parse_csv(sky_ctx *c, const char *text, int64_t nbytes, int64_t *ids_out, double *values_out, int64_t cap,
                  int64_t *n_out, int64_t *counts_out) {
    GUARD_BEGIN
    ARG_CHECK(c && n_out && (nbytes == 0 || text), "null argument");
    ARG_CHECK(nbytes >= 0 && nbytes < ((int64_t)1 << 40), "nbytes out of range");
    SKY_TRY(bind(c));
    SKY_TRY(c->csv_text.ensure((size_t)std::max<int64_t>(nbytes, 1)));
    if (nbytes) HIP_TRY(hipMemcpyAsync(c->csv_text.p, text, (size_t)nbytes, hipMemcpyHostToDevice, c->st));
    // records are at most nbytes/2 + 1 ("x\n" is the shortest non-empty record)
    const int64_t rmax = nbytes / 2 + 1;
    SKY_TRY(c->h_ids.ensure((size_t)rmax * 8));
    SKY_TRY(c->h_vals.ensure((size_t)rmax * c->D * 8));
    int64_t n = 0;
    SKY_TRY(sky_parse_csv_dev(c, c->csv_text.as<char>(), nbytes, c->h_ids.as<int64_t>(), c->h_vals.as<double>(), rmax,
                              &n, counts_out, nullptr));
    *n_out = n;
    if (n > cap) {
        set_error("output capacity too small for the accepted records");
        return SKY_E_CAPACITY;
    }
    ARG_CHECK(n == 0 || (ids_out && values_out), "null output buffers");
    if (n) {
        HIP_TRY(hipMemcpyAsync(ids_out, c->h_ids.p, (size_t)n * 8, hipMemcpyDeviceToHost, c->st));
        HIP_TRY(hipMemcpyAsync(values_out, c->h_vals.p, (size_t)n * c->D * 8, hipMemcpyDeviceToHost, c->st));
    }
    HIP_TRY(hipStreamSynchronize(c->st));
    return SKY_OK;
    GUARD_END
}

int sky_format_csv_dev(sky_ctx *c, const int64_t *d_ids, const double *d_values, int64_t n, char *d_text, int64_t cap,
                       int64_t *nbytes_out) {
    GUARD_BEGIN
    ARG_CHECK(c && nbytes_out && (n == 0 || (d_ids && d_values)), "null argument");
    ARG_CHECK(n >= 0 && n < (int64_t)0x7fffffffLL, "n out of range");
    SKY_TRY(bind(c));
    const size_t n1 = (size_t)std::max<int64_t>(n, 1);
    SKY_TRY(c->csv_keep.ensure(n1 * 4));
    SKY_TRY(c->csv_pos.ensure(n1 * 4 + 16));
    SKY_TRY(c->csv_scr.ensure(scan_scratch_words(n1) * 4));
    SKY_TRY(c->csv_counts.ensure(64));
    unsigned long long *d_te = c->csv_counts.as<unsigned long long>();
    HIP_TRY(hipMemsetAsync(d_te, 0, 16, c->st));
    launch_csv_fmt_len(d_ids, d_values, n, c->D, c->csv_keep.as<uint32_t>(), d_te, c->st);
    unsigned long long h_te[2] = {};
    HIP_TRY(hipMemcpyAsync(h_te, d_te, 16, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    if (h_te[1]) {
        set_error("sky_format_csv_dev formats integral values |v| < 2^53 only");
        return SKY_E_ARG;
    }
    *nbytes_out = (int64_t)h_te[0];
    if (!d_text || cap == 0) return SKY_OK;
    if ((int64_t)h_te[0] > cap) {
        set_error("text capacity too small");
        return SKY_E_CAPACITY;
    }
    ARG_CHECK(h_te[0] < 0xffffffffull, "formatted text must stay below 4 GiB per call");
    scan_excl_u32(c->csv_keep.as<uint32_t>(), c->csv_pos.as<uint32_t>(), (size_t)n, c->csv_pos.as<uint32_t>() + n1,
                  c->csv_scr.as<uint32_t>(), c->st);
    launch_csv_fmt_write(d_ids, d_values, n, c->D, c->csv_pos.as<uint32_t>(), reinterpret_cast<uint8_t *>(d_text),
                         c->st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->st));
    return SKY_OK;
    GUARD_END
}

int sky_profile_sort_dev(sky_ctx *c, uint64_t *d_keys, uint32_t *d_vals, int64_t n, int32_t *passes_out,
                         double *ms_out) {
    GUARD_BEGIN
    ARG_CHECK(c && d_keys && d_vals && n >= 0 && n < (int64_t)0xffffffffLL, "bad arguments");
    SKY_TRY(bind(c));
    const uint32_t m = (uint32_t)n;
    SKY_TRY(c->prof_k.ensure((size_t)std::max<int64_t>(n, 1) * 8));
    SKY_TRY(c->prof_v.ensure((size_t)std::max<int64_t>(n, 1) * 4));
    SKY_TRY(c->prof_scr.ensure(radix_scratch_words(m) * 4 + 64));
    SKY_TRY(c->csv_counts.ensure(64 + 256 * 8));
    unsigned long long *d_orand = c->csv_counts.as<unsigned long long>();
    radix_key_orand(d_keys, m, d_orand, c->st);
    unsigned long long orand[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(orand, d_orand, 16, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    uint32_t *err = reinterpret_cast<uint32_t *>(d_orand + 4);
    HIP_TRY(hipMemsetAsync(err, 0, 4, c->st));
    hipEvent_t a = c->take_event(), b = c->take_event();
    HIP_TRY(hipEventRecord(a, c->st));
    hipError_t lerr = hipSuccess;
    const bool alt = radix_sort_pairs(d_keys, d_vals, c->prof_k.as<uint64_t>(), c->prof_v.as<uint32_t>(), m, orand[0],
                                      orand[1], c->prof_scr.as<uint32_t>(), err, c->st, &lerr);
    HIP_TRY(lerr);
    HIP_TRY(hipEventRecord(b, c->st));
    if (alt) {
        HIP_TRY(hipMemcpyAsync(d_keys, c->prof_k.p, (size_t)n * 8, hipMemcpyDeviceToDevice, c->st));
        HIP_TRY(hipMemcpyAsync(d_vals, c->prof_v.p, (size_t)n * 4, hipMemcpyDeviceToDevice, c->st));
    }
    uint32_t h_err = 0;
    HIP_TRY(hipMemcpyAsync(&h_err, err, 4, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, a, b));
    c->event_pool.push_back(a);
    c->event_pool.push_back(b);
    if (h_err) {
        set_error("radix sort look-back spin bound reached");
        return SKY_E_HIP;
    }
    if (passes_out) *passes_out = radix_last_passes();
    if (ms_out) *ms_out = ms;
    return SKY_OK;
    GUARD_END
}

int sky_profile_pairs_dev(sky_ctx *c, const double *d_values, const int32_t *d_keys, int64_t n, uint32_t *d_fates_out,
                          int32_t *kind_out, double *ms_out) {
    GUARD_BEGIN
    ARG_CHECK(c && d_values && d_keys && d_fates_out && n >= 0 && n < (int64_t)0x7fffffffLL, "bad arguments");
    SKY_TRY(bind(c));
    const int D = c->D;
    const uint32_t m = (uint32_t)n;
    const size_t DP = (size_t)padded_dims<double>(D);
    SKY_TRY(c->prof_v.ensure((size_t)std::max<int64_t>(n, 1) * DP * 8));
    SKY_TRY(c->prof_k.ensure((size_t)std::max<int64_t>(n, 1) * 8));
    SKY_TRY(c->prof_scr.ensure(64));
    uint32_t *d_flags = c->prof_scr.as<uint32_t>();
    HIP_TRY(hipMemsetAsync(d_flags, 0, 4, c->st));
    launch_prof_slots(D, d_values, d_keys, m, c->prof_v.as<double>(), c->prof_k.as<uint64_t>(), d_flags, c->st);
    uint32_t fl = 0;
    HIP_TRY(hipMemcpyAsync(&fl, d_flags, 4, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    // the compare type the query's brute pass would take: packed u16 for integer rows with a
    // tie-free score, f32 when every value is an f32, else f64
    const bool f64 = (fl & kFlagNotF32) != 0;
    const bool u16 = !f64 && !(fl & kFlagNotU16) && !(fl & kFlagScoreTies);
    HIP_TRY(hipMemsetAsync(d_fates_out, 0, (size_t)std::max<int64_t>(n, 1) * 4, c->st));
    hipEvent_t a = c->take_event(), b = c->take_event();
    HIP_TRY(hipEventRecord(a, c->st));
    launch_brute_pairs(D, !f64, u16, c->prof_v.p, c->prof_k.as<uint64_t>(), m, d_fates_out, c->st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(b, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, a, b));
    c->event_pool.push_back(a);
    c->event_pool.push_back(b);
    if (kind_out) *kind_out = u16 ? 0 : (f64 ? 2 : 1);
    if (ms_out) *ms_out = ms;
    return SKY_OK;
    GUARD_END
}
