// abi_common.h — status-code plumbing shared by the extern "C" translation units.
#pragma once
#include "ctx.h"

#include <new>
#include <string>

using namespace sky;

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) {                                                           \
            set_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " #expr);   \
            return SKY_E_HIP;                                                             \
        }                                                                                 \
    } while (0)
#define SKY_TRY(expr)                \
    do {                             \
        int r_ = (expr);             \
        if (r_ != SKY_OK) return r_; \
    } while (0)
#define ARG_CHECK(cond, msg)          \
    do {                              \
        if (!(cond)) {                \
            set_error(msg);           \
            return SKY_E_ARG;         \
        }                             \
    } while (0)
#define GUARD_BEGIN try {
#define GUARD_END                                             \
    }                                                         \
    catch (const std::bad_alloc &) {                          \
        set_error("host allocation failed");                  \
        return SKY_E_NOMEM;                                   \
    }                                                         \
    catch (...) {                                             \
        set_error("internal error");                          \
        return SKY_E_HIP;                                     \
    }

static inline int bind(sky_ctx *c) {
    // hipGetLastError() is per thread and sticky: drop whatever another library
    // (e.g. torch) left behind so our launch checks only see our own failures
    (void)hipGetLastError();
    HIP_TRY(hipSetDevice(c->dev));
    return SKY_OK;
}


static inline void store_stats(sky_ctx *c, const Pipe &p) {
    c->K_last = p.K;
    c->lsz.assign(p.h_lsz.begin(), p.h_lsz.end());
    c->surv.assign(p.h_surv.begin(), p.h_surv.end());
    c->counters[0] = p.n;
    c->counters[1] = p.m;
    c->counters[2] = p.mr;
    c->counters[3] = p.mg;
    c->counters[4] = p.nout;
    c->counters[5] = p.sfs_rounds;
    c->counters[6] = p.sfs_pairs_upper;
    c->counters[7] = (p.f64 ? 1 : 0) | (p.ties ? 2 : 0) | (p.u16 ? 4 : 0) | (p.last_planned ? 8 : 0) |
                     (p.last_plan_miss ? 16 : 0) | (p.last_tiny ? 32 : 0) | (p.mbr_tiles << 8);
    c->dom_w = p.dom_w;
}

static inline void finish_profile(sky_ctx *c) {
    if (!c->profile) return;
    hipStreamSynchronize(c->st);
    for (int i = 0; i < SKY_PHASES; i++) {
        float ms = 0;
        c->phase_ms[i] = 0;
        if (c->pt.marked[i] && c->pt.marked[i + 1] &&
            hipEventElapsedTime(&ms, c->pt.ev[i], c->pt.ev[i + 1]) == hipSuccess)
            c->phase_ms[i] = ms;
    }
    c->ktimer_collect();
}

