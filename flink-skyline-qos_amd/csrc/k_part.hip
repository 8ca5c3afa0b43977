// k_part.hip — the per-key operator state (sky_part_*) updated incrementally.
//
// SkylineLocalProcessor.processBuffer (FlinkSkyline.java:417-444) sets S <- SKY(S u B) for
// every 5000-tuple buffer B.  The state is held as
//   reps     distinct vectors (f64 [R][D]), alive flag, number of tuples per rep
//   tuples   ids and rep index in insertion order (T entries, Tdead of them on dead reps)
// and an insert costs O(|B| (|B| + R)) pair tests plus O(|B|) writes, independent of the
// number of (duplicate) tuples in S:
//   k_part_pairs   B vs B, B vs alive S reps  -> dom_b (any dominator), eq_s (equal S rep),
//                  eq_b (first equal earlier batch tuple);  S reps vs B -> dom_s
//   k_part_flags   per batch tuple: kept (not dominated), new rep (kept, first of its vector,
//                  no equal S rep) -> two exclusive scans
//   k_part_write   kept tuples appended (ids, rep), new reps appended, joined reps counted
//   k_part_kill    dominated S reps die; their tuples count as dead (compacted lazily)
// S reps are never dominated by each other, a tuple equal to a rep shares its fate (equal
// vectors never dominate each other), and a rep killed by b kills every batch tuple equal to
// it too (b dominates them), so no surviving tuple joins a dying rep.
// NaN in the batch: every state-changing kernel is skipped (the flag is read back once), so a
// rejected batch leaves the state untouched (SKY_E_NAN), as the round-1 path did.
#include "sky_internal.h"

namespace sky {

constexpr int kPartX = 128;          // x rows per LDS tile
constexpr uint32_t kPartChunk = 256;    // x rows per workgroup (grid.y): many small workgroups

// dominance as ServiceTuple.dominates (ServiceTuple.java:67-77): <= everywhere, < somewhere
template <int D>
__global__ __launch_bounds__(kThreads) void k_part_pairs(const double *__restrict__ y, uint32_t ny,
                                                         const double *__restrict__ x, uint32_t nx,
                                                         const uint8_t *__restrict__ x_alive, int same_set,
                                                         const uint32_t *__restrict__ nanflag,
                                                         uint32_t *__restrict__ dom, uint32_t *__restrict__ eq) {
    __shared__ double s_x[kPartX * D];
    if (*nanflag) return;
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    const bool valid = j < ny;
    double v[D];
#pragma unroll
    for (int d = 0; d < D; d++) v[d] = valid ? y[(size_t)j * D + d] : 0.0;
    const uint32_t c0 = blockIdx.y * kPartChunk;
    const uint32_t c1 = min(nx, c0 + kPartChunk);
    bool dm = false;
    uint32_t emin = 0xffffffffu;
    for (uint32_t t0 = c0; t0 < c1; t0 += kPartX) {
        const uint32_t cn = min((uint32_t)kPartX, c1 - t0);
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < cn * D; q += kThreads) s_x[q] = x[(size_t)t0 * D + q];
        __syncthreads();
        if (!valid) continue;
        for (uint32_t i = 0; i < cn; i++) {
            const uint32_t xi = t0 + i;
            bool le = true, ge = true;
#pragma unroll
            for (int d = 0; d < D; d++) {
                const double a = s_x[i * D + d];
                le &= a <= v[d];
                ge &= a >= v[d];
            }
            const bool skip = (same_set && xi == j) || (x_alive && !x_alive[xi]);
            dm |= !skip && le && !ge;
            // equal vectors: the earliest one (same set: an EARLIER batch tuple only, so the
            // first occurrence has none and becomes the new rep)
            if (!skip && le && ge && xi < emin && (!same_set || xi < j)) emin = xi;
        }
    }
    if (valid && dm) atomicOr(&dom[j], 1u);
    if (valid && eq && emin != 0xffffffffu) atomicMin(&eq[j], emin);
}

__global__ __launch_bounds__(kThreads) void k_part_flags(uint32_t nb, const uint32_t *__restrict__ dom_b,
                                                         const uint32_t *__restrict__ eq_s,
                                                         const uint32_t *__restrict__ eq_b, uint32_t *__restrict__ keep,
                                                         uint32_t *__restrict__ fresh) {
    const uint32_t b = blockIdx.x * kThreads + threadIdx.x;
    if (b >= nb) return;
    const bool k = dom_b[b] == 0u;
    keep[b] = k ? 1u : 0u;
    fresh[b] = (k && eq_s[b] == 0xffffffffu && eq_b[b] == 0xffffffffu) ? 1u : 0u;
}

template <int D>
__global__ __launch_bounds__(kThreads) void k_part_write(uint32_t nb, const int64_t *__restrict__ bids,
                                                         const double *__restrict__ bvals,
                                                         const uint32_t *__restrict__ keep,
                                                         const uint32_t *__restrict__ keep_pos,
                                                         const uint32_t *__restrict__ fresh,
                                                         const uint32_t *__restrict__ fresh_pos,
                                                         const uint32_t *__restrict__ eq_s,
                                                         const uint32_t *__restrict__ eq_b, uint32_t R, uint32_t T,
                                                         const uint32_t *__restrict__ nanflag,
                                                         double *__restrict__ rrows, uint8_t *__restrict__ ralive,
                                                         uint32_t *__restrict__ rcnt, int64_t *__restrict__ tids,
                                                         uint32_t *__restrict__ trep) {
    const uint32_t b = blockIdx.x * kThreads + threadIdx.x;
    const bool act = b < nb && !*nanflag && keep[b];
    // the tuples of a batch mostly join one rep (duplicate-heavy keys): one atomic per wave then
    uint32_t rep = 0xffffffffu;
    if (act) {
        const uint32_t e = eq_s[b];
        rep = e != 0xffffffffu ? e : R + fresh_pos[eq_b[b] != 0xffffffffu ? eq_b[b] : b];
    }
    const uint64_t am = __ballot(act);
    if (!am) return;
    const uint32_t r0 = __shfl(rep, __ffsll((unsigned long long)am) - 1, 64);
    const bool uni = __ballot(act && rep != r0) == 0ull;
    if (uni && (threadIdx.x & 63) == (uint32_t)(__ffsll((unsigned long long)am) - 1))
        atomicAdd(&rcnt[r0], (uint32_t)__popcll(am));
    if (!act) return;
    if (!uni) atomicAdd(&rcnt[rep], 1u);
    if (fresh[b]) {
        const uint32_t r = R + fresh_pos[b];
#pragma unroll
        for (int d = 0; d < D; d++) rrows[(size_t)r * D + d] = bvals[(size_t)b * D + d];
        ralive[r] = 1;
    }
    const uint32_t t = T + keep_pos[b];
    tids[t] = bids[b];
    trep[t] = rep;
}

__global__ __launch_bounds__(kThreads) void k_part_kill(uint32_t R, const uint32_t *__restrict__ dom_s,
                                                        const uint32_t *__restrict__ nanflag,
                                                        uint8_t *__restrict__ ralive, const uint32_t *__restrict__ rcnt,
                                                        unsigned long long *__restrict__ dead) {
    const uint32_t s = blockIdx.x * kThreads + threadIdx.x;
    if (s >= R || *nanflag) return;
    if (dom_s[s] && ralive[s]) {
        ralive[s] = 0;
        atomicAdd(dead, (unsigned long long)rcnt[s]);
    }
}

// ---- compaction (dead reps and their tuples) and read-out -------------------------------
__global__ __launch_bounds__(kThreads) void k_part_rkeep(uint32_t R, const uint8_t *__restrict__ ralive,
                                                         uint32_t *__restrict__ keep) {
    const uint32_t s = blockIdx.x * kThreads + threadIdx.x;
    if (s < R) keep[s] = ralive[s] ? 1u : 0u;
}

template <int D>
__global__ __launch_bounds__(kThreads) void k_part_rmove(uint32_t R, const uint32_t *__restrict__ keep,
                                                         const uint32_t *__restrict__ pos,
                                                         const double *__restrict__ rows, const uint32_t *__restrict__ cnt,
                                                         double *__restrict__ rows2, uint32_t *__restrict__ cnt2,
                                                         uint8_t *__restrict__ alive2) {
    const uint32_t s = blockIdx.x * kThreads + threadIdx.x;
    if (s >= R || !keep[s]) return;
    const uint32_t p = pos[s];
#pragma unroll
    for (int d = 0; d < D; d++) rows2[(size_t)p * D + d] = rows[(size_t)s * D + d];
    cnt2[p] = cnt[s];
    alive2[p] = 1;
}

__global__ __launch_bounds__(kThreads) void k_part_tkeep(uint32_t T, const uint32_t *__restrict__ trep,
                                                         const uint8_t *__restrict__ ralive, uint32_t *__restrict__ keep) {
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t < T) keep[t] = ralive[trep[t]] ? 1u : 0u;
}

__global__ __launch_bounds__(kThreads) void k_part_tmove(uint32_t T, const uint32_t *__restrict__ keep,
                                                         const uint32_t *__restrict__ pos,
                                                         const uint32_t *__restrict__ rpos,
                                                         const int64_t *__restrict__ ids, const uint32_t *__restrict__ trep,
                                                         int64_t *__restrict__ ids2, uint32_t *__restrict__ trep2) {
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t >= T || !keep[t]) return;
    const uint32_t p = pos[t];
    ids2[p] = ids[t];
    trep2[p] = rpos[trep[t]];
}

template <int D>
__global__ __launch_bounds__(kThreads) void k_part_rows_out(uint32_t T, const uint32_t *__restrict__ trep,
                                                            const double *__restrict__ rrows, double *__restrict__ out) {
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t >= T) return;
    const uint32_t r = trep[t];
#pragma unroll
    for (int d = 0; d < D; d++) out[(size_t)t * D + d] = rrows[(size_t)r * D + d];
}

// ---- launchers ---------------------------------------------------------------------------
static inline unsigned nbk(size_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

void launch_part_pairs(int D, const double *y, uint32_t ny, const double *x, uint32_t nx, const uint8_t *x_alive,
                       bool same_set, const uint32_t *nanflag, uint32_t *dom, uint32_t *eq, hipStream_t st) {
    if (!ny || !nx) return;
    const dim3 g(nbk(ny), (nx + kPartChunk - 1) / kPartChunk);
    SKY_DISPATCH_D(D, (k_part_pairs<DD><<<g, kThreads, 0, st>>>(y, ny, x, nx, x_alive, same_set ? 1 : 0, nanflag,
                                                                 dom, eq)));
}

void launch_part_flags(uint32_t nb, const uint32_t *dom_b, const uint32_t *eq_s, const uint32_t *eq_b, uint32_t *keep,
                       uint32_t *fresh, hipStream_t st) {
    if (nb) k_part_flags<<<nbk(nb), kThreads, 0, st>>>(nb, dom_b, eq_s, eq_b, keep, fresh);
}

void launch_part_write(int D, uint32_t nb, const int64_t *bids, const double *bvals, const uint32_t *keep,
                       const uint32_t *keep_pos, const uint32_t *fresh, const uint32_t *fresh_pos, const uint32_t *eq_s,
                       const uint32_t *eq_b, uint32_t R, uint32_t T, const uint32_t *nanflag, double *rrows,
                       uint8_t *ralive, uint32_t *rcnt, int64_t *tids, uint32_t *trep, hipStream_t st) {
    if (!nb) return;
    SKY_DISPATCH_D(D, (k_part_write<DD><<<nbk(nb), kThreads, 0, st>>>(nb, bids, bvals, keep, keep_pos, fresh, fresh_pos,
                                                                      eq_s, eq_b, R, T, nanflag, rrows, ralive, rcnt,
                                                                      tids, trep)));
}

void launch_part_kill(uint32_t R, const uint32_t *dom_s, const uint32_t *nanflag, uint8_t *ralive, const uint32_t *rcnt,
                      unsigned long long *dead, hipStream_t st) {
    if (R) k_part_kill<<<nbk(R), kThreads, 0, st>>>(R, dom_s, nanflag, ralive, rcnt, dead);
}

void launch_part_rkeep(uint32_t R, const uint8_t *ralive, uint32_t *keep, hipStream_t st) {
    if (R) k_part_rkeep<<<nbk(R), kThreads, 0, st>>>(R, ralive, keep);
}

void launch_part_rmove(int D, uint32_t R, const uint32_t *keep, const uint32_t *pos, const double *rows,
                       const uint32_t *cnt, double *rows2, uint32_t *cnt2, uint8_t *alive2, hipStream_t st) {
    if (!R) return;
    SKY_DISPATCH_D(D, (k_part_rmove<DD><<<nbk(R), kThreads, 0, st>>>(R, keep, pos, rows, cnt, rows2, cnt2, alive2)));
}

void launch_part_tkeep(uint32_t T, const uint32_t *trep, const uint8_t *ralive, uint32_t *keep, hipStream_t st) {
    if (T) k_part_tkeep<<<nbk(T), kThreads, 0, st>>>(T, trep, ralive, keep);
}

void launch_part_tmove(uint32_t T, const uint32_t *keep, const uint32_t *pos, const uint32_t *rpos, const int64_t *ids,
                       const uint32_t *trep, int64_t *ids2, uint32_t *trep2, hipStream_t st) {
    if (T) k_part_tmove<<<nbk(T), kThreads, 0, st>>>(T, keep, pos, rpos, ids, trep, ids2, trep2);
}

void launch_part_rows_out(int D, uint32_t T, const uint32_t *trep, const double *rrows, double *out, hipStream_t st) {
    if (!T) return;
    SKY_DISPATCH_D(D, (k_part_rows_out<DD><<<nbk(T), kThreads, 0, st>>>(T, trep, rrows, out)));
}

}  // namespace sky
