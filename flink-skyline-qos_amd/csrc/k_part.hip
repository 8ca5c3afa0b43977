// k_part.hip — the per-key operator state (sky_part_*) updated incrementally.
//
// SkylineLocalProcessor.processBuffer (FlinkSkyline.java:417-444) sets S <- SKY(S u B) for
// every 5000-tuple buffer B.  The state is held as
//   reps     distinct vectors (f64 [R][D]), alive flag, number of tuples per rep
//   tuples   ids and rep index in insertion order (T entries, Tdead of them on dead reps)
// and an insert costs O(|B| (|B| + R)) pair tests plus O(|B|) writes, independent of the
// number of (duplicate) tuples in S:
//   k_parts_pairs  B vs B, B vs alive S reps  -> dom_b (any dominator), eq_s (equal S rep),
//                  eq_b (first equal earlier batch tuple);  S reps vs B -> dom_s
//   k_parts_commit per batch tuple: kept (not dominated), new rep (kept, first of its vector, no
//                  equal S rep); kept tuples appended (ids, rep), new reps appended, joined reps
//                  counted; dominated S reps die, their tuples count as dead (compacted lazily)
// S reps are never dominated by each other, a tuple equal to a rep shares its fate (equal
// vectors never dominate each other), and a rep killed by b kills every batch tuple equal to
// it too (b dominates them), so no surviving tuple joins a dying rep.
// NaN: the host checks the batch while staging it, and a batch holding one is rejected before
// any launch (SKY_E_NAN), so the state never sees it.
#include "sky_internal.h"

namespace sky {

constexpr int kPartX = 128;          // x rows per LDS tile
constexpr uint32_t kPartChunk = 256;    // x rows per workgroup (grid.y): many small workgroups

// ---- batched, asynchronous insert (sky_parts_insert) ---------------------------------------
// One call inserts one batch into each of G parts (the full buffers of several Flink keys) with
// four launches and no host read: k_fill_multi (flags), k_parts_pairs (work items over every
// part), k_parts_commit (one workgroup per part).  Counts live on the device (PartDesc::dcnt);
// launches are sized by host-side bounds and clamp to the device counts; the commit mirrors
// the new counts into host-mapped memory (seqlock) so that the host tightens its bounds
// without synchronising.

// dominance as ServiceTuple.dominates (ServiceTuple.java:67-77): <= everywhere, < somewhere
// mode 0: batch y vs batch x (dom_b, eq_b: first EARLIER equal batch tuple)
// mode 1: batch y vs alive state reps x (dom_b, eq_s: first equal rep)
// mode 2: state reps y vs batch x (dom_s)
template <int D>
__global__ __launch_bounds__(kThreads) void k_parts_pairs(const PartDesc *__restrict__ descs,
                                                          const PartItem *__restrict__ items) {
    __shared__ double s_x[kPartX * D];
    const PartItem it = items[blockIdx.x];
    const PartDesc &d = descs[it.part];
    const uint32_t R0 = d.dcnt[0];
    const int mode = (int)it.mode;
    const double *y = mode == 2 ? d.rrows : d.bvals;
    const uint32_t ny = mode == 2 ? min(R0, d.rb) : d.nb;
    const double *x = mode == 1 ? d.rrows : d.bvals;
    const uint32_t nx = mode == 1 ? min(R0, d.rb) : d.nb;
    const uint32_t j = it.y0 + threadIdx.x;
    const bool valid = j < ny;
    if (it.y0 >= ny || it.x0 >= nx) return;
    double v[D];
#pragma unroll
    for (int q = 0; q < D; q++) v[q] = valid ? y[(size_t)j * D + q] : 0.0;
    const uint32_t c1 = min(nx, it.x0 + kPartChunk);
    bool dm = false;
    uint32_t emin = 0xffffffffu;
    for (uint32_t t0 = it.x0; t0 < c1; t0 += kPartX) {
        const uint32_t cn = min((uint32_t)kPartX, c1 - t0);
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < cn * D; q += kThreads) s_x[q] = x[(size_t)t0 * D + q];
        __syncthreads();
        if (!valid) continue;
        for (uint32_t i = 0; i < cn; i++) {
            const uint32_t xi = t0 + i;
            bool le = true, ge = true;
#pragma unroll
            for (int q = 0; q < D; q++) {
                const double a = s_x[i * D + q];
                le &= a <= v[q];
                ge &= a >= v[q];
            }
            const bool skip = (mode == 0 && xi == j) || (mode == 1 && !d.ralive[xi]);
            dm |= !skip && le && !ge;
            if (!skip && le && ge && xi < emin && (mode != 0 || xi < j)) emin = xi;
        }
    }
    if (!valid) return;
    if (mode == 2) {
        if (dm) d.dom_s[j] = 1u;
        return;
    }
    if (dm) d.dom_b[j] = 1u;
    if (emin != 0xffffffffu) atomicMin(mode == 0 ? &d.eq_b[j] : &d.eq_s[j], emin);
}

// exclusive rank of a 0/1 flag over the 1024 threads, and the block total
__device__ __forceinline__ uint32_t rank1024(bool f, uint32_t *s_w, uint32_t &total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m = __ballot(f);
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    __syncthreads();
    if (lane == 0) s_w[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int w = 0; w < 16; w++) {
        const uint32_t c = s_w[w];
        off += w < wave ? c : 0u;
        tot += c;
    }
    total = tot;
    return off + (uint32_t)__popcll(m & lt);
}

// one workgroup per part: kept batch tuples appended (insertion order), new reps appended,
// tuples joining an existing rep counted, dominated reps killed; the new counts to the device
// and to the host mirror
template <int D>
__global__ __launch_bounds__(1024) void k_parts_commit(const PartDesc *__restrict__ descs) {
    __shared__ uint32_t s_w[16];
    __shared__ unsigned long long s_dead;
    const PartDesc &d = descs[blockIdx.x];
    const uint32_t R0 = d.dcnt[0], T0 = d.dcnt[1];
    const uint32_t nb = d.nb;
    if (threadIdx.x == 0) s_dead = 0;
    uint32_t kbase = 0, fbase = 0;
    for (uint32_t c0 = 0; c0 < nb; c0 += 1024) {
        const uint32_t b = c0 + threadIdx.x;
        const bool valid = b < nb;
        const bool keep = valid && d.dom_b[b] == 0u;
        const bool fresh = keep && d.eq_s[b] == 0xffffffffu && d.eq_b[b] == 0xffffffffu;
        uint32_t kt, ft;
        const uint32_t kp = kbase + rank1024(keep, s_w, kt);
        const uint32_t fp = fbase + rank1024(fresh, s_w, ft);
        if (valid) {
            d.kpos[b] = kp;
            d.fpos[b] = fp;
        }
        if (fresh) {
            const uint32_t r = R0 + fp;
#pragma unroll
            for (int q = 0; q < D; q++) d.rrows[(size_t)r * D + q] = d.bvals[(size_t)b * D + q];
            d.ralive[r] = 1;
            d.rcnt[r] = 0;
        }
        kbase += kt;
        fbase += ft;
    }
    __syncthreads();                           // the new reps and positions are visible
    for (uint32_t c0 = 0; c0 < nb; c0 += 1024) {
        const uint32_t b = c0 + threadIdx.x;
        const bool act = b < nb && d.dom_b[b] == 0u;
        uint32_t rep = 0xffffffffu;
        if (act) {
            const uint32_t e = d.eq_s[b];
            rep = e != 0xffffffffu ? e : R0 + d.fpos[d.eq_b[b] != 0xffffffffu ? d.eq_b[b] : b];
            const uint32_t t = T0 + d.kpos[b];
            d.tids[t] = d.bids[b];
            d.trep[t] = rep;
        }
        // the tuples of a batch mostly join one rep (duplicate-heavy keys): one atomic per wave
        const uint64_t am = __ballot(act);
        if (am) {
            const int leader = __ffsll((unsigned long long)am) - 1;
            const uint32_t r0 = __shfl(rep, leader, 64);
            const bool uni = __ballot(act && rep != r0) == 0ull;
            if (uni) {
                if ((int)(threadIdx.x & 63) == leader) atomicAdd(&d.rcnt[r0], (uint32_t)__popcll(am));
            } else if (act) {
                atomicAdd(&d.rcnt[rep], 1u);
            }
        }
    }
    __syncthreads();                           // joins done before the kills read rcnt
    unsigned long long killed = 0;
    const uint32_t rs = min(R0, d.rb);
    for (uint32_t s = threadIdx.x; s < rs; s += 1024) {
        if (d.dom_s[s] && d.ralive[s]) {
            d.ralive[s] = 0;
            killed += d.rcnt[s];
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) killed += __shfl_xor(killed, o, 64);
    if ((threadIdx.x & 63) == 0 && killed) atomicAdd(&s_dead, killed);
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t R1 = R0 + fbase, T1 = T0 + kbase;
        const unsigned long long dead = ((unsigned long long)d.dcnt[3] << 32 | d.dcnt[2]) + s_dead;
        d.dcnt[0] = R1;
        d.dcnt[1] = T1;
        d.dcnt[2] = (uint32_t)dead;
        d.dcnt[3] = (uint32_t)(dead >> 32);
        if (d.mirror) {                        // seqlock: begin, data, end (the host checks begin == end)
            volatile uint32_t *m = d.mirror;
            m[0] = d.seq;
            __threadfence_system();
            m[1] = R1;
            m[2] = T1;
            m[3] = (uint32_t)dead;
            m[4] = (uint32_t)(dead >> 32);
            __threadfence_system();
            m[5] = d.seq;
        }
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

void launch_parts_insert(int D, const PartDesc *descs, int nparts, const PartItem *items, uint32_t nitems,
                         hipStream_t st) {
    if (nitems) SKY_DISPATCH_D(D, (k_parts_pairs<DD><<<nitems, kThreads, 0, st>>>(descs, items)));
    if (nparts) SKY_DISPATCH_D(D, (k_parts_commit<DD><<<nparts, 1024, 0, st>>>(descs)));
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
