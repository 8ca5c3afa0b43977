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

// ---- batch pruners (k_parts_prune) --------------------------------------------------------
// Before any pair test, each part's batch is reduced to its UNDECIDED tuples U: kPartPruners
// batch tuples p_c minimise positive-weight linear criteria (a dominator never has a larger
// criterion value: rounding is monotone), and every batch tuple is classified against them in
// order c = 0, 1, ...: dominated by p_c (dropped: dom_b = 1), equal to p_c (class c: shares the
// fate of p_c, the class's first index is its equal-earlier tuple), or neither (undecided).  U =
// the undecided tuples plus each non-empty class's pruner.  Then
//   - a dominator of y in U is a pruned tuple t (its pruner, or a pruner before it, dominates y
//     and reaches U as a class pruner), a class member (its pruner is in U, same vector) or in U;
//   - an equal batch tuple of an undecided y is undecided too (a pruner dominating or equal to
//     it would dominate or equal y);
//   - a state rep dominated by a batch tuple is dominated by a member of U (same argument);
// so B x B and the state tests run over U only: O(|U| (|U| + R)) pair tests instead of
// O(|B| (|B| + R)).  On the reference streams a 5000-tuple buffer keeps a few hundred tuples.
template <int D>
__device__ __forceinline__ double part_crit(const double (&v)[D], int c) {
    // c = 0: the sum; c >= 1: the sum plus 3 x dimension (c - 1) * D / (kPartPruners - 1)
    double s = 0.0;
    const int dk = c == 0 ? -1 : ((c - 1) * D) / (kPartPruners - 1);
#pragma unroll
    for (int q = 0; q < D; q++) s += q == dk ? 4.0 * v[q] : v[q];
    return s;
}

template <int D>
__global__ __launch_bounds__(1024) void k_parts_prune(const PartDesc *__restrict__ descs) {
    __shared__ double s_bv[16][kPartPruners];
    __shared__ uint32_t s_bi[16][kPartPruners];
    __shared__ double s_pr[kPartPruners][D];
    __shared__ uint32_t s_pi[kPartPruners], s_fe[kPartPruners], s_u;
    const PartDesc &d = descs[blockIdx.x];
    const uint32_t nb = d.nb;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double bv[kPartPruners];
    uint32_t bi[kPartPruners];
#pragma unroll
    for (int c = 0; c < kPartPruners; c++) {
        bv[c] = __longlong_as_double(0x7ff0000000000000ll);
        bi[c] = 0xffffffffu;
    }
    // per thread: increasing b, so the first minimum is kept (ties -> the smallest index)
    for (uint32_t b = threadIdx.x; b < nb; b += 1024) {
        double v[D];
#pragma unroll
        for (int q = 0; q < D; q++) v[q] = d.bvals[(size_t)b * D + q];
#pragma unroll
        for (int c = 0; c < kPartPruners; c++) {
            const double s = part_crit<D>(v, c);
            if (s < bv[c] || bi[c] == 0xffffffffu) {
                bv[c] = s;
                bi[c] = b;
            }
        }
    }
    // (value, index) minimum over the block: waves, then the 16 wave results
#pragma unroll
    for (int c = 0; c < kPartPruners; c++) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const double ov = __shfl_xor(bv[c], o, 64);
            const uint32_t oi = (uint32_t)__shfl_xor((int)bi[c], o, 64);
            if (oi != 0xffffffffu && (bi[c] == 0xffffffffu || ov < bv[c] || (ov == bv[c] && oi < bi[c]))) {
                bv[c] = ov;
                bi[c] = oi;
            }
        }
        if (lane == 0) {
            s_bv[wave][c] = bv[c];
            s_bi[wave][c] = bi[c];
        }
    }
    if (threadIdx.x == 0) s_u = 0;
    __syncthreads();
    if (threadIdx.x < kPartPruners) {
        const int c = threadIdx.x;
        double v = s_bv[0][c];
        uint32_t i = s_bi[0][c];
        for (int w = 1; w < 16; w++) {
            const double ov = s_bv[w][c];
            const uint32_t oi = s_bi[w][c];
            if (oi != 0xffffffffu && (i == 0xffffffffu || ov < v || (ov == v && oi < i))) {
                v = ov;
                i = oi;
            }
        }
        s_pi[c] = i;
        s_fe[c] = 0xffffffffu;
    }
    __syncthreads();
    if (threadIdx.x < kPartPruners * D) {
        const int c = threadIdx.x / D, q = threadIdx.x % D;
        s_pr[c][q] = s_pi[c] != 0xffffffffu ? d.bvals[(size_t)s_pi[c] * D + q] : 0.0;
    }
    __syncthreads();
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t c0 = 0; c0 < nb; c0 += 1024) {
        const uint32_t b = c0 + threadIdx.x;
        const bool valid = b < nb;
        uint32_t cls = 0xffffffffu;
        bool dom = false;
        if (valid) {
            double v[D];
#pragma unroll
            for (int q = 0; q < D; q++) v[q] = d.bvals[(size_t)b * D + q];
            for (int c = 0; c < kPartPruners; c++) {
                if (s_pi[c] == 0xffffffffu) break;
                bool le = true, ge = true;
#pragma unroll
                for (int q = 0; q < D; q++) {
                    le &= s_pr[c][q] <= v[q];
                    ge &= s_pr[c][q] >= v[q];
                }
                if (le && !ge) {
                    dom = true;
                    break;
                }
                if (le) {
                    cls = (uint32_t)c;
                    break;
                }
            }
            if (dom) d.dom_b[b] = 1u;
            d.eqp[b] = cls;
            if (cls != 0xffffffffu) atomicMin(&s_fe[cls], b);
        }
        const bool inU = valid && !dom && (cls == 0xffffffffu || b == s_pi[cls]);
        const uint64_t um = __ballot(inU);
        uint32_t base = 0;
        if (lane == 0 && um) base = atomicAdd(&s_u, (uint32_t)__popcll(um));
        base = (uint32_t)__shfl((int)base, 0, 64);
        if (inU) d.uidx[base + (uint32_t)__popcll(um & lt)] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) d.meta[0] = s_u;
    if (threadIdx.x < kPartPruners) {
        d.meta[1 + threadIdx.x] = s_pi[threadIdx.x];
        d.meta[1 + kPartPruners + threadIdx.x] = s_fe[threadIdx.x];
    }
}

// dominance as ServiceTuple.dominates (ServiceTuple.java:67-77): <= everywhere, < somewhere
// mode 0: undecided y vs undecided x (dom_b, eq_b: first EARLIER equal batch tuple)
// mode 1: undecided y vs alive state reps x (dom_b, eq_s: first equal rep)
// mode 2: state reps y vs undecided x (dom_s)
// Launch sizes come from the batch size (a bound of |U|, which lives on the device): work items
// past |U| return at once.
template <int D>
__global__ __launch_bounds__(kThreads) void k_parts_pairs(const PartDesc *__restrict__ descs,
                                                          const PartItem *__restrict__ items) {
    __shared__ double s_x[kPartX * D];
    __shared__ uint32_t s_xi[kPartX];
    const PartItem it = items[blockIdx.x];
    const PartDesc &d = descs[it.part];
    const uint32_t R0 = d.dcnt[0];
    const uint32_t nu = min(d.meta[0], d.nb);
    const int mode = (int)it.mode;
    const uint32_t ny = mode == 2 ? min(R0, d.rb) : nu;
    const uint32_t nx = mode == 1 ? min(R0, d.rb) : nu;
    if (it.y0 >= ny || it.x0 >= nx) return;
    const uint32_t yi = it.y0 + threadIdx.x;
    const bool valid = yi < ny;
    // y: its row and its index (batch index for modes 0 / 1, rep index for mode 2)
    const uint32_t j = valid ? (mode == 2 ? yi : d.uidx[yi]) : 0u;
    const double *ysrc = mode == 2 ? d.rrows : d.bvals;
    double v[D];
#pragma unroll
    for (int q = 0; q < D; q++) v[q] = valid ? ysrc[(size_t)j * D + q] : 0.0;
    const uint32_t c1 = min(nx, it.x0 + kPartChunk);
    bool dm = false;
    uint32_t emin = 0xffffffffu;
    for (uint32_t t0 = it.x0; t0 < c1; t0 += kPartX) {
        const uint32_t cn = min((uint32_t)kPartX, c1 - t0);
        __syncthreads();
        if (mode == 1) {
            for (uint32_t q = threadIdx.x; q < cn * D; q += kThreads) s_x[q] = d.rrows[(size_t)t0 * D + q];
            if (threadIdx.x < cn) s_xi[threadIdx.x] = d.ralive[t0 + threadIdx.x] ? t0 + threadIdx.x : 0xffffffffu;
        } else {
            if (threadIdx.x < cn) s_xi[threadIdx.x] = d.uidx[t0 + threadIdx.x];
            __syncthreads();
            for (uint32_t q = threadIdx.x; q < cn * D; q += kThreads)
                s_x[q] = d.bvals[(size_t)s_xi[q / D] * D + q % D];
        }
        __syncthreads();
        if (!valid) continue;
        for (uint32_t i = 0; i < cn; i++) {
            const uint32_t xo = s_xi[i];
            bool le = true, ge = true;
#pragma unroll
            for (int q = 0; q < D; q++) {
                const double a = s_x[i * D + q];
                le &= a <= v[q];
                ge &= a >= v[q];
            }
            const bool skip = (mode == 0 && xo == j) || (mode == 1 && xo == 0xffffffffu);
            dm |= !skip && le && !ge;
            if (!skip && le && ge && xo < emin && (mode != 0 || xo < j)) emin = xo;
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
    // the members of a pruner class take the fate of its pruner (same vector); the class's
    // first index is their first equal batch tuple
    for (uint32_t b = threadIdx.x; b < nb; b += 1024) {
        const uint32_t c = d.eqp[b];
        if (c == 0xffffffffu) continue;
        const uint32_t r = d.meta[1 + c], fe = d.meta[1 + kPartPruners + c];
        if (b != r) {
            d.dom_b[b] = d.dom_b[r];
            d.eq_s[b] = d.eq_s[r];
        }
        d.eq_b[b] = fe < b ? fe : 0xffffffffu;
    }
    __syncthreads();
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
    if (nparts) SKY_DISPATCH_D(D, (k_parts_prune<DD><<<nparts, 1024, 0, st>>>(descs)));
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
