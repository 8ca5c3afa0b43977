// k_part.hip — the per-key operator state (sky_part_*) updated incrementally.
//
// SkylineLocalProcessor.processBuffer (FlinkSkyline.java:417-444) sets S <- SKY(S u B) for
// every 5000-tuple buffer B.  The state is held as
//   reps     distinct vectors (f64 [R][D]), alive flag, number of tuples per rep
//   tuples   ids and rep index in insertion order (T entries, Tdead of them on dead reps)
// and an insert costs O(|U| (|U| + R)) pair tests (U: the batch tuples its pruners leave
// undecided) plus O(|B|) work, independent of the number of (duplicate) tuples in S:
//   k_parts_crit / k_parts_classify  batch pruners: every batch tuple dropped (dominated by a
//                  pruner), in a pruner's class (equal to it) or undecided (U)
//   k_parts_pairs  U vs U, U vs alive S reps  -> dom_b (any dominator), eq_s (equal S rep),
//                  eq_b (first equal earlier batch tuple);  S reps vs U -> dom_s
//   k_parts_count / k_parts_place / k_parts_join  per batch tuple: kept (not dominated), new rep
//                  (kept, first of its vector, no equal S rep); kept tuples appended (ids, rep),
//                  new reps appended, joined reps counted; dominated S reps die, their tuples
//                  count as dead (compacted lazily)
// S reps are never dominated by each other, a tuple equal to a rep shares its fate (equal
// vectors never dominate each other), and a rep killed by b kills every batch tuple equal to
// it too (b dominates them), so no surviving tuple joins a dying rep.
// NaN: the host checks the batch while staging it, and a batch holding one is rejected before
// any launch (SKY_E_NAN), so the state never sees it.
#include "sky_internal.h"


#include <algorithm>

namespace sky {

constexpr int kPartX = 128;          // x rows per LDS tile
constexpr uint32_t kPartChunk = 256;    // x rows per workgroup (grid.y): many small workgroups

// ---- batched, asynchronous insert (sky_parts_insert) ---------------------------------------
// One call inserts one batch into each of G parts (the full buffers of several Flink keys) with
// six launches and no host read (grid = batch slice x part, except the pair pass: one
// workgroup per work item).  Counts live on the device (PartDesc::dcnt); launches are sized by
// host-side bounds and clamp to the device counts; the part's last slice mirrors the new counts
// into host-mapped memory (seqlock) so that the host tightens its bounds without synchronising.

// ---- batch pruners (k_parts_crit, k_parts_classify) ----------------------------------------
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

// The insert's kernels work on SLICES of kPartSlice batch tuples (grid.x = slice, grid.y =
// part; 256 threads, 4 tuples each, b = slice * 1024 + k * 256 + thread): a 5000-tuple buffer
// spreads over 5 workgroups per part instead of one 1024-thread workgroup, whose dependent
// chain of loads, reductions and barriers (one CU) took 20-30 us per call.
constexpr int kSliceIt = kPartSlice / kThreads;    // tuples per thread

// (value, index) lexicographic minimum: the smaller criterion, then the smaller index
__device__ __forceinline__ void vi_min(double &v, uint32_t &i, double ov, uint32_t oi) {
    if (oi != 0xffffffffu && (i == 0xffffffffu || ov < v || (ov == v && oi < i))) {
        v = ov;
        i = oi;
    }
}

// K1: per slice, the (criterion, index) minimum of each criterion; slice 0 also resets the
// part's insert words (|U|, first indices, killed tuples, tickets)
template <int D>
__device__ __forceinline__ void parts_crit(const PartDesc *__restrict__ descs, uint32_t slice, uint32_t part,
                                               uint32_t nsl_grid) {
    __shared__ double s_bv[kThreads / 64][kPartPruners];
    __shared__ uint32_t s_bi[kThreads / 64][kPartPruners];
    const PartDesc &d = descs[part];
    const uint32_t nb = d.nb, s0 = slice * kPartSlice;
    if (s0 >= nb) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (slice == 0 && threadIdx.x < kPartMeta) d.meta[threadIdx.x] = threadIdx.x >= 1 + kPartPruners &&
                                                                          threadIdx.x < 1 + 2 * kPartPruners
                                                                          ? 0xffffffffu : 0u;
    double rv[kSliceIt][D];
#pragma unroll
    for (int k = 0; k < kSliceIt; k++) {
        const uint32_t b = min(s0 + k * kThreads + threadIdx.x, nb - 1u);
#pragma unroll
        for (int q = 0; q < D; q++) rv[k][q] = d.bvals[(size_t)b * D + q];
    }
    double bv[kPartPruners];
    uint32_t bi[kPartPruners];
#pragma unroll
    for (int c = 0; c < kPartPruners; c++) {
        bv[c] = 0.0;
        bi[c] = 0xffffffffu;
    }
#pragma unroll
    for (int k = 0; k < kSliceIt; k++) {
        const uint32_t b = s0 + k * kThreads + threadIdx.x;
        if (b >= nb) continue;
#pragma unroll
        for (int c = 0; c < kPartPruners; c++) vi_min(bv[c], bi[c], part_crit<D>(rv[k], c), b);
    }
#pragma unroll
    for (int c = 0; c < kPartPruners; c++) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1)
            vi_min(bv[c], bi[c], __shfl_xor(bv[c], o, 64), (uint32_t)__shfl_xor((int)bi[c], o, 64));
        if (lane == 0) {
            s_bv[wave][c] = bv[c];
            s_bi[wave][c] = bi[c];
        }
    }
    __syncthreads();
    if (threadIdx.x < kPartPruners) {
        const int c = threadIdx.x;
        double v = s_bv[0][c];
        uint32_t i = s_bi[0][c];
        for (int w = 1; w < kThreads / 64; w++) vi_min(v, i, s_bv[w][c], s_bi[w][c]);
        d.sl_v[slice * kPartPruners + c] = v;
        d.sl_i[slice * kPartPruners + c] = i;
    }
}
template <int D>
__global__ __launch_bounds__(kThreads) void k_parts_crit(const PartDesc *__restrict__ descs) {
    parts_crit<D>(descs, blockIdx.x, blockIdx.y, gridDim.x);
}

// K2: the pruners (the minima over the part's slices, reduced by every workgroup itself), then
// each tuple of the slice classified: dropped / pruner class / undecided (appended to U)
template <int D>
__device__ __forceinline__ void parts_classify(const PartDesc *__restrict__ descs, uint32_t slice, uint32_t part,
                                               uint32_t nsl_grid) {
    __shared__ double s_pr[kPartPruners][D];
    __shared__ uint32_t s_pi[kPartPruners], s_fe[kPartPruners];
    const PartDesc &d = descs[part];
    const uint32_t nb = d.nb, s0 = slice * kPartSlice;
    // the insert's dom_s (per bounded rep) starts here, spread over the part's workgroups
    for (uint32_t r = slice * kThreads + threadIdx.x; r < d.rb; r += nsl_grid * kThreads) d.dom_s[r] = 0u;
    if (s0 >= nb) return;
    const int lane = threadIdx.x & 63;
    const uint32_t nsl = (nb + kPartSlice - 1) / kPartSlice;
    if (threadIdx.x < kPartPruners) {
        const int c = threadIdx.x;
        double v = 0.0;
        uint32_t i = 0xffffffffu;
        for (uint32_t q = 0; q < nsl; q++) vi_min(v, i, d.sl_v[q * kPartPruners + c], d.sl_i[q * kPartPruners + c]);
        s_pi[c] = i;
        s_fe[c] = 0xffffffffu;
        if (slice == 0) d.meta[1 + c] = i;
    }
    __syncthreads();
    if (threadIdx.x < kPartPruners * D) {
        const int c = threadIdx.x / D, q = threadIdx.x % D;
        s_pr[c][q] = s_pi[c] != 0xffffffffu ? d.bvals[(size_t)s_pi[c] * D + q] : 0.0;
    }
    double rv[kSliceIt][D];
#pragma unroll
    for (int k = 0; k < kSliceIt; k++) {
        const uint32_t b = min(s0 + k * kThreads + threadIdx.x, nb - 1u);
#pragma unroll
        for (int q = 0; q < D; q++) rv[k][q] = d.bvals[(size_t)b * D + q];
    }
    __syncthreads();
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int k = 0; k < kSliceIt; k++) {
        const uint32_t b = s0 + k * kThreads + threadIdx.x;
        const bool valid = b < nb;
        uint32_t cls = 0xffffffffu;
        bool dom = false;
        if (valid) {
            for (int c = 0; c < kPartPruners; c++) {
                if (s_pi[c] == 0xffffffffu) break;
                bool le = true, ge = true;
#pragma unroll
                for (int q = 0; q < D; q++) {
                    le &= s_pr[c][q] <= rv[k][q];
                    ge &= s_pr[c][q] >= rv[k][q];
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
            d.dom_b[b] = dom ? 1u : 0u;
            d.eq_s[b] = 0xffffffffu;
            d.eq_b[b] = 0xffffffffu;
            d.eqp[b] = cls;
            if (cls != 0xffffffffu) atomicMin(&s_fe[cls], b);
        }
        const bool inU = valid && !dom && (cls == 0xffffffffu || b == s_pi[cls]);
        const uint64_t um = __ballot(inU);
        uint32_t base = 0;
        if (lane == 0 && um) base = atomicAdd(&d.meta[0], (uint32_t)__popcll(um));
        base = (uint32_t)__shfl((int)base, 0, 64);
        if (inU) d.uidx[base + (uint32_t)__popcll(um & lt)] = b;
    }
    __syncthreads();
    if (threadIdx.x < kPartPruners && s_fe[threadIdx.x] != 0xffffffffu)
        atomicMin(&d.meta[1 + kPartPruners + threadIdx.x], s_fe[threadIdx.x]);
}
template <int D>
__global__ __launch_bounds__(kThreads) void k_parts_classify(const PartDesc *__restrict__ descs) {
    parts_classify<D>(descs, blockIdx.x, blockIdx.y, gridDim.x);
}

// dominance as ServiceTuple.dominates (ServiceTuple.java:67-77): <= everywhere, < somewhere
// mode 0: undecided y vs undecided x (dom_b, eq_b: first EARLIER equal batch tuple)
// mode 1: undecided y vs alive state reps x (dom_b, eq_s: first equal rep)
// mode 2: state reps y vs undecided x (dom_s)
// Launch sizes come from the batch size (a bound of |U|, which lives on the device): work items
// past |U| return at once.
template <int D>
__device__ __forceinline__ void parts_pairs(const PartDesc *__restrict__ descs, const PartItem *__restrict__ items,
                                            uint32_t item) {
    __shared__ double s_x[kPartX * D];
    __shared__ uint32_t s_xi[kPartX];
    const PartItem it = items[item];
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
template <int D>
__global__ __launch_bounds__(kThreads) void k_parts_pairs(const PartDesc *__restrict__ descs,
                                                          const PartItem *__restrict__ items) {
    parts_pairs<D>(descs, items, blockIdx.x);
}

// Ka: per slice, the pruner classes resolved (a class member takes the fate of its pruner, same
// vector; the class's first index is its equal-earlier tuple), kept / new-rep counts; and the
// state reps the batch dominates die (no kept tuple joins a dying rep: its dominator dominates
// every tuple equal to it), their tuples counted dead
template <int D>
__device__ __forceinline__ void parts_count(const PartDesc *__restrict__ descs, uint32_t slice, uint32_t part,
                                               uint32_t nsl_grid) {
    __shared__ uint32_t s_k[kThreads / 64], s_f[kThreads / 64];
    const PartDesc &d = descs[part];
    const uint32_t nb = d.nb, s0 = slice * kPartSlice;
    const uint32_t R0 = d.dcnt[0];
    {
        uint32_t killed = 0;
        const uint32_t rs = min(R0, d.rb);
        for (uint32_t r = slice * kThreads + threadIdx.x; r < rs; r += nsl_grid * kThreads)
            if (d.dom_s[r] && d.ralive[r]) {
                d.ralive[r] = 0;
                killed += d.rcnt[r];
            }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) killed += (uint32_t)__shfl_xor((int)killed, o, 64);
        if ((threadIdx.x & 63) == 0 && killed) atomicAdd(&d.meta[2 + 2 * kPartPruners], killed);
    }
    if (s0 >= nb) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t db[kSliceIt], es[kSliceIt], eb[kSliceIt], cp[kSliceIt];
#pragma unroll
    for (int k = 0; k < kSliceIt; k++) {
        const uint32_t b = min(s0 + k * kThreads + threadIdx.x, nb - 1u);
        db[k] = d.dom_b[b];
        es[k] = d.eq_s[b];
        eb[k] = d.eq_b[b];
        cp[k] = d.eqp[b];
    }
    uint32_t nk = 0, nf = 0;
#pragma unroll
    for (int k = 0; k < kSliceIt; k++) {
        const uint32_t b = s0 + k * kThreads + threadIdx.x;
        if (b >= nb) continue;
        if (cp[k] != 0xffffffffu) {
            const uint32_t r = d.meta[1 + cp[k]], fe = d.meta[1 + kPartPruners + cp[k]];
            if (b != r) {
                db[k] = d.dom_b[r];
                es[k] = d.eq_s[r];
                d.dom_b[b] = db[k];
                d.eq_s[b] = es[k];
            }
            eb[k] = fe < b ? fe : 0xffffffffu;
            d.eq_b[b] = eb[k];
        }
        const bool keep = db[k] == 0u;
        nk += keep ? 1u : 0u;
        nf += keep && es[k] == 0xffffffffu && eb[k] == 0xffffffffu ? 1u : 0u;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        nk += (uint32_t)__shfl_xor((int)nk, o, 64);
        nf += (uint32_t)__shfl_xor((int)nf, o, 64);
    }
    if (lane == 0) {
        s_k[wave] = nk;
        s_f[wave] = nf;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tk = 0, tf = 0;
        for (int w = 0; w < kThreads / 64; w++) {
            tk += s_k[w];
            tf += s_f[w];
        }
        d.sl_k[slice] = tk;
        d.sl_k[slice + ((nb + kPartSlice - 1) / kPartSlice)] = tf;
    }
}
template <int D>
__global__ __launch_bounds__(kThreads) void k_parts_count(const PartDesc *__restrict__ descs) {
    parts_count<D>(descs, blockIdx.x, blockIdx.y, gridDim.x);
}

// Kb: positions (the slices before this one, then ballots) of the kept tuples and the new reps;
// the new reps' rows appended
template <int D>
__device__ __forceinline__ void parts_place(const PartDesc *__restrict__ descs, uint32_t slice, uint32_t part,
                                               uint32_t nsl_grid) {
    __shared__ uint32_t s_kc[kSliceIt][kThreads / 64], s_fc[kSliceIt][kThreads / 64];
    const PartDesc &d = descs[part];
    const uint32_t nb = d.nb, s0 = slice * kPartSlice;
    if (s0 >= nb) return;
    const uint32_t R0 = d.dcnt[0];
    const uint32_t nsl = (nb + kPartSlice - 1) / kPartSlice;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint32_t ko = 0, fo = 0;
    for (uint32_t q = 0; q < slice; q++) {
        ko += d.sl_k[q];
        fo += d.sl_k[nsl + q];
    }
    uint64_t km[kSliceIt], fm[kSliceIt];
#pragma unroll
    for (int k = 0; k < kSliceIt; k++) {
        const uint32_t b = min(s0 + k * kThreads + threadIdx.x, nb - 1u);
        const bool valid = s0 + k * kThreads + threadIdx.x < nb;
        const bool keep = valid && d.dom_b[b] == 0u;
        const bool fresh = keep && d.eq_s[b] == 0xffffffffu && d.eq_b[b] == 0xffffffffu;
        km[k] = __ballot(keep);
        fm[k] = __ballot(fresh);
        if (lane == 0) {
            s_kc[k][wave] = (uint32_t)__popcll(km[k]);
            s_fc[k][wave] = (uint32_t)__popcll(fm[k]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSliceIt; k++) {
        uint32_t kw = 0, fw = 0, kt = 0, ft = 0;
#pragma unroll
        for (int w = 0; w < kThreads / 64; w++) {
            kw += w < wave ? s_kc[k][w] : 0u;
            fw += w < wave ? s_fc[k][w] : 0u;
            kt += s_kc[k][w];
            ft += s_fc[k][w];
        }
        const uint32_t b = s0 + k * kThreads + threadIdx.x;
        if ((km[k] >> lane) & 1ull) d.kpos[b] = ko + kw + (uint32_t)__popcll(km[k] & lt);
        if ((fm[k] >> lane) & 1ull) {
            const uint32_t fp = fo + fw + (uint32_t)__popcll(fm[k] & lt);
            d.fpos[b] = fp;
            const uint32_t r = R0 + fp;
#pragma unroll
            for (int q = 0; q < D; q++) d.rrows[(size_t)r * D + q] = d.bvals[(size_t)b * D + q];
            d.ralive[r] = 1;
            d.rcnt[r] = 0;
        }
        ko += kt;
        fo += ft;
    }
}
template <int D>
__global__ __launch_bounds__(kThreads) void k_parts_place(const PartDesc *__restrict__ descs) {
    parts_place<D>(descs, blockIdx.x, blockIdx.y, gridDim.x);
}

// Kc: the kept tuples appended (id, rep) at their positions, the tuples joining a rep counted
// (duplicate-heavy keys: one atomic per wave); the part's last slice to finish (a ticket)
// writes the new counts to the device and to the host mirror
template <int D>
__device__ __forceinline__ void parts_join(const PartDesc *__restrict__ descs, uint32_t slice, uint32_t part,
                                               uint32_t nsl_grid) {
    __shared__ bool s_last;
    const PartDesc &d = descs[part];
    const uint32_t nb = d.nb, s0 = slice * kPartSlice;
    if (s0 >= nb) return;
    const uint32_t R0 = d.dcnt[0], T0 = d.dcnt[1];
    const int lane = threadIdx.x & 63;
    uint32_t db[kSliceIt], es[kSliceIt], eb[kSliceIt], kp[kSliceIt];
#pragma unroll
    for (int k = 0; k < kSliceIt; k++) {
        const uint32_t b = min(s0 + k * kThreads + threadIdx.x, nb - 1u);
        db[k] = s0 + k * kThreads + threadIdx.x < nb ? d.dom_b[b] : 1u;
        es[k] = d.eq_s[b];
        eb[k] = d.eq_b[b];
        kp[k] = d.kpos[b];
    }
#pragma unroll
    for (int k = 0; k < kSliceIt; k++) {
        const uint32_t b = s0 + k * kThreads + threadIdx.x;
        const bool act = db[k] == 0u;
        uint32_t rep = 0xffffffffu;
        if (act) {
            rep = es[k] != 0xffffffffu ? es[k] : R0 + d.fpos[eb[k] != 0xffffffffu ? eb[k] : b];
            const uint32_t t = T0 + kp[k];
            d.tids[t] = d.bids[b];
            d.trep[t] = rep;
        }
        const uint64_t am = __ballot(act);
        if (am) {
            const int leader = __ffsll((unsigned long long)am) - 1;
            const uint32_t r0 = (uint32_t)__shfl((int)rep, leader, 64);
            const bool uni = __ballot(act && rep != r0) == 0ull;
            if (uni) {
                if (lane == leader) atomicAdd(&d.rcnt[r0], (uint32_t)__popcll(am));
            } else if (act) {
                atomicAdd(&d.rcnt[rep], 1u);
            }
        }
    }
    // the last slice of the part: every slice has read the old counts by now
    __syncthreads();
    const uint32_t nsl = (nb + kPartSlice - 1) / kPartSlice;
    if (threadIdx.x == 0) s_last = atomicAdd(&d.meta[3 + 2 * kPartPruners], 1u) == nsl - 1u;
    __syncthreads();
    if (!s_last || threadIdx.x != 0) return;
    uint32_t tk = 0, tf = 0;
    for (uint32_t q = 0; q < nsl; q++) {
        tk += d.sl_k[q];
        tf += d.sl_k[nsl + q];
    }
    const uint32_t R1 = R0 + tf, T1 = T0 + tk;
    const unsigned long long dead = ((unsigned long long)d.dcnt[3] << 32 | d.dcnt[2]) +
                                    d.meta[2 + 2 * kPartPruners];
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
template <int D>
__global__ __launch_bounds__(kThreads) void k_parts_join(const PartDesc *__restrict__ descs) {
    parts_join<D>(descs, blockIdx.x, blockIdx.y, gridDim.x);
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

// ---- the global merge of device-resident per-key states (sky_parts_global_merge) -----------
// GlobalSkylineAggregator (FlinkSkyline.java:515-569) over the keys' local skylines without
// moving them through host memory: the alive reps of every part (origin = list index, weight =
// tuples on the rep) run through the single-partition pipeline; the surviving reps are flagged,
// and every part's tuples (list order, then insertion order) whose rep survives are written.
__global__ __launch_bounds__(kThreads) void k_pgm_prep(uint32_t R, const uint32_t *__restrict__ rcnt, int32_t k,
                                                       int32_t *__restrict__ origin, int64_t *__restrict__ w) {
    const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
    if (r >= R) return;
    origin[r] = k;
    w[r] = (int64_t)rcnt[r];
}
__global__ __launch_bounds__(kThreads) void k_pgm_flags(uint32_t n, const int64_t *__restrict__ surv_idx,
                                                        uint8_t *__restrict__ flag) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    flag[surv_idx[i]] = 1;
}
// per tuple of the concatenated lists: its rep survives?
// (a caller-given rep index past its list's rep count -- sky_global_merge_reps -- selects nothing
// and sets *err)
__global__ __launch_bounds__(kThreads) void k_pgm_tflag(const PgmList *__restrict__ lists, int nl, uint32_t ttot,
                                                        const uint8_t *__restrict__ flag,
                                                        uint32_t *__restrict__ tsel, uint32_t *__restrict__ err) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= ttot) return;
    int lo = 0, hi = nl - 1;                   // the list holding tuple i (toff ascending)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (lists[mid].toff <= i) lo = mid;
        else hi = mid - 1;
    }
    const PgmList &L = lists[lo];
    const uint32_t r = L.trep[i - L.toff];
    if (r >= L.nrep) {
        tsel[i] = 0u;
        *err = 1u;
        return;
    }
    tsel[i] = flag[L.roff + r] ? 1u : 0u;
}
__global__ __launch_bounds__(kThreads) void k_pgm_write(const PgmList *__restrict__ lists, int nl, uint32_t ttot,
                                                        const uint32_t *__restrict__ tsel,
                                                        const uint32_t *__restrict__ tpos, int64_t *__restrict__ ids_out,
                                                        int32_t *__restrict__ org_out) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= ttot || !tsel[i]) return;
    int lo = 0, hi = nl - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (lists[mid].toff <= i) lo = mid;
        else hi = mid - 1;
    }
    const PgmList &L = lists[lo];
    const uint32_t o = tpos[i];
    ids_out[o] = L.tids[i - L.toff];
    org_out[o] = L.part_id;
}

void launch_pgm_prep(uint32_t R, const uint32_t *rcnt, int32_t k, int32_t *origin, int64_t *w, hipStream_t st) {
    if (R) k_pgm_prep<<<(R + kThreads - 1) / kThreads, kThreads, 0, st>>>(R, rcnt, k, origin, w);
}
void launch_pgm_flags(uint32_t n, const int64_t *surv_idx, uint8_t *flag, hipStream_t st) {
    if (n) k_pgm_flags<<<(n + kThreads - 1) / kThreads, kThreads, 0, st>>>(n, surv_idx, flag);
}
void launch_pgm_tuples(const PgmList *lists, int nl, uint32_t ttot, const uint8_t *flag, uint32_t *tsel,
                       uint32_t *tpos, uint32_t *d_total, uint32_t *scratch, int64_t *ids_out, int32_t *org_out,
                       uint32_t *err, hipStream_t st) {
    if (!ttot) return;
    const unsigned g = (ttot + kThreads - 1) / kThreads;
    k_pgm_tflag<<<g, kThreads, 0, st>>>(lists, nl, ttot, flag, tsel, err);
    scan_excl_u32(tsel, tpos, ttot, d_total, scratch, st);
    k_pgm_write<<<g, kThreads, 0, st>>>(lists, nl, ttot, tsel, tpos, ids_out, org_out);
}

void launch_parts_insert(int D, const PartDesc *descs, int nparts, uint32_t max_slices, const PartItem *items,
                         uint32_t nitems, hipStream_t st) {
    if (!nparts || !max_slices) return;
    const dim3 g(max_slices, (unsigned)nparts);
    SKY_DISPATCH_D(D, (k_parts_crit<DD><<<g, kThreads, 0, st>>>(descs)));
    SKY_DISPATCH_D(D, (k_parts_classify<DD><<<g, kThreads, 0, st>>>(descs)));
    if (nitems) SKY_DISPATCH_D(D, (k_parts_pairs<DD><<<nitems, kThreads, 0, st>>>(descs, items)));
    SKY_DISPATCH_D(D, (k_parts_count<DD><<<g, kThreads, 0, st>>>(descs)));
    SKY_DISPATCH_D(D, (k_parts_place<DD><<<g, kThreads, 0, st>>>(descs)));
    SKY_DISPATCH_D(D, (k_parts_join<DD><<<g, kThreads, 0, st>>>(descs)));
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
