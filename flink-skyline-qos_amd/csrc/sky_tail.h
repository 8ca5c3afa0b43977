// sky_tail.h -- the brute route's output counts, their scan, the stats and the final read in one
// workgroup (k_sfs.hip k_tail_counts).  Host-side declarations, not part of the C ABI.
#pragma once
#include "sky_internal.h"

namespace sky {

struct TailArgs {
    const uint32_t *tile_hist = nullptr;       // [tiles][KM] duplicates per tile
    const uint32_t *tile_cand = nullptr;       // [tiles] candidates in G per tile (k_fate_tables)
    const uint8_t *pruner_fate = nullptr;      // [KM]
    int KM = 0, K = 1, Kp = 1;
    uint32_t ntiles = 0;
    uint32_t *out_cnt = nullptr, *out_off = nullptr;
    uint32_t *totals = nullptr;                // [3] out: the output total
    const unsigned long long *lsz = nullptr, *surv = nullptr;   // [kStatShards][K]
    unsigned long long *statk = nullptr;       // [2K] out
    const uint32_t *segalive = nullptr, *segn = nullptr, *flags = nullptr, *dup_cnt = nullptr;
    uint32_t *pin = nullptr;                   // host-mapped: the final read (tiny_pin_layout)
    uint32_t pin_off[5] = {};
};
// k_out_hist_count + the tile scan + k_stat_reduce + the final read's gather, one launch
void launch_tail_counts(const TailArgs &a, hipStream_t st);

}  // namespace sky
