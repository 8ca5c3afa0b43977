// sky_common.h — constants shared by host orchestration and gfx950 kernels.
#pragma once
#include <stdint.h>
#include "../../include/skyline_hip.h"

namespace sky {

constexpr int kMaxD = SKY_MAX_DIMS;
constexpr int kMaxK = SKY_MAX_PARTITIONS;
constexpr int kThreads = 256;                 // 4 waves of 64
constexpr int kItems = 8;                     // tuples per thread per tile
constexpr int kTile = kThreads * kItems;      // 2048 tuples per workgroup tile
constexpr int kStatShards = 1024;             // |L_k| / survivors_k accumulators are [shard][K], reduced on device

// per-tuple status word (u16): high byte = partition key, low byte = code
constexpr uint16_t kCodeDropped = 0;          // dominated by a pruner / key never queried
constexpr uint16_t kCodeCandidate = 255;      // goes to sort + SFS
constexpr uint16_t kCodeFate0 = 251;          // candidate after the fate pass: 251 + (inL | inG << 1)
constexpr uint16_t kCodeDeferred = 250;       // MR-Angle key left to k_filter_deferred (rewritten there)
// codes 1..254: exact duplicate of pruner (code-1) of its partition

// flag bits (device u32)
constexpr uint32_t kFlagNotF32 = 1u;          // some candidate value is not exactly an f32
constexpr uint32_t kFlagNaN = 2u;             // a NaN was seen
constexpr uint32_t kFlagScoreTies = 4u;       // score key is not strictly monotone
constexpr uint32_t kFlagRadixSpin = 16u;      // a radix look-back hit its spin bound (result invalid)
constexpr uint32_t kFlagNotU16 = 8u;          // some candidate value is not an integer in [0, 65535]
constexpr uint32_t kFlagMbrQueue = 32u;       // the pair pass's work items outgrew their queue (no pass ran: invalid)

// padded row width in elements so every row starts 16-byte aligned
template <typename T>
constexpr int padded_dims(int D) { return sizeof(T) == 4 ? (D + 3) & ~3 : (D + 1) & ~1; }

}  // namespace sky
