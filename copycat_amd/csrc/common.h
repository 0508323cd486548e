// common.h — shared device/host definitions of the MI355X commit-apply engine (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/copycat_apply.h"

namespace cc {

// ---- geometry -----------------------------------------------------------------------------------------
constexpr int kWave = 64;                 // CDNA wavefront
constexpr int kResPerBucket = 64;         // one apply wave owns 64 resource slots (lane = slot % 64)
constexpr int kBucketShift = 6;
constexpr int kMaxBuckets = 4096;         // => max_resources <= 262144
constexpr int kPartWaves = 4;             // partition workgroup = 4 waves
constexpr int kPartThreads = kPartWaves * kWave;
constexpr int kWaveTile = 4096;           // commits per wave per partition tile
constexpr int kTile = kPartWaves * kWaveTile;  // 16384 commits per partition tile
constexpr int kScanGroups = 16;           // row groups of the tile-prefix scan (1024-thread WG)
constexpr uint32_t kNoRes = 0xFFFFFFFFu;

// device error bits (d_err)
constexpr uint32_t kErrUnsupported = 1u;
constexpr uint32_t kErrEvents = 2u;

// staging record meta word: pos(32) | op(8) | flags(8) | lane(6)
__host__ __device__ inline uint64_t pack_meta(uint32_t pos, uint32_t op, uint32_t flags, uint32_t lane) {
  return (uint64_t)pos | ((uint64_t)(op & 0xFF) << 32) | ((uint64_t)(flags & 0xFF) << 40) | ((uint64_t)(lane & 63) << 48);
}
__host__ __device__ inline uint32_t meta_pos(uint64_t m) { return (uint32_t)m; }
__host__ __device__ inline uint32_t meta_op(uint64_t m) { return (uint32_t)(m >> 32) & 0xFF; }
__host__ __device__ inline uint32_t meta_flags(uint64_t m) { return (uint32_t)(m >> 40) & 0xFF; }
__host__ __device__ inline uint32_t meta_lane(uint64_t m) { return (uint32_t)(m >> 48) & 63; }

struct alignas(16) u64x2 {
  uint64_t x, y;
};

// AtomicValueState per slot: meta = tag | (has_current << 8); value payload separately.
__host__ __device__ inline uint32_t vmeta(uint32_t tag, uint32_t cur) { return (tag & 0xFF) | ((cur & 1) << 8); }

__device__ inline uint32_t lane_id() { return __lane_id(); }
__device__ inline uint64_t lanemask_lt() {
  const uint32_t l = __lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}
__device__ inline uint64_t ballot(bool p) { return __ballot(p); }

// ---- ops registered per resource type (ResourceStateMachine.init + Copycat reflection configure) -----
__host__ __device__ inline bool op_registered(uint32_t type, uint32_t op) {
  if (op == CC_OP_DELETE) return type != CC_RES_NONE;
  switch (type) {
    case CC_RES_VALUE: return op >= 50 && op <= 55;
    case CC_RES_MAP: return op >= 60 && op <= 72;
    case CC_RES_LOCK: return op == 115 || op == 116;
    case CC_RES_ELECTION: return op >= 110 && op <= 112;
    case CC_RES_GROUP: return op >= 120 && op <= 123;
  }
  return false;
}
// ops this build applies on the GPU (others raise CC_ERR_UNSUPPORTED for the batch)
__host__ __device__ inline bool op_on_gpu(uint32_t type, uint32_t op) {
  if (type == CC_RES_VALUE) return op == CC_OP_DELETE || (op >= 50 && op <= 53);
  return false;
}

}  // namespace cc
