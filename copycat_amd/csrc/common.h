// common.h — shared device/host definitions of the MI355X commit-apply engine (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/copycat_apply.h"

namespace cc {

// ---- geometry -----------------------------------------------------------------------------------------
constexpr int kWave = 64;                 // CDNA wavefront
constexpr int kLaneRes = 64;              // an apply wave owns 64 resource slots (lane = slot % 64)
constexpr int kApplyWaves = 4;            // apply workgroup = 4 waves = one super-bucket of 256 slots
constexpr int kSbShift = 8;               // super-bucket = slot >> 8
constexpr int kMaxSb = 512;               // => max_resources <= 131072 with 256-slot super-buckets
constexpr int kPT = 1024;                 // partition workgroup threads (16 waves)
constexpr int kPW = kPT / kWave;
constexpr int kTile = 16384;              // commits per partition tile (one workgroup)
constexpr int kChunk = 4096;              // commits per LDS-staged chunk of a tile
constexpr int kScanGroups = 16;           // row groups of the tile-prefix scan (1024-thread WG)
constexpr int kApplyPer = 8;              // staging records per apply thread per chunk (prefetch depth)
constexpr int kMaxTiles = 1024;           // tiles per sub-batch => sub-batch <= 16M commits
constexpr uint32_t kNoRes = 0xFFFFFFFFu;

// device error bits (d_err)
constexpr uint32_t kErrUnsupported = 1u;
constexpr uint32_t kErrEvents = 2u;

// staging record meta word (u32): op(8) | flags(8) | slot-within-super-bucket(<=10 bits) << 16
__host__ __device__ inline uint32_t smeta_op(uint32_t m) { return m & 0xFF; }
__host__ __device__ inline uint32_t smeta_flags(uint32_t m) { return (m >> 8) & 0xFF; }
__host__ __device__ inline uint32_t smeta_slot(uint32_t m) { return m >> 16; }

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

// Workgroup barrier that orders LDS only.  __syncthreads() also drains every outstanding global load and
// store of the wave (s_waitcnt vmcnt(0)), which would kill the cross-chunk prefetches the streaming kernels
// rely on; none of the engine's kernels exchanges global-memory data between threads of a workgroup.
__device__ inline void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

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
