// engine_internal.h — launch-parameter structs shared by the engine's translation units.
#pragma once
#include "common.h"

namespace cc {

// Optional per-kernel timing (HIP events recorded on the launch stream around each kernel).
enum KernelId { K_PART_COUNT = 0, K_PART_SCAN, K_PART_BASE, K_PART_SCATTER, K_APPLY_VALUE, K_NUM };
struct Marker {
  void (*fn)(void* ctx, int kernel, int begin, hipStream_t st);
  void* ctx;
  void operator()(int k, int begin, hipStream_t st) const {
    if (fn) fn(ctx, k, begin, st);
  }
};

// One sub-batch [lo, n) of a batch (absolute row indices; column and output pointers are whole-batch).
struct PartArgs {
  const uint32_t* inst;
  const uint8_t* op;
  const uint8_t* flags;
  const uint64_t* a;
  const uint64_t* b;
  uint64_t lo, n;
  const uint32_t* inst_res;
  uint32_t max_inst;
  uint32_t nb, nbits;
  uint32_t* counts;  // [tiles][nb]
  uint32_t* tot;     // [nb]
  uint32_t* base;    // [nb]
  uint64_t* st_meta;
  u64x2* st_ab;
  uint8_t* out_status;
  uint64_t* out_value;
  Marker mark;
};
int launch_partition(const PartArgs& a, hipStream_t st);

struct ValueArgs {
  const uint64_t* st_meta;
  const u64x2* st_ab;
  const uint32_t* base;
  const uint32_t* tot;
  uint32_t nb;
  uint32_t* val_meta;   // [nb*64]
  uint64_t* val_v;      // [nb*64]
  uint8_t* out_status;  // offset to the sub-batch start
  uint64_t* out_value;
  uint32_t* err;
  Marker mark;
};
int launch_apply_value(const ValueArgs& a, hipStream_t st);

}  // namespace cc
