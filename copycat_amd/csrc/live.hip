// Retained value commits (the compaction side of Commit.clean()), CC_CFG_VALUE_RETAINED.
//
// AtomicValueState keeps exactly one commit alive: `current`, the last successful set / compareAndSet /
// getAndSet (AtomicValueState.java:88-118,123-133,138-144); every other value commit is cleaned or closed by
// the time its successor applies, and delete() cleans `current` (:146-157).  So after a batch the retained
// commit of a value slot is: none if the slot has no current (val_meta bit 8, cleared by Delete), else the
// batch's last successful writer on that slot, else the retained commit from before the batch.
//   k_live_mark : per row, atomicMax(row + 1) into wrow[slot] for successful writers (one pass, 7 B/row + the
//                 inst_res / res_type gathers; CAS rows also read their 8 B result).
//   k_live_fold : per value slot, resolve wrow against has_current and index[], then clear wrow.
#include "engine_internal.h"

namespace cc {

__global__ void k_live_mark(const uint32_t* __restrict__ inst, const uint8_t* __restrict__ op,
                            const uint8_t* __restrict__ status, const uint64_t* __restrict__ value, uint64_t n,
                            const uint32_t* __restrict__ inst_res, const uint8_t* __restrict__ res_type,
                            uint32_t max_inst, unsigned long long* __restrict__ wrow) {
  // Rows are walked from the end of the batch (grid-stride, descending) and a slot whose recorded row is already
  // later is skipped with a plain load: wrow only grows, so a stale (cached) read can only under-state it and a skip
  // is always safe.  After the first sweep nearly every slot holds a late row, so few rows reach the atomic.
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = n - 1 - k;
    const uint8_t o = op[i];
    if (o != CC_OP_VALUE_SET && o != CC_OP_VALUE_CAS && o != CC_OP_VALUE_GETANDSET) continue;
    if (CC_STATUS_CODE(status[i]) != CC_ST_OK) continue;
    if (o == CC_OP_VALUE_CAS && value[i] != 1) continue;  // compareAndSet returned false: commit.clean()
    const uint32_t in = inst[i];
    if (in >= max_inst) continue;
    const uint32_t s = inst_res[in];
    if (s == kNoRes || res_type[s] != CC_RES_VALUE) continue;
    if (__builtin_nontemporal_load(&wrow[s]) > i) continue;
    atomicMax(&wrow[s], (unsigned long long)(i + 1));
  }
}

__global__ void k_live_fold(const uint64_t* __restrict__ index, const uint32_t* __restrict__ val_meta,
                            const uint8_t* __restrict__ res_type, uint32_t slots,
                            unsigned long long* __restrict__ wrow, uint64_t* __restrict__ live) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= slots) return;
  const unsigned long long w = wrow[s];
  if (res_type[s] != CC_RES_VALUE) {
    live[s] = 0;
  } else if (!((val_meta[s] >> 8) & 1)) {
    live[s] = 0;  // no current: deleted after its last writer (or never written)
  } else if (w) {
    live[s] = index[w - 1];
  }
  if (w) wrow[s] = 0;
}

int launch_value_live(const uint32_t* inst, const uint8_t* op, const uint8_t* status, const uint64_t* value,
                      const uint64_t* index, uint64_t n, const uint32_t* inst_res, const uint8_t* res_type,
                      uint32_t max_inst, const uint32_t* val_meta, uint32_t slots, unsigned long long* wrow,
                      uint64_t* live, hipStream_t st) {
  const uint64_t want = (n + 255) / 256;
  const uint32_t blocks = (uint32_t)(want < 8192 ? (want ? want : 1) : 8192);
  hipLaunchKernelGGL(k_live_mark, dim3(blocks), dim3(256), 0, st, inst, op, status, value, n, inst_res, res_type,
                     max_inst, wrow);
  hipLaunchKernelGGL(k_live_fold, dim3((slots + 255) / 256), dim3(256), 0, st, index, val_meta, res_type, slots, wrow,
                     live);
  return hipGetLastError() != hipSuccess;
}

}  // namespace cc
