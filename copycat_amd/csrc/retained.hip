// retained.hip — the bulk compaction view (cc_retained_bitmap): every log index some state machine still holds
// without clean(), as a bitmap over a log range, built on the device from the engine's state in one pass per
// structure.  The union over all resource slots of cc_read_retained (engine.hip), which follows the reference's clean
// sites: AtomicValueState `current` + listeners (AtomicValueState.java:41-63,88-157), MapState / SetState entries
// (MapState.java:89-228: replaced, removed and expired entries are cleaned), LockState holder unless delete() cleaned
// it + waiters whose timeout has not fired (LockState.java:41-98), LeaderElectionState leader + listeners
// (LeaderElectionState.java:35-108), MembershipGroupState members (MembershipGroupState.java:47-81), QueueState
// elements less a head element() cleaned (QueueState.java:51-199); the host adds pending group schedules and the
// commits dropped without clean() (leak lists; ResourceManagerCommit.clean :79-81 is never called for them).
#include "common.h"
#include "engine_internal.h"

namespace cc {

__device__ inline void ret_mark(uint64_t idx, uint64_t first, uint64_t count, unsigned long long* bm) {
  const uint64_t d = idx - first;  // idx < first wraps above count
  if (idx >= first && d < count) atomicOr(bm + (d >> 6), 1ull << (d & 63));
}

// value slots: the retained `current` (live.hip post-pass, CC_CFG_VALUE_RETAINED)
__global__ void k_ret_value(const uint8_t* __restrict__ res_type, const uint64_t* __restrict__ val_live, uint32_t slots,
                            uint64_t first, uint64_t count, unsigned long long* __restrict__ bm) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < slots && res_type[s] == CC_RES_VALUE && val_live[s]) ret_mark(val_live[s], first, count, bm);
}

// map / set table entries: used, present, not of a deleted map, timer not due at the engine clock
__global__ void k_ret_map(const uint32_t* __restrict__ word, const uint64_t* __restrict__ ci, const uint64_t* __restrict__ dl,
                          const uint64_t* __restrict__ clock, uint64_t entries, uint64_t first, uint64_t count,
                          unsigned long long* __restrict__ bm) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= entries) return;
  const uint32_t w = word[i];
  if (!(w & kMwUsed) || !(w & kMwPresent) || (w & kMwDead)) return;
  if (dl && dl[i] && dl[i] <= *clock) return;
  ret_mark(ci[i], first, count, bm);
}

// coordination blocks: one wave per slot, lanes over the block's entries
__global__ void k_ret_coord(const uint8_t* __restrict__ res_type, const uint8_t* __restrict__ coord, uint32_t ccap,
                            uint32_t slots, const uint64_t* __restrict__ clock, uint64_t first, uint64_t count,
                            unsigned long long* __restrict__ bm) {
  const uint32_t s = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave), l = threadIdx.x & 63;
  if (s >= slots) return;
  const uint32_t type = res_type[s];
  if (type != CC_RES_VALUE && type != CC_RES_LOCK && type != CC_RES_ELECTION && type != CC_RES_GROUP && type != CC_RES_QUEUE)
    return;
  const uint8_t* blk = coord + (uint64_t)s * coord_block(ccap);
  const CoordHdr h = *reinterpret_cast<const CoordHdr*>(blk);
  const CoordEnt* q = reinterpret_cast<const CoordEnt*>(blk + sizeof(CoordHdr));
  const uint64_t clk = *clock;
  if (l == 0 && (type == CC_RES_LOCK || type == CC_RES_ELECTION) && (h.flags & kCoHeld) && !(h.flags & kCoCleaned))
    ret_mark(h.idx, first, count, bm);  // the holder / leader commit
  const bool ring = type == CC_RES_LOCK || type == CC_RES_QUEUE;
  for (uint32_t i = l; i < h.n && i < ccap; i += kWave) {
    const CoordEnt& x = q[ring ? ((h.head + i) & (ccap - 1)) : i];
    if (type == CC_RES_LOCK && x.x != kNoDeadline && x.x <= clk) continue;  // tryLock timeout fired: cleaned
    if (type == CC_RES_QUEUE && (x.pad & kQCleaned)) continue;            // head element() cleaned in place
    ret_mark(x.idx, first, count, bm);
  }
}

// host-known indices (pending group schedules, leak lists)
__global__ void k_ret_list(const uint64_t* __restrict__ idx, uint64_t n, uint64_t first, uint64_t count,
                           unsigned long long* __restrict__ bm) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ret_mark(idx[i], first, count, bm);
}

__global__ void k_ret_popc(const unsigned long long* __restrict__ bm, uint64_t words, unsigned long long* __restrict__ out) {
  uint64_t c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x)
    c += (uint64_t)__popcll(bm[i]);
  for (int d = 32; d; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, (unsigned long long)c);
}

int launch_retained(const RetainedArgs& a, hipStream_t st) {
  const uint64_t words = (a.count + 63) / 64;
  unsigned long long* bm = reinterpret_cast<unsigned long long*>(a.bitmap);
  if (hipMemsetAsync(bm, 0, words * 8, st) != hipSuccess) return -1;
  if (a.val_live)
    hipLaunchKernelGGL(k_ret_value, dim3((a.slots + 255) / 256), dim3(256), 0, st, a.res_type, a.val_live, a.slots, a.first,
                       a.count, bm);
  if (a.tbl_word)
    hipLaunchKernelGGL(k_ret_map, dim3((unsigned)((a.entries + 255) / 256)), dim3(256), 0, st, a.tbl_word, a.tbl_ci,
                       a.tbl_dl, a.clock, a.entries, a.first, a.count, bm);
  if (a.coord)
    hipLaunchKernelGGL(k_ret_coord, dim3((a.slots + 3) / 4), dim3(256), 0, st, a.res_type, a.coord, a.coord_cap, a.slots,
                       a.clock, a.first, a.count, bm);
  if (a.list_n)
    hipLaunchKernelGGL(k_ret_list, dim3((unsigned)((a.list_n + 255) / 256)), dim3(256), 0, st, a.list, a.list_n, a.first,
                       a.count, bm);
  if (a.total) {
    if (hipMemsetAsync(a.total, 0, 8, st) != hipSuccess) return -1;
    const uint64_t blocks = std::min<uint64_t>((words + 255) / 256, 1024);
    hipLaunchKernelGGL(k_ret_popc, dim3((unsigned)std::max<uint64_t>(blocks, 1)), dim3(256), 0, st, bm, words, a.total);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
