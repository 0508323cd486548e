// map_clear.hip — MapState.clear applied in the stream, outside TTL mode.
//
// MapState.clear (collections/src/main/java/io/atomix/collections/state/MapState.java:255-274) removes every entry of
// the map (its iterator removes them one by one, cancelling their timers; with no timer the result is an empty map
// whose HashMap keeps its table).  As a barrier (map_wide.hip) a clear ends the segment: a host round trip, a
// partition and a region apply for the rows before it, a scan of the table.  In the stream it is an epoch instead:
//
//   per batch      k_map_barriers lists the map clear rows (common.h ClrCtx); the list is sorted by (map, row) with
//                  per-map offsets (k_clr_keys, k_clr_off);
//   per sub-batch  k_clr_sub flags the maps cleared in the sub-batch (kMfClr) and gives every map its clears before
//                  the sub-batch and within it (at most 127: the host
//                  ends a sub-batch earlier for a map cleared more often); a commit's epoch is the clears of its map
//                  in [lo, row) (k_apply_map, at the top of its chunk: MRec meta bits 25-31 in LDS); a commit whose
//                  epoch differs from the one its entry's state is at (the previous commit of the entry, or the epoch
//                  the entry reached in an earlier chunk) sees the entry absent before it -- the transformer CLEAR.el
//                  of map_ops.h's family (a commit is still one element of the scan); at the end of the launch an
//                  entry whose state predates its map's last clear of the sub-batch is dropped (DEAD, as k_map_drop);
//                  a cleared map's keys are not hot-routed (k_hot_bind);
//   sizes          the flagged maps' insertions / removals are events (k_msize_count; their per-tile counts are left
//                  out of the exact tracking), the clears join them (k_clr_events), and after the sort one wave per map
//                  replays its run forward from the size at the sub-batch start: +1 / -1 / reset to 0, the peak ->
//                  the capacity level (HashMap.resize never shrinks; clear() keeps the table) and its timeline, the
//                  size / isEmpty rows answered on the way (k_clr_replay); a small map's HashMap model is emptied at
//                  the clear (map_small.hip k_small_replay);
//   generation     a cleared map's compacted-key generation moves on after the sub-batch (k_clr_gen: the keys a
//                  compaction dropped at the launch start predate the clears);
//   containsValue  in-stream answers restart their count at a clear (map_cv.hip: events carry the epoch).
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "engine_internal.h"

namespace cc {

// per batch: (map slot << 32 | row) of every in-stream clear row
__global__ void k_clr_keys(const uint32_t* __restrict__ rows, uint32_t n, const uint32_t* __restrict__ inst,
                           const uint32_t* __restrict__ inst_res, uint64_t* __restrict__ keys) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t row = rows[i];
    keys[i] = ((uint64_t)inst_res[inst[row]] << 32) | row;  // (listed through the registry: a map slot)
  }
}
// per batch: off[m] = the first sorted key of map m (m = 0..R)
__global__ void k_clr_off(const uint64_t* __restrict__ keys, uint32_t n, uint32_t R, uint32_t* __restrict__ off) {
  for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m <= R; m += gridDim.x * blockDim.x) {
    uint32_t a = 0, b = n;
    const uint64_t k = (uint64_t)m << 32;
    while (a < b) {
      const uint32_t mid = (a + b) >> 1;
      if (keys[mid] < k) a = mid + 1; else b = mid;
    }
    off[m] = a;
  }
}

int launch_clr_batch(const ClrBatchArgs& a, hipStream_t st) {
  if (a.n == 0) return 0;
  const uint32_t g = std::min<uint32_t>(1024, (a.n + 255) / 256);
  hipLaunchKernelGGL(k_clr_keys, dim3(g), dim3(256), 0, st, a.rows, a.n, a.inst, a.inst_res, a.keys);
  size_t tb = a.temp_bytes;
  if (hipcub::DeviceRadixSort::SortKeys(a.temp, tb, a.keys, a.keys2, (int)a.n, 0, 64, st) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_clr_off, dim3((a.R + 256) / 256), dim3(256), 0, st, a.keys2, a.n, a.R, a.off);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
size_t clr_sort_temp_bytes(uint32_t n) {
  size_t need = 0;
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, need, (uint64_t*)nullptr, (uint64_t*)nullptr, (int)n, 0, 64, (hipStream_t)0);
  return need;
}

// per sub-batch: every map's clears before [lo, hi) and within it
__global__ void k_clr_sub(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ off, uint32_t R, uint64_t lo,
                          uint64_t hi, uint32_t* __restrict__ base, uint8_t* __restrict__ eend, uint8_t* __restrict__ mflag,
                          uint32_t* __restrict__ err) {
  for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < R; m += gridDim.x * blockDim.x) {
    const uint32_t a0 = off[m], b0 = off[m + 1];
    auto lb = [&](uint64_t row) {
      uint32_t a = a0, b = b0;
      const uint64_t k = ((uint64_t)m << 32) | row;
      while (a < b) {
        const uint32_t mid = (a + b) >> 1;
        if (keys[mid] < k) a = mid + 1; else b = mid;
      }
      return a;
    };
    const uint32_t pl = a0 == b0 ? a0 : lb(lo), ph = a0 == b0 ? a0 : lb(hi);
    base[m] = pl - a0;
    if (ph - pl > 127u) atomicOr(err, kErrCapacity);  // (the host cuts sub-batches so that this never holds)
    eend[m] = (uint8_t)min(ph - pl, 127u);
    // kMfClr marks the maps cleared in THIS sub-batch: the others keep the exact size tracking and hot-key routing
    const uint8_t f = mflag[m];
    const uint8_t g = (uint8_t)((f & ~kMfClr) | (ph > pl ? kMfClr : 0u));
    if (g != f) mflag[m] = g;
  }
}

// per sub-batch: the clears of [lo, hi) join the map events (code 3: the size resets to 0)
__global__ void k_clr_events(const uint64_t* __restrict__ keys, uint32_t n, uint64_t lo, uint64_t hi,
                             const uint64_t* __restrict__ index, uint64_t* __restrict__ ev_key, uint32_t* __restrict__ ev_val,
                             EvPay* __restrict__ ev_pay, uint32_t cap, uint32_t* __restrict__ ctl) {
  const uint64_t idx0 = index[lo];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t k = keys[i], row = k & 0xFFFFFFFFull, m = k >> 32;
    if (row < lo || row >= hi) continue;
    const uint64_t d = (index[row] - idx0) & ((1ull << 40) - 1);
    const uint32_t at = atomicAdd(ctl, 1u);
    if (at < cap) {
      ev_key[at] = (m << 44) | (d << 4) | 3u;
      ev_val[at] = at;
      ev_pay[at] = EvPay{0, (uint32_t)row, 0};
    }
  }
}

int launch_clr_sub(const ClrSubArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_clr_sub, dim3((a.R + 255) / 256), dim3(256), 0, st, a.keys, a.off, a.R, a.lo, a.hi, a.base, a.eend,
                     a.mflag, a.err);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_clr_events(const ClrSubArgs& a, hipStream_t st) {
  if (a.n == 0) return 0;
  hipLaunchKernelGGL(k_clr_events, dim3(std::min<uint32_t>(1024, (a.n + 255) / 256)), dim3(256), 0, st, a.keys, a.n, a.lo,
                     a.hi, a.index, a.ev_key, a.ev_val, a.ev_pay, a.ev_cap, a.ev_ctl);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// after the sub-batch's map apply: a cleared map's compacted-key generation moves on
__global__ void k_clr_gen(const uint8_t* __restrict__ eend, uint32_t R, uint64_t* __restrict__ cgen) {
  for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < R; m += gridDim.x * blockDim.x)
    if (eend[m]) ++cgen[m];
}
int launch_clr_gen(const ClrSubArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_clr_gen, dim3((a.R + 255) / 256), dim3(256), 0, st, a.eend, a.R, a.cgen);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// One wave per run of a cleared map (the sorted event buffer, map_small.hip k_small_seg): the size from the sub-batch
// start, +1 insert / -1 removal / 0 at a clear, in log order (a segmented scan: a clear starts a segment at 0); the
// peak -> capacity level and the level timeline; size / isEmpty rows answered with the size before them.
__global__ __launch_bounds__(256) void k_clr_replay(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                                    const EvPay* __restrict__ pay, const uint32_t* __restrict__ ctl,
                                                    const uint32_t* __restrict__ seg, const uint32_t* __restrict__ nseg,
                                                    const uint8_t* __restrict__ mflag, uint32_t* __restrict__ msize,
                                                    uint32_t* __restrict__ mpcap, unsigned long long* __restrict__ lvl_at,
                                                    const uint64_t* __restrict__ idx0p, uint8_t* __restrict__ out_status,
                                                    uint64_t* __restrict__ out_value) {
  const uint32_t E = ctl[0], ns = *nseg, l = __lane_id();
  const uint32_t waves = gridDim.x * (blockDim.x / kWave);
  for (uint32_t r = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave); r < ns; r += waves) {
    const uint32_t start = seg[r];
    const uint32_t m = (uint32_t)(key[start] >> 44);
    if (!(mflag[m] & kMfClr)) continue;
    int64_t size = msize[m];  // at the sub-batch start (the exact tracking leaves this map's counts out)
    int64_t peak = size;      // (within the sub-batch: the level reached before is mpcap already)
    for (uint32_t b = start;; b += kWave) {
      const uint32_t i = b + l;
      const bool in = i < E && (uint32_t)(key[i] >> 44) == m;
      const uint64_t k = in ? key[i] : 0;
      const bool query = in && (k & 8u);
      const bool reset = in && !query && (k & 3u) == 3u;
      const int32_t dlt = !in || query || reset ? 0 : ((k & 3u) == 1u ? 1 : ((k & 3u) == 2u ? -1 : 0));
      int32_t inc = dlt;  // inclusive prefix of the deltas
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      int32_t lr = reset ? (int32_t)l : -1;  // the last reset at or before this lane
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int32_t y = __shfl_up(lr, d, 64);
        if (l >= (uint32_t)d) lr = max(lr, y);
      }
      const int32_t at_reset = __shfl(inc, lr < 0 ? 0 : lr, 64);
      const int64_t v = lr < 0 ? size + inc : (int64_t)(inc - at_reset);  // the size after this event
      if (query) {
        const uint32_t row = pay[val[i]].aux;
        if (k & 4u) {  // isEmpty
          out_status[row] = CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
          out_value[row] = v == 0 ? 1ull : 0ull;
        } else {  // size: an int
          out_status[row] = CC_STATUS(CC_ST_OK, CC_TAG_INT);
          out_value[row] = (uint64_t)v;
        }
      }
      // the peak so far (the running maximum over the lanes before this one and the chunk start's)
      int64_t pk = in ? v : INT64_MIN;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int64_t y = __shfl_up(pk, d, 64);
        if (l >= (uint32_t)d) pk = max(pk, y);
      }
      const int64_t pk_prev = __shfl_up(pk, 1, 64);  // (every lane shuffles: a read of an inactive lane is 0)
      const int64_t before = l == 0 ? peak : max(peak, pk_prev);
      if (lvl_at && in && dlt > 0 && v > before)  // an insertion growing the table (the capacity-level timeline)
        lvl_reached(lvl_at, m, cap_level((uint64_t)max<int64_t>(before, 0)), cap_level((uint64_t)v),
                    *idx0p + ((k >> 4) & ((1ull << 40) - 1)));
      peak = max(peak, (int64_t)__shfl(pk, 63, 64));
      const int32_t lr63 = __shfl(lr, 63, 64), inc63 = __shfl(inc, 63, 64), inc_lr = __shfl(inc, lr63 < 0 ? 0 : lr63, 64);
      size = lr63 < 0 ? size + inc63 : (int64_t)(inc63 - inc_lr);
      if (__ballot(in) != ~0ull) break;
    }
    if (l == 0) {
      msize[m] = (uint32_t)max<int64_t>(size, 0);
      atomicMax(&mpcap[m], cap_level((uint64_t)max<int64_t>(peak, 0)));
    }
  }
}

int launch_clr_replay(const ClrReplayArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_clr_replay, dim3(256), dim3(256), 0, st, a.key, a.val, a.pay, a.ctl, a.seg, a.nseg, a.mflag, a.msize,
                     a.mpcap, a.lvl_at, a.idx0, a.out_status, a.out_value);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
