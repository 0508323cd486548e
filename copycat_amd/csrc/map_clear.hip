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
//                  a cleared map's hot keys take the same epochs in the hot-key path (apply_map_hot.hip: CLEAR.el in the
//                  piece scan, the state cleared before a commit of a later epoch);
//   sizes          the flagged maps' insertions / removals are events (k_msize_count; their per-tile counts are left
//                  out of the exact tracking), the clears join them (k_clr_events), and after the sort a scan with resets
//                  over all events gives each map's sizes from the one at the sub-batch start: +1 / -1 / 0, the peak ->
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
    // kMfClr marks the maps cleared in THIS sub-batch: the others keep the exact size tracking (atomic on the flag
    // word: neighbouring maps' bytes share it; only the engine stream writes the flags, common.h)
    const uint8_t f = mflag[m];
    if (ph > pl && !(f & kMfClr)) mflag_or(mflag, m, kMfClr);
    else if (ph == pl && (f & kMfClr)) mflag_and(mflag, m, (uint8_t)~kMfClr);
  }
}

// per sub-batch: every map's epoch at the start of each row bucket, bit 7 set when one of its clears falls inside the
// bucket (clr_epoch's first step; 0 for a map not cleared in the sub-batch)
__global__ void k_clr_btab(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ off,
                           const uint32_t* __restrict__ base, const uint8_t* __restrict__ eend,
                           const uint8_t* __restrict__ mflag, uint32_t R, uint32_t nb, uint32_t bshift, uint64_t lo,
                           uint8_t* __restrict__ btab) {
  const uint64_t total = (uint64_t)R * nb;
  for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t m = (uint32_t)(x / nb), b = (uint32_t)(x % nb);
    if (!(mflag[m] & kMfClr)) {
      btab[x] = 0;
      continue;
    }
    const uint64_t* p = keys + off[m] + base[m];
    const uint64_t row = lo + ((uint64_t)b << bshift);
    const uint32_t ne = eend[m];
    uint32_t a = 0, c = ne;
    while (a < c) {  // the clears before the bucket's first row
      const uint32_t mid = (a + c) >> 1;
      if ((p[mid] & 0xFFFFFFFFull) < row) a = mid + 1; else c = mid;
    }
    const bool inside = a < ne && (p[a] & 0xFFFFFFFFull) < row + (1ull << bshift);  // a clear inside the bucket
    btab[x] = (uint8_t)(a | (inside ? 0x80u : 0u));
  }
}

// per sub-batch: the clears of [lo, hi) join the map events (code 3: the size resets to 0)
__global__ void k_clr_events(const uint64_t* __restrict__ keys, uint32_t n, uint64_t lo, uint64_t hi,
                             const uint64_t* __restrict__ index, uint64_t* __restrict__ ev_key, uint32_t* __restrict__ ev_val,
                             EvPay* __restrict__ ev_pay, uint32_t cap, uint32_t* __restrict__ ctl, uint32_t* __restrict__ err) {
  const uint64_t idx0 = index[lo];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t k = keys[i], row = k & 0xFFFFFFFFull, m = k >> 32;
    if (row < lo || row >= hi) continue;
    const uint64_t d = index[row] - idx0;
    if (d >> kEvPosBits) atomicOr(err, kErrSpan);
    const uint32_t at = atomicAdd(ctl, 1u);
    if (at < cap) {
      ev_key[at] = (m << kEvMapShift) | ((d & kEvPosMask) << 4) | 3u;
      ev_val[at] = at;
      ev_pay[at] = EvPay{0, (uint32_t)row, 0};
    }
  }
}

int launch_clr_sub(const ClrSubArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_clr_sub, dim3((a.R + 255) / 256), dim3(256), 0, st, a.keys, a.off, a.R, a.lo, a.hi, a.base, a.eend,
                     a.mflag, a.err);
  const uint64_t cells = (uint64_t)a.R * a.nb;
  hipLaunchKernelGGL(k_clr_btab, dim3((uint32_t)std::min<uint64_t>(4096, (cells + 255) / 256)), dim3(256), 0, st, a.keys,
                     a.off, a.base, a.eend, a.mflag, a.R, a.nb, a.bshift, a.lo, a.btab);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_clr_events(const ClrSubArgs& a, hipStream_t st) {
  if (a.n == 0) return 0;
  hipLaunchKernelGGL(k_clr_events, dim3(std::min<uint32_t>(1024, (a.n + 255) / 256)), dim3(256), 0, st, a.keys, a.n, a.lo,
                     a.hi, a.index, a.ev_key, a.ev_val, a.ev_pay, a.ev_cap, a.ev_ctl, a.err);
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

// The cleared maps' sizes over the sorted event buffer (map_small.hip k_small_seg's order: one map's events together, in
// log order), flat over all events: the size after each event is a scan with resets -- +1 insert, -1 removal, reset
// to 0 at a clear, reset to (size at the sub-batch start +- the event) at a map's first event -- and the peak since the
// map's first event rides the same scan (a running maximum split at the first reset: before it relative, after it
// absolute).  One hipcub scan of 16-byte elements, then one pass per event answers size / isEmpty rows, records the
// capacity-level timeline and, at a map's last event, writes its size and capacity level.  (It was one wave per map
// walking its run 64 events per step: a hot map's ~1M events per sub-batch took 3.4 ms of serial chunks.)
constexpr int32_t kClrNeg = -(1 << 30);  // "no value" of a running maximum (sizes stay below 2^30)
struct ClrS {
  int32_t v;     // the size after the span (absolute when f & 1, else the span's net change)
  int32_t pre;   // the highest size before the span's first reset, relative to the size entering it
  int32_t post;  // the highest absolute size from the span's first reset on
  uint32_t f;    // 1: the span holds a reset (a clear or a map's first event); 2: it holds a map's first event
};
struct ClrCompose {
  __device__ ClrS operator()(const ClrS& a, const ClrS& b) const {
    if (b.f & 2u) return b;  // (a map's first event: nothing before it matters)
    ClrS r;
    r.f = a.f | b.f;
    r.v = (b.f & 1u) ? b.v : a.v + b.v;
    const int32_t mid = a.v + b.pre;  // b's values before its first reset, on top of a
    if (a.f & 1u) {
      r.pre = a.pre;
      r.post = max(max(a.post, mid), (b.f & 1u) ? b.post : kClrNeg);
    } else {
      r.pre = max(a.pre, mid);
      r.post = (b.f & 1u) ? b.post : kClrNeg;
    }
    return r;
  }
};
__device__ inline int32_t clr_delta(uint64_t k) {
  if (k & 8u) return 0;  // a size / isEmpty query
  const uint32_t c = (uint32_t)(k & 3u);
  return c == 1u ? 1 : (c == 2u ? -1 : 0);
}
struct ClrElem {
  const uint64_t* key;
  const uint32_t* msize;
  __device__ ClrS operator()(uint32_t i) const {
    const uint64_t k = key[i];
    const uint32_t m = (uint32_t)(k >> kEvMapShift);
    const bool clear = !(k & 8u) && (k & 3u) == 3u;
    const int32_t d = clr_delta(k);
    if (i == 0 || (uint32_t)(key[i - 1] >> kEvMapShift) != m) {  // the map's first event: from its size at the sub-batch start
      const int32_t s0 = (int32_t)msize[m];
      const int32_t v = clear ? 0 : s0 + d;
      return ClrS{v, kClrNeg, max(s0, v), 3u};
    }
    if (clear) return ClrS{0, kClrNeg, 0, 1u};
    return ClrS{d, d, kClrNeg, 0u};
  }
};
using ClrIt = hipcub::TransformInputIterator<ClrS, ClrElem, hipcub::CountingInputIterator<uint32_t>>;

__global__ __launch_bounds__(256) void k_clr_finish(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                                    const EvPay* __restrict__ pay, const ClrS* __restrict__ S, uint32_t E,
                                                    const uint8_t* __restrict__ mflag, uint32_t* __restrict__ msize,
                                                    uint32_t* __restrict__ mpcap, unsigned long long* __restrict__ lvl_at,
                                                    const uint64_t* __restrict__ idx0p, uint8_t* __restrict__ out_status,
                                                    uint64_t* __restrict__ out_value) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < E; i += gridDim.x * blockDim.x) {
    const uint64_t k = key[i];
    const uint32_t m = (uint32_t)(k >> kEvMapShift);
    if (!(mflag[m] & kMfClr)) continue;  // (small / size-queried maps: map_small.hip)
    const ClrS x = S[i];
    const int32_t v = x.v;
    if (k & 8u) {
      const uint32_t row = pay[val[i]].aux;
      if (k & 4u) {  // isEmpty
        out_status[row] = CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
        out_value[row] = v == 0 ? 1ull : 0ull;
      } else {  // size: an int
        out_status[row] = CC_STATUS(CC_ST_OK, CC_TAG_INT);
        out_value[row] = (uint64_t)v;
      }
    }
    const bool first = i == 0 || (uint32_t)(key[i - 1] >> kEvMapShift) != m;
    if (lvl_at && clr_delta(k) > 0) {  // an insertion growing the table (the capacity-level timeline)
      const int32_t before = first ? v - 1 : S[i - 1].post;  // (the peak so far, the start size included)
      if (v > before)
        lvl_reached(lvl_at, m, cap_level((uint64_t)max(before, 0)), cap_level((uint64_t)v),
                    *idx0p + ((k >> 4) & kEvPosMask));
    }
    if (i + 1 == E || (uint32_t)(key[i + 1] >> kEvMapShift) != m) {  // the map's last event
      msize[m] = (uint32_t)max(v, 0);
      atomicMax(&mpcap[m], cap_level((uint64_t)max(x.post, 0)));
    }
  }
}

size_t clr_scan_temp_bytes(uint32_t cap) {
  size_t need = 0;
  ClrIt it(hipcub::CountingInputIterator<uint32_t>(0), ClrElem{nullptr, nullptr});
  (void)hipcub::DeviceScan::InclusiveScan(nullptr, need, it, (ClrS*)nullptr, ClrCompose{}, (int)cap, (hipStream_t)0);
  return need;
}
size_t clr_scan_bytes_per_event() { return sizeof(ClrS); }

int launch_clr_replay(const ClrReplayArgs& a, uint32_t E, hipStream_t st) {
  if (E == 0) return 0;
  ClrIt it(hipcub::CountingInputIterator<uint32_t>(0), ClrElem{a.key, a.msize});
  size_t tb = a.temp_bytes;
  ClrS* S = static_cast<ClrS*>(a.scan);
  if (hipcub::DeviceScan::InclusiveScan(a.temp, tb, it, S, ClrCompose{}, (int)E, st) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_clr_finish, dim3(std::min<uint32_t>(2048, (E + 255) / 256)), dim3(256), 0, st, a.key, a.val, a.pay, S,
                     E, a.mflag, a.msize, a.mpcap, a.lvl_at, a.idx0, a.out_status, a.out_value);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
