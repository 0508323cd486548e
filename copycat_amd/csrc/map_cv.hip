// map_cv.hip — MapState.containsValue answered in the stream, outside TTL mode, for maps that hold no null value.
//
// MapState.containsValue (collections/src/main/java/io/atomix/collections/state/MapState.java:49-60) walks
// map.values() and returns true at the first value equal to the operand; a stored null met first throws
// NullPointerException.  With no null stored the answer is order-free: true iff some present entry of the
// map holds the operand (same tag, same canonical payload) at the row.  Such rows need no barrier (map_wide.hip):
//
//   per batch   k_map_barriers lists the containsValue rows of maps (candidates) and flags their maps (kMfCv);
//               k_cv_nullrows finds, per flagged map, the first row that stores a null value (put / putIfAbsent /
//               replace / replaceIfPresent with a NULL value tag) or deletes the map; k_cv_maynull marks the flagged
//               maps that hold a null at the batch start; k_cv_classify keeps a candidate in the stream when its map
//               holds no null before it (else it becomes a barrier row, answered by map_wide.hip in HashMap order);
//   per sub-batch  the in-stream rows' operands go into a device hash set (k_cv_query, one position per operand,
//               plus a query event at the row's log position); k_cv_count0 counts, per operand, the present entries
//               that hold it at the sub-batch start; the map apply kernels (k_apply_map, k_hot_apply) report every
//               commit of a flagged map that moves a set operand into or out of an entry (common.h cv_change: an
//               event at the commit's log position); after the apply the events are sorted by (operand, log
//               position, kind) and one wave per operand walks its run: the count at each query = the initial count
//               plus the changes before it; the answer is count > 0 (k_cv_answer writes the row's result over the
//               placeholder the apply left, map_ops.h map_orphan).
//
// A query sorts after the commit whose index it carries (a query takes the index of the command before it) and
// before the next command.  Cost per sub-batch with in-stream rows: one pass over the table words (and the values of
// the flagged maps' entries), one set probe per value change of a flagged map, a sort of the events.
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "engine_internal.h"

namespace cc {

__device__ inline bool cv_stores(uint32_t op) {
  return op == CC_OP_MAP_PUT || op == CC_OP_MAP_PUTIFABSENT || op == CC_OP_MAP_REPLACE || op == CC_OP_MAP_REPLACEIFPRESENT;
}

// per batch: the first row of each flagged map that stores a null (or deletes the map: k_map_barriers lists those).
// 16 rows per thread and step from one 16-byte load of the op and flags columns each (a row per thread with byte
// loads was 1.9 ms per 1e9 rows); the rare null-storing rows resolve their map.
__device__ inline void cv_null_row(uint64_t i, const uint32_t* __restrict__ inst, const uint32_t* __restrict__ inst_res,
                                   uint32_t max_inst, const uint8_t* __restrict__ mflag, uint32_t* __restrict__ mfirst) {
  const uint32_t in = inst[i];
  if (in >= max_inst) return;
  const uint32_t r = inst_res[in];
  if (r == kNoRes || !(mflag[r] & kMfCv)) return;
  atomicMin(&mfirst[r], (uint32_t)i);
}
__global__ void k_cv_nullrows(const uint32_t* __restrict__ inst, const uint8_t* __restrict__ op,
                              const uint8_t* __restrict__ flags, uint64_t n, const uint32_t* __restrict__ inst_res,
                              uint32_t max_inst, const uint8_t* __restrict__ mflag, const uint32_t* __restrict__ cvq_n,
                              uint32_t* __restrict__ mfirst) {
  if (*cvq_n == 0) return;
  const bool al = ((reinterpret_cast<uintptr_t>(op) | reinterpret_cast<uintptr_t>(flags)) & 15) == 0;
  const uint64_t groups = (n + 15) / 16;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i0 = 16 * g;
    if (al && i0 + 16 <= n) {
      const uint4 o4 = reinterpret_cast<const uint4*>(op)[g], f4 = reinterpret_cast<const uint4*>(flags)[g];
      const uint32_t ow[4] = {o4.x, o4.y, o4.z, o4.w}, fw[4] = {f4.x, f4.y, f4.z, f4.w};
      uint32_t hit = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint32_t o = (ow[q / 4] >> (8 * (q % 4))) & 0xFFu, f = (fw[q / 4] >> (8 * (q % 4))) & 0xFFu;
        hit |= (cv_stores(o) && CC_FLAG_TAG_A(f) == CC_TAG_NULL ? 1u : 0u) << q;
      }
      for (; hit; hit &= hit - 1) cv_null_row(i0 + (uint32_t)__ffs(hit) - 1, inst, inst_res, max_inst, mflag, mfirst);
    } else {
      for (uint64_t i = i0; i < n && i < i0 + 16; ++i)
        if (cv_stores(op[i]) && CC_FLAG_TAG_A(flags[i]) == CC_TAG_NULL) cv_null_row(i, inst, inst_res, max_inst, mflag, mfirst);
    }
  }
}

// per batch: flagged maps holding a null value now
__global__ void k_cv_maynull(const uint32_t* __restrict__ word, uint64_t entries, const uint8_t* __restrict__ mflag,
                             const uint32_t* __restrict__ cvq_n, uint8_t* __restrict__ maynull) {
  if (*cvq_n == 0) return;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < entries; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t w = word[e];
    if (!(w & kMwUsed) || (w & kMwDead) || !(w & kMwPresent) || mw_vtag(w) != CC_TAG_NULL) continue;
    const uint32_t m = w & kMwSlotMask;
    if (mflag[m] & kMfCv) maynull[m] = 1;  // (every writer stores 1)
  }
}

// per batch: each candidate in the stream or a barrier
__global__ void k_cv_classify(const uint32_t* __restrict__ cvq, const uint32_t* __restrict__ cvq_n, uint32_t cvq_cap,
                              const uint32_t* __restrict__ inst, const uint32_t* __restrict__ inst_res,
                              const uint8_t* __restrict__ maynull, const uint32_t* __restrict__ mfirst,
                              uint32_t* __restrict__ bar, uint32_t* __restrict__ bar_n, uint32_t bar_cap,
                              uint32_t* __restrict__ isc, uint32_t* __restrict__ isc_n) {
  const uint32_t n = min(*cvq_n, cvq_cap);
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const uint32_t row = cvq[q];
    const uint32_t r = inst_res[inst[row]];  // (listed through the same registry: a map slot)
    if (maynull[r] || row > mfirst[r]) {
      const uint32_t k = atomicAdd(bar_n, 1u);
      if (k < bar_cap) bar[k] = row;
    } else {
      isc[atomicAdd(isc_n, 1u)] = row;
    }
  }
}

int launch_cv_batch(const CvBatchArgs& a, hipStream_t st) {
  if (hipMemsetAsync(a.maynull, 0, a.R, st) != hipSuccess) return -1;
  if (hipMemsetAsync(a.isc_n, 0, sizeof(uint32_t), st) != hipSuccess) return -1;
  const uint32_t g1 = (uint32_t)std::min<uint64_t>(2048, (a.n / 16 + 256) / 256);
  if (g1) hipLaunchKernelGGL(k_cv_nullrows, dim3(g1), dim3(256), 0, st, a.inst, a.op, a.flags, a.n, a.inst_res, a.max_inst,
                             a.mflag, a.cvq_n, a.mfirst);
  const uint32_t g2 = (uint32_t)std::min<uint64_t>(4096, (a.entries + 255) / 256);
  if (g2) hipLaunchKernelGGL(k_cv_maynull, dim3(g2), dim3(256), 0, st, a.tbl_word, a.entries, a.mflag, a.cvq_n, a.maynull);
  hipLaunchKernelGGL(k_cv_classify, dim3(1024), dim3(256), 0, st, a.cvq, a.cvq_n, a.cvq_cap, a.inst, a.inst_res, a.maynull,
                     a.mfirst, a.bar, a.bar_n, a.bar_cap, a.isc, a.isc_n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t cv_rows_temp_bytes(uint32_t n) {
  size_t need = 0;
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, need, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 32, (hipStream_t)0);
  return need;
}
int cv_sort_rows(uint32_t* rows, uint32_t* rows2, uint32_t n, void* temp, size_t temp_bytes, hipStream_t st) {
  size_t tb = temp_bytes;
  return hipcub::DeviceRadixSort::SortKeys(temp, tb, rows, rows2, (int)n, 0, 32, st) == hipSuccess ? 0 : -1;
}

// ---- per sub-batch -------------------------------------------------------------------------------------------
__device__ inline void cv_operand(uint32_t row, const uint32_t* __restrict__ inst, const uint8_t* __restrict__ flags,
                                  const uint64_t* __restrict__ a, const uint32_t* __restrict__ inst_res, uint32_t& m,
                                  uint32_t& tag, uint64_t& v) {
  m = inst_res[inst[row]];
  tag = CC_FLAG_TAG_A(flags[row]);
  v = tag ? a[row] : 0;
}

// the operands into the set by fingerprint (one position each; k_cv_verify / k_cv_fix give two operands that share a
// fingerprint a position each)
__global__ void k_cv_query(CvSubArgs a) {
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < a.isc_n; q += gridDim.x * blockDim.x) {
    const uint32_t row = a.isc[q];
    uint32_t m, tag;
    uint64_t v;
    cv_operand(row, a.inst, a.flags, a.a, a.inst_res, m, tag, v);
    bool exact;
    const uint64_t k = cv_key(m, tag, v, exact);
    const uint32_t b = cv_bloom_bit(k, a.cv.bbits);
    atomicOr(const_cast<uint32_t*>(a.cv.bloom) + (b >> 5), 1u << (b & 31));
    uint32_t p = cv_slot0(k, a.cv.mask);
    for (;;) {
      unsigned long long c = a.set[p].k64;
      if (c == 0ull) {
        c = atomicCAS(&a.set[p].k64, 0ull, (unsigned long long)k);
        if (c == 0ull) {  // claimed: the operand itself, for the fingerprint check
          a.set[p].v = v;
          a.set[p].meta = (m & kMwSlotMask) | (tag << 17);
          break;
        }
      }
      if (c == k) break;
      p = (p + 1) & a.cv.mask;
    }
  }
}

// Operands whose fingerprint another operand claimed (after k_cv_query: every claimer's operand is written) are
// listed (a.coll); the fingerprint hash is 63 bits, so this is adversarial input only.
__global__ void k_cv_verify(CvSubArgs a) {
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < a.isc_n; q += gridDim.x * blockDim.x) {
    uint32_t m, tag;
    uint64_t v;
    cv_operand(a.isc[q], a.inst, a.flags, a.a, a.inst_res, m, tag, v);
    bool exact;
    const uint64_t k = cv_key(m, tag, v, exact);
    if (exact) continue;
    uint32_t p = cv_slot0(k, a.cv.mask);
    while (a.set[p].k64 != k) p = (p + 1) & a.cv.mask;
    if (a.set[p].v != v || a.set[p].meta != ((m & kMwSlotMask) | (tag << 17))) a.coll[atomicAdd(a.coll_n, 1u)] = q;
  }
}

// The listed operands, one thread in list order: each gets a position of its own with its fingerprint, further along
// the probe sequence (an operand listed twice finds the position its first listing claimed).  cv_find matches the
// operand itself at every position that carries a hashed fingerprint.
__global__ void k_cv_fix(CvSubArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint32_t nc = *a.coll_n;
  for (uint32_t i = 0; i < nc; ++i) {
    uint32_t m, tag;
    uint64_t v;
    cv_operand(a.isc[a.coll[i]], a.inst, a.flags, a.a, a.inst_res, m, tag, v);
    bool exact;
    const uint64_t k = cv_key(m, tag, v, exact);
    const uint32_t meta = (m & kMwSlotMask) | (tag << 17);
    for (uint32_t p = cv_slot0(k, a.cv.mask);; p = (p + 1) & a.cv.mask) {
      const uint64_t c = a.set[p].k64;
      if (c == k && a.set[p].v == v && a.set[p].meta == meta) break;  // (listed before)
      if (c == 0) {
        a.set[p].k64 = k;
        a.set[p].v = v;
        a.set[p].meta = meta;
        break;
      }
    }
  }
}

// a query event per row, at its operand's own position
__global__ void k_cv_qevents(CvSubArgs a) {
  uint32_t err = 0;
  const uint64_t idx0 = a.index[a.lo];
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < a.isc_n; q += gridDim.x * blockDim.x) {
    const uint32_t row = a.isc[q];
    uint32_t m, tag;
    uint64_t v;
    cv_operand(row, a.inst, a.flags, a.a, a.inst_res, m, tag, v);
    const uint32_t p = cv_find(a.set, a.cv.mask, m, tag, v);
    // value: the row in the sub-batch | its clear epoch << 25 (map_clear.hip; 0 without clears in the stream)
    const uint32_t ep = a.clr.mflag && (a.clr.mflag[m] & kMfClr) ? clr_epoch(a.clr, m, row) : 0u;
    cv_event(a.cv, p, a.index[row] - idx0, 2u, (row - (uint32_t)a.lo) | (ep << 25), err);
  }
  if (err) atomicOr(a.err, err);
}

// per operand: the flagged maps' present entries holding it at the sub-batch start
__global__ void k_cv_count0(CvSubArgs a) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a.entries; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t w = a.tbl_word[e];
    if (!(w & kMwUsed) || (w & kMwDead) || !(w & kMwPresent)) continue;
    const uint32_t m = w & kMwSlotMask;
    if (!(a.cv.mflag[m] & kMfCv)) continue;
    const uint32_t t = mw_vtag(w);
    const uint32_t q = cv_lookup(a.cv, m, t, t ? a.tbl_val[e] : 0);
    if (q != ~0u) atomicAdd(&a.cnt[q], 1u);
  }
}

int launch_cv_prepare(const CvSubArgs& a, hipStream_t st) {
  if (hipMemsetAsync(a.set, 0, sizeof(CvEnt) * ((uint64_t)a.cv.mask + 1), st) != hipSuccess) return -1;
  if (hipMemsetAsync(a.cnt, 0, sizeof(uint32_t) * ((uint64_t)a.cv.mask + 1), st) != hipSuccess) return -1;
  if (hipMemsetAsync(a.cv.ctl, 0, sizeof(uint32_t), st) != hipSuccess) return -1;
  if (hipMemsetAsync(const_cast<uint32_t*>(a.cv.bloom), 0, (1ull << a.cv.bbits) / 8, st) != hipSuccess) return -1;
  const uint32_t gq = std::min<uint32_t>(1024, (a.isc_n + 255) / 256);
  if (hipMemsetAsync(a.coll_n, 0, sizeof(uint32_t), st) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_cv_query, dim3(gq), dim3(256), 0, st, a);
  hipLaunchKernelGGL(k_cv_verify, dim3(gq), dim3(256), 0, st, a);
  hipLaunchKernelGGL(k_cv_fix, dim3(1), dim3(64), 0, st, a);
  hipLaunchKernelGGL(k_cv_qevents, dim3(gq), dim3(256), 0, st, a);
  const uint32_t ge = (uint32_t)std::min<uint64_t>(4096, (a.entries + 255) / 256);
  hipLaunchKernelGGL(k_cv_count0, dim3(ge), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---- answers ----------------------------------------------------------------------------------------------------
__global__ void k_cv_seg(const uint64_t* __restrict__ key, uint32_t E, uint32_t* __restrict__ seg, uint32_t* __restrict__ nseg) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < E; i += gridDim.x * blockDim.x)
    if (i == 0 || (key[i] >> 42) != (key[i - 1] >> 42)) seg[atomicAdd(nseg, 1u)] = i;
}

// One wave per operand run (sorted by log position): the running count of entries holding it; a query's answer.
// With clears in the stream every event carries its clear epoch (non-decreasing along the run): the count restarts
// at 0 in each new epoch (cnt0, the count at the sub-batch start, belongs to epoch 0).
__global__ __launch_bounds__(256) void k_cv_answer(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                                   uint32_t E, const uint32_t* __restrict__ seg,
                                                   const uint32_t* __restrict__ nseg, const uint32_t* __restrict__ cnt,
                                                   uint64_t lo, uint8_t* __restrict__ out_status,
                                                   uint64_t* __restrict__ out_value) {
  const uint32_t ns = *nseg, l = __lane_id();
  const uint32_t waves = gridDim.x * (blockDim.x / kWave);
  for (uint32_t r = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave); r < ns; r += waves) {
    const uint32_t start = seg[r];
    const uint64_t q = key[start] >> 42;
    int64_t c = cnt[q];
    uint32_t cep = 0;  // the epoch c belongs to
    for (uint32_t b = start;; b += kWave) {
      const uint32_t i = b + l;
      const bool in = i < E && (key[i] >> 42) == q;
      const uint32_t kind = in ? (uint32_t)(key[i] & 3u) : 3u;
      const uint32_t vv = in ? val[i] : 0u;
      const uint32_t ep = in ? (kind == 2u ? vv >> 25 : vv) : 0xFFFFFFFFu;
      const int32_t dlt = kind == 1u ? 1 : (kind == 0u ? -1 : 0);
      int32_t inc = dlt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      // the first lane of this lane's epoch in the chunk (epochs are non-decreasing along the run)
      const uint32_t pep = __shfl_up(ep, 1, 64);
      int32_t fs = (l == 0 || pep != ep) ? (int32_t)l : 0;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int32_t y = __shfl_up(fs, d, 64);
        if (l >= (uint32_t)d) fs = max(fs, y);
      }
      // deltas before the epoch's lanes (every lane takes part in the shuffle: a lane reading an inactive one gets 0)
      const int32_t at_prev = __shfl(inc, fs > 0 ? fs - 1 : 0, 64);
      const int32_t before = fs == 0 ? 0 : at_prev;
      const int64_t base = ep == cep ? c : 0;  // (a later epoch starts from an empty map)
      if (in && kind == 2u) {
        const uint64_t row = lo + (vv & ((1u << 25) - 1));
        out_status[row] = (uint8_t)CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
        out_value[row] = base + (fs == 0 ? inc : inc - before) > 0 ? 1ull : 0ull;
      }
      // carry: the last in-lane's epoch and count
      const uint64_t inb = __ballot(in);
      const int32_t last = 63 - __clzll((long long)inb);
      const uint32_t lep = (uint32_t)__shfl((int)ep, last, 64);
      const int32_t lfs = __shfl(fs, last, 64), linc = __shfl(inc, last, 64);
      const int32_t lat_prev = __shfl(inc, lfs > 0 ? lfs - 1 : 0, 64);
      const int32_t lbefore = lfs == 0 ? 0 : lat_prev;
      c = (lep == cep ? c : 0) + (lfs == 0 ? linc : linc - lbefore);
      cep = lep;
      if (inb != ~0ull) break;
    }
  }
}

size_t cv_sort_temp_bytes(uint32_t cap) {
  size_t need = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, need, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (int)cap, 0, 64, (hipStream_t)0);
  return need;
}

int launch_cv_answer(const CvSubArgs& a, uint32_t E, hipStream_t st) {
  if (E == 0) return 0;
  if (E > a.cv.cap) return -2;
  size_t tb = a.temp_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(a.temp, tb, a.cv.ev_key, a.key2, a.cv.ev_val, a.val2, (int)E, 0, 64, st) != hipSuccess)
    return -1;
  if (hipMemsetAsync(a.nseg, 0, sizeof(uint32_t), st) != hipSuccess) return -1;
  const uint32_t g = std::min<uint32_t>(1024, (E + 255) / 256);
  hipLaunchKernelGGL(k_cv_seg, dim3(g), dim3(256), 0, st, a.key2, E, a.seg, a.nseg);
  hipLaunchKernelGGL(k_cv_answer, dim3(1024), dim3(256), 0, st, a.key2, a.val2, E, a.seg, a.nseg, a.cnt, a.lo, a.out_status,
                     a.out_value);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
