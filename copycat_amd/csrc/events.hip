// events.hip — the published events of a sub-batch, in the caller's order: by log row, then by the order in
// which the commit published them (Session.publish order, ManagedResourceSession.java:64-71).
//
// apply_coord.hip leaves each commit's event count at its staging position (ev_cnt) and the events themselves,
// tagged with (staging position, emission index), in an arena in whatever order workgroups finished.
//   k_ev_rows    : per partition tile: the counts back in row order (through cpos), an exclusive scan inside
//                  the tile, and row_of[staging position] = row for commits that published;
//   k_ev_tiles   : one workgroup: exclusive scan of the tile totals on top of the events already written by
//                  earlier sub-batches; capacity / no-stream checks;
//   k_ev_perm    : every arena event's output position (tile offset + row offset + emission index) -> perm[];
//   k_ev_out     : the output rows in order, each gathering its arena record: the six output columns are
//                  written contiguously (scattered 1-byte stores to them were the cost of the old one-pass
//                  scatter, k_ev_scatter, kept for A/B under CC_EV_SCATTER).
#include <cstdlib>

#include "common.h"
#include "engine_internal.h"

namespace cc {

constexpr int kER = kPT;  // 1024 threads per tile
constexpr int kERPer = kTile / kER;

// Per tile: thread t owns rows [16 t, 16 t + 16) (two 16-byte loads of cpos); a staged commit that published
// gets row_of (its row) and ev_loc (the tile-relative offset of its first event), both at its staging position.
__global__ __launch_bounds__(kER) void k_ev_rows(const uint16_t* __restrict__ cpos, uint64_t n, const uint16_t* __restrict__ ev_cnt,
                                                 uint32_t* __restrict__ row_of, uint32_t* __restrict__ ev_loc,
                                                 uint32_t* __restrict__ tile_sum) {
  static_assert(kERPer == 16, "two uint4 of cpos per thread");
  __shared__ uint32_t wsum[kER / kWave];
  // the tile's row_of / ev_loc are assembled in LDS and written out whole (scattered 4-byte stores to HBM cost a
  // partly written line each); positions of commits that published nothing carry stale values nobody reads
  __shared__ uint32_t lrow[kTile], lloc[kTile];
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  const uint64_t r0 = (uint64_t)blockIdx.x * kTile + (uint64_t)t * kERPer;
  const uint32_t tbase = blockIdx.x * kTile;
  uint32_t pp[kERPer];
  {
    // (cpos has a full tile for every tile of the sub-batch: the rows past n read as unknown sessions below)
    const uint4 v0 = reinterpret_cast<const uint4*>(cpos + r0)[0], v1 = reinterpret_cast<const uint4*>(cpos + r0)[1];
    const uint32_t ww[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      pp[2 * q] = ww[q] & 0xFFFF;
      pp[2 * q + 1] = ww[q] >> 16;
    }
  }
  uint32_t c[kERPer], sum = 0;
#pragma unroll
  for (int q = 0; q < kERPer; ++q) {
    c[q] = r0 + q < n && pp[q] != 0xFFFF ? ev_cnt[tbase + pp[q]] : 0u;
    sum += c[q];
  }
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (l >= (uint32_t)d) inc += y;
  }
  if (l == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t run = inc - sum, total = 0;
  for (uint32_t q = 0; q < kER / kWave; ++q) {
    if (q < w) run += wsum[q];
    total += wsum[q];
  }
#pragma unroll
  for (int q = 0; q < kERPer; ++q) {
    if (c[q]) {
      lrow[pp[q]] = (uint32_t)(r0 + q);
      lloc[pp[q]] = run;
    }
    run += c[q];
  }
  if (t == 0) tile_sum[blockIdx.x] = total;
  __syncthreads();
  for (uint32_t k = t; k < (uint32_t)kTile; k += kER) {
    row_of[tbase + k] = lrow[k];
    ev_loc[tbase + k] = lloc[k];
  }
}

__global__ __launch_bounds__(kER) void k_ev_tiles(const uint32_t* __restrict__ tile_sum, uint32_t tiles,
                                                  unsigned long long* __restrict__ ev_total, uint64_t* __restrict__ tile_off,
                                                  const unsigned long long* __restrict__ arena_n, uint64_t arena_cap,
                                                  uint64_t out_cap, int has_out, uint32_t* __restrict__ err_out) {
  __shared__ unsigned long long wsum[kER / kWave];
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  const unsigned long long base = *ev_total;
  unsigned long long v = t < tiles ? tile_sum[t] : 0, inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long y = __shfl_up(inc, d, 64);
    if (l >= (uint32_t)d) inc += y;
  }
  if (l == 63) wsum[w] = inc;
  __syncthreads();
  unsigned long long run = inc - v, total = 0;
  for (uint32_t q = 0; q < kER / kWave; ++q) {
    if (q < w) run += wsum[q];
    total += wsum[q];
  }
  if (t < tiles) tile_off[t] = base + run;
  __syncthreads();
  if (t == 0) {
    *ev_total = base + total;
    uint32_t err = 0;
    if (*arena_n > arena_cap || (has_out && base + total > out_cap)) err |= kErrEvents;
    if (!has_out && total) err |= kErrUnsupported;  // events published but no stream to publish them to
    if (err) atomicOr(err_out, err);
  }
}

__global__ void k_ev_scatter(const EvRec* __restrict__ arena, const unsigned long long* __restrict__ arena_n,
                             uint64_t arena_cap, const uint32_t* __restrict__ row_of, const uint32_t* __restrict__ ev_loc,
                             const uint64_t* __restrict__ tile_off, uint64_t lo, uint64_t out_cap, uint32_t* __restrict__ pos,
                             uint32_t* __restrict__ target, uint8_t* __restrict__ code, uint8_t* __restrict__ src,
                             uint8_t* __restrict__ tag, uint64_t* __restrict__ payload) {
  const uint64_t ne = *arena_n < arena_cap ? *arena_n : arena_cap;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += (uint64_t)gridDim.x * blockDim.x) {
    const EvRec r = arena[e];
    const uint32_t i = row_of[r.g];
    const uint64_t dst = tile_off[r.g / kTile] + ev_loc[r.g] + r.k;
    if (dst >= out_cap) continue;
    pos[dst] = (uint32_t)(lo + i);
    target[dst] = r.target;
    code[dst] = r.code;
    src[dst] = r.src;
    tag[dst] = r.tag;
    payload[dst] = r.payload;
  }
}

__global__ void k_ev_perm(const EvRec* __restrict__ arena, const unsigned long long* __restrict__ arena_n,
                          uint64_t arena_cap, const uint32_t* __restrict__ row_of, const uint32_t* __restrict__ ev_loc,
                          const uint64_t* __restrict__ tile_off, uint32_t* __restrict__ perm) {
  const uint64_t ne = *arena_n < arena_cap ? *arena_n : arena_cap;
  const uint64_t base = tile_off[0];
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t g = arena[e].g;
    const uint16_t k = arena[e].k;
    const uint64_t d = tile_off[g / kTile] + ev_loc[g] + k - base;
    if (d < arena_cap) perm[d] = (uint32_t)e;  // (more events than the arena holds: the call fails, kErrEvents)
  }
}

__global__ void k_ev_out(const EvRec* __restrict__ arena, const unsigned long long* __restrict__ arena_n,
                         uint64_t arena_cap, const uint32_t* __restrict__ perm,
                         const uint32_t* __restrict__ row_of, const uint64_t* __restrict__ tile_off,
                         const unsigned long long* __restrict__ ev_total, uint64_t lo, uint64_t out_cap,
                         uint32_t* __restrict__ pos, uint32_t* __restrict__ target, uint8_t* __restrict__ code,
                         uint8_t* __restrict__ src, uint8_t* __restrict__ tag, uint64_t* __restrict__ payload) {
  const uint64_t base = tile_off[0], end = *ev_total < out_cap ? *ev_total : out_cap;
  const uint64_t ne = *arena_n < arena_cap ? *arena_n : arena_cap;
  if (*arena_n > arena_cap) return;  // the arena overflowed: perm is incomplete and the call fails (kErrEvents)
  for (uint64_t d = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; d < end; d += (uint64_t)gridDim.x * blockDim.x) {
    if (d - base >= ne) break;
    const EvRec r = arena[perm[d - base]];
    pos[d] = (uint32_t)(lo + row_of[r.g]);
    target[d] = r.target;
    code[d] = r.code;
    src[d] = r.src;
    tag[d] = r.tag;
    payload[d] = r.payload;
  }
}

int launch_events(const EventArgs& a, hipStream_t st) {
  if (a.tiles == 0) return 0;
  a.mark(K_EVENTS, 1, st);
  hipLaunchKernelGGL(k_ev_rows, dim3(a.tiles), dim3(kER), 0, st, a.cpos, a.hi - a.lo, a.ev_cnt, a.row_of, a.ev_loc,
                     a.tile_sum);
  hipLaunchKernelGGL(k_ev_tiles, dim3(1), dim3(kER), 0, st, a.tile_sum, a.tiles, a.ev_total, a.tile_off, a.arena_n,
                     a.arena_cap, a.out_cap, a.out_pos ? 1 : 0, a.err);
  static const bool one_pass = getenv("CC_EV_SCATTER") != nullptr;
  if (a.out_pos && (one_pass || !a.perm)) {
    hipLaunchKernelGGL(k_ev_scatter, dim3(1024), dim3(256), 0, st, a.arena, a.arena_n, a.arena_cap, a.row_of, a.ev_loc,
                       a.tile_off, a.lo, a.out_cap, a.out_pos, a.out_target, a.out_code, a.out_src, a.out_tag,
                       a.out_payload);
  } else if (a.out_pos) {
    hipLaunchKernelGGL(k_ev_perm, dim3(1024), dim3(256), 0, st, a.arena, a.arena_n, a.arena_cap, a.row_of, a.ev_loc,
                       a.tile_off, a.perm);
    hipLaunchKernelGGL(k_ev_out, dim3(2048), dim3(256), 0, st, a.arena, a.arena_n, a.arena_cap, a.perm, a.row_of, a.tile_off, a.ev_total, a.lo,
                       a.out_cap, a.out_pos, a.out_target, a.out_code, a.out_src, a.out_tag, a.out_payload);
  }
  a.mark(K_EVENTS, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
