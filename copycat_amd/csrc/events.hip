// events.hip — the published events of a sub-batch, in the caller's order: by log row, then by the order in
// which the commit published them (Session.publish order, ManagedResourceSession.java:64-71).
//
// apply_coord.hip leaves each commit's event count at its staging position (ev_cnt) and the events themselves,
// tagged with (staging position, emission index), in an arena in whatever order workgroups finished.
//   k_ev_rows    : per partition tile: the counts back in row order (through cpos), an exclusive scan inside
//                  the tile, and row_of[staging position] = row for commits that published;
//   k_ev_tiles   : one workgroup: exclusive scan of the tile totals on top of the events already written by
//                  earlier sub-batches; capacity / no-stream checks;
// Default order pass (round 3): the arena is bucketed by partition tile, and each tile's events are placed from LDS
// tables, with no random gathers of per-row arrays:
//   k_ev_count   : per tile, the events its commits published (ev_cnt over the tile's staging positions);
//   k_ev_tiles   : (as above) the tiles' output offsets;
//   k_ev_chist   : per arena chunk of kEvChunk events, events per tile (ccnt[chunk][tile]);
//   k_ev_cscan   : per tile, the chunks' bucket bases (exclusive scan over chunks from the tile's offset);
//   k_ev_place   : every arena event to its tile's bucket (order inside a bucket is free);
//   k_ev_tile_out: per tile, the per-row event offsets rebuilt in LDS (cpos + ev_cnt), then each of the tile's events
//                  written to its output row (tile offset + row offset + emission index).
// The previous order pass (CC_EV_V1=1, A/B): k_ev_rows as above writes row_of / ev_loc per staging position;
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

// ---- the tile-bucketed order pass ---------------------------------------------------------------------------
constexpr int kEC = 256;  // threads of the counting / bucketing kernels

// events per tile: ev_cnt summed over the tile's staging positions below the sub-batch's row count (memset per
// sub-batch; positions without a staged commit hold 0)
__global__ __launch_bounds__(kEC) void k_ev_count(const uint16_t* __restrict__ ev_cnt, uint64_t n, uint32_t* __restrict__ tile_sum) {
  __shared__ uint32_t wsum[kEC / kWave];
  const uint32_t t = threadIdx.x, l = t & 63, w = t >> 6;
  const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
  const uint64_t end = t0 + kTile < n ? t0 + kTile : n;
  uint32_t s = 0;
  for (uint64_t i = t0 + 8 * (uint64_t)t; i < end; i += 8 * kEC) {
    if (i + 8 <= end) {
      const uint4 v = *reinterpret_cast<const uint4*>(ev_cnt + i);
      const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) s += (x[q] & 0xFFFFu) + (x[q] >> 16);
    } else {
      for (uint64_t k = i; k < end; ++k) s += ev_cnt[k];
    }
  }
#pragma unroll
  for (int d = 32; d; d >>= 1) s += __shfl_xor(s, d, 64);
  if (l == 0) wsum[w] = s;
  __syncthreads();
  if (t == 0) {
    uint32_t tot = 0;
    for (int q = 0; q < kEC / kWave; ++q) tot += wsum[q];
    tile_sum[blockIdx.x] = tot;
  }
}

// per arena chunk: events per tile
__global__ __launch_bounds__(kEC) void k_ev_chist(const EvRec* __restrict__ arena, const unsigned long long* __restrict__ arena_n,
                                                 uint64_t arena_cap, uint32_t tiles, uint32_t* __restrict__ ccnt) {
  __shared__ uint32_t h[kMaxTiles];
  const uint64_t ne = *arena_n < arena_cap ? *arena_n : arena_cap;
  const uint64_t c0 = (uint64_t)blockIdx.x * kEvChunk;
  if (c0 >= ne) return;
  for (uint32_t k = threadIdx.x; k < tiles; k += kEC) h[k] = 0;
  __syncthreads();
  const uint64_t c1 = c0 + kEvChunk < ne ? c0 + kEvChunk : ne;
  for (uint64_t e = c0 + threadIdx.x; e < c1; e += kEC) atomicAdd(&h[arena[e].g / kTile], 1u);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < tiles; k += kEC) ccnt[(uint64_t)blockIdx.x * tiles + k] = h[k];
}

// per tile (one workgroup): the bucket base of each chunk's events of the tile (exclusive prefix over chunks, from the
// tile's offset in the sub-batch's output); thread t owns a contiguous range of chunks
__global__ __launch_bounds__(kEC) void k_ev_cscan(const unsigned long long* __restrict__ arena_n, uint64_t arena_cap,
                                                 uint32_t tiles, const uint64_t* __restrict__ tile_off,
                                                 uint32_t* __restrict__ ccnt) {
  __shared__ uint32_t wsum[kEC / kWave];
  const uint32_t T = blockIdx.x, t = threadIdx.x, w = t >> 6, l = t & 63;
  const uint64_t ne = *arena_n < arena_cap ? *arena_n : arena_cap;
  const uint32_t chunks = (uint32_t)((ne + kEvChunk - 1) / kEvChunk);
  const uint32_t per = (chunks + kEC - 1) / kEC, c0 = t * per, c1 = min(c0 + per, chunks);
  uint32_t sum = 0;
  for (uint32_t c = c0; c < c1; ++c) sum += ccnt[(uint64_t)c * tiles + T];
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (l >= (uint32_t)d) inc += y;
  }
  if (l == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t run = (uint32_t)(tile_off[T] - tile_off[0]) + inc - sum;
  for (uint32_t q = 0; q < w; ++q) run += wsum[q];
  for (uint32_t c = c0; c < c1; ++c) {
    uint32_t* p = ccnt + (uint64_t)c * tiles + T;
    const uint32_t x = *p;
    *p = run;
    run += x;
  }
}

// every event of the chunk to its tile's bucket (base of the (chunk, tile) piece + rank inside it)
__global__ __launch_bounds__(kEC) void k_ev_place(const EvRec* __restrict__ arena, const unsigned long long* __restrict__ arena_n,
                                                 uint64_t arena_cap, uint32_t tiles, const uint32_t* __restrict__ ccnt,
                                                 EvRec* __restrict__ bucket) {
  __shared__ uint32_t h[kMaxTiles];
  const uint64_t ne = *arena_n < arena_cap ? *arena_n : arena_cap;
  const uint64_t c0 = (uint64_t)blockIdx.x * kEvChunk;
  if (c0 >= ne) return;
  for (uint32_t k = threadIdx.x; k < tiles; k += kEC) h[k] = ccnt[(uint64_t)blockIdx.x * tiles + k];
  __syncthreads();
  const uint64_t c1 = c0 + kEvChunk < ne ? c0 + kEvChunk : ne;
  for (uint64_t e = c0 + threadIdx.x; e < c1; e += kEC) {
    const EvRec r = arena[e];
    const uint32_t d = atomicAdd(&h[r.g / kTile], 1u);
    if (d < arena_cap) bucket[d] = r;
  }
}

constexpr int kEvWin = 4096;   // output events assembled per window in k_ev_tile_out
constexpr int kEvMaxWin = 15;  // more windows than this in one tile: events stored straight to their rows (and the
                               // windowed path's row offsets stay below 65,536: u16)
// per tile: the rows' event offsets in LDS, then the tile's events to their output rows, one window at a time
__global__ __launch_bounds__(kER) void k_ev_tile_out(const uint16_t* __restrict__ cpos, uint64_t n, const uint16_t* __restrict__ ev_cnt,
                                                    const uint32_t* __restrict__ tile_sum, const uint64_t* __restrict__ tile_off,
                                                    const EvRec* __restrict__ bucket, const unsigned long long* __restrict__ arena_n,
                                                    uint64_t arena_cap, uint64_t lo, uint64_t out_cap,
                                                    uint32_t* __restrict__ pos, uint32_t* __restrict__ target,
                                                    uint8_t* __restrict__ code, uint8_t* __restrict__ src,
                                                    uint8_t* __restrict__ tag, uint64_t* __restrict__ payload) {
  __shared__ uint32_t wsum[kER / kWave];
  __shared__ uint16_t srow[kTile];    // staging position -> row in the tile
  __shared__ uint16_t soff16[kTile];  // staging position -> offset of its commit's first event in the tile's output
  // one output window of kEvWin events, assembled in LDS so the six columns are written contiguously; a tile past
  // kEvMaxWin windows keeps its (u32) row offsets in the same bytes instead (16-bit offsets and 4,096-event windows:
  // c5's ~6K events per tile take two windows, each re-reading the tile's list, where 2,048-event windows took three)
  __shared__ __align__(16) uint8_t wbuf[kEvWin * 20];
  static_assert(kEvWin * 20 >= kTile * 4, "the direct path's u32 offsets fit the window bytes");
  static_assert(kEvWin * kEvMaxWin < 65536, "windowed offsets are u16");
  uint32_t* const wpos = reinterpret_cast<uint32_t*>(wbuf);
  uint32_t* const wtgt = wpos + kEvWin;
  uint32_t* const wcts = wtgt + kEvWin;
  uint64_t* const wpay = reinterpret_cast<uint64_t*>(wcts + kEvWin);
  uint32_t* const soff32 = reinterpret_cast<uint32_t*>(wbuf);
  if (*arena_n > arena_cap) return;  // the arena overflowed: the call fails (kErrEvents)
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63, T = blockIdx.x;
  const uint32_t nev = tile_sum[T];
  const bool direct = nev > (uint32_t)(kEvWin * kEvMaxWin);  // block-uniform
  const uint64_t r0 = (uint64_t)T * kTile + (uint64_t)t * kERPer;
  const uint32_t tbase = T * kTile;
  uint32_t pp[kERPer];
  {
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
  uint32_t run = inc - sum;
  for (uint32_t q = 0; q < w; ++q) run += wsum[q];
#pragma unroll
  for (int q = 0; q < kERPer; ++q) {
    if (c[q]) {
      srow[pp[q]] = (uint16_t)(t * kERPer + q);
      if (direct) soff32[pp[q]] = run;
      else soff16[pp[q]] = (uint16_t)run;
    }
    run += c[q];
  }
  __syncthreads();
  const uint64_t toff = tile_off[T], b0 = toff - tile_off[0];
  if (b0 + nev > arena_cap || toff + nev > out_cap) return;  // (the call fails: kErrEvents from k_ev_tiles)
  // Each window re-reads the tile's event list (from L2): nev^2 / kEvWin record reads per tile.  A tile whose fan-out
  // makes that more than kEvMaxWin windows (group / election bursts) writes each event straight to its output row
  // instead: scattered stores, linear in nev.
  if (direct) {
    for (uint32_t i = t; i < nev; i += kER) {
      const EvRec r = bucket[b0 + i];
      const uint32_t sp = r.g - tbase;
      const uint64_t d = toff + soff32[sp] + r.k;
      pos[d] = (uint32_t)(lo + tbase + srow[sp]);
      target[d] = r.target;
      code[d] = (uint8_t)r.code;
      src[d] = (uint8_t)r.src;
      tag[d] = (uint8_t)r.tag;
      payload[d] = r.payload;
    }
    return;
  }
  for (uint32_t w0 = 0; w0 < nev; w0 += kEvWin) {  // block-uniform
    const uint32_t wn = nev - w0 < (uint32_t)kEvWin ? nev - w0 : (uint32_t)kEvWin;
    for (uint32_t i = t; i < nev; i += kER) {  // the tile's events (re-read per window from L2)
      const EvRec r = bucket[b0 + i];
      const uint32_t sp = r.g - tbase;
      const uint32_t d = soff16[sp] + r.k - w0;
      if (d < wn) {
        wpos[d] = (uint32_t)(lo + tbase + srow[sp]);
        wtgt[d] = r.target;
        wcts[d] = (uint32_t)r.code | ((uint32_t)r.src << 8) | ((uint32_t)r.tag << 16);
        wpay[d] = r.payload;
      }
    }
    __syncthreads();
    for (uint32_t i = t; i < wn; i += kER) {
      const uint64_t d = toff + w0 + i;
      const uint32_t cts = wcts[i];
      pos[d] = wpos[i];
      target[d] = wtgt[i];
      code[d] = (uint8_t)cts;
      src[d] = (uint8_t)(cts >> 8);
      tag[d] = (uint8_t)(cts >> 16);
      payload[d] = wpay[i];
    }
    __syncthreads();
  }
}

// Events of a batch applied as two calls (more barrier rows than one listing holds, engine.hip): the second call's
// rows start at h, so its events' rows move by h.
__global__ void k_ev_shift(uint32_t* __restrict__ pos, uint64_t n, uint32_t by) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) pos[i] += by;
}

int launch_ev_shift(uint32_t* pos, uint64_t n, uint32_t by, hipStream_t st) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_ev_shift, dim3((uint32_t)std::min<uint64_t>(1024, (n + 255) / 256)), dim3(256), 0, st, pos, n, by);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_events(const EventArgs& a, hipStream_t st) {
  if (a.tiles == 0) return 0;
  a.mark(K_EVENTS, 1, st);
  static const bool v1 = diag_env("CC_EV_V1") || diag_env("CC_EV_SCATTER");
  if (!v1 && a.bucket && a.ccnt) {
    const uint32_t chunks = (uint32_t)ev_chunk_cap(a.arena_cap);
    hipLaunchKernelGGL(k_ev_count, dim3(a.tiles), dim3(kEC), 0, st, a.ev_cnt, a.hi - a.lo, a.tile_sum);
    hipLaunchKernelGGL(k_ev_tiles, dim3(1), dim3(kER), 0, st, a.tile_sum, a.tiles, a.ev_total, a.tile_off, a.arena_n,
                       a.arena_cap, a.out_cap, a.out_pos ? 1 : 0, a.err);
    if (a.out_pos) {
      hipLaunchKernelGGL(k_ev_chist, dim3(chunks), dim3(kEC), 0, st, a.arena, a.arena_n, a.arena_cap, a.tiles, a.ccnt);
      hipLaunchKernelGGL(k_ev_cscan, dim3(a.tiles), dim3(kEC), 0, st, a.arena_n, a.arena_cap, a.tiles, a.tile_off, a.ccnt);
      hipLaunchKernelGGL(k_ev_place, dim3(chunks), dim3(kEC), 0, st, a.arena, a.arena_n, a.arena_cap, a.tiles, a.ccnt,
                         a.bucket);
      hipLaunchKernelGGL(k_ev_tile_out, dim3(a.tiles), dim3(kER), 0, st, a.cpos, a.hi - a.lo, a.ev_cnt, a.tile_sum,
                         a.tile_off, a.bucket, a.arena_n, a.arena_cap, a.lo, a.out_cap, a.out_pos, a.out_target, a.out_code,
                         a.out_src, a.out_tag, a.out_payload);
    }
    a.mark(K_EVENTS, 0, st);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  hipLaunchKernelGGL(k_ev_rows, dim3(a.tiles), dim3(kER), 0, st, a.cpos, a.hi - a.lo, a.ev_cnt, a.row_of, a.ev_loc,
                     a.tile_sum);
  hipLaunchKernelGGL(k_ev_tiles, dim3(1), dim3(kER), 0, st, a.tile_sum, a.tiles, a.ev_total, a.tile_off, a.arena_n,
                     a.arena_cap, a.out_cap, a.out_pos ? 1 : 0, a.err);
  static const bool one_pass = diag_env("CC_EV_SCATTER");
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
