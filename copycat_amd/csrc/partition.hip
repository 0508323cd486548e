// partition.hip — stable group-by of a commit batch into per-bucket lists (bucket = resource slot / 64).
//
// Why: the reference applies commits one at a time in log order on one thread (ResourceManager.java:56-72);
// commits on DIFFERENT resources are independent (ResourceManager multiplexes isolated state machines,
// ResourceManager.java:37-39) but commits on the SAME resource form a sequential chain.  The engine therefore
// regroups a batch so that one wave owns 64 resources and sees exactly their commits, still in log order.
//
// Pipeline per sub-batch (all kernels stream their inputs coalesced; no global atomics):
//   k_part_count   : per 16384-commit tile, a histogram over buckets (LDS atomics) -> counts[tile][bucket]
//   k_part_scan    : per 64-bucket stripe, exclusive prefix over tiles (in place) + bucket totals
//   k_part_base    : exclusive scan of bucket totals -> bucket base offsets
//   k_part_scatter : per tile, stable multisplit: each wave walks its 4096 commits in steps of 64, ranks
//                    same-bucket lanes with ballots, and writes 24-byte staging records at
//                    base[b] + tile_prefix[b] + wave_prefix[b] + rank.  Commits on unknown instances get
//                    their UNKNOWN_SESSION status here (ResourceManager.java:60-69).
#include "common.h"
#include "engine_internal.h"

namespace cc {

// ResourceManager.operateResource dispatch (ResourceManager.java:60-62): instance slot -> resource slot.
__device__ inline uint32_t resolve(const uint32_t* __restrict__ inst_res, uint32_t max_inst, uint32_t s) {
  return s < max_inst ? inst_res[s] : kNoRes;
}

__global__ __launch_bounds__(kPartThreads) void k_part_count(const uint32_t* __restrict__ inst, uint64_t lo, uint64_t n,
                                                          const uint32_t* __restrict__ inst_res, uint32_t max_inst,
                                                          uint32_t nb, uint32_t* __restrict__ counts) {
  extern __shared__ uint32_t hist[];  // [nb]
  for (uint32_t b = threadIdx.x; b < nb; b += kPartThreads) hist[b] = 0;
  __syncthreads();
  const uint64_t t0 = lo + (uint64_t)blockIdx.x * kTile;
  const uint64_t t1 = t0 + kTile < n ? t0 + kTile : n;
  for (uint64_t i = t0 + threadIdx.x; i < t1; i += kPartThreads) {
    const uint32_t r = resolve(inst_res, max_inst, inst[i]);
    if (r != kNoRes) atomicAdd(&hist[r >> kBucketShift], 1u);
  }
  __syncthreads();
  uint32_t* row = counts + (uint64_t)blockIdx.x * nb;
  for (uint32_t b = threadIdx.x; b < nb; b += kPartThreads) row[b] = hist[b];
}

// One 1024-thread workgroup per stripe of 64 buckets: 16 row groups x 64 bucket lanes.
__global__ __launch_bounds__(1024) void k_part_scan(uint32_t* __restrict__ counts, uint32_t tiles, uint32_t nb,
                                                   uint32_t* __restrict__ tot) {
  __shared__ uint32_t part[kScanGroups][kWave];
  const uint32_t l = threadIdx.x & 63, g = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x * kWave + l;
  const uint32_t per = (tiles + kScanGroups - 1) / kScanGroups;
  const uint32_t r0 = g * per;
  const uint32_t r1 = r0 + per < tiles ? r0 + per : tiles;
  uint32_t s = 0;
  if (b < nb)
    for (uint32_t t = r0; t < r1; ++t) s += counts[(uint64_t)t * nb + b];
  part[g][l] = s;
  __syncthreads();
  uint32_t pre = 0;
  for (uint32_t q = 0; q < g; ++q) pre += part[q][l];
  if (g == kScanGroups - 1 && b < nb) tot[b] = pre + s;
  if (b < nb)
    for (uint32_t t = r0; t < r1; ++t) {
      const uint64_t k = (uint64_t)t * nb + b;
      const uint32_t c = counts[k];
      counts[k] = pre;
      pre += c;
    }
}

// Exclusive scan of nb (<= 4096) bucket totals in one 1024-thread workgroup.
__global__ __launch_bounds__(1024) void k_part_base(const uint32_t* __restrict__ tot, uint32_t nb, uint32_t* __restrict__ base) {
  __shared__ uint32_t wsum[16];
  const uint32_t t = threadIdx.x, l = t & 63, w = t >> 6;
  uint32_t v[4], s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = t * 4 + k;
    v[k] = i < nb ? tot[i] : 0;
    s += v[k];
  }
  // inclusive wave scan of s
  uint32_t inc = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (l >= (uint32_t)d) inc += y;
  }
  if (l == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t wpre = 0;
  for (uint32_t q = 0; q < w; ++q) wpre += wsum[q];
  uint32_t run = wpre + inc - s;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = t * 4 + k;
    if (i < nb) base[i] = run;
    run += v[k];
  }
}

__global__ __launch_bounds__(kPartThreads) void k_part_scatter(const uint32_t* __restrict__ inst, const uint8_t* __restrict__ op,
                                                            const uint8_t* __restrict__ flags, const uint64_t* __restrict__ ca,
                                                            const uint64_t* __restrict__ cb, uint64_t lo, uint64_t n,
                                                            const uint32_t* __restrict__ inst_res, uint32_t max_inst,
                                                            uint32_t nb, uint32_t nbits, const uint32_t* __restrict__ offs,
                                                            const uint32_t* __restrict__ base, uint64_t* __restrict__ st_meta,
                                                            u64x2* __restrict__ st_ab, uint8_t* __restrict__ out_status,
                                                            uint64_t* __restrict__ out_value) {
  extern __shared__ uint32_t woff_flat[];  // [kPartWaves][nb]
  auto woff = [&](uint32_t q, uint32_t b) -> uint32_t& { return woff_flat[q * nb + b]; };
  const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint64_t tile0 = lo + (uint64_t)blockIdx.x * kTile;
  const uint64_t w0 = tile0 + (uint64_t)w * kWaveTile;
  const uint64_t w1 = w0 + kWaveTile < n ? w0 + kWaveTile : n;

  // phase 1: per-wave bucket counts of this wave's 4096-commit sub-tile
  for (uint32_t b = threadIdx.x; b < nb; b += kPartThreads)
#pragma unroll
    for (int q = 0; q < kPartWaves; ++q) woff(q, b) = 0;
  __syncthreads();
  for (uint64_t i = w0 + l; i < w1; i += kWave) {
    const uint32_t r = resolve(inst_res, max_inst, inst[i]);
    if (r != kNoRes) atomicAdd(&woff(w, r >> kBucketShift), 1u);
  }
  __syncthreads();
  // phase 2: wave-level exclusive offsets = bucket base + tile prefix + earlier waves of this tile
  const uint32_t* trow = offs + (uint64_t)blockIdx.x * nb;
  for (uint32_t b = threadIdx.x; b < nb; b += kPartThreads) {
    uint32_t run = base[b] + trow[b];
#pragma unroll
    for (int q = 0; q < kPartWaves; ++q) {
      const uint32_t c = woff(q, b);
      woff(q, b) = run;
      run += c;
    }
  }
  __syncthreads();
  // phase 3: stable scatter, 64 commits per step, same-bucket lanes ranked by ballot
  uint32_t* my = woff_flat + w * nb;
  const uint64_t lt = lanemask_lt();
  for (uint64_t s0 = w0; s0 < w1; s0 += kWave) {
    const uint64_t i = s0 + l;
    const bool in = i < w1;
    const uint32_t r = in ? resolve(inst_res, max_inst, inst[i]) : kNoRes;
    const bool live = r != kNoRes;
    if (in && !live) {  // ResourceManagerException "unknown resource session" (ResourceManager.java:64-68)
      out_status[i] = CC_STATUS(CC_ST_UNKNOWN_SESSION, CC_TAG_NULL);
      out_value[i] = 0;
    }
    const uint32_t b = live ? (r >> kBucketShift) : 0;
    uint64_t peers = ballot(live);
    for (uint32_t k = 0; k < nbits; ++k) {
      const bool bit = (b >> k) & 1u;
      const uint64_t m = ballot(live && bit);
      peers &= bit ? m : ~m;
    }
    uint32_t dst = 0;
    if (live) dst = my[b] + (uint32_t)__popcll(peers & lt);
    if (live && (peers & lt) == 0) my[b] += (uint32_t)__popcll(peers);
    if (live) {
      st_meta[dst] = pack_meta((uint32_t)(i - lo), op[i], flags[i], r & (kResPerBucket - 1));
      u64x2 ab;
      ab.x = ca[i];
      ab.y = cb[i];
      st_ab[dst] = ab;
    }
  }
}

int launch_partition(const PartArgs& a, hipStream_t st) {
  const uint32_t tiles = (uint32_t)((a.n - a.lo + kTile - 1) / kTile);
  if (tiles == 0) return 0;
  a.mark(K_PART_COUNT, 1, st);
  hipLaunchKernelGGL(k_part_count, dim3(tiles), dim3(kPartThreads), a.nb * sizeof(uint32_t), st, a.inst, a.lo, a.n,
                     a.inst_res, a.max_inst, a.nb, a.counts);
  a.mark(K_PART_COUNT, 0, st);
  a.mark(K_PART_SCAN, 1, st);
  hipLaunchKernelGGL(k_part_scan, dim3((a.nb + kWave - 1) / kWave), dim3(1024), 0, st, a.counts, tiles, a.nb, a.tot);
  a.mark(K_PART_SCAN, 0, st);
  a.mark(K_PART_BASE, 1, st);
  hipLaunchKernelGGL(k_part_base, dim3(1), dim3(1024), 0, st, a.tot, a.nb, a.base);
  a.mark(K_PART_BASE, 0, st);
  a.mark(K_PART_SCATTER, 1, st);
  hipLaunchKernelGGL(k_part_scatter, dim3(tiles), dim3(kPartThreads), kPartWaves * a.nb * sizeof(uint32_t), st, a.inst,
                     a.op, a.flags, a.a, a.b, a.lo, a.n, a.inst_res, a.max_inst, a.nb, a.nbits, a.counts, a.base,
                     a.st_meta, a.st_ab, a.out_status, a.out_value);
  a.mark(K_PART_SCATTER, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
