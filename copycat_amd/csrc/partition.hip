// partition.hip — stable group-by of a commit batch into per-super-bucket lists (super-bucket = 256 resource
// slots = one apply workgroup), written as contiguous runs.
//
// Why: the reference applies commits one at a time in log order on one thread (ResourceManager.java:56-72);
// commits on DIFFERENT resources are independent (ResourceManager multiplexes isolated state machines,
// ResourceManager.java:37-39) but commits on the SAME resource form a sequential chain.  The engine therefore
// regroups a batch so that one workgroup owns 256 resources and sees exactly their commits, in log order.
//
// Pipeline per sub-batch [lo, hi) (no global atomics; every global access coalesced):
//   k_part_count   : per 16384-commit tile, a histogram over super-buckets (LDS atomics) -> counts[tile][sb]
//   k_part_scan    : per 64-super-bucket stripe, exclusive prefix over tiles (in place) + totals
//   k_part_base    : exclusive scan of the totals -> super-bucket base offsets in the staging list
//   k_part_scatter : per tile, 4 chunks of 4096 commits: a stable multisplit of the chunk in LDS (ranking
//                    inside a wave by LDS atomics, per-wave prefix sums across the 16 waves), then the chunk is
//                    written out super-bucket by super-bucket, so every staging run is contiguous (no
//                    partial-line writes), plus each commit's chunk-sorted position and per-chunk run tables.
//   k_unpermute    : per chunk, reads the chunk's result runs contiguously into LDS and writes results in log
//                    order (unknown sessions get their UNKNOWN_SESSION status here, ResourceManager.java:60-69).
#include "common.h"
#include "engine_internal.h"

namespace cc {

// ResourceManager.operateResource dispatch (ResourceManager.java:60-62): instance slot -> resource slot.
__device__ inline uint32_t resolve(const uint32_t* __restrict__ inst_res, uint32_t max_inst, uint32_t s) {
  return s < max_inst ? inst_res[s] : kNoRes;
}

__global__ __launch_bounds__(kPT) void k_part_count(const uint32_t* __restrict__ inst, uint64_t lo, uint64_t hi,
                                                 const uint32_t* __restrict__ inst_res, uint32_t max_inst, uint32_t sb,
                                                 uint32_t sb_shift, uint32_t* __restrict__ counts) {
  extern __shared__ uint32_t hist[];  // [sb]
  for (uint32_t b = threadIdx.x; b < sb; b += kPT) hist[b] = 0;
  lds_barrier();
  const uint64_t t0 = lo + (uint64_t)blockIdx.x * kTile;  // multiple of 4 (tiles and sub-batches are)
  const uint64_t t1 = t0 + kTile < hi ? t0 + kTile : hi;
  const uint64_t q1 = t1 / 4;
#pragma unroll 4
  for (uint64_t q = t0 / 4 + threadIdx.x; q < q1; q += kPT) {
    const uint4 v = reinterpret_cast<const uint4*>(inst)[q];
    const uint32_t r0 = resolve(inst_res, max_inst, v.x), r1 = resolve(inst_res, max_inst, v.y);
    const uint32_t r2 = resolve(inst_res, max_inst, v.z), r3 = resolve(inst_res, max_inst, v.w);
    if (r0 != kNoRes) atomicAdd(&hist[r0 >> sb_shift], 1u);
    if (r1 != kNoRes) atomicAdd(&hist[r1 >> sb_shift], 1u);
    if (r2 != kNoRes) atomicAdd(&hist[r2 >> sb_shift], 1u);
    if (r3 != kNoRes) atomicAdd(&hist[r3 >> sb_shift], 1u);
  }
  for (uint64_t i = q1 * 4 + threadIdx.x; i < t1; i += kPT) {  // ragged tail (< 4 commits)
    const uint32_t r = resolve(inst_res, max_inst, inst[i]);
    if (r != kNoRes) atomicAdd(&hist[r >> sb_shift], 1u);
  }
  lds_barrier();
  uint32_t* row = counts + (uint64_t)blockIdx.x * sb;
  for (uint32_t b = threadIdx.x; b < sb; b += kPT) row[b] = hist[b];
}

// One 1024-thread workgroup per stripe of 64 columns: 16 row groups x 64 column lanes.
__global__ __launch_bounds__(1024) void k_part_scan(uint32_t* __restrict__ counts, uint32_t tiles, uint32_t cols,
                                                   uint32_t* __restrict__ tot) {
  __shared__ uint32_t part[kScanGroups][kWave];
  const uint32_t l = threadIdx.x & 63, g = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x * kWave + l;
  const uint32_t per = (tiles + kScanGroups - 1) / kScanGroups;
  const uint32_t r0 = g * per;
  const uint32_t r1 = r0 + per < tiles ? r0 + per : tiles;
  uint32_t s = 0;
  if (b < cols) {
#pragma unroll 8
    for (uint32_t t = r0; t < r1; ++t) s += counts[(uint64_t)t * cols + b];
  }
  part[g][l] = s;
  lds_barrier();
  uint32_t pre = 0;
  for (uint32_t q = 0; q < g; ++q) pre += part[q][l];
  if (g == kScanGroups - 1 && b < cols) tot[b] = pre + s;
  if (b < cols)
#pragma unroll 8
    for (uint32_t t = r0; t < r1; ++t) {
      const uint64_t k = (uint64_t)t * cols + b;
      const uint32_t c = counts[k];
      counts[k] = pre;
      pre += c;
    }
}

// Exclusive scan of one value per thread of a block of up to 1024 threads; every thread must call it.
// Returns the exclusive prefix of this thread and writes the block total to *total.
__device__ inline uint32_t block_exscan(uint32_t v, uint32_t* wsum /*[16] LDS*/, uint32_t* total) {
  const uint32_t t = threadIdx.x, l = t & 63, w = t >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (l >= (uint32_t)d) inc += y;
  }
  lds_barrier();  // wsum may still be read by a previous call
  if (l == 63) wsum[w] = inc;
  lds_barrier();
  uint32_t wpre = 0, all = 0;
  for (uint32_t q = 0; q < blockDim.x / 64; ++q) {
    const uint32_t x = wsum[q];
    if (q < w) wpre += x;
    all += x;
  }
  *total = all;
  return wpre + inc - v;
}

// Exclusive scan of the super-bucket totals (<= 4096, 4 per thread) -> base offsets.
__global__ __launch_bounds__(1024) void k_part_base(const uint32_t* __restrict__ tot, uint32_t cols, uint32_t* __restrict__ base) {
  __shared__ uint32_t wsum[16];
  const uint32_t t = threadIdx.x;
  uint32_t v[4], s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = t * 4 + k;
    v[k] = i < cols ? tot[i] : 0;
    s += v[k];
  }
  uint32_t total;
  uint32_t run = block_exscan(s, wsum, &total);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = t * 4 + k;
    if (i < cols) base[i] = run;
    run += v[k];
  }
}

size_t scatter_lds_bytes(uint32_t sb) {
  return (size_t)kChunk * (16 + 4 + 2) + (size_t)kPW * sb * 4 + (size_t)4 * sb * 4 + 16 * 4;
}

// LDS layout (dynamic): rab[kChunk] u64x2 | rmeta[kChunk] u32 | rsb[kChunk] u16 | wc[kPW][sb] u32 |
//                       toff, trun, ctot, kstart [sb] u32 | wsum[16] u32
//
// Per chunk c (4096 commits) the kernel also records, for k_unpermute:
//   cpos[i]           u16  chunk-sorted position of commit i (0xFFFF: unknown session)
//   ckst[c][0..sb]    u16  chunk-sorted start of each super-bucket's run, ckst[c][sb] = live commits
//   crun[c][0..sb-1]  u32  staging position of that run
__global__ __launch_bounds__(kPT) void k_part_scatter(const uint32_t* __restrict__ inst, const uint8_t* __restrict__ op,
                                                   const uint8_t* __restrict__ flags, const uint64_t* __restrict__ ca,
                                                   const uint64_t* __restrict__ cb, uint64_t lo, uint64_t hi,
                                                   const uint32_t* __restrict__ inst_res, uint32_t max_inst, uint32_t sb,
                                                   uint32_t sb_shift, const uint32_t* __restrict__ offs,
                                                   const uint32_t* __restrict__ base, uint32_t* __restrict__ st_meta,
                                                   u64x2* __restrict__ st_ab, uint16_t* __restrict__ cpos,
                                                   uint16_t* __restrict__ ckst, uint32_t* __restrict__ crun) {
  extern __shared__ __align__(16) uint8_t smem[];
  u64x2* rab = reinterpret_cast<u64x2*>(smem);
  uint32_t* rmeta = reinterpret_cast<uint32_t*>(rab + kChunk);
  uint16_t* rsb = reinterpret_cast<uint16_t*>(rmeta + kChunk);
  uint32_t* wc = reinterpret_cast<uint32_t*>(rsb + kChunk);  // [kPW][sb]
  uint32_t* toff = wc + kPW * sb;
  uint32_t* trun = toff + sb;
  uint32_t* ctot = trun + sb;
  uint32_t* kstart = ctot + sb;
  uint32_t* wsum = kstart + sb;

  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  const uint32_t rmask = (1u << sb_shift) - 1;
  const uint64_t tile0 = lo + (uint64_t)blockIdx.x * kTile;
  const uint32_t* trow = offs + (uint64_t)blockIdx.x * sb;
  for (uint32_t k = t; k < sb; k += kPT) {
    toff[k] = base[k] + trow[k];
    trun[k] = 0;
  }

  constexpr int J = kChunk / kPT;  // commits per thread per chunk
  // commit (w, j, l) of chunk ch is cbase + w*(64*J) + j*64 + l: log order = (w, j, l)
  // Prefetch in two stages so no wave ever stalls on the instance->resource gather right after its load:
  // raw columns of chunk c+1 are requested at the top of chunk c, their gathers after chunk c's ranking.
  uint32_t res[J], meta[J], ninst[J], nmeta[J];
  u64x2 ab[J], nab[J];
  auto load_raw = [&](uint64_t cbase, uint32_t (&in)[J], uint32_t (&mt)[J], u64x2 (&aa)[J]) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const uint64_t i = cbase + (uint64_t)w * (kWave * J) + (uint64_t)j * kWave + l;
      in[j] = kNoRes;
      mt[j] = 0;
      aa[j] = u64x2{0, 0};
      if (i < hi) {
        in[j] = inst[i];
        mt[j] = (uint32_t)op[i] | ((uint32_t)flags[i] << 8);
        aa[j].x = ca[i];
        aa[j].y = cb[i];
      }
    }
  };
  auto gather = [&](const uint32_t (&in)[J], uint32_t (&rr)[J]) {
#pragma unroll
    for (int j = 0; j < J; ++j) rr[j] = in[j] == kNoRes ? kNoRes : resolve(inst_res, max_inst, in[j]);
  };
  load_raw(tile0, ninst, meta, ab);
  gather(ninst, res);
  for (uint32_t ch = 0; ch < kTile / kChunk; ++ch) {
    const uint64_t cbase = tile0 + (uint64_t)ch * kChunk;
    if (cbase >= hi) break;  // block-uniform
    const uint64_t cglob = (cbase - lo) / kChunk;
    const bool more = ch + 1 < kTile / kChunk && cbase + kChunk < hi;
    if (more) load_raw(cbase + kChunk, ninst, nmeta, nab);
    for (uint32_t k = t; k < kPW * sb; k += kPT) wc[k] = 0;
    lds_barrier();
    // 1. rank by super-bucket inside each wave: the wave's own counter table, LDS atomics with return
    //    (same-address lanes of one instruction resolve in lane order on gfx950 — checked at engine start)
    uint32_t key[J], loc[J];
    bool live[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      live[j] = res[j] != kNoRes;
      key[j] = live[j] ? (res[j] >> sb_shift) : 0;
      loc[j] = live[j] ? atomicAdd(&wc[w * sb + key[j]], 1u) : 0;
    }
    uint32_t nres[J];
    if (more) gather(ninst, nres);
    lds_barrier();
    // 2. per super-bucket: exclusive prefix over waves and chunk totals; then chunk-sorted starts
    for (uint32_t k = t; k < sb; k += kPT) {
      uint32_t run = 0;
      for (uint32_t q = 0; q < kPW; ++q) {
        const uint32_t c = wc[q * sb + k];
        wc[q * sb + k] = run;
        run += c;
      }
      ctot[k] = run;
    }
    lds_barrier();
    uint32_t nlive = 0;
    for (uint32_t k0 = 0; k0 < sb; k0 += kPT) {  // block-uniform loop
      const uint32_t k = k0 + t;
      uint32_t part;
      const uint32_t ex = block_exscan(k < sb ? ctot[k] : 0, wsum, &part);
      if (k < sb) kstart[k] = nlive + ex;
      nlive += part;
    }
    lds_barrier();
    // 3. place records in LDS in sorted order; per-commit chunk position; chunk tables
    for (uint32_t k = t; k <= sb; k += kPT) {
      ckst[cglob * (sb + 1) + k] = (uint16_t)(k < sb ? kstart[k] : nlive);
      if (k < sb) crun[cglob * sb + k] = toff[k] + trun[k];
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const uint64_t i = cbase + (uint64_t)w * (kWave * J) + (uint64_t)j * kWave + l;
      if (i >= hi) continue;
      if (!live[j]) {
        cpos[i - lo] = 0xFFFF;
        continue;
      }
      const uint32_t s = kstart[key[j]] + wc[w * sb + key[j]] + loc[j];
      rab[s] = ab[j];
      rmeta[s] = meta[j] | ((res[j] & rmask) << 16);
      rsb[s] = (uint16_t)key[j];
      cpos[i - lo] = (uint16_t)s;
    }
    lds_barrier();
    // 4. write the chunk out super-bucket by super-bucket (contiguous runs)
    for (uint32_t s = t; s < nlive; s += kPT) {
      const uint32_t k = rsb[s];
      const uint32_t g = toff[k] + trun[k] + (s - kstart[k]);
      st_meta[g] = rmeta[s];
      st_ab[g] = rab[s];
    }
    lds_barrier();
    for (uint32_t k = t; k < sb; k += kPT) trun[k] += ctot[k];
    lds_barrier();
    if (more) {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        res[j] = nres[j];
        meta[j] = nmeta[j];
        ab[j] = nab[j];
      }
    }
  }
}

// One workgroup per 4096-commit chunk: gather the chunk's result runs (contiguous in staging order) into LDS,
// then emit results in log order through the chunk positions — every global access coalesced.
__global__ __launch_bounds__(kPT) void k_unpermute(const uint16_t* __restrict__ cpos, const uint16_t* __restrict__ ckst,
                                                const uint32_t* __restrict__ crun, uint32_t sb, uint64_t n,
                                                const uint8_t* __restrict__ rst_status,
                                                const uint64_t* __restrict__ rst_value, uint8_t* __restrict__ out_status,
                                                uint64_t* __restrict__ out_value) {
  __shared__ uint64_t lv[kChunk];
  __shared__ uint8_t ls[kChunk];
  __shared__ uint16_t kst[kMaxSb + 1];
  __shared__ uint32_t run[kMaxSb];
  const uint32_t t = threadIdx.x;
  const uint64_t c = blockIdx.x;
  const uint64_t i0 = c * kChunk;
  for (uint32_t k = t; k <= sb; k += kPT) {
    kst[k] = ckst[c * (sb + 1) + k];
    if (k < sb) run[k] = crun[c * sb + k];
  }
  lds_barrier();
  const uint32_t nlive = kst[sb];
  for (uint32_t s = t; s < nlive; s += kPT) {
    // run of s: the last k with kst[k] <= s (empty runs share their start with the next run)
    uint32_t a = 0, b = sb;  // invariant: kst[a] <= s < kst[b] (kst[sb] = nlive > s)
    while (b - a > 1) {
      const uint32_t m = (a + b) >> 1;
      if (kst[m] <= s) a = m; else b = m;
    }
    const uint32_t g = run[a] + (s - kst[a]);
    ls[s] = rst_status[g];
    lv[s] = rst_value[g];
  }
  lds_barrier();
  const uint8_t unk = CC_STATUS(CC_ST_UNKNOWN_SESSION, CC_TAG_NULL);
  const uint64_t i1 = i0 + kChunk < n ? i0 + kChunk : n;
  if (i1 - i0 == (uint64_t)kChunk) {  // full chunk: 4 commits per thread, vector stores
    const uint64_t q = i0 / 4 + t;
    const uint2 pp = reinterpret_cast<const uint2*>(cpos)[q];
    const uint16_t p[4] = {(uint16_t)(pp.x & 0xFFFF), (uint16_t)(pp.x >> 16), (uint16_t)(pp.y & 0xFFFF), (uint16_t)(pp.y >> 16)};
    uint32_t sw = 0;
    uint64_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = p[k] != 0xFFFF;
      sw |= (uint32_t)(ok ? ls[p[k]] : unk) << (8 * k);
      v[k] = ok ? lv[p[k]] : 0;
    }
    reinterpret_cast<uint32_t*>(out_status)[q] = sw;
    u64x2* ov = reinterpret_cast<u64x2*>(out_value) + 2 * q;
    ov[0] = u64x2{v[0], v[1]};
    ov[1] = u64x2{v[2], v[3]};
  } else {
    for (uint64_t i = i0 + t; i < i1; i += kPT) {
      const uint16_t p = cpos[i];
      out_status[i] = p != 0xFFFF ? ls[p] : unk;
      out_value[i] = p != 0xFFFF ? lv[p] : 0;
    }
  }
}

int launch_partition(const PartArgs& a, hipStream_t st) {
  const uint32_t tiles = (uint32_t)((a.hi - a.lo + kTile - 1) / kTile);
  if (tiles == 0) return 0;
  a.mark(K_PART_COUNT, 1, st);
  hipLaunchKernelGGL(k_part_count, dim3(tiles), dim3(kPT), a.sb * sizeof(uint32_t), st, a.inst, a.lo, a.hi, a.inst_res,
                     a.max_inst, a.sb, a.sb_shift, a.counts);
  a.mark(K_PART_COUNT, 0, st);
  a.mark(K_PART_SCAN, 1, st);
  hipLaunchKernelGGL(k_part_scan, dim3((a.sb + kWave - 1) / kWave), dim3(1024), 0, st, a.counts, tiles, a.sb, a.tot);
  a.mark(K_PART_SCAN, 0, st);
  a.mark(K_PART_BASE, 1, st);
  hipLaunchKernelGGL(k_part_base, dim3(1), dim3(1024), 0, st, a.tot, a.sb, a.base);
  a.mark(K_PART_BASE, 0, st);
  a.mark(K_PART_SCATTER, 1, st);
  hipLaunchKernelGGL(k_part_scatter, dim3(tiles), dim3(kPT), scatter_lds_bytes(a.sb), st, a.inst, a.op, a.flags, a.a, a.b,
                     a.lo, a.hi, a.inst_res, a.max_inst, a.sb, a.sb_shift, a.counts, a.base, a.st_meta, a.st_ab,
                     a.cpos, a.ckst, a.crun);
  a.mark(K_PART_SCATTER, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_unpermute(const UnpermuteArgs& a, hipStream_t st) {
  const uint64_t n = a.hi - a.lo;
  const uint64_t chunks = (n + kChunk - 1) / kChunk;
  if (chunks == 0) return 0;
  a.mark(K_UNPERMUTE, 1, st);
  hipLaunchKernelGGL(k_unpermute, dim3((uint32_t)chunks), dim3(kPT), 0, st, a.cpos, a.ckst, a.crun, a.sb, n, a.rst_status,
                     a.rst_value, a.out_status + a.lo, a.out_value + a.lo);
  a.mark(K_UNPERMUTE, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
