// partition.hip — tile-local stable group-by of a commit batch by super-bucket (256 resource slots = one apply
// workgroup), and the inverse permutation of the results.
//
// Why: the reference applies commits one at a time in log order on one thread (ResourceManager.java:56-72);
// commits on DIFFERENT resources are independent (ResourceManager multiplexes isolated state machines,
// ResourceManager.java:37-39) but commits on the SAME resource form a sequential chain.  The engine therefore
// regroups a batch so that one workgroup owns 256 resources and sees exactly their commits, in log order.
//
// Super-buckets: value resources by slot (slot >> 8, 256 slots each); map commits by hash(map, key) into
// one of 2^map_bits table regions that follow them (a map's keys are independent chains).
//
// Layout: the sub-batch is cut into 16384-commit tiles; tile t owns staging positions [t*16384, (t+1)*16384)
// and stores its live commits there sorted by super-bucket (stable, so log order within each run).  The run
// of super-bucket k in tile t starts at ttab[t][k] (tile-local); ttab[t][sb] = live commits of the tile.
// No global scan is needed: the apply workgroup of super-bucket k walks its run in every tile, in tile order.
//
//   k_part_tile  : per tile: (0) histogram of the tile over super-buckets -> tile-local run starts;
//                  (1..) chunks of 4096 commits (2048 when map commits share the batch): a stable multisplit of
//                  the chunk in LDS (ranking inside a
//                  wave by LDS atomics with return, per-wave prefix sums across the 16 waves), then the chunk is
//                  written out run by run (contiguous stores), and each commit's tile-local position -> cpos.
//   k_unpermute  : per tile: the tile's staged results are read contiguously into LDS and written back in log
//                  order through cpos (unknown sessions get UNKNOWN_SESSION here, ResourceManager.java:60-69).
#include "common.h"
#include "engine_internal.h"

#include <cstdlib>

namespace cc {

#ifdef CC_PHASE_TIMING
__device__ unsigned long long g_ph_part[kPhases], g_ph_unperm[kPhases];  // g_ph_part: k_part_tile
#endif

// ResourceManager.operateResource dispatch (ResourceManager.java:60-62): instance slot -> resource slot.
__device__ inline uint32_t resolve(const uint32_t* __restrict__ inst_res, uint32_t max_inst, uint32_t s) {
  return s < max_inst ? inst_res[s] : kNoRes;
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

// Value-only engines: the tile histogram (tile-local run starts = the ttab row) in its own launch, so that the
// partition workgroups start streaming their tile at once instead of reading it twice.  512 threads per tile,
// 32 commits each (16-byte loads of the instance column, then the instance -> resource gathers).
constexpr int kHT = 512;
__global__ __launch_bounds__(kHT) void k_tile_hist(const uint32_t* __restrict__ inst, uint64_t lo, uint64_t hi,
                                                   const uint32_t* __restrict__ inst_res, uint32_t max_inst, uint32_t sb,
                                                   uint16_t* __restrict__ ttab) {
  __shared__ uint32_t h[kMaxSb];
  __shared__ uint32_t wsum[kHT / kWave];
  const uint32_t t = threadIdx.x;
  for (uint32_t k = t; k < sb; k += kHT) h[k] = 0;
  __syncthreads();
  const uint64_t tile0 = lo + (uint64_t)blockIdx.x * kTile;
  const uint64_t tile1 = tile0 + kTile < hi ? tile0 + kTile : hi;
  const uint64_t q1 = tile1 / 4;
  constexpr int kQ = kTile / 4 / kHT;  // uint4 groups per thread (8)
  uint4 v[kQ];
#pragma unroll
  for (int k = 0; k < kQ; ++k) {
    const uint64_t q = tile0 / 4 + t + (uint64_t)k * kHT;
    v[k] = q < q1 ? reinterpret_cast<const uint4*>(inst)[q] : make_uint4(kNoRes, kNoRes, kNoRes, kNoRes);
  }
#pragma unroll
  for (int k = 0; k < kQ; ++k) {
    const uint32_t x[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t r = resolve(inst_res, max_inst, x[e]);
      if (r != kNoRes) atomicAdd(&h[r >> kSbShift], 1u);
    }
  }
  for (uint64_t i = q1 * 4 + t; i < tile1; i += kHT) {  // ragged tail (< 4 commits)
    if (i < tile0) continue;
    const uint32_t r = resolve(inst_res, max_inst, inst[i]);
    if (r != kNoRes) atomicAdd(&h[r >> kSbShift], 1u);
  }
  __syncthreads();
  uint16_t* row = ttab + (uint64_t)blockIdx.x * (sb + 1);
  uint32_t run = 0;
  for (uint32_t k0 = 0; k0 < sb; k0 += kHT) {  // block-uniform; sb <= kMaxSb
    const uint32_t k = k0 + t;
    const uint32_t c = k < sb ? h[k] : 0;
    uint32_t inc = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if ((t & 63) >= (uint32_t)d) inc += y;
    }
    __syncthreads();
    if ((t & 63) == 63) wsum[t >> 6] = inc;
    __syncthreads();
    uint32_t pre = 0, all = 0;
    for (uint32_t q = 0; q < kHT / kWave; ++q) {
      pre += q < (t >> 6) ? wsum[q] : 0;
      all += wsum[q];
    }
    if (k < sb) row[k] = (uint16_t)(run + pre + inc - c);
    run += all;
  }
  if (t == 0) row[sb] = (uint16_t)run;  // live commits of the tile (<= 16384)
}

// Per-wave counters are packed u16 pairs (a wave ranks at most 256 commits of a chunk): wc[w][k/2]; the
// per-super-bucket tile offsets, run fills, chunk totals and chunk starts are u16 (a tile holds 16384 commits).
size_t tile_lds_bytes(uint32_t sb, bool maps, size_t chunk, bool ids) {
  const size_t rec = 16 + 4 + 2 + (maps ? 4 + 8 + 8 : 0);
  const size_t hw = (sb + 1) / 2;
  const size_t hot = maps ? kHotSlots * 4 + kHotMax * (8 + 8 + 4) : 0;
  return chunk * rec + (size_t)kPW * hw * 4 + 4 * (2 * hw) * 2 + 16 * 4 + hot + (maps && ids ? chunk * 8 : 0);
}

// LDS layout (dynamic): rab[C] u64x2 | [EXT: rkey[C] u64 | ridx[C] u64 | rres[C] u32] | rmeta[C] u32 |
//   rsb[C] u16 | wc[kPW][hw] u32 | toff, trun, ctot, kstart [2hw] u16 | wsum[16] u32 |
//   [EXT: hot keys: hslot[kHotSlots] u32 | hh64[kHotMax] u64 | hkey[kHotMax] u64 | hident[kHotMax] u32]
//
// Super-bucket of a commit: value resources by slot (slot >> 8); map commits by hash(map, key tag, key) into
// the map regions that follow the value super-buckets; commits of a hot key (apply_map_hot.hip) into that
// key's own bucket after the regions.
#ifndef CC_PART_WPE
#define CC_PART_WPE 4  // waves per SIMD one 1024-thread workgroup needs
#endif
template <int J, bool EXT>
__global__ __launch_bounds__(kPT, CC_PART_WPE) void k_part_tile(const uint32_t* __restrict__ inst, const uint8_t* __restrict__ op,
                                                const uint8_t* __restrict__ flags, const uint64_t* __restrict__ ca,
                                                const uint64_t* __restrict__ cb, const uint64_t* __restrict__ ckey,
                                                const uint64_t* __restrict__ cidx, const uint64_t* __restrict__ caux,
                                                const uint64_t* __restrict__ ctime, const uint64_t* __restrict__ clock_base,
                                                uint32_t ext_flags, uint64_t lo, uint64_t hi,
                                                const uint32_t* __restrict__ inst_res, const uint8_t* __restrict__ res_type,
                                                const uint8_t* __restrict__ sb_kind, uint32_t max_inst, uint32_t sb, uint32_t sb_val, uint32_t map_bits,
                                                uint32_t sbq_base,
                                                const HotKey* __restrict__ hot, const uint32_t* __restrict__ hot_n,
                                                uint32_t* __restrict__ st_meta, u64x2* __restrict__ st_ab,
                                                uint32_t* __restrict__ st_res, uint64_t* __restrict__ st_key,
                                                uint64_t* __restrict__ st_idx, uint16_t* __restrict__ cpos,
                                                uint16_t* __restrict__ ttab) {
  constexpr int C = J * kPT;  // commits per chunk
  extern __shared__ __align__(16) uint8_t smem[];
  u64x2* rab = reinterpret_cast<u64x2*>(smem);
  uint64_t* rkey = reinterpret_cast<uint64_t*>(rab + C);
  uint64_t* ridx = rkey + (EXT ? C : 0);
  uint32_t* rres = reinterpret_cast<uint32_t*>(ridx + (EXT ? C : 0));
  uint32_t* rmeta = rres + (EXT ? C : 0);
  uint16_t* rsb = reinterpret_cast<uint16_t*>(rmeta + C);
  uint32_t* wc = reinterpret_cast<uint32_t*>(rsb + C);  // [kPW][hw] packed u16 pairs
  const uint32_t hw = (sb + 1) / 2;
  uint16_t* toff = reinterpret_cast<uint16_t*>(wc + kPW * hw);
  uint16_t* trun = toff + 2 * hw;
  uint16_t* ctot = trun + 2 * hw;
  uint16_t* kstart = ctot + 2 * hw;
  uint32_t* wsum = reinterpret_cast<uint32_t*>(kstart + 2 * hw);
  uint32_t* ctot32 = reinterpret_cast<uint32_t*>(ctot);  // packed view for LDS atomics
  uint32_t* hslot = wsum + 16;
  uint64_t* hh64 = reinterpret_cast<uint64_t*>(hslot + (EXT ? kHotSlots : 0));
  uint64_t* hkey = hh64 + kHotMax;
  uint32_t* hident = reinterpret_cast<uint32_t*>(hkey + kHotMax);

  PH_DECL
  uint32_t nhot = 0;
  const uint64_t cbase0 = EXT && clock_base ? *clock_base : 0;
  const bool deferred = (ext_flags & kExtDeferred) != 0;
  if (EXT && map_bits) {
    nhot = *hot_n;
    for (uint32_t q = threadIdx.x; q < kHotSlots; q += kPT) hslot[q] = 0xFFFFFFFFu;
    if (threadIdx.x < nhot) {
      const HotKey hk = hot[threadIdx.x];
      hh64[threadIdx.x] = hk.h64;
      hkey[threadIdx.x] = hk.key;
      hident[threadIdx.x] = hk.ident;
    }
    lds_barrier();
    if (threadIdx.x < nhot) {
      uint32_t q = (uint32_t)(hh64[threadIdx.x] >> 32) & (kHotSlots - 1);
      while (atomicCAS(&hslot[q], 0xFFFFFFFFu, threadIdx.x) != 0xFFFFFFFFu) q = (q + 1) & (kHotSlots - 1);
    }
  }
  const uint32_t sb_hot = sb_val + (EXT && map_bits ? (1u << map_bits) : 0u);
  auto route = [&](uint32_t r, uint32_t f, uint64_t key) -> uint32_t {
    if (EXT && is_keyed(res_type[r])) {
      const uint32_t kt = CC_FLAG_KTAG(f);
      const uint64_t h = map_hash(r, kt, key);
      if (nhot) {
        const uint32_t id = mw_ident(r, kt);
        for (uint32_t q = (uint32_t)(h >> 32) & (kHotSlots - 1);; q = (q + 1) & (kHotSlots - 1)) {
          const uint32_t x = hslot[q];
          if (x == 0xFFFFFFFFu) break;
          if (hh64[x] == h && hident[x] == id && hkey[x] == key) return sb_hot + x;
        }
      }
      return sb_val + (uint32_t)(h >> (64 - map_bits));
    }
    if (EXT && sbq_base && sb_kind[r >> kSbShift]) return sbq_base + (r >> 6);  // quarter bucket (k_apply_coord)
    return r >> kSbShift;
  };
  auto hist_add = [&](uint32_t k) { atomicAdd(&ctot32[k >> 1], 1u << (16 * (k & 1))); };

  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  const uint64_t tile0 = lo + (uint64_t)blockIdx.x * kTile;
  const uint64_t tile1 = tile0 + kTile < hi ? tile0 + kTile : hi;
  const uint32_t tbase = blockIdx.x * kTile;  // staging region of this tile (relative to lo)

  // 0. histogram of the whole tile -> tile-local run starts (ttab row)
  for (uint32_t k = t; k < hw; k += kPT) ctot32[k] = 0;
  lds_barrier();
  if (!EXT) {
    const uint64_t q1 = tile1 / 4;
#pragma unroll 4
    for (uint64_t q = tile0 / 4 + t; q < q1; q += kPT) {
      const uint4 v = reinterpret_cast<const uint4*>(inst)[q];
      const uint32_t r0 = resolve(inst_res, max_inst, v.x), r1 = resolve(inst_res, max_inst, v.y);
      const uint32_t r2 = resolve(inst_res, max_inst, v.z), r3 = resolve(inst_res, max_inst, v.w);
      if (r0 != kNoRes) hist_add(r0 >> kSbShift);
      if (r1 != kNoRes) hist_add(r1 >> kSbShift);
      if (r2 != kNoRes) hist_add(r2 >> kSbShift);
      if (r3 != kNoRes) hist_add(r3 >> kSbShift);
    }
    for (uint64_t i = q1 * 4 + t; i < tile1; i += kPT) {  // ragged tail (< 4 commits)
      const uint32_t r = resolve(inst_res, max_inst, inst[i]);
      if (r != kNoRes) hist_add(r >> kSbShift);
    }
  } else {
#pragma unroll 4
    for (uint64_t i = tile0 + t; i < tile1; i += kPT) {
      const uint32_t r = resolve(inst_res, max_inst, inst[i]);
      if (r == kNoRes) continue;
      const bool m = is_keyed(res_type[r]);
      hist_add(route(r, m ? flags[i] : 0u, m ? ckey[i] : 0ull));
    }
  }
  lds_barrier();
  {
    uint16_t* row = ttab + (uint64_t)blockIdx.x * (sb + 1);
    uint32_t run = 0;
    for (uint32_t k0 = 0; k0 < sb; k0 += kPT) {  // block-uniform
      const uint32_t k = k0 + t;
      uint32_t part;
      const uint32_t ex = block_exscan(k < sb ? ctot[k] : 0, wsum, &part);
      if (k < sb) {
        toff[k] = run + ex;
        trun[k] = 0;
        row[k] = (uint16_t)(run + ex);
      }
      run += part;
    }
    if (t == 0) row[sb] = (uint16_t)run;  // live commits of the tile (<= 16384)
  }
  PH(0);

  // commit (w, j, l) of a chunk is cbase + w*(64*J) + j*64 + l: log order = (w, j, l).
  // Prefetch in two stages so no wave stalls on the instance->resource gather right after its load:
  // raw columns of chunk c+1 are requested at the top of chunk c, their gathers after chunk c's ranking.
  uint32_t res[J], meta[J], ninst[J], nmeta[J], xs[J], nxs[J];
  u64x2 ab[J], nab[J];
  uint64_t key[J], idx[J], nkey[J], nidx[J];
  auto load_raw = [&](uint64_t cbase, uint32_t (&in)[J], uint32_t (&mt)[J], u64x2 (&aa)[J], uint64_t (&kk)[J],
                      uint64_t (&ii)[J]) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const uint64_t i = cbase + (uint64_t)w * (kWave * J) + (uint64_t)j * kWave + l;
      in[j] = kNoRes;
      mt[j] = 0;
      aa[j] = u64x2{0, 0};
      kk[j] = 0;
      ii[j] = 0;
      if (i < hi) {
        in[j] = inst[i];
        mt[j] = (uint32_t)op[i] | ((uint32_t)flags[i] << 8);
        aa[j].x = ca[i];
        aa[j].y = cb[i];
      }
    }
  };
  // gathers: instance -> resource; with extended staging (maps, coordination, value events) the log index and
  // per type: map key + ttl sign; lock (clock at which due timeouts fire, timeout) + clock; others the key.
  // xs = the record's extended slot word: the map slot for map commits, the instance slot otherwise.
  // Records for k_apply_value are encoded for its walk (common.h value_encode).
  auto gather = [&](uint64_t cbase, const uint32_t (&in)[J], uint32_t (&rr)[J], uint32_t (&mt)[J], u64x2 (&aa)[J],
                    uint64_t (&kk)[J], uint64_t (&ii)[J], uint32_t (&xx)[J]) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      rr[j] = in[j] == kNoRes ? kNoRes : resolve(inst_res, max_inst, in[j]);
      xx[j] = in[j];
      if (!EXT && rr[j] != kNoRes) value_encode(mt[j] & 0xFF, (mt[j] >> 8) & 0xFF, aa[j].x, aa[j].y, mt[j], aa[j]);
      if (EXT && rr[j] != kNoRes) {
        const uint32_t ty = res_type[rr[j]];
        const uint64_t i = cbase + (uint64_t)w * (kWave * J) + (uint64_t)j * kWave + l;
        if (is_keyed(ty)) {
          if (ty == CC_RES_SET) {  // a set element is a map key holding Boolean TRUE (SetState.java:49-66)
            const uint32_t mop = set_as_map_op(mt[j] & 0xFF);
            uint32_t fl = (mt[j] >> 8) & 0xFF;
            if (mop == CC_OP_MAP_PUTIFABSENT) {
              fl = (fl & ~7u) | CC_TAG_BOOL;
              aa[j].x = 1;
            }
            mt[j] = (mt[j] & ~0xFFFFu) | mop | (fl << 8);
          } else if (ty == CC_RES_MULTIMAP) {  // a multimap key is a map key holding Boolean TRUE
            uint32_t fl = (mt[j] >> 8) & 0xFF;
            const uint32_t mop = mmap_as_map_op(mt[j] & 0xFF, fl & 7u);
            if (mop == CC_OP_MAP_PUTIFABSENT) {
              fl = (fl & ~7u) | CC_TAG_BOOL;
              aa[j].x = 1;
            }
            mt[j] = (mt[j] & ~0xFFFFu) | mop | (fl << 8);
          }
          kk[j] = ckey[i];
          ii[j] = cidx ? cidx[i] : 0;
          xx[j] = rr[j];
          if (caux && (int64_t)caux[i] > 0 && ty != CC_RES_MULTIMAP) mt[j] |= kMetaTtl;
        } else if (ty == CC_RES_VALUE && !sb_kind[rr[j] >> kSbShift]) {
          value_encode(mt[j] & 0xFF, (mt[j] >> 8) & 0xFF, aa[j].x, aa[j].y, mt[j], aa[j]);
        } else {
          ii[j] = cidx ? cidx[i] : 0;
          if (ty == CC_RES_LOCK) {  // deterministic log clock (time is non-decreasing within a batch)
            const uint64_t ti = ctime ? ctime[i] : 0;
            const uint64_t clk = ti > cbase0 ? ti : cbase0;
            uint64_t prev = cbase0;
            if (i > 0 && ctime) prev = ctime[i - 1] > cbase0 ? ctime[i - 1] : cbase0;
            aa[j].x = deferred ? prev : clk;
            aa[j].y = caux ? caux[i] : 0;
            kk[j] = clk;
          } else {
            kk[j] = ckey ? ckey[i] : 0;
          }
        }
      }
    }
  };
  load_raw(tile0, ninst, meta, ab, key, idx);
  gather(tile0, ninst, res, meta, ab, key, idx, xs);
  for (uint32_t ch = 0; ch < kTile / C; ++ch) {
    const uint64_t cbase = tile0 + (uint64_t)ch * C;
    if (cbase >= hi) break;  // block-uniform
    const bool more = ch + 1 < kTile / C && cbase + C < hi;
    if (more) load_raw(cbase + C, ninst, nmeta, nab, nkey, nidx);
    for (uint32_t k = t; k < kPW * hw; k += kPT) wc[k] = 0;
    lds_barrier();
    PH(6);
    // 1. rank by super-bucket inside each wave: the wave's own counter table, LDS atomics with return
    //    (same-address lanes of one instruction resolve in lane order on gfx950 — checked at engine start)
    uint32_t sk[J], loc[J];
    bool live[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      live[j] = res[j] != kNoRes;
      sk[j] = live[j] ? route(res[j], (meta[j] >> 8) & 0xFF, key[j]) : 0;
      const uint32_t sh = 16 * (sk[j] & 1);
      loc[j] = live[j] ? (atomicAdd(&wc[w * hw + (sk[j] >> 1)], 1u << sh) >> sh) & 0xFFFF : 0;
    }
    uint32_t nres[J];
    if (more) gather(cbase + C, ninst, nres, nmeta, nab, nkey, nidx, nxs);
    lds_barrier();
    PH(1);
    // 2. per super-bucket: exclusive prefix over waves (packed halves) and chunk totals; chunk-sorted starts
    for (uint32_t kw = t; kw < hw; kw += kPT) {
      uint32_t r0 = 0, r1 = 0;
      for (uint32_t q = 0; q < kPW; ++q) {
        const uint32_t c = wc[q * hw + kw];
        wc[q * hw + kw] = r0 | (r1 << 16);
        r0 += c & 0xFFFF;
        r1 += c >> 16;
      }
      ctot32[kw] = r0 | (r1 << 16);
    }
    lds_barrier();
    PH(2);
    uint32_t nlive = 0;
    for (uint32_t k0 = 0; k0 < sb; k0 += kPT) {  // block-uniform
      const uint32_t k = k0 + t;
      uint32_t part;
      const uint32_t ex = block_exscan(k < sb ? ctot[k] : 0, wsum, &part);
      if (k < sb) kstart[k] = nlive + ex;
      nlive += part;
    }
    lds_barrier();
    PH(3);
    // 3. place records in LDS in sorted order; per-commit tile-local position
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const uint64_t i = cbase + (uint64_t)w * (kWave * J) + (uint64_t)j * kWave + l;
      if (i >= hi) continue;
      if (!live[j]) {
        cpos[i - lo] = 0xFFFF;
        continue;
      }
      const uint32_t pre = (wc[w * hw + (sk[j] >> 1)] >> (16 * (sk[j] & 1))) & 0xFFFF;
      const uint32_t within = pre + loc[j];
      const uint32_t s = kstart[sk[j]] + within;
      rab[s] = ab[j];
      rmeta[s] = meta[j] | ((res[j] & ((1u << kSbShift) - 1)) << 16);
      rsb[s] = (uint16_t)sk[j];
      if (EXT) {
        rres[s] = xs[j];
        rkey[s] = key[j];
        ridx[s] = idx[j];
      }
      cpos[i - lo] = (uint16_t)(toff[sk[j]] + trun[sk[j]] + within);
    }
    lds_barrier();
    PH(4);
    // 4. write the chunk out run by run (contiguous)
    for (uint32_t s = t; s < nlive; s += kPT) {
      const uint32_t k = rsb[s];
      const uint32_t g = tbase + toff[k] + trun[k] + (s - kstart[k]);
      st_meta[g] = rmeta[s];
      st_ab[g] = rab[s];
      if (EXT) {
        st_res[g] = rres[s];
        st_key[g] = rkey[s];
        st_idx[g] = ridx[s];
      }
    }
    lds_barrier();
    PH(5);
    for (uint32_t k = t; k < sb; k += kPT) trun[k] += ctot[k];
    if (more) {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        res[j] = nres[j];
        meta[j] = nmeta[j];
        ab[j] = nab[j];
        key[j] = nkey[j];
        idx[j] = nidx[j];
        xs[j] = nxs[j];
      }
    }
  }
  PH_FLUSH(g_ph_part);
}

// Persistent over tiles (tile T = blockIdx.x + k * gridDim.x): the tile's staged results (contiguous, tile-local)
// are in LDS while they are written back in log order through cpos; the NEXT tile's results and cpos are loaded
// into registers (16-byte loads) during that scatter and moved to LDS at the top of the next iteration.
// NT threads per workgroup, TL commits per tile: (1024, 16384) for the shared pipeline, (512, 8192) for value_path.hip.
template <int NT, int TL>
__global__ __launch_bounds__(NT) void k_unpermute(const uint16_t* __restrict__ cpos, uint32_t tiles, uint64_t n,
                                                const uint8_t* __restrict__ rst_status,
                                                const uint64_t* __restrict__ rst_value, uint8_t* __restrict__ out_status,
                                                uint64_t* __restrict__ out_value, uint8_t* __restrict__ dummy_status,
                                                uint64_t* __restrict__ dummy_value) {
  constexpr int kUnVal = TL / (2 * NT);  // u64x2 value loads per thread per tile (8)
  constexpr int kUnPos = TL / (4 * NT);  // 4-commit cpos groups per thread per tile (4)
  __shared__ uint4 lv2[TL / 2];
  __shared__ uint4 ls4[TL / 16];
  PH_DECL
  const uint64_t* lv = reinterpret_cast<const uint64_t*>(lv2);
  const uint8_t* ls = reinterpret_cast<const uint8_t*>(ls4);
  const uint32_t t = threadIdx.x;
  // Prefetch registers as named scalars (an array here is kept in scratch by the compiler, which would make
  // every prefetch wait).  Staging buffers hold whole tiles (the sub-batch is a multiple of TL): full-tile
  // loads stay in bounds; the prefetch is unconditional (the last tile is re-read).
  static_assert(kUnVal == 8 && kUnPos == 4, "unpermute prefetch registers");
  uint4 rs, v0, v1, v2, v3, v4, v5, v6, v7;
  uint2 p0, p1, p2, p3;
  auto load = [&](uint32_t TT) {
    const uint64_t i0 = (uint64_t)TT * TL;
    const uint4* sv = reinterpret_cast<const uint4*>(rst_value + i0) + t;
    const uint2* sp = reinterpret_cast<const uint2*>(cpos + i0) + t;
    rs = reinterpret_cast<const uint4*>(rst_status + i0)[t];
    v0 = sv[0 * NT]; v1 = sv[1 * NT]; v2 = sv[2 * NT]; v3 = sv[3 * NT];
    v4 = sv[4 * NT]; v5 = sv[5 * NT]; v6 = sv[6 * NT]; v7 = sv[7 * NT];
    p0 = sp[0 * NT]; p1 = sp[1 * NT]; p2 = sp[2 * NT]; p3 = sp[3 * NT];
  };
  uint32_t T = blockIdx.x;
  load(T < tiles ? T : tiles - 1);
  const uint8_t unk = CC_STATUS(CC_ST_UNKNOWN_SESSION, CC_TAG_NULL);
  uint64_t tail_i = ~0ull, tail_v0 = 0, tail_v1 = 0, tail_v2 = 0;
  uint32_t tail_sw = 0;
  for (; T < tiles; T += gridDim.x) {
    lds_barrier();  // the previous tile's scatter is done reading LDS
    ls4[t] = rs;
    lv2[t + 0 * NT] = v0; lv2[t + 1 * NT] = v1; lv2[t + 2 * NT] = v2; lv2[t + 3 * NT] = v3;
    lv2[t + 4 * NT] = v4; lv2[t + 5 * NT] = v5; lv2[t + 6 * NT] = v6; lv2[t + 7 * NT] = v7;
    const uint2 pp[kUnPos] = {p0, p1, p2, p3};
    lds_barrier();
    PH(0);
    load(T + gridDim.x < tiles ? T + gridDim.x : tiles - 1);
    const uint64_t i0 = (uint64_t)T * TL;
    // 4-commit groups wholly inside the batch go to the outputs; the others to the dummy rows (unconditional
    // stores: see k_part_value), and the one group that straddles the batch end is written after the loop
#pragma unroll
    for (int k = 0; k < kUnPos; ++k) {
      const uint64_t i = i0 + 4 * (uint64_t)(t + k * NT);  // commits i .. i+3
      const uint32_t p[4] = {pp[k].x & 0xFFFF, pp[k].x >> 16, pp[k].y & 0xFFFF, pp[k].y >> 16};
      uint32_t sw = 0;
      uint64_t v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = p[q] != 0xFFFF;
        sw |= (uint32_t)(ok ? ls[p[q]] : unk) << (8 * q);
        v[q] = ok ? lv[p[q]] : 0;
      }
      const bool in = i + 4 <= n;
      uint32_t* os = in ? reinterpret_cast<uint32_t*>(out_status) + i / 4 : reinterpret_cast<uint32_t*>(dummy_status) + t;
      u64x2* ov = in ? reinterpret_cast<u64x2*>(out_value) + i / 2 : reinterpret_cast<u64x2*>(dummy_value) + 2 * t;
      *os = sw;
      ov[0] = u64x2{v[0], v[1]};
      ov[1] = u64x2{v[2], v[3]};
      if (!in && i < n) {  // the straddling group (at most one in the grid): remember it for after the loop
        tail_sw = sw;
        tail_v0 = v[0];
        tail_v1 = v[1];
        tail_v2 = v[2];
        tail_i = i;
      }
    }
    PH(1);
  }
  if (tail_i != ~0ull) {  // commits tail_i .. n-1 (1 to 3 of them)
    const uint64_t vv[3] = {tail_v0, tail_v1, tail_v2};
    for (int q = 0; q < 3 && tail_i + q < n; ++q) {
      out_status[tail_i + q] = (uint8_t)(tail_sw >> (8 * q));
      out_value[tail_i + q] = vv[q];
    }
  }
  PH_FLUSH(g_ph_unperm);
}

int phase_read_value(uint64_t* out);
int phase_read_partv(uint64_t* out);
int phase_read_coord(uint64_t* out);
int phase_read_map(uint64_t* out);
int phase_read_partx(uint64_t* out);
int phase_read_v3(int kernel, uint64_t* out);
int phase_read(int kernel, uint64_t* out) {
#ifdef CC_PHASE_TIMING
  if ((kernel == K_PART_TILE || kernel == K_APPLY_VALUE) && getenv("CC_V3_PHASES")) return phase_read_v3(kernel, out);
  if (kernel == K_APPLY_VALUE) return phase_read_value(out);
  if (kernel == K_APPLY_MAP) return phase_read_map(out);
  if (kernel == K_PART_TILE && getenv("CC_PART_EXT_PHASES")) return phase_read_partx(out);
  if (kernel == K_APPLY_COORD) return phase_read_coord(out);
  if (kernel == K_PART_TILE && (getenv("CC_PART_VALUE") || getenv("CC_PART_V2_PHASES"))) return phase_read_partv(out);
  unsigned long long z[kPhases] = {};
  if (kernel != K_UNPERMUTE && kernel != K_PART_TILE) return CC_ERR_INVALID;
  const void* sym = kernel == K_PART_TILE ? HIP_SYMBOL(g_ph_part) : HIP_SYMBOL(g_ph_unperm);
  if (hipMemcpyFromSymbol(out, sym, sizeof z) != hipSuccess || hipMemcpyToSymbol(sym, z, sizeof z) != hipSuccess)
    return CC_ERR_HIP;
  return CC_OK;
#else
  (void)kernel;
  (void)out;
  return CC_ERR_UNSUPPORTED;
#endif
}

int launch_partition(const PartArgs& a, hipStream_t st) {
  const uint32_t tiles = (uint32_t)((a.hi - a.lo + kTile - 1) / kTile);
  if (tiles == 0) return 0;
  const bool ext = a.ext;
  a.mark(K_PART_TILE, 1, st);
  if (!ext && a.v3) {  // value_path.hip: 8192-commit tiles
    const int rc = launch_part_v3(a, (uint32_t)((a.hi - a.lo + kV3Tile - 1) / kV3Tile), st);
    a.mark(K_PART_TILE, 0, st);
    return rc;
  }
  static const bool part_value = getenv("CC_PART_VALUE") != nullptr;  // experiment: persistent value partition
  static const bool part_tile_v1 = getenv("CC_PART_V1") != nullptr;   // A/B: the previous value partition
  if (!ext && part_value) {  // tile histograms, then the persistent value partition (partition_value.hip)
    if (a.res16) {
      if (launch_tile_hist16(a, tiles, st)) return -1;
    } else {
      hipLaunchKernelGGL(k_tile_hist, dim3(tiles), dim3(kHT), 0, st, a.inst, a.lo, a.hi, a.inst_res, a.max_inst, a.sb, a.ttab);
    }
    if (launch_part_value(a, tiles, st)) return -1;
  } else if (!ext && !part_tile_v1) {  // value-only engines: partition_value.hip k_part_v2
    if (launch_part_v2(a, tiles, st)) return -1;
  } else if (!ext) {
    hipLaunchKernelGGL((k_part_tile<kChunk / kPT, false>), dim3(tiles), dim3(kPT), tile_lds_bytes(a.sb, false, kChunk), st, a.inst,
                       a.op, a.flags, a.a, a.b, a.key, a.index, a.aux, a.time, a.clock_base, a.ext_flags, a.lo, a.hi, a.inst_res, a.res_type, a.sb_kind, a.max_inst, a.sb,
                       a.sb_val, a.map_bits, a.sbq_base, a.hot, a.hot_n, a.st_meta, a.st_ab, nullptr, nullptr, nullptr, a.cpos, a.ttab);
  } else {  // extended staging: partition_ext.hip k_part_ext
    if (launch_part_ext(a, tiles, st)) return -1;
  }
  a.mark(K_PART_TILE, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_unpermute(const UnpermuteArgs& a, hipStream_t st) {
  const uint64_t n = a.hi - a.lo;
  const uint64_t tiles = (n + kTile - 1) / kTile;
  if (tiles == 0) return 0;
  a.mark(K_UNPERMUTE, 1, st);
  if (a.v3) {  // value_path.hip tiles: two 512-thread workgroups per CU
    const uint64_t t3 = (n + kV3Tile - 1) / kV3Tile;
    const uint32_t grid = (uint32_t)(t3 < 2 * kPersistGrid ? t3 : 2 * kPersistGrid);
    hipLaunchKernelGGL((k_unpermute<512, kV3Tile>), dim3(grid), dim3(512), 0, st, a.cpos, (uint32_t)t3, n, a.rst_status,
                       a.rst_value, a.out_status + a.lo, a.out_value + a.lo, a.dummy_status, a.dummy_value);
  } else {
    const uint32_t grid = (uint32_t)(tiles < kPersistGrid ? tiles : kPersistGrid);
    hipLaunchKernelGGL((k_unpermute<kPT, kTile>), dim3(grid), dim3(kPT), 0, st, a.cpos, (uint32_t)tiles, n, a.rst_status,
                       a.rst_value, a.out_status + a.lo, a.out_value + a.lo, a.dummy_status, a.dummy_value);
  }
  a.mark(K_UNPERMUTE, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
