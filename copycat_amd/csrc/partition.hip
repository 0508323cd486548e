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
//   the partition : k_part_ext (partition_ext.hip; engines with maps / coordination / value events) or k_part_v4
//                   (value_path.hip; value-only engines): a stable multisplit of each tile in LDS, the tile's
//                   records written run by run, each commit's tile-local position -> cpos.
//   k_unpermute  : per tile: the tile's staged results are read contiguously into LDS and written back in log
//                  order through cpos (unknown sessions get UNKNOWN_SESSION here, ResourceManager.java:60-69).
#include "common.h"
#include "engine_internal.h"

#include <cstdlib>

namespace cc {

#ifdef CC_PHASE_TIMING
__device__ unsigned long long g_ph_part[kPhases], g_ph_unperm[kPhases];  // g_ph_part: k_part_tile
#endif

// Per-wave counters are packed u16 pairs (a wave ranks at most 256 commits of a chunk): wc[w][k/2]; the
// per-super-bucket tile offsets, run fills, chunk totals and chunk starts are u16 (a tile holds 16384 commits).
size_t tile_lds_bytes(uint32_t sb, bool maps, size_t chunk, bool ids) {
  const size_t rec = 16 + 4 + 2 + (maps ? 4 + 8 + 8 : 0);
  const size_t hw = (sb + 1) / 2;
  const size_t hot = maps ? kHotSlots * 4 + kHotMax * (8 + 8 + 4) : 0;
  return chunk * rec + (size_t)kPW * hw * 4 + 4 * (2 * hw) * 2 + 16 * 4 + hot + (maps && ids ? chunk * 8 : 0);
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
int phase_read_coord(uint64_t* out);
int phase_read_map(uint64_t* out);
int phase_read_small(uint64_t* out);
int phase_read_partx(uint64_t* out);
int phase_read_v3(int kernel, uint64_t* out);
int phase_read(int kernel, uint64_t* out) {
#ifdef CC_PHASE_TIMING
  if ((kernel == K_PART_TILE || kernel == K_APPLY_VALUE) && getenv("CC_V3_PHASES")) return phase_read_v3(kernel, out);
  if (kernel == K_APPLY_VALUE) return phase_read_value(out);
  if (kernel == K_APPLY_MAP && getenv("CC_SMALL_PHASES")) return phase_read_small(out);
  if (kernel == K_APPLY_MAP) return phase_read_map(out);
  if (kernel == K_PART_TILE && getenv("CC_PART_EXT_PHASES")) return phase_read_partx(out);
  if (kernel == K_APPLY_COORD) return phase_read_coord(out);
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
  a.mark(K_PART_TILE, 1, st);
  // value-only engines: value_path.hip k_part_v4 (8192-commit tiles); else partition_ext.hip k_part_ext
  const int rc = a.ext ? launch_part_ext(a, tiles, st)
                       : launch_part_v3(a, (uint32_t)((a.hi - a.lo + kV3Tile - 1) / kV3Tile), st);
  a.mark(K_PART_TILE, 0, st);
  return rc;
}

int launch_unpermute(const UnpermuteArgs& a, hipStream_t st) {
  const uint64_t n = a.hi - a.lo;
  const uint64_t tiles = (n + kTile - 1) / kTile;
  if (tiles == 0) return 0;
  a.mark(K_UNPERMUTE, 1, st);
  if (a.v3) {  // value_path.hip: packed result words over the records (k_unpermute_v3)
    if (launch_unpermute_v3(a, a.words, st)) return -1;
  } else {
    const uint32_t grid = (uint32_t)(tiles < kPersistGrid ? tiles : kPersistGrid);
    hipLaunchKernelGGL((k_unpermute<kPT, kTile>), dim3(grid), dim3(kPT), 0, st, a.cpos, (uint32_t)tiles, n, a.rst_status,
                       a.rst_value, a.out_status + a.lo, a.out_value + a.lo, a.dummy_status, a.dummy_value);
  }
  a.mark(K_UNPERMUTE, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
