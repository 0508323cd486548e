// partition_value.hip — the partition of value-only engines (the c2 headline path): a stable group-by of the
// commit batch by super-bucket (256 AtomicValueState slots = one k_apply_value workgroup) into the tile-local
// staging layout of partition.hip (run of super-bucket k in tile T at T*16384 + ttab[T][k]).
//
// Reference: ResourceManager.operateResource (ResourceManager.java:56-72) resolves each commit's instance to its
// resource and hands it to that resource's state machine; commits of different resources are independent
// (ResourceManager.java:37-39), commits of one resource keep their log order.  The partition does the
// instance -> resource resolution (unknown instances are dropped here and answered UNKNOWN_SESSION by
// k_unpermute) and the per-resource ordering is kept by stability.
//
// k_tile_hist (partition.hip) has already written every tile's run starts (the ttab row).  k_part_value is
// persistent: 256 workgroups of 1024 threads walk the tiles (T = blockIdx.x + k * gridDim.x) in chunks of 4096
// commits.  Per chunk, four LDS barriers:
//   R  rank: every wave ranks its 256 commits per super-bucket with LDS atomics with return on its own counter
//      row (same-address lanes of one instruction resolve in lane order on gfx950, checked at engine start);
//   S  one wave: per super-bucket, exclusive prefix over the 16 waves, chunk totals, the chunk-sorted run starts
//      and the tile-local base of each run piece (run start + records of earlier chunks);
//   P  the sorted order of the chunk (perm) and each commit's tile-local position (cpos);
//   W  write the sorted chunk out: contiguous stores of every run piece.
// R moves the chunk from registers into an LDS buffer in log order and immediately reloads the registers with the
// next chunk (the instance column two chunks ahead, so the instance -> resource gather never waits on a fresh
// load): the loads are in flight for a whole chunk.  P only writes the sorted order (perm) and W copies from the
// log-order buffer through it.  Every global load and store of an iteration is unconditional (past-the-end rows
// read row `lo` and write the dummy rows after the staging area), so the compiler counts outstanding memory
// operations exactly and no wait lands on a prefetch.
#include "common.h"
#include "engine_internal.h"

namespace cc {

#ifdef CC_PHASE_TIMING
__device__ unsigned long long g_ph_partv[kPhases];
int phase_read_partv(uint64_t* out) {
  unsigned long long z[kPhases] = {};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ph_partv), sizeof z) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_ph_partv), z, sizeof z) != hipSuccess)
    return CC_ERR_HIP;
  return CC_OK;
}
#endif

constexpr int kVPJ = 4;                  // commits per thread per chunk
constexpr int kVPC = kVPJ * kPT;         // 4096 commits per chunk
constexpr int kVPChunks = kTile / kVPC;  // chunks per tile
constexpr uint32_t kVPDead = 1u << 31;  // meta bit of a register row: past the batch end or unknown instance

// KP = super-buckets owned per lane of the scan wave (even: whole counter pairs); sb <= 64 * KP.
template <int KP, bool RES16>
__global__ __launch_bounds__(kPT) void k_part_value(const uint32_t* __restrict__ inst, const uint16_t* __restrict__ res16,
                                                 const uint8_t* __restrict__ op,
                                                 const uint8_t* __restrict__ flags, const uint64_t* __restrict__ ca,
                                                 const uint64_t* __restrict__ cb, uint64_t lo, uint64_t hi,
                                                 uint32_t tiles, const uint32_t* __restrict__ inst_res, uint32_t max_inst,
                                                 uint32_t sb, uint64_t dummy,
                                                 uint32_t* __restrict__ st_meta, u64x2* __restrict__ st_ab,
                                                 uint16_t* __restrict__ cpos, const uint16_t* __restrict__ ttab) {
  __shared__ uint4 rawab[kVPC];               // the chunk in log order: encoded operands
  __shared__ uint32_t rawmeta[kVPC];          //   meta word (value_encode | slot-in-super-bucket << 16)
  __shared__ uint16_t perm[kVPC];             // sorted position s -> log-order index in the chunk
  __shared__ uint16_t rsb[kVPC];              // sorted position s -> super-bucket
  __shared__ uint32_t wc[2][kPW][kMaxSb / 2];  // per-wave counters (packed u16 pairs), double-buffered
  __shared__ uint32_t tpos[kMaxSb];           // tile-local position of sorted record s of run k = tpos[k] + s
  __shared__ uint16_t kst[kMaxSb];            // chunk-sorted start of run k
  __shared__ uint32_t tnext[kMaxSb];          // tile-local position of run k's next piece (run start + pieces)
  __shared__ uint32_t nlive_s;
  PH_DECL
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  const uint32_t hw = (sb + 1) / 2;
  const uint32_t total_q = (tiles - blockIdx.x + gridDim.x - 1) / gridDim.x * kVPChunks;  // this workgroup's chunks
  for (uint32_t k = t; k < 2 * kPW * (kMaxSb / 2); k += kPT) (&wc[0][0][0])[k] = 0;

  // chunk q of this workgroup: tile blockIdx.x + (q / 4) * gridDim.x, commits [base, base + 4096)
  auto tile_of = [&](uint32_t q) -> uint32_t { return blockIdx.x + (q / kVPChunks) * gridDim.x; };
  auto chunk_base = [&](uint32_t q) -> uint64_t {
    return lo + (uint64_t)tile_of(q) * kTile + (uint64_t)(q % kVPChunks) * kVPC;
  };
  // Loop-carried registers, named (register arrays end up in scratch): per j the resource r, the dead bit ok,
  // op and flags (combined only when used: no ALU right behind a load), the operands ab, and ip = the raw instance
  // of the next chunk.
#define CC_J4(X) X(0) X(1) X(2) X(3)
#define CC_DECL(J) uint32_t r##J = 0, dd##J = 1, ip##J = 0; uint16_t rs##J = 0xFFFF; uint8_t opb##J = 0, flb##J = 0; \
                   uint4 ab##J = make_uint4(0, 0, 0, 0);
  CC_J4(CC_DECL)
#undef CC_DECL
  // row i of chunk base B for j: B + w*256 + j*64 + l (log order = (w, j, l)); rows past `hi` read row `lo`
#define CC_ROW(B, J) ((B) + (uint64_t)w * (kWave * kVPJ) + (uint64_t)(J) * kWave + l)
#define CC_CLAMP(I) ((I) < hi ? (I) : lo)
#define CC_LD_INST(J) if (!RES16) { const uint64_t i = CC_ROW(bi, J); ip##J = inst[CC_CLAMP(i)]; }
  // chunk B: the instance -> resource gather (its instances ip were loaded one chunk earlier) and raw columns
#define CC_LD_RAW(J)                                                                  \
  {                                                                                   \
    const uint64_t i = CC_ROW(br, J);                                                 \
    const uint64_t ic = CC_CLAMP(i);                                                  \
    if (RES16) { /* resolved by k_tile_hist16: 0xFFFF = unknown instance */            \
      dd##J = i < hi ? 0u : 1u;                                                       \
      rs##J = res16[ic - lo];                                                         \
    } else {                                                                          \
      dd##J = (i < hi && ip##J < max_inst) ? 0u : 1u;                                 \
      r##J = inst_res[ip##J < max_inst ? ip##J : 0u];                                 \
    }                                                                                 \
    opb##J = op[ic];                                                                  \
    flb##J = flags[ic];                                                               \
    const uint64_t a_ = ca[ic], b_ = cb[ic];                                          \
    ab##J = make_uint4((uint32_t)a_, (uint32_t)(a_ >> 32), (uint32_t)b_, (uint32_t)(b_ >> 32)); \
  }
  // the run starts of the next chunk's tile (loaded with every chunk; wave 0 uses them at a tile start)
  uint16_t nrow[KP];
#define CC_LD_ROW(TT)                                                                \
  {                                                                                  \
    const uint16_t* row_ = ttab + (uint64_t)(TT) * (sb + 1);                         \
    _Pragma("unroll") for (int e = 0; e < KP; ++e) {                                 \
      const uint32_t k = l * KP + e;                                                 \
      nrow[e] = row_[k < sb ? k : sb];                                               \
    }                                                                                \
  }
#pragma unroll
  for (int e = 0; e < KP; ++e) nrow[e] = 0;
  if (total_q) {
    { const uint64_t bi = chunk_base(0); CC_J4(CC_LD_INST) }
    { const uint64_t br = chunk_base(0); CC_J4(CC_LD_RAW) }
    { const uint64_t bi = chunk_base(total_q > 1 ? 1 : 0); CC_J4(CC_LD_INST) }
    CC_LD_ROW(tile_of(0))
    // as many stores as a chunk issues after its loads (cpos 4 + write-out 8): the loop header then sees the same
    // outstanding-operation count from the prologue as from the back edge, so its waits stay exact
#pragma unroll
    for (int e = 0; e < 3 * kVPJ; ++e) reinterpret_cast<volatile uint32_t*>(st_meta)[dummy + t] = (uint32_t)e;
  }
  PH(0);

  for (uint32_t q = 0; q < total_q; ++q) {
    const uint32_t cur = q & 1;
    const uint32_t T = tile_of(q);
    const uint64_t cbase = chunk_base(q);
    lds_barrier();  // the previous chunk's write-out is done reading the raw buffer
    if (w == 0 && q % kVPChunks == 0) {  // a new tile: its run starts (k_tile_hist, loaded with the chunk)
#pragma unroll
      for (int e = 0; e < KP; ++e) {
        const uint32_t k = l * KP + e;
        if (k < sb) tnext[k] = nrow[e];
      }
    }
    // ---- R: the chunk (in registers since the previous chunk) -> encoded, into the raw LDS buffer in log order;
    //      rank inside the wave; then the registers take the next chunk's loads (in flight for a whole chunk)
    uint32_t sk[kVPJ], loc[kVPJ];
#define CC_RANK(J)                                                                              \
    {                                                                                           \
      if (RES16) r##J = rs##J == 0xFFFF ? kNoRes : (uint32_t)rs##J;                             \
      const bool live = dd##J == 0 && r##J != kNoRes;                                           \
      sk[J] = live ? (r##J >> kSbShift) : 0u;                                                   \
      const uint32_t sh = 16 * (sk[J] & 1);                                                     \
      loc[J] = live ? (atomicAdd(&wc[cur][w][sk[J] >> 1], 1u << sh) >> sh) & 0xFFFFu : 0xFFFFu; \
      uint32_t m_;                                                                              \
      u64x2 xy;                                                                                 \
      value_encode(opb##J, flb##J, (uint64_t)ab##J.x | ((uint64_t)ab##J.y << 32),               \
                   (uint64_t)ab##J.z | ((uint64_t)ab##J.w << 32), m_, xy);                      \
      const uint32_t ix = w * (kWave * kVPJ) + (J) * kWave + l;                                 \
      rawmeta[ix] = m_ | ((r##J & ((1u << kSbShift) - 1)) << 16);                               \
      rawab[ix] = make_uint4((uint32_t)xy.x, (uint32_t)(xy.x >> 32), (uint32_t)xy.y, (uint32_t)(xy.y >> 32)); \
    }
    CC_J4(CC_RANK)
#undef CC_RANK
    {
      const uint32_t q1 = q + 1 < total_q ? q + 1 : q, q2 = q + 2 < total_q ? q + 2 : q1;
      CC_LD_ROW(tile_of(q1))  // first: the compiler packs these u16 right away, they must not wait on the rest
      { const uint64_t br = chunk_base(q1); CC_J4(CC_LD_RAW) }
      { const uint64_t bi = chunk_base(q2); CC_J4(CC_LD_INST) }
    }
    for (uint32_t k = t; k < kPW * hw; k += kPT) wc[cur ^ 1][k / hw][k % hw] = 0;
    lds_barrier();
    PH(1);
    // ---- S: one wave; lane l owns super-buckets [l*KP, l*KP + KP)
    if (w == 0) {
      uint32_t tot[KP];
#pragma unroll
      for (int e = 0; e < KP; e += 2) {
        const uint32_t pr = (l * KP + e) / 2;
        uint32_t acc = 0;
        if (pr < hw) {
#pragma unroll
          for (int qq = 0; qq < kPW; ++qq) {
            const uint32_t c = wc[cur][qq][pr];
            wc[cur][qq][pr] = acc;
            acc += c;
          }
        }
        tot[e] = acc & 0xFFFFu;
        tot[e + 1] = acc >> 16;
      }
      uint32_t mine = 0;
#pragma unroll
      for (int e = 0; e < KP; ++e) mine += tot[e];
      uint32_t inc = mine;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      uint32_t ks = inc - mine;
#pragma unroll
      for (int e = 0; e < KP; ++e) {
        const uint32_t k = l * KP + e;
        if (k < sb) {
          const uint32_t tn = tnext[k];
          kst[k] = (uint16_t)ks;
          tpos[k] = tn - ks;
          tnext[k] = tn + tot[e];
        }
        ks += tot[e];
      }
      if (l == 63) nlive_s = inc;
    }
    lds_barrier();
    PH(2);
    // ---- P: sorted position of every record (perm, rsb) and every commit's tile-local position (cpos;
    //      0xFFFF: unknown instance)
    const uint64_t crel = cbase - lo;
#define CC_PLACE(J)                                                                             \
    {                                                                                           \
      uint32_t cp = 0xFFFFu;                                                                    \
      if (loc[J] != 0xFFFFu) {                                                                  \
        const uint32_t k = sk[J];                                                               \
        const uint32_t pre = (wc[cur][w][k >> 1] >> (16 * (k & 1))) & 0xFFFFu;                  \
        const uint32_t s = kst[k] + pre + loc[J];                                               \
        perm[s] = (uint16_t)(w * (kWave * kVPJ) + (J) * kWave + l);                             \
        rsb[s] = (uint16_t)k;                                                                   \
        cp = tpos[k] + s;                                                                       \
      }                                                                                         \
      cpos[crel + (CC_ROW(cbase, J) - cbase)] = (uint16_t)cp;                                   \
    }
    CC_J4(CC_PLACE)
#undef CC_PLACE
    lds_barrier();
    PH(3);
    // ---- W: contiguous stores of the sorted chunk (rows past the chunk's live count go to the dummy rows)
    {
      const uint32_t nl = nlive_s;
      const uint64_t tb = (uint64_t)T * kTile;
#pragma unroll
      for (int e = 0; e < kVPJ; ++e) {
        const uint32_t s = t + e * kPT;
        const uint32_t k = rsb[s] & (kMaxSb - 1);  // garbage past nl: not used
        const uint32_t ri = perm[s] & (kVPC - 1);
        const uint64_t g = s < nl ? tb + tpos[k] + s : dummy + t;
        st_meta[g] = rawmeta[ri];
        reinterpret_cast<uint4*>(st_ab)[g] = rawab[ri];
      }
    }
    PH(4);
  }
#undef CC_LD_ROW
#undef CC_LD_RAW
#undef CC_LD_INST
#undef CC_CLAMP
#undef CC_ROW
#undef CC_J4
  PH_FLUSH(g_ph_partv);
}

// ---- k_part_v2: the default value-only partition (one 1024-thread workgroup per 16384-commit tile) ----------------
// Differences from k_part_tile<4, false>: every thread loads the instance column of all 16 of its tile commits (the
// chunk mapping (chunk, wave, j, lane)) and chunk 0's raw columns before anything waits, resolves the 16 instances
// with one batch of gathers, builds the tile histogram from those registers and keeps the resolved resources for the
// chunks (the instance column is read once and gathered once per commit); the 4 chunks are unrolled (their
// registers stay registers); the per-chunk wave prefixes, chunk totals and run starts are one wave's work (no block
// scan), so a chunk has 4 barriers.
constexpr int kV2J = 4;                   // commits per thread per chunk
constexpr int kV2C = kV2J * kPT;          // 4096 commits per chunk
constexpr int kV2N = kTile / kV2C;        // 4 chunks per tile

template <int KP>
__global__ __launch_bounds__(kPT) void k_part_v2(const uint32_t* __restrict__ inst, const uint8_t* __restrict__ op,
                                                 const uint8_t* __restrict__ flags, const uint64_t* __restrict__ ca,
                                                 const uint64_t* __restrict__ cb, uint64_t lo, uint64_t hi,
                                                 const uint32_t* __restrict__ inst_res, uint32_t max_inst, uint32_t sb,
                                                 uint32_t* __restrict__ st_meta, u64x2* __restrict__ st_ab,
                                                 uint16_t* __restrict__ cpos, uint16_t* __restrict__ ttab) {
  __shared__ uint4 rab[kV2C];                  // the chunk in sorted order: encoded operands
  __shared__ uint32_t rmeta[kV2C];             //   meta word (value_encode | slot-in-super-bucket << 16)
  __shared__ uint16_t rsb[kV2C];               //   super-bucket
  __shared__ uint32_t wc[kPW][kMaxSb / 2];     // per-wave counters (packed u16 pairs) -> per-wave exclusive prefixes
  __shared__ uint32_t hist[kMaxSb / 2];        // tile histogram (packed u16 pairs)
  __shared__ uint16_t tpos[kMaxSb];            // tile-local position of run k's next piece
  __shared__ uint16_t kst[kMaxSb];             // chunk-sorted start of run k
  __shared__ uint32_t nlive_s;
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  PH_DECL
  const uint32_t hw = (sb + 1) / 2;
  const uint64_t tile0 = lo + (uint64_t)blockIdx.x * kTile;
  const uint32_t tbase = blockIdx.x * kTile;  // staging region of this tile (relative to lo)
  for (uint32_t k = t; k < hw; k += kPT) hist[k] = 0;
  for (uint32_t k = t; k < (uint32_t)(kPW * (kMaxSb / 2)); k += kPT) (&wc[0][0])[k] = 0;
  // commit (c, w, j, l) of the tile: tile0 + c*4096 + w*256 + j*64 + l (log order)
  auto row_of = [&](int c, int j) -> uint64_t { return tile0 + (uint64_t)c * kV2C + (uint64_t)w * (kWave * kV2J) + (uint64_t)j * kWave + l; };
  uint32_t r[kV2N][kV2J];
#pragma unroll
  for (int c = 0; c < kV2N; ++c)
#pragma unroll
    for (int j = 0; j < kV2J; ++j) {
      const uint64_t i = row_of(c, j);
      r[c][j] = i < hi ? inst[i] : kNoRes;
    }
  uint8_t ob[kV2J], fb[kV2J];
  uint64_t av[kV2J], bv[kV2J];
  auto load_raw = [&](int c) {
#pragma unroll
    for (int j = 0; j < kV2J; ++j) {
      const uint64_t i = row_of(c, j), ic = i < hi ? i : lo;
      ob[j] = op[ic];
      fb[j] = flags[ic];
      av[j] = ca[ic];
      bv[j] = cb[ic];
    }
  };
  load_raw(0);
#pragma unroll
  for (int c = 0; c < kV2N; ++c)
#pragma unroll
    for (int j = 0; j < kV2J; ++j) r[c][j] = r[c][j] < max_inst ? inst_res[r[c][j]] : kNoRes;
  lds_barrier();  // hist / wc zeroed
  PH(0);
#pragma unroll
  for (int c = 0; c < kV2N; ++c)
#pragma unroll
    for (int j = 0; j < kV2J; ++j)
      if (r[c][j] != kNoRes) {
        const uint32_t k = r[c][j] >> kSbShift;
        atomicAdd(&hist[k >> 1], 1u << (16 * (k & 1)));
      }
  lds_barrier();
  if (w == 0) {  // tile-local run starts: one wave, lane l owns super-buckets [l*KP, l*KP + KP)
    uint32_t cnt[KP], mine = 0;
#pragma unroll
    for (int e = 0; e < KP; ++e) {
      const uint32_t k = l * KP + e;
      cnt[e] = k < sb ? (hist[k >> 1] >> (16 * (k & 1))) & 0xFFFFu : 0u;
      mine += cnt[e];
    }
    uint32_t inc = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (l >= (uint32_t)d) inc += y;
    }
    uint32_t run = inc - mine;
    uint16_t* row = ttab + (uint64_t)blockIdx.x * (sb + 1);
#pragma unroll
    for (int e = 0; e < KP; ++e) {
      const uint32_t k = l * KP + e;
      if (k < sb) {
        tpos[k] = (uint16_t)run;
        row[k] = (uint16_t)run;
      }
      run += cnt[e];
    }
    if (l == 63) row[sb] = (uint16_t)inc;  // live commits of the tile (<= 16384)
  }
  PH(1);
  // (tpos is first read after the next barrier)
#pragma unroll
  for (int c = 0; c < kV2N; ++c) {
    // encode and rank this chunk's records (registers: loaded one chunk ahead); then the next chunk's loads
    uint32_t sk[kV2J], loc[kV2J], mt[kV2J];
    uint4 xy4[kV2J];
#pragma unroll
    for (int j = 0; j < kV2J; ++j) {
      const bool live = r[c][j] != kNoRes;
      u64x2 xy;
      value_encode(ob[j], fb[j], av[j], bv[j], mt[j], xy);
      mt[j] |= (r[c][j] & ((1u << kSbShift) - 1)) << 16;
      xy4[j] = make_uint4((uint32_t)xy.x, (uint32_t)(xy.x >> 32), (uint32_t)xy.y, (uint32_t)(xy.y >> 32));
      sk[j] = live ? (r[c][j] >> kSbShift) : 0u;
      const uint32_t sh = 16 * (sk[j] & 1);
      loc[j] = live ? (atomicAdd(&wc[w][sk[j] >> 1], 1u << sh) >> sh) & 0xFFFFu : 0xFFFFu;
    }
    PH(2);
    if (c + 1 < kV2N) load_raw(c + 1);
    lds_barrier();
    PH(3);
    if (w == 0) {  // per super-bucket: exclusive prefix over the waves (in place), chunk totals, chunk-sorted starts
      uint32_t tot[KP];
#pragma unroll
      for (int e = 0; e < KP; e += 2) {
        const uint32_t pr = (l * KP + e) / 2;
        uint32_t acc = 0;
        if (pr < hw) {
#pragma unroll
          for (int q = 0; q < kPW; ++q) {
            const uint32_t x = wc[q][pr];
            wc[q][pr] = acc;
            acc += x;
          }
        }
        tot[e] = acc & 0xFFFFu;
        tot[e + 1] = acc >> 16;
      }
      uint32_t mine = 0;
#pragma unroll
      for (int e = 0; e < KP; ++e) mine += tot[e];
      uint32_t inc = mine;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      uint32_t ks = inc - mine;
#pragma unroll
      for (int e = 0; e < KP; ++e) {
        const uint32_t k = l * KP + e;
        if (k < sb) kst[k] = (uint16_t)ks;
        ks += tot[e];
      }
      if (l == 63) nlive_s = inc;
    }
    lds_barrier();
    PH(4);
    // place the records in sorted order; every commit's tile-local position (0xFFFF: unknown instance)
#pragma unroll
    for (int j = 0; j < kV2J; ++j) {
      const uint64_t i = row_of(c, j);
      uint32_t cp = 0xFFFFu;
      if (loc[j] != 0xFFFFu) {
        const uint32_t k = sk[j];
        const uint32_t pre = (wc[w][k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
        const uint32_t sp = kst[k] + pre + loc[j];
        rab[sp] = xy4[j];
        rmeta[sp] = mt[j];
        rsb[sp] = (uint16_t)k;
        cp = tpos[k] + pre + loc[j];
      }
      if (i < hi) cpos[i - lo] = (uint16_t)cp;
    }
    lds_barrier();
    PH(5);
    // write the chunk out run by run (contiguous); the next chunk's counters are cleared behind the reads
    const uint32_t nl = nlive_s;
    for (uint32_t sp = t; sp < nl; sp += kPT) {
      const uint32_t k = rsb[sp];
      const uint32_t g = tbase + tpos[k] + (sp - kst[k]);
      st_meta[g] = rmeta[sp];
      reinterpret_cast<uint4*>(st_ab)[g] = rab[sp];
    }
    for (uint32_t k = t; k < (uint32_t)(kPW * hw); k += kPT) wc[k / hw][k % hw] = 0;
    lds_barrier();
    PH(6);
    if (w == 0) {  // run k's next piece starts after this chunk's records of k
#pragma unroll
      for (int e = 0; e < KP; ++e) {
        const uint32_t k = l * KP + e;
        if (k < sb) tpos[k] = (uint16_t)(tpos[k] + ((k + 1 < sb ? kst[k + 1] : nl) - kst[k]));
      }
    }
    // (tpos is next read after the next chunk's first barrier)
  }
  PH_FLUSH(g_ph_partv);
}

// inst_res (u32, kNoRes = closed) -> a u16 copy for k_tile_hist16's LDS table (0xFFFF = closed), padded to 8.
__global__ void k_res16_table(const uint32_t* __restrict__ inst_res, uint32_t n, uint32_t npad, uint16_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < npad) out[i] = i < n && inst_res[i] != kNoRes ? (uint16_t)inst_res[i] : (uint16_t)0xFFFF;
}

// Value-only engines with < 65535 resources and <= 65536 instances: the tile histograms with the instance ->
// resource table resident in LDS (128 KB of u16), persistent over tiles; the resolved resource of every commit
// goes to the u16 column res16 (sub-batch relative), which k_part_value<_, true> reads instead of re-resolving.
// The random 4-byte table lookups (one L2 request per lane) are the dominant cost of resolving in global memory.
constexpr int kHT16 = 1024;
__global__ __launch_bounds__(kHT16) void k_tile_hist16(const uint32_t* __restrict__ inst, uint64_t lo, uint64_t hi,
                                                       uint32_t tiles, const uint16_t* __restrict__ tab16, uint32_t ntab,
                                                       uint32_t sb, uint16_t* __restrict__ ttab, uint16_t* __restrict__ res16) {
  __shared__ uint16_t tab[65536];
  __shared__ uint32_t h[kMaxSb];
  __shared__ uint32_t wsum[kHT16 / kWave];
  const uint32_t t = threadIdx.x, l = t & 63, w = t >> 6;
  for (uint32_t q = t; q < ntab / 8; q += kHT16) reinterpret_cast<uint4*>(tab)[q] = reinterpret_cast<const uint4*>(tab16)[q];
  const uint32_t nt = ntab;
  for (uint32_t T = blockIdx.x; T < tiles; T += gridDim.x) {
    for (uint32_t k = t; k < sb; k += kHT16) h[k] = 0;
    __syncthreads();
    const uint64_t tile0 = lo + (uint64_t)T * kTile;
    const uint64_t tile1 = tile0 + kTile < hi ? tile0 + kTile : hi;
    constexpr int kQ = kTile / 4 / kHT16;  // 4-commit groups per thread (4)
    uint4 v[kQ];
#pragma unroll
    for (int k = 0; k < kQ; ++k) {
      const uint64_t i = tile0 + 4 * ((uint64_t)t + (uint64_t)k * kHT16);
      v[k] = i + 4 <= tile1 ? reinterpret_cast<const uint4*>(inst)[i / 4] : make_uint4(kNoRes, kNoRes, kNoRes, kNoRes);
      if (i + 4 > tile1)  // the batch's ragged end
        for (int e = 0; e < 4; ++e)
          if (i + e < tile1) (&v[k].x)[e] = inst[i + e];
    }
#pragma unroll
    for (int k = 0; k < kQ; ++k) {
      const uint64_t i = tile0 + 4 * ((uint64_t)t + (uint64_t)k * kHT16);
      const uint32_t x[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
      uint32_t rr[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        rr[e] = x[e] < nt ? tab[x[e]] : 0xFFFFu;
        if (rr[e] != 0xFFFFu) atomicAdd(&h[rr[e] >> kSbShift], 1u);
      }
      if (i < tile1)  // the tile's whole region exists in the staging column (the sub-batch is whole tiles)
        reinterpret_cast<uint2*>(res16)[(i - lo) / 4] = make_uint2(rr[0] | (rr[1] << 16), rr[2] | (rr[3] << 16));
    }
    __syncthreads();
    uint16_t* row = ttab + (uint64_t)T * (sb + 1);
    uint32_t run = 0;
    for (uint32_t k0 = 0; k0 < sb; k0 += kHT16) {  // block-uniform
      const uint32_t k = k0 + t;
      const uint32_t c = k < sb ? h[k] : 0;
      uint32_t inc = c;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      if (l == 63) wsum[w] = inc;
      __syncthreads();
      uint32_t pre = 0, all = 0;
      for (uint32_t q = 0; q < kHT16 / kWave; ++q) {
        pre += q < w ? wsum[q] : 0;
        all += wsum[q];
      }
      if (k < sb) row[k] = (uint16_t)(run + pre + inc - c);
      run += all;
      __syncthreads();
    }
    if (t == 0) row[sb] = (uint16_t)run;  // live commits of the tile (<= 16384)
  }
}

int launch_tile_hist16(const PartArgs& a, uint32_t tiles, hipStream_t st) {
  const uint32_t npad = (a.max_inst + 7) / 8 * 8;
  hipLaunchKernelGGL(k_res16_table, dim3((npad + 255) / 256), dim3(256), 0, st, a.inst_res, a.max_inst, npad, a.inst_res16);
  const uint32_t grid = tiles < (uint32_t)kPersistGrid ? tiles : (uint32_t)kPersistGrid;
  hipLaunchKernelGGL(k_tile_hist16, dim3(grid), dim3(kHT16), 0, st, a.inst, a.lo, a.hi, tiles, (const uint16_t*)a.inst_res16,
                     npad, a.sb, a.ttab, a.res16);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_part_v2(const PartArgs& a, uint32_t tiles, hipStream_t st) {
  const uint32_t kp = (a.sb + kWave - 1) / kWave;  // super-buckets per lane of the scan wave
  if (a.sb > (uint32_t)kMaxSb) return -1;
#define CC_LAUNCH(KP)                                                                                                 \
  hipLaunchKernelGGL((k_part_v2<KP>), dim3(tiles), dim3(kPT), 0, st, a.inst, a.op, a.flags, a.a, a.b, a.lo, a.hi,      \
                     a.inst_res, a.max_inst, a.sb, a.st_meta, a.st_ab, a.cpos, a.ttab)
  if (kp <= 2) CC_LAUNCH(2);
  else if (kp <= 4) CC_LAUNCH(4);
  else CC_LAUNCH(8);
#undef CC_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_part_value(const PartArgs& a, uint32_t tiles, hipStream_t st) {
  const uint32_t grid = tiles < (uint32_t)kPersistGrid ? tiles : (uint32_t)kPersistGrid;
  const uint32_t kp = (a.sb + kWave - 1) / kWave;  // super-buckets per lane of the scan wave
#define CC_LAUNCH(KP, R16)                                                                                            \
  hipLaunchKernelGGL((k_part_value<KP, R16>), dim3(grid), dim3(kPT), 0, st, a.inst, (const uint16_t*)a.res16, a.op, a.flags, \
                     a.a, a.b, a.lo, a.hi, tiles, a.inst_res, a.max_inst, a.sb, a.dummy, a.st_meta, a.st_ab, a.cpos,    \
                     (const uint16_t*)a.ttab)
  if (a.res16) {
    if (kp <= 2) CC_LAUNCH(2, true);
    else if (kp <= 4) CC_LAUNCH(4, true);
    else CC_LAUNCH(8, true);
  } else {
    if (kp <= 2) CC_LAUNCH(2, false);
    else if (kp <= 4) CC_LAUNCH(4, false);
    else CC_LAUNCH(8, false);
  }
#undef CC_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
