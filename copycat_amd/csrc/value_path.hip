// value_path.hip — the value-only engine pipeline (the c2 headline): k_part_v4 -> k_apply_value_v3 -> k_unpermute.
//
// A stable group-by of the sub-batch by super-bucket (256 AtomicValueState slots), one walk per slot in log order,
// then the results back to log order, shaped for HBM bytes and CU occupancy:
//
//  * one 8-byte staging record per commit: the meta (slot, op class, the two value tags) and the operands packed as
//    small two's complement numbers (the CAS update as a difference from the expected value); a commit whose
//    operands do not fit keeps its row in the tile instead and the apply reads them from the batch's a / b columns;
//  * 8192-commit tiles, each ranked whole in one persistent 1024-thread workgroup per CU and written out of an LDS
//    image in full lines; the apply walks each slot in registers while loader waves stage the next chunk.
//
// Reference semantics are AtomicValueState's (atomic/src/main/java/io/atomix/atomic/state/AtomicValueState.java):
// get :77-83, set :114-118, compareAndSet :123-133, getAndSet :138-144, delete :146-157; dispatch and unknown
// sessions ResourceManager.operateResource :56-72 (UNKNOWN_SESSION rows are answered by the unpermute).
#include "common.h"
#include "engine_internal.h"

namespace cc {

#ifdef CC_PHASE_TIMING  // diagnostics build: phase clocks of k_part_v4 (g_ph_v3p) and k_apply_value_v3 (g_ph_v3a)
__device__ unsigned long long g_ph_v3p[kPhases], g_ph_v3a[kPhases];
int phase_read_v3(int kernel, uint64_t* out) {
  unsigned long long z[kPhases] = {};
  const void* sym = kernel == K_PART_TILE ? HIP_SYMBOL(g_ph_v3p) : HIP_SYMBOL(g_ph_v3a);
  if (hipMemcpyFromSymbol(out, sym, sizeof z) != hipSuccess || hipMemcpyToSymbol(sym, z, sizeof z) != hipSuccess)
    return CC_ERR_HIP;
  return CC_OK;
}
#endif


// ---- the 8-byte value record -------------------------------------------------------------------------------
// w = meta (18 bits) | payload (46 bits) << 18
//   meta: slot-in-super-bucket 0..7 | class 8..10 | compare tag 11..13 | new tag 14..16 | escaped 17
//   payload, set / getAndSet: the canonical new value as a 46-bit two's complement number (sign-extended back);
//            CAS: the canonical expected value as a 32-bit two's complement number | (update - expected) as a 14-bit
//            one << 32;
//            escaped (an operand that does not fit): the commit's row in its 8192-commit tile; the apply reads the
//            operands from the batch's a / b columns there (exact for every input; only the bytes moved differ).
// A DistributedAtomicLong CAS loop (DistributedAtomicLong.java:117-146) expects a value the resource holds and updates
// it by a small delta, so its records never escape while the values stay within +-2^31; the 16-byte record of round 3
// (full expected value + 33-bit delta) moved 8 more bytes per commit through the partition's writes and the apply's
// reads.
enum : uint32_t { kC3Get = 0, kC3Set = 1, kC3Cas = 2, kC3Gas = 3, kC3Del = 4, kC3Lis = 5, kC3Unk = 6 };
constexpr int kV3ExpBits = 32, kV3DeltaBits = 14, kV3SetBits = 46;
static_assert(kV3ExpBits + kV3DeltaBits == kV3SetBits && 18 + kV3SetBits == 64, "the record's payload field");
static_assert(kV3Tile <= (1 << 13), "the record's row field");

__device__ inline bool v3_fits(uint64_t x, int bits) {  // x == sign-extension of its low `bits` bits
  return (uint64_t)(((int64_t)(x << (64 - bits))) >> (64 - bits)) == x;
}

// (An escaped record's row, < 8192, is ORed in where the partition places the record: v3_set_row.)
__device__ inline uint64_t v3_encode(uint32_t op, uint32_t flags, uint64_t a, uint64_t b, uint32_t slot) {
  const uint32_t ta = CC_FLAG_TAG_A(flags), tb = CC_FLAG_TAG_B(flags);
  const uint64_t pa = ta ? a : 0, pb = tb ? b : 0;  // canonical NULL payload
  uint32_t cls = kC3Unk, ct = 0, nt = 0, esc = 0;
  uint64_t pl = 0;
  if (op == CC_OP_VALUE_GET) {
    cls = kC3Get;
  } else if (op == CC_OP_VALUE_SET || op == CC_OP_VALUE_GETANDSET) {
    cls = op == CC_OP_VALUE_SET ? kC3Set : kC3Gas;
    nt = ta;
    esc = v3_fits(pa, kV3SetBits) ? 0u : 1u;
    pl = pa;
  } else if (op == CC_OP_VALUE_CAS) {
    cls = kC3Cas;
    ct = ta;
    nt = tb;
    const uint64_t d = pb - pa;
    esc = v3_fits(pa, kV3ExpBits) && v3_fits(d, kV3DeltaBits) ? 0u : 1u;
    pl = (pa & 0xFFFFFFFFull) | (d << kV3ExpBits);
  } else if (op == CC_OP_DELETE) {
    cls = kC3Del;
  } else if (op == CC_OP_VALUE_LISTEN || op == CC_OP_VALUE_UNLISTEN) {
    cls = kC3Lis;
  }
  pl = esc ? 0ull : pl;
  return (uint64_t)(slot | (cls << 8) | (ct << 11) | (nt << 14) | (esc << 17)) | (pl << 18);
}
__device__ inline uint32_t v3_slot(uint64_t r) { return (uint32_t)r & 0xFFu; }
__device__ inline uint64_t v3_set_row(uint64_t r, uint32_t row) {
  return ((r >> 17) & 1u) ? (r | ((uint64_t)row << 18)) : r;
}

// The record -> value_walk's form (common.h value_encode: meta word, canonical compare value x, canonical new
// value y).  tile_row0 = the batch row of the record's tile start (escaped operands are read from ca / cb there).
__device__ inline void v3_decode(uint64_t r, const uint64_t* __restrict__ ca, const uint64_t* __restrict__ cb,
                                 uint64_t tile_row0, uint32_t& m, uint64_t& x, uint64_t& y) {
  const uint32_t lo = (uint32_t)r;
  const uint32_t slot = lo & 0xFFu, cls = (lo >> 8) & 7u, ct = (lo >> 11) & 7u, nt = (lo >> 14) & 7u;
  // class -> the walk's op bits (value_encode): get R, set W, CAS C + status OK|BOOL, getAndSet W|R, delete D,
  // listen / unlisten L (not applied here: flagged), anything else the precomputed UNKNOWN_OP status
  uint32_t bits = CC_STATUS(CC_ST_UNKNOWN_OP, CC_TAG_NULL);
  bits = cls == kC3Get ? kVrR : bits;
  bits = cls == kC3Set ? kVrW : bits;
  bits = cls == kC3Cas ? (kVrC | CC_STATUS(CC_ST_OK, CC_TAG_BOOL)) : bits;
  bits = cls == kC3Gas ? (kVrW | kVrR) : bits;
  bits = cls == kC3Del ? kVrD : bits;
  bits = cls == kC3Lis ? kVrL : bits;
  m = bits | (nt << 13) | (slot << 16) | (ct << 24);
  const bool cas = cls == kC3Cas, wr = cls == kC3Set || cls == kC3Gas;
  if ((lo >> 17) & 1u) {  // escaped (rare): the operands from the batch columns
    const uint64_t row = tile_row0 + ((r >> 18) & (kV3Tile - 1));
    x = cas && ct ? ca[row] : 0;
    y = cas ? (nt ? cb[row] : 0) : (wr && nt ? ca[row] : 0);
  } else {
    const uint64_t e = (uint64_t)(int64_t)(int32_t)(uint32_t)(r >> 18);
    x = cas ? e : 0;
    y = cas ? e + (uint64_t)((int64_t)r >> (64 - kV3DeltaBits)) : (wr ? (uint64_t)((int64_t)r >> 18) : 0);
  }
}

// ---- the packed result ----------------------------------------------------------------------------------------
// The apply writes each result over its record: payload (56-bit two's complement) | status (7 bits: code | tag << 4,
// tags <= 6) << 56 | escaped << 63.  A payload that does not fit (escaped) is written whole to rst_value at the
// same staging position, where the unpermute reads it.  (9 B per commit in two arrays before: a status byte array
// whose lines were written in ~32-byte pieces by different workgroups, and the value array.)
constexpr int kV3ResBits = 56;
__device__ inline uint64_t v3_pack_result(uint32_t status, uint64_t v, bool esc) {
  return (esc ? (1ull << 63) : (v & ((1ull << kV3ResBits) - 1))) | ((uint64_t)(status & 0x7Fu) << kV3ResBits);
}

// ---- k_part_v4: one persistent 1024-thread workgroup per CU, one pass per 8192-commit tile --------------------
// Same output as the round-3 k_part_v3 (the tile's records grouped by super-bucket in log order, its ttab row and cpos), but
// the whole tile is ranked at once and placed into a 128 KiB LDS image of the tile's staging region, which is then
// written out contiguously: every 128-byte line of the staging area is written whole by one instruction (k_part_v3
// wrote each run piece per 2048-commit chunk, and lines shared by two pieces reached HBM as partial writes: 22.6 B
// written per commit for 18).  Thread (w, j, l) holds commit w*512 + j*64 + l of the tile in registers (the
// tile's rows are wave-contiguous, so per-wave lane-ordered counters give a stable rank); after the placement the
// registers take the NEXT tile's loads, which are in flight while this tile's image is written out.
// LDS hazards: each wave zeroes its own counter row at the top of a tile (its previous readers -- wave 0's scan and
// the wave's own placement -- finished before the previous tile's B3); img / kst are rewritten only after the next
// tile's B1 / B2, which every thread reaches after its own write-out reads.
constexpr int kP4T = 1024;
constexpr int kP4W = kP4T / kWave;    // 16 waves
constexpr int kP4J = kV3Tile / kP4T;  // 8 commits per thread
static_assert(kP4J == 8, "k_part_v4 keeps 8 commits per thread in registers");

template <int KP, int KSB>
__global__ __launch_bounds__(kP4T) void k_part_v4(const uint32_t* __restrict__ inst, const uint8_t* __restrict__ op,
                                                const uint8_t* __restrict__ flags, const uint64_t* __restrict__ ca,
                                                const uint64_t* __restrict__ cb, uint64_t lo, uint64_t hi,
                                                const uint32_t* __restrict__ inst_res, uint32_t max_inst, uint32_t sb,
                                                uint32_t tiles, uint64_t* __restrict__ st_rec, uint16_t* __restrict__ cpos,
                                                uint16_t* __restrict__ ttab) {
  __shared__ uint64_t img[kV3Tile];          // the tile's records in staging order
  __shared__ uint32_t wc[kP4W][kMaxSb / 2];  // per-wave counters (packed u16 pairs) -> per-wave exclusive prefixes
  __shared__ uint16_t kst[kMaxSb + 1];       // tile-local run starts (+ live count)
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  const uint32_t hw = (sb + 1) / 2;
  uint32_t T = blockIdx.x;
  if (T >= tiles) return;
  PH_DECL
  // of2[j / 2] >> 16 * (j % 2) = op | flags << 8 of row j (two rows per register).  A full tile's op and flags columns arrive as 4-row words (opw / flw: lane l of
  // wave w holds rows w*512 + i*256 + 4l .. +3), one load instruction per 256 rows instead of one per 64 (the 16
  // byte loads per thread were issue-bound in the address unit: 19.4 -> 15.1 us per tile without them), and are
  // spread to the rank layout (row w*512 + j*64 + l) by lane shuffles at the top of the tile; a partial tile or an
  // unaligned column loads bytes.
  uint32_t ri[kP4J], of2[kP4J / 2], opw[2], flw[2];
  uint64_t av[kP4J], bv[kP4J];
  bool wide = false;
  const bool opfl_al = ((((uintptr_t)op) | ((uintptr_t)flags) | (uintptr_t)lo) & 3u) == 0;
  auto rowq = [&](int j) -> uint32_t { return w * (kWave * kP4J) + (uint32_t)j * kWave + l; };
  auto load = [&](uint32_t TT) {
    const uint64_t t0 = lo + (uint64_t)TT * kV3Tile;
    const uint32_t nr = (uint32_t)(hi - t0 < (uint64_t)kV3Tile ? hi - t0 : (uint64_t)kV3Tile);
    wide = opfl_al && nr == (uint32_t)kV3Tile;  // block-uniform
    if (wide) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint64_t ic = t0 + w * (kWave * kP4J) + (uint32_t)i * (4 * kWave) + 4u * l;
        opw[i] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(op + ic));
        flw[i] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(flags + ic));
      }
    }
#pragma unroll
    for (int j = 0; j < kP4J; ++j) {
      const uint32_t q = rowq(j);
      const uint64_t ic = t0 + (q < nr ? q : 0u);  // rows past the batch end re-read row 0 (ignored)
      ri[j] = __builtin_nontemporal_load(inst + ic);
#ifdef CC_DIAG_NO_OPFL  // diagnostics build only: op / flags not loaded (wrong results; the byte loads' issue cost)
      if (j % 2 == 0) of2[j / 2] = 0x11321132u;
#else
      if (!wide) {
        const uint32_t v = (uint32_t)__builtin_nontemporal_load(op + ic) | ((uint32_t)__builtin_nontemporal_load(flags + ic) << 8);
        of2[j / 2] = j % 2 ? (of2[j / 2] | (v << 16)) : v;
      }
#endif
      av[j] = __builtin_nontemporal_load(ca + ic);
      bv[j] = __builtin_nontemporal_load(cb + ic);
    }
  };
  // (at the top of a tile: the words landed with the instance column the gathers there wait for)
  auto unpack = [&]() {
#ifndef CC_DIAG_NO_OPFL
    if (!wide) return;
#pragma unroll
    for (int j = 0; j < kP4J; ++j) {
      const int src = (j % 4) * 16 + (int)(l >> 2);
      const uint32_t sh = 8u * (l & 3u);
      const uint32_t o = ((uint32_t)__shfl((int)opw[j / 4], src, kWave) >> sh) & 0xFFu;
      const uint32_t f = ((uint32_t)__shfl((int)flw[j / 4], src, kWave) >> sh) & 0xFFu;
      of2[j / 2] = j % 2 ? (of2[j / 2] | ((o | (f << 8)) << 16)) : (o | (f << 8));
    }
#endif
  };
  load(T);
  for (;;) {
    const uint64_t tile0 = lo + (uint64_t)T * kV3Tile;
    const uint32_t tbase = T * kV3Tile;
    const uint32_t nrow = (uint32_t)(hi - tile0 < (uint64_t)kV3Tile ? hi - tile0 : (uint64_t)kV3Tile);
    for (uint32_t k = l; k < hw; k += kWave) wc[w][k] = 0;
    uint32_t r[kP4J], loc[kP4J];
#pragma unroll
    for (int j = 0; j < kP4J; ++j) {  // instance -> resource (unconditional gathers, then the select)
      const bool ok = rowq(j) < nrow && ri[j] < max_inst;
      const uint32_t g = inst_res[ok ? ri[j] : 0u];
      r[j] = ok ? g : kNoRes;
    }
    unpack();  // (while the gathers fly)
#pragma unroll
    for (int j = 0; j < kP4J; ++j) {
      const uint32_t k = r[j] >> KSB, sh = 16 * (k & 1);
      loc[j] = r[j] != kNoRes ? (atomicAdd(&wc[w][k >> 1], 1u << sh) >> sh) & 0xFFFFu : 0xFFFFu;
    }
    PH(0);
    lds_barrier();  // B1: counters complete
    PH(1);
    if (w == 0) {   // per super-bucket: exclusive prefix over the waves (in place), totals, tile-local run starts
      uint32_t tot[KP];
#pragma unroll
      for (int e = 0; e < KP; e += 2) {
        const uint32_t pr = (l * KP + e) / 2;
        uint32_t acc = 0;
        if (pr < hw) {
#pragma unroll
          for (int q = 0; q < kP4W; ++q) {
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
      uint32_t run = inc - mine;
      uint16_t* row = ttab + (uint64_t)T * (sb + 1);
#pragma unroll
      for (int e = 0; e < KP; ++e) {
        const uint32_t k = l * KP + e;
        if (k < sb) {
          kst[k] = (uint16_t)run;
          row[k] = (uint16_t)run;
        }
        run += tot[e];
      }
      if (l == 63) {
        kst[sb] = (uint16_t)inc;
        row[sb] = (uint16_t)inc;
      }
    }
    PH(2);
    lds_barrier();  // B2: prefixes and run starts
    PH(3);
#pragma unroll
    for (int j = 0; j < kP4J; ++j) {
      const uint32_t q = rowq(j);
      uint32_t cp = 0xFFFFu;
      if (loc[j] != 0xFFFFu) {
        const uint32_t k = r[j] >> KSB, sh = 16 * (k & 1);
        const uint32_t sp = kst[k] + ((wc[w][k >> 1] >> sh) & 0xFFFFu) + loc[j];
        const uint32_t ofj = of2[j / 2] >> (16 * (j % 2));
        img[sp] = v3_set_row(v3_encode(ofj & 0xFFu, (ofj >> 8) & 0xFFu, av[j], bv[j], r[j] & ((1u << KSB) - 1)), q);
        cp = sp;
      }
      if (q < nrow) cpos[tbase + q] = (uint16_t)cp;
    }
    const uint32_t Tn = T + gridDim.x;
    if (Tn < tiles) load(Tn);  // the raw registers are free: the next tile's loads fly during the write-out
    PH(4);
    lds_barrier();             // B3: the image is complete
    PH(5);
    // whole tile region, unconditionally (a fixed store count; rows past the live count are never read), 16 B a lane
#pragma unroll
    for (int m = 0; m < kP4J / 2; ++m)
      reinterpret_cast<uint4*>(st_rec + tbase)[t + m * kP4T] = reinterpret_cast<const uint4*>(img)[t + m * kP4T];
    PH(6);
    if (Tn >= tiles) break;
    T = Tn;
  }
#ifdef CC_PHASE_TIMING
  PH_FLUSH(g_ph_v3p);
#endif
}

// ---- k_apply_value_v3: walker / loader waves (apply_value.hip k_apply_value_ws) over 8-byte records ------------
// One 1024-thread workgroup per super-bucket: waves 0-3 walk (thread t = slot t, AtomicValueState in registers),
// waves 4-15 load, decode, rank and place the next chunk (3072 records) into the other LDS buffer and store the
// previous chunk's results.  The super-bucket's list is its run in every 8192-commit tile, in tile (= log) order.
//
// LDS hazards (the chunk pipeline; cf. the k_apply_map chunk-0 race):
//   * buffer b is placed by the loaders during iteration i-1 and walked during iteration i; the one workgroup
//     barrier per iteration separates the two, and the walkers' in-place results in b are read back by the loaders'
//     store_results only in iteration i+1 (after the next barrier);
//   * wcnt[b] / pbase are rewritten by `prepare` only after the loaders' arrival barrier (loader_barrier), which every
//     loader wave reaches after its own ranking of the same chunk; wcnt[b^1] is cleared after that arrival barrier,
//     and was last read (placement bases of the chunk before) before the previous workgroup barrier;
//   * rstart / rpre (the run table) are written once, before the first workgroup barrier, and never rebuilt.
constexpr int kWsPer = 4;
constexpr uint32_t kNoPos3 = 0xFFFFFFFFu;
// NS slots per super-bucket: 256 (1024-thread workgroups: 4 walker + 12 loader waves, 3072-record chunks, one
// workgroup per CU) or 128 (512-thread workgroups: 2 walker + 6 loader waves, 1536-record chunks, 79 KB of LDS: two
// workgroups per CU, so one workgroup's per-chunk loader chain -- rank, arrival barrier, placement bases, placement
// -- overlaps the other's; with one workgroup per CU that chain, not the bytes, bounded the launch: 0.60 ms/step
// with contiguous loads and no walk at all, profiles/r03/diag1).
template <int NS>
struct V3A {
  static constexpr int WW = NS / kWave;               // walker waves
  static constexpr int LW = NS == 128 ? 6 : 12;       // loader waves
  static constexpr int T = (WW + LW) * kWave;         // workgroup threads
  static constexpr int W = T / kWave;
  static constexpr int CH = LW * kWave * kWsPer;      // records per chunk
  static constexpr int NP = NS / 2;                   // packed u16 counter pairs
  static constexpr int SPL = NS / kWave;              // slots per loader lane in the placement bases
  static constexpr int TPT = (kV3MaxTiles + T - 1) / T;  // run-table tiles per thread
  static constexpr int MINW = NS == 128 ? 4 : 1;      // waves per SIMD asked of the register allocator
};

__device__ inline uint32_t v3_value_walk(uint32_t m, uint64_t x, uint64_t y, uint32_t& ms, uint64_t& v, uint64_t& rv) {
  const uint32_t tag = ms & 0xFFu;
  // compareAndSet :124 (value == null && expect == null) || (value != null && value.equals(expect))
  const bool eq = vrec_ctag(m) == tag && v == x;
  const bool is_c = (m & kVrC) != 0, is_r = (m & kVrR) != 0, is_d = (m & kVrD) != 0;
  const bool wr = (m & kVrW) != 0 || (is_c && eq);
  rv = is_r ? v : ((is_c && eq) ? 1ull : 0ull);
  const uint32_t st = is_r ? (tag << 4) : (m & 0xFFu);
  ms = wr ? (vrec_ntag(m) | 0x100u) : (is_d ? 0u : ms);
  v = wr ? y : (is_d ? 0ull : v);
  return st;
}

// Largest r in [0, tiles) with rpre[r] <= c (two-round 64-ary search by the whole wave; tiles <= 4096).
__device__ inline uint32_t v3_find_run(const uint32_t* rpre, uint32_t tiles, uint32_t c) {
  const uint32_t l = __lane_id();
  const uint32_t step = (tiles + kWave - 1) / kWave;
  uint32_t cand = l * step;
  uint64_t b = __ballot(cand < tiles && rpre[cand] <= c);
  const uint32_t base = (uint32_t)(63 - __clzll((long long)b)) * step;
  cand = base + l;
  b = __ballot(l < step && cand < tiles && rpre[cand] <= c);
  return base + (uint32_t)(63 - __clzll((long long)b));
}

__device__ inline void v3_loader_barrier(uint32_t* ctr, uint32_t target) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if (__lane_id() == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int NS>
__global__ __launch_bounds__(V3A<NS>::T, V3A<NS>::MINW) void k_apply_value_v3(uint64_t* __restrict__ st_rec,
                                                        const uint64_t* __restrict__ ca, const uint64_t* __restrict__ cb,
                                                        uint64_t lo, const uint16_t* __restrict__ ttab, uint32_t tiles,
                                                        uint32_t sb, uint32_t* __restrict__ val_meta,
                                                        uint64_t* __restrict__ val_v, uint64_t* __restrict__ rst_value,
                                                        uint64_t dummy,
                                                        uint32_t* __restrict__ err_out) {
  using P = V3A<NS>;
#ifdef CC_DIAG  // diagnostics build only (-DCC_DIAG=1: no walk, 2: contiguous positions -- wrong results by design; 4: internal checks only, common.h kErrSmallFlag)
  constexpr uint32_t diag = CC_DIAG;
#else
  constexpr uint32_t diag = 0;
#endif
  constexpr int kWsLW = P::LW, kWsCh = P::CH, kAVT = P::T, kAVW = P::W, kVSlots3 = NS, kVPairs3 = P::NP;
  constexpr uint32_t kL0 = P::WW * kWave;       // first loader thread
  __shared__ u64x2 sab[2][kWsCh];               // chunk buffers sorted by slot; results in place {value, status}
  __shared__ uint32_t sm[2][kWsCh];             //   meta words
  __shared__ uint32_t wcnt[2][kWsLW][kVPairs3];  // per-loader-wave slot counts (packed u16 pairs), double-buffered
  __shared__ uint16_t pbase[kWsLW][kVSlots3];   // per loader wave: sorted position of its first record of each slot
  __shared__ uint32_t sstart[2][kVSlots3 + 1];  // slot run starts of each buffer (+ total)
  __shared__ uint16_t rb0[kV3MaxTiles];         // start of this super-bucket's run inside tile r
  __shared__ uint32_t rpre[kV3MaxTiles + 1];    // records of this super-bucket before tile r
  __shared__ uint32_t wsum[kAVW];
  __shared__ uint32_t lbar;
  auto rstart = [&](uint32_t r) -> uint32_t { return r * kV3Tile + rb0[r]; };  // staging position of run r

  const uint32_t s = blockIdx.x, t = threadIdx.x, w = t >> 6, l = t & 63;
  const bool walker = t < kL0;
  const uint32_t lw = walker ? 0u : w - P::WW;
  uint32_t ms = 0;
  uint64_t sv = 0;
  if (walker) {
    ms = val_meta[(uint64_t)s * kVSlots3 + t];
    sv = val_v[(uint64_t)s * kVSlots3 + t];
  }
  for (uint32_t k = t; k < (uint32_t)(2 * kWsLW * kVPairs3); k += kAVT) (&wcnt[0][0][0])[k] = 0;
  if (t == 0) lbar = 0;
  {  // the super-bucket's list = its run in every tile, in tile order; thread t owns tiles TPT*t .. TPT*t + TPT-1
    uint32_t len[P::TPT], lsum = 0;
#pragma unroll
    for (int q = 0; q < P::TPT; ++q) {
      const uint32_t tt = P::TPT * t + q;
      len[q] = 0;
      if (tt < tiles) {
        const uint16_t* row = ttab + (uint64_t)tt * (sb + 1);
        const uint32_t b0 = row[s], b1 = row[s + 1];
        rb0[tt] = (uint16_t)b0;
        len[q] = b1 - b0;
      }
      lsum += len[q];
    }
    uint32_t inc = lsum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (l >= (uint32_t)d) inc += y;
    }
    if (l == 63) wsum[w] = inc;
    lds_barrier();
    uint32_t pre = inc - lsum, all = 0;
    for (uint32_t q = 0; q < (uint32_t)kAVW; ++q) {
      const uint32_t x = wsum[q];
      if (q < w) pre += x;
      all += x;
    }
#pragma unroll
    for (int q = 0; q < P::TPT; ++q) {
      if (P::TPT * t + q < tiles) rpre[P::TPT * t + q] = pre;
      pre += len[q];
    }
    if (t == 0) rpre[tiles] = all;
    lds_barrier();
  }
  const uint32_t cnt = rpre[tiles];
  const uint32_t nch = (cnt + kWsCh - 1) / kWsCh;
  uint32_t err = 0;
#ifdef CC_PHASE_TIMING
  // thread 0 (walker): 0 walk, 1 wait; thread 256 (loader): 2 result store, 3 rank, 4 loader + workgroup barriers,
  // 5 clear + placement bases, 6 decode + place, 7 load issue
  uint64_t wph_last = wall_clock64(), wph[kPhases] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto WPH = [&](int k) {
    if (t == 0 || t == kL0) {
      const uint64_t n_ = wall_clock64();
      wph[k] += n_ - wph_last;
      wph_last = n_;
    }
  };
#else
  auto WPH = [&](int) {};
#endif

  // loader registers: the chunk to place next (rr, g; loaded one chunk ahead), the sorted / staging positions of the
  // chunk being walked (pp, gp) and of the chunk before it (qp, gq: its results are stored during the walk)
#define CC_J4(X) X(0) X(1) X(2) X(3)
#define CC_DECL(J) uint32_t g##J = kNoPos3, pp##J = 0, gp##J = kNoPos3, qp##J = 0, gq##J = kNoPos3; uint64_t rr##J = 0;
  CC_J4(CC_DECL)
#undef CC_DECL
  // record c0 + lw*256 + j*64 + l of the list (log order = (loader wave, j, lane)); past the end: staging position 0.
  // Staging position of list record c: the run r holding it gives rstart[r] + c - rpre[r]; one 64-ary search per wave
  // and chunk finds the wave's first run, lane k then holds window run rrow + k, and rows find their runs with ballots.
#define CC_LOAD1(J)                                                                               \
  {                                                                                               \
    const uint32_t crow = c0w + (J) * kWave, c = crow + l;                                        \
    uint32_t gpos = 0;                                                                            \
    if (crow < cnt) { /* wave-uniform */                                                          \
      if (win) {                                                                                  \
        uint32_t ri = (uint32_t)__popcll(__ballot(wB <= crow));                                   \
        uint64_t mb = __ballot(wB > crow && wB <= crow + (kWave - 1));                            \
        while (mb) {                                                                              \
          const uint32_t bk = (uint32_t)__builtin_amdgcn_readlane((int)wB, __ffsll((long long)mb) - 1); \
          ri += c >= bk ? 1u : 0u;                                                                \
          mb &= mb - 1;                                                                           \
        }                                                                                         \
        const uint32_t rs_ = (uint32_t)__shfl((int)wS, (int)ri, 64);                              \
        const uint32_t rp_ = (uint32_t)__shfl((int)wP, (int)ri, 64);                              \
        if (c < cnt) gpos = rs_ + (c - rp_);                                                      \
      } else {                                                                                    \
        uint32_t r = v3_find_run(rpre, tiles, crow);                                              \
        if (c < cnt) {                                                                            \
          while (rpre[r + 1] <= c) ++r;                                                           \
          gpos = rstart(r) + (c - rpre[r]);                                                       \
        }                                                                                         \
      }                                                                                           \
    }                                                                                             \
    if (diag & 2u) gpos = c < cnt ? c : 0u; /* diagnostics: contiguous positions (wrong results) */ \
    g##J = c < cnt ? gpos : kNoPos3;                                                              \
    rr##J = st_rec[gpos];                                                                         \
  }
#define CC_LOAD_CHUNK(C0)                                                                         \
  {                                                                                               \
    const uint32_t c0w = (C0) + lw * (kWave * kWsPer);                                            \
    uint32_t wB = 0xFFFFFFFFu, wS = 0, wP = 0;                                                    \
    bool win = false;                                                                             \
    if (c0w < cnt) {                                                                              \
      const uint32_t rrow = v3_find_run(rpre, tiles, c0w);                                        \
      const uint32_t kr = rrow + l;                                                               \
      wB = kr + 1 <= tiles ? rpre[kr + 1] : 0xFFFFFFFFu;                                          \
      wS = kr < tiles ? rstart(kr) : 0u;                                                          \
      wP = kr < tiles ? rpre[kr] : 0u;                                                            \
      const uint32_t lastc = c0w + kWave * kWsPer - 1 < cnt ? c0w + kWave * kWsPer - 1 : cnt - 1; \
      win = (uint32_t)__shfl((int)wB, 63, 64) > lastc;                                            \
    }                                                                                             \
    CC_J4(CC_LOAD1)                                                                               \
  }
  uint32_t bar_n = 0;  // loader-barrier arrivals expected so far
  // rank / place the registers' chunk into buffer b (loaders only)
  auto prepare = [&](uint32_t b) {
    uint32_t rank[kWsPer], slot[kWsPer];
    const uint64_t rv4[kWsPer] = {rr0, rr1, rr2, rr3};
    const uint32_t gv[kWsPer] = {g0, g1, g2, g3};
#pragma unroll
    for (int j = 0; j < kWsPer; ++j) {
      slot[j] = v3_slot(rv4[j]);
      const uint32_t sh = 16 * (slot[j] & 1);
      rank[j] = gv[j] != kNoPos3 ? (atomicAdd(&wcnt[b][lw][slot[j] >> 1], 1u << sh) >> sh) & 0xFFFFu : 0u;
    }
    WPH(3);
    bar_n += kWsLW;
    v3_loader_barrier(&lbar, bar_n);  // every loader wave has ranked this chunk into wcnt[b]
    WPH(4);
    // the other counter buffer was last read before the previous workgroup barrier: clear it for the next chunk
    for (uint32_t k = t - kL0; k < (uint32_t)(kWsLW * kVPairs3); k += kWsLW * kWave) (&wcnt[b ^ 1][0][0])[k] = 0;
    // this wave's placement bases: lane l owns slots SPL*l .. SPL*l + SPL-1 (counter pairs SPL/2*l ..)
    constexpr int PPL = P::SPL / 2;
    uint32_t acc[PPL], own[PPL];
#pragma unroll
    for (int e = 0; e < PPL; ++e) acc[e] = own[e] = 0;
#pragma unroll
    for (int q = 0; q < kWsLW; ++q) {
#pragma unroll
      for (int e = 0; e < PPL; ++e) {
        const uint32_t cv = wcnt[b][q][PPL * l + e];
        if ((uint32_t)q == lw) own[e] = acc[e];
        acc[e] += cv;
      }
    }
    uint32_t mine = 0;
#pragma unroll
    for (int e = 0; e < PPL; ++e) mine += (acc[e] & 0xFFFFu) + (acc[e] >> 16);
    uint32_t inc = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (l >= (uint32_t)d) inc += y;
    }
    uint32_t run = inc - mine;
#pragma unroll
    for (int e = 0; e < PPL; ++e) {
      const uint32_t k = P::SPL * l + 2 * e;
      pbase[lw][k] = (uint16_t)(run + (own[e] & 0xFFFFu));
      if (lw == 0) sstart[b][k] = run;  // the walkers' run starts (read after the workgroup barrier)
      run += acc[e] & 0xFFFFu;
      pbase[lw][k + 1] = (uint16_t)(run + (own[e] >> 16));
      if (lw == 0) sstart[b][k + 1] = run;
      run += acc[e] >> 16;
    }
    if (lw == 0 && l == 63) sstart[b][kVSlots3] = inc;
    WPH(5);
    // lanes read bases other lanes of this wave just wrote: LDS keeps one wave's accesses in order
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
#define CC_PLACE1(J)                                                                \
    {                                                                               \
      pp##J = 0;                                                                    \
      gp##J = g##J;                                                                 \
      if (g##J != kNoPos3) {                                                        \
        uint32_t m_;                                                                \
        uint64_t x_, y_;                                                            \
        v3_decode(rr##J, ca, cb, lo + (uint64_t)(g##J / kV3Tile) * kV3Tile, m_, x_, y_); \
        pp##J = pbase[lw][slot[J]] + rank[J];                                       \
        sm[b][pp##J] = m_;                                                          \
        sab[b][pp##J] = u64x2{x_, y_};                                              \
      }                                                                             \
    }
    CC_J4(CC_PLACE1)
#undef CC_PLACE1
    WPH(6);
  };
  // the previous chunk's results (buffer b) back to the records' staging positions, over the records themselves
  // (each record is read once, by this workgroup, a chunk earlier): one packed word per result (v3_pack_result),
  // unconditional stores (rows past the end go to the dummy words); an escaped value also goes to rst_value
  auto store_results = [&](uint32_t b) {
#define CC_STORE1(J)                                                                \
    {                                                                               \
      const uint64_t gx = gq##J != kNoPos3 ? (uint64_t)gq##J : dummy + t;           \
      const u64x2 r_ = sab[b][qp##J];                                               \
      const bool esc_ = !v3_fits(r_.x, kV3ResBits);                                 \
      st_rec[gx] = v3_pack_result((uint32_t)r_.y, r_.x, esc_);                      \
      if (esc_ && gq##J != kNoPos3) rst_value[gx] = r_.x;                            \
    }
    CC_J4(CC_STORE1)
#undef CC_STORE1
  };

  if (!walker) {
    CC_LOAD_CHUNK(0)
    prepare(0);
    CC_LOAD_CHUNK(kWsCh)
  }
  lds_barrier();
  for (uint32_t i = 0; i < nch; ++i) {
    const uint32_t b = i & 1;
    if (walker) {
      const uint32_t start = sstart[b][t], run = (diag & 1u) ? 0u : sstart[b][t + 1] - start;
      if (run) {
        uint32_t mA[4], mB[4];
        u64x2 xA[4], xB[4];
        const uint32_t last = start + run - 1;
        auto fetch = [&](uint32_t k0, uint32_t (&mm)[4], u64x2 (&xx)[4]) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t pq = start + k0 + q <= last ? start + k0 + q : last;
            mm[q] = sm[b][pq];
            xx[q] = sab[b][pq];
          }
        };
        auto walk4 = [&](uint32_t k0, const uint32_t (&mm)[4], const u64x2 (&xx)[4]) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (k0 + q < run) {
              uint64_t rv;
              const uint32_t stt = v3_value_walk(mm[q], xx[q].x, xx[q].y, ms, sv, rv);
              if (mm[q] & kVrL) err |= kErrUnsupported;
              // the result over the record, one 16-byte LDS write: with 2 reads + 1 write per record, a group of 4
              // records' reads plus the previous group's writes stay within the 15 outstanding LDS operations a
              // wave can wait on precisely (two writes per record overflowed it and serialised the pipeline)
              sab[b][start + k0 + q] = u64x2{rv, (uint64_t)stt};
            }
          }
        };
        fetch(0, mA, xA);
        for (uint32_t k0 = 0; k0 < run; k0 += 8) {
          fetch(k0 + 4, mB, xB);
          walk4(k0, mA, xA);
          if (k0 + 4 >= run) break;
          fetch(k0 + 8, mA, xA);
          walk4(k0 + 4, mB, xB);
        }
      }
    } else {
      store_results(b ^ 1);  // chunk i-1 (i = 0: the dummy rows)
      WPH(2);
#define CC_SHIFT1(J) qp##J = pp##J; gq##J = gp##J;
      CC_J4(CC_SHIFT1)
#undef CC_SHIFT1
      prepare(b ^ 1);        // chunk i+1 (past the end: no live records)
      CC_LOAD_CHUNK((i + 2) * kWsCh)
      WPH(7);
    }
    if (walker) WPH(0);
    lds_barrier();  // buffer hand-over: b walked (results in place), b^1 placed
    WPH(walker ? 1 : 4);
  }
  if (!walker && nch) store_results((nch - 1) & 1);  // the last chunk (qp / gq since its walk)
#ifdef CC_PHASE_TIMING
  if (t == 0 || t == kL0)
    for (int q = 0; q < kPhases; ++q) atomicAdd(&g_ph_v3a[q], (unsigned long long)wph[q]);
#endif
#undef CC_LOAD_CHUNK
#undef CC_LOAD1
#undef CC_J4
  if (walker) {
    val_meta[(uint64_t)s * kVSlots3 + t] = ms;
    val_v[(uint64_t)s * kVSlots3 + t] = sv;
  }
  if (err) atomicOr(err_out, err);
}

// ---- k_unpermute_v3: the packed results back to log order ----------------------------------------------------
// partition.hip k_unpermute over packed result words: per 8192-commit tile (persistent, two 512-thread workgroups per
// CU), the tile's staged words are read contiguously into LDS (the next tile's are loaded into registers meanwhile),
// then each thread writes 4-row groups in log order through cpos: status bytes as one u32, values as two 16-byte
// stores.  Unknown-session rows (cpos 0xFFFF) get UNKNOWN_SESSION here (ResourceManager.java:60-69).
constexpr int kU3T = 512;
template <int NT, int TL>
__global__ __launch_bounds__(NT) void k_unpermute_v3(const uint16_t* __restrict__ cpos, uint32_t tiles, uint64_t n,
                                                   const uint64_t* __restrict__ words, const uint64_t* __restrict__ esc_value,
                                                   uint8_t* __restrict__ out_status, uint64_t* __restrict__ out_value,
                                                   uint8_t* __restrict__ dummy_status, uint64_t* __restrict__ dummy_value) {
  constexpr int kUnVal = TL / (2 * NT);  // 16-byte word-pair loads per thread per tile (8)
  constexpr int kUnPos = TL / (4 * NT);  // 4-commit cpos groups per thread per tile (4)
  static_assert(kUnVal == 8 && kUnPos == 4, "unpermute prefetch registers");
  __shared__ uint4 lw2[TL / 2];
  const uint64_t* lw = reinterpret_cast<const uint64_t*>(lw2);
  const uint32_t t = threadIdx.x;
  // prefetch registers as named scalars (an array would live in scratch and make every prefetch wait)
  uint4 v0, v1, v2, v3, v4, v5, v6, v7;
  uint2 p0, p1, p2, p3;
  auto load = [&](uint32_t TT) {
    const uint64_t i0 = (uint64_t)TT * TL;
    const uint4* sv = reinterpret_cast<const uint4*>(words + i0) + t;
    const uint2* sp = reinterpret_cast<const uint2*>(cpos + i0) + t;
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
    lw2[t + 0 * NT] = v0; lw2[t + 1 * NT] = v1; lw2[t + 2 * NT] = v2; lw2[t + 3 * NT] = v3;
    lw2[t + 4 * NT] = v4; lw2[t + 5 * NT] = v5; lw2[t + 6 * NT] = v6; lw2[t + 7 * NT] = v7;
    const uint2 pp[kUnPos] = {p0, p1, p2, p3};
    lds_barrier();
    load(T + gridDim.x < tiles ? T + gridDim.x : tiles - 1);
    const uint64_t i0 = (uint64_t)T * TL;
#pragma unroll
    for (int k = 0; k < kUnPos; ++k) {
      const uint64_t i = i0 + 4 * (uint64_t)(t + k * NT);  // commits i .. i+3
      const uint32_t p[4] = {pp[k].x & 0xFFFF, pp[k].x >> 16, pp[k].y & 0xFFFF, pp[k].y >> 16};
      uint32_t sw = 0;
      uint64_t v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = p[q] != 0xFFFF;
        const uint64_t wd = ok ? lw[p[q]] : 0;
        uint64_t x = (uint64_t)(((int64_t)(wd << (64 - kV3ResBits))) >> (64 - kV3ResBits));
        if (wd >> 63) x = esc_value[i0 + p[q]];  // escaped payload (rare)
        sw |= (uint32_t)(ok ? (uint32_t)(wd >> kV3ResBits) & 0x7Fu : unk) << (8 * q);
        v[q] = x;
      }
      const bool in = i + 4 <= n;
      uint32_t* os = in ? reinterpret_cast<uint32_t*>(out_status) + i / 4 : reinterpret_cast<uint32_t*>(dummy_status) + t;
      u64x2* ov = in ? reinterpret_cast<u64x2*>(out_value) + i / 2 : reinterpret_cast<u64x2*>(dummy_value) + 2 * t;
      *os = sw;
      ov[0] = u64x2{v[0], v[1]};
      ov[1] = u64x2{v[2], v[3]};
      if (!in && i < n) {  // the straddling group (at most one in the grid): written after the loop
        tail_sw = sw;
        tail_v0 = v[0];
        tail_v1 = v[1];
        tail_v2 = v[2];
        tail_i = i;
      }
    }
  }
  if (tail_i != ~0ull) {  // commits tail_i .. n-1 (1 to 3 of them)
    const uint64_t vv[3] = {tail_v0, tail_v1, tail_v2};
    for (int q = 0; q < 3 && tail_i + q < n; ++q) {
      out_status[tail_i + q] = (uint8_t)(tail_sw >> (8 * q));
      out_value[tail_i + q] = vv[q];
    }
  }
}

int launch_unpermute_v3(const UnpermuteArgs& a, const uint64_t* words, hipStream_t st) {
  const uint64_t n = a.hi - a.lo;
  const uint64_t t3 = (n + kV3Tile - 1) / kV3Tile;
  const uint32_t grid = (uint32_t)(t3 < 2 * kPersistGrid ? t3 : 2 * kPersistGrid);
  hipLaunchKernelGGL((k_unpermute_v3<kU3T, kV3Tile>), dim3(grid), dim3(kU3T), 0, st, a.cpos, (uint32_t)t3, n, words,
                     a.rst_value, a.out_status + a.lo, a.out_value + a.lo, a.dummy_status, a.dummy_value);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Slots per value super-bucket: 256.  (128-slot buckets -- two 512-thread apply workgroups per CU -- measured slower
// on c2: apply 0.91 -> 0.98, partition 0.88 -> 0.92 ms/step, profiles/r03/ab_ns128: the apply is bound by the loaders'
// instruction and LDS throughput, not by the latency a second workgroup would hide, and 16-record runs over-fetch.)
int launch_part_v3(const PartArgs& a, uint32_t tiles, hipStream_t st) {
  if (a.sb > (uint32_t)kMaxSb || tiles > (uint32_t)kV3MaxTiles) return -1;
  const uint32_t grid = tiles < (uint32_t)kPersistGrid ? tiles : (uint32_t)kPersistGrid;
  const uint32_t kp = (a.sb + kWave - 1) / kWave;  // super-buckets per lane of the scan wave
#define CC_LAUNCH4(KP)                                                                                                 \
  hipLaunchKernelGGL((k_part_v4<KP, 8>), dim3(grid), dim3(kP4T), 0, st, a.inst, a.op, a.flags, a.a, a.b, a.lo, a.hi,   \
                     a.inst_res, a.max_inst, a.sb, tiles, reinterpret_cast<uint64_t*>(a.st_ab), a.cpos, a.ttab)
  if (kp <= 2) CC_LAUNCH4(2);
  else if (kp <= 4) CC_LAUNCH4(4);
  else CC_LAUNCH4(8);
#undef CC_LAUNCH4
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_apply_value_v3(const ValueArgs& a, hipStream_t st) {
  if (a.tiles > (uint32_t)kV3MaxTiles) return -1;
  hipLaunchKernelGGL(k_apply_value_v3<256>, dim3(a.sb_val), dim3(V3A<256>::T), 0, st,
                     reinterpret_cast<uint64_t*>(a.st_ab), a.ca, a.cb, a.lo, a.ttab, a.tiles, a.sb, a.val_meta, a.val_v,
                     a.rst_value, a.dummy, a.err);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
