// apply_value.hip — AtomicValueState apply (also DistributedAtomicLong, whose add is a client-side CAS loop).
//
// One 256-thread workgroup owns one super-bucket = 256 AtomicValueState instances: thread t holds slot t's
// state in registers for the whole launch.  It walks the super-bucket's staging list (its run in every tile,
// tile order = log order; built by partition.hip) in chunks of 2048 records, prefetching the next chunk into registers while it resolves the
// current one: a stable counting sort of the chunk by slot (ballot ranking + per-slot prefix sums in LDS)
// gives every slot its commits in log order, and each thread applies its slot's chain sequentially — the
// same order the reference's single state-machine thread would (ResourceManager.java:56-72).  Results are
// staged in LDS and written back to the records' staging positions; k_unpermute returns them to log order.
//
// Per-op semantics restate AtomicValueState (atomic/src/main/java/io/atomix/atomic/state/AtomicValueState.java):
//   get :77-83, set :114-118, compareAndSet :123-133, getAndSet :138-144, delete :146-157.
// `ttl` is never serialized for these commands (AtomicValueCommands.java:125-133,181-191,227-235),
// so no TTL timer can exist.  Listen/Unlisten (:41-63) publish events: not applied by this build (flagged).
#include "common.h"
#include "engine_internal.h"

namespace cc {

struct ValState {
  uint32_t meta;  // tag | has_current << 8
  uint64_t v;
};

// Applies one committed AtomicValue op to the state; returns the status byte, result payload in rv.
// Branch-free (selects only): a wave's lanes carry different ops, and a switch would run every case.
__device__ inline uint32_t value_apply(uint32_t op, uint32_t flags, uint64_t a, uint64_t b, ValState& s, uint64_t& rv,
                                       uint32_t& err) {
  const uint32_t ta = CC_FLAG_TAG_A(flags), tb = CC_FLAG_TAG_B(flags);
  const uint64_t pa = ta ? a : 0, pb = tb ? b : 0;  // canonical NULL payload
  const uint32_t tag = s.meta & 0xFF, cur = (s.meta >> 8) & 1;
  const bool is_get = op == CC_OP_VALUE_GET;        // get :77-83   return current != null ? value : null
  const bool is_set = op == CC_OP_VALUE_SET;        // set :114-118 value = v
  const bool is_cas = op == CC_OP_VALUE_CAS;        // compareAndSet :123-133
  const bool is_gas = op == CC_OP_VALUE_GETANDSET;  // getAndSet :138-144 result = old value
  const bool is_del = op == CC_OP_DELETE;           // delete :146-157 (current != null) -> value = current = null
  const bool is_lis = op == CC_OP_VALUE_LISTEN || op == CC_OP_VALUE_UNLISTEN;
  // (value == null && expect == null) || (value != null && expect != null && value.equals(expect))
  const bool eq = (tag == CC_TAG_NULL && ta == CC_TAG_NULL) || (tag != CC_TAG_NULL && tag == ta && s.v == pa);
  const bool write = is_set || is_gas || (is_cas && eq);
  const bool clear = is_del && cur;
  // result
  uint32_t rtag = CC_TAG_NULL;
  rv = 0;
  if ((is_get && cur) || is_gas) { rtag = tag; rv = s.v; }
  if (is_cas) { rtag = CC_TAG_BOOL; rv = eq ? 1 : 0; }
  const bool known = is_get || is_set || is_cas || is_gas || is_del || is_lis;
  if (is_lis) err |= kErrUnsupported;
  // state
  const uint32_t ntag = is_cas ? tb : ta;
  const uint64_t nv = is_cas ? pb : pa;
  s.meta = write ? vmeta(ntag, 1) : (clear ? 0u : s.meta);
  s.v = write ? nv : (clear ? 0ull : s.v);
  // IllegalStateException "unknown operation type" (ResourceStateMachineExecutor.java:78)
  return known ? CC_STATUS(CC_ST_OK, rtag) : CC_STATUS(CC_ST_UNKNOWN_OP, CC_TAG_NULL);
}

constexpr int kAT = kApplyWaves * kWave;  // 256 threads = 256 slots of the super-bucket
constexpr int kACh = kAT * kApplyPer;     // 2048 records per chunk
constexpr int kSbSlots = kApplyWaves * kLaneRes;
constexpr int kWaveRecs = kWave * kApplyPer;  // records of a chunk per wave (contiguous)

// One workgroup per super-bucket; thread t owns slot t (its AtomicValueState lives in two registers).
// Per chunk of 2048 staging records (wave w holds records w*512 + j*64 + lane, so log order = (w, j, lane)):
//   1. a stable counting sort of the chunk by slot: each wave ranks its records with LDS atomics with return
//      on its own 256-counter table (same-address lanes resolve in lane order on gfx950, and the wave's
//      instructions are in program order), the owner of each slot prefixes the 4 wave counts, a block scan
//      gives each slot's run start;
//   2. thread t walks its slot's run sequentially — the reference's one-commit-at-a-time order, per slot;
//   3. results go back through LDS to staging order and out contiguously.
__global__ __launch_bounds__(kAT) void k_apply_value(const uint32_t* __restrict__ st_meta, const u64x2* __restrict__ st_ab,
                                                    const uint16_t* __restrict__ ttab, uint32_t tiles, uint32_t sb,
                                                    const uint8_t* __restrict__ sb_kind,
                                                    uint32_t* __restrict__ val_meta, uint64_t* __restrict__ val_v,
                                                    uint8_t* __restrict__ rst_status, uint64_t* __restrict__ rst_value,
                                                    uint32_t* __restrict__ err_out) {
  __shared__ u64x2 sab[kACh];
  __shared__ uint32_t sm[kACh];
  __shared__ uint16_t sidx[kACh];
  __shared__ uint64_t rval[kACh];
  __shared__ uint8_t rstat[kACh];
  __shared__ uint32_t wcnt[kApplyWaves][kSbSlots];  // per-wave slot counts (zeroed after use)
  __shared__ uint32_t wpre[kApplyWaves][kSbSlots];  // per-wave slot prefixes
  __shared__ uint32_t sstart[kSbSlots];
  __shared__ uint32_t wsum[kApplyWaves];
  __shared__ uint32_t rstart[kMaxTiles];     // staging position of this super-bucket's run in tile t
  __shared__ uint32_t rpre[kMaxTiles + 1];   // records of this super-bucket before tile t

  const uint32_t s = blockIdx.x, t = threadIdx.x, w = t >> 6, l = t & 63;
  if (sb_kind && sb_kind[s]) return;  // holds coordination resources / value events: k_apply_coord
  ValState st_reg{val_meta[(uint64_t)s * kSbSlots + t], val_v[(uint64_t)s * kSbSlots + t]};
#pragma unroll
  for (int q = 0; q < kApplyWaves; ++q) wcnt[q][t] = 0;
  // the super-bucket's list = its run in every tile, in tile order (tile-local layout of partition.hip)
  {
    constexpr int PT = kMaxTiles / kAT;  // tiles per thread
    uint32_t len[PT], sum = 0;
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint32_t tt = t * PT + k;
      len[k] = 0;
      if (tt < tiles) {
        const uint16_t* row = ttab + (uint64_t)tt * (sb + 1);
        const uint32_t b0 = row[s], b1 = row[s + 1];
        rstart[tt] = tt * kTile + b0;
        len[k] = b1 - b0;
      }
      sum += len[k];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (l >= (uint32_t)d) inc += y;
    }
    if (l == 63) wsum[w] = inc;
    lds_barrier();
    uint32_t run = inc - sum;
    for (uint32_t q = 0; q < w; ++q) run += wsum[q];
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint32_t tt = t * PT + k;
      if (tt < tiles) rpre[tt] = run;
      run += len[k];
    }
    if (t == kAT - 1) rpre[tiles] = run;
    lds_barrier();
  }
  const uint32_t cnt = rpre[tiles];
  uint32_t err = 0;

  uint32_t m[kApplyPer], nm[kApplyPer], pos[kApplyPer], npos[kApplyPer];
  u64x2 ab[kApplyPer], nab[kApplyPer];
  uint32_t cur = 0;  // this thread's run cursor (its records are visited in increasing order)
  auto load = [&](uint32_t c0, uint32_t (&mm)[kApplyPer], u64x2 (&aa)[kApplyPer], uint32_t (&pp)[kApplyPer]) {
#pragma unroll
    for (int j = 0; j < kApplyPer; ++j) {
      const uint32_t c = c0 + w * kWaveRecs + j * kWave + l;
      mm[j] = 0;
      aa[j] = u64x2{0, 0};
      pp[j] = 0;
      if (c < cnt) {
        while (rpre[cur + 1] <= c) ++cur;
        const uint32_t g = rstart[cur] + (c - rpre[cur]);
        pp[j] = g;
        mm[j] = st_meta[g];
        aa[j] = st_ab[g];
      }
    }
  };
  load(0, m, ab, pos);
  lds_barrier();
  for (uint32_t c0 = 0; c0 < cnt; c0 += kACh) {
    // the next chunk's records stream in during this whole chunk
    load(c0 + kACh, nm, nab, npos);
    // 1a. rank each record among the wave's earlier records of its slot
    uint32_t rank[kApplyPer], slot[kApplyPer];
#pragma unroll
    for (int j = 0; j < kApplyPer; ++j) {
      const bool live = c0 + w * kWaveRecs + j * kWave + l < cnt;
      slot[j] = smeta_slot(m[j]) & (kSbSlots - 1);
      rank[j] = live ? atomicAdd(&wcnt[w][slot[j]], 1u) : 0xFFFFFFFFu;
    }
    lds_barrier();
    // 1b. owner of slot t: prefix over the 4 waves; run length; reset the counters
    uint32_t run = 0;
#pragma unroll
    for (int q = 0; q < kApplyWaves; ++q) {
      const uint32_t c = wcnt[q][t];
      wpre[q][t] = run;
      wcnt[q][t] = 0;
      run += c;
    }
    // 1c. block exclusive scan of the run lengths -> run starts
    uint32_t inc = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (l >= (uint32_t)d) inc += y;
    }
    if (l == 63) wsum[w] = inc;
    lds_barrier();
    uint32_t start = inc - run;
    for (uint32_t q = 0; q < w; ++q) start += wsum[q];
    sstart[t] = start;
    lds_barrier();
    // 1d. place records in slot order
#pragma unroll
    for (int j = 0; j < kApplyPer; ++j) {
      if (rank[j] == 0xFFFFFFFFu) continue;
      const uint32_t p = sstart[slot[j]] + wpre[w][slot[j]] + rank[j];
      sm[p] = m[j];
      sab[p] = ab[j];
      sidx[p] = (uint16_t)(w * kWaveRecs + j * kWave + l);
    }
    lds_barrier();
    // 2. thread t applies its slot's commits in log order, state in registers (next record's LDS reads
    //    are issued before the current one is applied)
    if (run) {
      uint32_t mm = sm[start];
      u64x2 abv = sab[start];
      uint32_t ci = sidx[start];
      for (uint32_t k = 0; k < run; ++k) {
        const uint32_t pn = k + 1 < run ? start + k + 1 : start + k;
        const uint32_t mm2 = sm[pn];
        const u64x2 abv2 = sab[pn];
        const uint32_t ci2 = sidx[pn];
        uint64_t rv;
        const uint32_t stt = value_apply(smeta_op(mm), smeta_flags(mm), abv.x, abv.y, st_reg, rv, err);
        rstat[ci] = (uint8_t)stt;
        rval[ci] = rv;
        mm = mm2;
        abv = abv2;
        ci = ci2;
      }
    }
    lds_barrier();
    // 3. results back to the records' staging positions (contiguous within each run)
#pragma unroll
    for (int j = 0; j < kApplyPer; ++j) {
      const uint32_t ci = w * kWaveRecs + j * kWave + l;
      if (c0 + ci < cnt) {
        rst_status[pos[j]] = rstat[ci];
        rst_value[pos[j]] = rval[ci];
      }
    }
    lds_barrier();
#pragma unroll
    for (int j = 0; j < kApplyPer; ++j) {
      m[j] = nm[j];
      ab[j] = nab[j];
      pos[j] = npos[j];
    }
  }
  val_meta[(uint64_t)s * kSbSlots + t] = st_reg.meta;
  val_v[(uint64_t)s * kSbSlots + t] = st_reg.v;
  if (err) atomicOr(err_out, err);
}

// Engine-start self-check of the hardware property the stable rankings rely on: LDS atomics with return
// from one wave instruction that hit the same address are resolved in lane order.  *bad counts violations.
__global__ __launch_bounds__(256) void k_selfcheck_lds_order(uint32_t* __restrict__ bad) {
  __shared__ uint32_t tbl[256];
  const uint32_t t = threadIdx.x, l = t & 63;
  uint32_t x = 0x9E3779B9u ^ (t * 2654435761u) ^ (blockIdx.x * 40503u);
  uint32_t v = 0;
  for (uint32_t it = 0; it < 32; ++it) {
    tbl[t] = 0;
    lds_barrier();
    x = x * 1664525u + 1013904223u;
    const uint32_t key = ((x >> 8) & ((1u << (it & 3)) - 1)) + (t >> 6) * 64;
    const uint32_t old = atomicAdd(&tbl[key], 1u);
    for (uint32_t j = 0; j < 64; ++j) {  // uniform loop: every lane takes part in each shuffle
      const uint32_t kj = __shfl(key, j, 64), oj = __shfl(old, j, 64);
      if (j < l && kj == key && oj >= old) ++v;
    }
    lds_barrier();
  }
  if (v) atomicAdd(bad, v);
}

int launch_selfcheck(uint32_t* d_bad, hipStream_t st) {
  hipLaunchKernelGGL(k_selfcheck_lds_order, dim3(64), dim3(256), 0, st, d_bad);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_apply_value(const ValueArgs& a, hipStream_t st) {
  a.mark(K_APPLY_VALUE, 1, st);
  hipLaunchKernelGGL(k_apply_value, dim3(a.sb_val), dim3(kAT), 0, st, a.st_meta, a.st_ab, a.ttab, a.tiles, a.sb, a.sb_kind, a.val_meta,
                     a.val_v, a.rst_status, a.rst_value, a.err);
  a.mark(K_APPLY_VALUE, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
