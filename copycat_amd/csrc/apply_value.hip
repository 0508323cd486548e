// apply_value.hip — AtomicValueState apply (also DistributedAtomicLong, whose add is a client-side CAS loop).
//
// One 256-thread workgroup owns one super-bucket = 256 AtomicValueState instances: thread t holds slot t's
// state in registers for the whole launch.  It walks the super-bucket's staging list (log order, built by
// partition.hip) in chunks of 2048 records, prefetching the next chunk into registers while it resolves the
// current one: a stable counting sort of the chunk by slot (ballot ranking + per-slot prefix sums in LDS)
// gives every slot its commits in log order, and each thread applies its slot's chain sequentially — the
// same order the reference's single state-machine thread would (ResourceManager.java:56-72).  Results are
// staged in LDS and written back contiguously in staging order; k_unpermute returns them to log order.
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
__device__ inline uint32_t value_apply(uint32_t op, uint32_t flags, uint64_t a, uint64_t b, ValState& s, uint64_t& rv,
                                       uint32_t& err) {
  const uint32_t ta = CC_FLAG_TAG_A(flags), tb = CC_FLAG_TAG_B(flags);
  const uint64_t pa = ta ? a : 0, pb = tb ? b : 0;  // canonical NULL payload
  const uint32_t tag = s.meta & 0xFF, cur = (s.meta >> 8) & 1;
  rv = 0;
  switch (op) {
    case CC_OP_VALUE_GET:  // return current != null ? value : null
      if (cur) {
        rv = s.v;
        return CC_STATUS(CC_ST_OK, tag);
      }
      return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
    case CC_OP_VALUE_SET:  // cleanCurrent(); value = v; setCurrent(commit)
      s.meta = vmeta(ta, 1);
      s.v = pa;
      return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
    case CC_OP_VALUE_CAS: {  // (value == null && expect == null) || (value != null && expect != null && value.equals(expect))
      const bool eq = (tag == CC_TAG_NULL && ta == CC_TAG_NULL) ||
                      (tag != CC_TAG_NULL && ta != CC_TAG_NULL && tag == ta && s.v == pa);
      if (eq) {
        s.meta = vmeta(tb, 1);
        s.v = pb;
      }
      rv = eq ? 1 : 0;
      return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
    }
    case CC_OP_VALUE_GETANDSET: {  // result = value; value = v; setCurrent
      rv = s.v;
      const uint32_t rt = tag;
      s.meta = vmeta(ta, 1);
      s.v = pa;
      return CC_STATUS(CC_ST_OK, rt);
    }
    case CC_OP_DELETE:  // if (current != null) { current = null; value = null; }
      if (cur) {
        s.meta = 0;
        s.v = 0;
      }
      return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
    case CC_OP_VALUE_LISTEN:
    case CC_OP_VALUE_UNLISTEN:
      err |= kErrUnsupported;
      return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
    default:  // IllegalStateException "unknown operation type" (ResourceStateMachineExecutor.java:78)
      return CC_STATUS(CC_ST_UNKNOWN_OP, CC_TAG_NULL);
  }
}

constexpr int kAT = kApplyWaves * kWave;  // 256 threads = 256 slots of the super-bucket
constexpr int kACh = kAT * kApplyPer;     // 2048 records per chunk
constexpr int kSbSlots = kApplyWaves * kLaneRes;
constexpr int kGroups = kApplyPer * kApplyWaves;  // (j, wave) groups of 64 records, in log order

// One workgroup per super-bucket; thread t owns slot t (its AtomicValueState lives in two registers).
// Per chunk of 2048 staging records (record c = j*256 + t, log order = (j, wave, lane)):
//   1. a stable counting sort of the chunk by slot: ballot ranking inside each (j, wave) group, per-group
//      per-slot counts in LDS (tagged with the chunk number, so the table is never cleared), each owner
//      thread scans its slot's 32 group counts, a block scan gives each slot's run start;
//   2. thread t walks its slot's run sequentially — the reference's one-commit-at-a-time order, per slot;
//   3. results go back through LDS to staging order and out contiguously.
__global__ __launch_bounds__(kAT) void k_apply_value(const uint32_t* __restrict__ st_meta, const u64x2* __restrict__ st_ab,
                                                    const uint32_t* __restrict__ base, const uint32_t* __restrict__ tot,
                                                    uint32_t* __restrict__ val_meta, uint64_t* __restrict__ val_v,
                                                    uint8_t* __restrict__ rst_status, uint64_t* __restrict__ rst_value,
                                                    uint32_t* __restrict__ err_out) {
  __shared__ u64x2 sab[kACh];
  __shared__ uint32_t sm[kACh];
  __shared__ uint16_t sidx[kACh];
  __shared__ uint64_t rval[kACh];
  __shared__ uint8_t rstat[kACh];
  __shared__ uint32_t gcnt[kGroups][kSbSlots];  // (chunk+1) << 12 | value (count, then prefix); else stale
  __shared__ uint32_t sstart[kSbSlots];
  __shared__ uint32_t wsum[kApplyWaves];

  const uint32_t s = blockIdx.x, t = threadIdx.x, w = t >> 6, l = t & 63;
  const uint64_t lt = lanemask_lt();
  ValState st_reg{val_meta[(uint64_t)s * kSbSlots + t], val_v[(uint64_t)s * kSbSlots + t]};
  for (uint32_t q = t; q < kGroups * kSbSlots; q += kAT) (&gcnt[0][0])[q] = 0;
  const uint32_t lo = base[s], cnt = tot[s];
  uint32_t err = 0;

  uint32_t m[kApplyPer];
  u64x2 ab[kApplyPer];
#pragma unroll
  for (int j = 0; j < kApplyPer; ++j) {
    const uint32_t c = j * kAT + t;
    m[j] = 0;
    ab[j] = u64x2{0, 0};
    if (c < cnt) {
      m[j] = st_meta[lo + c];
      ab[j] = st_ab[lo + c];
    }
  }
  __syncthreads();
  uint32_t chunk_tag = 0;
  for (uint32_t c0 = 0; c0 < cnt; c0 += kACh) {
    chunk_tag += 1u << 12;
    // 1a. rank inside each (j, wave) group by slot (8 ballots); group leaders publish counts
    uint32_t rank[kApplyPer], slot[kApplyPer];
#pragma unroll
    for (int j = 0; j < kApplyPer; ++j) {
      const bool live = c0 + j * kAT + t < cnt;
      slot[j] = smeta_slot(m[j]) & (kSbSlots - 1);
      uint64_t peers = ballot(live);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool bit = (slot[j] >> k) & 1u;
        const uint64_t mk = ballot(live && bit);
        peers &= bit ? mk : ~mk;
      }
      rank[j] = live ? (uint32_t)__popcll(peers & lt) : 0xFFFFFFFFu;
      if (live && (peers & lt) == 0) gcnt[j * kApplyWaves + w][slot[j]] = chunk_tag | (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // 1b. owner of slot t: exclusive prefix over the 32 groups; run length
    uint32_t run = 0;
#pragma unroll 8
    for (int g = 0; g < kGroups; ++g) {
      const uint32_t v = gcnt[g][t];
      const uint32_t c = (v & ~0xFFFu) == chunk_tag ? (v & 0xFFFu) : 0;
      gcnt[g][t] = chunk_tag | run;  // prefix, tagged
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
    __syncthreads();
    uint32_t start = inc - run;
    for (uint32_t q = 0; q < w; ++q) start += wsum[q];
    sstart[t] = start;
    __syncthreads();
    // 1d. place records in slot order
#pragma unroll
    for (int j = 0; j < kApplyPer; ++j) {
      if (rank[j] == 0xFFFFFFFFu) continue;
      const uint32_t p = sstart[slot[j]] + (gcnt[j * kApplyWaves + w][slot[j]] & 0xFFFu) + rank[j];
      sm[p] = m[j];
      sab[p] = ab[j];
      sidx[p] = (uint16_t)(j * kAT + t);
    }
    __syncthreads();
    // prefetch the next chunk while this one resolves
#pragma unroll
    for (int j = 0; j < kApplyPer; ++j) {
      const uint32_t c = c0 + kACh + j * kAT + t;
      m[j] = 0;
      ab[j] = u64x2{0, 0};
      if (c < cnt) {
        m[j] = st_meta[lo + c];
        ab[j] = st_ab[lo + c];
      }
    }
    // 2. thread t applies its slot's commits in log order, state in registers
    for (uint32_t k = 0; k < run; ++k) {
      const uint32_t p = start + k;
      const uint32_t mm = sm[p];
      const u64x2 abv = sab[p];
      uint64_t rv;
      const uint32_t stt = value_apply(smeta_op(mm), smeta_flags(mm), abv.x, abv.y, st_reg, rv, err);
      const uint32_t ci = sidx[p];
      rstat[ci] = (uint8_t)stt;
      rval[ci] = rv;
    }
    __syncthreads();
    // 3. results back in staging order, contiguous
    const uint32_t nhere = cnt - c0 < (uint32_t)kACh ? cnt - c0 : (uint32_t)kACh;
    for (uint32_t c = t; c < nhere; c += kAT) {
      rst_status[lo + c0 + c] = rstat[c];
      rst_value[lo + c0 + c] = rval[c];
    }
    __syncthreads();
  }
  val_meta[(uint64_t)s * kSbSlots + t] = st_reg.meta;
  val_v[(uint64_t)s * kSbSlots + t] = st_reg.v;
  if (err) atomicOr(err_out, err);
}

int launch_apply_value(const ValueArgs& a, hipStream_t st) {
  a.mark(K_APPLY_VALUE, 1, st);
  hipLaunchKernelGGL(k_apply_value, dim3(a.sb), dim3(kAT), 0, st, a.st_meta, a.st_ab, a.base, a.tot, a.val_meta, a.val_v,
                     a.rst_status, a.rst_value, a.err);
  a.mark(K_APPLY_VALUE, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
