// apply_value.hip — AtomicValueState apply (also DistributedAtomicLong, whose add is a client-side CAS loop).
//
// One 256-thread workgroup owns one super-bucket = 256 AtomicValueState instances, held in LDS for the whole
// launch.  It walks the super-bucket's staging list (log order, built by partition.hip) in chunks of 2048
// records, prefetching the next chunk into registers while it resolves the current one:
//   1. a stable 2-bit multisplit of the chunk in LDS hands wave w exactly the records of its 64 slots;
//   2. each wave resolves its records 64 at a time, IN LOG ORDER, with ballots:
//        peers(j) = lanes whose record targets the same slot as lane j   (6 ballots over the slot bits)
//        rank(j)  = popcount(peers(j) & lanes-below-j)                    (position in that chain)
//      round k applies every record of rank k — all on distinct slots — as an LDS read-modify-write;
//   3. the chunk's results are staged in LDS and written back contiguously (staging order); k_unpermute
//      later returns them to log order.
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

constexpr int kAT = kApplyWaves * kWave;  // 256 threads
constexpr int kACh = kAT * kApplyPer;     // 2048 records per chunk
constexpr int kSbSlots = kApplyWaves * kLaneRes;

__global__ __launch_bounds__(kAT) void k_apply_value(const uint32_t* __restrict__ st_meta, const u64x2* __restrict__ st_ab,
                                                    const uint32_t* __restrict__ base, const uint32_t* __restrict__ tot,
                                                    uint32_t* __restrict__ val_meta, uint64_t* __restrict__ val_v,
                                                    uint8_t* __restrict__ rst_status, uint64_t* __restrict__ rst_value,
                                                    uint32_t* __restrict__ err_out) {
  __shared__ uint32_t smeta[kSbSlots];
  __shared__ uint64_t sv[kSbSlots];
  __shared__ u64x2 lab[kACh];
  __shared__ uint32_t lmeta[kACh];
  __shared__ uint16_t lidx[kACh];
  __shared__ uint64_t rval[kACh];
  __shared__ uint8_t rstat[kACh];
  __shared__ uint32_t gcnt[kApplyPer][kApplyWaves][kApplyWaves];
  __shared__ uint32_t kseg[kApplyWaves + 1];

  const uint32_t s = blockIdx.x, t = threadIdx.x, w = t >> 6, l = t & 63;
  const uint64_t lt = lanemask_lt();
  for (uint32_t q = t; q < kSbSlots; q += kAT) {
    smeta[q] = val_meta[(uint64_t)s * kSbSlots + q];
    sv[q] = val_v[(uint64_t)s * kSbSlots + q];
  }
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
  for (uint32_t c0 = 0; c0 < cnt; c0 += kACh) {
    // prefetch the next chunk while this one resolves
    uint32_t nm[kApplyPer];
    u64x2 nab[kApplyPer];
#pragma unroll
    for (int j = 0; j < kApplyPer; ++j) {
      const uint32_t c = c0 + kACh + j * kAT + t;
      nm[j] = 0;
      nab[j] = u64x2{0, 0};
      if (c < cnt) {
        nm[j] = st_meta[lo + c];
        nab[j] = st_ab[lo + c];
      }
    }
    // 1. stable multisplit of the chunk (order c = j*256 + t) by owning wave = slot >> 6
    uint32_t rank[kApplyPer], key[kApplyPer];
    bool live[kApplyPer];
#pragma unroll
    for (int j = 0; j < kApplyPer; ++j) {
      live[j] = c0 + j * kAT + t < cnt;
      key[j] = (smeta_slot(m[j]) >> 6) & (kApplyWaves - 1);
      const uint64_t lv = ballot(live[j]);
      const uint64_t b0 = ballot(live[j] && (key[j] & 1));
      const uint64_t b1 = ballot(live[j] && (key[j] & 2));
      const uint64_t mk0 = lv & ~b0 & ~b1, mk1 = b0 & ~b1, mk2 = b1 & ~b0, mk3 = b0 & b1;
      const uint64_t mine = key[j] == 0 ? mk0 : key[j] == 1 ? mk1 : key[j] == 2 ? mk2 : mk3;
      rank[j] = (uint32_t)__popcll(mine & lt);
      if (l < kApplyWaves) {
        const uint64_t mk = l == 0 ? mk0 : l == 1 ? mk1 : l == 2 ? mk2 : mk3;
        gcnt[j][w][l] = (uint32_t)__popcll(mk);
      }
    }
    __syncthreads();
    if (t < kApplyWaves) {
      uint32_t run = 0;
      for (int j = 0; j < kApplyPer; ++j)
        for (int q = 0; q < kApplyWaves; ++q) {
          const uint32_t c = gcnt[j][q][t];
          gcnt[j][q][t] = run;
          run += c;
        }
      kseg[t + 1] = run;  // segment sizes, prefixed below
    }
    __syncthreads();
    if (t == 0) {
      kseg[0] = 0;
      for (int k = 1; k <= kApplyWaves; ++k) kseg[k] += kseg[k - 1];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kApplyPer; ++j) {
      if (!live[j]) continue;
      const uint32_t p = kseg[key[j]] + gcnt[j][w][key[j]] + rank[j];
      lmeta[p] = m[j];
      lab[p] = ab[j];
      lidx[p] = (uint16_t)(j * kAT + t);
    }
    __syncthreads();
    // 2. wave w resolves its segment against its 64 slots, in log order
    const uint32_t seg_lo = kseg[w], seg_hi = kseg[w + 1];
    for (uint32_t q0 = seg_lo; q0 < seg_hi; q0 += kWave) {
      const uint32_t q = q0 + l;
      const bool lv = q < seg_hi;
      const uint32_t mm = lv ? lmeta[q] : 0;
      const u64x2 abv = lv ? lab[q] : u64x2{0, 0};
      const uint32_t rr = smeta_slot(mm) & 63;
      uint64_t peers = ballot(lv);
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const bool bit = (rr >> k) & 1u;
        const uint64_t mk = ballot(lv && bit);
        peers &= bit ? mk : ~mk;
      }
      const uint32_t rk = (uint32_t)__popcll(peers & lt);
      const uint32_t si = w * kLaneRes + rr;
      uint32_t st = 0;
      uint64_t rv = 0;
      bool pending = lv;
      for (uint32_t k = 0; ballot(pending) != 0; ++k) {
        if (pending && rk == k) {
          ValState vs{smeta[si], sv[si]};
          st = value_apply(smeta_op(mm), smeta_flags(mm), abv.x, abv.y, vs, rv, err);
          smeta[si] = vs.meta;
          sv[si] = vs.v;
          pending = false;
        }
      }
      if (lv) {
        const uint32_t c = lidx[q];
        rstat[c] = (uint8_t)st;
        rval[c] = rv;
      }
    }
    __syncthreads();
    // 3. results back in staging order, contiguous
    const uint32_t nhere = cnt - c0 < (uint32_t)kACh ? cnt - c0 : (uint32_t)kACh;
    for (uint32_t c = t; c < nhere; c += kAT) {
      rst_status[lo + c0 + c] = rstat[c];
      rst_value[lo + c0 + c] = rval[c];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kApplyPer; ++j) {
      m[j] = nm[j];
      ab[j] = nab[j];
    }
  }
  for (uint32_t q = t; q < kSbSlots; q += kAT) {
    val_meta[(uint64_t)s * kSbSlots + q] = smeta[q];
    val_v[(uint64_t)s * kSbSlots + q] = sv[q];
  }
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
