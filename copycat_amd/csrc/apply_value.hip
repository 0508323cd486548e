// apply_value.hip — AtomicValueState apply (also DistributedAtomicLong, whose add is a client-side CAS loop).
//
// One wave owns one bucket = 64 AtomicValueState instances (lane l <-> slot bucket*64 + l).  The wave
// walks its bucket's staging list (log order, built by partition.hip) 64 records per step.  Records of one
// step may hit the same resource several times; they are resolved IN LOG ORDER with ballots:
//   peers(j) = lanes whose record targets the same slot as lane j   (6 ballots over the slot bits)
//   rank(j)  = popcount(peers(j) & lanes-below-j)                    (its position in that chain)
// and round k applies every record of rank k — all targeting distinct slots — against the state held in
// LDS (read-modify-write, no atomics).  Rounds per step = the longest same-slot chain in the step.
//
// The per-op semantics restate AtomicValueState (atomic/src/main/java/io/atomix/atomic/state/AtomicValueState.java):
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

// Applies one committed AtomicValue op to (tag, v, cur); returns the status byte, result payload in *rv.
__device__ inline uint32_t value_apply(uint32_t op, uint32_t flags, uint64_t a, uint64_t b, ValState& s, uint64_t& rv,
                                       uint32_t& err) {
  const uint32_t ta = CC_FLAG_TAG_A(flags), tb = CC_FLAG_TAG_B(flags);
  const uint64_t pa = ta ? a : 0, pb = tb ? b : 0;  // canonical NULL payload
  const uint32_t tag = s.meta & 0xFF, cur = (s.meta >> 8) & 1;
  rv = 0;
  switch (op) {
    case CC_OP_VALUE_GET:  // return current != null ? value : null
      if (cur) { rv = s.v; return CC_STATUS(CC_ST_OK, tag); }
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

__global__ __launch_bounds__(256) void k_apply_value(const uint64_t* __restrict__ st_meta, const u64x2* __restrict__ st_ab,
                                                     const uint32_t* __restrict__ base, const uint32_t* __restrict__ tot,
                                                     uint32_t nb, uint32_t* __restrict__ val_meta, uint64_t* __restrict__ val_v,
                                                     uint8_t* __restrict__ out_status, uint64_t* __restrict__ out_value,
                                                     uint32_t* __restrict__ err_out) {
  __shared__ uint32_t sm[4][kWave];
  __shared__ uint64_t sv[4][kWave];
  const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint32_t bucket = blockIdx.x * 4 + w;
  if (bucket >= nb) return;  // wave-uniform
  const uint32_t slot = bucket * kResPerBucket + l;
  sm[w][l] = val_meta[slot];
  sv[w][l] = val_v[slot];
  const uint32_t lo = base[bucket], cnt = tot[bucket];
  const uint64_t lt = lanemask_lt();
  uint32_t err = 0;

  // software pipeline: records of step s+1 are loaded while step s resolves
  uint64_t meta = 0;
  u64x2 ab{0, 0};
  if (l < cnt) {
    meta = st_meta[lo + l];
    ab = st_ab[lo + l];
  }
  for (uint32_t s0 = 0; s0 < cnt; s0 += kWave) {
    const bool live = s0 + l < cnt;
    uint64_t nmeta = 0;
    u64x2 nab{0, 0};
    const uint32_t nj = s0 + kWave + l;
    if (nj < cnt) {
      nmeta = st_meta[lo + nj];
      nab = st_ab[lo + nj];
    }
    const uint32_t t = meta_lane(meta);
    uint64_t peers = ballot(live);
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const bool bit = (t >> k) & 1u;
      const uint64_t m = ballot(live && bit);
      peers &= bit ? m : ~m;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & lt);
    uint32_t st = 0;
    uint64_t rv = 0;
    bool pending = live;
    for (uint32_t k = 0; ballot(pending) != 0; ++k) {
      if (pending && rank == k) {
        ValState s{sm[w][t], sv[w][t]};
        st = value_apply(meta_op(meta), meta_flags(meta), ab.x, ab.y, s, rv, err);
        sm[w][t] = s.meta;
        sv[w][t] = s.v;
        pending = false;
      }
    }
    if (live) {
      const uint32_t pos = meta_pos(meta);
      out_status[pos] = (uint8_t)st;
      out_value[pos] = rv;
    }
    meta = nmeta;
    ab = nab;
  }
  val_meta[slot] = sm[w][l];
  val_v[slot] = sv[w][l];
  if (err) atomicOr(err_out, err);
}

int launch_apply_value(const ValueArgs& a, hipStream_t st) {
  a.mark(K_APPLY_VALUE, 1, st);
  hipLaunchKernelGGL(k_apply_value, dim3((a.nb + 3) / 4), dim3(256), 0, st, a.st_meta, a.st_ab, a.base, a.tot, a.nb,
                     a.val_meta, a.val_v, a.out_status, a.out_value, a.err);
  a.mark(K_APPLY_VALUE, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
