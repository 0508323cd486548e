// map_ops.h — MapState key-op semantics shared by the region kernel (apply_map.hip) and the hot-key scan
// (apply_map_hot.hip).  Restates collections/src/main/java/io/atomix/collections/state/MapState.java:
//   containsKey :38-44, get :65-72, getOrDefault :77-84, put :89-110, putIfAbsent :115-133, remove :138-154,
//   removeIfPresent :159-178, replace :183-202, replaceIfPresent :207-228 (stores `value`, compares `replace`).
#pragma once
#include "common.h"

namespace cc {

__device__ inline bool map_key_op(uint32_t op) { return op == 60 || (op >= 62 && op <= 69); }
__device__ inline bool map_binds(uint32_t op) { return op == CC_OP_MAP_PUT || op == CC_OP_MAP_PUTIFABSENT; }
__device__ inline bool map_reads_ttl(uint32_t op) {
  return op == CC_OP_MAP_PUT || op == CC_OP_MAP_PUTIFABSENT || op == CC_OP_MAP_REPLACE || op == CC_OP_MAP_REPLACEIFPRESENT;
}

// Applies one committed key op to an entry (w: word with PRESENT + value tag, v: value payload).
// Returns the status byte; rv = result payload; `wrote` = the entry now holds this commit (commit index),
// `created` = a new HashMap node was created (insert index).
__device__ inline uint32_t map_apply(uint32_t op, uint32_t flags, uint64_t a, uint64_t b, uint32_t& w, uint64_t& v,
                                     uint64_t& rv, bool& wrote, bool& created) {
  const uint32_t ta = CC_FLAG_TAG_A(flags), tb = CC_FLAG_TAG_B(flags);
  const uint64_t pa = ta ? a : 0, pb = tb ? b : 0;  // canonical NULL payload
  const bool P = (w & kMwPresent) != 0;
  const uint32_t T = P ? mw_vtag(w) : CC_TAG_NULL;
  const uint64_t V = P ? v : 0;
  auto store = [&](uint32_t tag, uint64_t x) {
    w = (w & ~(kMwVtagMask | kMwUnseen)) | kMwPresent | (tag << 21);
    v = x;
  };
  auto erase = [&]() {
    w &= ~(kMwPresent | kMwVtagMask);
    v = 0;
  };
  wrote = created = false;
  rv = 0;
  switch (op) {
    case CC_OP_MAP_CONTAINSKEY:
      rv = P;
      return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
    case CC_OP_MAP_GET:  // a key mapped to null is present and returns null
      rv = V;
      return CC_STATUS(CC_ST_OK, T);
    case CC_OP_MAP_GETORDEFAULT:
      rv = P ? V : pa;
      return CC_STATUS(CC_ST_OK, P ? T : ta);
    case CC_OP_MAP_PUT:
      rv = V;
      store(ta, pa);
      wrote = true;
      created = !P;
      return CC_STATUS(CC_ST_OK, T);
    case CC_OP_MAP_PUTIFABSENT:
      if (P) {
        rv = V;
        return CC_STATUS(CC_ST_OK, T);
      }
      store(ta, pa);
      wrote = created = true;
      return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
    case CC_OP_MAP_REMOVE:
      rv = V;
      erase();
      return CC_STATUS(CC_ST_OK, T);
    case CC_OP_MAP_REMOVEIFPRESENT: {
      // fail: absent, or stored null and value not null, or stored non-null and !stored.equals(value)
      const bool fail = !P || (T == CC_TAG_NULL && ta != CC_TAG_NULL) || (T != CC_TAG_NULL && !(T == ta && V == pa));
      if (!fail) erase();
      rv = !fail;
      return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
    }
    case CC_OP_MAP_REPLACE:
      if (!P) return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      rv = V;
      store(ta, pa);
      wrote = true;
      return CC_STATUS(CC_ST_OK, T);
    case CC_OP_MAP_REPLACEIFPRESENT: {
      const bool ok = P && ((T == CC_TAG_NULL && tb == CC_TAG_NULL) || (T != CC_TAG_NULL && T == tb && V == pb));
      if (ok) {
        store(ta, pa);
        wrote = true;
      }
      rv = ok;
      return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
    }
  }
  return CC_STATUS(CC_ST_UNKNOWN_OP, CC_TAG_NULL);
}

// Result of a commit that has no entry in the region: unknown op, an op not applied here, or a key op on a key
// that is absent for the whole chunk.
__device__ inline uint32_t map_orphan(uint32_t op, uint32_t meta, uint32_t flags, uint64_t a, uint64_t b, uint64_t& rv,
                                      uint32_t& err) {
  rv = 0;
  if (!op_registered(CC_RES_MAP, op)) return CC_STATUS(CC_ST_UNKNOWN_OP, CC_TAG_NULL);
  // size / isEmpty are answered in the stream after the sub-batch (map_small.hip k_size_answer; k_ttl_replay in TTL mode),
  // containsValue rows that reach a region (the batch answers them in the stream) by map_cv.hip k_cv_answer; a clear
  // that reaches a region is applied in the stream (map_clear.hip: MapState.clear returns nothing)
  if (op == CC_OP_MAP_SIZE || op == CC_OP_MAP_ISEMPTY || op == CC_OP_MAP_CONTAINSVALUE || op == CC_OP_MAP_CLEAR)
    return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
  if (!map_key_op(op) || (map_reads_ttl(op) && (meta & kMetaTtl))) {
    err |= kErrUnsupported;
    return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
  }
  uint32_t w = kMwUsed;
  uint64_t v = 0;
  bool wrote, created;
  return map_apply(op, flags, a, b, w, v, rv, wrote, created);
}

// ---- key ops as transformers of one entry's state (absent | present(value, node)) ------------------------
//   put(v)          absent -> present(v, new node)     present -> present(v, same node)
//   putIfAbsent(v)  absent -> present(v, new node)     present -> unchanged
//   remove          absent -> absent                   present -> absent
//   replace(v)      absent -> absent                   present -> present(v, same node)
//   containsKey, get, getOrDefault: identity
// The family is closed under composition: each branch of a composite ends absent, unchanged, or present with
// the value of some commit and a node created by some commit (or the input's node), so a composite is two
// branch outcomes holding commit references and a scan over it is exact.  removeIfPresent/replaceIfPresent
// compare the stored value and are outside the family (their keys are applied sequentially).
constexpr uint32_t kBrAbsent = 0, kBrKeep = 1, kBrPresent = 2;
constexpr uint32_t kOrig = 0xFFFFFFFFu;

struct Br {
  uint32_t kind, v, n;  // outcome; value record; node record (kOrig: the input's node)
};
struct Comp {
  Br A, P;  // outcome when the entry is absent / present before the run
};

__device__ inline Comp comp_identity() { return Comp{{kBrAbsent, 0, 0}, {kBrKeep, 0, 0}}; }

// g applied to present(value v, node n)
__device__ inline Br apply_present(const Comp& g, uint32_t v, uint32_t n) {
  if (g.P.kind == kBrKeep) return Br{kBrPresent, v, n};
  if (g.P.kind == kBrPresent) return Br{kBrPresent, g.P.v, g.P.n == kOrig ? n : g.P.n};
  return Br{kBrAbsent, 0, 0};
}
// f first, then g
__device__ inline Comp compose(const Comp& f, const Comp& g) {
  Comp r;
  r.A = f.A.kind == kBrAbsent ? g.A : apply_present(g, f.A.v, f.A.n);
  if (f.P.kind == kBrKeep) r.P = g.P;
  else if (f.P.kind == kBrPresent) r.P = apply_present(g, f.P.v, f.P.n);
  else r.P = g.A;
  return r;
}

// a value-comparing op that is applied (replaceIfPresent with ttl > 0 is not: it fails the batch)
__device__ inline bool compares_value(uint32_t m) {
  const uint32_t op = smeta_op(m);
  return op == CC_OP_MAP_REMOVEIFPRESENT || (op == CC_OP_MAP_REPLACEIFPRESENT && !(m & kMetaTtl));
}
__device__ inline bool map_applied(uint32_t m) {
  const uint32_t op = smeta_op(m);
  return map_key_op(op) && !(map_reads_ttl(op) && (m & kMetaTtl));
}

// transformer of the commit staged at g (meta m)
__device__ inline Comp element(uint32_t m, uint32_t g) {
  Comp c = comp_identity();
  if (!map_applied(m)) return c;  // unknown op / not applied on the GPU: identity (result from map_orphan)
  switch (smeta_op(m)) {
    case CC_OP_MAP_PUT:
      c.A = Br{kBrPresent, g, g};
      c.P = Br{kBrPresent, g, kOrig};
      break;
    case CC_OP_MAP_PUTIFABSENT:
      c.A = Br{kBrPresent, g, g};
      break;
    case CC_OP_MAP_REMOVE:
      c.P = Br{kBrAbsent, 0, 0};
      break;
    case CC_OP_MAP_REPLACE:
      c.P = Br{kBrPresent, g, kOrig};
      break;
  }
  return c;
}

__device__ inline Comp comp_shfl_up(const Comp& c, int d) {
  Comp o;
  o.A.kind = __shfl_up(c.A.kind, d, 64);
  o.A.v = __shfl_up(c.A.v, d, 64);
  o.A.n = __shfl_up(c.A.n, d, 64);
  o.P.kind = __shfl_up(c.P.kind, d, 64);
  o.P.v = __shfl_up(c.P.v, d, 64);
  o.P.n = __shfl_up(c.P.n, d, 64);
  return o;
}

// A composite applied to an entry state (word w0, value v0, commit index ci0, insert index ins0): the state
// (word, value) map_apply works on, plus commit/insert index.  References are record slots of an LDS chunk.
__device__ inline void materialize_lds(const Comp& c, uint32_t w0, uint64_t v0, uint64_t ci0, uint64_t ins0,
                                       const uint32_t* rmeta, const u64x2* rab, const uint64_t* ridx, uint32_t& w,
                                       uint64_t& v, uint64_t& ci, uint64_t& ins) {
  const Br b = (w0 & kMwPresent) ? c.P : c.A;
  if (b.kind == kBrKeep) {
    w = w0;
    v = v0;
    ci = ci0;
    ins = ins0;
  } else if (b.kind == kBrAbsent) {
    w = w0 & ~(kMwPresent | kMwVtagMask);
    v = 0;
    ci = ci0;
    ins = ins0;
  } else {
    const uint32_t tag = CC_FLAG_TAG_A(smeta_flags(rmeta[b.v]));
    w = (w0 & ~(kMwVtagMask | kMwUnseen)) | kMwPresent | (tag << 21);
    v = tag ? rab[b.v].x : 0;
    ci = ridx[b.v];
    ins = b.n == kOrig ? ins0 : ridx[b.n];
  }
}

// The same, for a kernel that keeps the commit / insert indices in HBM: the (word, value) state and the chunk
// records whose commit rewrote the commit index (vref) and created the node (nref); kOrig: unchanged.
__device__ inline void materialize_ref(const Comp& c, uint32_t w0, uint64_t v0, const uint32_t* rmeta, const u64x2* rab,
                                       uint32_t& w, uint64_t& v, uint32_t& vref, uint32_t& nref) {
  const Br b = (w0 & kMwPresent) ? c.P : c.A;
  vref = nref = kOrig;
  if (b.kind == kBrKeep) {
    w = w0;
    v = v0;
  } else if (b.kind == kBrAbsent) {
    w = w0 & ~(kMwPresent | kMwVtagMask);
    v = 0;
  } else {
    const uint32_t tag = CC_FLAG_TAG_A(smeta_flags(rmeta[b.v]));
    w = (w0 & ~(kMwVtagMask | kMwUnseen)) | kMwPresent | (tag << 21);
    v = tag ? rab[b.v].x : 0;
    vref = b.v;
    nref = b.n;
  }
}

// in-order inclusive scan of one Comp per lane across a wave
__device__ inline Comp wave_scan(Comp c, uint32_t l) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const Comp o = comp_shfl_up(c, d);
    if (l >= (uint32_t)d) c = compose(o, c);
  }
  return c;
}

}  // namespace cc
