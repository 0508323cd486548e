// workload.cpp — deterministic synthetic committed-command streams (host side, seeded splitmix64).
//
// These are the benches' and tests' inputs, not part of the apply path.  Each generator writes SoA columns
// in the layout of cc_batch (include/copycat_apply.h).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/copycat_apply.h"

namespace {
struct SplitMix64 {
  uint64_t s;
  explicit SplitMix64(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint64_t below(uint64_t n) { return (uint64_t)(((unsigned __int128)next() * n) >> 64); }
};
}  // namespace

extern "C" {

// Config 2 stream: DistributedAtomicLong "add delta" client model (DistributedAtomicLong.java:117-146).
// Each add on a uniformly chosen resource r emits, in log order:
//   fresh cache (prob 1 - p_cold - p_stale):  CompareAndSet(E, E' + delta)             -> succeeds
//   cold cache  (prob p_cold):                Get; CompareAndSet(E, E' + delta)        -> succeeds
//   stale cache (prob p_stale):               CompareAndSet(stale, stale + delta) -> fails; Get; CAS(E, E'+delta)
// where E is the current value (null for a fresh resource, A4) and E' = E != null ? E : 0; delta ~ U[-1000, 1000].
// Values are java.lang.Long.  Instance slot = first_inst + r.  Returns the number of rows written (= n).
uint64_t wl_atomic_long(uint64_t n, uint32_t resources, uint32_t first_inst, uint64_t seed, uint32_t p_cold_ppm,
                        uint32_t p_stale_ppm, uint64_t index0, uint64_t* index, uint64_t* time, uint32_t* inst,
                        uint8_t* op, uint8_t* flags, uint64_t* a, uint64_t* b) {
  SplitMix64 rng(seed);
  std::vector<uint8_t> tag(resources, CC_TAG_NULL);
  std::vector<int64_t> val(resources, 0);
  uint64_t i = 0;
  auto emit = [&](uint32_t r, uint8_t o, uint8_t ta, uint64_t pa, uint8_t tb, uint64_t pb) {
    if (i >= n) return;
    if (index) index[i] = index0 + i;
    if (time) time[i] = (index0 + i) / 1024;  // ~1 ms of log time per 1024 entries
    inst[i] = first_inst + r;
    op[i] = o;
    flags[i] = CC_FLAGS(ta, tb, 0);
    a[i] = pa;
    b[i] = pb;
    ++i;
  };
  auto cas = [&](uint32_t r, uint8_t et, int64_t ev, int64_t delta) {
    const int64_t base = et == CC_TAG_NULL ? 0 : ev;
    const int64_t upd = (int64_t)((uint64_t)base + (uint64_t)delta);  // wrapping Long add
    emit(r, CC_OP_VALUE_CAS, et, (uint64_t)ev, CC_TAG_LONG, (uint64_t)upd);
    const bool ok = (tag[r] == CC_TAG_NULL && et == CC_TAG_NULL) || (tag[r] != CC_TAG_NULL && et == tag[r] && ev == val[r]);
    if (ok) {
      tag[r] = CC_TAG_LONG;
      val[r] = upd;
    }
    return ok;
  };
  while (i < n) {
    const uint32_t r = (uint32_t)rng.below(resources);
    const int64_t delta = (int64_t)rng.below(2001) - 1000;
    const uint64_t u = rng.below(1000000);
    if (u < p_stale_ppm) {
      const int64_t stale = (tag[r] == CC_TAG_NULL ? 0 : val[r]) + 1 + (int64_t)rng.below(1000);
      cas(r, CC_TAG_LONG, stale, delta);  // fails
      emit(r, CC_OP_VALUE_GET, 0, 0, 0, 0);
      cas(r, tag[r], tag[r] == CC_TAG_NULL ? 0 : val[r], delta);
    } else if (u < (uint64_t)p_stale_ppm + p_cold_ppm) {
      emit(r, CC_OP_VALUE_GET, 0, 0, 0, 0);
      cas(r, tag[r], tag[r] == CC_TAG_NULL ? 0 : val[r], delta);
    } else {
      cas(r, tag[r], tag[r] == CC_TAG_NULL ? 0 : val[r], delta);
    }
  }
  return i;
}

// Config 2 stream, one bench step of a run: the same client model as wl_atomic_long, continued from the model
// state (state_tag/state_val per resource: the value every client's CAS expects, updated in place to the state after
// the n emitted rows), generated on `threads` threads with the same rows for any thread count.
// Every add ends with a CAS that succeeds, so the value an add's CASes expect is the resource's value before the
// step plus the deltas of the earlier adds on it (a per-resource prefix sum):
//   pass 1 (parallel over chunks of adds): add k draws (resource, delta, kind, stale offset) from a counter-based
//           generator keyed by (seed, k); rows per chunk (fresh 1, cold 2, stale 3 rows per add); per-chunk
//           per-resource delta sums;
//   pass 2 (parallel over resources): the model state at the start of every chunk (exclusive prefix over chunks);
//   pass 3 (parallel over chunks): walk the chunk's adds from that state and write its rows contiguously.
// Row i gets log index index0 + i * index_stride (a rank's share of one global log: stride = world size) and log time
// index / 1024.  Only emitted rows change the model (an add cut off at row n leaves the rest unapplied).
uint64_t wl_atomic_long_step(uint64_t n, uint32_t resources, uint32_t first_inst, uint64_t seed, uint32_t p_cold_ppm,
                             uint32_t p_stale_ppm, uint64_t index0, uint64_t index_stride, uint8_t* state_tag,
                             int64_t* state_val, uint32_t threads, uint64_t* index, uint64_t* time, uint32_t* inst,
                             uint8_t* op, uint8_t* flags, uint64_t* a, uint64_t* b) {
  if (!resources || !n) return 0;
  const uint32_t T = std::max<uint32_t>(1, threads);
  const uint64_t R = resources;
  struct Add { uint32_t r; int16_t delta; uint8_t kind; uint16_t stale; };  // kind: 0 fresh, 1 cold, 2 stale
  auto draw = [&](uint64_t k) {
    SplitMix64 g(seed ^ (k * 0xD1B54A32D192ED03ull) ^ 0x5DEECE66Dull);
    Add x;
    x.r = (uint32_t)g.below(resources);
    x.delta = (int16_t)((int64_t)g.below(2001) - 1000);
    const uint64_t u = g.below(1000000);
    x.kind = u < p_stale_ppm ? 2 : (u < (uint64_t)p_stale_ppm + p_cold_ppm ? 1 : 0);
    x.stale = (uint16_t)g.below(1000);
    return x;
  };
  auto run = [&](auto&& fn, uint64_t count) {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < T; ++t) th.emplace_back([&, t] { for (uint64_t c = t; c < count; c += T) fn(c); });
    for (auto& x : th) x.join();
  };
  // chunks: enough adds for n rows (every add emits at least one row; ~1.4 on average)
  constexpr uint64_t kChunk = 1 << 20;
  const double rows_per_add = 1.0 + (p_cold_ppm + 2.0 * p_stale_ppm) / 1e6;
  uint64_t chunks = (uint64_t)((double)n / rows_per_add / kChunk) + 2;
  std::vector<Add> adds;
  std::vector<uint64_t> crow;
  std::vector<int64_t> dsum;   // [chunks][R] per-chunk delta sums
  std::vector<uint8_t> seen;   // [chunks][R]
  for (uint64_t have = 0;;) {  // (re)draw with more chunks if the estimate fell short
    adds.resize(chunks * kChunk);
    crow.assign(chunks + 1, 0);
    dsum.assign(chunks * R, 0);
    seen.assign(chunks * R, 0);
    run([&](uint64_t c) {
      uint64_t rows = 0;
      int64_t* ds = dsum.data() + c * R;
      uint8_t* sn = seen.data() + c * R;
      for (uint64_t k = c * kChunk; k < (c + 1) * kChunk; ++k) {
        const Add x = adds[k] = draw(k);
        rows += 1 + x.kind;
        ds[x.r] = (int64_t)((uint64_t)ds[x.r] + (uint64_t)(int64_t)x.delta);
        sn[x.r] = 1;
      }
      crow[c + 1] = rows;
    }, chunks);
    for (uint64_t c = 0; c < chunks; ++c) crow[c + 1] += crow[c];
    if (crow[chunks] >= n) break;
    have = chunks;
    chunks = have * 2;
  }
  // pass 2: model state at the start of every chunk (in place: dsum/seen of chunk c become the prefix before c)
  std::vector<uint8_t> tag0(state_tag, state_tag + R);
  std::vector<int64_t> val0(state_val, state_val + R);
  run([&](uint64_t t) {
    for (uint64_t r = t; r < R; r += T) {
      uint8_t tg = tag0[r];
      int64_t v = val0[r];
      for (uint64_t c = 0; c < chunks; ++c) {
        const int64_t d = dsum[c * R + r];
        const uint8_t s = seen[c * R + r];
        dsum[c * R + r] = v;
        seen[c * R + r] = tg;
        if (s) {
          v = (int64_t)((uint64_t)(tg == CC_TAG_NULL ? 0 : v) + (uint64_t)d);
          tg = CC_TAG_LONG;
        }
      }
    }
  }, T);
  // pass 3: rows, chunk by chunk from each chunk's start state; the chunk holding row n - 1 leaves the final state
  run([&](uint64_t c) {
    uint64_t i = crow[c];
    if (i >= n) return;
    std::vector<uint8_t> tg(seen.begin() + c * R, seen.begin() + (c + 1) * R);
    std::vector<int64_t> vl(dsum.begin() + c * R, dsum.begin() + (c + 1) * R);
    for (uint64_t k = c * kChunk; k < (c + 1) * kChunk && i < n; ++k) {
      const Add& x = adds[k];
      auto emit = [&](uint8_t o, uint8_t ta, uint64_t pa, uint8_t tb, uint64_t pb) {
        if (i >= n) return false;
        const uint64_t idx = index0 + i * index_stride;
        if (index) index[i] = idx;
        if (time) time[i] = idx / 1024;
        inst[i] = first_inst + x.r;
        op[i] = o;
        flags[i] = CC_FLAGS(ta, tb, 0);
        a[i] = pa;
        b[i] = pb;
        ++i;
        return true;
      };
      uint8_t& t = tg[x.r];
      int64_t& v = vl[x.r];
      auto cas = [&](uint8_t et, int64_t ev) {
        const int64_t upd = (int64_t)((uint64_t)(et == CC_TAG_NULL ? 0 : ev) + (uint64_t)(int64_t)x.delta);
        if (!emit(CC_OP_VALUE_CAS, et, (uint64_t)ev, CC_TAG_LONG, (uint64_t)upd)) return;
        if ((t == CC_TAG_NULL && et == CC_TAG_NULL) || (t != CC_TAG_NULL && et == t && ev == v)) {
          t = CC_TAG_LONG;
          v = upd;
        }
      };
      if (x.kind == 2) {  // stale cache: CAS(stale) fails, Get, CAS(current)
        cas(CC_TAG_LONG, (t == CC_TAG_NULL ? 0 : v) + 1 + (int64_t)x.stale);
        emit(CC_OP_VALUE_GET, 0, 0, 0, 0);
        cas(t, t == CC_TAG_NULL ? 0 : v);
      } else if (x.kind == 1) {  // cold cache: Get, CAS(current)
        emit(CC_OP_VALUE_GET, 0, 0, 0, 0);
        cas(t, t == CC_TAG_NULL ? 0 : v);
      } else {
        cas(t, t == CC_TAG_NULL ? 0 : v);
      }
    }
    if (crow[c + 1] >= n) {  // the last chunk with rows: its walk ends in the state after row n - 1
      memcpy(state_tag, tg.data(), R);
      memcpy(state_val, vl.data(), 8 * R);
    }
  }, chunks);
  return n;
}

// Adversarial AtomicValue stream for parity tests: every op (Get/Set/CAS/GetAndSet/Delete), every value tag
// (NULL/LONG/INT/BOOL/HANDLE) over a tiny value domain (so equals hits and misses), unknown instance slots,
// ops of other resource types (UNKNOWN_OP), and a hot set of `hot` resources receiving p_hot_ppm of the rows
// (long same-slot chains inside one 64-row step).
uint64_t wl_value_random(uint64_t n, uint32_t resources, uint32_t first_inst, uint32_t max_inst, uint64_t seed,
                         uint32_t hot, uint32_t p_hot_ppm, uint64_t index0, uint64_t* index, uint64_t* time, uint32_t* inst,
                         uint8_t* op, uint8_t* flags, uint64_t* a, uint64_t* b) {
  SplitMix64 rng(seed);
  static const uint8_t ops[] = {CC_OP_VALUE_GET, CC_OP_VALUE_SET, CC_OP_VALUE_CAS, CC_OP_VALUE_CAS, CC_OP_VALUE_CAS,
                                CC_OP_VALUE_GETANDSET, CC_OP_VALUE_GET};
  auto rand_val = [&](uint8_t& t, uint64_t& p) {
    const uint64_t k = rng.below(16);
    t = k < 3 ? CC_TAG_NULL : (k < 11 ? CC_TAG_LONG : (k < 13 ? CC_TAG_INT : (k < 15 ? CC_TAG_BOOL : CC_TAG_HANDLE)));
    p = t == CC_TAG_BOOL ? rng.below(2) : rng.below(4);
    if (t == CC_TAG_NULL) p = rng.next();  // non-canonical payload under NULL must be ignored
    if (t == CC_TAG_LONG && rng.below(8) == 0) p = ~p;  // negative longs
    if (t == CC_TAG_INT && (p & 1)) p = (uint64_t)(int64_t)(int32_t)(0x80000000u | (uint32_t)p);
  };
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t r = hot && rng.below(1000000) < p_hot_ppm ? (uint32_t)rng.below(hot) : (uint32_t)rng.below(resources);
    uint64_t k = rng.below(1000);
    uint8_t o = ops[rng.below(sizeof ops)];
    uint32_t s = first_inst + r;
    if (k < 3) s = max_inst + (uint32_t)rng.below(1000);                     // beyond the table
    else if (k < 6) o = (uint8_t)(60 + rng.below(13));                       // a MapState op on a value resource
    else if (k < 8) o = CC_OP_DELETE;                                        // DeleteCommand
    uint8_t ta, tb;
    uint64_t pa, pb;
    rand_val(ta, pa);
    rand_val(tb, pb);
    if (index) index[i] = index0 + i;
    if (time) time[i] = (index0 + i) / 1024;
    inst[i] = s;
    op[i] = o;
    flags[i] = CC_FLAGS(ta, tb, 0);
    a[i] = pa;
    b[i] = pb;
  }
  return n;
}

// MapState parity stream (adversarial): every key op, all key and value tags, null values, hot keys, ops of
// other resource types on a map (UNKNOWN_OP) and unknown instance slots.  Map m is instance slot first_inst + m.
// aux (ttl) is 0 or negative (no timer); small value domains make the conditional ops hit.
// value_compare_ops = 0 replaces removeIfPresent/replaceIfPresent by remove/replace.
uint64_t wl_map_random(uint64_t n, uint32_t maps, uint32_t first_inst, uint32_t max_inst, uint32_t keys, uint64_t seed,
                       uint32_t hot, uint32_t p_hot_ppm, uint64_t index0, uint64_t* index, uint64_t* time, uint32_t* inst,
                       uint8_t* op, uint8_t* flags, uint64_t* key, uint64_t* a, uint64_t* b, uint64_t* aux,
                       uint32_t value_compare_ops) {
  SplitMix64 rng(seed);
  static const uint8_t ops[] = {CC_OP_MAP_PUT, CC_OP_MAP_PUT, CC_OP_MAP_PUT, CC_OP_MAP_PUT, CC_OP_MAP_PUT,
                                CC_OP_MAP_PUTIFABSENT, CC_OP_MAP_PUTIFABSENT, CC_OP_MAP_GET, CC_OP_MAP_GET, CC_OP_MAP_GET,
                                CC_OP_MAP_GETORDEFAULT, CC_OP_MAP_CONTAINSKEY, CC_OP_MAP_REMOVE, CC_OP_MAP_REMOVE,
                                CC_OP_MAP_REMOVEIFPRESENT, CC_OP_MAP_REMOVEIFPRESENT, CC_OP_MAP_REPLACE, CC_OP_MAP_REPLACE,
                                CC_OP_MAP_REPLACEIFPRESENT, CC_OP_MAP_REPLACEIFPRESENT};
  auto rand_val = [&](uint8_t& t, uint64_t& p) {
    const uint64_t k = rng.below(16);
    t = k < 3 ? CC_TAG_NULL : (k < 11 ? CC_TAG_LONG : (k < 13 ? CC_TAG_INT : (k < 15 ? CC_TAG_BOOL : CC_TAG_HANDLE)));
    p = t == CC_TAG_BOOL ? rng.below(2) : rng.below(3);
    if (t == CC_TAG_NULL) p = rng.next();  // non-canonical payload under NULL must be ignored
    if (t == CC_TAG_LONG && rng.below(8) == 0) p = ~p;
  };
  for (uint64_t i = 0; i < n; ++i) {
    const bool is_hot = hot && rng.below(1000000) < p_hot_ppm;
    const uint32_t m = is_hot ? (uint32_t)rng.below(std::min(hot, maps)) : (uint32_t)rng.below(maps);
    uint32_t kt = 0;
    uint64_t kp;
    if (is_hot) {
      kp = rng.below(hot);
    } else {
      const uint64_t q = rng.below(16);
      kt = q < 12 ? 0 : (q < 14 ? 1 : (q < 15 ? 2 : 3));  // LONG / INT / BOOL / HANDLE keys
      kp = kt == 2 ? rng.below(2) : rng.below(keys);
      if (kt == 0 && rng.below(4) == 0) kp = ~kp;  // negative longs (spread over the hash)
    }
    uint8_t o = ops[rng.below(sizeof ops)];
    if (!value_compare_ops && (o == CC_OP_MAP_REMOVEIFPRESENT || o == CC_OP_MAP_REPLACEIFPRESENT))
      o = o == CC_OP_MAP_REMOVEIFPRESENT ? CC_OP_MAP_REMOVE : CC_OP_MAP_REPLACE;
    uint32_t s = first_inst + m;
    const uint64_t k = rng.below(1000);
    if (k < 3) s = max_inst + (uint32_t)rng.below(1000);  // unknown instance slot
    else if (k < 6) o = (uint8_t)(50 + rng.below(4));     // an AtomicValue op on a map: UNKNOWN_OP
    uint8_t ta, tb;
    uint64_t pa, pb;
    rand_val(ta, pa);
    rand_val(tb, pb);
    if (index) index[i] = index0 + i;
    if (time) time[i] = (index0 + i) / 1024;
    inst[i] = s;
    op[i] = o;
    flags[i] = CC_FLAGS(ta, tb, kt);
    key[i] = kp;
    a[i] = pa;
    b[i] = pb;
    if (aux) aux[i] = rng.below(4) == 0 ? (uint64_t)(-(int64_t)rng.below(3)) : 0;  // ttl <= 0: no timer
  }
  return n;
}

// Coordination parity stream: resources [0, R) with types types[r] (CC_RES_LOCK / ELECTION / GROUP / VALUE),
// each with K instances: instance slot r*K + k (instance id 1000 + slot, set up by the caller).  Ops per type:
// lock/unlock with timeouts {-1, 0, 1..40 ms}; listen/unlisten/isLeader; join/leave/execute(member = an
// instance id of that group, callback = handle); value get/set/CAS/getAndSet/listen/unlisten.  Rare Delete,
// ops of other types (UNKNOWN_OP) and unknown instance slots.  Time = 1 + index / 8 ms (non-decreasing).
// The lock client model of wl_coord_random, kept across calls (a bench applies one step's stream after another).
struct CoordModel {
  struct Waiter { uint32_t k; uint64_t deadline; };
  std::vector<int32_t> holder;
  std::vector<std::vector<Waiter>> queue;
  explicit CoordModel(uint32_t R) : holder(R, -1), queue(R) {}
};
void* wl_coord_model_new(uint32_t R) { return new CoordModel(R); }
void wl_coord_model_free(void* m) { delete static_cast<CoordModel*>(m); }

uint64_t wl_coord_random_model(void* model, uint64_t n, uint32_t R, uint32_t K, const uint8_t* types, uint32_t max_inst,
                               uint64_t seed, uint32_t p_delete_ppm, uint64_t index0, uint64_t* index, uint64_t* time,
                               uint32_t* inst, uint8_t* op, uint8_t* flags, uint64_t* key, uint64_t* a, uint64_t* b,
                               uint64_t* aux) {
  SplitMix64 rng(seed);
  // client model for locks (so a waiter queue never exceeds K): a holder unlocks, a waiter sends unlock (fails:
  // not the holder), anyone else locks.  Tracks LockState exactly, timeouts included (either timer order:
  // the model removes a waiter once its deadline has passed, before the instance's next request).
  using Waiter = CoordModel::Waiter;
  CoordModel& M = *static_cast<CoordModel*>(model);
  std::vector<int32_t>& holder = M.holder;
  std::vector<std::vector<Waiter>>& queue = M.queue;
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t r = (uint32_t)rng.below(R), k = (uint32_t)rng.below(K);
    const uint64_t now = 1 + (index0 + i) / 8;
    uint32_t s = r * K + k;
    uint8_t o = 0, ta = 0, tb = 0;
    uint64_t pa = 0, pb = 0, ky = 0, ax = 0;
    const uint64_t u = rng.below(100);
    switch (types[r]) {
      case CC_RES_LOCK: {
        auto& q = queue[r];
        // waiters whose timeout passed are gone (conservatively: strictly before now, both timer orders agree)
        q.erase(std::remove_if(q.begin(), q.end(), [&](const Waiter& w) { return w.deadline + 1 < now; }), q.end());
        const bool waiting = std::any_of(q.begin(), q.end(), [&](const Waiter& w) { return w.k == k; });
        if (holder[r] == (int32_t)k || waiting || u < 10) {
          o = CC_OP_LOCK_UNLOCK;
          if (holder[r] == (int32_t)k) {
            if (q.empty()) holder[r] = -1;
            else { holder[r] = (int32_t)q.front().k; q.erase(q.begin()); }
          }
        } else {
          o = CC_OP_LOCK_LOCK;
          const uint64_t v = rng.below(10);
          ax = v < 6 ? (uint64_t)-1 : (v < 8 ? 0 : 1 + rng.below(40));
          if (holder[r] < 0) holder[r] = (int32_t)k;
          else if (ax != 0) q.push_back(Waiter{k, ax == (uint64_t)-1 ? ~0ull - 2 : now + ax});
        }
        break;
      }
      case CC_RES_ELECTION:
        o = u < 45 ? CC_OP_ELECT_LISTEN : (u < 90 ? CC_OP_ELECT_UNLISTEN : CC_OP_ELECT_ISLEADER);
        break;
      case CC_RES_GROUP:
        o = u < 45 ? CC_OP_GROUP_JOIN : (u < 85 ? CC_OP_GROUP_LEAVE : CC_OP_GROUP_EXECUTE);
        if (o == CC_OP_GROUP_EXECUTE) {
          ky = 1000 + r * K + rng.below(K);  // a member id of this group (maybe not joined)
          ta = CC_TAG_HANDLE;
          pa = rng.below(100);
        }
        break;
      default: {  // value
        static const uint8_t vops[] = {CC_OP_VALUE_GET, CC_OP_VALUE_SET, CC_OP_VALUE_CAS, CC_OP_VALUE_GETANDSET,
                                       CC_OP_VALUE_LISTEN, CC_OP_VALUE_UNLISTEN, CC_OP_VALUE_CAS};
        o = vops[rng.below(sizeof vops)];
        ta = rng.below(4) ? CC_TAG_LONG : CC_TAG_NULL;
        tb = rng.below(4) ? CC_TAG_LONG : CC_TAG_NULL;
        pa = rng.below(3);
        pb = rng.below(3);
      }
    }
    const uint64_t x = rng.below(1000000);
    if (types[r] != CC_RES_LOCK) {  // locks stay on the client model (Delete on a lock: KATs)
      if (x < p_delete_ppm) o = CC_OP_DELETE;
      else if (x < p_delete_ppm + 2000) {  // possibly another type's op (never schedule: not applied on the GPU)
        o = (uint8_t)(50 + rng.below(80));
        if (o == CC_OP_GROUP_SCHEDULE) o = CC_OP_GROUP_LEAVE;
      }
      else if (x < p_delete_ppm + 4000) s = max_inst + (uint32_t)rng.below(100);  // unknown instance slot
    }
    if (index) index[i] = index0 + i;
    if (time) time[i] = now;
    inst[i] = s;
    op[i] = o;
    flags[i] = CC_FLAGS(ta, tb, 0);
    key[i] = ky;
    a[i] = pa;
    b[i] = pb;
    if (aux) aux[i] = ax;
  }
  return n;
}

uint64_t wl_coord_random(uint64_t n, uint32_t R, uint32_t K, const uint8_t* types, uint32_t max_inst, uint64_t seed,
                         uint32_t p_delete_ppm, uint64_t index0, uint64_t* index, uint64_t* time, uint32_t* inst,
                         uint8_t* op, uint8_t* flags, uint64_t* key, uint64_t* a, uint64_t* b, uint64_t* aux) {
  CoordModel m(R);
  return wl_coord_random_model(&m, n, R, K, types, max_inst, seed, p_delete_ppm, index0, index, time, inst, op, flags, key,
                               a, b, aux);
}

// Config 3 stream: DistributedMap put/get/remove (45/45/10) over `pairs` (power of two) distinct
// (map, key) pairs spread over `maps` maps; pair rank ~ Zipf(s).  Rank r -> pair (r * 0x9E3779B1 + 0x7F4A7C15)
// mod pairs (a bijection), pair -> map pair % maps (instance slot first_inst + map), key = mix64(pair) (Long).
// Rows [row0, row0 + n) of the stream are written; any sub-range gives the same rows (chunks are seeded by
// their 64K-row block), so the bench can generate and upload a 1e9-row stream block by block on `threads`.
uint64_t wl_map_zipf(uint64_t row0, uint64_t n, uint32_t maps, uint32_t pairs, double s, uint32_t first_inst,
                     uint64_t seed, uint32_t threads, uint64_t* index, uint64_t* time, uint32_t* inst, uint8_t* op,
                     uint8_t* flags, uint64_t* key, uint64_t* a, uint64_t* b) {
  if (!pairs || (pairs & (pairs - 1)) || !maps) return 0;
  // Walker alias table over the Zipf pmf
  std::vector<double> pr(pairs);
  double z = 0;
  for (uint32_t r = 0; r < pairs; ++r) z += (pr[r] = 1.0 / std::pow((double)r + 1.0, s));
  std::vector<uint32_t> alias(pairs), small, large;
  std::vector<double> q(pairs);
  for (uint32_t r = 0; r < pairs; ++r) {
    q[r] = pr[r] / z * pairs;
    (q[r] < 1.0 ? small : large).push_back(r);
  }
  while (!small.empty() && !large.empty()) {
    const uint32_t l = small.back(), g = large.back();
    small.pop_back();
    alias[l] = g;
    q[g] -= 1.0 - q[l];
    if (q[g] < 1.0) {
      large.pop_back();
      small.push_back(g);
    }
  }
  for (uint32_t r : large) q[r] = 1.0, alias[r] = r;
  for (uint32_t r : small) q[r] = 1.0, alias[r] = r;
  std::vector<uint32_t> qthr(pairs);
  for (uint32_t r = 0; r < pairs; ++r) qthr[r] = (uint32_t)std::min(4294967295.0, q[r] * 4294967296.0);
  constexpr uint64_t kBlock = 65536;
  auto gen = [&](uint64_t blk0, uint64_t blk1) {
    for (uint64_t blk = blk0; blk < blk1; ++blk) {
      SplitMix64 rng(seed ^ (blk * 0xD1B54A32D192ED03ull));
      const uint64_t r0 = blk * kBlock;
      for (uint64_t rr = r0; rr < r0 + kBlock; ++rr) {
        const uint64_t x = rng.next(), y = rng.next(), w = rng.next();
        if (rr < row0 || rr >= row0 + n) continue;
        uint32_t rank = (uint32_t)(((x & 0xFFFFFFFFull) * pairs) >> 32);
        if ((uint32_t)(x >> 32) >= qthr[rank]) rank = alias[rank];
        const uint32_t pair = (uint32_t)(rank * 0x9E3779B1u + 0x7F4A7C15u) & (pairs - 1);
        SplitMix64 km(pair);
        const uint64_t i = rr - row0;
        const uint32_t u = (uint32_t)(y % 100);
        if (index) index[i] = 1 + rr;
        if (time) time[i] = (1 + rr) / 1024;
        inst[i] = first_inst + pair % maps;
        op[i] = u < 45 ? CC_OP_MAP_PUT : (u < 90 ? CC_OP_MAP_GET : CC_OP_MAP_REMOVE);
        flags[i] = CC_FLAGS(u < 45 ? CC_TAG_LONG : CC_TAG_NULL, CC_TAG_NULL, 0);
        key[i] = km.next();
        a[i] = u < 45 ? w : 0;
        b[i] = 0;
      }
    }
  };
  const uint64_t b0 = row0 / kBlock, b1 = (row0 + n + kBlock - 1) / kBlock;
  const uint32_t nt = std::max<uint32_t>(1, std::min<uint64_t>(threads ? threads : 1, b1 - b0));
  std::vector<std::thread> th;
  const uint64_t per = (b1 - b0 + nt - 1) / nt;
  for (uint32_t t = 0; t < nt; ++t) {
    const uint64_t lo = b0 + t * per, hi = std::min(b1, lo + per);
    if (lo < hi) th.emplace_back(gen, lo, hi);
  }
  for (auto& x : th) x.join();
  return n;
}

}  // extern "C"
