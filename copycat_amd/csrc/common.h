// common.h — shared device/host definitions of the MI355X commit-apply engine (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/copycat_apply.h"

namespace cc {

// ---- geometry -----------------------------------------------------------------------------------------
constexpr int kWave = 64;                 // CDNA wavefront
constexpr int kSbShift = 8;               // super-bucket = slot >> 8 (256 slots: one apply workgroup)
constexpr int kMaxSb = 512;               // => max_resources <= 131072 with 256-slot super-buckets
constexpr int kMapRegion = 2048;          // map table entries per region (one map apply workgroup, LDS-resident)
constexpr int kMaxMapSb = 2048;           // map regions => map_capacity <= 2M live entries (load <= 1/2)
constexpr int kMaxSbTotal = kMaxSb + kMaxMapSb;
constexpr int kPT = 1024;                 // partition workgroup threads (16 waves)
constexpr int kPW = kPT / kWave;
constexpr int kTile = 16384;              // commits per partition tile (one workgroup)
#ifndef CC_PART_CHUNK
#define CC_PART_CHUNK 4096
#endif
constexpr int kChunk = CC_PART_CHUNK;              // commits per LDS-staged chunk of a tile (value-only engines)
constexpr int kChunkMaps = 2048;          // ... when map commits (bigger records) share the partition
constexpr int kScanGroups = 16;           // row groups of the tile-prefix scan (1024-thread WG)
constexpr int kMaxTiles = 1024;           // tiles per sub-batch => sub-batch <= 16M commits
constexpr int kPersistGrid = 256;         // persistent tile loops: one 1024-thread workgroup per CU
constexpr int kV3Tile = 8192;             // value-only pipeline (value_path.hip): commits per partition tile
constexpr int kV3MaxTiles = 3072;         //   tiles per sub-batch (a value-only engine's sub-batch <= 24 Mi commits)
constexpr uint32_t kNoRes = 0xFFFFFFFFu;

// device error bits (d_err)
constexpr uint32_t kErrUnsupported = 1u;
constexpr uint32_t kErrEvents = 2u;
constexpr uint32_t kErrCapacity = 4u;
// hot map keys (apply_map_hot.hip): detected per sub-batch, applied by a multi-workgroup scan
#ifndef CC_HOT_MAX
#define CC_HOT_MAX 256
#endif
constexpr int kHotMax = CC_HOT_MAX;  // hot keys per sub-batch
constexpr int kHotSlots = 1024;     // LDS hash of the hot set in the partition kernel
#ifndef CC_HOT_PIECE
#define CC_HOT_PIECE 1024  // (4096: 16 commits per thread, ~48 KB of a wave's records in flight per step; 1024: the hot
#endif                     //  path 32.0 -> 23.3 ms per c3 step, profiles/r03/ab_hp)
constexpr int kHotPiece = CC_HOT_PIECE;  // commits per scan piece (one workgroup)
constexpr int kHotMaxPieces = (16 << 20) / kHotPiece;
struct HotKey {
  uint64_t h64;    // map_hash(slot, key tag, key)
  uint64_t key;
  uint32_t ident;  // mw_ident(slot, key tag)
  uint32_t pos;    // table entry (region * 2048 + index)
};     // a map table region is full

// staging record meta word (u32): op(8) | flags(8) | slot-within-super-bucket(<=10 bits) << 16
__host__ __device__ inline uint32_t smeta_op(uint32_t m) { return m & 0xFF; }
__host__ __device__ inline uint32_t smeta_flags(uint32_t m) { return (m >> 8) & 0xFF; }
__host__ __device__ inline uint32_t smeta_slot(uint32_t m) { return m >> 16; }

struct alignas(16) u64x2 {
  uint64_t x, y;
};

// AtomicValueState per slot: meta = tag | (has_current << 8); value payload separately.
__host__ __device__ inline uint32_t vmeta(uint32_t tag, uint32_t cur) { return (tag & 0xFF) | ((cur & 1) << 8); }

// Value records staged for k_apply_value are encoded by the partition (value_encode): the walk then needs no
// op decode and no tag canonicalisation.  meta = status byte of ops that do not return the current value
// (bits 0..7) | W 8 | C 9 | R 10 | D 11 | L 12 | new tag 13..15 | slot-in-super-bucket 16..23 | compare tag
// 24..26; operands = (canonical compare value, canonical new value).  Semantics: AtomicValueState.java
// get :77-83, set :114-118, compareAndSet :123-133, getAndSet :138-144, delete :146-157.
constexpr uint32_t kVrW = 1u << 8;   // unconditional write: set, getAndSet
constexpr uint32_t kVrC = 1u << 9;   // compareAndSet
constexpr uint32_t kVrR = 1u << 10;  // returns the current value: get, getAndSet
constexpr uint32_t kVrD = 1u << 11;  // delete
constexpr uint32_t kVrL = 1u << 12;  // listen / unlisten: events, not applied by k_apply_value (flagged)
__host__ __device__ inline uint32_t vrec_ntag(uint32_t m) { return (m >> 13) & 7u; }
__host__ __device__ inline uint32_t vrec_ctag(uint32_t m) { return (m >> 24) & 7u; }
__host__ __device__ inline void value_encode(uint32_t op, uint32_t flags, uint64_t a, uint64_t b, uint32_t& m, u64x2& xy) {
  const uint32_t ta = CC_FLAG_TAG_A(flags), tb = CC_FLAG_TAG_B(flags);
  const uint64_t pa = ta ? a : 0, pb = tb ? b : 0;  // canonical NULL payload
  uint32_t bits, ntag = 0, ctag = 0;
  uint64_t x = 0, y = 0;
  switch (op) {
    case CC_OP_VALUE_GET: bits = kVrR; break;
    case CC_OP_VALUE_SET: bits = kVrW; ntag = ta; y = pa; break;
    case CC_OP_VALUE_CAS: bits = kVrC | CC_STATUS(CC_ST_OK, CC_TAG_BOOL); ctag = ta; x = pa; ntag = tb; y = pb; break;
    case CC_OP_VALUE_GETANDSET: bits = kVrW | kVrR; ntag = ta; y = pa; break;
    case CC_OP_DELETE: bits = kVrD; break;
    case CC_OP_VALUE_LISTEN:
    case CC_OP_VALUE_UNLISTEN: bits = kVrL; break;
    default: bits = CC_STATUS(CC_ST_UNKNOWN_OP, CC_TAG_NULL);  // ResourceStateMachineExecutor.java:78
  }
  m = bits | (ntag << 13) | (ctag << 24);
  xy = u64x2{x, y};
}

__device__ inline uint32_t lane_id() { return __lane_id(); }
__device__ inline uint64_t lanemask_lt() {
  const uint32_t l = __lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}
__device__ inline uint64_t ballot(bool p) { return __ballot(p); }
// A slot in an append buffer for every active lane of the wave: one atomic per wave (an event buffer's counter is
// one address: per-lane atomics on it serialise), lanes in lane order.
__device__ inline uint32_t wave_append(uint32_t* ctr) {
  const uint64_t act = __ballot(1);
  const uint32_t leader = (uint32_t)__builtin_ctzll(act);
  uint32_t base = 0;
  if (__lane_id() == leader) base = atomicAdd(ctr, (uint32_t)__builtin_popcountll(act));
  base = (uint32_t)__shfl((int)base, (int)leader, 64);
  return base + (uint32_t)__builtin_popcountll(act & lanemask_lt());
}

// Workgroup barrier that orders LDS only.  __syncthreads() also drains every outstanding global load and
// store of the wave (s_waitcnt vmcnt(0)), which would kill the cross-chunk prefetches the streaming kernels
// rely on; none of the engine's kernels exchanges global-memory data between threads of a workgroup.
__device__ inline void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ---- optional in-kernel phase clocks (diagnostics build: -DCC_PHASE_TIMING, scripts/probes/phase_timing.py) --
// Thread 0 of every workgroup accumulates s_memrealtime ticks (100 MHz) between phase marks; the sums are added to
// a per-kernel __device__ array at the end and read back with cc_debug_phases.  Compiled out by default.
constexpr int kPhases = 8;
#ifdef CC_PHASE_TIMING
#define PH_DECL uint64_t ph_last_ = wall_clock64(); const uint64_t ph_t0_ = ph_last_; uint64_t ph_acc_[kPhases] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PH(k) do { if (threadIdx.x == 0) { const uint64_t n_ = wall_clock64(); ph_acc_[k] += n_ - ph_last_; ph_last_ = n_; } } while (0)
#define PH_FLUSH(buf) do { if (threadIdx.x == 0) for (int q_ = 0; q_ < kPhases; ++q_) atomicAdd(&(buf)[q_], (unsigned long long)ph_acc_[q_]); } while (0)
#else
#define PH_DECL
#define PH(k) do { } while (0)
#define PH_FLUSH(buf) do { } while (0)
#endif

// ---- ops registered per resource type (ResourceStateMachine.init + Copycat reflection configure) -----
__host__ __device__ inline bool op_registered(uint32_t type, uint32_t op) {
  if (op == CC_OP_DELETE) return type != CC_RES_NONE;
  switch (type) {
    case CC_RES_VALUE: return op >= 50 && op <= 55;
    case CC_RES_MAP: return op >= 60 && op <= 72;
    case CC_RES_LOCK: return op == 115 || op == 116;
    case CC_RES_ELECTION: return op >= 110 && op <= 112;
    case CC_RES_GROUP: return op >= 120 && op <= 123;
    case CC_RES_SET: return op >= 100 && op <= 105;
    case CC_RES_QUEUE: return op >= 90 && op <= 99;
    case CC_RES_MULTIMAP: return op == 75 || (op >= 78 && op <= 84);  // MultiMapState.java:37-207 (no 76 / 77)
  }
  return false;
}
// resources whose elements live in the map table (apply_map.hip): MapState and SetState
__host__ __device__ inline bool is_keyed(uint32_t type) {
  return type == CC_RES_MAP || type == CC_RES_SET || type == CC_RES_MULTIMAP;
}
// SetState ops as the MapState key ops they behave like (the result is rewritten by k_set_results):
// contains -> containsKey, add -> putIfAbsent(Boolean TRUE), remove -> remove; anything else -> 0 (unknown op)
__host__ __device__ inline uint32_t set_as_map_op(uint32_t op) {
  switch (op) {
    case CC_OP_SET_CONTAINS: return CC_OP_MAP_CONTAINSKEY;
    case CC_OP_SET_ADD: return CC_OP_MAP_PUTIFABSENT;
    case CC_OP_SET_REMOVE: return CC_OP_MAP_REMOVE;
    case CC_OP_SET_SIZE: return CC_OP_MAP_SIZE;
    case CC_OP_SET_ISEMPTY: return CC_OP_MAP_ISEMPTY;
    case CC_OP_SET_CLEAR: return CC_OP_MAP_CLEAR;
    case CC_OP_DELETE: return CC_OP_DELETE;
  }
  return 0;
}
// MultiMapState ops as MapState key ops (MultiMapState.java:37-207; results rewritten by k_keyed_results).  The
// state is the set of keys put (put registers the key's value map but never stores the value, :68-91), so a key
// is a map entry holding Boolean TRUE: containsKey -> containsKey; put -> putIfAbsent(TRUE), no TTL (the timer's
// callback throws before it changes anything, A18); get / size(key) / remove(key, value) change nothing ->
// containsKey; remove(key) -> remove; removeValue and clear drop every key (:140-165, every value map is
// empty) -> clear; anything else -> 0 (unknown op).
__host__ __device__ inline uint32_t mmap_as_map_op(uint32_t op, uint32_t tag_a) {
  switch (op) {
    case CC_OP_MMAP_CONTAINSKEY: return CC_OP_MAP_CONTAINSKEY;
    case CC_OP_MMAP_PUT: return CC_OP_MAP_PUTIFABSENT;
    case CC_OP_MMAP_GET: return CC_OP_MAP_CONTAINSKEY;
    case CC_OP_MMAP_SIZE: return CC_OP_MAP_CONTAINSKEY;
    case CC_OP_MMAP_REMOVE: return tag_a != CC_TAG_NULL ? CC_OP_MAP_CONTAINSKEY : CC_OP_MAP_REMOVE;
    case CC_OP_MMAP_REMOVEVALUE: return CC_OP_MAP_CLEAR;
    case CC_OP_MMAP_ISEMPTY: return CC_OP_MAP_ISEMPTY;
    case CC_OP_MMAP_CLEAR: return CC_OP_MAP_CLEAR;
    case CC_OP_DELETE: return CC_OP_DELETE;
  }
  return 0;
}
// ops this build applies on the GPU (others raise CC_ERR_UNSUPPORTED for the batch)
__host__ __device__ inline bool op_on_gpu(uint32_t type, uint32_t op) {
  if (type == CC_RES_VALUE) return op == CC_OP_DELETE || (op >= 50 && op <= 53);
  if (type == CC_RES_MAP) return op == 60 || (op >= 62 && op <= 69);  // key ops (whole-map ops: map_wide.hip)
  if (type == CC_RES_SET) return op >= 100 && op <= 102;
  if (type == CC_RES_MULTIMAP) return op == 75 || (op >= 78 && op <= 80) || op == 83;
  if (type == CC_RES_QUEUE) return op_registered(type, op);
  if (type == CC_RES_LOCK || type == CC_RES_ELECTION) return op_registered(type, op);
  if (type == CC_RES_GROUP) return op_registered(type, op);  // schedule rows are batch barriers (engine.hip)
  return false;
}

// Map key placement: (map slot, key tag, key) -> 64-bit hash; the top bits pick the table region (= map
// super-bucket), the low bits the first probe inside it.  Shared by the partition and the map apply kernel.
__host__ __device__ inline uint64_t map_hash(uint32_t res, uint32_t ktag, uint64_t key) {
  uint64_t h = key ^ ((uint64_t)res << 32) ^ ((uint64_t)ktag << 61) ^ 0x9E3779B97F4A7C15ull;
  h ^= h >> 30;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 27;
  h *= 0x94D049BB133111EBull;
  h ^= h >> 31;
  return h;
}
// map table entry word: slot(17) | ktag(2) << 17 | USED << 19 | PRESENT << 20 | vtag(3) << 21 | PENDING << 24 | DEAD << 25 |
// UNSEEN << 26
constexpr uint32_t kMwSlotMask = (1u << 17) - 1;
constexpr uint32_t kMwUsed = 1u << 19;
constexpr uint32_t kMwPresent = 1u << 20;
constexpr uint32_t kMwVtagMask = 7u << 21;
constexpr uint32_t kMwPending = 1u << 24;  // bound this round, key not yet visible (apply_map resolution)
constexpr uint32_t kMwDead = 1u << 25;     // entry of a deleted map: never matches, reclaimed by compaction
// an entry k_hot_bind inserted for a hot-key candidate that no commit has stored into yet: not a key the map ever
// held (left out of the bound-key counts and compaction drops that bound tree bins, map_wide.hip); cleared by a store
constexpr uint32_t kMwUnseen = 1u << 26;
constexpr uint32_t kMwIdentMask = kMwSlotMask | (3u << 17) | kMwUsed | kMwDead;
// coordination state blocks (apply_coord.hip): one per resource slot, fixed capacity
struct CoordHdr {
  uint32_t who;    // lock holder / election leader instance slot
  uint32_t flags;  // kCoHeld (held / has leader) | kCoCleaned
  uint64_t idx;    // holder / leader commit index
  uint32_t head;   // lock waiter ring head
  uint32_t n;      // waiters / listeners / members
  uint64_t pad;
};
struct CoordEnt {
  uint64_t x;     // lock waiter: timeout deadline (kNoDeadline: none); election listener / group member: instance id
  uint64_t idx;   // commit index
  uint32_t inst;  // instance slot
  uint32_t pad;
};
constexpr uint32_t kCoHeld = 1u, kCoCleaned = 2u;
// the resource was removed from ResourceManager.resources by a deleteResource whose delete() threw (a lock or
// election whose holder commit was already cleaned): its instances stay registered and every commit on them hits
// `resources.get(...) == null` -> NullPointerException (ResourceManager.java:62,71); close skips its handler
constexpr uint32_t kCoZombie = 4u;
constexpr uint64_t kNoDeadline = ~0ull;
// QueueState entry (CoordEnt.pad = value tag | kQCleaned): element() clean()ed the head it leaves in place
// (QueueState.java:111-124), so the log no longer retains that commit
constexpr uint32_t kQCleaned = 0x100u, kQTagMask = 0xFFu;
// a commit the state machine dropped without clean() (AtomicValueState.listen's listeners.put over an existing
// session :41-49, MembershipGroupState.close's members.remove :36-42): the log retains it for good.  Appended to
// the engine's leak log by the kernels, drained into the host's per-slot lists (cc_read_retained)
struct LeakRec {
  uint64_t idx;
  uint32_t slot, pad;
};
// entries per coordination block = cc_config.coord_cap (a power of two; 0 = the default CC_LOCK_QUEUE =
// CC_ELECTION_LISTENERS = CC_GROUP_MEMBERS = CC_VALUE_LISTENERS = CC_QUEUE_CAP = 64)
constexpr uint32_t kCoordCapDefault = 64;
constexpr uint32_t kCoordCapMax = 65536;
__host__ __device__ inline size_t coord_block(uint32_t cap) { return sizeof(CoordHdr) + (size_t)cap * sizeof(CoordEnt); }
// One staged record of the extended partition (map, set, multimap, coordination and value-event commits), one
// 48-byte record per staging position: a bucket's run is then one contiguous span per chunk (its cache lines are
// written whole while they sit in L2) instead of five column spans.  Value commits for k_apply_value keep the
// st_meta / st_ab columns.
struct XRec {
  u64x2 ab;       // operands (locks: the clock at which due timeouts fire, the timeout)
  uint64_t key;   // map key / group member / lock clock
  uint64_t idx;   // log index
  uint32_t meta;  // staging meta word (op | flags << 8 | slot low byte << 16 | kMetaTtl)
  uint32_t res;   // map commits: the map slot; others: the instance slot
  uint64_t pad;
};
static_assert(sizeof(XRec) == 48, "XRec is three 16-byte words");
// One staged map / set / multimap record (k_part_ext -> k_apply_map, k_hot_*, launch_map_size): 32 bytes.  The b
// operand is read only by replaceIfPresent (its compare value, MapState.java:207-228): from the batch's b column, by
// the record's row in its partition tile (rr >> 17), instead of 8 more bytes in every record.
// pfx[h] = scan pieces of the hot keys before h, for h <= nh (hot_len: each key's list length).  Wave 0 does it, 4 keys
// per lane with their loads in flight together, and a wave scan: one thread walking the keys waited for each load in
// turn (~256 dependent global round trips at the top of every workgroup of the hot / size kernels).  The caller
// synchronises the workgroup before reading pfx.
__device__ inline void hot_piece_prefix(const uint32_t* __restrict__ hot_len, uint32_t nh, uint32_t* pfx) {
  constexpr int PL = (kHotMax + kWave - 1) / kWave;
  if (threadIdx.x >= (uint32_t)kWave) return;
  const uint32_t l = threadIdx.x;
  uint32_t c[PL], sum = 0;
#pragma unroll
  for (int q = 0; q < PL; ++q) {
    const uint32_t h = l * PL + q;
    c[q] = h < nh ? (hot_len[h] + kHotPiece - 1) / kHotPiece : 0u;
    sum += c[q];
  }
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, kWave);
    if (l >= (uint32_t)d) inc += y;
  }
  uint32_t run = inc - sum;
#pragma unroll
  for (int q = 0; q < PL; ++q) {
    const uint32_t h = l * PL + q;
    if (h <= nh) pfx[h] = run;
    run += c[q];
  }
  if (l == kWave - 1 && nh == (uint32_t)(PL * kWave)) pfx[nh] = inc;
}

struct MRec {
  uint64_t a;     // value operand
  uint64_t key;
  uint64_t idx;   // log index
  uint32_t meta;  // op | flags << 8 | slot low byte << 16 | kMetaTtl
  uint32_t rr;    // map slot | row in the partition tile << 17
};
static_assert(sizeof(MRec) == 32, "MRec is two 16-byte words");
// one event of the per-sub-batch arena (apply_coord.hip -> events.hip)
struct EvRec {
  uint32_t g;       // staging position of the commit
  uint32_t target;  // instance slot
  uint64_t payload;
  uint16_t k;       // emission order within the commit
  uint8_t code, tag, src, pad[3];
};
constexpr uint32_t kErrTime = 8u;  // the time column decreased inside a batch
constexpr uint32_t kErrMapOrder = 16u;  // containsValue's HashMap iteration order is undetermined (map_wide.hip)
constexpr uint32_t kErrMapSize = 32u;   // a map's tracked size differs from its table at a barrier (internal check)
constexpr uint32_t kErrHandleHash = 64u;  // a HANDLE map key whose String.hashCode was never registered (cc_handle_hashes)
constexpr uint32_t kErrSmallFlag = 256u;
constexpr uint32_t kErrCoordFull = 512u;
constexpr uint32_t kErrSpan = 1024u;      // a sub-batch with map events spans 2^32 log indices (the host cuts them first)  // a coordination collection (lock queue, listeners, members, queue) is full  // (CC_DIAG builds) a map in the small-map window without its snapshot flag
constexpr uint32_t kErrCvKey = 128u;     // in-stream containsValue: an event past a 2^40-index span (internal check)

// java.util.HashMap placement of a map key: hash(key) = h ^ (h >>> 16), h = key.hashCode() -- Long (int)(v ^ v >>> 32),
// Integer v, Boolean 1231 / 1237, String (HANDLE) its registered String.hashCode (hh: sorted handles + hashes);
// ok = false for an unregistered HANDLE.  Key tags: 0 LONG, 1 INT, 2 BOOL, 3 HANDLE.
__device__ inline uint32_t java_key_hash(uint32_t ktag, uint64_t v, const uint64_t* __restrict__ hh_key,
                                         const int32_t* __restrict__ hh_val, uint32_t hh_n, bool& ok) {
  uint32_t h;
  ok = true;
  switch (ktag) {
    case 1: h = (uint32_t)v; break;
    case 2: h = v ? 1231u : 1237u; break;
    case 3: {
      uint32_t lo = 0, hi = hh_n;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (hh_key[mid] < v) lo = mid + 1; else hi = mid;
      }
      ok = lo < hh_n && hh_key[lo] == v;
      h = ok ? (uint32_t)hh_val[lo] : 0u;
      break;
    }
    default: h = (uint32_t)(v ^ (v >> 32)); break;
  }
  return h ^ (h >> 16);
}

// Keys compacted away from the map table (apply_map.hip: a region more than 3/4 bound re-inserts its present entries
// and drops the bound-but-absent ones), kept per (map, generation) in a device hash set with the log index at which
// the key's entry was first bound (its claim: tbl_claim).  A tree bin (capacity >= 128) needs 9 keys in one bin at
// once; the engine's test for "the deciding bin of an order-dependent containsValue may have been a tree bin" counts,
// per capacity level L, the distinct keys the map bound in that bin at level L's bin width before its table grew past
// L, since its last clear: the bound entries of the table plus this set's keys that are not bound now
// (map_wide.hip k_mw_order / k_mw_cset).  A clear / Delete bumps the map's generation (its old keys no longer count).
// meta: occupied << 31 | (generation & 0xFFF) << 19 | key tag << 17 | slot.
struct CsetEnt {
  uint64_t key;
  unsigned long long claim;  // the earliest claim of the key's entries that were compacted away
  uint32_t meta;
  uint32_t pad;
};
__device__ inline uint32_t cset_meta(uint32_t slot, uint32_t kt, uint64_t gen) {
  return 0x80000000u | ((uint32_t)(gen & 0xFFFu) << 19) | ((kt & 3u) << 17) | (slot & kMwSlotMask);
}
// (a key is inserted by the one workgroup compacting its region; a reader racing an insert of another key of the
// same map may miss a dedupe and add a duplicate: that only over-counts, toward refusing)
// An entry of a generation its map has left (a clear / Delete since: k_map_drop) is stale and taken over.
__device__ inline void cset_insert(CsetEnt* __restrict__ set, uint64_t mask, uint32_t* __restrict__ full, uint32_t slot,
                                   uint32_t kt, uint64_t key, const uint64_t* __restrict__ cgen, uint64_t claim) {
  const uint64_t gen = cgen[slot];
  const uint32_t meta = cset_meta(slot, kt, gen);
  uint64_t p = (map_hash(slot, kt, key) ^ (gen * 0x9E3779B97F4A7C15ull)) & mask;
  for (int step = 0; step < 128; ++step, p = (p + 1) & mask) {
    uint32_t m = __atomic_load_n(&set[p].meta, __ATOMIC_RELAXED);
    if (m != 0u && m != meta && ((m >> 19) & 0xFFFu) != (uint32_t)(cgen[m & kMwSlotMask] & 0xFFFu)) {
      const uint32_t was = atomicCAS(&set[p].meta, m, meta);  // a stale entry: reused
      if (was == m) {
        set[p].key = key;
        set[p].claim = claim;
        return;
      }
      m = was;
    }
    if (m == 0u) {
      m = atomicCAS(&set[p].meta, 0u, meta);
      if (m == 0u) {
        set[p].key = key;
        set[p].claim = claim;  // (one key is compacted by one workgroup at a time: no racing dedupe of it)
        return;
      }
    }
    if (m == meta && set[p].key == key) {
      atomicMin(&set[p].claim, (unsigned long long)claim);
      return;
    }
  }
  atomicOr(full, 1u);  // (the set is full: every later order-dependent test above capacity 64 refuses)
}
// A map's capacity-level timeline (cc_engine::d_lvl_at, kLvlSlots per map): the log index of the commit whose
// insertion grew its HashMap table to level L (capacity 16 << L), ~0 while not reached (0 for level 0).  A key counts
// toward level L's tree-bin test only if its entry was claimed before the table left level L (lvl_at[L + 1]).
constexpr uint32_t kLvlSlots = 32;
__device__ inline void lvl_reached(unsigned long long* __restrict__ lvl_at, uint32_t m, uint32_t from, uint32_t to,
                                   uint64_t idx) {
  for (uint32_t L = from + 1; L <= to && L < kLvlSlots; ++L) atomicMin(&lvl_at[(uint64_t)m * kLvlSlots + L], (unsigned long long)idx);
}
// The key's entry in the map table (an entry of its map and tag), or ~0 when it has none.  Probes its region from
// the key's first slot until an empty entry (map_hash: the top map_bits bits pick the region).
__device__ inline uint64_t tbl_find(const uint32_t* __restrict__ word, const uint64_t* __restrict__ tkey, uint32_t map_bits,
                                    uint32_t slot, uint32_t kt, uint64_t key) {
  const uint64_t h = map_hash(slot, kt, key);
  const uint64_t base = (h >> (64 - map_bits)) * (uint64_t)kMapRegion;
  const uint32_t ident = (slot & kMwSlotMask) | ((kt & 3u) << 17) | kMwUsed;  // (mw_ident)
  uint32_t p = (uint32_t)h & (kMapRegion - 1);
  for (int step = 0; step < kMapRegion; ++step, p = (p + 1) & (kMapRegion - 1)) {
    const uint32_t w = word[base + p];
    if (w == 0u) return ~0ull;
    if ((w & kMwIdentMask) == ident && tkey[base + p] == key) return base + p;
  }
  return ~0ull;
}

// A map's java.util.HashMap while its table is small (capacity <= 64; map_small.hip, small_jhm.h): the nodes of the
// live keys (their hashes, chain and red-black tree links, at most 49 at once), the bin heads, the capacity level
// (capacity = 16 << lvl) and the bins (mod 64) that became tree bins since the last clear.  Below capacity 64 a bin
// that reaches 9 keys resizes the table early (HashMap.treeifyBin); at 64 it becomes a red-black tree bin, followed
// node for node here; after the window (capacity 128) such a bin's order is no longer followed (tree_bins, sticky).
constexpr uint32_t kSmNodes = 64;
struct SmallMap {
  uint32_t n, lvl, flags, pad;  // (pad: the big model's slot while kSmBig; see kSmBigNew)
  uint64_t tree_bins;
  uint64_t used;            // node pool occupancy
  uint32_t jh[kSmNodes];    // node: the key's HashMap hash
  uint8_t nx[kSmNodes], pv[kSmNodes], pa[kSmNodes], lf[kSmNodes], rt[kSmNodes];  // links: node + 1 (0 = null)
  uint8_t nb[kSmNodes];     // bit 0 TreeNode, bit 1 red
  uint8_t tab[64];          // bin heads: node + 1 (0 = null)
  // (cold: read only when two live keys share a hash; k_small_replay keeps the part above in LDS, these in HBM)
  uint64_t key[kSmNodes];   // node: the key (tag in kt), for putTreeVal's compareTo / tieBreakOrder and removeNode
  uint8_t kt[kSmNodes];
};
constexpr uint32_t kSmHotBytes = (uint32_t)offsetof(SmallMap, key);
constexpr uint32_t kSmIn = 1u;       // the table is still small (capacity <= 64): followed node for node
constexpr uint32_t kSmTree = 2u;     // a bin became a tree bin since the last clear
constexpr uint32_t kSmUnknown = 4u;  // tracking stopped while small (kept for the snapshot format; never set now)
constexpr uint32_t kSmAmbig = 8u;    // a tree order the engine cannot know (two String keys with one hash in a tree bin;
                                     // a removal of a key the model does not hold): an order-dependent answer refuses
constexpr uint32_t kSmBig = 16u;     // the table left the window with a tree bin: followed node for node by a big model
                                     // (BigMap, big_jhm.h; SmallMap::pad is its slot)
constexpr uint32_t kSmBigNew = 32u;  // ... from this sub-batch's replay on: the small model's nodes are still here, and
                                     // SmallMap::pad is the position of the event that grew the table

// A map's java.util.HashMap after its table left the small window (capacity 128 and up) with a tree bin since its
// last clear (big_jhm.h, map_big.hip): every bin followed node for node, tree bins through HashMap.resize's
// TreeNode.split, so an order-dependent containsValue there is answered instead of refused.  An engine holds
// kBigSlots of them; a map that finds none free, or outgrows one (kBigNodes live keys, capacity 16 << kBigMaxLvl),
// falls back to the bounds of map_wide.hip k_mw_order (which refuse such an answer).
constexpr uint32_t kBigSlots = 16;
constexpr uint32_t kBigNodes = 4096;
constexpr uint32_t kBigMaxLvl = 9;  // capacity 8,192
constexpr uint32_t kBigTab = 16u << kBigMaxLvl;
struct BigNode {
  uint64_t key;
  uint32_t jh;                  // the key's HashMap hash
  uint16_t nx, pv, pa, lf, rt;  // links: node + 1 (0 = null)
  uint8_t nb, kt;               // bit 0 TreeNode, bit 1 red; the key's tag
};
struct BigHdr {
  uint32_t owner;  // map slot + 1 (0: free)
  uint32_t n, lvl, flags;
  uint32_t top;    // nodes [1, top] handed out so far
  uint32_t free;   // released nodes, linked through nx
  unsigned long long resume;  // kBigResume: the position of the event at which the map left the window
};
struct BigMap {
  BigHdr h;
  uint16_t tab[kBigTab];  // bin heads: node + 1
  BigNode nd[kBigNodes];
};
constexpr uint32_t kBigResume = 0x100u;  // BigHdr::flags: converted from the small model this sub-batch, before its
                                         // resize to 128; events up to `resume` were applied by the small replay
// per-map flags of the batch (cc_engine::d_msmall), written on the engine stream only: bit 0 the table is small (events
// followed key by key; a SNAPSHOT of the small-map models' kSmIn, see below), bit 1 the
// batch asks the map's size / isEmpty (events followed for the in-stream answers); either makes every insertion /
// removal of the map an event (region commits: k_msize_count; hot-key commits: k_hot_apply)
constexpr uint8_t kMfSmall = 1u, kMfSize = 2u;
// bit 2: the batch answers containsValue rows of the map in the stream (map_cv.hip): its commits report value changes
constexpr uint8_t kMfCv = 4u;
// bit 3: the sub-batch clears the map in the stream (map_clear.hip): its sizes come from event replay and its commits
// carry their clear epoch (region and hot-key commits alike)
constexpr uint8_t kMfClr = 8u;
// The small-map window invariant (race-free by construction, engine_state.h SmSet): a map's kSmIn (its model, written
// by k_small_replay) and its kMfSmall snapshot only go 1 -> 0 inside a batch (a table only grows past 64; they go to
// 1 only at resource creation / snapshot restore, between batches, with no replay pending).  The replay, which may
// run on the side stream beside the next sub-batch, never writes d_msmall: it marks a map that left the window in its
// own buffer (cc_engine::d_msm_left, one per event-buffer set), and k_small_fold clears kMfSmall from those marks on
// the engine stream once that stream has waited for the replay.  So no kernel of a sub-batch reads a byte another
// stream writes meanwhile; the snapshot may lag the models by one sub-batch (a map that left still emits its events
// for one more sub-batch, and the replay skips them: its model says it left).  Engine-stream kernels read the
// snapshot, never a model's kSmIn, while a replay may be pending (k_small_chains, ChainKeep).
// the flag bytes are set by concurrent threads of one kernel: OR through the aligned word (the array is padded to it)
__device__ inline void mflag_or(uint8_t* mflag, uint32_t m, uint8_t bit) {
  atomicOr(reinterpret_cast<uint32_t*>(mflag + (m & ~3u)), (uint32_t)bit << (8 * (m & 3u)));
}
__device__ inline void mflag_and(uint8_t* mflag, uint32_t m, uint8_t keep) {
  atomicAnd(reinterpret_cast<uint32_t*>(mflag + (m & ~3u)), ~((uint32_t)(uint8_t)~keep << (8 * (m & 3u))));
}
// a map commit's size change for the exact size tracking (map_wide.hip launch_map_size): slot << 2 | 1 insert, 2 remove
__device__ inline uint32_t msz_word(uint32_t slot, bool was, bool now) {
  return (slot << 2) | (now && !was ? 1u : !now && was ? 2u : 0u);
}

// a map record's operands: (a, b), b gathered from the batch's b column for the one op that reads it (see MRec)
__device__ inline u64x2 mrec_ab(const MRec& r, const uint64_t* __restrict__ cb, uint64_t lo, uint32_t g) {
  const uint32_t fl = smeta_flags(r.meta);
  const bool needs_b = smeta_op(r.meta) == CC_OP_MAP_REPLACEIFPRESENT && CC_FLAG_TAG_B(fl) != CC_TAG_NULL;
  return u64x2{r.a, needs_b ? cb[lo + (uint64_t)(g / kTile) * kTile + (r.rr >> 17)] : 0ull};
}

// log2(HashMap capacity / 16) after the size peaked at p (resize doubles the table when ++size > 0.75 capacity)
__host__ __device__ inline uint32_t cap_level(uint64_t p) {  // the least lv with p <= 12 << lv (closed form)
  const uint64_t q = (p + 11) / 12;                          // ceil(p / 12): lv = ceil(log2(q))
  return q <= 1 ? 0u : (uint32_t)(64 - __builtin_clzll(q - 1));
}

// ---- TTL mode: map timers as size events (map_small.hip) -------------------------------------------------------
// In TTL mode a map's size also drops when a timer fires (MapState.java:91-93: the scheduled map.remove(key)), with no
// commit.  Every expiry becomes an event at the boundary where the reference fires it: the first row of the batch
// whose clock max(clock_before, time[r]) reaches the deadline, before that row (module mode) or after it (manager
// mode, deferred: boundary r + 1).  Events are keyed map << 36 | position << 4 | code, position 2 * (row
// - lo) + 1 for a commit of row `row`, 2 * (b - lo) for boundary b (before row b), code 1 insert / 2 remove, so a
// radix sort puts each map's commits and expiries in log order.  A sub-batch [lo, hi) owns the boundaries [bl, bh]:
// bh = hi, bl = lo at the batch start and after a barrier row, lo + 1 after another sub-batch (which owned lo).
// A map event's payload (map_small.hip), by emission slot: the sorted events carry the slot as their value.
// aux = the key's HashMap hash for an insertion / removal, the batch row for a size / isEmpty query.
constexpr uint32_t kEvPosBits = 32;                      // a map event's position field (a sub-batch's span)
constexpr uint32_t kEvMapShift = 4 + kEvPosBits;          // its map slot above it (the sort's key bits end there)
constexpr uint64_t kEvPosMask = (1ull << kEvPosBits) - 1;
struct EvPay {
  uint64_t key;   // the key (its tag in ktag): a small map's model tells keys with one hash apart by them
  uint32_t aux;
  uint32_t ktag;  // the key's tag (bits 0-1); at an alternating run's first removal, the events it implies << kSkipShift
};
constexpr uint32_t kSkipShift = 4;  // (map_small.hip k_small_chains)
struct TtlEmit {
  const uint64_t* time;   // the batch's time column (null: the clock is clock_before throughout)
  uint64_t n;             // rows in the batch
  uint64_t lo, bl, bh;
  uint64_t adv;           // cc_advance_time: every timer due in (clock_before, adv] fires, at position 0 (0: a batch)
  uint32_t deferred;
  const uint64_t* hh_key;  // String.hashCode of HANDLE keys (java_key_hash)
  const int32_t* hh_val;
  uint32_t hh_n;
  uint64_t* ev_key;        // the event buffer shared with launch_map_size's emission (SmallArgs::ev_key / ev_val)
  uint32_t* ev_val;
  EvPay* ev_pay;
  uint32_t ev_cap;
  uint32_t* ctl;           // ctl[0]: events appended
};

// One expiry of entry (word w, key) whose timer has deadline d, if the sub-batch owns its firing boundary.
__device__ inline void ttl_expiry_event(const TtlEmit& t, uint64_t cb, uint32_t w, uint64_t key, uint64_t d,
                                        uint32_t& err) {
  if (d <= cb) return;  // fired by the end of an earlier batch (or cc_advance_time)
  uint64_t pos = 0;
  if (t.adv) {
    if (d > t.adv) return;
  } else {
    uint64_t a = 0, b = t.n;  // the first row whose clock reaches d
    while (a < b) {
      const uint64_t mid = a + (b - a) / 2;
      const uint64_t c = t.time ? (t.time[mid] > cb ? t.time[mid] : cb) : cb;
      if (c >= d) b = mid;
      else a = mid + 1;
    }
    if (a >= t.n) return;  // not due in this batch
    const uint64_t bd = t.deferred ? a + 1 : a;
    if (bd < t.bl || bd > t.bh) return;
    pos = bd > t.lo ? 2 * (bd - t.lo) : 0;  // (a boundary before the sub-batch's first row: before all of it)
  }
  bool ok;
  const uint32_t jh = java_key_hash((w >> 17) & 3, key, t.hh_key, t.hh_val, t.hh_n, ok);
  if (!ok) err |= kErrHandleHash;
  const uint32_t at = wave_append(t.ctl);
  if (at < t.ev_cap) {
    t.ev_key[at] = ((uint64_t)(w & kMwSlotMask) << kEvMapShift) | ((pos & kEvPosMask) << 4) | 2u;
    t.ev_val[at] = at;
    t.ev_pay[at] = EvPay{key, jh, (w >> 17) & 3u};
  }
}

// extended staging (partition.hip) options
constexpr uint32_t kExtValue = 1u;     // value records carry the extended columns (value events on the GPU)
constexpr uint32_t kExtDeferred = 2u;  // manager-mode timer order
constexpr uint32_t kExtTimeCheck = 4u; // the partition checks time[i] >= time[i-1] for its rows (kErrTime)
// staging meta: op | flags << 8 | slot low byte << 16 | (map records) ttl > 0 << 24
constexpr uint32_t kMetaTtl = 1u << 24;
__host__ __device__ inline uint32_t mw_ident(uint32_t res, uint32_t ktag) { return (res & kMwSlotMask) | ((ktag & 3) << 17) | kMwUsed; }
__host__ __device__ inline uint32_t mw_vtag(uint32_t w) { return (w >> 21) & 7; }


// ---- containsValue in the stream (map_cv.hip) -------------------------------------------------------------------
// A sub-batch's in-stream containsValue operands (map slot, value tag, canonical value) live in a device hash set
// keyed by a 64-bit key: exact (bit 63 set) when the value fits 43 signed bits, else a fingerprint whose entries are
// verified against the stored operand (two operands that share a fingerprint get a position each: map_cv.hip k_cv_fix).
struct CvEnt {
  unsigned long long k64;  // 0: empty
  uint64_t v;
  uint32_t meta;           // slot | tag << 17
  uint32_t pad;
};
__host__ __device__ inline uint64_t cv_key(uint32_t m, uint32_t tag, uint64_t v, bool& exact) {
  const int64_t sv = (int64_t)v;
  exact = ((int64_t)((uint64_t)sv << 21) >> 21) == sv;
  if (exact) return (1ull << 63) | ((uint64_t)(tag & 7u) << 60) | ((uint64_t)(m & kMwSlotMask) << 43) | (v & ((1ull << 43) - 1));
  uint64_t h = (v ^ ((uint64_t)(m & kMwSlotMask) << 3 | (tag & 7u)) * 0xC2B2AE3D27D4EB4Full) * 0x9E3779B97F4A7C15ull;
  h ^= h >> 31;
  h = (h * 0xBF58476D1CE4E5B9ull) & ~(1ull << 63);
  return h ? h : 1ull;
}
__host__ __device__ inline uint32_t cv_slot0(uint64_t k64, uint32_t mask) {
  uint64_t h = k64 * 0x9E3779B97F4A7C15ull;
  return (uint32_t)(h >> 32) & mask;
}
// The operand's set position, or ~0 when the sub-batch asks no containsValue of it.  A hashed fingerprint (an operand
// past 43 bits) may be shared by two operands: the set then holds each at its own position, the second one further
// along the probe sequence (map_cv.hip k_cv_fix), so a position counts only when the operand itself matches.
__device__ inline uint32_t cv_find(const CvEnt* __restrict__ set, uint32_t mask, uint32_t m, uint32_t tag, uint64_t v) {
  bool exact;
  const uint64_t k = cv_key(m, tag, v, exact);
  uint32_t p = cv_slot0(k, mask);
  for (uint32_t step = 0; step <= mask; ++step, p = (p + 1) & mask) {
    const uint64_t c = set[p].k64;
    if (c == 0) return ~0u;
    if (c == k && (exact || (set[p].v == v && set[p].meta == ((m & kMwSlotMask) | (tag << 17))))) return p;
  }
  return ~0u;
}
// The containsValue context of a map apply kernel: the maps answered in the stream (mflag & kMfCv), their operand
// set, and the event buffer (key = operand << 42 | (log index - the sub-batch's first) << 2 | kind: 0 a matching
// value left an entry, 1 one entered it, 2 a query; value = the query's row - lo).  set == nullptr: off.
struct CvCtx {
  const uint8_t* mflag;
  const CvEnt* set;
  uint32_t mask;
  const uint32_t* bloom;  // a bit per operand key (cv_bloom_bit): a commit's value that is no operand skips the set
  uint32_t bbits;         // log2 of the filter's bits
  uint64_t* ev_key;
  uint32_t* ev_val;
  uint32_t cap;
  uint32_t* ctl;  // ctl[0]: events appended
  const uint64_t* idx0p;
};
__device__ inline void cv_event(const CvCtx& cv, uint32_t q, uint64_t d, uint32_t kind, uint32_t val, uint32_t& err) {
  if (d >> 40) err |= kErrCvKey;
  const uint32_t at = wave_append(cv.ctl);
  if (at < cv.cap) {
    cv.ev_key[at] = ((uint64_t)q << 42) | ((d & ((1ull << 40) - 1)) << 2) | kind;
    cv.ev_val[at] = val;
  } else {
    err |= kErrCapacity;
  }
}
__host__ __device__ inline uint32_t cv_bloom_bit(uint64_t k64, uint32_t bbits) {
  return (uint32_t)((k64 * 0xD6E8FEB86659FD93ull) >> (64 - bbits));
}
// cv_find behind the filter (one L2-resident bit instead of a probe of the 24-byte-entry set: nearly every stored
// value is no operand)
__device__ inline uint32_t cv_lookup(const CvCtx& cv, uint32_t m, uint32_t tag, uint64_t v) {
  bool exact;
  const uint64_t k = cv_key(m, tag, v, exact);
  const uint32_t b = cv_bloom_bit(k, cv.bbits);
  if (!((cv.bloom[b >> 5] >> (b & 31)) & 1u)) return ~0u;
  return cv_find(cv.set, cv.mask, m, tag, v);
}
// One commit's change of an entry (word / value before and after) in a map answered in the stream: the operand
// count events of the values that left and entered it.  idx(): the commit's log index (read only on an event).
template <class IdxF>
__device__ inline void cv_change(const CvCtx& cv, uint32_t w0, uint64_t v0, uint32_t w1, uint64_t v1, IdxF idx,
                                 uint32_t ep, uint32_t& err) {
  if (!cv.set) return;
  const uint32_t m = w1 & kMwSlotMask;
  if (!(cv.mflag[m] & kMfCv)) return;
  const bool p0 = (w0 & kMwPresent) != 0, p1 = (w1 & kMwPresent) != 0;
  const uint32_t t0 = mw_vtag(w0), t1 = mw_vtag(w1);
  if (p0 == p1 && (!p0 || (t0 == t1 && v0 == v1))) return;
  const uint32_t q0 = p0 ? cv_lookup(cv, m, t0, t0 ? v0 : 0) : ~0u;
  const uint32_t q1 = p1 ? cv_lookup(cv, m, t1, t1 ? v1 : 0) : ~0u;
  if (q0 == ~0u && q1 == ~0u) return;
  const uint64_t d = idx() - *cv.idx0p;
  if (q0 != ~0u) cv_event(cv, q0, d, 0u, ep, err);  // (value: the commit's clear epoch, map_clear.hip)
  if (q1 != ~0u) cv_event(cv, q1, d, 1u, ep, err);
}


// ---- clear in the stream (map_clear.hip) ------------------------------------------------------------------------
// A batch's in-stream clears as (map slot << 32 | row) sorted, with per-map offsets; per sub-batch, for every map the
// clears before the sub-batch (base) and within it (eend, < 128).  A commit's epoch = the clears of its map in
// [lo, row): a commit whose epoch differs from the one its entry was last at sees the entry absent first.
struct ClrCtx {
  const uint8_t* mflag;     // null: no clears in this sub-batch
  const uint64_t* clr;      // [n] (slot << 32 | row), ascending
  const uint32_t* off;      // [R + 1]
  const uint32_t* base;     // [R] clears of the map before this sub-batch (positions in clr from off[m])
  const uint8_t* eend;      // [R] clears of the map in this sub-batch
  uint64_t lo;              // the sub-batch's first row
  uint8_t* tbl_ep;          // [map_entries] a hot key's entry's epoch after k_hot_apply (k_apply_map resets it to 0)
  const uint8_t* btab;      // [R][nb] a cleared map's epoch at each row bucket's start (map_clear.hip k_clr_btab)
  uint32_t nb, bshift;      // buckets per map, log2 of the rows per bucket
};
constexpr uint32_t kMetaEpochShift = 25;  // MRec meta bits 25-31 (in LDS, k_apply_map): the commit's clear epoch
// the bucket's epoch (bit 7: a clear of the map falls inside the bucket), then only in such a bucket the map's few
// clears before the row: one load for most commits (0 for a map not cleared in the sub-batch); a binary search over
// the map's clears was ~10 dependent loads per commit of a cleared map
__device__ inline uint32_t clr_epoch(const ClrCtx& c, uint32_t m, uint64_t row) {
  uint32_t e = c.btab[(uint64_t)m * c.nb + (uint32_t)((row - c.lo) >> c.bshift)];
  if (!(e & 0x80u)) return e;
  e &= 0x7Fu;
  const uint32_t end = c.eend[m];
  if (e < end) {
    const uint64_t* p = c.clr + c.off[m] + c.base[m];  // the map's clears in this sub-batch, ascending
    while (e < end && (uint32_t)p[e] < (uint32_t)row) ++e;
  }
  return e;
}
}  // namespace cc
