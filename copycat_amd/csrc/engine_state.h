// engine_state.h — the engine handle (struct cc_engine) shared by the host-side translation units of
// libcopycat_apply.so: engine.hip (lifecycle, registry, batched apply driver, readback, snapshots) and
// manager.hip (the ResourceManager control plane, ResourceManager.java:77-264).  Host code only.
#pragma once
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "common.h"
#include "engine_internal.h"
#include "java_hashmap.h"

namespace cc {
// error reporting (cc_last_error) and the stream drain every registry update starts with
int set_err(int code, const char* what, hipError_t e = hipSuccess);
int quiesce(cc_engine* e);      // drains the streams, then applies the queued registry writes (dev_flush)
int sync_streams(cc_engine* e);  // drains the streams only (control-plane updates that queue their device writes)
int dev_flush(cc_engine* e);
// registry primitives (engine.hip): resource slots [first, first+count) of `type`; instance slots first+k ->
// resource res_first + k*res_stride, instance id id_first+k, owned by `client`; a successful deleteResource
int create_range(cc_engine* e, uint32_t first, uint32_t count, uint32_t type);
int open_range(cc_engine* e, uint32_t first, uint32_t count, uint32_t res_first, uint32_t res_stride, uint64_t id_first,
               uint64_t client);
int delete_slot(cc_engine* e, uint32_t slot);
int drain_leaks(cc_engine* e);  // the device leak log -> cc_engine::leaks
// a device checkpoint of the state a batch apply writes (engine.hip; synchronous): saved before an attempt of the
// prefix apply, restored when the attempt failed on a fixed capacity
int ckpt_save(cc_engine* e);
int ckpt_restore(cc_engine* e);

// Occupancy bitmap of a slot space with lowest-free / highest-free search (control-plane allocation: rare, so a
// word scan from a hint is enough).
struct SlotBits {
  std::vector<uint64_t> w;
  uint64_t n = 0, lo = 0;  // lo: no free slot below it
  void reset(uint64_t count) {
    n = count;
    w.assign((count + 63) / 64, 0);
    lo = 0;
  }
  bool test(uint64_t s) const { return (w[s >> 6] >> (s & 63)) & 1; }
  void set(uint64_t s) { w[s >> 6] |= 1ull << (s & 63); }
  void clear(uint64_t s) {
    w[s >> 6] &= ~(1ull << (s & 63));
    if (s < lo) lo = s;
  }
  int64_t lowest() {  // lowest free slot, -1 if none
    for (uint64_t i = lo >> 6; i < w.size(); ++i)
      if (~w[i]) {
        const uint64_t s = i * 64 + (uint64_t)__builtin_ctzll(~w[i]);
        lo = i * 64;
        return s < n ? (int64_t)s : -1;
      }
    lo = n;
    return -1;
  }
  int64_t highest() {  // highest free slot, -1 if none
    for (uint64_t i = w.size(); i-- > 0;) {
      uint64_t f = ~w[i];
      if (i == w.size() - 1 && (n & 63)) f &= (1ull << (n & 63)) - 1;
      if (f) return (int64_t)(i * 64 + 63 - (uint64_t)__builtin_clzll(f));
    }
    return -1;
  }
};
}  // namespace cc

#define HIPCHECK(x)                                                \
  do {                                                             \
    hipError_t _e = (x);                                           \
    if (_e != hipSuccess) return cc::set_err(CC_ERR_HIP, #x, _e);  \
  } while (0)

using namespace cc;  // internal header: the engine's host translation units all work in namespace cc

struct cc_engine {
  uint32_t coord_cap = 64;  // entries per coordination block (cc_config.coord_cap, a power of two)
  cc_config cfg{};
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t last_stream = nullptr;
  uint32_t sb = 0, sb_bits = 0;  // value super-buckets of 256 slots
  uint32_t map_bits = 0;         // 2^map_bits map table regions follow them (0: no maps)
  uint64_t map_entries = 0;
  // buckets of the partition: value super-buckets, map regions + hot keys, then (coordination on, when the partition's
  // LDS allows) one bucket per quarter super-bucket (64 slots) for every super-bucket run by k_apply_coord
  bool quarter = false;
  uint32_t sbq_base() const { return sb + (map_bits ? (1u << map_bits) + kHotMax : 0u); }
  uint32_t sb_total() const { return sbq_base() + (quarter ? 4 * sb : 0u); }
  uint64_t sub_batch = 0, sub_ext = 0, max_tiles = 0;  // sub_ext: the sub-batch once the engine is ext (<= 16 Mi)
  // host mirrors of the registry
  std::vector<uint8_t> res_type;     // [sb*256]
  std::vector<uint32_t> inst_res;    // [max_inst]
  std::vector<uint64_t> inst_id, inst_client;
  // ResourceManager.sessions (ResourceManager.java:37, a java.util.HashMap<Long, SessionHolder> keyed by instance
  // id): its iteration order orders the close / expire fan-out (ResourceManager.java:237-264; java_hashmap.h)
  cc::JavaLongHashMap sessions;
  // String.hashCode of HANDLE keys (host-interned Strings): java.util.HashMap's bins of MapState (containsValue
  // order, MapState.java:49-60).  Host map + a sorted device copy (handle, hash) for the map kernels.
  std::map<uint64_t, int32_t> hh;
  uint64_t* d_hh_key = nullptr;
  int32_t* d_hh_val = nullptr;
  uint32_t hh_n = 0, hh_cap = 0;
  // ResourceManager control plane (manager.hip; ResourceManager.java:37-39,269-295).  Resource ids and instance ids
  // are commit indices (:86-88,103,185); slots are the engine's dense handles for them.
  std::unordered_map<uint64_t, uint64_t> keys;       // ResourceManager.keys: host-interned key -> resource id
  std::unordered_map<uint64_t, uint32_t> res_by_id;  // ResourceManager.resources: resource id -> slot
  std::unordered_map<uint64_t, uint32_t> inst_by_id; // ResourceManager.sessions: instance id -> instance slot
  std::map<std::pair<uint32_t, uint64_t>, uint64_t> res_sessions;  // ResourceHolder.sessions: (slot, client) -> instance id
  std::vector<uint64_t> res_id, res_key;  // [slots] resource id; key (when res_has_key)
  std::vector<uint8_t> res_has_key;       // [slots] created through get/create (low-level slots have no key)
  std::vector<uint8_t> res_zombie;        // [slots] removed from `resources` by a deleteResource whose delete() threw
  cc::SlotBits used_res, used_inst;       // slot occupancy (allocation: values/maps low, coordination high; instances low)
  std::set<uint32_t> open_grp[16];        // per coordination type: 64-slot groups holding only that type, with room
  // Control-plane registry writes queued for the next device work (engine.hip dev_flush): a run of creates / opens
  // coalesces into one copy or fill per array instead of ~10 blocking copies per call.  Mirrored arrays (res_type,
  // sb_kind, inst_res + inst_id) upload their dirty host range; the others queue fills / copies per array, in order.
  struct DevWrite {
    uint8_t* dst;
    uint64_t bytes;
    int fill;                   // byte value, or -1: copy `data`
    std::vector<uint8_t> data;
  };
  std::map<const void*, std::vector<DevWrite>> dev_pend;
  uint64_t res_dirty_lo = ~0ull, res_dirty_hi = 0, inst_dirty_lo = ~0ull, inst_dirty_hi = 0;
  bool sb_kind_dirty = false;
  bool dev_dirty() const {
    return !dev_pend.empty() || !big_rel.empty() || res_dirty_hi || inst_dirty_hi || sb_kind_dirty;
  }
  // device registry + state
  uint32_t* d_inst_res = nullptr;
  uint8_t* d_res_type = nullptr;
  uint32_t* d_val_meta = nullptr;
  uint64_t* d_val_v = nullptr;
  uint64_t* d_val_live = nullptr;             // [slots] retained value commit index (CC_CFG_VALUE_RETAINED)
  unsigned long long* d_val_wrow = nullptr;   // [slots] last writer row + 1 of the current batch
  // workspace
  uint32_t* d_st_meta = nullptr;
  u64x2* d_st_ab = nullptr;
  uint16_t* d_cpos = nullptr;
  uint16_t* d_ttab = nullptr;
  uint8_t* d_rst_status = nullptr;
  uint64_t* d_rst_value = nullptr;
  uint32_t* d_err = nullptr;
  // pinned host words for the per-batch / per-sub-batch counter readbacks: a copy into pageable memory returns only
  // after its own round trip, so two counters read back cost two idle gaps of ~200 us on the GPU
  uint64_t* h_pin = nullptr;
  // map table (apply_map.hip) + map staging columns
  uint64_t* d_tbl_key = nullptr;
  uint32_t* d_tbl_word = nullptr;
  uint64_t* d_tbl_val = nullptr;
  uint64_t* d_tbl_ci = nullptr;
  uint64_t* d_tbl_ins = nullptr;
  XRec* d_xrec = nullptr;  // [sub_batch] extended staging records (partition_ext.hip)
  MRec* d_mrec = nullptr;  // [sub_batch] map / set / multimap records (same staging positions; maps only)
  // hot map keys (apply_map_hot.hip)
  HotKey* d_hot = nullptr;
  uint32_t* d_hot_n = nullptr;
  HotKey* d_hot_cand = nullptr;      // [kHotMax] the batch's hot keys (counted once per batch)
  uint32_t* d_hot_meta = nullptr;    // [sub_batch] hot-bucket records' meta words (k_part_ext -> k_hot_agg)
  uint32_t* d_hot_cand_n = nullptr;
  // whole-map ops (map_wide.hip): barrier rows of the current batch, per-map peak-size bounds, scratch
  uint32_t* d_bar = nullptr;       // [kBarCap]
  BarRow* d_bar_rows = nullptr;    // [bar_rows_cap] the batch's barrier rows' columns (k_bar_fields)
  uint32_t bar_rows_cap = 0;
  std::vector<BarRow> bar_rows;    // host copy, in row order (= bars)
  uint64_t* d_fb = nullptr;        // [3 * fb_cap] group-timer fire-bound search: deadlines, search starts, results
  uint32_t fb_cap = 0;
  uint32_t* d_bar_n = nullptr;
  uint32_t* d_mw_peak = nullptr;   // [max_resources]
  uint64_t* d_mw_drop = nullptr;   // [max_resources]
  uint64_t* d_mw_cgen = nullptr;   // [max_resources] the map's generation: bumped by clear / Delete (compacted-key set)
  CsetEnt* d_cset = nullptr;       // keys compacted away from the table, per (map, generation) (common.h CsetEnt)
  uint64_t cset_mask = 0;          // set entries - 1
  uint32_t* d_cset_full = nullptr; // the set overflowed
  uint64_t* d_tbl_claim = nullptr; // [map_entries] log index at which each entry was first bound
  unsigned long long* d_lvl_at = nullptr;
  uint64_t* d_half_count = nullptr;
  EvPay* d_sm_pay = nullptr;       // [sm_cap] map event payloads by emission slot (map_small.hip)  // a batch applied as two calls (kBarCap): the second call's event count  // [max_resources * kLvlSlots] capacity-level timeline (common.h)
  // exact map sizes / HashMap capacities (map_wide.hip launch_map_size; not in TTL mode)
  uint32_t* d_rst_msz = nullptr;   // [sub_batch + 4 kPT] each region map commit's map and size change, staging order
  uint32_t* d_hot_msz = nullptr;   // hot-key commits' size changes (HotArgs::hot_msz)
  uint32_t* d_msize = nullptr;     // [max_resources]
  uint32_t* d_mpcap = nullptr;     // [max_resources]
  uint32_t* d_msz_tcnt = nullptr;  // [max_tiles][max_resources]
  uint4* d_msz_list = nullptr;     // [kMszListCap]
  uint32_t* d_msz_list_n = nullptr;
  // maps whose HashMap table is still small (capacity <= 64): early resizes and tree bins (map_small.hip)
  SmallMap* d_msm = nullptr;       // [max_resources]
  BigMap* d_mbig = nullptr;        // [kBigSlots] maps that left the window with a tree bin (map_big.hip)
  std::vector<std::pair<uint32_t, uint32_t>> big_rel;  // resource slots created since the last flush: their big
                                                       // models are freed there (dev_flush, launch_big_release)
  uint8_t* d_msmall = nullptr;     // [max_resources] 1: in the window
  uint8_t* d_msm_left = nullptr;   // [3][max_resources] maps a replay saw leave the window: sets 0 / 1 (side-stream
                                   // replays), 2 (engine-stream replays); folded into d_msmall on the engine stream
  uint32_t* d_sm_ctl = nullptr;    // [4] events of the sub-batch, maps still in the window
  uint64_t *d_sm_key = nullptr, *d_sm_key2 = nullptr;  // [sm_cap] map events (small / size-queried maps; TTL mode: all)
  uint32_t *d_sm_val = nullptr, *d_sm_val2 = nullptr;
  uint32_t* d_sm_seg = nullptr;    // [max_resources + 1] run starts + count
  uint32_t* d_cvbloom = nullptr;  // the in-stream containsValue operands' filter (common.h CvCtx)
  uint32_t* d_sm_cseg = nullptr;  // the replayed events without implied chain events: runs, counts (map_small.hip)
  // Outside TTL mode the small-map replay of sub-batch i runs on a side stream while sub-batch i + 1 runs on the
  // engine's: the event buffers alternate between two sets (swapped at each sub-batch start), a set is reused only
  // after its replay finished (ev_rep), and the engine stream waits for the side stream before barrier rows, timers
  // and the batch's end (join_replay).  Race-free by construction (common.h, the small-map window invariant): the
  // replay writes only its models (d_msm, read by no engine-stream kernel while it may run), its set's exit marks
  // (d_msm_left) and, atomically, the capacity levels (mpcap, lvl_at: atomic max / min on both streams, and the one
  // engine-stream reader of mpcap inside a sub-batch, k_msize_scan, loads it atomically); every wait for a replay
  // (wait_replay) is followed on the engine stream by the fold of its marks into the d_msmall snapshot.
  struct SmSet {
    uint64_t *key = nullptr, *key2 = nullptr;
    uint32_t *val = nullptr, *val2 = nullptr;
    EvPay* pay = nullptr;
    uint32_t* cseg = nullptr;
  } sm_alt;
  bool sm_alt_on = false;
  hipStream_t side_st = nullptr;
  hipEvent_t ev_prep = nullptr, ev_rep[2] = {nullptr, nullptr};
  hipEvent_t ev_rb = nullptr;  // after the per-sub-batch counter readback (the unpermute runs while the host waits)
  bool rep_pending[2] = {false, false};
  int sm_cur = 0;
  // a sub-batch's replay waits to be launched until the next sub-batch's partition is running: the partition's
  // equal-sized tiles run in lockstep rounds over every CU, and a CU held by the replay cost them a round
  SmallArgs pend_sa{};
  bool pend = false;
  int pend_set = 0;
  void* d_sm_temp = nullptr;
  size_t sm_temp_bytes = 0;
  void* d_clr_scan = nullptr;  // the cleared maps' size scan (map_clear.hip), one element per map event
  void* d_clr_stemp = nullptr;
  size_t clr_scan_cap = 0, clr_stemp_bytes = 0;
  uint8_t* d_clr_btab = nullptr;  // [R][nb] clear epochs per row bucket (common.h ClrCtx)
  size_t clr_btab_bytes = 0;
  uint64_t sm_cap = 0;             // events the buffers hold (engine.hip small_cap_needed)
  bool small_live = false;         // some map may still be in the window (the host then reads the event count)
  // map size / isEmpty rows answered in the stream (outside TTL mode; map_small.hip k_size_answer)
  uint32_t* d_szq = nullptr;       // [szq_cap] the batch's size / isEmpty rows
  uint32_t* d_szq_n = nullptr;
  uint32_t szq_cap = 0;
  uint32_t szq_n = 0;              // this batch's
  bool szq_flagged = false;        // maps carry kMfSize / kMfCv from the last batch (cleared before the next scan)
  // containsValue in the stream (map_cv.hip)
  uint32_t* d_cvq = nullptr;       // [cvq_cap] the batch's candidate rows
  uint32_t* d_cvq_n = nullptr;     // [2]: candidates, rows kept in the stream
  uint32_t cvq_cap = 0;
  uint32_t* d_isc = nullptr;       // [cvq_cap] rows answered in the stream (sorted into d_isc2)
  uint32_t* d_isc2 = nullptr;
  uint32_t* d_mfirst = nullptr;    // [max_resources] first null-storing / deleting row of a flagged map
  uint8_t* d_maynull = nullptr;    // [max_resources]
  void* d_cv_rtemp = nullptr;      // row sort scratch
  size_t cv_rtemp_bytes = 0;
  std::vector<uint32_t> isc_rows;  // this batch's in-stream rows, ascending
  CvEnt* d_cvset = nullptr;        // [cvset_cap] operand set of a sub-batch
  uint32_t* d_cvcnt = nullptr;     // [cvset_cap]
  uint32_t cvset_cap = 0;
  uint64_t* d_cvev_key = nullptr;  // [cvev_cap] events (and sorted copies)
  uint64_t* d_cvev_key2 = nullptr;
  uint32_t* d_cvev_val = nullptr;
  uint32_t* d_cvev_val2 = nullptr;
  uint32_t* d_cvev_ctl = nullptr;
  uint32_t* d_cvseg = nullptr;     // [cvset_cap + 1] run starts (+ count)
  void* d_cvtemp = nullptr;
  size_t cvtemp_bytes = 0;
  uint32_t cvev_cap = 0;
  uint64_t stat_barriers = 0, stat_isc = 0, stat_subbatches = 0, stat_events = 0;  // cc_engine_counters
  // clears in the stream (map_clear.hip)
  uint32_t* d_clrq = nullptr;      // [clrq_cap] the batch's in-stream clear rows
  uint32_t* d_clrq_n = nullptr;
  uint32_t clrq_cap = 0;
  uint64_t* d_clr_keys = nullptr;  // [clrq_cap] scratch, then (slot << 32 | row) ascending in d_clr_keys2
  uint64_t* d_clr_keys2 = nullptr;
  uint32_t* d_clr_off = nullptr;   // [max_resources + 1]
  uint32_t* d_clr_base = nullptr;  // [max_resources]
  uint8_t* d_clr_eend = nullptr;   // [max_resources]
  uint8_t* d_tbl_ep = nullptr;     // [map_entries] hot entries' clear epochs within a sub-batch (0 between)
  void* d_clr_temp = nullptr;
  size_t clr_temp_bytes = 0;
  uint32_t clr_n = 0;              // this batch's
  std::vector<std::vector<uint32_t>> clr_heavy;  // rows of the maps cleared >= 128 times in this batch (sub-batch cuts)
  unsigned long long* d_mw_ctl = nullptr;  // [16]
  std::vector<uint32_t> bars;
  // map TTL timers (apply_map.hip k_apply_map<true>): entered on the first map row with ttl > 0, for good
  uint64_t* d_tbl_dl = nullptr;    // [map_entries] timer deadline per entry (0: none)
  uint32_t* d_map_row = nullptr;   // [sub_batch] staging position -> batch row
  uint32_t* d_ttl_seen = nullptr;
  bool ttl_live = false;
  bool has_sets = false;
  bool has_values = false;  // an AtomicValueState resource was ever created (else k_apply_value is not launched)
  bool has_mmaps = false;  // MultiMapState resources share the map table too (every Put lands in the leak log)  // SetState resources share the map table (results rewritten by k_set_results)
  // MembershipGroupState.schedule timers (MembershipGroupState.java:86-103): armed by schedule barrier rows, fired
  // at the batch boundary where the reference's fire_due runs (host-ordered by (deadline, id))
  struct GroupTimer {
    uint64_t deadline, id, member, payload;
    uint32_t slot, tag;
    uint64_t fire_b;  // boundary in the current batch (rows before it applied first); ~0: not in this batch
    uint64_t idx;     // the schedule commit's log index (retained until the timer fires, :86-103)
  };
  std::vector<GroupTimer> gtimers;
  uint64_t gtimer_seq = 0;
  uint32_t* d_hot_rpre = nullptr;
  uint32_t* d_hot_rstart = nullptr;
  uint32_t* d_hot_len = nullptr;
  uint32_t* d_hot_cond = nullptr;
  void* d_hot_agg = nullptr;
  void* d_hot_s0 = nullptr;
  void* d_hot_samp = nullptr;
  // extended staging (maps / coordination / value events) + coordination + events
  bool ext = false, coord_on = false;
  std::vector<uint8_t> sb_kind;      // [sb] 1: the super-bucket runs on k_apply_coord
  uint8_t* d_sb_kind = nullptr;
  uint64_t* d_inst_id = nullptr;     // instance slot -> instance id (election listeners, group members)
  uint8_t* d_coord = nullptr;        // [slots] coordination blocks
  uint64_t* d_clock = nullptr;       // the engine's log clock (max time applied / advanced)
  uint16_t* d_ev_cnt = nullptr;      // [sub_batch] events per staged commit
  uint32_t* d_row_of = nullptr;      // [sub_batch]
  uint32_t* d_ev_loc = nullptr;      // [sub_batch]
  uint32_t* d_tile_sum = nullptr;    // [max_tiles]
  uint64_t* d_tile_off = nullptr;    // [max_tiles]
  EvRec* d_arena = nullptr;
  EvRec* d_ev_bucket = nullptr;      // [arena_cap] the arena grouped by partition tile (events.hip)
  uint32_t* d_ev_ccnt = nullptr;     // [ev_chunk_cap(arena_cap) * max_tiles] per (arena chunk, tile) counts / bases
  uint32_t* d_ev_perm = nullptr;     // [arena_cap] event output order -> arena index (events.hip)
  unsigned long long* d_arena_n = nullptr;
  unsigned long long* d_ev_total = nullptr;
  uint64_t arena_cap = 0;
  // commits dropped without clean() (LeakRec, common.h): the kernels' device log, drained into per-slot host lists
  LeakRec* d_leak = nullptr;
  unsigned long long* d_leak_n = nullptr;
  uint64_t leak_cap = 0;
  std::map<uint32_t, std::vector<uint64_t>> leaks;  // ordered: snapshots are byte-deterministic
  uint64_t applied = 0;
  bool applied_pending = false;
  uint32_t last_err_bits = 0;        // the device error bits the last check_device_err read (common.h kErr*)
  bool span_cut = false;             // this batch's index range passes 2^32: sub-batches are cut at k_span_cut's row
  uint64_t* d_span_cut = nullptr;
  // the prefix apply's device checkpoint (cc_apply_batch_host_prefix): every device section the data path writes, as
  // one device-to-device copy, and the host fields it moves
  void* d_ckpt = nullptr;
  uint64_t ckpt_bytes = 0;
  struct Ckpt {
    uint64_t applied = 0;
    bool applied_pending = false, ttl_live = false, small_live = false;
    std::vector<GroupTimer> gtimers;
    uint64_t gtimer_seq = 0;
    std::map<uint32_t, std::vector<uint64_t>> leaks;
  } ckpt;
  uint64_t* d_last_index = nullptr;  // index[n-1] of the last batch (device copy)
  // device staging of the host-memory entry points (host_path.hip): grown on demand, kept between calls
  void* hw_buf[24] = {};
  size_t hw_cap[24] = {};
  // per-kernel profiling (cc_profile_enable)
  bool prof_on = false;
  std::vector<hipEvent_t> ev_pool;
  struct Pending { int kernel; hipEvent_t a, b; bool shared_a; };  // shared_a: a is an earlier Pending's b
  hipEvent_t last_end = nullptr;     // value-only engines: the last end marker, reused as the next begin marker
  hipStream_t last_end_st = nullptr;
  bool open_shared[K_NUM] = {};
  std::vector<Pending> pending;
  hipEvent_t open_ev[K_NUM] = {};
  double prof_ms[K_NUM] = {};
  uint64_t prof_n[K_NUM] = {};
};
