// engine_internal.h — launch-parameter structs shared by the engine's translation units.
#pragma once
#include <cstdlib>

#include "common.h"

// A/B and diagnostics switches read from the environment (CC_NO_HOT, CC_EV_V1, CC_EV_SCATTER, CC_PART_EXT_1024) exist
// only in -DCC_DIAG builds (copycat_amd/build.py build_variant); the product library never takes an untested path.
inline bool diag_env(const char* name) {
#ifdef CC_DIAG
  return getenv(name) != nullptr;
#else
  (void)name;
  return false;
#endif
}

namespace cc {

// Optional per-kernel timing (HIP events recorded on the launch stream around each kernel).
enum KernelId { K_PART_TILE = 0, K_APPLY_VALUE, K_UNPERMUTE, K_APPLY_MAP, K_MAP_HOT, K_APPLY_COORD, K_EVENTS, K_NUM };
struct Marker {
  void (*fn)(void* ctx, int kernel, int begin, hipStream_t st);
  void* ctx;
  void operator()(int k, int begin, hipStream_t st) const {
    if (fn) fn(ctx, k, begin, st);
  }
};

// Phase clocks of the diagnostics build (common.h PH_*): read and clear one kernel's sums (ticks of 10 ns).
int phase_read(int kernel, uint64_t* out /*[kPhases]*/);

// One sub-batch [lo, hi) of a batch (absolute row indices; column pointers are whole-batch; staging buffers
// are indexed relative to lo).
struct PartArgs {
  const uint32_t* inst;
  const uint8_t* op;
  const uint8_t* flags;
  const uint64_t* a;
  const uint64_t* b;
  const uint64_t* key;    // maps only
  const uint64_t* index;  // maps only (commit index of map entries)
  const uint64_t* aux;    // maps: ttl (> 0 not applied on the GPU); locks: timeout
  const uint64_t* time;   // locks: log time (clock)
  const uint64_t* clock_base;  // device: the engine clock before this batch
  uint32_t ext_flags;     // kExtValue | kExtDeferred | kExtTimeCheck
  uint32_t* err;          // device error bits (kExtTimeCheck: kErrTime)
  bool ext;               // extended staging (maps / coordination / value events)
  uint64_t lo, hi;
  const uint32_t* inst_res;
  const uint64_t* inst_id;   // coordination engines: instance ids, carried in XRec.pad for k_apply_coord (else null)
  const uint8_t* res_type;
  const uint8_t* sb_kind;  // value super-buckets run by k_apply_coord (their value records stay unencoded)
  uint32_t max_inst;
  uint32_t sb;        // super-buckets in total = sb_val + 2^map_bits (0 map bits: no maps)
  uint32_t sb_val;
  uint32_t map_bits;
  uint32_t sbq_base;  // non-zero: commits of super-buckets run by k_apply_coord go to quarter buckets sbq_base + slot/64
  const HotKey* hot;  // hot map keys of this sub-batch (maps only)
  const uint32_t* hot_n;
  uint32_t* st_meta;  // staging records [sub_batch], tile-local layout
  u64x2* st_ab;
  XRec* xrec;         // extended staging records (k_part_ext): coordination and value-event commits
  MRec* mrec;         // map / set / multimap commits' 32-byte records (same staging positions)
  uint32_t* hot_meta; // maps: the meta word of each hot-bucket record again, compact (k_hot_agg reads only these)
  ClrCtx clr{};       // clears in the stream: each map commit's clear epoch into its meta (bits 25-31, map_clear.hip)
  uint16_t* cpos;     // [sub_batch] tile-local staging position of commit lo+i (0xFFFF: unknown session)
  uint16_t* ttab;     // [tiles][sb+1] tile-local run starts (+ live count)
  uint64_t dummy;     // first of the kPT dummy staging rows after the staging area (= sub_batch)
  bool v3;               // value-only pipeline of value_path.hip (8192-commit tiles, 16-byte records in st_ab)
  Marker mark;
};
int launch_partition(const PartArgs& a, hipStream_t st);
int launch_part_ext(const PartArgs& a, uint32_t tiles, hipStream_t st);
int launch_part_v3(const PartArgs& a, uint32_t tiles, hipStream_t st);
size_t tile_lds_bytes(uint32_t sb, bool maps, size_t chunk, bool ids = false);  // ids: k_part_ext's instance-id plane
size_t part_ext_chunk(uint32_t sb, bool maps, bool ids);  // k_part_ext's chunk for sb buckets (0: its LDS cannot hold them)

struct ValueArgs {
  const uint32_t* st_meta;
  u64x2* st_ab;  // (value_path.hip: the records, then the packed results over them)
  const uint16_t* ttab;
  uint32_t tiles;
  uint32_t sb;           // total super-buckets (ttab row width - 1)
  uint32_t sb_val;       // value super-buckets (the apply grid)
  const uint8_t* sb_kind;  // non-zero: the super-bucket runs on k_apply_coord (may be null)
  uint32_t* val_meta;    // [sb*256]
  uint64_t* val_v;       // [sb*256]
  uint8_t* rst_status;   // staged results [sub_batch + kPT]
  uint64_t* rst_value;
  uint64_t dummy;        // first of the dummy result rows after the staging area (= sub_batch)
  uint32_t* err;
  bool v3;               // value_path.hip: 8-byte records, 8192-commit tiles
  const uint64_t* ca;    //   the batch's a / b columns (operands of escaped records) and the sub-batch's first row
  const uint64_t* cb;
  uint64_t lo;
  Marker mark;
};
int launch_apply_value(const ValueArgs& a, hipStream_t st);
int launch_apply_value_v3(const ValueArgs& a, hipStream_t st);
int launch_selfcheck(uint32_t* d_bad, hipStream_t st);

struct MapArgs {
  CvCtx cv{};          // in-stream containsValue (map_cv.hip): value-change events of the flagged maps
  ClrCtx clr{};        // clears in the stream (map_clear.hip): commit epochs, the end-of-launch drop
  const MRec* mrec;
  const uint64_t* cb;  // the batch's b column (replaceIfPresent's compare value, mrec_ab)
  uint64_t lo;         // the sub-batch's first row
  const uint16_t* ttab;
  uint32_t tiles;
  uint32_t sb;  // total super-buckets (ttab row width - 1)
  uint32_t sb_val;
  uint32_t map_bits;
  uint64_t* tbl_key;  // [2^map_bits * kMapRegion]
  uint32_t* tbl_word;
  uint64_t* tbl_val;
  uint64_t* tbl_ci;
  uint64_t* tbl_ins;
  uint64_t* tbl_claim;        // [entries] log index at which the entry was first bound (tree-bin test, map_wide.hip)
  const uint64_t* idx0;       // device: the sub-batch's first log index (index column + lo)
  uint64_t* dropped;  // [max_resources] compaction drops bound-but-absent entries: counted per map (map_wide.hip)
  const uint64_t* cgen; // [max_resources] map generations (bumped by clear / Delete)
  CsetEnt* cset;        // the compacted keys (common.h CsetEnt): each drop is inserted
  uint64_t cset_mask;
  uint32_t* cset_full;
  bool ttl;           // TTL mode: entries carry timer deadlines (k_apply_map<true>)
  uint64_t* tbl_dl;
  const uint32_t* map_row;     // [sub_batch] staging position -> batch row (launch_map_rows)
  const uint64_t* time;        // batch columns (absolute rows)
  const uint64_t* aux;
  const uint64_t* clock_base;  // device: the engine clock before this batch
  bool deferred;               // manager-mode timer order (CC_CFG_TIMERS_DEFERRED)
  uint8_t* rst_status;
  uint64_t* rst_value;
  uint32_t* rst_msz;           // [sub_batch] each commit's map and size change (msz_word), staging order
  TtlEmit ttl_emit;            // TTL mode: expiries the walk sees (a commit after its key's timer fired), as events
  uint32_t* err;
  Marker mark;
};
int launch_apply_map(const MapArgs& a, hipStream_t st);
// Exact map sizes and HashMap capacities (map_wide.hip): after a sub-batch's map kernels, per (tile, map) insert /
// remove counts from rst_msz, then per map a scan over its tiles (sizes at tile starts, capacity bounds per tile)
// and an exact in-tile pass for the few tiles whose counts alone leave the capacity open.  Engines with maps
// outside TTL mode.
constexpr uint32_t kMpInexact = 1u << 31;  // mpcap flag: the capacity level is a lower bound only (list overflow)
constexpr uint32_t kMszListCap = 1u << 18;  // (tile, map) pairs resolved exactly per sub-batch
struct MapSizeArgs {
  const uint16_t* ttab;
  const uint16_t* cpos;
  uint32_t tiles;
  uint64_t rows;               // rows of the sub-batch
  uint32_t sb;                 // ttab row width - 1
  uint32_t k0, k1;             // the map and hot-key buckets [k0, k1)
  uint32_t sb_hot;             // the first hot-key bucket
  const uint32_t* rst_msz;     // region records (k_apply_map)
  const HotKey* hot;           // hot-key records (k_hot_apply): codes per hot list position
  const uint32_t* hot_n;
  const uint32_t* hot_len;
  const uint32_t* hot_rpre;
  const uint32_t* hot_msz;
  const uint8_t* res_type;
  uint32_t max_resources;
  uint32_t* tcnt;              // [tiles][max_resources] (inserts | removes << 16) per (tile, map)
  uint32_t* msize;             // [max_resources] live size at the sub-batch boundary
  uint32_t* mpcap;             // [max_resources] log2(HashMap capacity / 16) of the peak size so far (| kMpInexact)
  uint4* list;                 // [kMszListCap] (tile, map, size at the tile's start) pairs for the exact pass
  uint32_t* list_n;
  // small maps (map_small.hip): events of the maps still in the window (null msmall: none is)
  const uint8_t* msmall;       // [max_resources] 1: the map's table is small (capacity <= 64), followed key by key
  const MRec* mrec;            // the sub-batch's map records (log index, key, key tag)
  const uint64_t* idx0;        // device: the log index of the sub-batch's first row
  const uint64_t* hh_key;      // String.hashCode of HANDLE keys (cc_handle_hashes), sorted by handle
  const int32_t* hh_val;
  uint32_t hh_n;
  uint64_t* ev_key;            // [ev_cap] map << kEvMapShift | (index - idx0) << 4 | code
  uint32_t* ev_val;            // [ev_cap] the emission slot (its payload: ev_pay)
  EvPay* ev_pay;               // [ev_cap] key, tag and HashMap hash
  uint32_t ev_cap;
  uint32_t* sm_ctl;            // [0] events emitted
  const uint32_t* map_row;     // TTL mode: every map's commits emitted, positioned by batch row (common.h TtlEmit)
  uint64_t lo;                 //   (the sub-batch's first row)
  unsigned long long* lvl_at;  // the capacity-level timeline (k_msize_exact records each resize's log index)
  const uint64_t* index;       // the batch's index column (absolute rows)
  uint32_t* err;
};
int launch_map_size(const MapSizeArgs& a, hipStream_t st);
struct SmallArgs {
  uint64_t *ev_key, *ev_key2;  // events and their sorted copy
  uint32_t *ev_val, *ev_val2;  // emission slots
  const EvPay* ev_pay;         // payloads by emission slot
  uint32_t cap;
  void* temp;                  // hipcub radix-sort scratch
  size_t temp_bytes;
  uint32_t* ctl;               // [0] events, [1] maps still in the window (after the replay)
  uint32_t* seg;               // [max_resources] run starts
  uint32_t* nseg;
  // outside TTL mode: the replayed maps' events without the ones alternating chains imply (k_small_chains), as
  // positions in the sorted buffer (written over ev_key), their count and runs: [max_resources] starts, then the
  // run count, then the event count (null: every event is replayed, TTL mode)
  uint32_t* cseg;
  hipEvent_t ev_prep;          // (a replay on another stream: recorded after the sort and compaction)
  bool defer;                  // outside TTL mode: sort and compact only; the replay kernel comes later
                               // (launch_small_replay_kernel)
  uint8_t* out_status;         // TTL mode: the size / isEmpty rows among the events are answered here (else null)
  uint64_t* out_value;
  SmallMap* state;             // [max_resources]
  BigMap* big;                 // [kBigSlots] the models of maps that left the window with a tree bin (null: none)
  uint8_t* msmall;             // the engine stream's snapshot of the window (common.h): read, never written, by the replay
  uint8_t* left;               // [max_resources] the replay's exit marks (one buffer per event-buffer set), folded by
                               // launch_small_fold on the engine stream after it waited for the replay
  uint32_t* err;
  uint32_t* mpcap;
  uint32_t max_resources;
  uint32_t* msize;             // TTL mode: every map's size / capacity from its events (k_ttl_replay); else null
  // the capacity-level timeline (common.h lvl_reached): an event's log index is idx0 + its offset, or in TTL mode
  // (positions by row, common.h TtlEmit) the index column at row lo + (position - 1) / 2
  unsigned long long* lvl_at;  // [max_resources * kLvlSlots] (null: not recorded)
  const uint64_t* idx0;
  const uint64_t* index;
  uint64_t lo;
};
// TTL mode: the table entries whose timers fire at a boundary the sub-batch owns -> expiry events (common.h TtlEmit)
int launch_ttl_scan(const TtlEmit& t, const uint64_t* clock_base, const uint32_t* word, const uint64_t* key,
                    const uint64_t* dl, uint64_t entries, uint32_t* err, hipStream_t st);
// sort, runs, replay (E events); the replay kernel itself on stream rst (after a.ev_prep, when rst != st)
int launch_small_replay(const SmallArgs& a, uint32_t E, hipStream_t st, hipStream_t rst);
int launch_small_replay_kernel(const SmallArgs& a, hipStream_t rst);
// map_big.hip: the big models' replay, over the same events as the small replay (orig: compacted positions, else
// every event; cnt: the event count; seg / nseg: the runs), on the small replay's stream after it
int launch_big_replay(const SmallArgs& a, const uint32_t* orig, const uint32_t* cnt, const uint32_t* seg,
                      const uint32_t* nseg, hipStream_t rst);
// a whole-map barrier's clear / Delete of map m on its big model
int launch_big_clear(BigMap* big, const SmallMap* state, uint32_t m, hipStream_t st);
// resource creation: the big models of the slots [first, first + count) are freed
int launch_big_release(BigMap* big, uint32_t first, uint32_t count, hipStream_t st);
int launch_small_finish(const SmallArgs& a, hipStream_t st);              // counters for the next sub-batch
// size / isEmpty rows of the sub-batch [lo, hi): emitted into the event buffer before the sort (query entries), then
// answered from the sorted buffer after the unpermute (the row's staged result is a placeholder)
struct SizeArgs {
  const uint32_t* szq;          // the batch's size / isEmpty rows (unordered)
  uint32_t szq_n;
  uint64_t lo, hi;              // the sub-batch's rows
  const uint32_t* inst;         // batch columns
  const uint8_t* op;
  const uint64_t* index;
  const uint32_t* inst_res;
  uint64_t* ev_key;
  uint32_t* ev_val;
  EvPay* ev_pay;
  uint32_t cap;
  uint32_t* ctl;                // [0] the event count
  const uint64_t* sorted_key;   // after the sort
  const uint32_t* sorted_val;
  const uint32_t* seg;
  const uint32_t* nseg;
  const uint32_t* msize;        // [max_resources] live sizes at the sub-batch end (exact tracking)
  uint8_t* out_status;          // the batch's result columns (absolute rows)
  uint64_t* out_value;
  bool ttl;                     // TTL mode: queries positioned by row (common.h TtlEmit), answered by k_ttl_replay
  uint32_t* err;                // kErrSpan: a sub-batch spanning 2^32 log indices
};
int launch_size_emit(const SizeArgs& a, hipStream_t st);
int launch_size_answer(const SizeArgs& a, hipStream_t st);
int launch_mflag_clear(uint8_t* mflag, uint32_t R, hipStream_t st);
int launch_small_fold(uint8_t* left, uint8_t* msmall, uint32_t R, hipStream_t st);
int launch_span_cut(const uint64_t* index, uint64_t lo, uint64_t hi, uint64_t* out, hipStream_t st);
size_t small_sort_temp_bytes(uint32_t cap);
int launch_small_clear(SmallMap* state, uint32_t m, hipStream_t st);
int launch_map_drop_resource(uint32_t* tbl_word, uint64_t entries, uint32_t slot, uint64_t* cgen, hipStream_t st);
int launch_map_rows(const uint16_t* cpos, uint64_t lo, uint64_t hi, uint32_t* map_row, hipStream_t st);

// Whole-map ops (containsValue / isEmpty / size / clear / Delete): barrier rows of a batch (map_wide.hip).
constexpr uint32_t kBarCap = 1u << 16;  // barrier rows per batch
// Also flags (ttl_seen = 1) a map put/putIfAbsent/replace/replaceIfPresent row with ttl > 0.
// Outside TTL mode map size / isEmpty rows are not barriers: they are listed in szq (rows) and their maps flagged
// (kMfSize in mflag), then answered in the stream (map_small.hip launch_size_answer).
int launch_map_barriers(const uint32_t* inst, const uint8_t* op, const uint64_t* aux, uint64_t n, const uint32_t* inst_res,
                        const uint8_t* res_type, uint32_t max_inst, uint32_t* bar, uint32_t* bar_n, uint32_t cap,
                        uint32_t* ttl_seen, uint32_t* szq, uint32_t* szq_n, uint32_t szq_cap, uint8_t* mflag,
                        uint32_t* cvq, uint32_t* cvq_n, uint32_t cvq_cap, uint32_t* mfirst, uint32_t R,
                        uint32_t* clrq, uint32_t* clrq_n, uint32_t clrq_cap, hipStream_t st);
// ---- containsValue in the stream (map_cv.hip) ----
struct CvBatchArgs {  // per batch: classify the candidates listed by k_map_barriers
  const uint32_t* inst;
  const uint8_t* op;
  const uint8_t* flags;
  uint64_t n;
  const uint32_t* inst_res;
  uint32_t max_inst;
  const uint8_t* mflag;
  const uint32_t* tbl_word;
  uint64_t entries;
  const uint32_t* cvq;
  const uint32_t* cvq_n;
  uint32_t cvq_cap;
  uint32_t* mfirst;   // per map: the first row that stores a null or deletes the map (~0: none)
  uint8_t* maynull;   // per map: holds a null value at the batch start
  uint32_t R;
  uint32_t* bar;
  uint32_t* bar_n;
  uint32_t bar_cap;
  uint32_t* isc;      // the rows answered in the stream (unsorted)
  uint32_t* isc_n;
};
int launch_cv_batch(const CvBatchArgs& a, hipStream_t st);
int cv_sort_rows(uint32_t* rows, uint32_t* rows2, uint32_t n, void* temp, size_t temp_bytes, hipStream_t st);
size_t cv_rows_temp_bytes(uint32_t n);
struct CvSubArgs {  // per sub-batch: the operand set, initial counts and query events, then the answers
  CvCtx cv;           // set / mask / events (the apply kernels get the same)
  ClrCtx clr;         // clears in the stream: a query's epoch (map_clear.hip)
  CvEnt* set;
  uint32_t* cnt;      // per set position: matching entries at the sub-batch start
  const uint32_t* isc;  // this sub-batch's in-stream rows (sorted)
  uint32_t isc_n;
  uint64_t lo;
  const uint32_t* inst;
  const uint8_t* flags;
  const uint64_t* a;
  const uint64_t* index;
  const uint32_t* inst_res;
  const uint32_t* tbl_word;
  const uint64_t* tbl_val;
  uint64_t entries;
  uint32_t* err;
  uint32_t* coll;     // operands whose fingerprint another claimed (k_cv_verify -> k_cv_fix), and their count
  uint32_t* coll_n;
  // answers
  uint64_t* key2;
  uint32_t* val2;
  uint32_t* seg;
  uint32_t* nseg;
  void* temp;
  size_t temp_bytes;
  uint8_t* out_status;
  uint64_t* out_value;
};
int launch_cv_prepare(const CvSubArgs& a, hipStream_t st);
// ---- clear in the stream (map_clear.hip) ----
struct ClrBatchArgs {
  const uint32_t* rows;  // the batch's in-stream clear rows
  uint32_t n;
  const uint32_t* inst;
  const uint32_t* inst_res;
  uint64_t* keys;        // [n] scratch
  uint64_t* keys2;       // [n] (slot << 32 | row), ascending
  uint32_t* off;         // [R + 1]
  uint32_t R;
  void* temp;
  size_t temp_bytes;
};
int launch_clr_batch(const ClrBatchArgs& a, hipStream_t st);
size_t clr_sort_temp_bytes(uint32_t n);
struct ClrSubArgs {
  const uint64_t* keys;  // sorted
  uint32_t n;
  const uint32_t* off;
  uint32_t R;
  uint64_t lo, hi;
  uint32_t* base;
  uint8_t* eend;
  uint8_t* mflag;  // kMfClr: cleared in this sub-batch
  uint8_t* btab;   // [R][nb] epochs at the row buckets' starts (common.h ClrCtx)
  uint32_t nb, bshift;
  uint32_t* err;
  const uint64_t* index;
  uint64_t* ev_key;
  uint32_t* ev_val;
  EvPay* ev_pay;
  uint32_t ev_cap;
  uint32_t* ev_ctl;
  uint64_t* cgen;
};
int launch_clr_sub(const ClrSubArgs& a, hipStream_t st);
int launch_clr_events(const ClrSubArgs& a, hipStream_t st);
int launch_clr_gen(const ClrSubArgs& a, hipStream_t st);
struct ClrReplayArgs {
  const uint64_t* key;  // the sorted map events
  const uint32_t* val;
  const EvPay* pay;
  const uint8_t* mflag;
  uint32_t* msize;
  uint32_t* mpcap;
  unsigned long long* lvl_at;
  const uint64_t* idx0;
  uint8_t* out_status;
  uint64_t* out_value;
  void* scan;         // [events] clr_scan_bytes_per_event() each
  void* temp;
  size_t temp_bytes;  // >= clr_scan_temp_bytes(events)
};
int launch_clr_replay(const ClrReplayArgs& a, uint32_t E, hipStream_t st);
size_t clr_scan_temp_bytes(uint32_t cap);
size_t clr_scan_bytes_per_event();
int launch_cv_answer(const CvSubArgs& a, uint32_t E, hipStream_t st);
size_t cv_sort_temp_bytes(uint32_t cap);
struct MapWideArgs {
  uint32_t slot, op, atag;
  uint64_t apay;
  uint64_t row;  // absolute row of the barrier in the batch
  uint32_t* tbl_word;
  const uint64_t* tbl_key;
  const uint64_t* tbl_val;
  const uint64_t* tbl_ins;
  const uint64_t* tbl_claim;   // first-bound log index of each entry, and each map's capacity-level timeline: a key
  const unsigned long long* lvl_at;  // counts at level L only if bound before the table left L (common.h)
  const uint64_t* tbl_dl;      // TTL mode: entry deadlines (null: no timers)
  uint64_t fire_clock;         // entries with a deadline <= this clock have expired at the barrier row
  uint64_t entries;
  uint32_t* peak_lo;           // [max_resources] lower bound on the map's peak size
  uint64_t* dropped;           // [max_resources] entries dropped by compaction / clear (upper-bound term)
  uint64_t* cgen;              // [max_resources] map generations: clear / Delete bump them
  const CsetEnt* cset;         // keys compacted away from the table (tree-bin test: k_mw_cset)
  uint64_t cset_n;
  const uint32_t* cset_full;
  uint32_t map_bits;
  uint32_t* msize;             // exact tracking (launch_map_size; null in TTL mode): the live size, and
  const uint32_t* mpcap;       //   log2(capacity / 16) of the peak (in TTL mode a lower bound for the bounds above)
  unsigned long long* ctl;     // [C_N] scratch
  const SmallMap* small;       // [max_resources] the small-table state (early resizes, tree bins; map_small.hip)
  const BigMap* big;           // [kBigSlots] the models of maps past the window with a tree bin (map_big.hip)
  const uint64_t* hh_key;      // String.hashCode of HANDLE keys (sorted by handle)
  const int32_t* hh_val;
  uint32_t hh_n;
  uint8_t* out_status;
  uint64_t* out_value;
  uint32_t* err;
};
int launch_map_wide(const MapWideArgs& a, hipStream_t st);
// MembershipGroupState.schedule barrier rows and their timers (apply_coord.hip)
int launch_group_schedule(const uint8_t* coord, uint32_t ccap, uint32_t slot, uint64_t member, uint64_t row, uint8_t* out_status,
                          uint64_t* out_value, uint32_t* found, hipStream_t st);
int launch_group_fire(const uint8_t* coord, uint32_t ccap, uint32_t slot, uint64_t member, uint32_t tag, uint64_t payload, uint32_t pos,
                      unsigned long long* ev_total, const cc_events* ev, uint32_t* err, hipStream_t st);
// SetState result rewrite after the batch (map_wide.hip)
int launch_value_live(const uint32_t* inst, const uint8_t* op, const uint8_t* status, const uint64_t* value,
                      const uint64_t* index, uint64_t n, const uint32_t* inst_res, const uint8_t* res_type,
                      uint32_t max_inst, const uint32_t* val_meta, uint32_t slots, unsigned long long* wrow,
                      uint64_t* live, hipStream_t st);
// set / multimap results of the map ops they ran as (map_wide.hip k_keyed_results)
struct KeyedResultArgs {
  const uint32_t* inst;
  const uint8_t* op;
  const uint8_t* flags;
  const uint64_t* index;
  uint64_t n;
  const uint32_t* inst_res;
  const uint8_t* res_type;
  uint32_t max_inst;
  uint8_t* status;
  uint64_t* value;
  LeakRec* leak;  // multimap Put commits (never cleaned)
  unsigned long long* leak_n;
  uint64_t leak_cap;
  uint32_t* err;
};
int launch_keyed_results(const KeyedResultArgs& a, hipStream_t st);

#ifndef CC_HOT_GRID_AGG
#define CC_HOT_GRID_AGG 1024
#endif
#ifndef CC_HOT_GRID_APPLY
#define CC_HOT_GRID_APPLY 1024
#endif
// workgroups of the hot-key scan kernels (grid-stride over pieces; -D overrides for A/B builds only)
constexpr int kHotGridAgg = CC_HOT_GRID_AGG;
constexpr int kHotGridApply = CC_HOT_GRID_APPLY;
// clears in the stream for the hot-key scan (map_clear.hip): commit epochs from their rows, the cleared maps' size
// events, the entry dropped when its state predates the map's last clear of the sub-batch
struct HotClr {
  ClrCtx clr;                // clr.mflag == nullptr: no clears in this batch
  const MRec* xr;
  uint64_t lo;
  uint64_t* ev_key;          // the map event buffer (map_small.hip SmallArgs)
  uint32_t* ev_val;
  EvPay* ev_pay;
  uint32_t ev_cap;
  uint32_t* ev_ctl;
  const uint64_t* idx0p;
  uint8_t* tbl_ep;           // [map_entries] the clear epoch a hot key's entry ends at (read by k_apply_map)
  // the map events of small / size-queried / cleared maps' hot commits (null: no such maps in this batch)
  const uint8_t* mflag;
  const uint64_t* hh_key;    // String.hashCode of HANDLE keys (java_key_hash)
  const int32_t* hh_val;
  uint32_t hh_n;
  uint32_t* err;
};
struct HotArgs {
  CvCtx cv{};  // in-stream containsValue (map_cv.hip)
  HotClr hc{};  // clears in the stream (map_clear.hip)
  // detection (before the partition)
  const uint32_t* inst;
  const uint8_t* flags;
  const uint64_t* key;
  uint64_t lo, hi;
  const uint32_t* inst_res;
  const uint8_t* res_type;
  uint32_t max_inst;
  // scan (after the partition)
  const MRec* mrec;
  const uint64_t* cb;  // the batch's b column (mrec_ab)
  const uint16_t* ttab;
  uint32_t tiles, sb, sb_val, map_bits;
  uint64_t* tbl_key;
  uint32_t* tbl_word;
  uint64_t* tbl_val;
  uint64_t* tbl_ci;
  uint64_t* tbl_ins;
  uint64_t* tbl_claim;    // [entries] first-bound log index of each entry (k_hot_bind claims with idx0)
  const uint64_t* idx0;   // device: the sub-batch's first log index
  HotKey* hot;
  uint32_t* hot_n;
  const uint8_t* msmall;  // [max_resources] maps in their small-table window (map_small.hip): never hot-routed
  HotKey* hot_cand;      // [kHotMax] the batch's hot keys by rank (k_hot_count), bound per sub-batch (k_hot_bind)
  const uint32_t* hot_meta;  // [sub_batch] meta word of each hot-bucket record (k_part_ext), read by k_hot_agg
  uint32_t* hot_cand_n;
  uint32_t* hot_rpre;    // [kHotMax][kMaxTiles + 1]
  uint32_t* hot_rstart;  // [kHotMax][kMaxTiles]
  uint32_t* hot_len;     // [kHotMax]
  uint32_t* hot_cond;    // [kHotMax]
  void* hot_agg;         // [kHotMax][kHotMaxPieces] composites
  void* hot_s0;          // [kHotMax] entry snapshots
  void* hot_samp;        // [65536] resolved detection sample (apply_map_hot.hip HotSamp)
  uint8_t* rst_status;
  uint64_t* rst_value;
  uint32_t* hot_msz;     // [(kHotMaxPieces + kHotMax) * kHotPiece / 16] 2-bit size-change codes per list position
  uint32_t* err;
  Marker mark;
};
int launch_map_hot_detect(const HotArgs& a, hipStream_t st);  // once per batch: sample + count (rows [lo, hi))
int launch_map_hot_bind(const HotArgs& a, hipStream_t st);    // per sub-batch: the candidates' table entries
int launch_map_hot_apply(const HotArgs& a, hipStream_t st);
size_t hot_agg_bytes();
size_t hot_s0_bytes();
size_t hot_samp_bytes();

struct CoordArgs {
  const XRec* xrec;
  const uint16_t* ttab;
  uint32_t tiles, sb, sb_val;
  uint32_t sbq_base;       // non-zero: the quarter buckets of the partition (else each workgroup filters its quarter)
  const uint8_t* sb_kind;
  const uint8_t* res_type;
  const uint64_t* inst_id;
  uint8_t* coord;
  uint32_t coord_cap;      // entries per coordination block (cc_config.coord_cap)
  uint32_t* val_meta;
  uint64_t* val_v;
  uint8_t* rst_status;
  uint64_t* rst_value;
  uint16_t* ev_cnt;
  EvRec* arena;
  unsigned long long* arena_n;
  uint64_t arena_cap;
  LeakRec* leak;           // leak log (LeakRec, common.h)
  unsigned long long* leak_n;
  uint64_t leak_cap;
  uint32_t* err;
  Marker mark;
};
int launch_apply_coord(const CoordArgs& a, hipStream_t st);
int phase_read_coord_wg(uint64_t* out);  // CC_PHASE_TIMING builds
int launch_time_check(const uint64_t* time, uint64_t n, uint64_t* clock, uint32_t* err, hipStream_t st);
int launch_clock_advance(const uint64_t* time, uint64_t n, uint64_t now, uint64_t* clock, hipStream_t st);

struct EventArgs {
  const uint16_t* cpos;
  uint64_t lo, hi;
  uint32_t tiles;
  const uint16_t* ev_cnt;
  uint32_t* row_of;
  uint32_t* ev_loc;
  uint32_t* tile_sum;
  uint64_t* tile_off;
  unsigned long long* ev_total;
  const EvRec* arena;
  const unsigned long long* arena_n;
  uint64_t arena_cap;
  uint32_t* perm;          // [arena_cap] output position - the sub-batch's first -> arena index (CC_EV_V1)
  EvRec* bucket;           // [arena_cap] the arena grouped by tile
  uint32_t* ccnt;          // [ev_chunk_cap(arena_cap) * tiles] per (arena chunk, tile) counts -> bases
  uint64_t out_cap;
  uint32_t* out_pos;
  uint32_t* out_target;
  uint8_t* out_code;
  uint8_t* out_src;
  uint8_t* out_tag;
  uint64_t* out_payload;
  uint32_t* err;
  Marker mark;
};
int launch_events(const EventArgs& a, hipStream_t st);
int launch_ev_shift(uint32_t* pos, uint64_t n, uint32_t by, hipStream_t st);
constexpr uint64_t kEvChunk = 8192;  // arena events per bucketing workgroup (events.hip)
inline uint64_t ev_chunk_cap(uint64_t arena_cap) { return (arena_cap + kEvChunk - 1) / kEvChunk; }

// Session close / expire fan-out (close.hip): m closes in fan-out order, grouped by resource.
struct CloseArgs {
  const uint32_t* cinst;   // [m] instance slots in fan-out order
  uint32_t m;
  const uint32_t* rlist;   // [nr] resources with a close handler among them
  const uint32_t* rstart;  // [nr + 1] -> items
  const uint32_t* items;   // positions, grouped by resource, ascending
  uint32_t nr;
  uint32_t* inst_res;
  const uint8_t* res_type;
  const uint64_t* inst_id;
  uint8_t* coord;          // null: no coordination blocks (then no state machine has a close handler)
  uint32_t coord_cap;      // entries per coordination block
  const uint32_t* pcl;     // [m] client rank of each position (positions are grouped by client, in client order)
  uint32_t* fail;          // [clients] per client: first position whose close throws (init m); that client's
                           // fan-out ends there (ResourceManager.close runs once per session), the others go on
  uint32_t* cnt;           // [m] events per close (zeroed)
  uint64_t* off;           // [m + 1]
  EvRec* arena;
  unsigned long long* arena_n;
  uint64_t arena_cap;
  LeakRec* leak;           // leak log: a group member removed by close (its join commit is never clean()ed)
  unsigned long long* leak_n;
  uint64_t leak_cap;
  uint64_t out_cap;
  uint32_t* out_pos;
  uint32_t* out_target;
  uint8_t* out_code;
  uint8_t* out_src;
  uint8_t* out_tag;
  uint64_t* out_payload;
  uint64_t* out_count;
  uint32_t* err;
};
int launch_close(const CloseArgs& a, hipStream_t st);

// One barrier row's columns, gathered on the device at the start of a batch (k_bar_fields): the host walks the
// batch's barrier rows from these instead of one blocking copy per field per row.
struct BarRow {
  uint64_t a, key, aux, idx;
  uint64_t t_prev, t_row;  // time[row - 1], time[row] (0 without a time column / at row 0)
  uint32_t inst;
  uint8_t op, flags, pad0, pad1;
  uint32_t pad2, pad3;
};
static_assert(sizeof(BarRow) == 64, "BarRow");
int launch_bar_fields(const uint32_t* rows, uint32_t nb, const uint32_t* inst, const uint8_t* op, const uint8_t* flags,
                      const uint64_t* a, const uint64_t* key, const uint64_t* aux, const uint64_t* index,
                      const uint64_t* time, BarRow* out, hipStream_t st);
// Group-timer fire boundaries, one device binary search per timer over the batch's time column: the first row r >=
// from[i] whose clock max(clock_before, time[r]) reaches deadline[i] -> r (+1 when timers are deferred), or ~0.
int launch_fire_bounds(const uint64_t* time, uint64_t n, uint64_t clock_before, const uint64_t* deadline,
                       const uint64_t* from, uint32_t m, bool deferred, uint64_t* out, hipStream_t st);

struct UnpermuteArgs {
  const uint16_t* cpos;
  const uint16_t* ttab;
  uint32_t sb;
  uint64_t lo, hi;
  const uint8_t* rst_status;
  const uint64_t* rst_value;
  uint8_t* out_status;  // whole-batch outputs
  uint64_t* out_value;
  uint8_t* dummy_status;  // 4 x kPT dummy result rows (after the staging area) for unconditional stores
  uint64_t* dummy_value;
  bool v3;                // value_path.hip tiles (8192 commits): packed result words in `words` (the records' area)
  const uint64_t* words;
  Marker mark;
};
int launch_unpermute(const UnpermuteArgs& a, hipStream_t st);
int launch_unpermute_v3(const UnpermuteArgs& a, const uint64_t* words, hipStream_t st);

// The bulk compaction view (retained.hip, cc_retained_bitmap): bit (i - first) of bitmap set iff log index i is held
// by a state machine without clean().
struct RetainedArgs {
  const uint8_t* res_type;
  uint32_t slots;
  const uint64_t* val_live;  // null: no value resources
  const uint32_t* tbl_word;  // null: no maps / sets
  const uint64_t* tbl_ci;
  const uint64_t* tbl_dl;    // null: no map timers
  uint64_t entries;
  const uint8_t* coord;      // null: no coordination blocks
  uint32_t coord_cap;
  const uint64_t* clock;
  const uint64_t* list;      // host-known indices (pending schedules, leak lists), uploaded
  uint64_t list_n;
  uint64_t first, count;
  uint64_t* bitmap;          // ceil(count / 64) words
  unsigned long long* total; // null or: the retained indices in the range (popcount)
};
int launch_retained(const RetainedArgs& a, hipStream_t st);

}  // namespace cc
