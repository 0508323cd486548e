// engine.hip — the C-ABI of include/copycat_apply.h: engine handle, resource/instance registry, and the
// batched apply driver (partition.hip -> apply_*.hip per sub-batch).
//
// Reference interface replaced: the Copycat StateMachine that ResourceManager implements
// (manager/src/main/java/io/atomix/manager/ResourceManager.java:35-264), applying committed entries
// one by one through ResourceManagerStateMachineExecutor.execute (:90-102) and
// ResourceStateMachineExecutor.executeCommand/executeQuery (resource/.../ResourceStateMachineExecutor.java:73-91).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <tuple>
#include <vector>

#include <cstdlib>

#include "engine_state.h"

using namespace cc;

static thread_local std::string g_err;

int cc::set_err(int code, const char* what, hipError_t e) {
  char buf[512];
  if (e != hipSuccess)
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
  else
    snprintf(buf, sizeof buf, "%s", what);
  g_err = buf;
  return code;
}

static hipEvent_t take_event(cc_engine* e) {
  if (!e->ev_pool.empty()) {
    hipEvent_t ev = e->ev_pool.back();
    e->ev_pool.pop_back();
    return ev;
  }
  hipEvent_t ev = nullptr;
  // timing-only markers: no system-scope fence (cache writeback + invalidate) when the event is recorded, which
  // cost the timed c2 step ~0.15 ms (2.28 vs 2.13 ms with the markers off); elapsed times stay exact
  if (hipEventCreateWithFlags(&ev, hipEventDisableSystemFence) != hipSuccess) (void)hipEventCreate(&ev);
  return ev;
}

static void mark_fn(void* ctx, int k, int begin, hipStream_t st) {
  cc_engine* e = (cc_engine*)ctx;
  // a value-only engine enqueues nothing between one kernel's end marker and the next kernel's begin marker inside a
  // batch, so that end event doubles as the begin event (4 events per sub-batch instead of 6: each recorded event
  // is a packet on the stream the timed step pays for)
  if (begin && !e->ext && e->last_end && e->last_end_st == st) {
    e->open_ev[k] = e->last_end;
    e->open_shared[k] = true;
    e->last_end = nullptr;
    return;
  }
  hipEvent_t ev = take_event(e);
  (void)hipEventRecord(ev, st);
  if (begin) {
    e->open_ev[k] = ev;
    e->open_shared[k] = false;
    e->last_end = nullptr;
  } else {
    e->pending.push_back({k, e->open_ev[k], ev, e->open_shared[k]});
    e->open_ev[k] = nullptr;
    e->last_end = ev;
    e->last_end_st = st;
  }
}

static Marker marker_of(cc_engine* e) { return Marker{e->prof_on ? &mark_fn : nullptr, e}; }

static void drain_profile(cc_engine* e) {
  for (auto& p : e->pending) {
    float ms = 0.f;
    if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      e->prof_ms[p.kernel] += ms;
      e->prof_n[p.kernel] += 1;
    }
    if (!p.shared_a) e->ev_pool.push_back(p.a);  // (a shared begin event is an earlier entry's end event)
    e->ev_pool.push_back(p.b);
  }
  e->pending.clear();
}

static void free_all(cc_engine* e) {
  drain_profile(e);
  for (hipEvent_t ev : e->ev_pool) (void)hipEventDestroy(ev);
  e->ev_pool.clear();
  void* ptrs[] = {e->d_inst_res, e->d_res_type, e->d_val_meta,   e->d_val_v,     e->d_st_meta, e->d_st_ab,
                  e->d_err,      e->d_last_index, e->d_cpos,    e->d_ttab,      e->d_rst_status, e->d_rst_value,
                  e->d_tbl_key,  e->d_tbl_word, e->d_tbl_val,   e->d_tbl_ci,    e->d_tbl_ins,    e->d_xrec,
                  e->d_hot,       e->d_hot_n,     e->d_hot_cand,   e->d_hot_cand_n, e->d_hot_meta, e->d_hot_rpre,   e->d_hot_rstart,
                  e->d_hot_len,  e->d_hot_cond, e->d_hot_agg,   e->d_hot_s0,    e->d_hot_samp, e->d_sb_kind,    e->d_inst_id,
                  e->d_coord,    e->d_clock,    e->d_ev_cnt,    e->d_row_of,    e->d_ev_loc,     e->d_tile_sum,
                  e->d_tile_off, e->d_arena,    e->d_ev_perm,   e->d_arena_n,   e->d_ev_total,
                  e->d_bar,      e->d_bar_n,    e->d_mw_peak,   e->d_mw_drop,   e->d_mw_ctl,    e->d_mw_cgen, e->d_cset, e->d_cset_full, e->d_tbl_claim, e->d_lvl_at, e->d_half_count,
                  e->d_tbl_dl,   e->d_map_row,  e->d_ttl_seen, e->d_val_live, e->d_val_wrow,
                  e->d_leak,     e->d_leak_n,   e->d_ev_bucket, e->d_ev_ccnt, e->d_rst_msz, e->d_hot_msz, e->d_msize,
                  e->d_mpcap,    e->d_msz_tcnt, e->d_msz_list, e->d_msz_list_n, e->d_msm,     e->d_mbig,     e->d_msmall,  e->d_msm_left, e->d_span_cut,
                  e->d_sm_ctl,   e->d_sm_key,   e->d_sm_key2,  e->d_sm_val,   e->d_sm_val2,    e->d_sm_seg, e->d_sm_temp, e->d_sm_pay,
                  e->d_szq,      e->d_szq_n,    e->d_mrec,    e->d_bar_rows, e->d_fb,
                  e->d_cvq,      e->d_cvq_n,    e->d_isc,     e->d_isc2,     e->d_mfirst,     e->d_maynull, e->d_cv_rtemp,
                  e->d_cvset,    e->d_cvcnt,    e->d_cvev_key, e->d_cvev_key2, e->d_cvev_val, e->d_cvev_val2, e->d_cvev_ctl,
                  e->d_cvseg,    e->d_cvtemp,   e->d_clrq,    e->d_clrq_n,   e->d_clr_keys,   e->d_clr_keys2, e->d_clr_off,
                  e->d_clr_base, e->d_clr_eend, e->d_clr_temp, e->d_tbl_ep, e->d_clr_scan, e->d_clr_stemp, e->d_clr_btab, e->d_sm_cseg, e->d_cvbloom};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (void*& p : e->hw_buf)
    if (p) (void)hipFree(p), p = nullptr;
  if (e->d_hh_key) (void)hipFree(e->d_hh_key);
  if (e->d_hh_val) (void)hipFree(e->d_hh_val);
  if (e->h_pin) (void)hipHostFree(e->h_pin);
  if (e->d_ckpt) (void)hipFree(e->d_ckpt);
  if (e->side_st) (void)hipStreamSynchronize(e->side_st);
  void* alt[] = {e->sm_alt.key, e->sm_alt.key2, e->sm_alt.val, e->sm_alt.val2, e->sm_alt.pay, e->sm_alt.cseg};
  for (void* p : alt)
    if (p) (void)hipFree(p);
  for (hipEvent_t ev : {e->ev_prep, e->ev_rep[0], e->ev_rep[1], e->ev_rb})
    if (ev) (void)hipEventDestroy(ev);
  if (e->side_st) (void)hipStreamDestroy(e->side_st);
  if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
}

constexpr uint64_t kLeakCap = 1u << 20;  // leak log entries between drains (16 MiB)

// The leak log with room for `need` entries past those already drained (an empty log is reallocated).
static int ensure_leak(cc_engine* e, uint64_t need) {
  if (!e->d_leak_n) {
    hipError_t x = hipMalloc(&e->d_leak_n, sizeof(unsigned long long));
    if (x == hipSuccess) x = hipMemset(e->d_leak_n, 0, sizeof(unsigned long long));
    if (x != hipSuccess) return set_err(CC_ERR_HIP, "leak log counter", x);
  }
  if (e->d_leak && e->leak_cap >= need) return CC_OK;
  if (e->d_leak) {
    int rc = drain_leaks(e);
    if (rc) return rc;
    (void)hipFree(e->d_leak);
    e->d_leak = nullptr;
  }
  const uint64_t cap = std::max<uint64_t>(need, kLeakCap);
  hipError_t x = hipMalloc(&e->d_leak, sizeof(LeakRec) * cap);
  if (x != hipSuccess) return set_err(CC_ERR_HIP, "hipMalloc leak log", x);
  e->leak_cap = cap;
  return CC_OK;
}

// The map event buffers (map_small.hip), sorted by hipcub: one event per map commit of a sub-batch at most; in TTL
// mode also one per expiry (at most one per commit that sees its key's timer fired, plus one per table entry).
static uint64_t small_cap_needed(const cc_engine* e) {
  return e->ttl_live ? 2 * e->sub_batch + e->map_entries : e->sub_batch;
}
static int launch_pending_replay(cc_engine* e, hipStream_t st);
static int wait_replay(cc_engine* e, int k, hipStream_t st);
static void free_sm_alt(cc_engine* e) {
  // (inside a batch: a replay not yet launched runs now, and every replay's exit marks fold into the snapshot on the
  // engine stream -- e->last_stream -- before the buffers go)
  if (e->last_stream) {
    (void)launch_pending_replay(e, e->last_stream);
    for (int k = 0; k < 2; ++k) (void)wait_replay(e, k, e->last_stream);
    (void)hipStreamSynchronize(e->last_stream);
  }
  if (e->side_st) (void)hipStreamSynchronize(e->side_st);
  e->rep_pending[0] = e->rep_pending[1] = false;
  void* alt[] = {e->sm_alt.key, e->sm_alt.key2, e->sm_alt.val, e->sm_alt.val2, e->sm_alt.pay, e->sm_alt.cseg};
  for (void* p : alt)
    if (p) (void)hipFree(p);
  e->sm_alt = cc_engine::SmSet{};
  e->sm_alt_on = false;
}
static int ensure_small(cc_engine* e) {
  const uint64_t cap = small_cap_needed(e);
  if (e->d_sm_key && e->sm_cap >= cap) return CC_OK;
  if (cap > 0xFFFFFFFFull) return set_err(CC_ERR_CAPACITY, "map event buffer beyond 2^32 entries");
  if (e->d_sm_key) {  // grown (TTL mode): the counters keep their buffer, the events are rebuilt per sub-batch
    free_sm_alt(e);  // (the side stream's replay is done with either set)
    void* ps[] = {e->d_sm_key, e->d_sm_key2, e->d_sm_val, e->d_sm_val2, e->d_sm_temp, e->d_sm_pay};
    for (void* p : ps) (void)hipFree(p);
    e->d_sm_key = e->d_sm_key2 = nullptr;
    e->d_sm_val = e->d_sm_val2 = nullptr;
    e->d_sm_pay = nullptr;
    e->d_sm_temp = nullptr;
  }
  const size_t tb = std::max<size_t>(small_sort_temp_bytes((uint32_t)cap), 256);
  hipError_t x = hipMalloc(&e->d_sm_key, 8 * cap);
  if (x == hipSuccess) x = hipMalloc(&e->d_sm_key2, 8 * cap);
  if (x == hipSuccess) x = hipMalloc(&e->d_sm_val, 4 * cap);
  if (x == hipSuccess) x = hipMalloc(&e->d_sm_val2, 4 * cap);
  if (x == hipSuccess) x = hipMalloc(&e->d_sm_pay, sizeof(EvPay) * cap);
  if (x == hipSuccess && !e->d_sm_seg) x = hipMalloc(&e->d_sm_seg, 4ull * (e->cfg.max_resources + 1));
  if (x == hipSuccess && !e->d_sm_cseg) x = hipMalloc(&e->d_sm_cseg, 4ull * (e->cfg.max_resources + 2));
  if (x == hipSuccess) x = hipMalloc(&e->d_sm_temp, tb);
  if (x != hipSuccess) return set_err(CC_ERR_HIP, "hipMalloc map events", x);
  e->sm_temp_bytes = tb;
  e->sm_cap = cap;
  return CC_OK;
}
// the second event-buffer set and the side stream of the overlapped small-map replay (engine_state.h SmSet)
static int ensure_sm_alt(cc_engine* e) {
  if (e->sm_alt_on) return CC_OK;
  const uint64_t cap = e->sm_cap;
  hipError_t x = hipSuccess;
  if (!e->side_st) x = hipStreamCreateWithFlags(&e->side_st, hipStreamNonBlocking);
  for (hipEvent_t* ev : {&e->ev_prep, &e->ev_rep[0], &e->ev_rep[1]})
    if (x == hipSuccess && !*ev) x = hipEventCreateWithFlags(ev, hipEventDisableTiming);
  if (x == hipSuccess) x = hipMalloc(&e->sm_alt.key, 8 * cap);
  if (x == hipSuccess) x = hipMalloc(&e->sm_alt.key2, 8 * cap);
  if (x == hipSuccess) x = hipMalloc(&e->sm_alt.val, 4 * cap);
  if (x == hipSuccess) x = hipMalloc(&e->sm_alt.val2, 4 * cap);
  if (x == hipSuccess) x = hipMalloc(&e->sm_alt.pay, sizeof(EvPay) * cap);
  if (x == hipSuccess) x = hipMalloc(&e->sm_alt.cseg, 4ull * (e->cfg.max_resources + 2));
  if (x != hipSuccess) return set_err(CC_ERR_HIP, "hipMalloc map events (second set)", x);
  e->sm_alt_on = true;
  return CC_OK;
}
// the deferred replay on the side stream, after what the engine stream has queued so far
static int launch_pending_replay(cc_engine* e, hipStream_t st) {
  if (!e->pend) return CC_OK;
  e->pend = false;
  HIPCHECK(hipEventRecord(e->ev_prep, st));
  HIPCHECK(hipStreamWaitEvent(e->side_st, e->ev_prep, 0));
  if (launch_small_replay_kernel(e->pend_sa, e->side_st)) return set_err(CC_ERR_HIP, "small-map replay launch", hipGetLastError());
  HIPCHECK(hipEventRecord(e->ev_rep[e->pend_set], e->side_st));
  e->rep_pending[e->pend_set] = true;
  return CC_OK;
}
// the engine stream waits for the side-stream replay of event-buffer set k, then folds its exit marks into the
// d_msmall snapshot (common.h, the small-map window invariant: the only place a replay's result reaches the flags)
static int wait_replay(cc_engine* e, int k, hipStream_t st) {
  if (!e->rep_pending[k]) return CC_OK;
  HIPCHECK(hipStreamWaitEvent(st, e->ev_rep[k], 0));
  e->rep_pending[k] = false;
  if (launch_small_fold(e->d_msm_left + (size_t)k * e->cfg.max_resources, e->d_msmall, e->cfg.max_resources, st))
    return set_err(CC_ERR_HIP, "small-map fold launch", hipGetLastError());
  return CC_OK;
}
// the engine stream waits for the side stream's replays (before barrier rows, timers, and the batch's end)
static int join_replay(cc_engine* e, hipStream_t st) {
  {
    int rc = launch_pending_replay(e, st);
    if (rc) return rc;
  }
  for (int k = 0; k < 2; ++k) {
    int rc = wait_replay(e, k, st);
    if (rc) return rc;
  }
  return CC_OK;
}

// the cleared maps' size scan (map_clear.hip): one element per map event, sized with the event buffer
static int ensure_clr_scan(cc_engine* e) {
  if (e->d_clr_scan && e->clr_scan_cap >= e->sm_cap) return CC_OK;
  if (e->d_clr_scan) (void)hipFree(e->d_clr_scan);
  if (e->d_clr_stemp) (void)hipFree(e->d_clr_stemp);
  e->d_clr_scan = e->d_clr_stemp = nullptr;
  const size_t tb = std::max<size_t>(clr_scan_temp_bytes((uint32_t)e->sm_cap), 256);
  hipError_t x = hipMalloc(&e->d_clr_scan, clr_scan_bytes_per_event() * e->sm_cap);
  if (x == hipSuccess) x = hipMalloc(&e->d_clr_stemp, tb);
  if (x != hipSuccess) return set_err(CC_ERR_HIP, "hipMalloc clear size scan", x);
  e->clr_scan_cap = e->sm_cap;
  e->clr_stemp_bytes = tb;
  return CC_OK;
}

// containsValue in the stream (map_cv.hip): the batch's in-stream rows sorted (device) and copied to the host, which
// cuts each sub-batch's slice of them.
constexpr uint32_t kCvMaxRows = 1u << 21;  // in-stream containsValue rows per sub-batch (a denser run shortens it)
static int cv_rows(cc_engine* e, uint32_t n2, hipStream_t st) {
  e->isc_rows.clear();
  if (n2 == 0) return CC_OK;
  const size_t need = std::max<size_t>(cv_rows_temp_bytes(e->cvq_cap), 256);
  if (!e->d_isc2 || need > e->cv_rtemp_bytes) {
    if (e->d_isc2) HIPCHECK(hipFree(e->d_isc2));
    if (e->d_cv_rtemp) HIPCHECK(hipFree(e->d_cv_rtemp));
    e->d_isc2 = nullptr;
    e->d_cv_rtemp = nullptr;
    HIPCHECK(hipMalloc(&e->d_isc2, sizeof(uint32_t) * e->cvq_cap));
    HIPCHECK(hipMalloc(&e->d_cv_rtemp, need));
    e->cv_rtemp_bytes = need;
  }
  if (cv_sort_rows(e->d_isc, e->d_isc2, n2, e->d_cv_rtemp, e->cv_rtemp_bytes, st))
    return set_err(CC_ERR_HIP, "containsValue row sort", hipGetLastError());
  e->isc_rows.resize(n2);
  HIPCHECK(hipMemcpyAsync(e->isc_rows.data(), e->d_isc2, sizeof(uint32_t) * n2, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  return CC_OK;
}
// clears in the stream (map_clear.hip): the batch's list sorted by (map, row) with per-map offsets on the device; the
// host keeps the rows of any map cleared 128 times or more (a sub-batch holds at most 127 clears of one map)
static int clr_rows(cc_engine* e, uint32_t n, const cc_batch* c, hipStream_t st) {
  e->clr_n = n;
  e->clr_heavy.clear();
  if (n == 0) return CC_OK;
  ClrBatchArgs cb{};
  cb.rows = e->d_clrq;
  cb.n = n;
  cb.inst = c->inst;
  cb.inst_res = e->d_inst_res;
  cb.keys = e->d_clr_keys;
  cb.keys2 = e->d_clr_keys2;
  cb.off = e->d_clr_off;
  cb.R = e->cfg.max_resources;
  cb.temp = e->d_clr_temp;
  cb.temp_bytes = e->clr_temp_bytes;
  if (launch_clr_batch(cb, st)) return set_err(CC_ERR_HIP, "clear list launch", hipGetLastError());
  if (n >= 128) {
    std::vector<uint64_t> keys(n);
    HIPCHECK(hipMemcpyAsync(keys.data(), e->d_clr_keys2, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    for (uint32_t a = 0; a < n;) {
      uint32_t b = a;
      while (b < n && (keys[b] >> 32) == (keys[a] >> 32)) ++b;
      if (b - a >= 128) {
        std::vector<uint32_t> rows(b - a);
        for (uint32_t q = a; q < b; ++q) rows[q - a] = (uint32_t)keys[q];
        e->clr_heavy.push_back(std::move(rows));
      }
      a = b;
    }
  }
  return CC_OK;
}

// the operand set (sized for kCvMaxRows operands) and the event buffers (two events per commit, one per query)
constexpr uint32_t kCvBloomMaxBits = 25;  // the operand filter: ~16 bits per operand, 2^16 .. 2^25 bits
static int ensure_cv(cc_engine* e) {
  if (e->d_cvset) return CC_OK;
  const uint32_t sc = 2 * kCvMaxRows;
  const uint64_t ec = 2ull * e->sub_batch + kCvMaxRows;
  if (ec > 0xFFFFFFFFull) return set_err(CC_ERR_CAPACITY, "containsValue event buffer beyond 2^32 entries");
  const size_t tb = std::max<size_t>(cv_sort_temp_bytes((uint32_t)ec), 256);
  hipError_t x = hipMalloc(&e->d_cvset, sizeof(CvEnt) * sc);
  if (x == hipSuccess) x = hipMalloc(&e->d_cvcnt, sizeof(uint32_t) * sc);
  if (x == hipSuccess) x = hipMalloc(&e->d_cvseg, sizeof(uint32_t) * (sc + 1));
  if (x == hipSuccess) x = hipMalloc(&e->d_cvev_key, 8 * ec);
  if (x == hipSuccess) x = hipMalloc(&e->d_cvev_key2, 8 * ec);
  if (x == hipSuccess) x = hipMalloc(&e->d_cvev_val, 4 * ec);
  if (x == hipSuccess) x = hipMalloc(&e->d_cvev_val2, 4 * ec);
  if (x == hipSuccess) x = hipMalloc(&e->d_cvev_ctl, sizeof(uint32_t) * 2);
  if (x == hipSuccess) x = hipMalloc(&e->d_cvtemp, tb);
  if (x == hipSuccess) x = hipMalloc(&e->d_cvbloom, (1ull << kCvBloomMaxBits) / 8);
  if (x != hipSuccess) return set_err(CC_ERR_HIP, "hipMalloc containsValue buffers", x);
  e->cvset_cap = sc;
  e->cvev_cap = (uint32_t)ec;
  e->cvtemp_bytes = tb;
  return CC_OK;
}

// Extended staging columns (maps, coordination, value events); with `coord`, the coordination blocks and the
// event buffers.  Allocated on first need (engine creation or the first coordination resource).
static int ensure_ext(cc_engine* e, bool coord) {
  auto alloc = [&](void** p, size_t bytes) -> int {
    if (*p) return CC_OK;
    hipError_t x = hipMalloc(p, bytes);
    if (x != hipSuccess) return set_err(CC_ERR_HIP, "hipMalloc (extended staging)", x);
    return CC_OK;
  };
  int rc = CC_OK;
  if (!e->ext) {
    if ((rc = alloc((void**)&e->d_xrec, sizeof(XRec) * e->sub_batch))) return rc;
    e->ext = true;
  }
  if (coord && !e->coord_on) {
    // coordination records carry their instance id (k_part_ext's id plane: 8 more LDS bytes per chunk commit), so the
    // partition must still fit with it; checked before anything is allocated or switched on
    if (part_ext_chunk(e->sbq_base(), e->map_bits != 0, true) == 0)
      return set_err(CC_ERR_CAPACITY, "map_capacity and max_resources together leave no room in the partition for "
                                      "coordination resources / value events");
    const uint64_t slots = (uint64_t)e->sb << kSbShift;
    e->arena_cap = std::max<uint64_t>(e->cfg.max_events, 1);
    if ((rc = alloc((void**)&e->d_coord, coord_block(e->coord_cap) * slots)) ||
        (rc = alloc((void**)&e->d_ev_cnt, sizeof(uint16_t) * e->sub_batch)) ||
        (rc = alloc((void**)&e->d_row_of, sizeof(uint32_t) * e->sub_batch)) ||
        (rc = alloc((void**)&e->d_ev_loc, sizeof(uint32_t) * e->sub_batch)) ||
        (rc = alloc((void**)&e->d_tile_sum, sizeof(uint32_t) * e->max_tiles)) ||
        (rc = alloc((void**)&e->d_tile_off, sizeof(uint64_t) * e->max_tiles)) ||
        (rc = alloc((void**)&e->d_arena, sizeof(EvRec) * e->arena_cap)) ||
        (rc = alloc((void**)&e->d_ev_perm, sizeof(uint32_t) * e->arena_cap)) ||
        (rc = alloc((void**)&e->d_ev_bucket, sizeof(EvRec) * e->arena_cap)) ||
        (rc = alloc((void**)&e->d_ev_ccnt, sizeof(uint32_t) * ev_chunk_cap(e->arena_cap) * e->max_tiles)) ||
        (rc = alloc((void**)&e->d_arena_n, sizeof(unsigned long long))) ||
        (rc = alloc((void**)&e->d_ev_total, sizeof(unsigned long long))) ||
        (rc = ensure_leak(e, kLeakCap)))
      return rc;
    hipError_t x = hipMemset(e->d_coord, 0, coord_block(e->coord_cap) * slots);
    if (x != hipSuccess) return set_err(CC_ERR_HIP, "memset coord", x);
    e->coord_on = true;
    // quarter buckets for k_apply_coord when the extended partition's LDS still fits with them
    e->quarter = part_ext_chunk(e->sbq_base() + 4 * e->sb, e->map_bits != 0, true) != 0;
  }
  return CC_OK;
}

static bool is_coord(uint32_t type) {
  return type == CC_RES_LOCK || type == CC_RES_ELECTION || type == CC_RES_GROUP || type == CC_RES_QUEUE;
}

extern "C" int cc_abi_version(void) { return CC_ABI_VERSION; }
extern "C" const char* cc_last_error(void) { return g_err.c_str(); }

extern "C" int cc_engine_create(const cc_config* cfg, cc_engine** out) {
  if (!cfg || !out) return set_err(CC_ERR_INVALID, "null config");
  if (cfg->max_resources == 0 || cfg->max_resources > (uint32_t)kMaxSb << kSbShift)
    return set_err(CC_ERR_CAPACITY, "max_resources must be in [1, 131072]");
  if (cfg->max_instances == 0 || cfg->max_batch == 0) return set_err(CC_ERR_INVALID, "max_instances/max_batch must be > 0");
  const uint32_t ccap = cfg->coord_cap ? cfg->coord_cap : kCoordCapDefault;
  if (ccap < kCoordCapDefault || ccap > kCoordCapMax || (ccap & (ccap - 1)))
    return set_err(CC_ERR_INVALID, "coord_cap must be 0 or a power of two in [64, 65536]");
  cc_engine* e = new cc_engine();
  e->cfg = *cfg;
  e->coord_cap = ccap;
  e->device = cfg->device;
  hipError_t he = hipSetDevice(e->device);
  if (he != hipSuccess) { delete e; return set_err(CC_ERR_HIP, "hipSetDevice", he); }
  e->sb = (cfg->max_resources + (1u << kSbShift) - 1) >> kSbShift;
  e->sb_bits = 0;
  while ((1u << e->sb_bits) < e->sb) ++e->sb_bits;
  if (cfg->map_capacity) {  // regions of 2048 entries, load <= 1/2
    if (cfg->map_capacity > (uint64_t)kMaxMapSb * kMapRegion / 2) {
      delete e;
      return set_err(CC_ERR_CAPACITY, "map_capacity must be <= 2097152");
    }
    e->map_bits = 1;
    while (((uint64_t)kMapRegion << e->map_bits) < 2 * cfg->map_capacity) ++e->map_bits;
    e->map_entries = (uint64_t)kMapRegion << e->map_bits;
    // the extended partition's per-bucket LDS counters must fit (with the instance-id plane when value events turn
    // the coordination path on from the start; a later coordination resource is checked in ensure_ext)
    if (part_ext_chunk(e->sbq_base(), true, (cfg->flags & CC_CFG_VALUE_EVENTS) != 0) == 0) {
      delete e;
      return set_err(CC_ERR_CAPACITY, "map_capacity and max_resources together exceed the partition's bucket capacity");
    }
  }
  // sub-batch: a multiple of the partition tile (keeps every sub-batch start 16 KiB-aligned).  The value-only pipeline
  // (value_path.hip: 8,192-commit tiles, kV3MaxTiles of them) takes up to 24 Mi commits per sub-batch, 24 Mi by default:
  // 100M commits in 4 sub-batches instead of 6, 12 launches per step instead of 18.  The extended path (maps,
  // coordination, value events; kMaxTiles tiles of kTile) stays at 16 Mi: sub_ext, used once the engine turns ext.
  uint64_t sub = cfg->sub_batch ? cfg->sub_batch : (uint64_t)kV3MaxTiles * kV3Tile;
  sub = std::min<uint64_t>(sub, cfg->max_batch);
  sub = (sub + kTile - 1) / kTile * kTile;
  sub = std::min<uint64_t>(sub, (uint64_t)kV3MaxTiles * kV3Tile);
  static_assert((uint64_t)kV3MaxTiles * kV3Tile >= (uint64_t)kMaxTiles * kTile, "the value-only sub-batch is the larger");
  static_assert(((uint64_t)kV3MaxTiles * kV3Tile) % kTile == 0, "a multiple of the partition tile");
  e->sub_batch = sub;
  e->sub_ext = std::min<uint64_t>(sub, (uint64_t)kMaxTiles * kTile);
  e->max_tiles = (sub + kTile - 1) / kTile;

  const uint64_t slots = (uint64_t)e->sb << kSbShift;
  e->res_type.assign(slots, CC_RES_NONE);
  e->inst_res.assign(cfg->max_instances, kNoRes);
  e->inst_id.assign(cfg->max_instances, 0);
  e->inst_client.assign(cfg->max_instances, 0);
  e->res_id.assign(slots, 0);
  e->res_key.assign(slots, 0);
  e->res_has_key.assign(slots, 0);
  e->res_zombie.assign(slots, 0);
  e->used_res.reset(cfg->max_resources);
  e->used_inst.reset(cfg->max_instances);
  auto fail = [&](const char* what, hipError_t x) {
    free_all(e);
    delete e;
    return set_err(CC_ERR_HIP, what, x);
  };
#define ALLOC(p, bytes)                                   \
  do {                                                    \
    hipError_t x = hipMalloc((void**)&(p), (bytes));      \
    if (x != hipSuccess) return fail("hipMalloc " #p, x); \
  } while (0)
  ALLOC(e->d_inst_res, sizeof(uint32_t) * cfg->max_instances);
  ALLOC(e->d_res_type, slots);
  ALLOC(e->d_val_meta, sizeof(uint32_t) * slots);
  ALLOC(e->d_val_v, sizeof(uint64_t) * slots);
  if (cfg->flags & CC_CFG_VALUE_RETAINED) {
    ALLOC(e->d_val_live, sizeof(uint64_t) * slots);
    ALLOC(e->d_val_wrow, sizeof(unsigned long long) * slots);
  }
  ALLOC(e->d_st_meta, sizeof(uint32_t) * (e->sub_batch + kPT));  // + dummy rows for unconditional stores
  ALLOC(e->d_st_ab, sizeof(u64x2) * (e->sub_batch + kPT));
  ALLOC(e->d_cpos, sizeof(uint16_t) * e->sub_batch);
  // (value-only engines: 2 tiles of 8192 per 16384 and 128-slot buckets -> 2 x (2 sb + 1) entries per 16384 commits)
  ALLOC(e->d_ttab, sizeof(uint16_t) * e->max_tiles * (e->sbq_base() + 4 * e->sb + 2));
  if (e->map_bits) {
    ALLOC(e->d_tbl_key, sizeof(uint64_t) * e->map_entries);
    ALLOC(e->d_mrec, sizeof(MRec) * e->sub_batch);
    ALLOC(e->d_tbl_word, sizeof(uint32_t) * e->map_entries);
    ALLOC(e->d_tbl_val, sizeof(uint64_t) * e->map_entries);
    ALLOC(e->d_tbl_ci, sizeof(uint64_t) * e->map_entries);
    ALLOC(e->d_tbl_ins, sizeof(uint64_t) * e->map_entries);
    ALLOC(e->d_hot, sizeof(HotKey) * kHotMax);
    ALLOC(e->d_hot_n, sizeof(uint32_t));
    ALLOC(e->d_hot_cand, sizeof(HotKey) * kHotMax);
    ALLOC(e->d_hot_meta, sizeof(uint32_t) * e->sub_batch);
    ALLOC(e->d_hot_cand_n, sizeof(uint32_t));
    ALLOC(e->d_mw_peak, sizeof(uint32_t) * cfg->max_resources);
    ALLOC(e->d_mw_drop, sizeof(uint64_t) * cfg->max_resources);
    ALLOC(e->d_mw_cgen, sizeof(uint64_t) * cfg->max_resources);
    e->cset_mask = std::max<uint64_t>(1u << 16, e->map_entries) - 1;  // (map_entries is a power of two)
    ALLOC(e->d_cset, sizeof(CsetEnt) * (e->cset_mask + 1));
    ALLOC(e->d_cset_full, sizeof(uint32_t));
    ALLOC(e->d_tbl_claim, sizeof(uint64_t) * e->map_entries);
    ALLOC(e->d_tbl_ep, e->map_entries);  // clears in the stream: hot entries' epochs (map_clear.hip)
    ALLOC(e->d_lvl_at, sizeof(unsigned long long) * kLvlSlots * cfg->max_resources);
    ALLOC(e->d_mw_ctl, sizeof(unsigned long long) * 64);
    ALLOC(e->d_msm, sizeof(SmallMap) * cfg->max_resources);
    ALLOC(e->d_mbig, sizeof(BigMap) * kBigSlots);
    ALLOC(e->d_msmall, (cfg->max_resources + 3) & ~3u);  // (padded to whole words: common.h mflag_or)
    ALLOC(e->d_msm_left, 3ull * cfg->max_resources);
    ALLOC(e->d_span_cut, sizeof(uint64_t));
    ALLOC(e->d_sm_ctl, sizeof(uint32_t) * 4);
    ALLOC(e->d_rst_msz, sizeof(uint32_t) * (e->sub_batch + 4 * kPT));
    ALLOC(e->d_hot_msz, sizeof(uint32_t) * (kHotMaxPieces + kHotMax) * (kHotPiece / 16));
    ALLOC(e->d_msize, sizeof(uint32_t) * cfg->max_resources);
    ALLOC(e->d_mpcap, sizeof(uint32_t) * cfg->max_resources);
    ALLOC(e->d_msz_tcnt, sizeof(uint32_t) * cfg->max_resources * e->max_tiles);  // [tile][map] counts
    ALLOC(e->d_msz_list, sizeof(uint4) * kMszListCap);
    ALLOC(e->d_msz_list_n, sizeof(uint32_t));
    ALLOC(e->d_tbl_dl, sizeof(uint64_t) * e->map_entries);
    ALLOC(e->d_map_row, sizeof(uint32_t) * e->sub_batch);
    ALLOC(e->d_hot_rpre, sizeof(uint32_t) * kHotMax * (kMaxTiles + 1));
    ALLOC(e->d_hot_rstart, sizeof(uint32_t) * kHotMax * kMaxTiles);
    ALLOC(e->d_hot_len, sizeof(uint32_t) * kHotMax);
    ALLOC(e->d_hot_cond, sizeof(uint32_t) * kHotMax);
    ALLOC(e->d_hot_agg, hot_agg_bytes());
    ALLOC(e->d_hot_s0, hot_s0_bytes());
    ALLOC(e->d_hot_samp, hot_samp_bytes());
  }
  ALLOC(e->d_rst_status, e->sub_batch + 4 * kPT);  // + dummy rows for unconditional result stores
  ALLOC(e->d_rst_value, sizeof(uint64_t) * (e->sub_batch + 4 * kPT));
  ALLOC(e->d_err, sizeof(uint32_t));
  {
    hipError_t x = hipHostMalloc((void**)&e->h_pin, 8 * sizeof(uint64_t), hipHostMallocDefault);
    if (x != hipSuccess) return fail("hipHostMalloc (counter readbacks)", x);
  }
  ALLOC(e->d_bar, sizeof(uint32_t) * kBarCap);
  ALLOC(e->d_bar_n, sizeof(uint32_t));
  ALLOC(e->d_ttl_seen, sizeof(uint32_t));
  ALLOC(e->d_last_index, sizeof(uint64_t));
  ALLOC(e->d_sb_kind, e->sb);
  ALLOC(e->d_inst_id, sizeof(uint64_t) * cfg->max_instances);
  ALLOC(e->d_clock, sizeof(uint64_t));
#undef ALLOC
  if ((he = hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking)) != hipSuccess) return fail("hipStreamCreate", he);
  e->last_stream = e->own_stream;
  if ((he = hipMemset(e->d_inst_res, 0xFF, sizeof(uint32_t) * cfg->max_instances)) != hipSuccess) return fail("memset", he);
  if ((he = hipMemset(e->d_res_type, 0, slots)) != hipSuccess) return fail("memset", he);
  if ((he = hipMemset(e->d_val_meta, 0, sizeof(uint32_t) * slots)) != hipSuccess) return fail("memset", he);
  if ((he = hipMemset(e->d_val_v, 0, sizeof(uint64_t) * slots)) != hipSuccess) return fail("memset", he);
  if (e->d_val_live) {
    if ((he = hipMemset(e->d_val_live, 0, sizeof(uint64_t) * slots)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_val_wrow, 0, sizeof(unsigned long long) * slots)) != hipSuccess) return fail("memset", he);
  }
  if ((he = hipMemset(e->d_err, 0, sizeof(uint32_t))) != hipSuccess) return fail("memset", he);
  if ((he = hipMemset(e->d_sb_kind, 0, e->sb)) != hipSuccess) return fail("memset", he);
  if ((he = hipMemset(e->d_clock, 0, sizeof(uint64_t))) != hipSuccess) return fail("memset", he);
  if ((he = hipMemset(e->d_last_index, 0, sizeof(uint64_t))) != hipSuccess) return fail("memset", he);
  e->sb_kind.assign(e->sb, 0);
  if (e->map_bits) {  // word 0 = empty entry
    if ((he = hipMemset(e->d_tbl_word, 0, sizeof(uint32_t) * e->map_entries)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_tbl_ci, 0, sizeof(uint64_t) * e->map_entries)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_tbl_ins, 0, sizeof(uint64_t) * e->map_entries)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_hot_n, 0, sizeof(uint32_t))) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_mw_peak, 0, sizeof(uint32_t) * cfg->max_resources)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_mw_drop, 0, sizeof(uint64_t) * cfg->max_resources)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_mw_cgen, 0, sizeof(uint64_t) * cfg->max_resources)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_cset, 0, sizeof(CsetEnt) * (e->cset_mask + 1))) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_cset_full, 0, sizeof(uint32_t))) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_tbl_claim, 0, sizeof(uint64_t) * e->map_entries)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_tbl_ep, 0, e->map_entries)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_lvl_at, 0xFF, sizeof(unsigned long long) * kLvlSlots * cfg->max_resources)) != hipSuccess)
      return fail("memset", he);
    if ((he = hipMemset(e->d_msize, 0, sizeof(uint32_t) * cfg->max_resources)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_mpcap, 0, sizeof(uint32_t) * cfg->max_resources)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_msm, 0, sizeof(SmallMap) * cfg->max_resources)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_mbig, 0, sizeof(BigMap) * kBigSlots)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_msmall, 0, cfg->max_resources)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_msm_left, 0, 3ull * cfg->max_resources)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_sm_ctl, 0, sizeof(uint32_t) * 4)) != hipSuccess) return fail("memset", he);
    if ((he = hipMemset(e->d_tbl_dl, 0, sizeof(uint64_t) * e->map_entries)) != hipSuccess) return fail("memset", he);
  }
  if ((he = hipDeviceSynchronize()) != hipSuccess) return fail("sync", he);
  // the stable rankings of k_part_scatter / k_apply_value need same-address LDS atomics of one wave
  // instruction to resolve in lane order: verify on this device before trusting any result
  if (launch_selfcheck(e->d_err, e->own_stream) != 0) return fail("selfcheck launch", hipGetLastError());
  uint32_t bad = 0;
  if ((he = hipMemcpyAsync(&bad, e->d_err, sizeof bad, hipMemcpyDeviceToHost, e->own_stream)) != hipSuccess ||
      (he = hipStreamSynchronize(e->own_stream)) != hipSuccess)
    return fail("selfcheck", he);
  if (bad) {
    free_all(e);
    delete e;
    return set_err(CC_ERR_STATE, "device self-check failed: LDS atomics are not lane-ordered on this device");
  }
  if ((he = hipMemset(e->d_err, 0, sizeof(uint32_t))) != hipSuccess) return fail("memset", he);
  if (e->map_bits || (cfg->flags & CC_CFG_VALUE_EVENTS)) {
    int rc = ensure_ext(e, (cfg->flags & CC_CFG_VALUE_EVENTS) != 0);
    if (rc) {
      free_all(e);
      delete e;
      return rc;
    }
  }
  *out = e;
  return CC_OK;
}

extern "C" int cc_engine_destroy(cc_engine* e) {
  if (!e) return CC_ERR_INVALID;
  (void)hipSetDevice(e->device);
  if (e->last_stream) (void)hipStreamSynchronize(e->last_stream);
  free_all(e);
  delete e;
  return CC_OK;
}

extern "C" void* cc_engine_stream(cc_engine* e) { return e ? (void*)e->own_stream : nullptr; }

static int check_device_err(cc_engine* e) {
  uint32_t err = 0;
  HIPCHECK(hipMemcpy(&err, e->d_err, sizeof err, hipMemcpyDeviceToHost));
  e->last_err_bits = err;  // (cc_apply_batch_host_prefix tells a full coordination collection from other failures)
  if (err) {
    HIPCHECK(hipMemset(e->d_err, 0, sizeof(uint32_t)));
    if (err & kErrTime) return set_err(CC_ERR_INVALID, "the time column must be non-decreasing within a batch");
    if (err & kErrMapOrder)
      return set_err(CC_ERR_STATE, "map containsValue: the answer depends on java.util.HashMap iteration order inside a "
                                   "bin that may have been a red-black tree bin, or on a table capacity the engine's "
                                   "bounds leave open (TTL mode)");
    if (err & kErrMapSize) return set_err(CC_ERR_STATE, "internal check: a map's tracked size differs from its table");
    if (err & kErrCvKey)
      return set_err(CC_ERR_STATE, "internal check: an in-stream containsValue event spans more than 2^40 log indices");
    if (err & kErrSmallFlag)
      return set_err(CC_ERR_STATE, "internal check (CC_DIAG): a map in the small-map window without its snapshot flag");
    if (err & kErrHandleHash)
      return set_err(CC_ERR_STATE, "a HANDLE map key's String.hashCode is not registered (cc_handle_hashes)");
    if (err & kErrSpan)
      return set_err(CC_ERR_STATE, "internal check: a sub-batch with map events spans 2^32 log indices (the index "
                                   "column must increase in log order)");
    if (err & kErrEvents) return set_err(CC_ERR_CAPACITY, "more events than the event stream / max_events holds");
    if (err & kErrCapacity)
      return set_err(CC_ERR_CAPACITY, "a fixed capacity was exceeded (map table region, leak log, event buffer)");
    if (err & kErrCoordFull)
      return set_err(CC_ERR_CAPACITY, "a coordination collection is full (coord_cap: lock queue, listeners, members, "
                                      "queue elements)");
    if (err & kErrUnsupported)
      return set_err(CC_ERR_UNSUPPORTED,
                     "batch contained an op this build does not apply on the GPU (AtomicValue Listen/Unlisten without "
                     "CC_CFG_VALUE_EVENTS; group "
                     "schedule) or published events with no event stream");
    return set_err(CC_ERR_STATE, "device-side check failed");
  }
  return CC_OK;
}

extern "C" int cc_sync(cc_engine* e) {
  if (!e) return CC_ERR_INVALID;
  HIPCHECK(hipSetDevice(e->device));
  HIPCHECK(hipStreamSynchronize(e->last_stream));
  if (e->applied_pending) {
    uint64_t li = 0;
    HIPCHECK(hipMemcpy(&li, e->d_last_index, sizeof li, hipMemcpyDeviceToHost));
    e->applied = std::max(e->applied, li);
    e->applied_pending = false;
  }
  return check_device_err(e);
}

// Registry updates are control-plane (the reference runs them as log commands too: ResourceManager.java:77-235);
// the host orders them against batches, so they first drain the stream the last batch ran on.
int cc::sync_streams(cc_engine* e) {
  HIPCHECK(hipSetDevice(e->device));
  HIPCHECK(hipStreamSynchronize(e->last_stream));
  return CC_OK;
}

int cc::quiesce(cc_engine* e) {
  int rc = sync_streams(e);
  if (rc) return rc;
  return e->dev_dirty() ? dev_flush(e) : CC_OK;
}

// queued registry writes (cc_engine::dev_pend): fills and copies per destination array, coalesced when contiguous
static void dev_fill(cc_engine* e, void* base, uint64_t off, int val, uint64_t bytes) {
  if (!bytes) return;
  auto& v = e->dev_pend[base];
  uint8_t* dst = (uint8_t*)base + off;
  if (!v.empty() && v.back().fill == val && v.back().dst + v.back().bytes == dst) {
    v.back().bytes += bytes;
    return;
  }
  v.push_back(cc_engine::DevWrite{dst, bytes, val, {}});
}
static void dev_copy(cc_engine* e, void* base, uint64_t off, const void* src, uint64_t bytes) {
  if (!bytes) return;
  auto& v = e->dev_pend[base];
  uint8_t* dst = (uint8_t*)base + off;
  const uint8_t* s = (const uint8_t*)src;
  if (!v.empty() && v.back().fill < 0 && v.back().dst + v.back().bytes == dst) {
    v.back().data.insert(v.back().data.end(), s, s + bytes);
    v.back().bytes += bytes;
    return;
  }
  v.push_back(cc_engine::DevWrite{dst, bytes, -1, std::vector<uint8_t>(s, s + bytes)});
}
static void mark_dirty(uint64_t& lo, uint64_t& hi, uint64_t a, uint64_t b) {
  lo = std::min(lo, a);
  hi = std::max(hi, b);
}

int cc::dev_flush(cc_engine* e) {
  // A run of consecutive fills of one value is written as its merged intervals (order inside such a run does not
  // matter; a copy or another value ends it): resources created one by one land in type-pure 64-slot groups, so their
  // blocks are not adjacent in creation order, and each had cost a fill of its own (~98K fills for c5's 32,768).
  for (auto& kv : e->dev_pend) {
    auto& v = kv.second;
    for (size_t a = 0; a < v.size();) {
      if (v[a].fill < 0) {
        HIPCHECK(hipMemcpy(v[a].dst, v[a].data.data(), v[a].bytes, hipMemcpyHostToDevice));
        ++a;
        continue;
      }
      size_t b = a + 1;
      while (b < v.size() && v[b].fill == v[a].fill) ++b;
      std::vector<std::pair<uint8_t*, uint64_t>> iv;  // [dst, dst + bytes)
      for (size_t k = a; k < b; ++k) iv.push_back({v[k].dst, v[k].bytes});
      std::sort(iv.begin(), iv.end());
      for (size_t k = 0; k < iv.size();) {
        uint8_t* lo = iv[k].first;
        uint8_t* hi = lo + iv[k].second;
        for (++k; k < iv.size() && iv[k].first <= hi; ++k) hi = std::max(hi, iv[k].first + iv[k].second);
        HIPCHECK(hipMemset(lo, v[a].fill, (size_t)(hi - lo)));
      }
      a = b;
    }
  }
  e->dev_pend.clear();
  for (const auto& r : e->big_rel) {  // (the new maps' slots: a big model of the map deleted from one is freed)
    if (launch_big_release(e->d_mbig, r.first, r.second, nullptr)) return set_err(CC_ERR_HIP, "big-model release", hipGetLastError());
    HIPCHECK(hipStreamSynchronize(nullptr));
  }
  e->big_rel.clear();
  if (e->res_dirty_hi) {
    HIPCHECK(hipMemcpy(e->d_res_type + e->res_dirty_lo, e->res_type.data() + e->res_dirty_lo,
                       e->res_dirty_hi - e->res_dirty_lo, hipMemcpyHostToDevice));
    e->res_dirty_lo = ~0ull;
    e->res_dirty_hi = 0;
  }
  if (e->inst_dirty_hi) {
    const uint64_t lo = e->inst_dirty_lo, n = e->inst_dirty_hi - lo;
    HIPCHECK(hipMemcpy(e->d_inst_res + lo, e->inst_res.data() + lo, sizeof(uint32_t) * n, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(e->d_inst_id + lo, e->inst_id.data() + lo, sizeof(uint64_t) * n, hipMemcpyHostToDevice));
    e->inst_dirty_lo = ~0ull;
    e->inst_dirty_hi = 0;
  }
  if (e->sb_kind_dirty) {
    HIPCHECK(hipMemcpy(e->d_sb_kind, e->sb_kind.data(), e->sb, hipMemcpyHostToDevice));
    e->sb_kind_dirty = false;
  }
  return CC_OK;
}

int cc::create_range(cc_engine* e, uint32_t first, uint32_t count, uint32_t type) {
  if (is_keyed(type) && !e->map_bits) return set_err(CC_ERR_CAPACITY, "map and set resources need cc_config.map_capacity > 0");
  if (type < CC_RES_VALUE || type > CC_RES_MULTIMAP) return set_err(CC_ERR_INVALID, "unknown resource type");
  if (type == CC_RES_SET) e->has_sets = true;
  if (type == CC_RES_VALUE) e->has_values = true;
  if (type == CC_RES_MULTIMAP) {
    e->has_mmaps = true;
    int rc = ensure_leak(e, kLeakCap);
    if (rc) return rc;
  }
  const uint64_t end = (uint64_t)first + count;
  if (end > e->cfg.max_resources) return set_err(CC_ERR_CAPACITY, "resource slot out of range");
  for (uint64_t s = first; s < end; ++s) {
    if (e->res_type[s] != CC_RES_NONE) return set_err(CC_ERR_INVALID, "resource slot already in use");
  }
  int rc = sync_streams(e);  // (its device writes are queued: dev_flush before the next device work)
  if (rc) return rc;
  const bool value_events = (e->cfg.flags & CC_CFG_VALUE_EVENTS) != 0;
  if (is_coord(type) && (rc = ensure_ext(e, true))) return rc;
  for (uint64_t s = first; s < end; ++s) {
    e->res_type[s] = (uint8_t)type;
    if (is_coord(type) || (type == CC_RES_VALUE && value_events)) e->sb_kind[s >> kSbShift] = 1;
    e->res_has_key[s] = 0;
    e->res_zombie[s] = 0;
    e->used_res.set(s);
  }
  mark_dirty(e->res_dirty_lo, e->res_dirty_hi, first, end);
  e->sb_kind_dirty = true;
  if (e->coord_on)
    dev_fill(e, e->d_coord, (uint64_t)first * coord_block(e->coord_cap), 0, coord_block(e->coord_cap) * (uint64_t)count);
  if (is_keyed(type)) {  // a new HashMap: capacity 16, no history
    dev_fill(e, e->d_mw_peak, sizeof(uint32_t) * first, 0, sizeof(uint32_t) * count);
    dev_fill(e, e->d_mw_drop, sizeof(uint64_t) * first, 0, sizeof(uint64_t) * count);
    // (d_mw_cgen is not reset: a reused slot must not see the compacted keys of the map deleted from it, whose delete
    // bumped the generation)
    dev_fill(e, e->d_msize, sizeof(uint32_t) * first, 0, sizeof(uint32_t) * count);
    dev_fill(e, e->d_mpcap, sizeof(uint32_t) * first, 0, sizeof(uint32_t) * count);
    {  // the capacity-level timeline: level 0 from the start, none of the others reached
      std::vector<unsigned long long> la((size_t)kLvlSlots * count, ~0ull);
      for (uint32_t k = 0; k < count; ++k) la[(size_t)k * kLvlSlots] = 0;
      dev_copy(e, e->d_lvl_at, sizeof(unsigned long long) * kLvlSlots * first, la.data(), sizeof(unsigned long long) * la.size());
    }
    // MapState's table followed key by key while small (map_small.hip); sets / multimaps have no order-dependent op
    std::vector<SmallMap> sm(count);
    const bool is_map = type == CC_RES_MAP;
    for (auto& x : sm) x.flags = is_map ? kSmIn : 0u;  // (TTL mode too: its commit + expiry events are replayed)
    dev_copy(e, e->d_msm, sizeof(SmallMap) * first, sm.data(), sizeof(SmallMap) * count);
    if (e->d_mbig) e->big_rel.push_back({first, count});
    dev_fill(e, e->d_msmall, first, is_map ? 1 : 0, count);
    if (is_map && !e->ttl_live) {
      e->small_live = true;
      // the count of maps still small (ctl[1], k_small_count) is stale until the next sub-batch's recount: a
      // nonzero one keeps the small-map events on for that sub-batch even if it emits none
      const uint32_t pending = 1;
      dev_copy(e, e->d_sm_ctl, sizeof(uint32_t), &pending, sizeof pending);
    }
  }
  // fresh state: AtomicValueState() {value = null; current = null}
  dev_fill(e, e->d_val_meta, sizeof(uint32_t) * first, 0, sizeof(uint32_t) * count);
  dev_fill(e, e->d_val_v, sizeof(uint64_t) * first, 0, sizeof(uint64_t) * count);
  if (e->d_val_live) dev_fill(e, e->d_val_live, sizeof(uint64_t) * first, 0, sizeof(uint64_t) * count);
  return CC_OK;
}

// Slot-level registration (the host picked the slot): the resource id is the slot number, as in the oracle's
// orc_resource_create; such a resource has no key (get/create never find it).
static int create_slots(cc_engine* e, uint32_t first, uint32_t count, uint32_t type) {
  int rc = create_range(e, first, count, type);
  if (rc) return rc;
  for (uint64_t s = first; s < (uint64_t)first + count; ++s) {
    e->res_id[s] = s;
    e->res_by_id[s] = (uint32_t)s;
  }
  return CC_OK;
}

extern "C" int cc_resource_create(cc_engine* e, uint32_t slot, uint32_t type) {
  if (!e) return CC_ERR_INVALID;
  return create_slots(e, slot, 1, type);
}

extern "C" int cc_resource_create_range(cc_engine* e, uint32_t first, uint32_t count, uint32_t type) {
  if (!e) return CC_ERR_INVALID;
  return create_slots(e, first, count, type);
}

extern "C" int cc_resource_delete(cc_engine* e, uint32_t slot) {
  if (!e || slot >= e->cfg.max_resources || e->res_type[slot] == CC_RES_NONE) return set_err(CC_ERR_INVALID, "unknown resource slot");
  if (e->res_zombie[slot]) return set_err(CC_ERR_INVALID, "resource slot was removed by a failed deleteResource");
  return delete_slot(e, slot);
}

// The device leak log into the per-slot host lists (the engine is quiesced).  An overflow was already reported by
// the batch that caused it (kErrCapacity); the entries past the log's end are lost.
int cc::drain_leaks(cc_engine* e) {
  if (!e->d_leak_n) return CC_OK;
  unsigned long long n = 0;
  HIPCHECK(hipMemcpy(&n, e->d_leak_n, sizeof n, hipMemcpyDeviceToHost));
  if (!n) return CC_OK;
  n = std::min<unsigned long long>(n, e->leak_cap);
  std::vector<LeakRec> v(n);
  HIPCHECK(hipMemcpy(v.data(), e->d_leak, sizeof(LeakRec) * n, hipMemcpyDeviceToHost));
  for (const LeakRec& r : v) e->leaks[r.slot].push_back(r.idx);
  HIPCHECK(hipMemset(e->d_leak_n, 0, sizeof(unsigned long long)));
  return CC_OK;
}

// ResourceManager.deleteResource after resource.stateMachine.delete() succeeded (ResourceManager.java:212-235).
int cc::delete_slot(cc_engine* e, uint32_t slot) {
  int rc = sync_streams(e);  // (its device writes are queued: dev_flush before the next device work)
  if (rc) return rc;
  const uint32_t old_type = e->res_type[slot];
  if ((rc = drain_leaks(e))) return rc;
  e->leaks.erase(slot);  // the per-slot view ends with the resource (its dropped commits stay in the log)
  // ResourceManager.deleteResource: delete() the state, close the executor, drop every instance of the resource.
  if (is_keyed(e->res_type[slot])) {  // MapState.delete :264-274 / SetState.delete :123-134 — entries die with it
    if (launch_map_drop_resource(e->d_tbl_word, e->map_entries, slot, e->d_mw_cgen, e->own_stream))
      return set_err(CC_ERR_HIP, "map drop launch", hipGetLastError());
    HIPCHECK(hipStreamSynchronize(e->own_stream));
  }
  if (e->map_bits) dev_fill(e, e->d_msmall, slot, 0, 1);  // no more small-map events for it
  e->res_type[slot] = CC_RES_NONE;
  // ResourceManagerStateMachineExecutor.close cancels the resource's timers
  e->gtimers.erase(std::remove_if(e->gtimers.begin(), e->gtimers.end(),
                                  [slot](const cc_engine::GroupTimer& g) { return g.slot == slot; }),
                   e->gtimers.end());
  if (e->coord_on) dev_fill(e, e->d_coord, (uint64_t)slot * coord_block(e->coord_cap), 0, coord_block(e->coord_cap));
  mark_dirty(e->res_dirty_lo, e->res_dirty_hi, slot, slot + 1);
  dev_fill(e, e->d_val_meta, sizeof(uint32_t) * slot, 0, sizeof(uint32_t));
  dev_fill(e, e->d_val_v, sizeof(uint64_t) * slot, 0, sizeof(uint64_t));
  if (e->d_val_live) dev_fill(e, e->d_val_live, sizeof(uint64_t) * slot, 0, sizeof(uint64_t));
  // :223-229 walks sessions.entrySet() and iterator.remove()s every holder of the resource: removed in that
  // iteration order (the red-black deletes of a tree bin depend on it)
  std::vector<uint32_t> gone;
  e->sessions.for_each([&](int64_t id) {
    auto it = e->inst_by_id.find((uint64_t)id);
    if (it != e->inst_by_id.end() && e->inst_res[it->second] == slot) gone.push_back(it->second);
  });
  for (uint32_t i = 0; i < e->cfg.max_instances; ++i)  // (every holder is registered in sessions; kept as a guard)
    if (e->inst_res[i] == slot && std::find(gone.begin(), gone.end(), i) == gone.end()) gone.push_back(i);
  for (uint32_t i : gone) {
    e->inst_res[i] = kNoRes;
    e->sessions.remove((int64_t)e->inst_id[i], /*movable=*/false);  // iterator.remove()
    e->inst_by_id.erase(e->inst_id[i]);
    e->used_inst.clear(i);
    mark_dirty(e->inst_dirty_lo, e->inst_dirty_hi, i, i + 1);
  }
  // ResourceManager.resources / keys / ResourceHolder.sessions
  auto rit = e->res_by_id.find(e->res_id[slot]);
  if (rit != e->res_by_id.end() && rit->second == slot) e->res_by_id.erase(rit);
  if (e->res_has_key[slot]) e->keys.erase(e->res_key[slot]);
  e->res_has_key[slot] = 0;
  e->res_sessions.erase(e->res_sessions.lower_bound({slot, 0}), e->res_sessions.lower_bound({slot + 1, 0}));
  e->used_res.clear(slot);
  if (old_type < 16) e->open_grp[old_type].insert(slot >> 6);  // room again in its group (manager.hip)
  return CC_OK;
}

int cc::open_range(cc_engine* e, uint32_t first, uint32_t count, uint32_t res_first, uint32_t res_stride,
                      uint64_t id_first, uint64_t client) {
  const uint64_t end = (uint64_t)first + count;
  if (end > e->cfg.max_instances) return set_err(CC_ERR_CAPACITY, "instance slot out of range");
  for (uint64_t k = 0; k < count; ++k) {
    const uint64_t r = (uint64_t)res_first + k * res_stride;
    if (r >= e->cfg.max_resources || e->res_type[r] == CC_RES_NONE) return set_err(CC_ERR_INVALID, "instance on unknown resource");
    if (e->inst_res[first + k] != kNoRes) return set_err(CC_ERR_INVALID, "instance slot already open");
    if (e->inst_by_id.count(id_first + k)) return set_err(CC_ERR_INVALID, "instance id already open");
  }
  int rc = sync_streams(e);  // (its device writes are queued: dev_flush before the next device work)
  if (rc) return rc;
  for (uint64_t k = 0; k < count; ++k) {
    e->inst_res[first + k] = (uint32_t)(res_first + k * res_stride);
    e->inst_id[first + k] = id_first + k;
    e->inst_client[first + k] = client;
    e->sessions.put((int64_t)(id_first + k));  // sessions.put(instance id, holder): HashMap.putVal of a new key
    e->inst_by_id[id_first + k] = (uint32_t)(first + k);
    e->used_inst.set(first + k);
  }
  mark_dirty(e->inst_dirty_lo, e->inst_dirty_hi, first, end);
  return CC_OK;
}

extern "C" int cc_instance_open(cc_engine* e, uint32_t inst, uint32_t res_slot, uint64_t instance_id, uint64_t client_session) {
  if (!e) return CC_ERR_INVALID;
  return open_range(e, inst, 1, res_slot, 0, instance_id, client_session);
}

extern "C" int cc_instance_open_range(cc_engine* e, uint32_t first, uint32_t count, uint32_t res_first, uint64_t id_first,
                                      uint64_t client_session) {
  if (!e) return CC_ERR_INVALID;
  return open_range(e, first, count, res_first, 1, id_first, client_session);
}

// Diagnostics (CC_DEBUG_SYNC=1): drain the stream after every launch of cc_apply_batch and name the launch whose
// kernels failed.
static const bool g_dbg_sync = getenv("CC_DEBUG_SYNC") != nullptr;
#define DBG_SYNC(what)                                                                          \
  do {                                                                                          \
    if (g_dbg_sync) {                                                                           \
      hipError_t _x = hipStreamSynchronize(st);                                                 \
      if (_x != hipSuccess) return set_err(CC_ERR_HIP, "CC_DEBUG_SYNC after " what, _x);        \
    }                                                                                           \
  } while (0)

// TTL mode: the map events appended so far (commits, expiries) -> every map's size and capacity, the small maps' key
// sets (map_small.hip: sort, runs, k_small_replay + k_ttl_replay), then the counters for the next round.
static int ttl_replay(cc_engine* e, hipStream_t st, const uint64_t* index = nullptr, uint64_t lo = 0,
                      const cc_results* out = nullptr) {
  uint32_t ctl[2] = {0, 0};
  HIPCHECK(hipMemcpyAsync(ctl, e->d_sm_ctl, sizeof ctl, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  SmallArgs sa{};
  sa.ev_key = e->d_sm_key;
  sa.ev_key2 = e->d_sm_key2;
  sa.ev_val = e->d_sm_val;
  sa.ev_val2 = e->d_sm_val2;
  sa.ev_pay = e->d_sm_pay;
  sa.cap = (uint32_t)e->sm_cap;
  sa.temp = e->d_sm_temp;
  sa.temp_bytes = e->sm_temp_bytes;
  sa.ctl = e->d_sm_ctl;
  sa.seg = e->d_sm_seg;
  sa.nseg = e->d_sm_seg + e->cfg.max_resources;
  sa.state = e->d_msm;
  sa.big = e->d_mbig;
  sa.msmall = e->d_msmall;
  sa.left = e->d_msm_left + 2ull * e->cfg.max_resources;  // (an engine-stream replay: folded right after it)
  sa.err = e->d_err;
  sa.mpcap = e->d_mpcap;
  sa.max_resources = e->cfg.max_resources;
  sa.msize = e->d_msize;
  sa.lvl_at = e->d_lvl_at;
  sa.index = index;  // (null for the expiry-only flushes: they grow no table)
  sa.lo = lo;
  sa.out_status = out ? out->status : nullptr;  // (the sub-batch's size / isEmpty rows among the events)
  sa.out_value = out ? out->value : nullptr;
  {
    int rc = join_replay(e, st);  // (an overlapped replay of an earlier sub-batch: the models it writes)
    if (rc) return rc;
  }
  const int rs = launch_small_replay(sa, ctl[0], st, st);
  if (rs) return rs == -1 ? set_err(CC_ERR_HIP, "TTL map events launch", hipGetLastError())
                          : set_err(CC_ERR_STATE, "TTL map events exceed their buffer");
  if (launch_small_finish(sa, st)) return set_err(CC_ERR_HIP, "map event counters", hipGetLastError());
  return CC_OK;
}

static TtlEmit ttl_emit_args(const cc_engine* e, const uint64_t* time, uint64_t n, uint64_t lo, uint64_t bl, uint64_t bh,
                             uint64_t adv) {
  TtlEmit t{};
  t.time = time;
  t.n = n;
  t.lo = lo;
  t.bl = bl;
  t.bh = bh;
  t.adv = adv;
  t.deferred = (e->cfg.flags & CC_CFG_TIMERS_DEFERRED) ? 1u : 0u;
  t.hh_key = e->d_hh_key;
  t.hh_val = e->d_hh_val;
  t.hh_n = e->hh_n;
  t.ev_key = e->d_sm_key;
  t.ev_val = e->d_sm_val;
  t.ev_pay = e->d_sm_pay;
  t.ev_cap = (uint32_t)e->sm_cap;
  t.ctl = e->d_sm_ctl;
  return t;
}

// TTL mode: the expiries of the boundaries [bl, bh] that no sub-batch owned (before a barrier row, at the batch end),
// or every timer due by `adv` (cc_advance_time), as size events.
static int ttl_flush(cc_engine* e, const uint64_t* time, uint64_t n, uint64_t bl, uint64_t bh, uint64_t adv,
                     hipStream_t st) {
  int rc = ensure_small(e);
  if (rc) return rc;
  const TtlEmit te = ttl_emit_args(e, time, n, bl, bl, bh, adv);
  if (launch_ttl_scan(te, e->d_clock, e->d_tbl_word, e->d_tbl_key, e->d_tbl_dl, e->map_entries, e->d_err, st))
    return set_err(CC_ERR_HIP, "TTL scan launch", hipGetLastError());
  return ttl_replay(e, st);
}

extern "C" int cc_apply_batch(cc_engine* e, const cc_batch* c, uint64_t n, const cc_results* out, const cc_events* ev,
                              void* stream) {
  if (!e || !c || !out) return set_err(CC_ERR_INVALID, "null argument");
  e->last_end = nullptr;  // (profiling markers: no begin marker is shared across calls)
  if (n == 0) return CC_OK;
  if (n > e->cfg.max_batch) return set_err(CC_ERR_CAPACITY, "batch larger than max_batch");
  if (!c->inst || !c->op || !c->flags || !c->a || !c->b || !out->status || !out->value)
    return set_err(CC_ERR_INVALID, "inst/op/flags/a/b columns and status/value outputs are required");
  HIPCHECK(hipSetDevice(e->device));
  hipStream_t st = stream ? (hipStream_t)stream : e->own_stream;
  if (st != e->last_stream) HIPCHECK(hipStreamSynchronize(e->last_stream));
  if (e->dev_dirty()) {  // registry writes queued by the control plane since the last device work
    int rc = quiesce(e);
    if (rc) return rc;
  }
  e->last_stream = st;
  if ((((uintptr_t)out->status) & 3) || (((uintptr_t)out->value) & 15) || (((uintptr_t)c->inst) & 15))
    return set_err(CC_ERR_INVALID, "inst and value must be 16-byte aligned, status 4-byte aligned");
  if (e->map_bits && !c->key) return set_err(CC_ERR_INVALID, "an engine with maps needs the key column");
  if (e->map_bits && !c->index)  // (log order of map events and the entries' claims: the tree-bin test, map_wide.hip)
    return set_err(CC_ERR_INVALID, "an engine with maps needs the index column");
  if (e->d_val_live && !c->index) return set_err(CC_ERR_INVALID, "CC_CFG_VALUE_RETAINED needs the index column");
  if (ev && (!ev->pos || !ev->target || !ev->code || !ev->src || !ev->tag || !ev->payload || !ev->count))
    return set_err(CC_ERR_INVALID, "event stream columns and count are required");
  // Whole-map ops are barriers (map_wide.hip): find them (one sync), then apply the rows between them as segments.
  e->bars.clear();
  uint64_t clock_before = 0;  // the engine clock before this batch (TTL mode and barrier rows need it on the host)
  e->szq_n = 0;
  e->isc_rows.clear();
  e->clr_n = 0;
  e->clr_heavy.clear();
  if (e->map_bits || e->coord_on) {
    uint32_t nb = 0, ttl_seen = 0;
    // Outside TTL mode map size / isEmpty, containsValue and clear rows are answered in the stream (listed, their maps
    // flagged); in TTL mode size / isEmpty rows are (the event replay answers them), the others are barriers.  A batch
    // that turns TTL mode on (or lists more than a list holds) is scanned again with TTL mode's lists (or larger ones).
    bool inline_size = e->map_bits && !e->ttl_live;
    bool inline_ttl = e->map_bits && e->ttl_live;
    for (int pass = 0;; ++pass) {
      if ((inline_size || inline_ttl) && !e->d_szq) {
        e->szq_cap = 1u << 20;
        HIPCHECK(hipMalloc(&e->d_szq, sizeof(uint32_t) * e->szq_cap));
        HIPCHECK(hipMalloc(&e->d_szq_n, sizeof(uint32_t)));
      }
      if (inline_size && !e->d_cvq) {  // containsValue candidates (map_cv.hip)
        e->cvq_cap = 1u << 20;
        HIPCHECK(hipMalloc(&e->d_cvq, sizeof(uint32_t) * e->cvq_cap));
        HIPCHECK(hipMalloc(&e->d_isc, sizeof(uint32_t) * e->cvq_cap));
        HIPCHECK(hipMalloc(&e->d_cvq_n, sizeof(uint32_t) * 2));
        HIPCHECK(hipMalloc(&e->d_mfirst, sizeof(uint32_t) * e->cfg.max_resources));
        HIPCHECK(hipMalloc(&e->d_maynull, e->cfg.max_resources));
        e->clrq_cap = 1u << 20;  // clears in the stream (map_clear.hip)
        HIPCHECK(hipMalloc(&e->d_clrq, sizeof(uint32_t) * e->clrq_cap));
        HIPCHECK(hipMalloc(&e->d_clrq_n, sizeof(uint32_t)));
        HIPCHECK(hipMalloc(&e->d_clr_keys, sizeof(uint64_t) * e->clrq_cap));
        HIPCHECK(hipMalloc(&e->d_clr_keys2, sizeof(uint64_t) * e->clrq_cap));
        HIPCHECK(hipMalloc(&e->d_clr_off, sizeof(uint32_t) * (e->cfg.max_resources + 1)));
        HIPCHECK(hipMalloc(&e->d_clr_base, sizeof(uint32_t) * e->cfg.max_resources));
        HIPCHECK(hipMalloc(&e->d_clr_eend, e->cfg.max_resources));
        e->clr_temp_bytes = std::max<size_t>(clr_sort_temp_bytes(e->clrq_cap), 256);
        HIPCHECK(hipMalloc(&e->d_clr_temp, e->clr_temp_bytes));
      }
      if (e->szq_flagged) {
        if (launch_mflag_clear(e->d_msmall, e->cfg.max_resources, st)) return set_err(CC_ERR_HIP, "map flags", hipGetLastError());
        e->szq_flagged = false;
      }
      HIPCHECK(hipMemsetAsync(e->d_ttl_seen, 0, sizeof(uint32_t), st));
      if (launch_map_barriers(c->inst, c->op, c->aux, n, e->d_inst_res, e->d_res_type, e->cfg.max_instances, e->d_bar,
                              e->d_bar_n, kBarCap, e->d_ttl_seen, inline_size || inline_ttl ? e->d_szq : nullptr,
                              inline_size || inline_ttl ? e->d_szq_n : nullptr, e->szq_cap, e->d_msmall,
                              inline_size ? e->d_cvq : nullptr, inline_size ? e->d_cvq_n : nullptr, e->cvq_cap,
                              inline_size ? e->d_mfirst : nullptr, e->cfg.max_resources,
                              inline_size ? e->d_clrq : nullptr, inline_size ? e->d_clrq_n : nullptr, e->clrq_cap, st))
        return set_err(CC_ERR_HIP, "map barrier scan launch", hipGetLastError());
      if (inline_size) {  // containsValue candidates: in the stream, or barriers (map_cv.hip)
        CvBatchArgs cb{};
        cb.inst = c->inst;
        cb.op = c->op;
        cb.flags = c->flags;
        cb.n = n;
        cb.inst_res = e->d_inst_res;
        cb.max_inst = e->cfg.max_instances;
        cb.mflag = e->d_msmall;
        cb.tbl_word = e->d_tbl_word;
        cb.entries = e->map_entries;
        cb.cvq = e->d_cvq;
        cb.cvq_n = e->d_cvq_n;
        cb.cvq_cap = e->cvq_cap;
        cb.mfirst = e->d_mfirst;
        cb.maynull = e->d_maynull;
        cb.R = e->cfg.max_resources;
        cb.bar = e->d_bar;
        cb.bar_n = e->d_bar_n;
        cb.bar_cap = kBarCap;
        cb.isc = e->d_isc;
        cb.isc_n = e->d_cvq_n + 1;
        if (launch_cv_batch(cb, st)) return set_err(CC_ERR_HIP, "containsValue classify launch", hipGetLastError());
      }
      uint32_t qn = 0, cvn[2] = {0, 0}, cln = 0;
      {  // (one round trip: every counter into the pinned words, then one synchronize)
        uint64_t* const pin = e->h_pin;
        uint32_t* const p32 = reinterpret_cast<uint32_t*>(pin + 1);
        HIPCHECK(hipMemcpyAsync(pin, e->d_clock, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(p32 + 0, e->d_bar_n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(p32 + 1, e->d_ttl_seen, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        if (inline_size || inline_ttl) HIPCHECK(hipMemcpyAsync(p32 + 2, e->d_szq_n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        if (inline_size) HIPCHECK(hipMemcpyAsync(p32 + 3, e->d_cvq_n, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        if (inline_size) HIPCHECK(hipMemcpyAsync(p32 + 5, e->d_clrq_n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        if (e->map_bits) {  // the batch's first and last log index (map event positions, below)
          HIPCHECK(hipMemcpyAsync(pin + 4, c->index, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
          HIPCHECK(hipMemcpyAsync(pin + 5, c->index + n - 1, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        }
        HIPCHECK(hipStreamSynchronize(st));
        // Map events are keyed by their position (log index - the sub-batch's first, 32 bits: common.h kEvPosBits).
        // A batch whose whole index range fits needs no cut; else each sub-batch ends before its first row 2^32 past
        // its start (k_span_cut, one round trip per sub-batch, only then)
        if (e->map_bits) e->span_cut = n && pin[5] - pin[4] >= (1ull << kEvPosBits);
        clock_before = pin[0];
        nb = p32[0];
        ttl_seen = p32[1];
        if (inline_size || inline_ttl) qn = p32[2];
        if (inline_size) cvn[0] = p32[3], cvn[1] = p32[4], cln = p32[5];
      }
      if (!inline_size && !inline_ttl) break;
      e->szq_flagged = qn > 0 || cvn[0] > 0 || cln > 0;
      if (inline_size && (ttl_seen || pass > 2)) {  // this batch turns TTL mode on: containsValue and clear become
        inline_size = false;                        // barriers again, size / isEmpty stay in the stream
        inline_ttl = pass <= 2;
        continue;
      }
      if (qn > e->szq_cap) {  // a larger list, then the same scan again
        HIPCHECK(hipFree(e->d_szq));
        e->d_szq = nullptr;
        e->szq_cap = qn;
        HIPCHECK(hipMalloc(&e->d_szq, sizeof(uint32_t) * e->szq_cap));
        continue;
      }
      if (cln > e->clrq_cap) {
        HIPCHECK(hipFree(e->d_clrq));
        HIPCHECK(hipFree(e->d_clr_keys));
        HIPCHECK(hipFree(e->d_clr_keys2));
        HIPCHECK(hipFree(e->d_clr_temp));
        e->clrq_cap = cln;
        HIPCHECK(hipMalloc(&e->d_clrq, sizeof(uint32_t) * e->clrq_cap));
        HIPCHECK(hipMalloc(&e->d_clr_keys, sizeof(uint64_t) * e->clrq_cap));
        HIPCHECK(hipMalloc(&e->d_clr_keys2, sizeof(uint64_t) * e->clrq_cap));
        e->clr_temp_bytes = std::max<size_t>(clr_sort_temp_bytes(e->clrq_cap), 256);
        HIPCHECK(hipMalloc(&e->d_clr_temp, e->clr_temp_bytes));
        continue;
      }
      if (cvn[0] > e->cvq_cap) {
        HIPCHECK(hipFree(e->d_cvq));
        HIPCHECK(hipFree(e->d_isc));
        e->cvq_cap = cvn[0];
        HIPCHECK(hipMalloc(&e->d_cvq, sizeof(uint32_t) * e->cvq_cap));
        HIPCHECK(hipMalloc(&e->d_isc, sizeof(uint32_t) * e->cvq_cap));
        continue;
      }
      e->szq_n = qn;
      if (inline_ttl) break;  // (TTL mode lists size / isEmpty rows only)
      int rc = cv_rows(e, cvn[1], st);  // the in-stream rows, sorted, on the host too
      if (rc) return rc;
      if ((rc = clr_rows(e, cln, c, st))) return rc;  // the in-stream clears: sorted by (map, row), offsets
      break;
    }
    if (ttl_seen && !e->ttl_live) {  // TTL mode for good: sizes and capacities from commit + expiry events
      e->ttl_live = true;
      e->small_live = false;  // (every map's events are replayed in TTL mode, the small ones' key sets included)
    }
    // The leak log (commits dropped without clean()) is drained before every batch of an engine that can add to it:
    // every multimap put, and with value events every re-listen (AtomicValueState.listen :41-49) may land there, at
    // most one entry per row, so the drained log gets room for n more; a coordination engine without value events
    // adds entries only in the close fan-out (cc_sessions_close sizes the log for that itself) but is drained here
    // too, so nothing accumulates across batches toward the log's end.
    if (e->has_mmaps || e->coord_on) {
      int rc = drain_leaks(e);
      const bool may_leak = e->has_mmaps || (e->cfg.flags & CC_CFG_VALUE_EVENTS);
      if (!rc && may_leak) rc = ensure_leak(e, n);
      if (rc) return rc;
    }
    if (nb > kBarCap) {
      // More barrier rows than one listing holds: the batch runs as two consecutive batches (a batch boundary is a
      // point of the log like any other: timers due by its clock have fired there in both timer orders, A8).  With an
      // event stream the second half's events are appended after the first's, their rows moved by h.
      if (n < 2)
        return set_err(CC_ERR_CAPACITY, "more whole-map ops and group schedules in one row than kBarCap");
      const uint64_t h = n / 2;
      auto shift = [h](const auto* p) { return p ? p + h : p; };
      const cc_batch c2{shift(c->index), shift(c->time), shift(c->inst), shift(c->op), shift(c->flags), shift(c->key),
                        shift(c->a), shift(c->b), shift(c->aux)};
      const cc_results o2{out->status + h, out->value + h};
      int rc = cc_apply_batch(e, c, h, out, ev, stream);
      if (rc || !ev || !e->coord_on) return rc ? rc : cc_apply_batch(e, &c2, n - h, &o2, ev, stream);
      uint64_t n1 = 0, n2 = 0;
      HIPCHECK(hipMemcpyAsync(&n1, ev->count, sizeof n1, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      if (n1 > ev->capacity) return set_err(CC_ERR_CAPACITY, "event stream capacity exceeded");
      if (!e->d_half_count) HIPCHECK(hipMalloc(&e->d_half_count, sizeof(uint64_t)));
      cc_events ev2 = *ev;
      ev2.pos += n1, ev2.target += n1, ev2.code += n1, ev2.src += n1, ev2.tag += n1, ev2.payload += n1;
      ev2.capacity -= n1;
      ev2.count = e->d_half_count;
      if ((rc = cc_apply_batch(e, &c2, n - h, &o2, &ev2, stream))) return rc;
      HIPCHECK(hipMemcpyAsync(&n2, e->d_half_count, sizeof n2, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      if (launch_ev_shift(ev2.pos, std::min(n2, ev2.capacity), (uint32_t)h, st))
        return set_err(CC_ERR_HIP, "event row shift launch", hipGetLastError());
      const uint64_t total = n1 + n2;
      HIPCHECK(hipMemcpyAsync(ev->count, &total, sizeof total, hipMemcpyHostToDevice, st));
      HIPCHECK(hipStreamSynchronize(st));  // (total is a host local)
      return CC_OK;
    }
    if (nb) {  // the barrier rows in log order, then their columns in one gather (one copy back, not one per field)
      e->bars.resize(nb);
      HIPCHECK(hipMemcpy(e->bars.data(), e->d_bar, sizeof(uint32_t) * nb, hipMemcpyDeviceToHost));
      std::sort(e->bars.begin(), e->bars.end());
      if (nb > e->bar_rows_cap) {
        if (e->d_bar_rows) HIPCHECK(hipFree(e->d_bar_rows));
        e->d_bar_rows = nullptr;
        e->bar_rows_cap = 0;
        HIPCHECK(hipMalloc(&e->d_bar_rows, sizeof(BarRow) * nb));
        e->bar_rows_cap = nb;
      }
      HIPCHECK(hipMemcpyAsync(e->d_bar, e->bars.data(), sizeof(uint32_t) * nb, hipMemcpyHostToDevice, st));
      if (launch_bar_fields(e->d_bar, nb, c->inst, c->op, c->flags, c->a, c->key, c->aux, c->index, c->time,
                            e->d_bar_rows, st))
        return set_err(CC_ERR_HIP, "barrier rows gather launch", hipGetLastError());
      e->bar_rows.resize(nb);
      HIPCHECK(hipMemcpyAsync(e->bar_rows.data(), e->d_bar_rows, sizeof(BarRow) * nb, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
    }
  }
  if (e->coord_on || e->ttl_live) {  // events of this batch start at 0; the log clock must not go backwards inside it
    if (e->coord_on) HIPCHECK(hipMemsetAsync(e->d_ev_total, 0, sizeof(unsigned long long), st));
    // (without barrier rows every row goes through k_part_ext, which checks it against the row before it)
    if (!e->bars.empty() && launch_time_check(c->time, n, e->d_clock, e->d_err, st))
      return set_err(CC_ERR_HIP, "time check", hipGetLastError());
  }
  // Group timers: where each pending one fires in this batch, and where the timer of each schedule row of the batch
  // would (the clock at row r is max(clock_before, time[r])): the first row r >= from whose clock reaches the deadline
  // -> the boundary the timer fires at (manager mode: after row r; module mode: before it, A8), or ~0 when no row of
  // this batch reaches it.  One device search for all of them (k_fire_bounds).
  const bool deferred = (e->cfg.flags & CC_CFG_TIMERS_DEFERRED) != 0;
  auto clock_at = [&](const BarRow& br) { return c->time ? std::max(br.t_row, clock_before) : clock_before; };
  std::vector<uint64_t> sched_dl(e->bars.size(), 0), sched_fb(e->bars.size(), ~0ull);  // per barrier (schedule rows)
  {
    std::vector<uint64_t> dl, from;
    std::vector<uint32_t> who;  // < gtimers.size(): a pending timer; else gtimers.size() + barrier index
    for (size_t q = 0; q < e->gtimers.size(); ++q) {
      dl.push_back(e->gtimers[q].deadline);
      from.push_back(0);
      who.push_back((uint32_t)q);
    }
    for (size_t k = 0; k < e->bars.size(); ++k) {
      const BarRow& br = e->bar_rows[k];
      if (br.op != CC_OP_GROUP_SCHEDULE) continue;
      const uint64_t delay = c->aux ? br.aux : 0;
      sched_dl[k] = clock_at(br) + ((int64_t)delay > 0 ? delay : 0);  // schedule :86-103
      dl.push_back(sched_dl[k]);
      from.push_back(deferred ? e->bars[k] : (uint64_t)e->bars[k] + 1);
      who.push_back((uint32_t)(e->gtimers.size() + k));
    }
    const uint32_t m = (uint32_t)dl.size();
    if (m) {
      if (m > e->fb_cap) {
        if (e->d_fb) HIPCHECK(hipFree(e->d_fb));
        e->d_fb = nullptr;
        e->fb_cap = 0;
        HIPCHECK(hipMalloc(&e->d_fb, sizeof(uint64_t) * 3 * m));
        e->fb_cap = m;
      }
      std::vector<uint64_t> res(m);
      HIPCHECK(hipMemcpyAsync(e->d_fb, dl.data(), 8ull * m, hipMemcpyHostToDevice, st));
      HIPCHECK(hipMemcpyAsync(e->d_fb + m, from.data(), 8ull * m, hipMemcpyHostToDevice, st));
      if (launch_fire_bounds(c->time, n, clock_before, e->d_fb, e->d_fb + m, m, deferred, e->d_fb + 2 * m, st))
        return set_err(CC_ERR_HIP, "timer bounds launch", hipGetLastError());
      HIPCHECK(hipMemcpyAsync(res.data(), e->d_fb + 2 * m, 8ull * m, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      for (uint32_t i = 0; i < m; ++i) {
        if (who[i] < e->gtimers.size()) e->gtimers[who[i]].fire_b = res[i];
        else sched_fb[who[i] - e->gtimers.size()] = res[i];
      }
    }
  }
  if (e->map_bits && !e->ttl_live) {  // the batch's hot map keys (apply_map_hot.hip): counted once, bound per sub-batch
    HotArgs hb{};
    hb.inst = c->inst;
    hb.flags = c->flags;
    hb.key = c->key;
    hb.lo = 0;
    hb.hi = n;
    hb.inst_res = e->d_inst_res;
    hb.res_type = e->d_res_type;
    hb.max_inst = e->cfg.max_instances;
    hb.hot_samp = e->d_hot_samp;
    hb.hot_cand = e->d_hot_cand;
    hb.hot_cand_n = e->d_hot_cand_n;
    if (launch_map_hot_detect(hb, st)) return set_err(CC_ERR_HIP, "hot-key detect launch", hipGetLastError());
  }
  uint64_t cur = 0;
  size_t bi = 0;
  uint64_t own_lo = 0;  // TTL mode: the first timer-firing boundary no sub-batch has owned yet (common.h TtlEmit)
  for (;;) {
  // the next thing in log order: a barrier row, or a group timer firing (timers first at the same boundary)
  const uint64_t bar_b = bi < e->bars.size() ? (uint64_t)e->bars[bi] : ~0ull;
  size_t tk = e->gtimers.size();
  for (size_t q = 0; q < e->gtimers.size(); ++q) {
    const auto& g = e->gtimers[q];
    if (g.fire_b == ~0ull || g.fire_b < cur) continue;
    if (tk == e->gtimers.size()) { tk = q; continue; }
    const auto& b = e->gtimers[tk];
    if (std::make_tuple(g.fire_b, g.deadline, g.id) < std::make_tuple(b.fire_b, b.deadline, b.id)) tk = q;
  }
  const uint64_t tim_b = tk < e->gtimers.size() ? e->gtimers[tk].fire_b : ~0ull;
  const int action = (tim_b != ~0ull && tim_b <= bar_b) ? 2 : (bar_b != ~0ull ? 1 : 0);
  const uint64_t seg_lo = cur;
  const uint64_t seg_hi = action == 2 ? tim_b : (action == 1 ? bar_b : n);
  for (uint64_t lo = seg_lo, hi; lo < seg_hi; lo = hi) {
    hi = std::min(seg_hi, lo + (e->ext ? e->sub_ext : e->sub_batch));
    if (e->sm_alt_on && !e->ttl_live) {  // the other event-buffer set, once its replay is done (engine_state.h SmSet)
      std::swap(e->d_sm_key, e->sm_alt.key);
      std::swap(e->d_sm_key2, e->sm_alt.key2);
      std::swap(e->d_sm_val, e->sm_alt.val);
      std::swap(e->d_sm_val2, e->sm_alt.val2);
      std::swap(e->d_sm_pay, e->sm_alt.pay);
      std::swap(e->d_sm_cseg, e->sm_alt.cseg);
      e->sm_cur ^= 1;
      int rc = wait_replay(e, e->sm_cur, st);  // (its replay's exit marks fold into the snapshot here)
      if (rc) return rc;
    }
    for (const auto& hv : e->clr_heavy) {  // at most 127 in-stream clears of one map per sub-batch (map_clear.hip)
      const size_t q = (size_t)(std::lower_bound(hv.begin(), hv.end(), (uint32_t)lo) - hv.begin());
      if (q + 127 < hv.size() && hv[q + 127] < hi) hi = hv[q + 127];
    }
    // this sub-batch's in-stream containsValue rows (at most kCvMaxRows: a denser run ends the sub-batch earlier)
    size_t cv_b = 0, cv_e = 0;
    if (!e->isc_rows.empty()) {
      cv_b = (size_t)(std::lower_bound(e->isc_rows.begin(), e->isc_rows.end(), (uint32_t)lo) - e->isc_rows.begin());
      cv_e = (size_t)(std::lower_bound(e->isc_rows.begin(), e->isc_rows.end(), (uint32_t)hi) - e->isc_rows.begin());
      if (cv_e - cv_b > kCvMaxRows) {
        cv_e = cv_b + kCvMaxRows;
        hi = e->isc_rows[cv_e];
      }
    }
    if (e->span_cut && !e->ttl_live) {  // (TTL mode positions events by row, 2 (row - lo) + 1: always within 32 bits)
      HIPCHECK(hipMemsetAsync(e->d_span_cut, 0xFF, sizeof(uint64_t), st));
      if (launch_span_cut(c->index, lo, hi, e->d_span_cut, st)) return set_err(CC_ERR_HIP, "span cut launch", hipGetLastError());
      HIPCHECK(hipMemcpyAsync(e->h_pin + 6, e->d_span_cut, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      if (e->h_pin[6] > lo && e->h_pin[6] < hi) hi = e->h_pin[6];
      if (!e->isc_rows.empty())  // (the in-stream containsValue rows of the shortened sub-batch)
        cv_e = (size_t)(std::lower_bound(e->isc_rows.begin(), e->isc_rows.end(), (uint32_t)hi) - e->isc_rows.begin());
    }
    const uint32_t cv_n = (uint32_t)(cv_e - cv_b);
    const bool clr_on = e->clr_n > 0;  // clears in the stream in this batch (map_clear.hip)
    ClrSubArgs ca{};
    ClrCtx cctx{};
    if (clr_on) {
      int rc = ensure_small(e);  // (the cleared maps' sizes ride the map event buffer)
      if (rc) return rc;
      ca.keys = e->d_clr_keys2;
      ca.n = e->clr_n;
      ca.off = e->d_clr_off;
      ca.R = e->cfg.max_resources;
      ca.lo = lo;
      ca.hi = hi;
      ca.base = e->d_clr_base;
      ca.eend = e->d_clr_eend;
      ca.mflag = e->d_msmall;
      ca.err = e->d_err;
      ca.index = c->index;
      ca.ev_key = e->d_sm_key;
      ca.ev_val = e->d_sm_val;
      ca.ev_pay = e->d_sm_pay;
      ca.ev_cap = (uint32_t)e->sm_cap;
      ca.ev_ctl = e->d_sm_ctl;
      ca.cgen = e->d_mw_cgen;
      {  // the epoch buckets: at most 1024 per map and ~64 MB in all
        uint32_t nbmax = 16;
        while (nbmax < 1024 && (uint64_t)(2 * nbmax) * e->cfg.max_resources <= (64ull << 20)) nbmax <<= 1;
        uint32_t sh = 0;
        while (((hi - lo + (1ull << sh) - 1) >> sh) > nbmax) ++sh;
        ca.bshift = sh;
        ca.nb = (uint32_t)((hi - lo + (1ull << sh) - 1) >> sh);
        const size_t need = (size_t)nbmax * e->cfg.max_resources;
        if (e->clr_btab_bytes < need) {
          if (e->d_clr_btab) (void)hipFree(e->d_clr_btab);
          e->d_clr_btab = nullptr;
          HIPCHECK(hipMalloc(&e->d_clr_btab, need));
          e->clr_btab_bytes = need;
        }
        ca.btab = e->d_clr_btab;
      }
      if (launch_clr_sub(ca, st)) return set_err(CC_ERR_HIP, "clear epochs launch", hipGetLastError());
      cctx = ClrCtx{e->d_msmall, e->d_clr_keys2, e->d_clr_off, e->d_clr_base, e->d_clr_eend, lo, e->d_tbl_ep,
                    e->d_clr_btab, ca.nb, ca.bshift};
    }
    CvSubArgs cva{};
    cva.clr = cctx;
    ++e->stat_subbatches;
    e->stat_isc += cv_n;
    const uint32_t tiles = (uint32_t)((hi - lo + kTile - 1) / kTile);
    SizeArgs sz{};       // this sub-batch's size / isEmpty rows (map_small.hip)
    bool sized = false;  // the event pipeline ran (its counters are reset after the answers)
    bool ttl_pending = false;  // TTL mode: the sub-batch's event replay, after the unpermute
    uint32_t cv_E = 0;         // in-stream containsValue events (final once the map apply kernels ran)
    bool cv_known = false;     // (read with the map events' count: one host round trip per sub-batch, not two)
    uint32_t sized_events = 0;
    if (e->map_bits && e->ttl_live) {  // TTL mode: every key goes through its region (timers are walked in order)
      HIPCHECK(hipMemsetAsync(e->d_hot_n, 0, sizeof(uint32_t), st));
    }
    HotArgs ha{};
    if (e->map_bits && !e->ttl_live) {  // hot map keys of this sub-batch (routed to their own buckets by the partition)
      ha.inst = c->inst;
      ha.flags = c->flags;
      ha.key = c->key;
      ha.lo = lo;
      ha.hi = hi;
      ha.inst_res = e->d_inst_res;
      ha.res_type = e->d_res_type;
      ha.max_inst = e->cfg.max_instances;
      ha.mrec = e->d_mrec;
      ha.cb = c->b;
      ha.ttab = e->d_ttab;
      ha.tiles = tiles;
      ha.sb = e->sb_total();
      ha.sb_val = e->sb;
      ha.map_bits = e->map_bits;
      ha.tbl_key = e->d_tbl_key;
      ha.tbl_word = e->d_tbl_word;
      ha.tbl_val = e->d_tbl_val;
      ha.tbl_ci = e->d_tbl_ci;
      ha.tbl_ins = e->d_tbl_ins;
      ha.tbl_claim = e->d_tbl_claim;
      ha.idx0 = c->index ? c->index + lo : nullptr;
      ha.hot = e->d_hot;
      ha.hot_n = e->d_hot_n;
      ha.hot_rpre = e->d_hot_rpre;
      ha.hot_rstart = e->d_hot_rstart;
      ha.hot_len = e->d_hot_len;
      ha.hot_cond = e->d_hot_cond;
      ha.hot_agg = e->d_hot_agg;
      ha.hot_s0 = e->d_hot_s0;
      ha.hot_samp = e->d_hot_samp;
      ha.hot_cand = e->d_hot_cand;
      ha.hot_cand_n = e->d_hot_cand_n;
      ha.hot_meta = e->d_hot_meta;
      ha.rst_status = e->d_rst_status;
      ha.rst_value = e->d_rst_value;
      ha.hot_msz = e->d_hot_msz;
      ha.msmall = nullptr;  // (every map's keys are hot-routed)
      if (e->small_live || e->szq_n || clr_on) {  // small / size-queried / cleared maps' hot commits: map events
        int rc = ensure_small(e);
        if (rc) return rc;
        if (!c->index) return set_err(CC_ERR_INVALID, "an engine with maps needs the index column (log order)");
        ha.hc.clr = cctx;  // (cleared maps: commit epochs, map_clear.hip)
        ha.hc.mflag = e->d_msmall;
        ha.hc.hh_key = e->d_hh_key;
        ha.hc.hh_val = e->d_hh_val;
        ha.hc.hh_n = e->hh_n;
        ha.hc.xr = e->d_mrec;
        ha.hc.lo = lo;
        ha.hc.ev_key = e->d_sm_key;
        ha.hc.ev_val = e->d_sm_val;
        ha.hc.ev_pay = e->d_sm_pay;
        ha.hc.ev_cap = (uint32_t)e->sm_cap;
        ha.hc.ev_ctl = e->d_sm_ctl;
        ha.hc.idx0p = c->index + lo;
        ha.hc.tbl_ep = e->d_tbl_ep;
      }
      ha.err = e->d_err;
      ha.mark = marker_of(e);
      static const bool no_hot = diag_env("CC_NO_HOT");  // diagnostics: every key through its region
      if (no_hot) HIPCHECK(hipMemsetAsync(e->d_hot_n, 0, sizeof(uint32_t), st));
      else if (launch_map_hot_bind(ha, st)) return set_err(CC_ERR_HIP, "hot-key bind launch", hipGetLastError()); DBG_SYNC("hot-key bind launch");
    }
    PartArgs pa{};
    pa.inst = c->inst;
    pa.op = c->op;
    pa.flags = c->flags;
    pa.a = c->a;
    pa.b = c->b;
    pa.key = c->key;
    pa.index = c->index;
    pa.aux = (e->coord_on || e->ttl_live) ? c->aux : nullptr;  // maps read ttl only in TTL mode (the scan saw none)
    pa.time = c->time;
    pa.clock_base = e->d_clock;
    pa.ext_flags = ((e->cfg.flags & CC_CFG_VALUE_EVENTS) ? kExtValue : 0u) | ((e->cfg.flags & CC_CFG_TIMERS_DEFERRED) ? kExtDeferred : 0u) |
                   ((e->coord_on || e->ttl_live) && e->bars.empty() ? kExtTimeCheck : 0u);
    pa.err = e->d_err;
    pa.ext = e->ext;
    pa.lo = lo;
    pa.hi = hi;
    pa.inst_res = e->d_inst_res;
    pa.inst_id = e->coord_on ? e->d_inst_id : nullptr;
    pa.res_type = e->d_res_type;
    pa.sb_kind = e->d_sb_kind;
    pa.max_inst = e->cfg.max_instances;
    pa.sb = e->sb_total();
    pa.sb_val = e->sb;
    pa.sbq_base = e->quarter ? e->sbq_base() : 0u;
    pa.map_bits = e->map_bits;
    pa.hot = e->d_hot;
    pa.hot_n = e->d_hot_n;
    pa.st_meta = e->d_st_meta;
    pa.st_ab = e->d_st_ab;
    pa.xrec = e->d_xrec;
    pa.mrec = e->d_mrec;
    pa.hot_meta = e->d_hot_meta;
    pa.clr = cctx;  // (each map commit's clear epoch into its meta word)
    pa.cpos = e->d_cpos;
    pa.ttab = e->d_ttab;
    pa.dummy = e->sub_batch;
    const bool v3 = !e->ext;  // value-only engines: value_path.hip
    pa.v3 = v3;
    // the sub-batch's results back to log order (every staged result is written by then); launched early, beside
    // the host's counter readback, when nothing after that point writes staged results (below)
    bool unpermuted = false;
    auto unpermute = [&]() -> int {
      UnpermuteArgs ua{};
      ua.cpos = e->d_cpos;
      ua.ttab = e->d_ttab;
      ua.sb = e->sb_total();
      ua.lo = lo;
      ua.hi = hi;
      ua.rst_status = e->d_rst_status;
      ua.rst_value = e->d_rst_value;
      ua.out_status = out->status;
      ua.out_value = out->value;
      ua.dummy_status = e->d_rst_status + e->sub_batch;
      ua.dummy_value = e->d_rst_value + e->sub_batch;
      ua.v3 = v3;
      ua.words = reinterpret_cast<const uint64_t*>(e->d_st_ab);
      ua.mark = marker_of(e);
      if (launch_unpermute(ua, st)) return set_err(CC_ERR_HIP, "unpermute launch", hipGetLastError());
      unpermuted = true;
      return CC_OK;
    };

    pa.mark = marker_of(e);
    if (launch_partition(pa, st)) {
      const hipError_t x = hipGetLastError();
      if (x == hipSuccess) return set_err(CC_ERR_CAPACITY, "the partition's LDS cannot hold this engine's buckets");
      return set_err(CC_ERR_HIP, "partition launch", x);
    }
    DBG_SYNC("partition launch");
    {
      int rc = launch_pending_replay(e, st);  // (the previous sub-batch's small-map replay, beside this one's work)
      if (rc) return rc;
    }
    if (e->map_bits && e->ttl_live && launch_map_rows(e->d_cpos, lo, hi, e->d_map_row, st))
      return set_err(CC_ERR_HIP, "map rows launch", hipGetLastError());
    ValueArgs va{};
    va.st_meta = e->d_st_meta;
    va.st_ab = e->d_st_ab;
    va.ttab = e->d_ttab;
    va.tiles = v3 ? (uint32_t)((hi - lo + kV3Tile - 1) / kV3Tile) : tiles;
    va.v3 = v3;

    va.ca = c->a;
    va.cb = c->b;
    va.lo = lo;
    va.sb = e->sb_total();
    va.sb_val = e->sb;
    va.sb_kind = e->d_sb_kind;
    va.val_meta = e->d_val_meta;
    va.val_v = e->d_val_v;
    va.rst_status = e->d_rst_status;
    va.rst_value = e->d_rst_value;
    va.dummy = e->sub_batch;
    va.err = e->d_err;
    va.mark = marker_of(e);
    if ((e->has_values || !e->ext) && launch_apply_value(va, st)) return set_err(CC_ERR_HIP, "apply launch", hipGetLastError()); DBG_SYNC("apply launch");
    if (cv_n) {  // in-stream containsValue: operand set, initial counts, query events (map_cv.hip)
      int rc = ensure_cv(e);
      if (rc) return rc;
      uint32_t sc = 1024;
      while (sc < 2 * cv_n) sc <<= 1;
      cva.cv.mflag = e->d_msmall;
      cva.cv.set = e->d_cvset;
      cva.cv.mask = sc - 1;
      cva.cv.bloom = e->d_cvbloom;
      cva.cv.bbits = 16;
      while (cva.cv.bbits < kCvBloomMaxBits && (1ull << cva.cv.bbits) < 16ull * cv_n) ++cva.cv.bbits;
      cva.cv.ev_key = e->d_cvev_key;
      cva.cv.ev_val = e->d_cvev_val;
      cva.cv.cap = e->cvev_cap;
      cva.cv.ctl = e->d_cvev_ctl;
      cva.cv.idx0p = c->index + lo;
      cva.set = e->d_cvset;
      cva.cnt = e->d_cvcnt;
      cva.isc = e->d_isc2 + cv_b;
      cva.isc_n = cv_n;
      cva.lo = lo;
      cva.inst = c->inst;
      cva.flags = c->flags;
      cva.a = c->a;
      cva.index = c->index;
      cva.inst_res = e->d_inst_res;
      cva.tbl_word = e->d_tbl_word;
      cva.tbl_val = e->d_tbl_val;
      cva.entries = e->map_entries;
      cva.err = e->d_err;
      cva.key2 = e->d_cvev_key2;
      cva.val2 = e->d_cvev_val2;
      cva.seg = e->d_cvseg;
      cva.nseg = e->d_cvseg + e->cvset_cap;
      cva.coll = e->d_cvseg;          // (free until the answers' runs: the prepare's collision list)
      cva.coll_n = e->d_cvev_ctl + 1;
      cva.temp = e->d_cvtemp;
      cva.temp_bytes = e->cvtemp_bytes;
      cva.out_status = out->status;
      cva.out_value = out->value;
      if (launch_cv_prepare(cva, st)) return set_err(CC_ERR_HIP, "containsValue prepare launch", hipGetLastError());
      ha.cv = cva.cv;
    }
    if (e->map_bits) {
      if (!e->ttl_live && launch_map_hot_apply(ha, st)) return set_err(CC_ERR_HIP, "hot-key apply launch", hipGetLastError());
      MapArgs ma{};
      ma.cv = cva.cv;
      ma.clr = cctx;
      ma.mrec = e->d_mrec;
      ma.cb = c->b;
      ma.lo = lo;
      ma.ttab = e->d_ttab;
      ma.tiles = tiles;
      ma.sb = e->sb_total();
      ma.sb_val = e->sb;
      ma.map_bits = e->map_bits;
      ma.tbl_key = e->d_tbl_key;
      ma.tbl_word = e->d_tbl_word;
      ma.tbl_val = e->d_tbl_val;
      ma.tbl_ci = e->d_tbl_ci;
      ma.tbl_ins = e->d_tbl_ins;
      ma.tbl_claim = e->d_tbl_claim;
      ma.idx0 = c->index ? c->index + lo : nullptr;
      ma.dropped = e->d_mw_drop;
      ma.cgen = e->d_mw_cgen;
      ma.cset = e->d_cset;
      ma.cset_mask = e->cset_mask;
      ma.cset_full = e->d_cset_full;
      ma.ttl = e->ttl_live;
      ma.tbl_dl = e->d_tbl_dl;
      ma.map_row = e->d_map_row;
      ma.time = c->time;
      ma.aux = c->aux;
      ma.clock_base = e->d_clock;
      ma.deferred = (e->cfg.flags & CC_CFG_TIMERS_DEFERRED) != 0;
      ma.rst_status = e->d_rst_status;
      ma.rst_value = e->d_rst_value;
      ma.rst_msz = e->d_rst_msz;
      ma.err = e->d_err;
      ma.mark = marker_of(e);
      TtlEmit te{};
      if (e->ttl_live) {  // this sub-batch owns the timer-firing boundaries [own_lo, hi] (common.h TtlEmit)
        int rc = ensure_small(e);
        if (rc) return rc;
        te = ttl_emit_args(e, c->time, n, lo, own_lo, hi, 0);
        ma.ttl_emit = te;
      }
      if (launch_apply_map(ma, st)) return set_err(CC_ERR_HIP, "map apply launch", hipGetLastError()); DBG_SYNC("map apply launch");
      if (clr_on && launch_clr_gen(ca, st)) return set_err(CC_ERR_HIP, "clear generation launch", hipGetLastError());
      if (e->ttl_live) {  // exact sizes and capacities in TTL mode: the sub-batch's commits and expiries as events
        if (launch_ttl_scan(te, e->d_clock, e->d_tbl_word, e->d_tbl_key, e->d_tbl_dl, e->map_entries, e->d_err, st))
          return set_err(CC_ERR_HIP, "TTL scan launch", hipGetLastError());
        MapSizeArgs za{};
        za.ttab = e->d_ttab;
        za.cpos = e->d_cpos;
        za.tiles = tiles;
        za.rows = hi - lo;
        za.sb = e->sb_total();
        za.k0 = e->sb;
        za.k1 = e->sbq_base();
        za.sb_hot = e->sb + (1u << e->map_bits);
        za.rst_msz = e->d_rst_msz;
        za.hot = e->d_hot;
        za.hot_n = e->d_hot_n;  // (0: no hot keys in TTL mode)
        za.hot_len = e->d_hot_len;
        za.hot_rpre = e->d_hot_rpre;
        za.hot_msz = e->d_hot_msz;
        za.res_type = e->d_res_type;
        za.max_resources = e->cfg.max_resources;
        za.tcnt = e->d_msz_tcnt;
        za.msize = e->d_msize;
        za.mpcap = e->d_mpcap;
        za.list = e->d_msz_list;
        za.list_n = e->d_msz_list_n;
        za.mrec = e->d_mrec;
        za.hh_key = e->d_hh_key;
        za.hh_val = e->d_hh_val;
        za.hh_n = e->hh_n;
        za.ev_key = e->d_sm_key;
        za.ev_val = e->d_sm_val;
        za.ev_pay = e->d_sm_pay;
        za.ev_cap = (uint32_t)e->sm_cap;
        za.sm_ctl = e->d_sm_ctl;
        za.map_row = e->d_map_row;
        za.lo = lo;
        za.lvl_at = e->d_lvl_at;
        za.index = c->index;
        za.err = e->d_err;
        if (launch_map_size(za, st)) return set_err(CC_ERR_HIP, "map size launch", hipGetLastError());
        own_lo = hi + 1;
        if (e->szq_n) {  // this sub-batch's size / isEmpty rows join the events at their rows' positions
          sz.szq = e->d_szq;
          sz.szq_n = e->szq_n;
          sz.lo = lo;
          sz.hi = hi;
          sz.inst = c->inst;
          sz.op = c->op;
          sz.index = c->index;
          sz.inst_res = e->d_inst_res;
          sz.ev_key = e->d_sm_key;
          sz.ev_val = e->d_sm_val;
          sz.ev_pay = e->d_sm_pay;
          sz.cap = (uint32_t)e->sm_cap;
          sz.ctl = e->d_sm_ctl;
          sz.err = e->d_err;
          sz.ttl = true;
          if (launch_size_emit(sz, st)) return set_err(CC_ERR_HIP, "size query launch", hipGetLastError());
        }
        ttl_pending = true;  // (the replay answers them: after the unpermute's placeholders)
      } else {  // exact map sizes and HashMap capacities (containsValue's iteration order)
        MapSizeArgs za{};
        za.ttab = e->d_ttab;
        za.cpos = e->d_cpos;
        za.tiles = tiles;
        za.rows = hi - lo;
        za.sb = e->sb_total();
        za.k0 = e->sb;
        za.k1 = e->sbq_base();
        za.sb_hot = e->sb + (1u << e->map_bits);
        za.rst_msz = e->d_rst_msz;
        za.hot = e->d_hot;
        za.hot_n = e->d_hot_n;
        za.hot_len = e->d_hot_len;
        za.hot_rpre = e->d_hot_rpre;
        za.hot_msz = e->d_hot_msz;
        za.res_type = e->d_res_type;
        za.max_resources = e->cfg.max_resources;
        za.tcnt = e->d_msz_tcnt;
        za.msize = e->d_msize;
        za.mpcap = e->d_mpcap;
        za.list = e->d_msz_list;
        za.list_n = e->d_msz_list_n;
        za.err = e->d_err;
        za.lvl_at = e->d_lvl_at;
        za.index = c->index;
        za.lo = lo;
        if (e->small_live || e->szq_n || clr_on) {  // small / size-queried / cleared maps: their insertions / removals
          int rc = ensure_small(e);
          if (rc) return rc;
          if (!c->index) return set_err(CC_ERR_INVALID, "an engine with maps needs the index column (log order)");
          za.msmall = e->d_msmall;
          za.mrec = e->d_mrec;
          za.idx0 = c->index + lo;
          za.hh_key = e->d_hh_key;
          za.hh_val = e->d_hh_val;
          za.hh_n = e->hh_n;
          za.ev_key = e->d_sm_key;
          za.ev_val = e->d_sm_val;
          za.ev_pay = e->d_sm_pay;
          za.ev_cap = (uint32_t)e->sm_cap;
          za.sm_ctl = e->d_sm_ctl;
        }
        if (launch_map_size(za, st)) return set_err(CC_ERR_HIP, "map size launch", hipGetLastError()); DBG_SYNC("map size launch");
        if (e->szq_n) {  // this sub-batch's size / isEmpty rows join the events
          sz.szq = e->d_szq;
          sz.szq_n = e->szq_n;
          sz.lo = lo;
          sz.hi = hi;
          sz.inst = c->inst;
          sz.op = c->op;
          sz.index = c->index;
          sz.inst_res = e->d_inst_res;
          sz.ev_key = e->d_sm_key;
          sz.ev_val = e->d_sm_val;
          sz.ev_pay = e->d_sm_pay;
          sz.cap = (uint32_t)e->sm_cap;
          sz.ctl = e->d_sm_ctl;
          sz.err = e->d_err;
          sz.sorted_key = e->d_sm_key2;
          sz.sorted_val = e->d_sm_val2;
          sz.seg = e->d_sm_seg;
          sz.nseg = e->d_sm_seg + e->cfg.max_resources;
          sz.msize = e->d_msize;
          sz.out_status = out->status;
          sz.out_value = out->value;
          if (launch_size_emit(sz, st)) return set_err(CC_ERR_HIP, "size query launch", hipGetLastError());
        }
        if (clr_on && launch_clr_events(ca, st)) return set_err(CC_ERR_HIP, "clear events launch", hipGetLastError());
        if (e->small_live || e->szq_n || clr_on) {
          uint32_t ctl[2] = {0, 0};
          uint32_t* const p32 = reinterpret_cast<uint32_t*>(e->h_pin);  // (pinned: one round trip for both)
          HIPCHECK(hipMemcpyAsync(p32, e->d_sm_ctl, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
          if (cv_n) HIPCHECK(hipMemcpyAsync(p32 + 2, e->d_cvev_ctl, sizeof cv_E, hipMemcpyDeviceToHost, st));
          if (!e->coord_on) {  // (the coordination apply, launched below, writes staged results: then no early unpermute)
            if (!e->ev_rb) HIPCHECK(hipEventCreateWithFlags(&e->ev_rb, hipEventDisableTiming));
            HIPCHECK(hipEventRecord(e->ev_rb, st));
            int rc = unpermute();  // (on the GPU while the host waits for the counters)
            if (rc) return rc;
            HIPCHECK(hipEventSynchronize(e->ev_rb));
          } else {
            HIPCHECK(hipStreamSynchronize(st));
          }
          ctl[0] = p32[0];
          ctl[1] = p32[1];
          if (cv_n) memcpy(&cv_E, p32 + 2, sizeof cv_E);
          cv_known = cv_n != 0;
          e->stat_events += ctl[0];
          SmallArgs sa{};
          sa.ev_key = e->d_sm_key;
          sa.ev_key2 = e->d_sm_key2;
          sa.ev_val = e->d_sm_val;
          sa.ev_val2 = e->d_sm_val2;
          sa.ev_pay = e->d_sm_pay;
          sa.cap = (uint32_t)e->sm_cap;
          sa.temp = e->d_sm_temp;
          sa.temp_bytes = e->sm_temp_bytes;
          sa.ctl = e->d_sm_ctl;
          sa.seg = e->d_sm_seg;
          sa.nseg = e->d_sm_seg + e->cfg.max_resources;
          sa.cseg = e->d_sm_cseg;
          sa.state = e->d_msm;
          sa.big = e->d_mbig;
          sa.msmall = e->d_msmall;
          sa.left = e->d_msm_left + 2ull * e->cfg.max_resources;  // (on this stream: folded right after it)
          sa.err = e->d_err;
          sa.mpcap = e->d_mpcap;
          sa.max_resources = e->cfg.max_resources;
          sa.lvl_at = e->d_lvl_at;
          sa.idx0 = c->index + lo;
          // the replay overlaps the next sub-batch on the side stream (engine_state.h SmSet), launched once that
          // sub-batch's partition is queued (launch_pending_replay)
          static const bool no_side = diag_env("CC_NO_SIDE_REPLAY");  // diagnostics: the replay on the engine stream
          if (ctl[0] && !no_side) {
            int rc = ensure_sm_alt(e);
            if (rc) return rc;
            sa.defer = true;
            sa.left = e->d_msm_left + (size_t)e->sm_cur * e->cfg.max_resources;  // (folded by wait_replay)
          }
          const int rs = launch_small_replay(sa, ctl[0], st, st);
          if (sa.defer && !rs) {
            e->pend_sa = sa;
            e->pend = true;
            e->pend_set = e->sm_cur;
          }
          if (rs) return rs == -1 ? set_err(CC_ERR_HIP, "small-map replay launch", hipGetLastError())
                                  : set_err(CC_ERR_STATE, "small-map events exceed their buffer");
          if (e->small_live && ctl[0] == 0 && ctl[1] == 0) e->small_live = false;  // (ctl[1]: maps small after the last replay)
          sized = true;
          sized_events = ctl[0];
        }
      }
    }
    if (e->coord_on) {
      HIPCHECK(hipMemsetAsync(e->d_ev_cnt, 0, sizeof(uint16_t) * (hi - lo), st));
      HIPCHECK(hipMemsetAsync(e->d_arena_n, 0, sizeof(unsigned long long), st));
      CoordArgs ca{};
      ca.xrec = e->d_xrec;
      ca.ttab = e->d_ttab;
      ca.tiles = tiles;
      ca.sb = e->sb_total();
      ca.sb_val = e->sb;
      ca.sbq_base = e->quarter ? e->sbq_base() : 0u;
      ca.sb_kind = e->d_sb_kind;
      ca.res_type = e->d_res_type;
      ca.inst_id = e->d_inst_id;
      ca.coord = e->d_coord;
      ca.coord_cap = e->coord_cap;
      ca.val_meta = e->d_val_meta;
      ca.val_v = e->d_val_v;
      ca.rst_status = e->d_rst_status;
      ca.rst_value = e->d_rst_value;
      ca.ev_cnt = e->d_ev_cnt;
      ca.arena = e->d_arena;
      ca.arena_n = e->d_arena_n;
      ca.arena_cap = e->arena_cap;
      ca.leak = e->d_leak;
      ca.leak_n = e->d_leak_n;
      ca.leak_cap = e->leak_cap;
      ca.err = e->d_err;
      ca.mark = marker_of(e);
      if (launch_apply_coord(ca, st)) return set_err(CC_ERR_HIP, "coordination apply launch", hipGetLastError()); DBG_SYNC("coordination apply launch");
    }
    if (!unpermuted) {
      int rc = unpermute();
      if (rc) return rc;
    }
    DBG_SYNC("unpermute launch");
    if (cv_n) {  // in-stream containsValue answers over the unpermute's placeholders (map_cv.hip)
      if (!cv_known) {
        HIPCHECK(hipMemcpyAsync(e->h_pin, e->d_cvev_ctl, sizeof cv_E, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        memcpy(&cv_E, e->h_pin, sizeof cv_E);
      }
      const int rc = launch_cv_answer(cva, cv_E, st);
      if (rc) return rc == -2 ? set_err(CC_ERR_CAPACITY, "containsValue events exceed their buffer")
                              : set_err(CC_ERR_HIP, "containsValue answer launch", hipGetLastError());
    }
    if (ttl_pending) {  // TTL mode: sizes, capacities, small maps' key sets, and the size / isEmpty rows' answers
      int rc = ttl_replay(e, st, c->index, lo, out);
      if (rc) return rc;
    }
    if (sized) {  // size / isEmpty answers over the unpermute's placeholders; then the next sub-batch's counters
      if (e->szq_n && sized_events && launch_size_answer(sz, st))
        return set_err(CC_ERR_HIP, "size answer launch", hipGetLastError());
      if (clr_on && sized_events) {  // the cleared maps' sizes, capacities and size / isEmpty rows (map_clear.hip)
        ClrReplayArgs cr{};
        cr.key = e->d_sm_key2;
        cr.val = e->d_sm_val2;
        cr.pay = e->d_sm_pay;
        cr.mflag = e->d_msmall;
        cr.msize = e->d_msize;
        cr.mpcap = e->d_mpcap;
        cr.lvl_at = e->d_lvl_at;
        cr.idx0 = c->index + lo;
        cr.out_status = out->status;
        cr.out_value = out->value;
        int rc = ensure_clr_scan(e);
        if (rc) return rc;
        cr.scan = e->d_clr_scan;
        cr.temp = e->d_clr_stemp;
        cr.temp_bytes = e->clr_stemp_bytes;
        if (launch_clr_replay(cr, sized_events, st)) return set_err(CC_ERR_HIP, "clear replay launch", hipGetLastError());
      }
      SmallArgs sf{};
      sf.ctl = e->d_sm_ctl;
      sf.msmall = e->d_msmall;
      sf.max_resources = e->cfg.max_resources;
      if (launch_small_finish(sf, st)) return set_err(CC_ERR_HIP, "small-map counters", hipGetLastError());
    }
    if (e->coord_on) {
      EventArgs ea{};
      ea.cpos = e->d_cpos;
      ea.lo = lo;
      ea.hi = hi;
      ea.tiles = tiles;
      ea.ev_cnt = e->d_ev_cnt;
      ea.row_of = e->d_row_of;
      ea.ev_loc = e->d_ev_loc;
      ea.tile_sum = e->d_tile_sum;
      ea.tile_off = e->d_tile_off;
      ea.ev_total = e->d_ev_total;
      ea.arena = e->d_arena;
      ea.arena_n = e->d_arena_n;
      ea.arena_cap = e->arena_cap;
      ea.perm = e->d_ev_perm;
      ea.bucket = e->d_ev_bucket;  // the tile-bucketed order pass (CC_EV_V1=1: the gather pass)
      ea.ccnt = e->d_ev_ccnt;
      if (ev) {
        ea.out_cap = ev->capacity;
        ea.out_pos = ev->pos;
        ea.out_target = ev->target;
        ea.out_code = ev->code;
        ea.out_src = ev->src;
        ea.out_tag = ev->tag;
        ea.out_payload = ev->payload;
      }
      ea.err = e->d_err;
      ea.mark = marker_of(e);
      if (launch_events(ea, st)) return set_err(CC_ERR_HIP, "events launch", hipGetLastError()); DBG_SYNC("events launch");
    }
  }
  {
    int rc = join_replay(e, st);  // (barrier rows, timers and the caller read the small maps' models)
    if (rc) return rc;
  }
  if (action == 2) {  // a group timer fires here (MembershipGroupState.java:92-98)
    cc_engine::GroupTimer gt = e->gtimers[tk];
    e->gtimers.erase(e->gtimers.begin() + (ptrdiff_t)tk);
    const uint32_t pos = (uint32_t)(deferred ? seg_hi - 1 : seg_hi);
    if (launch_group_fire(e->d_coord, e->coord_cap, gt.slot, gt.member, gt.tag, gt.payload, pos, e->d_ev_total, ev, e->d_err, st))
      return set_err(CC_ERR_HIP, "group timer launch", hipGetLastError());
    cur = seg_hi;
    continue;
  }
  if (action == 0) {
    if (e->map_bits && e->ttl_live && own_lo <= n) {  // the boundaries after the last sub-batch (manager mode: row n)
      int rc = ttl_flush(e, c->time, n, own_lo, n, 0, st);
      if (rc) return rc;
    }
    break;
  }
  {  // the barrier row, against the state as it stands after the rows before it
    const uint64_t row = seg_hi;
    ++e->stat_barriers;
    const BarRow& br = e->bar_rows[bi];
    const size_t bk = bi;
    cur = row + 1;
    ++bi;
    if (e->map_bits && e->ttl_live) {  // the timers that fire up to this row's boundary, as size events (TtlEmit)
      if (own_lo <= row) {
        int rc = ttl_flush(e, c->time, n, own_lo, row, 0, st);
        if (rc) return rc;
      }
      own_lo = row + 1;
    }
    uint32_t res = 0;
    const uint32_t in = br.inst;
    const uint8_t op = br.op, fl = br.flags;
    const uint64_t a = br.a;
    // (k_map_barriers listed the row through the device registry; the host mirror must agree before its slot
    // indexes any per-resource array)
    if (row >= n || in >= e->cfg.max_instances || (res = e->inst_res[in]) >= e->cfg.max_resources ||
        !(is_keyed(e->res_type[res]) || e->res_type[res] == CC_RES_GROUP))
      return set_err(CC_ERR_STATE, "barrier row does not resolve to a map / set / multimap / group on the host registry");
    if (e->res_type[res] == CC_RES_GROUP) {  // schedule :86-103 (member = key, callback = a, delay = aux)
      const uint64_t member = br.key;
      if (launch_group_schedule(e->d_coord, e->coord_cap, res, member, row, out->status, out->value, e->d_ttl_seen, st))
        return set_err(CC_ERR_HIP, "group schedule launch", hipGetLastError());
      uint32_t found = 0;
      HIPCHECK(hipMemcpyAsync(&found, e->d_ttl_seen, sizeof found, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      if (found) {
        cc_engine::GroupTimer gt{};
        gt.deadline = sched_dl[bk];
        gt.id = ++e->gtimer_seq;
        gt.member = member;
        gt.tag = CC_FLAG_TAG_A(fl);
        gt.payload = gt.tag == CC_TAG_NULL ? 0 : a;
        gt.slot = res;
        gt.idx = br.idx;
        gt.fire_b = sched_fb[bk];
        e->gtimers.push_back(gt);
      }
      continue;
    }
    MapWideArgs mw{};
    mw.slot = res;
    mw.op = e->res_type[res] == CC_RES_SET        ? set_as_map_op(op)
            : e->res_type[res] == CC_RES_MULTIMAP ? mmap_as_map_op(op, CC_FLAG_TAG_A(fl))
                                                  : op;
    mw.atag = CC_FLAG_TAG_A(fl);
    mw.apay = a;
    mw.row = row;
    mw.tbl_word = e->d_tbl_word;
    mw.tbl_key = e->d_tbl_key;
    mw.tbl_val = e->d_tbl_val;
    mw.tbl_ins = e->d_tbl_ins;
    mw.tbl_claim = e->d_tbl_claim;
    mw.lvl_at = e->d_lvl_at;
    if (e->ttl_live) {  // the clock at which the reference last fired timers before this row (A8)
      uint64_t t0 = clock_before, t1 = clock_before;
      if (c->time) {
        t1 = std::max(br.t_row, clock_before);
        if (row > 0) t0 = std::max(br.t_prev, clock_before);
      }
      mw.tbl_dl = e->d_tbl_dl;
      mw.fire_clock = (e->cfg.flags & CC_CFG_TIMERS_DEFERRED) ? t0 : t1;
    }
    mw.entries = e->map_entries;
    mw.peak_lo = e->d_mw_peak;
    mw.dropped = e->d_mw_drop;
    mw.cgen = e->d_mw_cgen;
    mw.cset = e->d_cset;
    mw.cset_n = e->cset_mask + 1;
    mw.cset_full = e->d_cset_full;
    mw.map_bits = e->map_bits;
    mw.msize = e->d_msize;  // exact in both modes (TTL mode: commit + expiry events, map_small.hip)
    mw.mpcap = e->d_mpcap;
    mw.ctl = e->d_mw_ctl;
    mw.small = e->res_type[res] == CC_RES_MAP ? e->d_msm : nullptr;
    mw.big = e->d_mbig;
    mw.hh_key = e->d_hh_key;
    mw.hh_val = e->d_hh_val;
    mw.hh_n = e->hh_n;
    mw.out_status = out->status;
    mw.out_value = out->value;
    mw.err = e->d_err;
    if (launch_map_wide(mw, st)) return set_err(CC_ERR_HIP, "whole-map op launch", hipGetLastError()); DBG_SYNC("whole-map op launch");
    if (e->res_type[res] == CC_RES_MAP && (mw.op == CC_OP_MAP_CLEAR || mw.op == CC_OP_DELETE) &&
        (launch_big_clear(e->d_mbig, e->d_msm, res, st) || launch_small_clear(e->d_msm, res, st)))
      return set_err(CC_ERR_HIP, "small-map clear launch", hipGetLastError());
  }
  }
  if (e->has_sets || e->has_mmaps) {
    KeyedResultArgs ka{c->inst,     c->op,          c->flags, c->index,     n,           e->d_inst_res, e->d_res_type,
                       e->cfg.max_instances, out->status, out->value, e->d_leak, e->d_leak_n, e->leak_cap, e->d_err};
    if (launch_keyed_results(ka, st)) return set_err(CC_ERR_HIP, "set / multimap results launch", hipGetLastError()); DBG_SYNC("set / multimap results launch");
  }
  // Retained value commits (live.hip): after every value op of the batch has applied.  The post-pass attributes
  // each row through the END-of-batch inst_res / res_type / val_meta: correct because the registry cannot change
  // inside a cc_apply_batch call (resource create/delete, instance open/close are host calls that quiesce the
  // stream between batches; no op applied on the device rebinds an instance or retypes a slot).
  if (e->d_val_live) {
    if (launch_value_live(c->inst, c->op, out->status, out->value, c->index, n, e->d_inst_res, e->d_res_type,
                          e->cfg.max_instances, e->d_val_meta, e->cfg.max_resources, e->d_val_wrow, e->d_val_live, st))
      return set_err(CC_ERR_HIP, "retained value launch", hipGetLastError());
  }
  if (e->coord_on && ev) HIPCHECK(hipMemcpyAsync(ev->count, e->d_ev_total, sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
  if (e->coord_on || e->map_bits) {  // the log clock (timers: lock timeouts, map TTL)
    if (launch_clock_advance(c->time, n, 0, e->d_clock, st)) return set_err(CC_ERR_HIP, "clock", hipGetLastError()); DBG_SYNC("clock");
  }
  if (c->index) {  // the applied watermark = index of the batch's last entry
    HIPCHECK(hipMemcpyAsync(e->d_last_index, c->index + (n - 1), sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
    e->applied_pending = true;
  }
  return CC_OK;
}

// String.hashCode of HANDLE keys (java.util.HashMap bins of MapState, MapState.java:33,49-60): merged into the host
// map, then the sorted (handle, hash) table is uploaded whole (control plane: rare, and small next to a batch).
extern "C" int cc_handle_hashes(cc_engine* e, const uint64_t* h_handles, const int32_t* h_hashes, uint64_t count) {
  if (!e || (count && (!h_handles || !h_hashes))) return set_err(CC_ERR_INVALID, "null argument");
  if (count == 0) return CC_OK;
  int rc = quiesce(e);
  if (rc) return rc;
  for (uint64_t i = 0; i < count; ++i) {
    auto it = e->hh.find(h_handles[i]);
    if (it != e->hh.end() && it->second != h_hashes[i])
      return set_err(CC_ERR_INVALID, "a handle's String.hashCode cannot change (interned Strings are immutable)");
    e->hh[h_handles[i]] = h_hashes[i];
  }
  const uint32_t n = (uint32_t)e->hh.size();
  if (n > e->hh_cap) {
    const uint32_t cap = std::max<uint32_t>(n, e->hh_cap * 2);
    uint64_t* k = nullptr;
    int32_t* v = nullptr;
    HIPCHECK(hipMalloc(&k, 8ull * cap));
    if (hipMalloc(&v, 4ull * cap) != hipSuccess) {
      (void)hipFree(k);
      return set_err(CC_ERR_HIP, "hipMalloc handle hashes");
    }
    if (e->d_hh_key) (void)hipFree(e->d_hh_key);
    if (e->d_hh_val) (void)hipFree(e->d_hh_val);
    e->d_hh_key = k;
    e->d_hh_val = v;
    e->hh_cap = cap;
  }
  std::vector<uint64_t> hk;
  std::vector<int32_t> hv;
  hk.reserve(n);
  hv.reserve(n);
  for (const auto& kv : e->hh) hk.push_back(kv.first), hv.push_back(kv.second);
  HIPCHECK(hipMemcpy(e->d_hh_key, hk.data(), 8ull * n, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(e->d_hh_val, hv.data(), 4ull * n, hipMemcpyHostToDevice));
  e->hh_n = n;
  return CC_OK;
}

extern "C" int cc_applied_index_async(cc_engine* e, uint64_t* d_out, void* stream) {
  if (!e || !d_out) return set_err(CC_ERR_INVALID, "null argument");
  HIPCHECK(hipSetDevice(e->device));
  hipStream_t st = stream ? (hipStream_t)stream : e->own_stream;
  if (st != e->last_stream) HIPCHECK(hipStreamSynchronize(e->last_stream));
  e->last_stream = st;
  // the device copy of the last batch's last index (kept up to date stream-ordered by cc_apply_batch)
  HIPCHECK(hipMemcpyAsync(d_out, e->d_last_index, sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
  return CC_OK;
}

extern "C" int cc_engine_counters(cc_engine* e, uint64_t* out, uint32_t n) {
  if (!e || (n && !out)) return CC_ERR_INVALID;
  uint64_t v[5] = {e->stat_barriers, e->stat_isc, e->stat_subbatches, e->stat_events, 0};
  if (n > 4 && e->d_mbig) {  // (the owners of the big models: one strided read after the stream drains)
    int rc = cc_sync(e);
    if (rc) return rc;
    uint32_t own[kBigSlots];
    HIPCHECK(hipMemcpy2D(own, sizeof(uint32_t), &e->d_mbig->h.owner, sizeof(BigMap), sizeof(uint32_t), kBigSlots,
                         hipMemcpyDeviceToHost));
    for (uint32_t b = 0; b < kBigSlots; ++b) v[4] += own[b] != 0;
  }
  for (uint32_t i = 0; i < n && i < 5; ++i) out[i] = v[i];
  return CC_OK;
}

extern "C" int cc_applied_index(cc_engine* e, uint64_t* out) {
  if (!e || !out) return CC_ERR_INVALID;
  int rc = cc_sync(e);
  *out = e->applied;
  return rc;
}

// HashMap.hash of a java.lang.Long key: h = (int)(v ^ v >>> 32); h ^ h >>> 16

// The closing instances (client rank, slot) -> ResourceManager.close(Session) fan-out, in client rank order
// (ResourceManager.java:250-264); `count` clients.  The two entry points below build `by_client`.
static int sessions_close_core(cc_engine* e, const std::vector<std::pair<uint64_t, uint32_t>>& by_client, uint64_t count,
                               const cc_events* d_events, hipStream_t st, uint64_t* h_closed);

static int sessions_close_args(cc_engine* e, const cc_events* d_events) {
  if (d_events && (!d_events->pos || !d_events->target || !d_events->code || !d_events->src || !d_events->tag ||
                   !d_events->payload || !d_events->count))
    return set_err(CC_ERR_INVALID, "event stream columns and count are required");
  return CC_OK;
}

// ResourceManager.close(Session) for each client session of h_clients, in that order (ResourceManager.java:250-264).
extern "C" int cc_sessions_close(cc_engine* e, const uint64_t* h_clients, uint64_t count, const cc_events* d_events,
                                 void* stream, uint64_t* h_closed) {
  if (!e || (count && !h_clients)) return set_err(CC_ERR_INVALID, "null argument");
  int rc = sessions_close_args(e, d_events);
  if (rc) return rc;
  rc = quiesce(e);
  if (rc) return rc;
  hipStream_t st = stream ? (hipStream_t)stream : e->own_stream;
  e->last_stream = st;
  // the fan-out order: client order, then each client's instances in HashMap order of `sessions`
  std::vector<std::pair<uint64_t, uint32_t>> by_client;  // (client rank, slot) candidates
  {
    std::vector<std::pair<uint64_t, uint64_t>> rank(count);  // (client, rank), sorted for lookup
    for (uint64_t i = 0; i < count; ++i) rank[i] = {h_clients[i], i};
    std::sort(rank.begin(), rank.end());
    for (uint32_t i = 0; i < e->cfg.max_instances; ++i) {
      if (e->inst_res[i] == kNoRes) continue;
      auto it = std::lower_bound(rank.begin(), rank.end(), std::make_pair(e->inst_client[i], (uint64_t)0));
      if (it != rank.end() && it->first == e->inst_client[i]) by_client.emplace_back(it->second, i);
    }
  }
  return sessions_close_core(e, by_client, count, d_events, st, h_closed);
}

static int sessions_close_core(cc_engine* e, const std::vector<std::pair<uint64_t, uint32_t>>& by_client, uint64_t count,
                               const cc_events* d_events, hipStream_t st, uint64_t* h_closed) {
  struct Close { uint64_t crank, okey; uint32_t slot; };
  std::vector<Close> order;
  order.reserve(by_client.size());
  if (!by_client.empty()) {  // the closing instances' positions in sessions.values() iteration order
    std::vector<std::pair<uint64_t, uint64_t>> pos;  // (instance id, position), only the closing instances'
    pos.reserve(by_client.size());
    for (auto& bc : by_client) pos.emplace_back(e->inst_id[bc.second], ~0ull);
    std::sort(pos.begin(), pos.end());
    uint64_t q = 0;
    e->sessions.for_each([&](int64_t id) {
      auto it = std::lower_bound(pos.begin(), pos.end(), std::make_pair((uint64_t)id, (uint64_t)0));
      if (it != pos.end() && it->first == (uint64_t)id) it->second = q;
      ++q;
    });
    for (auto& bc : by_client) {
      const uint32_t i = bc.second;
      auto it = std::lower_bound(pos.begin(), pos.end(), std::make_pair(e->inst_id[i], (uint64_t)0));
      if (it == pos.end() || it->first != e->inst_id[i] || it->second == ~0ull)
        return set_err(CC_ERR_STATE, "an open instance is missing from the sessions map");
      order.push_back(Close{bc.first, it->second, i});
    }
  }
  std::sort(order.begin(), order.end(), [](const Close& x, const Close& y) {
    return x.crank != y.crank ? x.crank < y.crank : x.okey < y.okey;
  });
  const uint32_t m = (uint32_t)order.size();
  if (h_closed) *h_closed = 0;
  if (m == 0) {
    if (d_events) HIPCHECK(hipMemsetAsync(d_events->count, 0, sizeof(uint64_t), st));
    HIPCHECK(hipStreamSynchronize(st));
    return CC_OK;
  }
  // positions grouped by resource (only state machines with a close handler: value, election, group)
  std::vector<uint32_t> cinst(m), rlist, rstart, items;
  std::vector<std::pair<uint32_t, uint32_t>> rp;
  for (uint32_t p = 0; p < m; ++p) {
    cinst[p] = order[p].slot;
    const uint32_t r = e->inst_res[order[p].slot];
    const uint8_t ty = e->res_type[r];
    // a resource a failed deleteResource left behind is not in `resources` any more: no close handler (:253-257)
    if (e->res_zombie[r]) continue;
    if (ty == CC_RES_VALUE || ty == CC_RES_ELECTION || ty == CC_RES_GROUP) rp.emplace_back(r, p);
  }
  std::sort(rp.begin(), rp.end());
  for (size_t q = 0; q < rp.size(); ++q) {
    if (q == 0 || rp[q].first != rp[q - 1].first) {
      rlist.push_back(rp[q].first);
      rstart.push_back((uint32_t)q);
    }
    items.push_back(rp[q].second);
  }
  rstart.push_back((uint32_t)rp.size());
  const uint32_t nr = (uint32_t)rlist.size();
  // client rank of every position (order is sorted by client rank first)
  const uint32_t nc = (uint32_t)count;
  std::vector<uint32_t> pcl(m);
  for (uint32_t p = 0; p < m; ++p) pcl[p] = (uint32_t)order[p].crank;
  // device scratch: cinst | rlist | rstart | items | cnt | pcl | fail[nc], off
  const size_t n32 = (size_t)m + nr + (nr + 1) + items.size() + m + m + nc;
  uint32_t* d32 = nullptr;
  uint64_t* d_off = nullptr;
  HIPCHECK(hipMalloc(&d32, sizeof(uint32_t) * n32));
  if (hipMalloc(&d_off, sizeof(uint64_t) * (m + 1)) != hipSuccess) {
    (void)hipFree(d32);
    return set_err(CC_ERR_HIP, "hipMalloc close offsets");
  }
  std::vector<uint32_t> h32;
  h32.reserve(n32);
  h32.insert(h32.end(), cinst.begin(), cinst.end());
  h32.insert(h32.end(), rlist.begin(), rlist.end());
  h32.insert(h32.end(), rstart.begin(), rstart.end());
  h32.insert(h32.end(), items.begin(), items.end());
  h32.insert(h32.end(), (size_t)m, 0u);
  h32.insert(h32.end(), pcl.begin(), pcl.end());
  h32.insert(h32.end(), (size_t)nc, m);
  // every closed instance may drop one commit without clean() (a group member removed by close,
  // MembershipGroupState.java:36-42; a value listener): the drained leak log gets room for m more.  Only the
  // coordination handlers (groups, elections, value listeners) can leak; other engines skip the drain.
  if (e->coord_on) {
    int rc2 = drain_leaks(e);
    if (!rc2) rc2 = ensure_leak(e, m);
    if (rc2) {
      (void)hipFree(d32);
      (void)hipFree(d_off);
      return rc2;
    }
  }
  CloseArgs ca{};
  ca.cinst = d32;
  ca.m = m;
  ca.rlist = d32 + m;
  ca.rstart = d32 + m + nr;
  ca.items = d32 + m + nr + nr + 1;
  ca.cnt = d32 + m + nr + nr + 1 + items.size();
  ca.pcl = ca.cnt + m;
  ca.fail = ca.cnt + m + m;
  ca.nr = nr;
  ca.off = d_off;
  ca.inst_res = e->d_inst_res;
  ca.res_type = e->d_res_type;
  ca.inst_id = e->d_inst_id;
  ca.coord = e->coord_on ? e->d_coord : nullptr;
  ca.coord_cap = e->coord_cap;
  ca.arena = e->d_arena;
  ca.arena_n = e->d_arena_n;
  ca.arena_cap = e->coord_on ? e->arena_cap : 0;
  ca.err = e->d_err;
  ca.leak = e->d_leak;
  ca.leak_n = e->d_leak_n;
  ca.leak_cap = e->leak_cap;
  unsigned long long zero_n = 0, *d_zero = nullptr;
  if (!ca.arena_n) {  // no coordination state: no handler can publish; the scan still needs a counter
    if (hipMalloc(&d_zero, sizeof zero_n) != hipSuccess) {
      (void)hipFree(d32);
      (void)hipFree(d_off);
      return set_err(CC_ERR_HIP, "hipMalloc close counter");
    }
    ca.arena_n = d_zero;
  }
  if (d_events) {
    ca.out_cap = d_events->capacity;
    ca.out_pos = d_events->pos;
    ca.out_target = d_events->target;
    ca.out_code = d_events->code;
    ca.out_src = d_events->src;
    ca.out_tag = d_events->tag;
    ca.out_payload = d_events->payload;
    ca.out_count = d_events->count;
  }
  std::vector<uint32_t> fail(nc, m);
  hipError_t x = hipMemcpyAsync(d32, h32.data(), sizeof(uint32_t) * n32, hipMemcpyHostToDevice, st);
  if (x == hipSuccess) x = hipMemsetAsync(ca.arena_n, 0, sizeof(unsigned long long), st);
  if (x == hipSuccess && launch_close(ca, st)) x = hipGetLastError();
  if (x == hipSuccess) x = hipMemcpyAsync(fail.data(), ca.fail, sizeof(uint32_t) * nc, hipMemcpyDeviceToHost, st);
  if (x == hipSuccess) x = hipStreamSynchronize(st);
  (void)hipFree(d32);
  (void)hipFree(d_off);
  if (d_zero) (void)hipFree(d_zero);
  if (x != hipSuccess) return set_err(CC_ERR_HIP, "session close", x);
  // the host mirrors of ResourceManager.sessions and ResourceHolder.sessions (:253-261); a close that threw has
  // already removed its ResourceHolder.sessions entry but keeps its holder
  uint64_t closed = 0;
  for (uint32_t p = 0; p < m; ++p) {
    const uint32_t stop = fail[pcl[p]];
    if (p > stop) continue;  // after the close that threw: this client's loop had ended
    const uint32_t i = cinst[p], r = e->inst_res[i];
    if (!e->res_zombie[r]) e->res_sessions.erase({r, e->inst_client[i]});
    if (p == stop) continue;
    e->inst_res[i] = kNoRes;
    e->sessions.remove((int64_t)e->inst_id[i], /*movable=*/false);  // iterator.remove()
    e->inst_by_id.erase(e->inst_id[i]);
    e->used_inst.clear(i);
    ++closed;
  }
  if (h_closed) *h_closed = closed;
  return check_device_err(e);
}

// Expired sessions from cc_expire_sweep's bitmap (bit s = client session id s), closed in ascending id order:
// ResourceManager.expire (:238-247; no covered state machine overrides expire) then the close fan-out.
extern "C" int cc_sessions_expire(cc_engine* e, const uint64_t* d_bitmap, uint64_t sessions, const cc_events* d_events,
                                  void* stream, uint64_t* h_closed) {
  if (!e || (sessions && !d_bitmap)) return set_err(CC_ERR_INVALID, "null argument");
  int rc = sessions_close_args(e, d_events);
  if (rc) return rc;
  rc = quiesce(e);
  if (rc) return rc;
  hipStream_t st = stream ? (hipStream_t)stream : e->own_stream;
  e->last_stream = st;
  const uint64_t words = (sessions + 63) / 64;
  std::vector<uint64_t> bm(words);
  if (words) HIPCHECK(hipMemcpy(bm.data(), d_bitmap, sizeof(uint64_t) * words, hipMemcpyDeviceToHost));
  if (sessions % 64) bm[words - 1] &= (1ull << (sessions % 64)) - 1;  // (ids >= sessions are not sessions)
  // the expired clients in ascending id order: a client's rank is the set bits before its own (per-word prefix), so
  // each open instance finds its client's rank with one bit test -- no sorted id list, no search per instance (the
  // c5 step closed nothing after its first expiry and still spent ~0.5 ms here sorting and searching 32K ids)
  std::vector<uint64_t> pre(words + 1, 0);
  for (uint64_t wi = 0; wi < words; ++wi) pre[wi + 1] = pre[wi] + (uint64_t)__builtin_popcountll(bm[wi]);
  std::vector<std::pair<uint64_t, uint32_t>> by_client;  // (client rank, slot)
  for (uint32_t i = 0; i < e->cfg.max_instances; ++i) {
    if (e->inst_res[i] == kNoRes) continue;
    const uint64_t sid = e->inst_client[i];
    if (sid >= sessions || !((bm[sid >> 6] >> (sid & 63)) & 1)) continue;
    const uint64_t below = (sid & 63) ? bm[sid >> 6] & ((1ull << (sid & 63)) - 1) : 0ull;
    by_client.emplace_back(pre[sid >> 6] + (uint64_t)__builtin_popcountll(below), i);
  }
  return sessions_close_core(e, by_client, pre[words], d_events, st, h_closed);
}

extern "C" int cc_read_value_state(cc_engine* e, uint32_t first, uint32_t count, uint8_t* h_tag, uint64_t* h_value,
                                   uint8_t* h_has_current) {
  if (!e || (uint64_t)first + count > e->cfg.max_resources) return set_err(CC_ERR_INVALID, "range");
  int rc = quiesce(e);
  if (rc) return rc;
  std::vector<uint32_t> meta(count);
  HIPCHECK(hipMemcpy(meta.data(), e->d_val_meta + first, sizeof(uint32_t) * count, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(h_value, e->d_val_v + first, sizeof(uint64_t) * count, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < count; ++i) {
    const bool live = e->res_type[first + i] == CC_RES_VALUE;
    h_tag[i] = live ? (uint8_t)(meta[i] & 0xFF) : 0;
    h_has_current[i] = live ? (uint8_t)((meta[i] >> 8) & 1) : 0;
    if (!live) h_value[i] = 0;
  }
  return CC_OK;
}

extern "C" int cc_read_value_retained(cc_engine* e, uint32_t first, uint32_t count, uint64_t* h_index) {
  if (!e || !h_index || (uint64_t)first + count > e->cfg.max_resources) return set_err(CC_ERR_INVALID, "range");
  if (!e->d_val_live) return set_err(CC_ERR_INVALID, "engine created without CC_CFG_VALUE_RETAINED");
  int rc = quiesce(e);
  if (rc) return rc;
  HIPCHECK(hipMemcpy(h_index, e->d_val_live + first, sizeof(uint64_t) * count, hipMemcpyDeviceToHost));
  return CC_OK;
}

// The live entries of one map / set slot (all slots: ~0u), sorted by (slot, key tag, key).
namespace {
struct MapRow {
  uint32_t slot;
  uint8_t kt;
  uint64_t k;
  uint8_t vt;
  uint64_t v, ci;
};
}  // namespace
static int read_map_rows(cc_engine* e, uint32_t slot, std::vector<MapRow>& rows) {
  int rc = quiesce(e);
  if (rc) return rc;
  const uint64_t n = e->map_entries;
  std::vector<uint64_t> key(n), val(n), ci(n);
  std::vector<uint32_t> word(n);
  HIPCHECK(hipMemcpy(key.data(), e->d_tbl_key, 8 * n, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(word.data(), e->d_tbl_word, 4 * n, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(val.data(), e->d_tbl_val, 8 * n, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(ci.data(), e->d_tbl_ci, 8 * n, hipMemcpyDeviceToHost));
  std::vector<uint64_t> dl;
  uint64_t clock = 0;
  if (e->ttl_live) {  // every timer due by the engine clock has fired (MapState TTL removal)
    dl.resize(n);
    HIPCHECK(hipMemcpy(dl.data(), e->d_tbl_dl, 8 * n, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(&clock, e->d_clock, sizeof clock, hipMemcpyDeviceToHost));
  }
  static const uint8_t ktag_tag[4] = {CC_TAG_LONG, CC_TAG_INT, CC_TAG_BOOL, CC_TAG_HANDLE};
  rows.clear();
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t w = word[i];
    if (!dl.empty() && dl[i] && dl[i] <= clock) continue;
    const uint32_t s = w & kMwSlotMask;
    if ((w & kMwUsed) && (w & kMwPresent) && !(w & kMwDead) && (slot == ~0u || s == slot))
      rows.push_back(MapRow{s, ktag_tag[(w >> 17) & 3], key[i], (uint8_t)mw_vtag(w), val[i], ci[i]});
  }
  std::sort(rows.begin(), rows.end(), [](const MapRow& x, const MapRow& y) {
    return x.slot != y.slot ? x.slot < y.slot : (x.kt != y.kt ? x.kt < y.kt : x.k < y.k);
  });
  return CC_OK;
}

extern "C" int cc_read_map_entries(cc_engine* e, uint32_t slot, uint64_t cap, uint64_t* count, uint8_t* h_key_tag,
                                   uint64_t* h_key, uint8_t* h_value_tag, uint64_t* h_value, uint64_t* h_commit_index) {
  if (!e || !count || slot >= e->cfg.max_resources || !is_keyed(e->res_type[slot]))
    return set_err(CC_ERR_INVALID, "not a map or set slot");
  if (cap && (!h_key_tag || !h_key || !h_value_tag || !h_value)) return set_err(CC_ERR_INVALID, "null output");
  std::vector<MapRow> rows;
  int rc = read_map_rows(e, slot, rows);
  if (rc) return rc;
  *count = rows.size();
  const uint64_t m = std::min<uint64_t>(cap, rows.size());
  for (uint64_t i = 0; i < m; ++i) {
    h_key_tag[i] = rows[i].kt;
    h_key[i] = rows[i].k;
    h_value_tag[i] = rows[i].vt;
    h_value[i] = rows[i].v;
    if (h_commit_index) h_commit_index[i] = rows[i].ci;
  }
  return CC_OK;
}

extern "C" int cc_read_map_table(cc_engine* e, uint64_t cap, uint64_t* count, uint32_t* h_slot, uint8_t* h_key_tag,
                                 uint64_t* h_key, uint8_t* h_value_tag, uint64_t* h_value, uint64_t* h_commit_index) {
  if (!e || !count) return set_err(CC_ERR_INVALID, "null argument");
  if (!e->map_bits) return set_err(CC_ERR_INVALID, "engine without maps");
  if (cap && (!h_slot || !h_key_tag || !h_key || !h_value_tag || !h_value)) return set_err(CC_ERR_INVALID, "null output");
  std::vector<MapRow> rows;
  int rc = read_map_rows(e, ~0u, rows);
  if (rc) return rc;
  *count = rows.size();
  const uint64_t m = std::min<uint64_t>(cap, rows.size());
  for (uint64_t i = 0; i < m; ++i) {
    h_slot[i] = rows[i].slot;
    h_key_tag[i] = rows[i].kt;
    h_key[i] = rows[i].k;
    h_value_tag[i] = rows[i].vt;
    h_value[i] = rows[i].v;
    if (h_commit_index) h_commit_index[i] = rows[i].ci;
  }
  return CC_OK;
}

static int read_block(cc_engine* e, uint32_t slot, uint32_t type, CoordHdr& h, std::vector<CoordEnt>& ents, uint64_t* clock) {
  if (!e || slot >= e->cfg.max_resources || e->res_type[slot] != type || !e->coord_on)
    return set_err(CC_ERR_INVALID, "slot does not hold a resource of that type");
  int rc = quiesce(e);
  if (rc) return rc;
  std::vector<uint8_t> blk(coord_block(e->coord_cap));
  HIPCHECK(hipMemcpy(blk.data(), e->d_coord + (uint64_t)slot * coord_block(e->coord_cap), coord_block(e->coord_cap), hipMemcpyDeviceToHost));
  memcpy(&h, blk.data(), sizeof h);
  ents.resize(e->coord_cap);
  memcpy(ents.data(), blk.data() + sizeof(CoordHdr), sizeof(CoordEnt) * e->coord_cap);
  if (clock) HIPCHECK(hipMemcpy(clock, e->d_clock, sizeof(uint64_t), hipMemcpyDeviceToHost));
  return CC_OK;
}

extern "C" int cc_read_lock_state(cc_engine* e, uint32_t slot, int64_t* holder, uint64_t* holder_index,
                                  uint8_t* holder_cleaned, uint64_t cap, uint64_t* count, uint32_t* h_queue_inst,
                                  uint64_t* h_queue_index) {
  CoordHdr h;
  std::vector<CoordEnt> q;
  uint64_t clock = 0;
  int rc = read_block(e, slot, CC_RES_LOCK, h, q, &clock);
  if (rc) return rc;
  const bool held = h.flags & kCoHeld;
  if (holder) *holder = held ? (int64_t)h.who : -1;
  if (holder_index) *holder_index = held ? h.idx : 0;
  if (holder_cleaned) *holder_cleaned = held && (h.flags & kCoCleaned) ? 1 : 0;
  uint64_t n = 0;
  for (uint32_t i = 0; i < h.n; ++i) {  // timeouts due at the engine clock have fired (LockState.java:54-58)
    const CoordEnt& x = q[(h.head + i) & (e->coord_cap - 1)];
    if (x.x != kNoDeadline && x.x <= clock) continue;
    if (n < cap) {
      if (h_queue_inst) h_queue_inst[n] = x.inst;
      if (h_queue_index) h_queue_index[n] = x.idx;
    }
    ++n;
  }
  if (count) *count = n;
  return CC_OK;
}

extern "C" int cc_read_election_state(cc_engine* e, uint32_t slot, int64_t* leader, uint64_t* leader_index, uint64_t cap,
                                      uint64_t* count, uint32_t* h_listener_inst, uint64_t* h_listener_index) {
  CoordHdr h;
  std::vector<CoordEnt> q;
  int rc = read_block(e, slot, CC_RES_ELECTION, h, q, nullptr);
  if (rc) return rc;
  const bool has = h.flags & kCoHeld;
  if (leader) *leader = has ? (int64_t)h.who : -1;
  if (leader_index) *leader_index = has ? h.idx : 0;
  for (uint32_t i = 0; i < h.n && i < cap; ++i) {
    if (h_listener_inst) h_listener_inst[i] = q[i].inst;
    if (h_listener_index) h_listener_index[i] = q[i].idx;
  }
  if (count) *count = h.n;
  return CC_OK;
}

extern "C" int cc_read_group_members(cc_engine* e, uint32_t slot, uint64_t cap, uint64_t* count, uint64_t* h_ids) {
  CoordHdr h;
  std::vector<CoordEnt> q;
  int rc = read_block(e, slot, CC_RES_GROUP, h, q, nullptr);
  if (rc) return rc;
  for (uint32_t i = 0; i < h.n && i < cap; ++i)
    if (h_ids) h_ids[i] = q[i].x;
  if (count) *count = h.n;
  return CC_OK;
}

// Every commit the slot's state machine holds without having clean()ed it, ascending (the
// oracle's orc_read_retained restates the same sites).
extern "C" int cc_read_retained(cc_engine* e, uint32_t slot, uint64_t cap, uint64_t* count, uint64_t* h_index) {
  if (!e || !count || slot >= e->cfg.max_resources || e->res_type[slot] == CC_RES_NONE)
    return set_err(CC_ERR_INVALID, "unknown resource slot");
  if (cap && !h_index) return set_err(CC_ERR_INVALID, "null output");
  const uint32_t type = e->res_type[slot];
  if (type == CC_RES_VALUE && !e->d_val_live)
    return set_err(CC_ERR_INVALID, "engine created without CC_CFG_VALUE_RETAINED");
  int rc = quiesce(e);
  if (rc) return rc;
  if ((rc = drain_leaks(e))) return rc;
  std::vector<uint64_t> v;
  auto it = e->leaks.find(slot);
  if (it != e->leaks.end()) v = it->second;
  CoordHdr h{};
  std::vector<CoordEnt> q;
  if (is_coord(type) || (type == CC_RES_VALUE && e->coord_on)) {
    if ((rc = read_block(e, slot, type, h, q, nullptr))) return rc;
  }
  switch (type) {
    case CC_RES_VALUE: {  // current (AtomicValueState.java:88-157) + listeners :41-63
      uint64_t cur = 0;
      HIPCHECK(hipMemcpy(&cur, e->d_val_live + slot, sizeof cur, hipMemcpyDeviceToHost));
      if (cur) v.push_back(cur);
      for (uint32_t i = 0; i < h.n; ++i) v.push_back(q[i].idx);
      break;
    }
    case CC_RES_MAP:
    case CC_RES_SET: {  // MapState / SetState: each entry's commit (removal and TTL expiry clean it)
      uint64_t n = 0;
      if ((rc = cc_read_map_entries(e, slot, 0, &n, nullptr, nullptr, nullptr, nullptr, nullptr))) return rc;
      std::vector<uint8_t> kt(n), vt(n);
      std::vector<uint64_t> k(n), val(n), ci(n);
      if ((rc = cc_read_map_entries(e, slot, n, &n, kt.data(), k.data(), vt.data(), val.data(), ci.data()))) return rc;
      v.insert(v.end(), ci.begin(), ci.end());
      break;
    }
    case CC_RES_LOCK: {  // holder unless delete() cleaned it; waiters whose timeout has not fired (LockState :41-98)
      uint64_t n = 0, held_idx = 0;
      int64_t holder = -1;
      uint8_t cleaned = 0;
      if ((rc = cc_read_lock_state(e, slot, &holder, &held_idx, &cleaned, 0, &n, nullptr, nullptr))) return rc;
      std::vector<uint64_t> wi(n);
      if ((rc = cc_read_lock_state(e, slot, &holder, &held_idx, &cleaned, n, &n, nullptr, wi.data()))) return rc;
      if (holder >= 0 && !cleaned) v.push_back(held_idx);
      v.insert(v.end(), wi.begin(), wi.end());
      break;
    }
    case CC_RES_ELECTION:  // leader unless delete() cleaned it + listeners (LeaderElectionState :35-108)
      if ((h.flags & kCoHeld) && !(h.flags & kCoCleaned)) v.push_back(h.idx);
      for (uint32_t i = 0; i < h.n; ++i) v.push_back(q[i].idx);
      break;
    case CC_RES_GROUP:  // members + pending schedule commits (MembershipGroupState :47-103)
      for (uint32_t i = 0; i < h.n; ++i) v.push_back(q[i].idx);
      for (const auto& g : e->gtimers)
        if (g.slot == slot) v.push_back(g.idx);
      break;
    case CC_RES_MULTIMAP:  // every Put (MultiMapState.put :68-91 neither cleans nor closes it): the leak lists
      break;
    case CC_RES_QUEUE:  // elements, less the head element() clean()ed (QueueState :51-199)
      for (uint32_t i = 0; i < h.n; ++i) {
        const CoordEnt& x = q[(h.head + i) & (e->coord_cap - 1)];
        if (!(x.pad & kQCleaned)) v.push_back(x.idx);
      }
      break;
  }
  std::sort(v.begin(), v.end());
  *count = v.size();
  for (uint64_t i = 0; i < v.size() && i < cap; ++i) h_index[i] = v[i];
  return CC_OK;
}

// Every slot's retained commits at once (the union of cc_read_retained over all resource slots) as a bitmap over
// [first, first + count), built on the device (retained.hip); the compactor's per-batch feed.
extern "C" int cc_retained_bitmap(cc_engine* e, uint64_t first, uint64_t count, uint64_t* d_bitmap, uint64_t* h_count) {
  if (!e || (count && !d_bitmap) || ((uintptr_t)d_bitmap & 7)) return set_err(CC_ERR_INVALID, "null or misaligned bitmap");
  if (count == 0) {
    if (h_count) *h_count = 0;
    return CC_OK;
  }
  const uint64_t slots = (uint64_t)e->sb << kSbShift;
  bool values = false;
  for (uint32_t s = 0; s < e->cfg.max_resources; ++s) values |= e->res_type[s] == CC_RES_VALUE;
  if (values && !e->d_val_live) return set_err(CC_ERR_INVALID, "engine created without CC_CFG_VALUE_RETAINED");
  int rc = quiesce(e);
  if (rc) return rc;
  if ((rc = drain_leaks(e))) return rc;
  std::vector<uint64_t> host;  // pending MembershipGroup.schedule commits + commits dropped without clean()
  for (const auto& g : e->gtimers)
    if (g.idx >= first && g.idx - first < count) host.push_back(g.idx);
  for (const auto& kv : e->leaks)
    for (uint64_t i : kv.second)
      if (i >= first && i - first < count) host.push_back(i);
  uint64_t* d_list = nullptr;
  unsigned long long* d_total = nullptr;
  HIPCHECK(hipMalloc(&d_total, sizeof(unsigned long long) * (1 + host.size())));
  d_list = reinterpret_cast<uint64_t*>(d_total + 1);
  hipError_t x = host.empty() ? hipSuccess
                              : hipMemcpyAsync(d_list, host.data(), 8 * host.size(), hipMemcpyHostToDevice, e->own_stream);
  RetainedArgs ra{};
  ra.res_type = e->d_res_type;
  ra.slots = (uint32_t)std::min<uint64_t>(slots, e->cfg.max_resources);
  ra.val_live = values ? e->d_val_live : nullptr;
  ra.tbl_word = e->map_bits ? e->d_tbl_word : nullptr;
  ra.tbl_ci = e->d_tbl_ci;
  ra.tbl_dl = e->ttl_live ? e->d_tbl_dl : nullptr;
  ra.entries = e->map_entries;
  ra.coord = e->coord_on ? e->d_coord : nullptr;
  ra.coord_cap = e->coord_cap;
  ra.clock = e->d_clock;
  ra.list = d_list;
  ra.list_n = host.size();
  ra.first = first;
  ra.count = count;
  ra.bitmap = d_bitmap;
  ra.total = d_total;
  if (x == hipSuccess && launch_retained(ra, e->own_stream)) x = hipGetLastError();
  unsigned long long total = 0;
  if (x == hipSuccess) x = hipMemcpyAsync(&total, d_total, sizeof total, hipMemcpyDeviceToHost, e->own_stream);
  if (x == hipSuccess) x = hipStreamSynchronize(e->own_stream);
  (void)hipFree(d_total);
  if (x != hipSuccess) return set_err(CC_ERR_HIP, "retained bitmap", x);
  if (h_count) *h_count = total;
  return CC_OK;
}

extern "C" int cc_advance_time_events(cc_engine* e, uint64_t now, const cc_events* d_events) {
  if (!e) return CC_ERR_INVALID;
  int rc = quiesce(e);
  if (rc) return rc;
  if (e->coord_on) {  // due group timers fire in (deadline, id) order; events at pos 0xFFFFFFFF (no commit)
    HIPCHECK(hipMemsetAsync(e->d_ev_total, 0, sizeof(unsigned long long), e->own_stream));
    std::sort(e->gtimers.begin(), e->gtimers.end(), [](const cc_engine::GroupTimer& x, const cc_engine::GroupTimer& y) {
      return x.deadline != y.deadline ? x.deadline < y.deadline : x.id < y.id;
    });
    uint64_t clk = 0;  // the reference fires everything due by max(clock, now)
    HIPCHECK(hipMemcpy(&clk, e->d_clock, sizeof clk, hipMemcpyDeviceToHost));
    const uint64_t thr = std::max(clk, now);
    size_t k = 0;
    for (; k < e->gtimers.size() && e->gtimers[k].deadline <= thr; ++k) {
      const auto& gt = e->gtimers[k];
      if (launch_group_fire(e->d_coord, e->coord_cap, gt.slot, gt.member, gt.tag, gt.payload, 0xFFFFFFFFu, e->d_ev_total, d_events, e->d_err,
                            e->own_stream))
        return set_err(CC_ERR_HIP, "group timer launch", hipGetLastError());
    }
    e->gtimers.erase(e->gtimers.begin(), e->gtimers.begin() + (ptrdiff_t)k);
    if (d_events) HIPCHECK(hipMemcpyAsync(d_events->count, e->d_ev_total, sizeof(uint64_t), hipMemcpyDeviceToDevice, e->own_stream));
  }
  if (e->map_bits && e->ttl_live) {  // map timers due by the new clock fire: their keys leave (sizes, small maps)
    uint64_t clk = 0;
    HIPCHECK(hipMemcpy(&clk, e->d_clock, sizeof clk, hipMemcpyDeviceToHost));
    if (now > clk) {
      rc = ttl_flush(e, nullptr, 0, 0, 0, now, e->own_stream);
      if (rc) return rc;
    }
  }
  if (launch_clock_advance(nullptr, 0, now, e->d_clock, e->own_stream)) return set_err(CC_ERR_HIP, "clock", hipGetLastError());
  HIPCHECK(hipStreamSynchronize(e->own_stream));
  return check_device_err(e);
}

extern "C" int cc_advance_time(cc_engine* e, uint64_t now) { return cc_advance_time_events(e, now, nullptr); }

static const char* kKernelNames[K_NUM] = {"k_part_tile", "k_apply_value", "k_unpermute", "k_apply_map", "k_map_hot",
                                          "k_apply_coord", "k_events"};

// ---- snapshot / restore (restart without replaying the whole log) -------------------
// Layout: SnapHdr, then the sections below in order, each a u64 byte count followed by the bytes.  Host
// mirrors travel with the device arrays so a fresh engine of the same configuration resumes exactly.
namespace {
constexpr uint64_t kSnapMagic = 0x37304E5053434343ull;  // "CCCSPN07"
constexpr uint32_t kSnapRetained = 4u;                   // SnapHdr.flags: CC_CFG_VALUE_RETAINED section present
struct SnapHdr {
  uint64_t magic;
  uint32_t abi, flags;  // flags: 1 coord blocks, 2 map TTL mode, 4 retained value commits
  uint32_t max_resources, max_instances, map_bits, sb;
  uint64_t applied;
  uint32_t coord_cap, pad;
};
struct Section {
  void* dev;
  void* host;
  uint64_t bytes;
};
}  // namespace

static std::vector<Section> snap_sections(cc_engine* e) {
  const uint64_t slots = (uint64_t)e->sb << kSbShift, mi = e->cfg.max_instances, mr = e->cfg.max_resources;
  std::vector<Section> v = {
      {nullptr, e->res_type.data(), slots},
      {nullptr, e->inst_res.data(), 4 * mi},
      {nullptr, e->inst_id.data(), 8 * mi},
      {nullptr, e->inst_client.data(), 8 * mi},
      {nullptr, e->sb_kind.data(), e->sb},
      {e->d_inst_res, nullptr, 4 * mi},
      {e->d_res_type, nullptr, slots},
      {e->d_val_meta, nullptr, 4 * slots},
      {e->d_val_v, nullptr, 8 * slots},
      {e->d_sb_kind, nullptr, e->sb},
      {e->d_inst_id, nullptr, 8 * mi},
      {e->d_clock, nullptr, 8},
      {nullptr, e->res_id.data(), 8 * slots},
      {nullptr, e->res_key.data(), 8 * slots},
      {nullptr, e->res_has_key.data(), slots},
      {nullptr, e->res_zombie.data(), slots},
  };
  if (e->d_val_live) v.push_back({e->d_val_live, nullptr, 8 * slots});
  if (e->map_bits) {
    const uint64_t n = e->map_entries;
    v.push_back({e->d_tbl_key, nullptr, 8 * n});
    v.push_back({e->d_tbl_word, nullptr, 4 * n});
    v.push_back({e->d_tbl_val, nullptr, 8 * n});
    v.push_back({e->d_tbl_ci, nullptr, 8 * n});
    v.push_back({e->d_tbl_ins, nullptr, 8 * n});
    v.push_back({e->d_tbl_dl, nullptr, 8 * n});
    v.push_back({e->d_mw_peak, nullptr, 4 * mr});
    v.push_back({e->d_mw_drop, nullptr, 8 * mr});
    v.push_back({e->d_mw_cgen, nullptr, 8 * mr});
    v.push_back({e->d_cset, nullptr, sizeof(CsetEnt) * (e->cset_mask + 1)});
    v.push_back({e->d_cset_full, nullptr, 4});
    v.push_back({e->d_tbl_claim, nullptr, 8 * n});
    v.push_back({e->d_lvl_at, nullptr, 8ull * kLvlSlots * mr});
    v.push_back({e->d_msize, nullptr, 4 * mr});
    v.push_back({e->d_mpcap, nullptr, 4 * mr});
    v.push_back({e->d_msm, nullptr, sizeof(SmallMap) * mr});
    v.push_back({e->d_mbig, nullptr, sizeof(BigMap) * kBigSlots});
    v.push_back({e->d_msmall, nullptr, mr});
  }
  if (e->coord_on) v.push_back({e->d_coord, nullptr, coord_block(e->coord_cap) * slots});
  return v;
}

// ---- the prefix apply's checkpoint (host_path.hip cc_apply_batch_host_prefix) -------------------------------------
// The device sections of a snapshot (the state every batch apply may write), the applied index and the leak log's
// count, copied device to device into one engine-owned buffer; the host fields a batch moves beside them.
static std::vector<Section> ckpt_sections(cc_engine* e) {
  std::vector<Section> v;
  for (const Section& x : snap_sections(e))
    if (x.dev) v.push_back(x);
  v.push_back({e->d_last_index, nullptr, sizeof(uint64_t)});
  if (e->d_leak_n) v.push_back({e->d_leak_n, nullptr, sizeof(unsigned long long)});
  return v;
}

int cc::ckpt_save(cc_engine* e) {
  int rc = quiesce(e);
  if (rc) return rc;
  const auto secs = ckpt_sections(e);
  uint64_t need = 0;
  for (const Section& x : secs) need += (x.bytes + 255) & ~255ull;
  if (need > e->ckpt_bytes) {
    if (e->d_ckpt) HIPCHECK(hipFree(e->d_ckpt));
    e->d_ckpt = nullptr;
    e->ckpt_bytes = 0;
    HIPCHECK(hipMalloc(&e->d_ckpt, need));
    e->ckpt_bytes = need;
  }
  uint8_t* p = (uint8_t*)e->d_ckpt;
  for (const Section& x : secs) {
    HIPCHECK(hipMemcpyAsync(p, x.dev, x.bytes, hipMemcpyDeviceToDevice, e->last_stream));
    p += (x.bytes + 255) & ~255ull;
  }
  HIPCHECK(hipStreamSynchronize(e->last_stream));
  e->ckpt.applied = e->applied;
  e->ckpt.applied_pending = e->applied_pending;
  e->ckpt.ttl_live = e->ttl_live;
  e->ckpt.small_live = e->small_live;
  e->ckpt.gtimers = e->gtimers;
  e->ckpt.gtimer_seq = e->gtimer_seq;
  e->ckpt.leaks = e->leaks;
  return CC_OK;
}

int cc::ckpt_restore(cc_engine* e) {
  (void)hipStreamSynchronize(e->last_stream);  // (a failed call may have left work queued)
  if (e->side_st) (void)hipStreamSynchronize(e->side_st);
  uint8_t* p = (uint8_t*)e->d_ckpt;
  for (const Section& x : ckpt_sections(e)) {
    HIPCHECK(hipMemcpyAsync(x.dev, p, x.bytes, hipMemcpyDeviceToDevice, e->last_stream));
    p += (x.bytes + 255) & ~255ull;
  }
  HIPCHECK(hipMemsetAsync(e->d_err, 0, sizeof(uint32_t), e->last_stream));
  if (e->map_bits) HIPCHECK(hipMemsetAsync(e->d_msm_left, 0, 3ull * e->cfg.max_resources, e->last_stream));
  HIPCHECK(hipStreamSynchronize(e->last_stream));
  e->applied = e->ckpt.applied;
  e->applied_pending = e->ckpt.applied_pending;
  e->ttl_live = e->ckpt.ttl_live;
  e->small_live = e->ckpt.small_live;
  e->gtimers = e->ckpt.gtimers;
  e->gtimer_seq = e->ckpt.gtimer_seq;
  e->leaks = e->ckpt.leaks;
  e->rep_pending[0] = e->rep_pending[1] = false;
  e->pend = false;
  return CC_OK;
}

static uint64_t leak_entries(const cc_engine* e) {
  uint64_t n = 0;
  for (const auto& kv : e->leaks) n += kv.second.size();
  return n;
}

extern "C" int cc_snapshot_size(cc_engine* e, uint64_t* bytes) {
  if (!e || !bytes) return CC_ERR_INVALID;
  int rc = quiesce(e);  // the leak log's entries are counted from the host lists
  if (rc) return rc;
  if ((rc = drain_leaks(e))) return rc;
  std::vector<uint8_t> sess;
  e->sessions.save(sess);
  uint64_t total = sizeof(SnapHdr) + 16 + e->gtimers.size() * sizeof(cc_engine::GroupTimer) + 8 +
                   e->res_sessions.size() * 24 + 8 + leak_entries(e) * 16 + 8 + sess.size() + 8 + e->hh.size() * 16;
  for (const Section& x : snap_sections(e)) total += 8 + x.bytes;
  *bytes = total;
  return CC_OK;
}

extern "C" int cc_snapshot_save(cc_engine* e, void* h_buf, uint64_t cap) {
  if (!e || !h_buf) return CC_ERR_INVALID;
  int rc = cc_sync(e);  // results of every batch so far are final (and the applied watermark is current)
  if (rc) return rc;
  uint64_t need = 0;
  if ((rc = cc_snapshot_size(e, &need))) return rc;
  if (cap < need) return set_err(CC_ERR_CAPACITY, "snapshot buffer smaller than cc_snapshot_size");
  SnapHdr h{};
  h.magic = kSnapMagic;
  h.abi = CC_ABI_VERSION;
  h.flags = (e->coord_on ? 1u : 0u) | (e->ttl_live ? 2u : 0u) | (e->d_val_live ? kSnapRetained : 0u);
  h.max_resources = e->cfg.max_resources;
  h.max_instances = e->cfg.max_instances;
  h.map_bits = e->map_bits;
  h.sb = e->sb;
  h.applied = e->applied;
  h.coord_cap = e->coord_cap;
  uint8_t* p = (uint8_t*)h_buf;
  memcpy(p, &h, sizeof h);
  p += sizeof h;
  for (const Section& x : snap_sections(e)) {
    memcpy(p, &x.bytes, 8);
    p += 8;
    if (x.dev) HIPCHECK(hipMemcpy(p, x.dev, x.bytes, hipMemcpyDeviceToHost));
    else memcpy(p, x.host, x.bytes);
    p += x.bytes;
  }
  {
    std::vector<uint8_t> sess;  // ResourceManager.sessions' java.util.HashMap structure (close order)
    e->sessions.save(sess);
    const uint64_t sb = sess.size();
    memcpy(p, &sb, 8);
    memcpy(p + 8, sess.data(), sb);
    p += 8 + sb;
    const uint64_t nh = e->hh.size();  // String.hashCode of HANDLE keys: (handle, hash) pairs
    memcpy(p, &nh, 8);
    p += 8;
    for (const auto& kv : e->hh) {
      const uint64_t t[2] = {kv.first, (uint64_t)(uint32_t)kv.second};
      memcpy(p, t, 16);
      p += 16;
    }
  }
  const uint64_t ng = e->gtimers.size();  // pending MembershipGroup.schedule timers
  memcpy(p, &ng, 8);
  memcpy(p + 8, &e->gtimer_seq, 8);
  if (ng) memcpy(p + 16, e->gtimers.data(), ng * sizeof(cc_engine::GroupTimer));
  p += 16 + ng * sizeof(cc_engine::GroupTimer);
  const uint64_t ns = e->res_sessions.size();  // ResourceHolder.sessions: (slot, client, instance id) triples
  memcpy(p, &ns, 8);
  p += 8;
  for (const auto& kv : e->res_sessions) {
    const uint64_t t[3] = {kv.first.first, kv.first.second, kv.second};
    memcpy(p, t, 24);
    p += 24;
  }
  const uint64_t nl = leak_entries(e);  // commits dropped without clean(): (slot, log index) pairs
  memcpy(p, &nl, 8);
  p += 8;
  for (const auto& kv : e->leaks)
    for (uint64_t idx : kv.second) {
      const uint64_t t[2] = {kv.first, idx};
      memcpy(p, t, 16);
      p += 16;
    }
  return CC_OK;
}

// Remaining bytes from p hold at least `count` records of `rec` bytes (no pointer arithmetic on the count: a corrupt
// count cannot wrap the check).
static bool snap_room(const uint8_t* p, const uint8_t* end, uint64_t count, uint64_t rec) {
  return p <= end && count <= (uint64_t)(end - p) / rec;
}

extern "C" int cc_snapshot_restore(cc_engine* e, const void* h_buf, uint64_t size) {
  if (!e || !h_buf || size < sizeof(SnapHdr)) return set_err(CC_ERR_INVALID, "snapshot too small");
  SnapHdr h;
  memcpy(&h, h_buf, sizeof h);
  if (h.magic != kSnapMagic || h.abi != CC_ABI_VERSION) return set_err(CC_ERR_INVALID, "not a snapshot of this engine ABI");
  if (h.max_resources != e->cfg.max_resources || h.max_instances != e->cfg.max_instances || h.map_bits != e->map_bits ||
      h.sb != e->sb || h.coord_cap != e->coord_cap)
    return set_err(CC_ERR_INVALID, "snapshot configuration (max_resources/max_instances/map_capacity/coord_cap) differs");
  if (((h.flags & kSnapRetained) != 0) != (e->d_val_live != nullptr))  // the section lists would differ
    return set_err(CC_ERR_INVALID, "snapshot and engine differ in CC_CFG_VALUE_RETAINED");
  if (e->coord_on && !(h.flags & 1u))  // the engine's coordination blocks have no section to come from
    return set_err(CC_ERR_INVALID, "snapshot has no coordination state but the engine does");
  const uint8_t* const base = (const uint8_t*)h_buf + sizeof h;
  const uint8_t* const end = (const uint8_t*)h_buf + size;
  // 1. validate the whole buffer before any engine state changes: a rejected snapshot leaves the engine as it was
  std::vector<uint64_t> sizes;
  for (const Section& x : snap_sections(e)) sizes.push_back(x.bytes);
  if ((h.flags & 1u) && !e->coord_on) sizes.push_back(coord_block(e->coord_cap) * ((uint64_t)e->sb << kSbShift));
  const uint8_t* p = base;
  for (uint64_t want : sizes) {
    uint64_t b = 0;
    if (!snap_room(p, end, 1, 8)) return set_err(CC_ERR_INVALID, "snapshot truncated");
    memcpy(&b, p, 8);
    p += 8;
    if (b != want || !snap_room(p, end, b, 1)) return set_err(CC_ERR_INVALID, "snapshot section size mismatch");
    p += b;
  }
  uint64_t sbytes = 0, nh = 0;
  cc::JavaLongHashMap sessions;
  if (!snap_room(p, end, 1, 8)) return set_err(CC_ERR_INVALID, "snapshot truncated");
  memcpy(&sbytes, p, 8);
  p += 8;
  if (!snap_room(p, end, sbytes, 1) || sessions.load(p, sbytes) != sbytes)
    return set_err(CC_ERR_INVALID, "snapshot: malformed sessions table");
  p += sbytes;
  if (!snap_room(p, end, 1, 8)) return set_err(CC_ERR_INVALID, "snapshot truncated");
  memcpy(&nh, p, 8);
  p += 8;
  if (!snap_room(p, end, nh, 16)) return set_err(CC_ERR_INVALID, "snapshot truncated (handle hashes)");
  const uint8_t* const hh_at = p;
  p += nh * 16;
  uint64_t ng = 0, ns = 0, nl = 0;
  if (!snap_room(p, end, 2, 8)) return set_err(CC_ERR_INVALID, "snapshot truncated");
  memcpy(&ng, p, 8);
  p += 16;
  if (!snap_room(p, end, ng, sizeof(cc_engine::GroupTimer))) return set_err(CC_ERR_INVALID, "snapshot truncated (group timers)");
  p += ng * sizeof(cc_engine::GroupTimer);
  if (!snap_room(p, end, 1, 8)) return set_err(CC_ERR_INVALID, "snapshot truncated");
  memcpy(&ns, p, 8);
  p += 8;
  if (!snap_room(p, end, ns, 24)) return set_err(CC_ERR_INVALID, "snapshot truncated (resource sessions)");
  p += ns * 24;
  if (!snap_room(p, end, 1, 8)) return set_err(CC_ERR_INVALID, "snapshot truncated");
  memcpy(&nl, p, 8);
  p += 8;
  if (!snap_room(p, end, nl, 16)) return set_err(CC_ERR_INVALID, "snapshot truncated (leak lists)");
  // 2. apply
  int rc = quiesce(e);
  if (rc) return rc;
  if ((h.flags & 1u) && (rc = ensure_ext(e, true))) return rc;
  e->ttl_live = (h.flags & 2u) != 0;
  p = base;
  for (const Section& x : snap_sections(e)) {
    p += 8;
    if (x.dev) HIPCHECK(hipMemcpy(x.dev, p, x.bytes, hipMemcpyHostToDevice));
    else memcpy(x.host, p, x.bytes);
    p += x.bytes;
  }
  p = hh_at + nh * 16;  // (the sessions table and handle hashes were parsed above)
  memcpy(&e->gtimer_seq, p + 8, 8);
  p += 16;
  e->gtimers.resize(ng);
  if (ng) memcpy(e->gtimers.data(), p, ng * sizeof(cc_engine::GroupTimer));
  p += ng * sizeof(cc_engine::GroupTimer) + 8;
  e->res_sessions.clear();
  for (uint64_t i = 0; i < ns; ++i, p += 24) {
    uint64_t t[3];
    memcpy(t, p, 24);
    e->res_sessions[{(uint32_t)t[0], t[1]}] = t[2];
  }
  p += 8;
  e->leaks.clear();
  for (uint64_t i = 0; i < nl; ++i, p += 16) {
    uint64_t t[2];
    memcpy(t, p, 16);
    e->leaks[(uint32_t)t[0]].push_back(t[1]);
  }
  if (e->d_leak_n) HIPCHECK(hipMemset(e->d_leak_n, 0, sizeof(unsigned long long)));
  // the control-plane maps and slot occupancy follow from the restored arrays
  e->keys.clear();
  e->res_by_id.clear();
  e->inst_by_id.clear();
  e->used_res.reset(e->cfg.max_resources);
  e->used_inst.reset(e->cfg.max_instances);
  for (uint32_t s = 0; s < e->cfg.max_resources; ++s) {
    if (e->res_type[s] == CC_RES_NONE) continue;
    e->used_res.set(s);
    if (e->res_has_key[s]) e->keys[e->res_key[s]] = e->res_id[s];
    if (!e->res_zombie[s]) e->res_by_id[e->res_id[s]] = s;
  }
  for (auto& og : e->open_grp) og.clear();  // groups of one coordination type with room (manager.hip)
  for (uint32_t g = 0; g * 64 < e->cfg.max_resources; ++g) {
    uint32_t type = CC_RES_NONE, used = 0;
    bool mixed = false;
    for (uint32_t s = g * 64; s < g * 64 + 64 && s < e->cfg.max_resources; ++s) {
      if (e->res_type[s] == CC_RES_NONE && !e->used_res.test(s)) continue;
      ++used;
      if (type == CC_RES_NONE) type = e->res_type[s];
      else if (type != e->res_type[s]) mixed = true;
    }
    if (!mixed && type != CC_RES_NONE && used < 64 && type < 16) e->open_grp[type].insert(g);
  }
  for (uint32_t i = 0; i < e->cfg.max_instances; ++i) {
    if (e->inst_res[i] == kNoRes) continue;
    e->used_inst.set(i);
    e->inst_by_id[e->inst_id[i]] = i;
  }
  e->applied = h.applied;
  e->applied_pending = false;
  HIPCHECK(hipMemcpy(e->d_last_index, &e->applied, sizeof(uint64_t), hipMemcpyHostToDevice));
  e->has_sets = std::find(e->res_type.begin(), e->res_type.end(), (uint8_t)CC_RES_SET) != e->res_type.end();
  e->has_values = e->has_values || std::find(e->res_type.begin(), e->res_type.end(), (uint8_t)CC_RES_VALUE) != e->res_type.end();
  e->has_mmaps = std::find(e->res_type.begin(), e->res_type.end(), (uint8_t)CC_RES_MULTIMAP) != e->res_type.end();
  if (e->has_mmaps && (rc = ensure_leak(e, kLeakCap))) return rc;
  e->sessions = std::move(sessions);
  e->small_live = e->map_bits && !e->ttl_live;  // (the next sub-batch recounts the maps still small)
  if (e->map_bits)  // (no replay is pending here: the restored snapshot flags start with no exit marks)
    HIPCHECK(hipMemset(e->d_msm_left, 0, 3ull * e->cfg.max_resources));
  if (e->small_live) {  // (ctl[1] nonzero until that recount: see resource creation)
    const uint32_t pending[2] = {0, 1};
    HIPCHECK(hipMemcpy(e->d_sm_ctl, pending, sizeof pending, hipMemcpyHostToDevice));
  }
  {
    std::vector<uint64_t> hk(nh);
    std::vector<int32_t> hv(nh);
    const uint8_t* q = hh_at;
    for (uint64_t i = 0; i < nh; ++i, q += 16) {
      uint64_t t[2];
      memcpy(t, q, 16);
      hk[i] = t[0];
      hv[i] = (int32_t)(uint32_t)t[1];
    }
    e->hh.clear();
    if (nh && (rc = cc_handle_hashes(e, hk.data(), hv.data(), nh))) return rc;
  }
  HIPCHECK(hipMemset(e->d_err, 0, sizeof(uint32_t)));
  return CC_OK;
}

extern "C" int cc_profile_enable(cc_engine* e, int on) {
  if (!e) return CC_ERR_INVALID;
  e->prof_on = on != 0;
  return CC_OK;
}

extern "C" int cc_profile_reset(cc_engine* e) {
  if (!e) return CC_ERR_INVALID;
  HIPCHECK(hipSetDevice(e->device));
  drain_profile(e);
  for (int k = 0; k < K_NUM; ++k) {
    e->prof_ms[k] = 0;
    e->prof_n[k] = 0;
  }
  return CC_OK;
}

extern "C" int cc_debug_phases(cc_engine* e, int kernel, uint64_t* ticks) {
#ifdef CC_PHASE_TIMING
  if (e && ticks && kernel == 64) {  // diagnostics: k_apply_coord's per-workgroup (start, end), 2 x 4096 entries
    HIPCHECK(hipStreamSynchronize(e->last_stream));
    return phase_read_coord_wg(ticks);
  }
#endif
  if (!e || !ticks || kernel < 0 || kernel >= K_NUM) return CC_ERR_INVALID;
  HIPCHECK(hipSetDevice(e->device));
  HIPCHECK(hipStreamSynchronize(e->last_stream));
  const int rc = phase_read(kernel, ticks);
  return rc == CC_OK ? CC_OK : set_err(rc, "phase clocks: not a CC_PHASE_TIMING build, or not instrumented kernel");
}

extern "C" int cc_profile_read(cc_engine* e, int kernel, double* total_ms, uint64_t* launches, const char** name) {
  if (!e || kernel < 0 || kernel >= K_NUM) return CC_ERR_INVALID;
  HIPCHECK(hipSetDevice(e->device));
  drain_profile(e);
  if (total_ms) *total_ms = e->prof_ms[kernel];
  if (launches) *launches = e->prof_n[kernel];
  if (name) *name = kKernelNames[kernel];
  return CC_OK;
}
