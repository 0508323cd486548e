/*
 * copycat_apply.h — C-ABI of the MI355X batched commit-apply engine.
 *
 * This is the drop-in boundary for ONE hot path of madjam/copycat (Atomix 0.1.0 on Copycat 1.0.0-beta4):
 * applying a batch of committed Raft log entries to many multiplexed resource state machines.
 * In the reference that path is, per committed entry, on one state-machine thread:
 *
 *   Copycat apply loop [not vendored]
 *     -> ResourceManager.operateResource           manager/src/main/java/io/atomix/manager/ResourceManager.java:56-72
 *     -> ResourceManagerStateMachineExecutor.execute manager/.../ResourceManagerStateMachineExecutor.java:90-102
 *     -> ResourceStateMachineExecutor.executeCommand resource/.../ResourceStateMachineExecutor.java:73-91
 *     -> AtomicValueState / MapState / LockState / LeaderElectionState / MembershipGroupState methods
 *
 * The engine replaces that chain for a whole batch: the host encodes the batch into the SoA columns of
 * cc_batch (one row per commit, in log order) and calls cc_apply_batch(); hand-written gfx950 kernels
 * produce one (status, value) row per commit plus an event stream.
 *
 * Conventions
 *  - Every call returns an int: CC_OK (0) or a negative CC_ERR_* code.  Per-commit failures (the Java
 *    exceptions) never fail the call: they are reported in the commit's status byte.
 *  - A handle is used from one host thread at a time (the reference applies on one thread too).
 *  - Pointers named d_* are device (HBM) pointers; h_* are host pointers.  `stream` is a hipStream_t
 *    passed as void* (NULL = the legacy default stream).  Device calls are stream-ordered and
 *    asynchronous; results are final after cc_sync() or a sync on the caller's stream.
 *  - No torch, no C++ types: plain C so that a JNI / Panama FFM / ctypes stub can bind it
 *    (INTEGRATION.md shows the bindings).
 */
#ifndef COPYCAT_APPLY_H
#define COPYCAT_APPLY_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CC_ABI_VERSION 5

/* ---- return codes ------------------------------------------------------------------------------ */
#define CC_OK               0
#define CC_ERR_INVALID     -1  /* bad argument / handle */
#define CC_ERR_HIP         -2  /* HIP runtime error (message: cc_last_error) */
#define CC_ERR_CAPACITY    -3  /* batch / resource / instance / table capacity exceeded */
#define CC_ERR_UNSUPPORTED -4  /* an op or resource type this build does not run on the GPU */
#define CC_ERR_STATE       -5  /* engine state corrupt (a device-side check failed) */

/* ---- resource (state machine) types; ResourceManager.getResource instantiates one per key ----------
 * ResourceManager.java:92 `commit.operation().type().newInstance()`                                    */
#define CC_RES_NONE      0
#define CC_RES_VALUE     1  /* AtomicValueState  atomic/.../state/AtomicValueState.java:32 (also DistributedAtomicLong) */
#define CC_RES_MAP       2  /* MapState          collections/.../state/MapState.java:32 */
#define CC_RES_LOCK      3  /* LockState         coordination/.../state/LockState.java:33 */
#define CC_RES_ELECTION  4  /* LeaderElectionState coordination/.../state/LeaderElectionState.java:31 */
#define CC_RES_GROUP     5  /* MembershipGroupState coordination/.../state/MembershipGroupState.java:33 */
#define CC_RES_SET       6  /* SetState          collections/.../state/SetState.java:32 (shares the map table) */
#define CC_RES_QUEUE     7  /* QueueState        collections/.../state/QueueState.java:33 (a FIFO of CC_QUEUE_CAP) */
#define CC_RES_MULTIMAP  8  /* MultiMapState     collections/.../state/MultiMapState.java:30 (shares the map table) */
#define CC_QUEUE_CAP    64

/* ---- op codes = Catalyst @SerializeWith ids of the inner operation ------------- */
#define CC_OP_DELETE            1   /* ResourceStateMachine.DeleteCommand (no wire id) ResourceStateMachine.java:53 */
/* AtomicValueCommands.java:93-260 */
#define CC_OP_VALUE_GET        50   /* query */
#define CC_OP_VALUE_SET        51
#define CC_OP_VALUE_CAS        52   /* CompareAndSet(expect=a, update=b) */
#define CC_OP_VALUE_GETANDSET  53
#define CC_OP_VALUE_LISTEN     54
#define CC_OP_VALUE_UNLISTEN   55
/* MapCommands.java:134-450 */
#define CC_OP_MAP_CONTAINSKEY   60  /* query */
#define CC_OP_MAP_CONTAINSVALUE 61  /* query */
#define CC_OP_MAP_PUT           62
#define CC_OP_MAP_PUTIFABSENT   63
#define CC_OP_MAP_GET           64  /* query */
#define CC_OP_MAP_GETORDEFAULT  65  /* query */
#define CC_OP_MAP_REMOVE        66
#define CC_OP_MAP_REMOVEIFPRESENT 67
#define CC_OP_MAP_REPLACE       68
#define CC_OP_MAP_REPLACEIFPRESENT 69
#define CC_OP_MAP_ISEMPTY       70  /* query */
#define CC_OP_MAP_SIZE          71  /* query */
#define CC_OP_MAP_CLEAR         72
/* LeaderElectionCommands.java:80-99 */
/* QueueState (collections/.../state/QueueCommands.java:133-235): the element travels in operand a */
#define CC_OP_QUEUE_CONTAINS   90  /* query */
#define CC_OP_QUEUE_ADD        91
#define CC_OP_QUEUE_OFFER      92
#define CC_OP_QUEUE_PEEK       93  /* query */
#define CC_OP_QUEUE_POLL       94
#define CC_OP_QUEUE_ELEMENT    95
#define CC_OP_QUEUE_REMOVE     96  /* a = element, or NULL: remove the head */
#define CC_OP_QUEUE_SIZE       97  /* query */
#define CC_OP_QUEUE_ISEMPTY    98  /* query */
#define CC_OP_QUEUE_CLEAR      99
/* SetState (collections/.../state/SetCommands.java:133-238): the element travels in the key column (key tag in
 * CC_FLAGS), the ttl of Add in aux */
#define CC_OP_SET_CONTAINS     100  /* query */
#define CC_OP_SET_ADD          101
#define CC_OP_SET_REMOVE       102
#define CC_OP_SET_SIZE         103  /* query */
#define CC_OP_SET_ISEMPTY      104  /* query */
#define CC_OP_SET_CLEAR        105
/* MultiMapState (collections/.../state/MultiMapCommands.java:205-441): the key travels in the key column (key tag
 * in CC_FLAGS), the value in operand a, Put's ttl in aux.  ContainsEntry and ContainsValue have no handler in
 * MultiMapState (unknown operation).  MultiMapState.put never stores its value (:76-82): the state is the set of
 * keys put and not removed since; every Put commit stays retained (never cleaned or closed).               */
#define CC_OP_MMAP_CONTAINSKEY   75  /* query */
#define CC_OP_MMAP_CONTAINSENTRY 76  /* query (no handler) */
#define CC_OP_MMAP_CONTAINSVALUE 77  /* query (no handler) */
#define CC_OP_MMAP_PUT           78
#define CC_OP_MMAP_GET           79  /* query */
#define CC_OP_MMAP_REMOVE        80  /* a = value, or NULL: remove the key */
#define CC_OP_MMAP_REMOVEVALUE   81  /* a = value */
#define CC_OP_MMAP_ISEMPTY       82  /* query */
#define CC_OP_MMAP_SIZE          83  /* query */
#define CC_OP_MMAP_CLEAR         84

#define CC_OP_ELECT_LISTEN     110
#define CC_OP_ELECT_UNLISTEN   111
#define CC_OP_ELECT_ISLEADER   112  /* query */
/* LockCommands.java:59-93 */
#define CC_OP_LOCK_LOCK        115
#define CC_OP_LOCK_UNLOCK      116
/* MembershipGroupCommands.java:62-140 */
#define CC_OP_GROUP_JOIN       120
#define CC_OP_GROUP_LEAVE      121
#define CC_OP_GROUP_SCHEDULE   122
#define CC_OP_GROUP_EXECUTE    123

/* ---- canonical tagged values: Java equals == (tag, payload) equality ---------- */
#define CC_TAG_NULL    0
#define CC_TAG_LONG    1   /* java.lang.Long, payload = two's complement i64 */
#define CC_TAG_INT     2   /* java.lang.Integer, payload = sign-extended i32 */
#define CC_TAG_BOOL    3   /* java.lang.Boolean, payload 0/1 */
#define CC_TAG_HANDLE  4   /* host-interned object (String, Runnable callback ...) */
#define CC_TAG_SET     5   /* result only: Set<Long> of MembershipGroupState.join; payload = member count,
                              members are written to the aux-result stream */
#define CC_TAG_LIST    6   /* result only: a Collection (MultiMapState get / remove(key)); payload = element count */

/* flags column: bits 0-2 tag(a), bits 3-5 tag(b), bits 6-7 key tag (keys are never null,
 * KeyCommand asserts notNull MapCommands.java:77): 0 LONG, 1 INT, 2 BOOL, 3 HANDLE.               */
#define CC_FLAGS(tag_a, tag_b, ktag) ((uint8_t)(((tag_a) & 7u) | (((tag_b) & 7u) << 3) | (((ktag) & 3u) << 6)))
#define CC_FLAG_TAG_A(f) ((f) & 7u)
#define CC_FLAG_TAG_B(f) (((f) >> 3) & 7u)
#define CC_FLAG_KTAG(f)  (((f) >> 6) & 3u)

/* ---- per-commit status (the Java exception class) ----------------------------------
 * status byte = code | (result tag << 4)                                                          */
#define CC_ST_OK               0
#define CC_ST_UNKNOWN_SESSION  1  /* ResourceManagerException "unknown resource session" ResourceManager.java:65 */
#define CC_ST_UNKNOWN_OP       2  /* IllegalStateException "unknown operation type" ResourceStateMachineExecutor.java:78 */
#define CC_ST_ILLEGAL_STATE    3  /* IllegalStateException "not the lock holder" LockState.java:70 */
#define CC_ST_ILLEGAL_ARGUMENT 4  /* IllegalArgumentException "unknown member" MembershipGroupState.java:89,112 */
#define CC_ST_NULL_POINTER     5  /* NullPointerException in MapState.containsValue MapState.java:52 */
#define CC_ST_TYPE_MISMATCH    6  /* ResourceManagerException "inconsistent resource type" ResourceManager.java:120,181 */
#define CC_ST_UNKNOWN_RESOURCE 7  /* ResourceManagerException "unknown resource" ResourceManager.java:216 */
#define CC_ST_NO_SUCH_ELEMENT  8  /* NoSuchElementException of ArrayDeque.element/remove() QueueState.java:113,144 */
#define CC_STATUS(code, tag)   ((uint8_t)(((code) & 15u) | (((tag) & 15u) << 4)))
#define CC_STATUS_CODE(s)      ((s) & 15u)
#define CC_STATUS_TAG(s)       (((s) >> 4) & 15u)

/* ---- event codes: Session.publish(event, msg) -> InstanceEvent{instance, msg}
 * ManagedResourceSession.java:64-71, InstanceEvent.java:29-80                                     */
#define CC_EV_CHANGE   1  /* AtomicValueState.change  AtomicValueState.java:68-72 */
#define CC_EV_LOCK     2  /* LockState "lock" true/false LockState.java:44,47,79 */
#define CC_EV_ELECT    3  /* LeaderElectionState "elect"(epoch=leader index) LeaderElectionState.java:44,60,80 */
#define CC_EV_JOIN     4  /* MembershipGroupState "join"(instance) :55 */
#define CC_EV_LEAVE    5  /* MembershipGroupState "leave"(instance) :40,75 */
#define CC_EV_EXECUTE  6  /* MembershipGroupState "execute"(callback) :95,115 */
#define CC_EV_MEMBER   7  /* not an event: one row per member of a join's Set<Long> result (ascending ids,
                             target = the joining instance, src CC_EVSRC_RESULT) MembershipGroupState.java:63 */

/* event source */
#define CC_EVSRC_COMMIT 0  /* published while applying commit `pos` */
#define CC_EVSRC_TIMER  1  /* published by a timer that fired at commit `pos` */
#define CC_EVSRC_CLOSE  2  /* published by a session close/expire fan-out */
#define CC_EVSRC_RESULT 3  /* a variable-length result row (CC_EV_MEMBER) */

/* ---- engine configuration ------------------------------------------------------------------------ */
typedef struct cc_config {
  uint32_t max_resources;   /* resource slots (ResourceManager.resources), <= 131072            */
  uint32_t max_instances;   /* instance-session slots (ResourceManager.sessions)               */
  uint64_t max_batch;       /* max commits per cc_apply_batch call                               */
  uint64_t max_events;      /* capacity of the device event stream per batch                      */
  uint64_t map_capacity;    /* live map entries across all CC_RES_MAP resources (0 = no maps; at most
                               2M: the table has 2^k regions of 2048 entries, >= 2 x map_capacity) */
  int32_t  device;          /* HIP device ordinal                                                  */
  uint32_t flags;           /* CC_CFG_* */
  uint64_t sub_batch;       /* commits per internal sub-batch (0 = default 24Mi; rounded up to a multiple
                               of 16384, at most 24Mi; an engine with maps, coordination resources or
                               value events runs its batches in sub-batches of at most 16Mi)        */
  uint32_t coord_cap;       /* entries per coordination resource: lock waiters, election listeners, group
                               members, value listeners, queue elements (0 = 64 = CC_LOCK_QUEUE; else a power
                               of two in [64, 65536]; CC_ERR_CAPACITY beyond).  Device memory per resource slot:
                               32 + 24 x coord_cap bytes; entries past the first 8 are walked in global memory. */
  uint32_t reserved32;
  uint64_t reserved[3];
} cc_config;

#define CC_CFG_TIMERS_DEFERRED 1u  /* manager-mode timer order (A8): due timers fire after the commit
                                      that advanced time (ResourceManagerStateMachineExecutor.java:104-109) */
#define CC_CFG_VALUE_RETAINED  4u  /* keep, per AtomicValue slot, the log index of the commit the state machine
                                      still retains (`current`, never clean()ed): cc_read_value_retained  */
#define CC_CFG_VALUE_EVENTS    2u  /* AtomicValue Listen/Unlisten + "change" events on the GPU (every value
                                      resource then runs on the event-capable kernel)              */

/* Coordination resources (lock / election / group / queue) keep their variable-size state in per-resource
 * blocks of cc_config.coord_cap entries; the defaults (coord_cap = 0): at most CC_LOCK_QUEUE waiters per lock,
 * CC_ELECTION_LISTENERS listeners per election, CC_GROUP_MEMBERS members per group, CC_VALUE_LISTENERS listeners per
 * value, CC_QUEUE_CAP elements per queue (CC_ERR_CAPACITY beyond).
 * The time column must be non-decreasing within a batch when lock timeouts are used (Raft log time).   */
#define CC_LOCK_QUEUE          64
#define CC_ELECTION_LISTENERS  64
#define CC_GROUP_MEMBERS       64
#define CC_VALUE_LISTENERS     64

/* ---- one batch of committed entries, SoA, log order ------------------------------------------------
 * Row i is InstanceCommand/InstanceQuery{instance, op} of log entry index[i]
 * (InstanceOperation.java:59-69; ResourceManagerCommit.index/time ResourceManagerCommit.java:54-66).
 * Columns an op does not use may hold anything; pointers of columns no op in the batch uses may be NULL. */
typedef struct cc_batch {
  const uint64_t* index;  /* log index (Commit.index())                                         */
  const uint64_t* time;   /* log time, ms (Commit.time()); drives TTL / timeout timers           */
  const uint32_t* inst;   /* instance-session slot (InstanceOperation.resource -> sessions map)  */
  const uint8_t*  op;     /* CC_OP_*                                                              */
  const uint8_t*  flags;  /* CC_FLAGS(tag a, tag b, key tag)                                      */
  const uint64_t* key;    /* map key / group member instance slot                                 */
  const uint64_t* a;      /* value / expect / default-less operand                                */
  const uint64_t* b;      /* update / replace / default operand                                   */
  const uint64_t* aux;    /* ttl / lock timeout / schedule delay (signed i64)                     */
} cc_batch;

/* per-commit results (caller-allocated, n rows) */
typedef struct cc_results {
  uint8_t*  status;       /* CC_STATUS(code, result tag) */
  uint64_t* value;        /* result payload                */
} cc_results;

/* event stream (caller-allocated, capacity rows); count written to *count (device u64) */
typedef struct cc_events {
  uint32_t* pos;          /* batch row that produced the event                          */
  uint32_t* target;       /* instance slot whose session receives it                    */
  uint8_t*  code;         /* CC_EV_*                                                     */
  uint8_t*  src;          /* CC_EVSRC_*                                                  */
  uint8_t*  tag;          /* payload tag                                                 */
  uint64_t* payload;
  uint64_t  capacity;
  uint64_t* count;        /* device pointer: number of events written (may exceed capacity:
                             then the call returns CC_ERR_CAPACITY on sync)                */
} cc_events;

typedef struct cc_engine cc_engine;

/* ---- lifecycle ------------------------------------------------------------------------------------ */
int  cc_abi_version(void);
const char* cc_last_error(void);
/* ResourceManager constructor + StateMachine.configure (ResourceManager.java:35-50) */
int  cc_engine_create(const cc_config* cfg, cc_engine** out);
int  cc_engine_destroy(cc_engine* e);
int  cc_sync(cc_engine* e);
/* The engine's stream (hipStream_t as void*). */
void* cc_engine_stream(cc_engine* e);

/* ---- resource and instance registry (host-side control commands) --------------------------------
 * New resource: ResourceManager.getResource/createResource new-key branch (ResourceManager.java:84-100,157-176);
 * the engine allocates state for `slot` (chosen by the host: resource id -> dense slot).       */
int  cc_resource_create(cc_engine* e, uint32_t slot, uint32_t type);
/* Bulk form: slots [first, first+count) all of `type`. */
int  cc_resource_create_range(cc_engine* e, uint32_t first, uint32_t count, uint32_t type);
/* ResourceManager.deleteResource (ResourceManager.java:212-235): delete() state, cancel timers,
 * and close every instance slot registered to the resource.                                   */
int  cc_resource_delete(cc_engine* e, uint32_t slot);
/* A ManagedResourceSession (ResourceManager.java:103-106,128-131,189-190): instance slot -> resource slot,
 * owned by client session `client_session`; `instance_id` is the Java instance id (= creating commit index). */
int  cc_instance_open(cc_engine* e, uint32_t inst, uint32_t res_slot, uint64_t instance_id, uint64_t client_session);
/* Bulk form: instance slot first+k -> resource slot res_first+k, instance id id_first+k, one client session. */
int  cc_instance_open_range(cc_engine* e, uint32_t first, uint32_t count, uint32_t res_first, uint64_t id_first,
                            uint64_t client_session);

/* ---- ResourceManager control commands (ResourceManager.java:77-235) ------------------------------------
 * GetResource / CreateResource / DeleteResource / ResourceExists commits, applied by the host between batches in log
 * order (manager.hip).  `key` is the host-interned GetResource.key String, `client` = commit.session().id(),
 * `index` = commit.index().  Resource ids and instance ids are commit indices; the engine picks the slots.
 * *status = CC_STATUS(CC_ST_OK, CC_TAG_LONG) with *instance_id = the ManagedResourceSession id (the Long the reference
 * returns) and *inst_slot = the instance slot its commits carry in cc_batch.inst; or CC_ST_TYPE_MISMATCH
 * ("inconsistent resource type" :119-121,178-181).  Return codes: CC_ERR_CAPACITY when no slot is free.       */
/* getResource :77-143 — a new key creates the resource (id = index); a client that already holds an instance of
 * the resource gets that instance back (ResourceHolder.sessions :137-141) */
int  cc_get_resource(cc_engine* e, uint64_t key, uint32_t type, uint64_t client, uint64_t index, uint64_t* instance_id,
                     uint32_t* inst_slot, uint8_t* status);
/* createResource :148-196 — always a new instance (id = index), not recorded in ResourceHolder.sessions */
int  cc_create_resource(cc_engine* e, uint64_t key, uint32_t type, uint64_t client, uint64_t index, uint64_t* instance_id,
                        uint32_t* inst_slot, uint8_t* status);
/* resourceExists :201-207 */
int  cc_resource_exists(cc_engine* e, uint64_t key, uint8_t* exists);
/* deleteResource :212-235 by RESOURCE id (clients send their instance id, so only the creating instance matches,
 * A13): *status = OK|BOOL (true), CC_ST_UNKNOWN_RESOURCE, or CC_ST_ILLEGAL_STATE when the state machine's delete()
 * throws (a lock / election whose holder commit was already cleaned): the resource then leaves `resources` but its
 * key and instances stay, and commits on those instances get CC_ST_NULL_POINTER (:62,71).                     */
int  cc_delete_resource(cc_engine* e, uint64_t resource_id, uint8_t* status);
/* id -> slot lookups of ResourceManager.sessions / resources (-1: none) */
int  cc_instance_slot(cc_engine* e, uint64_t instance_id, int64_t* slot);
int  cc_resource_slot(cc_engine* e, uint64_t resource_id, int64_t* slot);

/* java.lang.String.hashCode of HANDLE keys.  A HANDLE key is a host-interned String (GetResource / DistributedMap keys
 * are Strings); java.util.HashMap places it by String.hashCode, which the handle alone does not give.  Map resources
 * need it to answer containsValue in the reference's iteration order (MapState.java:49-60 walks map.values()) and
 * to follow the table's capacity exactly (HashMap.treeifyBin resizes a table below capacity 64 when one bin reaches 9
 * keys).  cc_wire_decode registers the Strings it interns itself; a host that interns Strings on its own registers
 * them here before the batch that uses them (a map operation that needs an unregistered key's hash fails the batch
 * with CC_ERR_STATE).  Registering a handle again with another hash is CC_ERR_INVALID. */
int  cc_handle_hashes(cc_engine* e, const uint64_t* h_handles, const int32_t* h_hashes, uint64_t count);

/* ---- the hot path --------------------------------------------------------------------------------
 * Apply n committed entries (device-resident columns) in log order.  Replaces the per-entry chain
 * ResourceManager.operateResource (ResourceManager.java:56-72) -> executors -> state machine method.
 * `events` may be NULL when no op in the batch publishes (then publishing ops fail with CC_ERR_UNSUPPORTED). */
/* Map containsValue/size/isEmpty/clear/Delete rows (MapState.java:49-60,233-274) read or reset a whole map: on
 * an engine with maps the call first scans the batch for them (one host sync), then applies the rows between
 * them as segments and each such row against the table as it stands at its log position.  A containsValue whose
 * answer depends on java.util.HashMap iteration order when the map's table capacity is not determined exactly
 * fails the batch with CC_ERR_STATE (see copycat_amd/csrc/map_wide.hip). */
/* d_out->status must be 4-byte aligned and d_out->value 16-byte aligned (hipMalloc / torch allocations are). */
int  cc_apply_batch(cc_engine* e, const cc_batch* d_cols, uint64_t n, const cc_results* d_out,
                    const cc_events* d_events, void* stream);
/* ---- host-memory entry points (copycat_amd/csrc/host_path.hip) -------------------------------------------------
 * For a host that holds no device pointers (a JVM through Panama FFM / JNI): host columns in,
 * host results and events out.  The engine stages them in device buffers it owns (grown on demand, kept between
 * calls); every call is synchronous.  A host event stream is a cc_events whose column pointers AND `count` point to
 * host memory: *count = the events published (when it exceeds `capacity` the call returns CC_ERR_CAPACITY after
 * copying the first `capacity` rows).  Events reach the client as Session.publish -> InstanceEvent{instance, msg}
 * (ManagedResourceSession.java:64-71, InstanceEvent.java:29-80): `target` is the instance slot whose session
 * receives the event, rows in publish order (log row, then the state machine's publish order). */
/* Host columns/results: H2D, apply, D2H, sync (PCIe-inclusive path).  Publishing ops fail with
 * CC_ERR_UNSUPPORTED here: use cc_apply_batch_host_events. */
int  cc_apply_batch_host(cc_engine* e, const cc_batch* h_cols, uint64_t n, const cc_results* h_out);
/* The same with the event stream (lock grants, elections, joins / leaves, executes, value changes). */
int  cc_apply_batch_host_events(cc_engine* e, const cc_batch* h_cols, uint64_t n, const cc_results* h_out,
                                const cc_events* h_events);
/* Highest log index applied so far (the applied watermark; all-gathered across GPUs by the host). */
int  cc_applied_index(cc_engine* e, uint64_t* out);
/* Cumulative path counters of the engine (observability; ABI 5): out[0] whole-map / schedule rows applied as batch
 * barriers, out[1] map containsValue rows answered in the stream (map_cv.hip), out[2] sub-batches launched,
 * out[3] map events sorted and replayed (small maps' HashMap models, size rows, cleared maps' sizes: map_small.hip),
 * out[4] big HashMap models held now (maps past capacity 64 with a tree bin: map_big.hip; reading it syncs).
 * n = entries of `out` to fill (at most 5). */
int  cc_engine_counters(cc_engine* e, uint64_t* out, uint32_t n);
/* The same watermark written stream-ordered into device memory (u64 at d_out) without a host sync: what a rank feeds
 * to the RCCL all-gather of applied watermarks after each batch. */
int  cc_applied_index_async(cc_engine* e, uint64_t* d_out, void* stream);

/* ---- snapshot / restore ---------------------------------------------------------------------------
 * Replaces recovery by full log replay (the reference replays Copycat's log, AbstractReplicaTest.java:82-84):
 * the engine's whole device state plus its host registry mirrors, as one host buffer.  Save syncs first;
 * restore needs an engine created with the same max_resources, max_instances and map_capacity. */
int  cc_snapshot_size(cc_engine* e, uint64_t* bytes);
int  cc_snapshot_save(cc_engine* e, void* h_buf, uint64_t cap);
int  cc_snapshot_restore(cc_engine* e, const void* h_buf, uint64_t size);

/* ---- state readback for parity checks ------------------------------------------------------------ */
/* AtomicValueState {value, current != null} for slots [first, first+count) (AtomicValueState.java:34-35) */
int  cc_read_value_state(cc_engine* e, uint32_t first, uint32_t count, uint8_t* h_tag, uint64_t* h_value,
                         uint8_t* h_has_current);
/* Log compaction (Commit.clean(), AtomicValueState.java:88-157): per value slot in [first, first+count), the
 * index of the one commit still retained (`current`), 0 if none.  Needs CC_CFG_VALUE_RETAINED.          */
int  cc_read_value_retained(cc_engine* e, uint32_t first, uint32_t count, uint64_t* h_index);
/* MapState.map of one map slot (MapState.java:33): *count = live entries; the first min(cap, count), sorted
 * by (key tag, key), go to the arrays (key tag as a CC_TAG_*; commit_index may be NULL).               */
int  cc_read_map_entries(cc_engine* e, uint32_t slot, uint64_t cap, uint64_t* count, uint8_t* h_key_tag, uint64_t* h_key,
                         uint8_t* h_value_tag, uint64_t* h_value, uint64_t* h_commit_index);
/* Every map / set slot's live entries in one pass over the table (bulk form of cc_read_map_entries): *count =
 * entries; the first min(cap, count), sorted by (slot, key tag, key), go to the arrays.                      */
int  cc_read_map_table(cc_engine* e, uint64_t cap, uint64_t* count, uint32_t* h_slot, uint8_t* h_key_tag, uint64_t* h_key,
                       uint8_t* h_value_tag, uint64_t* h_value, uint64_t* h_commit_index);

/* LockState (LockState.java:33-36) after the timers due at the engine clock: holder instance slot (-1 none),
 * its commit index and cleaned flag; *count = queued waiters, the first min(cap, count) to the arrays. */
int  cc_read_lock_state(cc_engine* e, uint32_t slot, int64_t* holder, uint64_t* holder_index, uint8_t* holder_cleaned,
                        uint64_t cap, uint64_t* count, uint32_t* h_queue_inst, uint64_t* h_queue_index);
/* LeaderElectionState (LeaderElectionState.java:31-33): leader instance slot (-1 none) + index, listeners in
 * insertion order. */
int  cc_read_election_state(cc_engine* e, uint32_t slot, int64_t* leader, uint64_t* leader_index, uint64_t cap,
                            uint64_t* count, uint32_t* h_listener_inst, uint64_t* h_listener_index);
/* MembershipGroupState.members (MembershipGroupState.java:33): member instance ids, ascending. */
int  cc_read_group_members(cc_engine* e, uint32_t slot, uint64_t cap, uint64_t* count, uint64_t* h_ids);
/* Log compaction for every state machine (Commit.clean()): the log indices of every commit
 * the slot's state machine still holds without having clean()ed it, ascending — *count of them, the first
 * min(cap, count) to h_index.  Value: `current` + listeners (AtomicValueState.java:41-157, needs
 * CC_CFG_VALUE_RETAINED); map / set: each entry's commit (MapState.java:279-287); lock: the holder unless
 * delete() cleaned it + waiters (LockState.java:41-98); election: the leader unless cleaned + listeners
 * (LeaderElectionState.java:35-108); group: members + pending schedule commits (MembershipGroupState.java:47-103);
 * queue: elements less the head element() cleaned (QueueState.java:51-199).  Plus the commits those state
 * machines drop without clean() — a listen that replaces a session's listener (AtomicValueState.java:41-49), a
 * member removed by close (MembershipGroupState.java:36-42) — which the log can never compact.            */
int  cc_read_retained(cc_engine* e, uint32_t slot, uint64_t cap, uint64_t* count, uint64_t* h_index);
/* Bulk compaction feed: bit (i - first) of d_bitmap (ceil(count / 64) u64 words in HBM, LSB first) is set iff
 * log index i in [first, first + count) is held by some resource's state machine without clean() -- the union over
 * every live resource slot of cc_read_retained, built on the device in one pass (retained.hip).  *h_count (may be
 * NULL) = the retained commits in the range.  A compactor calls it after a batch over (last compacted, commit index]:
 * clear bits are compactable (Commit.clean(), ResourceManagerCommit.java:79-81); a bit that cleared since the
 * previous call was released by a clean() in between.  Value resources need CC_CFG_VALUE_RETAINED.  Synchronous. */
int  cc_retained_bitmap(cc_engine* e, uint64_t first, uint64_t count, uint64_t* d_bitmap, uint64_t* h_count);
/* The same bitmap into host memory (ceil(count / 64) u64 words). */
int  cc_retained_bitmap_host(cc_engine* e, uint64_t first, uint64_t count, uint64_t* h_bitmap, uint64_t* h_count);
/* Log time advanced without a commit (ResourceManagerStateMachineExecutor timers): due lock
 * timeouts take effect (they publish nothing, LockState.java:54-58). */
int  cc_advance_time(cc_engine* e, uint64_t now);
/* Same, publishing the "execute" events of MembershipGroup.schedule timers that come due (pos 0xFFFFFFFF,
 * src CC_EVSRC_TIMER) to d_events; *d_events->count is written.  cc_advance_time fails with CC_ERR_UNSUPPORTED
 * when such an event is due and has no stream. */
int  cc_advance_time_events(cc_engine* e, uint64_t now, const cc_events* d_events);
/* The same with a host event stream. */
int  cc_advance_time_events_host(cc_engine* e, uint64_t now, const cc_events* h_events);

/* ---- session close / expire fan-out (ResourceManager.close :250-264, expire :238-247) -------------------
 * For each client session of h_clients, in order: every instance it owns, in java.util.HashMap iteration order of
 * ResourceManager.sessions, is closed on its state machine (LeaderElectionState.close :35-52 hands leadership to the
 * first listener, MembershipGroupState.close :36-42 publishes "leave", an AtomicValue listener is dropped; locks and
 * maps have no close handler) and leaves the dispatch table: later commits on it get CC_ST_UNKNOWN_SESSION.  Events
 * go to d_events (src CC_EVSRC_CLOSE, pos 0xFFFFFFFF) in fan-out order; *count is written.  A close that throws
 * (an election leader already cleaned by delete) ends that client's fan-out there, as the reference's loop does
 * (ResourceManager.close runs once per session; the remaining clients are closed): *h_closed = the instances closed.
 * Synchronous (control plane).                                              */
int  cc_sessions_close(cc_engine* e, const uint64_t* h_clients, uint64_t count, const cc_events* d_events, void* stream,
                       uint64_t* h_closed);
/* The expired set of cc_expire_sweep (bit s = client session id s, u64 words in HBM), closed in ascending id order. */
int  cc_sessions_expire(cc_engine* e, const uint64_t* d_bitmap, uint64_t sessions, const cc_events* d_events, void* stream,
                        uint64_t* h_closed);
/* Host-memory forms (see "host-memory entry points" above): events to a host cc_events (NULL: none may publish). */
int  cc_sessions_close_host(cc_engine* e, const uint64_t* h_clients, uint64_t count, const cc_events* h_events,
                            uint64_t* h_closed);
int  cc_sessions_expire_host(cc_engine* e, const uint64_t* h_bitmap, uint64_t sessions, const cc_events* h_events,
                             uint64_t* h_closed);

/* ---- per-kernel timing (HIP events recorded on the launch stream around every engine kernel) ----------
 * kernel ids: 0 k_part_tile, 1 k_apply_value, 2 k_unpermute, 3 k_apply_map, 4 k_map_hot (hot-key lists +
 * scan, apply_map_hot.hip), 5 k_apply_coord (coordination + value events), 6 k_events (event scan+scatter). */
#define CC_PROFILE_KERNELS 7
int  cc_profile_enable(cc_engine* e, int on);
int  cc_profile_reset(cc_engine* e);
/* Accumulated device time (ms) and launch count of one kernel since the last reset (synchronizes). */
int  cc_profile_read(cc_engine* e, int kernel, double* total_ms, uint64_t* launches, const char** name);

/* Diagnostics build only (-DCC_PHASE_TIMING; scripts/probes/phase_timing.py): per-phase s_memrealtime ticks
 * (10 ns) summed over the workgroups of kernel `kernel` (0 k_part_tile, 1 k_apply_value, 2 k_unpermute) since
 * the last read, CC_PHASES entries; CC_ERR_UNSUPPORTED in the product build. */
#define CC_PHASES 8
int cc_debug_phases(cc_engine* e, int kernel, uint64_t* ticks);

/* ---- leader quorum commit index (Copycat leader [not vendored]) ------------------------
 * Per group g: N = the quorum-th largest of d_match[r*groups + g], r < replicas (r = 0 is the leader's
 * last log index), quorum = replicas/2 + 1; new = (N >= d_term_start[g] && N > d_commit_in[g]) ? N : d_commit_in[g]. */
int  cc_quorum_commit(const uint64_t* d_match, uint32_t replicas, uint64_t groups, const uint64_t* d_term_start,
                      const uint64_t* d_commit_in, uint64_t* d_commit_out, void* stream);

/* ---- session / lease expiry sweep (Copycat sessions [not vendored]) ---------------------
 * Session s is expired iff now - d_last[s] > timeout (signed difference; a keep-alive in the future never
 * expires).  Bit s of d_bitmap (u64 words, LSB first) is set for expired sessions; *d_count (u64) += expired. */
int  cc_expire_sweep(const uint64_t* d_last, uint64_t sessions, uint64_t now, uint64_t timeout,
                     uint64_t* d_bitmap, uint64_t* d_count, void* stream);

/* ---- plain device memory: for cc_quorum_commit / cc_expire_sweep and hosts that keep columns resident in HBM --------
 * (hipMalloc / hipFree / hipMemcpy on the engine's HIP runtime; cc_memcpy and cc_memset synchronize `stream`) */
#define CC_MEMCPY_H2D 1
#define CC_MEMCPY_D2H 2
#define CC_MEMCPY_D2D 3
int  cc_device_alloc(int device, uint64_t bytes, void** d_out);
int  cc_device_free(void* d_ptr);
int  cc_memcpy(void* dst, const void* src, uint64_t bytes, int kind, void* stream);
int  cc_memset(void* d_ptr, int byte, uint64_t bytes, void* stream);

/* ---- Catalyst wire format -> columns (copycat_amd/csrc/wire.cpp) ----------------------
 * A committed resource entry is InstanceCommand / InstanceQuery (@SerializeWith 30 / 31): writeLong(instance id),
 * then serializer.writeObject(operation) (InstanceOperation.java:60-69); the operation's @SerializeWith id is the
 * CC_OP_* code and its fields follow its writeObject chain (wire.cpp kSchema cites each).  Manager entries
 * (GetResource 35, CreateResource 36, DeleteResource 37, ResourceExists 38) decode to control rows.
 * Catalyst (Serializer / Buffer) is not vendored: the identifier byte before a registered type id (0 null,
 * 1..4 an id of 1..4 bytes, 5 a class name), the ids of Long / Integer / Boolean / String, byte order and the
 * UTF-8 framing are cc_wire_codec fields; the defaults below are this engine's restatement of Catalyst 1.x
 * (parity unpinned: set them from the deployment's serializer registry). */
#define CC_WIRE_ID_BOOLEAN 129
#define CC_WIRE_ID_INTEGER 132
#define CC_WIRE_ID_LONG    133
#define CC_WIRE_ID_STRING  136
typedef struct cc_wire_codec {
  uint8_t  big_endian;          /* Catalyst Buffer byte order (1: big-endian, Java's)                        */
  uint8_t  utf8_presence_byte;  /* writeUTF8 writes a boolean "not null" byte before the length               */
  uint8_t  utf8_len_bytes;      /* width of writeUTF8's length prefix                                        */
  uint8_t  reserved8;
  int32_t  id_bool, id_int, id_long, id_string;  /* registered serializer ids                                  */
  uint64_t reserved[4];
} cc_wire_codec;
void cc_wire_codec_default(cc_wire_codec* c);
/* String values and resource keys become CC_TAG_HANDLE handles through an interner (equal bytes, equal handle:
 * Java String.equals); handles are first_handle, first_handle + 1, ... in order of first appearance. */
typedef struct cc_wire_interner cc_wire_interner;
int  cc_wire_interner_create(uint64_t first_handle, cc_wire_interner** out);
int  cc_wire_interner_destroy(cc_wire_interner* in);
int  cc_wire_intern(cc_wire_interner* in, const uint8_t* bytes, uint64_t len, uint64_t* handle);
int  cc_wire_lookup(cc_wire_interner* in, uint64_t handle, uint8_t* buf, uint64_t cap, uint64_t* len);
/* java.lang.String.hashCode of an interned String (its UTF-8 bytes decoded to UTF-16 code units). */
int  cc_wire_string_hash(cc_wire_interner* in, uint64_t handle, int32_t* hash);
/* decoded rows (host memory, n each).  kind 0: a resource operation (inst = the instance slot of the instance
 * id through the engine's session registry, max_instances when unknown -> CC_ST_UNKNOWN_SESSION when applied;
 * iid = the instance id itself; op/flags/key/a/b/aux as cc_batch).  With e == NULL (no engine: host-only
 * decoding) inst is not written and iid is required.  kind 35/36/38: get/create/exists with key = the key's handle, a = the
 * CC_RES_* of the state machine class (CC_RES_NONE when not one this engine runs); kind 37: delete, b = the
 * resource id.  index and time are the log entry's own (the caller's) and are not touched. */
typedef struct cc_wire_out {
  uint32_t* inst;   /* needs an engine */
  uint64_t* iid;    /* optional with an engine */
  uint8_t*  op;
  uint8_t*  flags;
  uint64_t* key;
  uint64_t* a;
  uint64_t* b;
  uint64_t* aux;
  uint8_t*  kind;
} cc_wire_out;
/* Entry i is buf[offsets[i], offsets[i+1]) of the buf_len-byte buffer (an entry that ends past buf_len fails with its
 * row; ABI 3 added buf_len).  Fails (CC_ERR_INVALID, *bad_row = the entry) on a truncated or
 * over-long entry, an unknown operation, a null key, or a value that is neither null, Long, Integer, Boolean
 * nor String (user objects have no canonical tag); rows before *bad_row are decoded. */
int  cc_wire_decode(cc_engine* e, const cc_wire_codec* codec, cc_wire_interner* in, const uint8_t* buf, uint64_t buf_len,
                    const uint64_t* offsets, uint64_t n, const cc_wire_out* out, uint64_t* bad_row);

/* ---- a batch applied up to the first commit the engine cannot hold (ABI 5; copycat_amd/csrc/host_path.hip) ----
 * Java's coordination collections are unbounded; the engine's hold cc_config.coord_cap entries.  Like
 * cc_apply_batch_host_events (h_events may be NULL), but a row that would add an entry to a full lock queue / listener
 * list / member set / queue is not applied: the call returns CC_ERR_CAPACITY with *h_applied = that row, the engine
 * state is exactly the state after rows [0, *h_applied), the events of those rows are in h_events, and rows from
 * *h_applied on are not applied (their result rows keep what the caller put there).  The host resumes at that row
 * (e.g. on an engine with a larger coord_cap restored from a snapshot, or treating the commit as failed).  On success
 * *h_applied = n.  Round 6: the same holds for a row whose map / set / multimap entry a full table region cannot
 * hold, and for a row whose events do not fit h_events' capacity (or max_events): the engine takes a device
 * checkpoint before each part of the batch and, when a part fails on one of those capacities, restores it and
 * applies the longest prefix that fits (bisection), so *h_applied is exactly that row and the state, results and
 * events are those after the rows before it.  A host with a full event stream drains it and resumes at that row. */
int  cc_apply_batch_host_prefix(cc_engine* e, const cc_batch* h_cols, uint64_t n, const cc_results* h_out,
                                const cc_events* h_events, uint64_t* h_applied);

/* ---- one global log, many engines (ABI 5; copycat_amd/csrc/split.cpp) -----------------------------
 * The reference multiplexes every resource in one Raft log (ResourceManager.java:37-39,56-72); with one engine per
 * GPU the host splits each committed batch by the rank that owns the row's resource, and merges the per-rank results
 * back into log order.  Host memory only: no engine and no GPU is involved.
 *
 * cc_split_batch: stable split of rows [0, n) of `in` (host columns; inst is required, any other column may be NULL
 * and then stays NULL).  rank_of_inst[s] (s < n_inst) is the rank owning instance slot s; a row whose inst >= n_inst
 * goes to rank 0 (whose engine answers UNKNOWN_SESSION).  counts[r] = rows of rank r.  With outs == NULL only the
 * counts are computed.  Otherwise outs[r] receives rank r's rows in log order: every column present in `in` must be
 * non-NULL in outs[r], with room for out_cap[r] rows; if counts[r] > out_cap[r] for any r the call returns
 * CC_ERR_CAPACITY with `counts` filled and nothing written.  rows (optional, world pointers, each optional) receives
 * each output row's row in `in`.  threads: worker threads (0 = hardware concurrency). */
typedef struct cc_batch_out {
  uint64_t* index;
  uint64_t* time;
  uint32_t* inst;
  uint8_t*  op;
  uint8_t*  flags;
  uint64_t* key;
  uint64_t* a;
  uint64_t* b;
  uint64_t* aux;
} cc_batch_out;
int  cc_split_batch(const cc_batch* in, uint64_t n, const uint8_t* rank_of_inst, uint32_t n_inst, uint32_t world,
                    uint32_t threads, const cc_batch_out* outs, const uint64_t* out_cap, uint64_t* counts,
                    uint64_t* const* rows);
/* cc_merge_results: the inverse for the result columns.  Row i of `out` (n rows) takes the next unread row of
 * parts[rank_of(inst[i])] (the same inst column and table the split used). */
int  cc_merge_results(const uint32_t* inst, uint64_t n, const uint8_t* rank_of_inst, uint32_t n_inst, uint32_t world,
                      uint32_t threads, const cc_results* parts, const cc_results* out);

#ifdef __cplusplus
}
#endif
#endif /* COPYCAT_APPLY_H */
