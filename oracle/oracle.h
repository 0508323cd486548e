/*
 * oracle.h — CPU restatement of the reference's commit-apply path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so, and only
 * as the checker / the timed CPU baseline.  The product (copycat_amd/, libcopycat_apply.so) never links,
 * loads or calls it.
 *
 * It restates, line by line, the Java state machines of madjam/copycat (Atomix 0.1.0-SNAPSHOT):
 *   ResourceManager.java:56-264, ResourceManagerStateMachineExecutor.java:90-116,
 *   ResourceStateMachineExecutor.java:73-117, ResourceStateMachine.java:33-54,
 *   AtomicValueState.java:41-157, MapState.java:38-274, LockState.java:41-98,
 *   LeaderElectionState.java:35-108, MembershipGroupState.java:36-125
 * (paths relative to the reference root; exact citations at each function in oracle.cpp).
 *
 * Parity pinning: the Java reference cannot run here (no JDK, no Copycat/Catalyst jars),
 * so this restatement is pinned by the known answers of the reference's own tests, transcribed into
 * tests/golden/kats.json (DistributedMapTest, DistributedAtomicValueTest, DistributedAtomicLongTest,
 * DistributedLockTest, DistributedLeaderElectionTest, DistributedMembershipGroupTest, AtomixReplicaTest),
 * plus hand-derived quirk KATs.  Copycat-side rules (quorum commit index, session
 * expiry, timer order) have no reference source here and are "parity unpinned" (see DESIGN.md).
 *
 * The column/record types are the engine's public ABI types (include/copycat_apply.h), so the same
 * batch can be fed to both.
 */
#ifndef COPYCAT_ORACLE_H
#define COPYCAT_ORACLE_H
#include <stdint.h>
#include "../include/copycat_apply.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc orc;

#define ORC_TIMERS_DEFERRED CC_CFG_TIMERS_DEFERRED

orc* orc_create(uint32_t max_resources, uint32_t max_instances, uint32_t flags);
void orc_destroy(orc* o);

/* registry (slot level, same contract as cc_resource_create / cc_resource_delete / cc_instance_open) */
int  orc_resource_create(orc* o, uint32_t slot, uint32_t type);
int  orc_resource_delete(orc* o, uint32_t slot);
int  orc_instance_open(orc* o, uint32_t inst, uint32_t res, uint64_t instance_id, uint64_t client_session);

/* ResourceManager control commands (ResourceManager.java:77-235), key = interned key handle.
 * They allocate resource / instance slots (lowest free) and return status codes like commits.     */
int  orc_get_resource(orc* o, uint64_t key, uint32_t type, uint64_t client_session, uint64_t index,
                      uint64_t* instance_id, uint32_t* inst_slot, uint8_t* status);
int  orc_create_resource(orc* o, uint64_t key, uint32_t type, uint64_t client_session, uint64_t index,
                         uint64_t* instance_id, uint32_t* inst_slot, uint8_t* status);
int  orc_delete_resource(orc* o, uint64_t resource_id, uint8_t* status);
int  orc_resource_exists(orc* o, uint64_t key);
int  orc_inst_slot_of(orc* o, uint64_t instance_id); /* -1 if unknown */
int  orc_res_slot_of(orc* o, uint64_t resource_id);  /* -1 if unknown */

/* apply a batch (host columns); results per row; events / set results accumulate (see below) */
int  orc_apply(orc* o, const cc_batch* cols, uint64_t n, uint8_t* status, uint64_t* value);
/* advance the deterministic clock (keep-alive ticks between batches) and fire due timers */
int  orc_advance_time(orc* o, uint64_t now);
/* The String behind a HANDLE key (UTF-16 code units): its hashCode / compareTo place it in java.util.HashMap's bins
 * and tree bins (containsValue order).  Unregistered handles hash like a Long of the handle. */
int  orc_handle_string(orc* o, uint64_t handle, const uint16_t* units, uint64_t n);
/* ResourceManager.close / expire (ResourceManager.java:237-264) for a client session */
int  orc_session_close(orc* o, uint64_t client_session);
int  orc_session_expire(orc* o, uint64_t client_session);
uint64_t orc_applied_index(orc* o);

/* event stream (in emission order) */
uint64_t orc_event_count(orc* o);
void orc_events_read(orc* o, uint32_t* pos, uint32_t* target, uint8_t* code, uint8_t* src, uint8_t* tag,
                     uint64_t* payload);
void orc_events_clear(orc* o);
/* set results of MembershipGroupState.join (pos, member instance id), members ascending per pos */
uint64_t orc_aux_count(orc* o);
void orc_aux_read(orc* o, uint32_t* pos, uint64_t* member);
void orc_aux_clear(orc* o);

/* state readback */
int  orc_read_value_retained(orc* o, uint32_t first, uint32_t count, uint64_t* index);
int  orc_read_value_state(orc* o, uint32_t first, uint32_t count, uint8_t* tag, uint64_t* value,
                          uint8_t* has_current);
int64_t orc_read_retained(orc* o, uint32_t slot, uint64_t cap, uint64_t* out);
int64_t orc_map_size(orc* o, uint32_t res);
/* entries sorted by (key tag, key); returns count written (<= cap) or -1 */
int64_t orc_map_entries(orc* o, uint32_t res, uint64_t cap, uint8_t* ktag, uint64_t* key, uint8_t* vtag,
                        uint64_t* val, uint64_t* commit_index);
/* lock: holder inst slot (-1 none), holder commit index, cleaned flag; queue of waiter inst slots */
int64_t orc_lock_state(orc* o, uint32_t res, int64_t* holder, uint64_t* holder_index, uint8_t* holder_cleaned,
                       uint64_t cap, uint32_t* queue_inst, uint64_t* queue_index);
int64_t orc_election_state(orc* o, uint32_t res, int64_t* leader, uint64_t* leader_index, uint64_t cap,
                           uint32_t* listener_inst, uint64_t* listener_index);
int64_t orc_group_members(orc* o, uint32_t res, uint64_t cap, uint64_t* member_ids);
uint64_t orc_pending_timers(orc* o);

/* Leader quorum commit index and session expiry sweep — the rules the engine defines (a14/a15, unpinned) */
void orc_quorum_commit(const uint64_t* match, uint32_t replicas, uint64_t groups, const uint64_t* term_start,
                       const uint64_t* commit_in, uint64_t* commit_out);
void orc_expire_sweep(const uint64_t* last, uint64_t sessions, uint64_t now, uint64_t timeout, uint64_t* bitmap,
                      uint64_t* count);

#ifdef __cplusplus
}
#endif
#endif
