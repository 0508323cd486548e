// manager.hip — the ResourceManager control plane on the host side of the engine (no kernels).
//
// Reference: ResourceManager.getResource :77-143, createResource :148-196, resourceExists :201-207 and
// deleteResource :212-235 (manager/src/main/java/io/atomix/manager/ResourceManager.java).  These commands share the
// Raft log with the resource commits but are rare; the host applies them between cc_apply_batch calls, in log order.
// They maintain the maps the hot path dispatches through:
//   keys        key -> resource id                (ResourceManager.keys :37)
//   res_by_id   resource id -> resource slot      (ResourceManager.resources :38)
//   inst_by_id  instance id -> instance slot      (ResourceManager.sessions :39; the device copy is inst_res)
//   res_sessions (slot, client session) -> instance id   (ResourceHolder.sessions :273)
// Ids are commit indices: a new key's resource id is the index of the commit that created it (:86-88,157-159), every
// new instance's id is the index of its commit (:103,128,185).  Slots are the engine's dense handles: value, map and
// set resources take the lowest free slot, coordination resources (lock, election, group, queue) the highest, so
// value super-buckets stay on the value-only apply kernel; and a coordination resource goes into a 64-slot group
// (one k_apply_coord walking wave) that holds only its type, so the walk runs the type-specialised code
// (apply_coord.hip TypeC) without divergence between types.  Instances take the lowest free instance slot.
#include <algorithm>
#include <cstring>

#include "engine_state.h"

using namespace cc;

namespace {

bool coord_type(uint32_t t) { return t == CC_RES_LOCK || t == CC_RES_ELECTION || t == CC_RES_GROUP || t == CC_RES_QUEUE; }

// every used slot of 64-slot group g holds `type`
bool group_holds_only(const cc_engine* e, uint32_t g, uint32_t type) {
  for (uint32_t s = g * 64; s < g * 64 + 64 && s < e->cfg.max_resources; ++s)
    if (e->used_res.test(s) && e->res_type[s] != type) return false;
  return true;
}

int alloc_res_slot(cc_engine* e, uint32_t type, uint32_t* slot) {
  if (coord_type(type)) {
    auto& open = e->open_grp[type];
    while (!open.empty()) {  // the highest group of this type with room
      const uint32_t g = *open.rbegin();
      const uint64_t word = e->used_res.w[g];
      const uint64_t valid = (uint64_t)g * 64 + 64 <= e->cfg.max_resources ? ~0ull : (1ull << (e->cfg.max_resources & 63)) - 1;
      if ((~word & valid) && group_holds_only(e, g, type)) {
        *slot = g * 64 + 63 - (uint32_t)__builtin_clzll(~word & valid);
        return CC_OK;
      }
      open.erase(g);
    }
    for (uint64_t g = e->cfg.max_resources / 64; g-- > 0;)  // else the highest empty group
      if (e->used_res.w[g] == 0) {
        open.insert((uint32_t)g);
        *slot = (uint32_t)(g * 64 + 63);
        return CC_OK;
      }
  }
  const int64_t s = coord_type(type) ? e->used_res.highest() : e->used_res.lowest();
  if (s < 0) return set_err(CC_ERR_CAPACITY, "no free resource slot (max_resources)");
  *slot = (uint32_t)s;
  return CC_OK;
}

int alloc_inst_slot(cc_engine* e, uint32_t* slot) {
  const int64_t s = e->used_inst.lowest();
  if (s < 0) return set_err(CC_ERR_CAPACITY, "no free instance slot (max_instances)");
  *slot = (uint32_t)s;
  return CC_OK;
}

// `new ManagedResourceSession(index, commit.session())` registered in ResourceManager.sessions (:103-107,128-131,189-190)
int open_instance(cc_engine* e, uint32_t rslot, uint64_t index, uint64_t client, uint64_t* instance_id, uint32_t* inst_slot) {
  uint32_t is = 0;
  int rc = alloc_inst_slot(e, &is);
  if (rc) return rc;
  if ((rc = open_range(e, is, 1, rslot, 0, index, client))) return rc;
  *instance_id = index;
  *inst_slot = is;
  return CC_OK;
}

// open_instance for `index` will succeed: a free instance slot and an unused instance id.  Checked before a new key's
// resource is registered, so a failed get / create leaves no keyed resource without an instance behind.
int instance_room(cc_engine* e, uint64_t index) {
  if (e->used_inst.lowest() < 0) return set_err(CC_ERR_CAPACITY, "no free instance slot (max_instances)");
  if (e->inst_by_id.count(index)) return set_err(CC_ERR_INVALID, "instance id (commit index) already open");
  return CC_OK;
}

// A new key: resource id = commit index, a fresh state machine of `type` (:84-100,155-176).
int new_resource(cc_engine* e, uint64_t key, uint32_t type, uint64_t index, uint32_t* rslot) {
  if (type < CC_RES_VALUE || type > CC_RES_MULTIMAP) return set_err(CC_ERR_INVALID, "unknown resource type");
  if (e->res_by_id.count(index)) return set_err(CC_ERR_INVALID, "resource id (commit index) already in use");
  uint32_t s = 0;
  int rc = alloc_res_slot(e, type, &s);
  if (rc) return rc;
  if ((rc = create_range(e, s, 1, type))) return rc;
  e->res_id[s] = index;
  e->res_key[s] = key;
  e->res_has_key[s] = 1;
  e->res_by_id[index] = s;
  e->keys[key] = index;
  *rslot = s;
  return CC_OK;
}

// the existing resource of a key, or TYPE_MISMATCH: `resources.get(id) == null || type differs` (:119-121,178-181)
bool existing(cc_engine* e, uint64_t rid, uint32_t type, uint32_t* rslot) {
  auto it = e->res_by_id.find(rid);
  if (it == e->res_by_id.end() || e->res_type[it->second] != type) return false;
  *rslot = it->second;
  return true;
}

int check_args(cc_engine* e, uint64_t* instance_id, uint32_t* inst_slot, uint8_t* status) {
  if (!e || !instance_id || !inst_slot || !status) return set_err(CC_ERR_INVALID, "null argument");
  return CC_OK;
}

}  // namespace

extern "C" int cc_get_resource(cc_engine* e, uint64_t key, uint32_t type, uint64_t client, uint64_t index,
                               uint64_t* instance_id, uint32_t* inst_slot, uint8_t* status) {
  int rc = check_args(e, instance_id, inst_slot, status);
  if (rc) return rc;
  *status = CC_STATUS(CC_ST_OK, CC_TAG_LONG);
  auto kit = e->keys.find(key);
  if (kit == e->keys.end()) {  // :84-113
    uint32_t rs = 0;
    if ((rc = instance_room(e, index)) || (rc = new_resource(e, key, type, index, &rs))) return rc;
    if ((rc = open_instance(e, rs, index, client, instance_id, inst_slot))) return rc;
    e->res_sessions[{rs, client}] = index;
    return CC_OK;
  }
  uint32_t rs = 0;
  if (!existing(e, kit->second, type, &rs)) {
    *status = CC_STATUS(CC_ST_TYPE_MISMATCH, CC_TAG_NULL);
    return CC_OK;
  }
  auto hit = e->res_sessions.find({rs, client});
  if (hit == e->res_sessions.end()) {  // :126-136 a new instance session for this client
    if ((rc = open_instance(e, rs, index, client, instance_id, inst_slot))) return rc;
    e->res_sessions[{rs, client}] = index;
    return CC_OK;
  }
  // :137-141 the client's open instance (the commit is cleaned)
  auto iit = e->inst_by_id.find(hit->second);
  if (iit == e->inst_by_id.end()) return set_err(CC_ERR_STATE, "ResourceHolder.sessions names a closed instance");
  *instance_id = hit->second;
  *inst_slot = iit->second;
  return CC_OK;
}

extern "C" int cc_create_resource(cc_engine* e, uint64_t key, uint32_t type, uint64_t client, uint64_t index,
                                  uint64_t* instance_id, uint32_t* inst_slot, uint8_t* status) {
  int rc = check_args(e, instance_id, inst_slot, status);
  if (rc) return rc;
  *status = CC_STATUS(CC_ST_OK, CC_TAG_LONG);
  uint32_t rs = 0;
  auto kit = e->keys.find(key);
  if (kit == e->keys.end()) {
    if ((rc = instance_room(e, index)) || (rc = new_resource(e, key, type, index, &rs))) return rc;
  } else if (!existing(e, kit->second, type, &rs)) {
    *status = CC_STATUS(CC_ST_TYPE_MISMATCH, CC_TAG_NULL);
    return CC_OK;
  }
  // :183-195 a unique instance every time, NOT added to ResourceHolder.sessions
  return open_instance(e, rs, index, client, instance_id, inst_slot);
}

extern "C" int cc_resource_exists(cc_engine* e, uint64_t key, uint8_t* exists) {
  if (!e || !exists) return set_err(CC_ERR_INVALID, "null argument");
  *exists = e->keys.count(key) ? 1 : 0;  // :201-207 keys.containsKey (a failed delete keeps the key)
  return CC_OK;
}

// :212-235.  The id is looked up in `resources`; clients send the INSTANCE id (InstanceClient.java:73-74), so only the
// creating instance can delete (A13).  `delete()` throws "commit closed" for a lock / election whose holder commit a
// DeleteCommand already cleaned: the resource is then gone from `resources` but its key and instances stay (zombie).
extern "C" int cc_delete_resource(cc_engine* e, uint64_t resource_id, uint8_t* status) {
  if (!e || !status) return set_err(CC_ERR_INVALID, "null argument");
  auto it = e->res_by_id.find(resource_id);
  if (it == e->res_by_id.end()) {
    *status = CC_STATUS(CC_ST_UNKNOWN_RESOURCE, CC_TAG_NULL);
    return CC_OK;
  }
  const uint32_t slot = it->second;
  const uint8_t type = e->res_type[slot];
  if ((type == CC_RES_LOCK || type == CC_RES_ELECTION) && e->coord_on) {
    int rc = quiesce(e);
    if (rc) return rc;
    CoordHdr h;
    HIPCHECK(hipMemcpy(&h, e->d_coord + (uint64_t)slot * coord_block(e->coord_cap), sizeof h, hipMemcpyDeviceToHost));
    if ((h.flags & kCoHeld) && (h.flags & kCoCleaned)) {  // LockState.delete :87-98 / LeaderElectionState.delete :100-108
      h.flags |= kCoZombie;
      HIPCHECK(hipMemcpy(e->d_coord + (uint64_t)slot * coord_block(e->coord_cap), &h, sizeof h, hipMemcpyHostToDevice));
      e->res_by_id.erase(it);
      e->res_zombie[slot] = 1;
      *status = CC_STATUS(CC_ST_ILLEGAL_STATE, CC_TAG_NULL);
      return CC_OK;
    }
  }
  int rc = delete_slot(e, slot);
  if (rc) return rc;
  *status = CC_STATUS(CC_ST_OK, CC_TAG_BOOL);  // returns true
  return CC_OK;
}

extern "C" int cc_instance_slot(cc_engine* e, uint64_t instance_id, int64_t* slot) {
  if (!e || !slot) return set_err(CC_ERR_INVALID, "null argument");
  auto it = e->inst_by_id.find(instance_id);
  *slot = it == e->inst_by_id.end() ? -1 : (int64_t)it->second;
  return CC_OK;
}

extern "C" int cc_resource_slot(cc_engine* e, uint64_t resource_id, int64_t* slot) {
  if (!e || !slot) return set_err(CC_ERR_INVALID, "null argument");
  auto it = e->res_by_id.find(resource_id);
  *slot = it == e->res_by_id.end() ? -1 : (int64_t)it->second;
  return CC_OK;
}
