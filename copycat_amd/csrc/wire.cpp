// wire.cpp — Catalyst wire format -> the engine's columns.
//
// A committed Atomix entry carries a Catalyst-serialized operation.  Resource operations are InstanceCommand /
// InstanceQuery (@SerializeWith 30 / 31, manager/.../resource/InstanceCommand.java:26, InstanceQuery.java:26):
// `writeLong(resource)` — the instance id — then `serializer.writeObject(operation)` (InstanceOperation.java:60-69).
// The inner operation's @SerializeWith id is this engine's op code (include/copycat_apply.h), and its fields follow
// its class's writeObject chain; kSchema below restates each one (file:line).  Manager operations
// (GetResource 35, CreateResource 36, DeleteResource 37, ResourceExists 38: manager/.../manager/*.java) are decoded
// into control rows for cc_get_resource / cc_create_resource / cc_delete_resource / cc_resource_exists.
//
// Catalyst itself (Serializer, Buffer) is not vendored: its byte-level conventions — the identifier
// byte before a registered type id, the ids of the boxed primitives and String, byte order, writeUTF8's
// framing — are parameters (cc_wire_codec) whose defaults restate Catalyst 1.x as documented in DESIGN.md; the
// byte layout is "parity unpinned", the field order per op is pinned to the reference's writeObject sources.
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "engine_state.h"

namespace {

// Catalyst Serializer identifier bytes: the width of the type id that follows (null has none)
enum : uint8_t { kIdNull = 0x00, kIdInt8 = 0x01, kIdInt16 = 0x02, kIdInt24 = 0x03, kIdInt32 = 0x04, kIdClass = 0x05 };

// operand slots of one op, in wire order
enum Field : uint8_t {
  F_END = 0,
  F_KEY,      // serializer.writeObject(key): a non-null key -> key column + key tag
  F_KEY_OPT,  // same, may be null (MultiMapCommands.Size() without a key): key 0
  F_A,        // serializer.writeObject(value) -> operand a
  F_B,        // serializer.writeObject(...) -> operand b
  F_AUX,      // buffer.writeLong(ttl / timeout / delay) -> aux
  F_LKEY,     // buffer.writeLong(member) -> key column, key tag LONG
};

struct Schema {
  uint8_t op;
  Field f[5];
};

// Field order per @SerializeWith id, from the writeObject chains of the reference's command classes.
const Schema kSchema[] = {
    // AtomicValueCommands.java: Get/Listen/Unlisten write nothing (:82,:249,:263); Set/GetAndSet write only the
    // value (:126,:228 — they override ValueCommand.writeObject, so ttl never travels, A2); CompareAndSet
    // expect, update (:182-184)
    {CC_OP_VALUE_GET, {F_END}},
    {CC_OP_VALUE_SET, {F_A, F_END}},
    {CC_OP_VALUE_CAS, {F_A, F_B, F_END}},
    {CC_OP_VALUE_GETANDSET, {F_A, F_END}},
    {CC_OP_VALUE_LISTEN, {F_END}},
    {CC_OP_VALUE_UNLISTEN, {F_END}},
    // MapCommands.java: KeyQuery/KeyCommand key (:88,:119-121); ContainsValue value (:166-168); KeyValueCommand
    // key, value (:200-202); TtlCommand key, value, ttl (:241-243); GetOrDefault key, default (:331-333);
    // ReplaceIfPresent key, value, ttl, replace (:421-423); IsEmpty/Size/Clear nothing
    {CC_OP_MAP_CONTAINSKEY, {F_KEY, F_END}},
    {CC_OP_MAP_CONTAINSVALUE, {F_A, F_END}},
    {CC_OP_MAP_PUT, {F_KEY, F_A, F_AUX, F_END}},
    {CC_OP_MAP_PUTIFABSENT, {F_KEY, F_A, F_AUX, F_END}},
    {CC_OP_MAP_GET, {F_KEY, F_END}},
    {CC_OP_MAP_GETORDEFAULT, {F_KEY, F_A, F_END}},
    {CC_OP_MAP_REMOVE, {F_KEY, F_END}},
    {CC_OP_MAP_REMOVEIFPRESENT, {F_KEY, F_A, F_END}},
    {CC_OP_MAP_REPLACE, {F_KEY, F_A, F_AUX, F_END}},
    {CC_OP_MAP_REPLACEIFPRESENT, {F_KEY, F_A, F_AUX, F_B, F_END}},
    {CC_OP_MAP_ISEMPTY, {F_END}},
    {CC_OP_MAP_SIZE, {F_END}},
    {CC_OP_MAP_CLEAR, {F_END}},
    // MultiMapCommands.java: KeyQuery key (:121-123); EntryQuery key, value (:190-192); ValueQuery value
    // (:154-156); TtlCommand key, value, ttl (:308-310); EntryCommand key, value (:267-269); RemoveValue value
    // (:399-400); Size is a KeyQuery whose key may be null (:420-430)
    {CC_OP_MMAP_CONTAINSKEY, {F_KEY, F_END}},
    {CC_OP_MMAP_CONTAINSENTRY, {F_KEY, F_A, F_END}},
    {CC_OP_MMAP_CONTAINSVALUE, {F_A, F_END}},
    {CC_OP_MMAP_PUT, {F_KEY, F_A, F_AUX, F_END}},
    {CC_OP_MMAP_GET, {F_KEY, F_END}},
    {CC_OP_MMAP_REMOVE, {F_KEY, F_A, F_END}},
    {CC_OP_MMAP_REMOVEVALUE, {F_A, F_END}},
    {CC_OP_MMAP_ISEMPTY, {F_END}},
    {CC_OP_MMAP_SIZE, {F_KEY_OPT, F_END}},
    {CC_OP_MMAP_CLEAR, {F_END}},
    // QueueCommands.java: ValueCommand / ValueQuery value (:87-88,:118-120); the rest nothing
    {CC_OP_QUEUE_CONTAINS, {F_A, F_END}},
    {CC_OP_QUEUE_ADD, {F_A, F_END}},
    {CC_OP_QUEUE_OFFER, {F_A, F_END}},
    {CC_OP_QUEUE_PEEK, {F_END}},
    {CC_OP_QUEUE_POLL, {F_END}},
    {CC_OP_QUEUE_ELEMENT, {F_END}},
    {CC_OP_QUEUE_REMOVE, {F_A, F_END}},
    {CC_OP_QUEUE_SIZE, {F_END}},
    {CC_OP_QUEUE_ISEMPTY, {F_END}},
    {CC_OP_QUEUE_CLEAR, {F_END}},
    // SetCommands.java: the element travels as the key column (ValueCommand / ValueQuery value :87-88,:118-120);
    // Add = TtlCommand element, ttl (:172-174)
    {CC_OP_SET_CONTAINS, {F_KEY, F_END}},
    {CC_OP_SET_ADD, {F_KEY, F_AUX, F_END}},
    {CC_OP_SET_REMOVE, {F_KEY, F_END}},
    {CC_OP_SET_SIZE, {F_END}},
    {CC_OP_SET_ISEMPTY, {F_END}},
    {CC_OP_SET_CLEAR, {F_END}},
    // LeaderElectionCommands.java: nothing (:50,:69)
    {CC_OP_ELECT_LISTEN, {F_END}},
    {CC_OP_ELECT_UNLISTEN, {F_END}},
    {CC_OP_ELECT_ISLEADER, {F_END}},
    // LockCommands.java: Lock timeout (:80-81); Unlock nothing
    {CC_OP_LOCK_LOCK, {F_AUX, F_END}},
    {CC_OP_LOCK_UNLOCK, {F_END}},
    // MembershipGroupCommands.java: Join/Leave nothing; Schedule member, delay, callback (:124-126); Execute
    // member, callback (:172-174)
    {CC_OP_GROUP_JOIN, {F_END}},
    {CC_OP_GROUP_LEAVE, {F_END}},
    {CC_OP_GROUP_SCHEDULE, {F_LKEY, F_AUX, F_A, F_END}},
    {CC_OP_GROUP_EXECUTE, {F_LKEY, F_A, F_END}},
};

const Schema* schema_of(uint32_t id) {
  static const std::vector<const Schema*> table = [] {  // (thread-safe one-time initialisation)
    std::vector<const Schema*> t(256, nullptr);
    for (const Schema& s : kSchema) t[s.op] = &s;
    return t;
  }();
  return id < 256 ? table[id] : nullptr;
}

// ResourceManager instantiates `type` by class name (GetResource.java:62-79, ResourceManager.java:92,165)
uint32_t res_type_of_class(const std::string& name) {
  static const std::pair<const char*, uint32_t> kClasses[] = {
      {"io.atomix.atomic.state.AtomicValueState", CC_RES_VALUE},
      {"io.atomix.collections.state.MapState", CC_RES_MAP},
      {"io.atomix.collections.state.SetState", CC_RES_SET},
      {"io.atomix.collections.state.QueueState", CC_RES_QUEUE},
      {"io.atomix.collections.state.MultiMapState", CC_RES_MULTIMAP},
      {"io.atomix.coordination.state.LockState", CC_RES_LOCK},
      {"io.atomix.coordination.state.LeaderElectionState", CC_RES_ELECTION},
      {"io.atomix.coordination.state.MembershipGroupState", CC_RES_GROUP},
  };
  for (const auto& c : kClasses)
    if (name == c.first) return c.second;
  return CC_RES_NONE;
}

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool be;
  bool ok = true;
  uint64_t uint(int n) {  // an n-byte unsigned integer in the codec's byte order
    if (!ok || end - p < n) {
      ok = false;
      return 0;
    }
    uint64_t v = 0;
    if (be)
      for (int i = 0; i < n; ++i) v = (v << 8) | p[i];
    else
      for (int i = n - 1; i >= 0; --i) v = (v << 8) | p[i];
    p += n;
    return v;
  }
  bool bytes(uint64_t n, const uint8_t*& out) {
    if (!ok || (uint64_t)(end - p) < n) return ok = false;
    out = p;
    p += n;
    return true;
  }
};

}  // namespace

struct cc_wire_interner {
  uint64_t next;
  std::unordered_map<std::string, uint64_t> ids;
  std::vector<std::string> strs;  // handle - first -> bytes
  uint64_t first;
  std::vector<int32_t> hashes;    // handle - first -> java.lang.String.hashCode
};

using namespace cc;

namespace {

// Catalyst writeUTF8 (KeyOperation.java:53-54; String values through the String serializer)
bool read_utf8(Reader& r, const cc_wire_codec& c, std::string& s, bool& null) {
  null = false;
  if (c.utf8_presence_byte && !r.uint(1)) {
    null = true;
    return r.ok;
  }
  const uint64_t n = r.uint(c.utf8_len_bytes);
  const uint8_t* b = nullptr;
  if (!r.bytes(n, b)) return false;
  s.assign((const char*)b, n);
  return true;
}

// java.lang.String.hashCode of the String decoded from UTF-8 bytes: s[0]*31^(n-1) + ... + s[n-1] over its UTF-16
// code units (a code point above U+FFFF is a surrogate pair; a malformed sequence decodes to U+FFFD, as Java's
// UTF-8 decoder replaces it).
int32_t java_string_hash(const std::string& s) {
  uint32_t h = 0;
  auto unit = [&](uint32_t u) { h = 31u * h + u; };
  const uint8_t* p = (const uint8_t*)s.data();
  const size_t n = s.size();
  for (size_t i = 0; i < n;) {
    const uint32_t b = p[i];
    uint32_t cp = 0xFFFD, len = 1;
    if (b < 0x80) cp = b;
    else if ((b >> 5) == 6 && i + 1 < n && (p[i + 1] >> 6) == 2) cp = ((b & 0x1F) << 6) | (p[i + 1] & 0x3F), len = 2;
    else if ((b >> 4) == 14 && i + 2 < n && (p[i + 1] >> 6) == 2 && (p[i + 2] >> 6) == 2)
      cp = ((b & 0x0F) << 12) | ((p[i + 1] & 0x3F) << 6) | (p[i + 2] & 0x3F), len = 3;
    else if ((b >> 3) == 30 && i + 3 < n && (p[i + 1] >> 6) == 2 && (p[i + 2] >> 6) == 2 && (p[i + 3] >> 6) == 2)
      cp = ((b & 0x07) << 18) | ((p[i + 1] & 0x3F) << 12) | ((p[i + 2] & 0x3F) << 6) | (p[i + 3] & 0x3F), len = 4;
    if ((len == 2 && cp < 0x80) || (len == 3 && (cp < 0x800 || (cp >= 0xD800 && cp < 0xE000))) ||
        (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)))
      cp = 0xFFFD;  // overlong / surrogate / out of range
    if (cp >= 0x10000) {
      unit(0xD800 + ((cp - 0x10000) >> 10));
      unit(0xDC00 + ((cp - 0x10000) & 0x3FF));
    } else {
      unit(cp);
    }
    i += len;
  }
  return (int32_t)h;
}

uint64_t intern(cc_wire_interner* in, const std::string& s) {
  auto it = in->ids.find(s);
  if (it != in->ids.end()) return it->second;
  const uint64_t h = in->next++;
  in->ids.emplace(s, h);
  in->strs.push_back(s);
  in->hashes.push_back(java_string_hash(s));
  return h;
}

// serializer.writeObject(value): null, or identifier + registered id + the type's serializer payload.
// -> (tag, payload); false: truncated, or a type with no canonical tag (a user class) -> *why
bool read_value(Reader& r, const cc_wire_codec& c, cc_wire_interner* in, uint32_t& tag, uint64_t& v, const char** why) {
  const uint8_t ident = (uint8_t)r.uint(1);
  if (!r.ok) return false;
  if (ident == kIdNull) {
    tag = CC_TAG_NULL;
    v = 0;
    return true;
  }
  int w = 0;
  switch (ident) {
    case kIdInt8: w = 1; break;
    case kIdInt16: w = 2; break;
    case kIdInt24: w = 3; break;
    case kIdInt32: w = 4; break;
    default:
      *why = ident == kIdClass ? "value of an unregistered class (serialized by class name)" : "unknown identifier byte";
      return false;
  }
  uint64_t raw = r.uint(w);
  if (!r.ok) return false;
  const int64_t id = (int64_t)(raw << (64 - 8 * w)) >> (64 - 8 * w);  // ids are signed
  if (id == c.id_long) {
    tag = CC_TAG_LONG;
    v = r.uint(8);
  } else if (id == c.id_int) {
    tag = CC_TAG_INT;
    v = (uint64_t)(int64_t)(int32_t)(uint32_t)r.uint(4);
  } else if (id == c.id_bool) {
    tag = CC_TAG_BOOL;
    v = r.uint(1) ? 1 : 0;
  } else if (id == c.id_string) {
    std::string s;
    bool null = false;
    if (!read_utf8(r, c, s, null)) return false;
    tag = null ? CC_TAG_NULL : CC_TAG_HANDLE;
    v = null ? 0 : intern(in, s);
  } else {
    *why = "value of a registered type with no canonical tag (only Long, Integer, Boolean, String and null travel)";
    return false;
  }
  return r.ok;
}

int decode_one(cc_engine* e, const cc_wire_codec& c, cc_wire_interner* in, const uint8_t* p, const uint8_t* end,
               uint64_t row, const cc_wire_out* out) {
  Reader r{p, end, c.big_endian != 0};
  const char* why = "truncated entry";
  auto fail = [&](const char* msg) { return set_err(CC_ERR_INVALID, (std::string("wire row ") + std::to_string(row) + ": " + msg).c_str()); };
  // the entry's operation: identifier + id
  auto read_id = [&](int64_t& id) -> bool {
    const uint8_t ident = (uint8_t)r.uint(1);
    int w = ident == kIdInt8 ? 1 : ident == kIdInt16 ? 2 : ident == kIdInt24 ? 3 : ident == kIdInt32 ? 4 : 0;
    if (!w) return false;
    const uint64_t raw = r.uint(w);
    id = (int64_t)(raw << (64 - 8 * w)) >> (64 - 8 * w);
    return r.ok;
  };
  int64_t top = 0;
  if (!read_id(top)) return fail("entry is not a registered Catalyst type");
  if (out->inst) out->inst[row] = e ? e->cfg.max_instances : 0;
  if (out->iid) out->iid[row] = 0;
  out->op[row] = 0;
  out->flags[row] = 0;
  out->key[row] = out->a[row] = out->b[row] = out->aux[row] = 0;
  out->kind[row] = 0;
  if (top == 35 || top == 36 || top == 38) {  // GetResource / CreateResource / ResourceExists: key [, type]
    std::string key, type;
    bool null = false;
    if (!read_utf8(r, c, key, null)) return fail(why);
    if (null) return fail("resource key is null");
    out->kind[row] = (uint8_t)top;
    out->key[row] = intern(in, key);
    if (top != 38) {  // buffer.writeInt(len).write(type name bytes) (GetResource.java:62-65, CreateResource.java:57-60)
      const uint64_t n = r.uint(4);
      const uint8_t* b = nullptr;
      if (!r.bytes(n, b)) return fail(why);
      out->a[row] = res_type_of_class(std::string((const char*)b, n));
    }
    return r.p == end ? CC_OK : fail("trailing bytes after the manager operation");
  }
  if (top == 37) {  // DeleteResource: writeLong(resource) (DeleteResource.java:56)
    out->kind[row] = 37;
    out->b[row] = r.uint(8);
    return r.ok && r.p == end ? CC_OK : fail(why);
  }
  if (top != 30 && top != 31) return fail("not an InstanceCommand / InstanceQuery / manager operation");
  const uint64_t iid = r.uint(8);  // InstanceOperation.writeObject: writeLong(resource) = the instance id
  int64_t id = 0;
  if (!read_id(id)) return fail("inner operation is not a registered Catalyst type");
  const Schema* s = (id >= 0 && id < 256) ? schema_of((uint32_t)id) : nullptr;
  if (!s) return fail("inner operation id is no resource operation this engine knows");
  if (out->iid) out->iid[row] = iid;
  if (e) {
    auto it = e->inst_by_id.find(iid);
    out->inst[row] = it == e->inst_by_id.end() ? e->cfg.max_instances : it->second;  // unknown: UNKNOWN_SESSION
  }
  out->op[row] = s->op;
  uint32_t ta = CC_TAG_NULL, tb = CC_TAG_NULL, kt = 0;
  for (int k = 0; k < 5 && s->f[k] != F_END; ++k) {
    uint32_t tag = 0;
    uint64_t v = 0;
    switch (s->f[k]) {
      case F_KEY:
      case F_KEY_OPT:
        if (!read_value(r, c, in, tag, v, &why)) return fail(why);
        if (tag == CC_TAG_NULL) {
          if (s->f[k] == F_KEY) return fail("null key (KeyCommand asserts notNull)");
          break;
        }
        kt = tag == CC_TAG_LONG ? 0u : tag == CC_TAG_INT ? 1u : tag == CC_TAG_BOOL ? 2u : 3u;
        out->key[row] = v;
        break;
      case F_A:
        if (!read_value(r, c, in, ta, v, &why)) return fail(why);
        out->a[row] = v;
        break;
      case F_B:
        if (!read_value(r, c, in, tb, v, &why)) return fail(why);
        out->b[row] = v;
        break;
      case F_AUX:
        out->aux[row] = r.uint(8);
        break;
      case F_LKEY:
        out->key[row] = r.uint(8);
        kt = 0;
        break;
      case F_END:
        break;
    }
    if (!r.ok) return fail("truncated entry");
  }
  if (r.p != end) return fail("trailing bytes after the operation's fields");
  out->flags[row] = CC_FLAGS(ta, tb, kt);
  return CC_OK;
}

}  // namespace

extern "C" void cc_wire_codec_default(cc_wire_codec* c) {
  if (!c) return;
  memset(c, 0, sizeof *c);
  c->big_endian = 1;
  c->utf8_presence_byte = 1;
  c->utf8_len_bytes = 2;
  c->id_bool = CC_WIRE_ID_BOOLEAN;
  c->id_int = CC_WIRE_ID_INTEGER;
  c->id_long = CC_WIRE_ID_LONG;
  c->id_string = CC_WIRE_ID_STRING;
}

extern "C" int cc_wire_interner_create(uint64_t first_handle, cc_wire_interner** out) {
  if (!out || !first_handle) return set_err(CC_ERR_INVALID, "interner: null output or handle 0");
  *out = new cc_wire_interner{first_handle, {}, {}, first_handle};
  return CC_OK;
}

extern "C" int cc_wire_interner_destroy(cc_wire_interner* in) {
  delete in;
  return CC_OK;
}

extern "C" int cc_wire_intern(cc_wire_interner* in, const uint8_t* bytes, uint64_t len, uint64_t* handle) {
  if (!in || !handle || (len && !bytes)) return set_err(CC_ERR_INVALID, "intern: null argument");
  *handle = intern(in, std::string((const char*)bytes, len));
  return CC_OK;
}

extern "C" int cc_wire_string_hash(cc_wire_interner* in, uint64_t handle, int32_t* hash) {
  if (!in || !hash || handle < in->first || handle - in->first >= in->hashes.size())
    return set_err(CC_ERR_INVALID, "unknown handle");
  *hash = in->hashes[handle - in->first];
  return CC_OK;
}

extern "C" int cc_wire_lookup(cc_wire_interner* in, uint64_t handle, uint8_t* buf, uint64_t cap, uint64_t* len) {
  if (!in || !len || handle < in->first || handle - in->first >= in->strs.size())
    return set_err(CC_ERR_INVALID, "lookup: unknown handle");
  const std::string& s = in->strs[handle - in->first];
  *len = s.size();
  if (buf) memcpy(buf, s.data(), std::min<uint64_t>(cap, s.size()));
  return CC_OK;
}

extern "C" int cc_wire_decode(cc_engine* e, const cc_wire_codec* codec, cc_wire_interner* in, const uint8_t* buf,
                              uint64_t buf_len, const uint64_t* offsets, uint64_t n, const cc_wire_out* out,
                              uint64_t* bad_row) {
  if (!in || !buf || !offsets || !out || !out->op || !out->flags || !out->key || !out->a || !out->b || !out->aux ||
      !out->kind || (e && !out->inst) || (!e && !out->iid))
    return set_err(CC_ERR_INVALID, "wire decode: null argument");
  cc_wire_codec c;
  if (codec) c = *codec;
  else cc_wire_codec_default(&c);
  if (c.utf8_len_bytes < 1 || c.utf8_len_bytes > 8) return set_err(CC_ERR_INVALID, "wire codec: utf8_len_bytes");
  for (uint64_t i = 0; i < n; ++i) {
    if (offsets[i + 1] < offsets[i]) {
      if (bad_row) *bad_row = i;
      return set_err(CC_ERR_INVALID, "wire decode: offsets decrease");
    }
    if (offsets[i + 1] > buf_len) {  // never read past the caller's buffer
      if (bad_row) *bad_row = i;
      return set_err(CC_ERR_INVALID, "wire decode: entry ends past the buffer");
    }
    const int rc = decode_one(e, c, in, buf + offsets[i], buf + offsets[i + 1], i, out);
    if (rc) {
      if (bad_row) *bad_row = i;
      return rc;
    }
  }
  if (e) {  // the String.hashCode of every String key decoded, for the engine's java.util.HashMap model
    std::vector<uint64_t> hk;
    std::vector<int32_t> hv;
    for (uint64_t i = 0; i < n; ++i)
      if (out->kind[i] == 0 && CC_FLAG_KTAG(out->flags[i]) == 3u && out->key[i] >= in->first &&
          out->key[i] - in->first < in->hashes.size() && !e->hh.count(out->key[i])) {
        hk.push_back(out->key[i]);
        hv.push_back(in->hashes[out->key[i] - in->first]);
      }
    if (!hk.empty()) return cc_handle_hashes(e, hk.data(), hv.data(), hk.size());
  }
  return CC_OK;
}
