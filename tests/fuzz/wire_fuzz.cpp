// wire_fuzz.cpp — host-only fuzz driver for cc_wire_decode (copycat_amd/csrc/wire.cpp), built with
// -fsanitize=address,undefined by tests/test_wire_asan.py (test infrastructure; never part of the product library).
//
// cc_wire_decode parses committed log bytes (InstanceOperation.writeObject/readObject,
// manager/src/main/java/io/atomix/resource/InstanceOperation.java:59-69), so every input below must come back as
// CC_OK or CC_ERR_INVALID, with no read outside the caller's buffer: each entry is decoded from a heap copy of
// exactly its bytes, so the sanitizer sees any overread.  Inputs: the committed fixture (tests/golden/wire_fixture.*),
// every truncation of every fixture entry, random byte flips, random splices of two entries, random garbage, and
// random codec parameters.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "engine_state.h"

namespace cc {
int set_err(int code, const char*, hipError_t) { return code; }  // the engine's cc_last_error store is not linked
}  // namespace cc
extern "C" int cc_handle_hashes(cc_engine*, const uint64_t*, const int32_t*, uint64_t) { return CC_OK; }

namespace {
uint64_t g_rng = 0x9E3779B97F4A7C15ull;
uint64_t rnd() {  // splitmix64
  uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
uint64_t n_ok = 0, n_invalid = 0;

bool decode(cc_wire_interner* in, const cc_wire_codec* codec, const std::vector<uint8_t>& bytes) {
  // an exact-size heap copy: one byte past it is an ASan report
  uint8_t* buf = (uint8_t*)malloc(bytes.empty() ? 1 : bytes.size());
  if (!bytes.empty()) memcpy(buf, bytes.data(), bytes.size());
  uint64_t offs[2] = {0, bytes.size()};
  uint8_t op, flags, kind;
  uint64_t key, a, b, aux, iid, bad = ~0ull;
  cc_wire_out out{};
  out.iid = &iid;
  out.op = &op;
  out.flags = &flags;
  out.key = &key;
  out.a = &a;
  out.b = &b;
  out.aux = &aux;
  out.kind = &kind;
  const int rc = cc_wire_decode(nullptr, codec, in, buf, bytes.size(), offs, 1, &out, &bad);
  free(buf);
  if (rc == CC_OK) ++n_ok;
  else if (rc == CC_ERR_INVALID) ++n_invalid;
  else {
    fprintf(stderr, "unexpected rc %d\n", rc);
    return false;
  }
  return true;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: wire_fuzz FIXTURE.bin OFFSETS.txt ITERATIONS\n");
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> blob;
  for (int c; (c = fgetc(f)) != EOF;) blob.push_back((uint8_t)c);
  fclose(f);
  std::vector<uint64_t> off;
  FILE* g = fopen(argv[2], "r");
  if (!g) return 2;
  for (unsigned long long x; fscanf(g, "%llu", &x) == 1;) off.push_back(x);
  fclose(g);
  const long iters = atol(argv[3]);
  cc_wire_interner* in = nullptr;
  if (cc_wire_interner_create(1, &in) != CC_OK) return 2;
  cc_wire_codec def;
  cc_wire_codec_default(&def);

  std::vector<std::vector<uint8_t>> ents;
  for (size_t i = 0; i + 1 < off.size(); ++i) ents.emplace_back(blob.begin() + off[i], blob.begin() + off[i + 1]);
  // the fixture decodes
  for (auto& e : ents) {
    const uint64_t before = n_ok;
    if (!decode(in, &def, e)) return 1;
    if (n_ok == before) {
      fprintf(stderr, "a fixture entry failed to decode\n");
      return 1;
    }
  }
  // every truncation of every entry
  for (auto& e : ents)
    for (size_t n = 0; n < e.size(); ++n)
      if (!decode(in, &def, std::vector<uint8_t>(e.begin(), e.begin() + n))) return 1;
  for (long it = 0; it < iters; ++it) {
    std::vector<uint8_t> x = ents[rnd() % ents.size()];
    cc_wire_codec c = def;
    switch (rnd() % 5) {
      case 0: {  // byte flips
        const int k = 1 + (int)(rnd() % 4);
        for (int j = 0; j < k && !x.empty(); ++j) x[rnd() % x.size()] ^= (uint8_t)(1 + rnd() % 255);
        break;
      }
      case 1: {  // splice: a prefix of one entry + a suffix of another
        const auto& y = ents[rnd() % ents.size()];
        x.resize(x.empty() ? 0 : rnd() % x.size());
        const size_t from = y.empty() ? 0 : rnd() % y.size();
        x.insert(x.end(), y.begin() + from, y.end());
        break;
      }
      case 2: {  // garbage
        x.resize(rnd() % 80);
        for (auto& b : x) b = (uint8_t)rnd();
        break;
      }
      case 3: {  // random codec parameters over a valid or flipped entry
        c.big_endian = rnd() & 1;
        c.utf8_presence_byte = rnd() & 1;
        c.utf8_len_bytes = 1 + (uint32_t)(rnd() % 8);
        if (!x.empty() && (rnd() & 1)) x[rnd() % x.size()] ^= 0x80;
        break;
      }
      default: {  // huge length fields: 0xFF runs at a random place
        if (!x.empty()) {
          const size_t at = rnd() % x.size();
          for (size_t j = at; j < x.size() && j < at + 8; ++j) x[j] = 0xFF;
        }
        break;
      }
    }
    if (!decode(in, &c, x)) return 1;
  }
  cc_wire_interner_destroy(in);
  printf("wire_fuzz: %llu decoded, %llu rejected as CC_ERR_INVALID\n", (unsigned long long)n_ok,
         (unsigned long long)n_invalid);
  return 0;
}
