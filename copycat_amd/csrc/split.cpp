// split.cpp — one global log, many engines (ABI 5).  Host code only.
//
// The reference multiplexes every resource in ONE Raft log (ResourceManager.java:37-39,56-72): a committed batch holds
// rows of every resource, in log order.  With one engine per GPU (resources sharded by slot), the host must split each
// committed batch by the rank that owns the row's resource before the H2D, and put the per-rank results back in log
// order afterwards.  Resources are independent state machines, so the only order to keep is log order WITHIN a rank
// (a stable split keeps it within every resource too).
//
// cc_split_batch is a multi-threaded count-then-scatter:
//   1. each thread counts its contiguous row range per rank (reads the inst column, 4 B/row, and the owner table);
//   2. exclusive prefix over (thread, rank): thread t's rows of rank r start after every earlier thread's;
//   3. each thread walks its range in blocks of kBlock rows: the block's owner bytes once (L1-resident), then one
//      sequential read of each column, stored to `world` output streams.
// HBM-side bytes: 4 (count) + 4 + 54 read, 54 written per row (+8 with row ids); the split is bound by the host's
// memory bandwidth.  cc_merge_results is the same walk backwards for the result columns (status 1 B, value 8 B).
#include <emmintrin.h>
#include <xmmintrin.h>

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "engine_state.h"

namespace {

constexpr uint32_t kBlock = 8192;  // rows per block (u16 staging slots; 64 KiB of u64 staging)

uint32_t pick_threads(uint32_t threads, uint64_t n) {
  uint32_t t = threads ? threads : std::max(1u, std::thread::hardware_concurrency());
  t = std::min<uint32_t>(t, 256);
  const uint64_t by_size = std::max<uint64_t>(1, n / (4 * kBlock));  // no thread gets less than 4 blocks
  return (uint32_t)std::min<uint64_t>(t, by_size);
}

template <class F>
void parallel(uint32_t threads, F f) {
  if (threads == 1) {
    f(0u);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(threads);
  for (uint32_t t = 0; t < threads; ++t) th.emplace_back(f, t);
  for (auto& x : th) x.join();
}

inline uint8_t owner(const uint32_t* inst, uint64_t i, const uint8_t* rank_of_inst, uint32_t n_inst) {
  const uint32_t s = inst[i];
  return s < n_inst ? rank_of_inst[s] : 0;  // an unknown instance: rank 0's engine answers UNKNOWN_SESSION
}

// per-thread counts per rank; returns false if an owner byte names no rank
bool count_ranks(const uint32_t* inst, uint64_t n, const uint8_t* rank_of_inst, uint32_t n_inst, uint32_t world,
                 uint32_t threads, std::vector<uint64_t>& cnt) {
  cnt.assign((size_t)threads * world, 0);
  std::vector<uint8_t> bad(threads, 0);
  parallel(threads, [&](uint32_t t) {
    const uint64_t lo = n * t / threads, hi = n * (t + 1) / threads;
    // four count tables, rows interleaved over them: consecutive rows of one rank do not wait on each other's
    // increment (a store-to-load chain through one counter costs several cycles per row)
    uint32_t c[4][256] = {};
    uint64_t tot[256] = {0};
    uint8_t mx = 0;
    for (uint64_t b = lo; b < hi; b += 1u << 30) {  // u32 counters: flushed every 2^30 rows
      const uint64_t e = std::min<uint64_t>(hi, b + (1u << 30));
      uint64_t i = b;
      for (; i + 4 <= e; i += 4) {
        const uint8_t r0 = owner(inst, i, rank_of_inst, n_inst), r1 = owner(inst, i + 1, rank_of_inst, n_inst);
        const uint8_t r2 = owner(inst, i + 2, rank_of_inst, n_inst), r3 = owner(inst, i + 3, rank_of_inst, n_inst);
        ++c[0][r0], ++c[1][r1], ++c[2][r2], ++c[3][r3];
        mx = std::max(mx, std::max(std::max(r0, r1), std::max(r2, r3)));
      }
      for (; i < e; ++i) {
        const uint8_t r = owner(inst, i, rank_of_inst, n_inst);
        mx = std::max(mx, r);
        ++c[0][r];
      }
      for (uint32_t r = 0; r < 256; ++r) tot[r] += (uint64_t)c[0][r] + c[1][r] + c[2][r] + c[3][r];
      std::memset(c, 0, sizeof c);
    }
    if (mx >= world) bad[t] = 1;
    std::copy(tot, tot + world, cnt.begin() + (size_t)t * world);
  });
  return std::find(bad.begin(), bad.end(), 1) == bad.end();
}

// Copies `bytes` to dst: the 64-byte lines wholly inside [dst, dst + bytes) with non-temporal stores (a plain store
// would first read each output line from memory: the write-allocate doubles the write traffic), the partial lines at
// either end with plain stores (a neighbouring run may own the rest of such a line).
inline void nt_copy(uint8_t* dst, const uint8_t* src, size_t bytes) {
  uint8_t* const end = dst + bytes;
  uint8_t* a = (uint8_t*)(((uintptr_t)dst + 63) & ~(uintptr_t)63);
  uint8_t* const z = (uint8_t*)((uintptr_t)end & ~(uintptr_t)63);
  if (a >= z) {
    std::memcpy(dst, src, bytes);
    return;
  }
  std::memcpy(dst, src, (size_t)(a - dst));
  src += a - dst;
  for (; a < z; a += 64, src += 64) {
    const __m128i x0 = _mm_loadu_si128((const __m128i*)src), x1 = _mm_loadu_si128((const __m128i*)(src + 16));
    const __m128i x2 = _mm_loadu_si128((const __m128i*)(src + 32)), x3 = _mm_loadu_si128((const __m128i*)(src + 48));
    _mm_stream_si128((__m128i*)a, x0);
    _mm_stream_si128((__m128i*)(a + 16), x1);
    _mm_stream_si128((__m128i*)(a + 32), x2);
    _mm_stream_si128((__m128i*)(a + 48), x3);
  }
  std::memcpy(z, src, (size_t)(end - z));
}

// One column of one block: the block's rows placed at their staging slots (dst: a stable counting sort by rank,
// computed once per block), then each rank's run copied out to its output stream as one contiguous piece.
template <class T>
inline void scatter(const T* in, T* const* out, const uint16_t* dst, uint32_t m, uint32_t world, const uint32_t* boff,
                    const uint64_t* pos, uint8_t* stage) {
  T* st = (T*)stage;
  constexpr uint32_t kLine = 64 / sizeof(T);
  // the same column of the next block is prefetched a line per line read (a prefetch past the end is harmless)
  uint32_t i = 0;
  for (; i + kLine <= m; i += kLine) {
    _mm_prefetch((const char*)(in + kBlock + i), _MM_HINT_T1);
    for (uint32_t j = 0; j < kLine; ++j) st[dst[i + j]] = in[i + j];
  }
  for (; i < m; ++i) st[dst[i]] = in[i];
  for (uint32_t r = 0; r < world; ++r)
    if (const uint32_t c = boff[r + 1] - boff[r])
      nt_copy((uint8_t*)(out[r] + pos[r]), (const uint8_t*)(st + boff[r]), (size_t)c * sizeof(T));
}

template <class T>
inline void gather(T* out, const T* const* in, const uint8_t* own, uint32_t m, uint64_t* cur) {
  for (uint32_t i = 0; i < m; ++i) {
    const uint8_t r = own[i];
    out[i] = in[r][cur[r]++];
  }
}

}  // namespace

extern "C" int cc_split_batch(const cc_batch* in, uint64_t n, const uint8_t* rank_of_inst, uint32_t n_inst,
                              uint32_t world, uint32_t threads, const cc_batch_out* outs, const uint64_t* out_cap,
                              uint64_t* counts, uint64_t* const* rows) {
  using cc::set_err;
  if (!in || !counts || (n && !in->inst) || (n_inst && !rank_of_inst)) return set_err(CC_ERR_INVALID, "split: null argument");
  if (world == 0 || world > 256) return set_err(CC_ERR_INVALID, "split: world must be in [1, 256]");
  const uint32_t T = pick_threads(threads, n);
  std::vector<uint64_t> cnt;
  if (!count_ranks(in->inst, n, rank_of_inst, n_inst, world, T, cnt))
    return set_err(CC_ERR_INVALID, "split: rank_of_inst names a rank >= world");
  for (uint32_t r = 0; r < world; ++r) {
    uint64_t s = 0;
    for (uint32_t t = 0; t < T; ++t) s += cnt[(size_t)t * world + r];
    counts[r] = s;
  }
  if (!outs) return CC_OK;
  if (!out_cap) return set_err(CC_ERR_INVALID, "split: null out_cap");
  // every column the input has, every output has (a missing input column stays missing)
  const void* const icol[9] = {in->index, in->time, in->inst, in->op, in->flags, in->key, in->a, in->b, in->aux};
  for (uint32_t r = 0; r < world; ++r) {
    if (counts[r] > out_cap[r]) return set_err(CC_ERR_CAPACITY, "split: a rank's output columns are too small");
    const void* const ocol[9] = {outs[r].index, outs[r].time, outs[r].inst, outs[r].op, outs[r].flags,
                                 outs[r].key,   outs[r].a,    outs[r].b,    outs[r].aux};
    for (int k = 0; k < 9; ++k)
      if (icol[k] && counts[r] && !ocol[k]) return set_err(CC_ERR_INVALID, "split: null output column");
  }
  // thread t's first output row of rank r
  std::vector<uint64_t> base((size_t)T * world);
  for (uint32_t r = 0; r < world; ++r) {
    uint64_t s = 0;
    for (uint32_t t = 0; t < T; ++t) base[(size_t)t * world + r] = s, s += cnt[(size_t)t * world + r];
  }
  std::vector<uint64_t*> o_u64[6];  // index, time, key, a, b, aux
  std::vector<uint32_t*> o_inst(world);
  std::vector<uint8_t*> o_op(world), o_fl(world);
  for (auto& v : o_u64) v.resize(world);
  for (uint32_t r = 0; r < world; ++r) {
    o_u64[0][r] = outs[r].index, o_u64[1][r] = outs[r].time, o_u64[2][r] = outs[r].key;
    o_u64[3][r] = outs[r].a, o_u64[4][r] = outs[r].b, o_u64[5][r] = outs[r].aux;
    o_inst[r] = outs[r].inst, o_op[r] = outs[r].op, o_fl[r] = outs[r].flags;
  }
  const uint64_t* i_u64[6] = {in->index, in->time, in->key, in->a, in->b, in->aux};
  parallel(T, [&](uint32_t t) {
    const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
    alignas(64) uint8_t own[kBlock];
    alignas(64) uint16_t dst[kBlock];
    std::vector<uint8_t> stage_v(sizeof(uint64_t) * kBlock + 64);
    uint8_t* const stage = (uint8_t*)(((uintptr_t)stage_v.data() + 63) & ~(uintptr_t)63);
    uint64_t pos[256];
    uint32_t boff[257];
    std::copy(base.begin() + (size_t)t * world, base.begin() + (size_t)(t + 1) * world, pos);
    for (uint64_t b = lo; b < hi; b += kBlock) {
      const uint32_t m = (uint32_t)std::min<uint64_t>(kBlock, hi - b);
      // the block's owners, then a stable counting sort by rank: four quarters of the block counted and placed
      // side by side (four independent counter chains per loop step), quarter q's rows of rank r after q-1's
      const bool quad = m % 4 == 0;  // every block but a thread's last one
      const uint32_t Q = quad ? m / 4 : m;
      for (uint32_t i = 0; i < m; ++i) own[i] = owner(in->inst, b + i, rank_of_inst, n_inst);
      uint32_t qc[4][256] = {};
      if (quad)
        for (uint32_t j = 0; j < Q; ++j) ++qc[0][own[j]], ++qc[1][own[Q + j]], ++qc[2][own[2 * Q + j]], ++qc[3][own[3 * Q + j]];
      else
        for (uint32_t i = 0; i < m; ++i) ++qc[0][own[i]];
      uint32_t bc[256], qo[4][256];
      boff[0] = 0;
      for (uint32_t r = 0; r < world; ++r) {
        bc[r] = qc[0][r] + qc[1][r] + qc[2][r] + qc[3][r];
        boff[r + 1] = boff[r] + bc[r];
        qo[0][r] = boff[r], qo[1][r] = qo[0][r] + qc[0][r], qo[2][r] = qo[1][r] + qc[1][r], qo[3][r] = qo[2][r] + qc[2][r];
      }
      if (quad)
        for (uint32_t j = 0; j < Q; ++j) {
          dst[j] = (uint16_t)qo[0][own[j]]++;
          dst[Q + j] = (uint16_t)qo[1][own[Q + j]]++;
          dst[2 * Q + j] = (uint16_t)qo[2][own[2 * Q + j]]++;
          dst[3 * Q + j] = (uint16_t)qo[3][own[3 * Q + j]]++;
        }
      else
        for (uint32_t i = 0; i < m; ++i) dst[i] = (uint16_t)qo[0][own[i]]++;
      scatter(in->inst + b, o_inst.data(), dst, m, world, boff, pos, stage);
      if (in->op) scatter(in->op + b, o_op.data(), dst, m, world, boff, pos, stage);
      if (in->flags) scatter(in->flags + b, o_fl.data(), dst, m, world, boff, pos, stage);
      for (int k = 0; k < 6; ++k)
        if (i_u64[k]) scatter(i_u64[k] + b, o_u64[k].data(), dst, m, world, boff, pos, stage);
      if (rows) {
        uint64_t* st = (uint64_t*)stage;
        for (uint32_t i = 0; i < m; ++i) st[dst[i]] = b + i;
        for (uint32_t r = 0; r < world; ++r)
          if (rows[r] && bc[r]) nt_copy((uint8_t*)(rows[r] + pos[r]), (const uint8_t*)(st + boff[r]), 8ull * bc[r]);
      }
      for (uint32_t r = 0; r < world; ++r) pos[r] += bc[r];
    }
    _mm_sfence();  // the streamed stores are globally visible before the join
  });
  return CC_OK;
}

extern "C" int cc_merge_results(const uint32_t* inst, uint64_t n, const uint8_t* rank_of_inst, uint32_t n_inst,
                                uint32_t world, uint32_t threads, const cc_results* parts, const cc_results* out) {
  using cc::set_err;
  if ((n && (!inst || !parts || !out || !out->status || !out->value)) || (n_inst && !rank_of_inst))
    return set_err(CC_ERR_INVALID, "merge: null argument");
  if (world == 0 || world > 256) return set_err(CC_ERR_INVALID, "merge: world must be in [1, 256]");
  const uint32_t T = pick_threads(threads, n);
  std::vector<uint64_t> cnt;
  if (!count_ranks(inst, n, rank_of_inst, n_inst, world, T, cnt))
    return set_err(CC_ERR_INVALID, "merge: rank_of_inst names a rank >= world");
  std::vector<const uint8_t*> ps(world);
  std::vector<const uint64_t*> pv(world);
  for (uint32_t r = 0; r < world; ++r) {
    uint64_t s = 0;
    for (uint32_t t = 0; t < T; ++t) s += cnt[(size_t)t * world + r];
    if (s && (!parts[r].status || !parts[r].value)) return set_err(CC_ERR_INVALID, "merge: null part column");
    ps[r] = parts[r].status, pv[r] = parts[r].value;
  }
  std::vector<uint64_t> base((size_t)T * world);
  for (uint32_t r = 0; r < world; ++r) {
    uint64_t s = 0;
    for (uint32_t t = 0; t < T; ++t) base[(size_t)t * world + r] = s, s += cnt[(size_t)t * world + r];
  }
  parallel(T, [&](uint32_t t) {
    const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
    uint8_t own[kBlock];
    uint64_t pos[256], cur[256];
    std::copy(base.begin() + (size_t)t * world, base.begin() + (size_t)(t + 1) * world, pos);
    for (uint64_t b = lo; b < hi; b += kBlock) {
      const uint32_t m = (uint32_t)std::min<uint64_t>(kBlock, hi - b);
      for (uint32_t i = 0; i < m; ++i) own[i] = owner(inst, b + i, rank_of_inst, n_inst);
      std::copy(pos, pos + world, cur);
      gather(out->status + b, ps.data(), own, m, cur);
      std::copy(pos, pos + world, cur);
      gather(out->value + b, pv.data(), own, m, cur);
      for (uint32_t i = 0; i < m; ++i) ++pos[own[i]];
    }
  });
  return CC_OK;
}
