// quorum.hip — leader-side quorum commit index and the session/lease expiry sweep (a15).
//
// Both live in Copycat 1.0.0-beta4 (copycat-server, not vendored in the reference: pom.xml:26), so the rule
// each kernel computes is defined by this engine and pinned by its own KATs (tests/test_oracle_kats.py):
//   quorum : commit = quorum-th largest matchIndex (leader's last index included), only if it is at least the
//            first index of the leader's term and larger than the old commit index (Raft §5.3, §5.4.2).
//   expiry : session s expired iff now - lastKeepAlive[s] > sessionTimeout (signed difference); the result is
//            a bitmap (1 bit per session) — the set ResourceManager.expire/close fan out over
//            (ResourceManager.java:237-264).
// Both are pure HBM streams: 16-byte loads per lane, no LDS, grid-stride.
#include "common.h"

namespace cc {

// quorum-th largest of R values (R small, in registers): selection by counting ranks.
template <int R>
__device__ inline uint64_t kth_largest(const uint64_t (&m)[R], int q) {
  // sort descending with a fully unrolled insertion network
  uint64_t s[R];
#pragma unroll
  for (int i = 0; i < R; ++i) s[i] = m[i];
#pragma unroll
  for (int i = 1; i < R; ++i)
#pragma unroll
    for (int j = i; j > 0; --j) {
      const uint64_t x = s[j - 1], y = s[j];
      s[j - 1] = x > y ? x : y;
      s[j] = x > y ? y : x;
    }
  uint64_t r = s[0];
#pragma unroll
  for (int i = 0; i < R; ++i)
    if (i == q - 1) r = s[i];
  return r;
}

template <int R>
__global__ __launch_bounds__(256) void k_quorum(const uint64_t* __restrict__ match, uint64_t groups,
                                                const uint64_t* __restrict__ term_start, const uint64_t* __restrict__ cin,
                                                uint64_t* __restrict__ cout) {
  constexpr int q = R / 2 + 1;
  const uint64_t pairs = groups / 2;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < pairs; p += stride) {
    uint64_t m0[R], m1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u64x2 v = reinterpret_cast<const u64x2*>(match + (uint64_t)r * groups)[p];
      m0[r] = v.x;
      m1[r] = v.y;
    }
    const u64x2 ts = reinterpret_cast<const u64x2*>(term_start)[p];
    const u64x2 ci = reinterpret_cast<const u64x2*>(cin)[p];
    const uint64_t n0 = kth_largest<R>(m0, q), n1 = kth_largest<R>(m1, q);
    u64x2 o;
    o.x = (n0 >= ts.x && n0 > ci.x) ? n0 : ci.x;
    o.y = (n1 >= ts.y && n1 > ci.y) ? n1 : ci.y;
    reinterpret_cast<u64x2*>(cout)[p] = o;
  }
  // odd tail
  if (blockIdx.x == 0 && threadIdx.x == 0 && (groups & 1)) {
    const uint64_t g = groups - 1;
    uint64_t m[R];
#pragma unroll
    for (int r = 0; r < R; ++r) m[r] = match[(uint64_t)r * groups + g];
    const uint64_t n = kth_largest<R>(m, q);
    cout[g] = (n >= term_start[g] && n > cin[g]) ? n : cin[g];
  }
}

// generic replica count (unaligned / unusual R): one group per thread, R <= 16
__global__ __launch_bounds__(256) void k_quorum_generic(const uint64_t* __restrict__ match, uint32_t R, uint64_t groups,
                                                        const uint64_t* __restrict__ term_start,
                                                        const uint64_t* __restrict__ cin, uint64_t* __restrict__ cout) {
  const uint32_t q = R / 2 + 1;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += stride) {
    uint64_t n = 0;
    for (uint32_t i = 0; i < R; ++i) {  // the value with exactly-(q-1)-larger rank: count larger/equal
      const uint64_t x = match[(uint64_t)i * groups + g];
      uint32_t gt = 0, ge = 0;
      for (uint32_t j = 0; j < R; ++j) {
        const uint64_t y = match[(uint64_t)j * groups + g];
        gt += y > x;
        ge += y >= x;
      }
      if (gt < q && ge >= q) n = x;
    }
    cout[g] = (n >= term_start[g] && n > cin[g]) ? n : cin[g];
  }
}

// spread the low 32 bits of x to the even bit positions of a 64-bit word
__device__ inline uint64_t spread32(uint64_t x) {
  x &= 0xFFFFFFFFull;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x << 2)) & 0x3333333333333333ull;
  x = (x | (x << 1)) & 0x5555555555555555ull;
  return x;
}

// Each wave covers 128 sessions per step (16 B per lane); the two ballots interleave into 2 bitmap words.
__global__ __launch_bounds__(256) void k_expire(const uint64_t* __restrict__ last, uint64_t sessions, uint64_t now,
                                                int64_t timeout, uint64_t* __restrict__ bitmap,
                                                unsigned long long* __restrict__ count) {
  const uint32_t l = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint64_t steps = (sessions + 127) / 128;
  uint32_t c = 0;
  for (uint64_t s = wave; s < steps; s += waves) {
    const uint64_t i0 = s * 128 + 2 * l;
    bool e0 = false, e1 = false;
    if (i0 + 1 < sessions) {
      const u64x2 v = reinterpret_cast<const u64x2*>(last)[i0 / 2];
      e0 = (int64_t)(now - v.x) > timeout;
      e1 = (int64_t)(now - v.y) > timeout;
    } else if (i0 < sessions) {
      e0 = (int64_t)(now - last[i0]) > timeout;
    }
    const uint64_t m0 = ballot(e0), m1 = ballot(e1);
    if (l == 0) {
      const uint64_t wlo = spread32(m0) | (spread32(m1) << 1);
      const uint64_t whi = spread32(m0 >> 32) | (spread32(m1 >> 32) << 1);
      const uint64_t w = s * 2;
      const uint64_t words = (sessions + 63) / 64;
      bitmap[w] = wlo;
      if (w + 1 < words) bitmap[w + 1] = whi;
      c += (uint32_t)__popcll(m0) + (uint32_t)__popcll(m1);
    }
  }
  // one counter update per workgroup: thousands of same-address atomics would serialize at the L2
  __shared__ uint32_t wc[4];
  if (l == 0) wc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tot = wc[0] + wc[1] + wc[2] + wc[3];
    if (tot) atomicAdd(count, (unsigned long long)tot);
  }
}

static int grid_for(uint64_t work, int per_block) {
  uint64_t g = (work + per_block - 1) / per_block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace cc

extern "C" int cc_quorum_commit(const uint64_t* d_match, uint32_t replicas, uint64_t groups, const uint64_t* d_term_start,
                                const uint64_t* d_commit_in, uint64_t* d_commit_out, void* stream) {
  using namespace cc;
  if (!d_match || !d_term_start || !d_commit_in || !d_commit_out || replicas == 0 || replicas > 16) return CC_ERR_INVALID;
  if (groups == 0) return CC_OK;
  hipStream_t st = (hipStream_t)stream;
  const bool aligned = ((groups & 1) == 0) && (((uintptr_t)d_match | (uintptr_t)d_term_start | (uintptr_t)d_commit_in |
                                                (uintptr_t)d_commit_out) & 15) == 0;
  const int grid = grid_for(groups / 2 + 1, 256);
  if (aligned && replicas == 5)
    hipLaunchKernelGGL(k_quorum<5>, dim3(grid), dim3(256), 0, st, d_match, groups, d_term_start, d_commit_in, d_commit_out);
  else if (aligned && replicas == 3)
    hipLaunchKernelGGL(k_quorum<3>, dim3(grid), dim3(256), 0, st, d_match, groups, d_term_start, d_commit_in, d_commit_out);
  else if (aligned && replicas == 7)
    hipLaunchKernelGGL(k_quorum<7>, dim3(grid), dim3(256), 0, st, d_match, groups, d_term_start, d_commit_in, d_commit_out);
  else
    hipLaunchKernelGGL(k_quorum_generic, dim3(grid_for(groups, 256)), dim3(256), 0, st, d_match, replicas, groups,
                       d_term_start, d_commit_in, d_commit_out);
  return hipGetLastError() == hipSuccess ? CC_OK : CC_ERR_HIP;
}

extern "C" int cc_expire_sweep(const uint64_t* d_last, uint64_t sessions, uint64_t now, uint64_t timeout, uint64_t* d_bitmap,
                               uint64_t* d_count, void* stream) {
  using namespace cc;
  if (!d_last || !d_bitmap || !d_count || (((uintptr_t)d_last) & 15)) return CC_ERR_INVALID;
  if (sessions == 0) return CC_OK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_expire, dim3(grid_for((sessions + 127) / 128, 16)), dim3(256), 0, st, d_last, sessions, now,
                     (int64_t)timeout, d_bitmap, (unsigned long long*)d_count);
  return hipGetLastError() == hipSuccess ? CC_OK : CC_ERR_HIP;
}
