// Probe: the LDS bank-conflict share of ranking by random slots, the way k_part_v4 / k_apply_value_v3 rank records
// (one LDS atomic with return per record on a wave's own row of counters), against conflict-free controls.
// Each kernel runs 1,024-thread workgroups, one per CU; every wave does kIters rounds of one atomicAdd per lane on
// its own counter row.  Kernels (one rocprofv3 --pmc pass reads SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE per kernel):
//   k_rand_u16   random slot in [0, 256), packed u16 pairs (128 dwords per row: the c2 partition / apply layout)
//   k_rand_u32   random slot in [0, 256), one u32 counter per slot (256 dwords per row)
//   k_rand_pad   random slot, u32 counters with a 65-dword row pitch per 64 slots (padding)
//   k_seq_u32    slot = lane (64 consecutive dwords: conflict-free control)
//   hipcc --offload-arch=gfx950 -O3 lds_random_conflicts.hip -o lds_random_conflicts
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kT = 1024, kW = kT / 64, kIters = 4096;

__device__ inline uint32_t mix(uint32_t x) {  // a cheap hash: random-looking slots, different per lane and round
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__global__ __launch_bounds__(kT) void k_rand_u16(uint32_t* out) {
  __shared__ uint32_t wc[kW][128];
  const uint32_t t = threadIdx.x, w = t >> 6;
  for (uint32_t k = t; k < kW * 128; k += kT) (&wc[0][0])[k] = 0;
  __syncthreads();
  uint32_t acc = 0;
  for (int i = 0; i < kIters; ++i) {
    const uint32_t s = mix(blockIdx.x * 0x9E3779B9u + i * kT + t) & 255u, sh = 16 * (s & 1);
    acc += (atomicAdd(&wc[w][s >> 1], 1u << sh) >> sh) & 0xFFFF;
  }
  if (acc == 0xFFFFFFFFu) out[0] = acc;
}

__global__ __launch_bounds__(kT) void k_rand_u32(uint32_t* out) {
  __shared__ uint32_t wc[kW][256];
  const uint32_t t = threadIdx.x, w = t >> 6;
  for (uint32_t k = t; k < kW * 256; k += kT) (&wc[0][0])[k] = 0;
  __syncthreads();
  uint32_t acc = 0;
  for (int i = 0; i < kIters; ++i) acc += atomicAdd(&wc[w][mix(blockIdx.x * 0x9E3779B9u + i * kT + t) & 255u], 1u);
  if (acc == 0xFFFFFFFFu) out[0] = acc;
}

__global__ __launch_bounds__(kT) void k_rand_pad(uint32_t* out) {
  __shared__ uint32_t wc[kW][4 * 65];
  const uint32_t t = threadIdx.x, w = t >> 6;
  for (uint32_t k = t; k < kW * 4 * 65; k += kT) (&wc[0][0])[k] = 0;
  __syncthreads();
  uint32_t acc = 0;
  for (int i = 0; i < kIters; ++i) {
    const uint32_t s = mix(blockIdx.x * 0x9E3779B9u + i * kT + t) & 255u;
    acc += atomicAdd(&wc[w][(s >> 6) * 65 + (s & 63)], 1u);
  }
  if (acc == 0xFFFFFFFFu) out[0] = acc;
}

__global__ __launch_bounds__(kT) void k_seq_u32(uint32_t* out) {
  __shared__ uint32_t wc[kW][256];
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  for (uint32_t k = t; k < kW * 256; k += kT) (&wc[0][0])[k] = 0;
  __syncthreads();
  uint32_t acc = 0;
  for (int i = 0; i < kIters; ++i) acc += atomicAdd(&wc[w][((i & 3) << 6) + l], 1u);
  if (acc == 0xFFFFFFFFu) out[0] = acc;
}

int main() {
  uint32_t* d;
  (void)hipMalloc(&d, 16);
  const dim3 g(256), b(kT);
  hipLaunchKernelGGL(k_rand_u16, g, b, 0, 0, d);
  hipLaunchKernelGGL(k_rand_u32, g, b, 0, 0, d);
  hipLaunchKernelGGL(k_rand_pad, g, b, 0, 0, d);
  hipLaunchKernelGGL(k_seq_u32, g, b, 0, 0, d);
  const hipError_t x = hipDeviceSynchronize();
  printf("%s\n", x == hipSuccess ? "ok" : hipGetErrorString(x));
  return x == hipSuccess ? 0 : 1;
}
