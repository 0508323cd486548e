// Probe: do LDS atomics with return (ds_add_rtn_u32) resolve lanes of ONE wave instruction that hit the same
// address in lane order on gfx950?  (If so, the returned value is a stable rank.)  Prints violations.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void probe(uint32_t keys_mod, uint32_t iters, uint32_t* viol, uint32_t seed) {
  __shared__ uint32_t tbl[1024];
  const uint32_t t = threadIdx.x, l = t & 63;
  uint32_t x = seed ^ (t * 2654435761u) ^ (blockIdx.x * 40503u);
  uint32_t bad = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    for (uint32_t k = t; k < 1024; k += blockDim.x) tbl[k] = 0;
    __syncthreads();
    x = x * 1664525u + 1013904223u;
    const uint32_t key = ((x >> 8) % keys_mod) + (t >> 6) * 64;  // per-wave private region (64 cells per wave)
    const uint32_t old = atomicAdd(&tbl[key], 1u);
    // check: among lanes of this wave with the same key, old must increase with lane id
    for (uint32_t j = 0; j < 64; ++j) {
      const uint32_t kj = __shfl(key, j, 64), oj = __shfl(old, j, 64);
      if (j < l && kj == key && oj >= old) bad++;
    }
    __syncthreads();
  }
  if (bad) atomicAdd(viol, bad);
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 4);
  for (uint32_t mod : {1u, 2u, 4u, 16u, 64u}) {
    for (int bs : {64, 256, 1024}) {
      hipMemset(d, 0, 4);
      hipLaunchKernelGGL(probe, dim3(1024), dim3(bs), 0, 0, mod, 64, d, 12345u + mod);
      uint32_t h = 0;
      hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
      printf("keys_mod=%u block=%d violations=%u\n", mod, bs, h);
    }
  }
  return 0;
}
