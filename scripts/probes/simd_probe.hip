// Probe (argument: dynamic LDS bytes per workgroup): where do the waves of k_apply_coord-shaped workgroups land, and
// how many run on one CU at once?  516 workgroups of 256 threads; every wave records its hardware id (XCC, SE, CU,
// SIMD) and every workgroup its start / end clock, so co-residency is counted from overlapping intervals (a workgroup
// dispatched onto a CU after another finished is not co-resident with it).  The questions: do the wave-0s of the
// workgroups sharing a CU (k_apply_coord's walkers) share one SIMD, and at which LDS size do three stop fitting?
//   hipcc --offload-arch=gfx950 -O2 simd_probe.hip -o /tmp/simd_probe && /tmp/simd_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(256, 3) void k_probe(uint32_t* out, unsigned long long* times, uint32_t spin) {
  extern __shared__ uint32_t pad[];
  const uint32_t t = threadIdx.x, w = t >> 6;
  pad[t] = t;
  __syncthreads();
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if ((t & 63) == 0) {
    out[(blockIdx.x * 4 + w) * 2] = hw;
    out[(blockIdx.x * 4 + w) * 2 + 1] = xcc;
  }
  // keep the workgroup resident a while so the whole grid is co-resident
  uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < spin) __builtin_amdgcn_s_sleep(2);
  if (pad[(t + 1) & 255] == 0xFFFFFFFFu) out[0] = 0;
  if (t == 0) {
    times[2 * blockIdx.x] = t0;
    times[2 * blockIdx.x + 1] = wall_clock64();
  }
}

int main(int argc, char** argv) {
  const int G = 516;
  const unsigned lds = argc > 1 ? (unsigned)atoi(argv[1]) : 52800u;
  printf("LDS %u B per workgroup\n", lds);
  uint32_t* d;
  unsigned long long* dt;
  (void)hipMalloc(&d, G * 4 * 2 * 4);
  (void)hipMalloc(&dt, G * 2 * 8);
  hipLaunchKernelGGL(k_probe, dim3(G), dim3(256), lds, 0, d, dt, 20000u);
  if (hipDeviceSynchronize() != hipSuccess) { printf("fail\n"); return 1; }
  std::vector<uint32_t> h(G * 8);
  (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  std::vector<unsigned long long> tm(G * 2);
  (void)hipMemcpy(tm.data(), dt, tm.size() * 8, hipMemcpyDeviceToHost);
  // per CU: the SIMDs of each resident workgroup's waves
  std::map<std::tuple<int, int, int, int>, std::vector<std::pair<int, std::vector<int>>>> cu;
  int same_simd_all = 0;
  for (int b = 0; b < G; ++b) {
    std::vector<int> simds;
    int key_x = 0, key_se = 0, key_sh = 0, key_cu = 0;
    for (int w = 0; w < 4; ++w) {
      const uint32_t hw = h[(b * 4 + w) * 2], xcc = h[(b * 4 + w) * 2 + 1];
      simds.push_back((hw >> 4) & 3);
      key_x = xcc & 0xF;
      key_se = (hw >> 13) & 7;
      key_sh = (hw >> 12) & 1;
      key_cu = (hw >> 8) & 15;
    }
    cu[{key_x, key_se, key_sh, key_cu}].push_back({b, simds});
  }
  int hist[5] = {0, 0, 0, 0, 0};  // CUs by the number of distinct SIMDs their wave-0s use
  int n = 0;
  for (auto& kv : cu) {
    int mask = 0;
    for (auto& p : kv.second) mask |= 1 << p.second[0];
    hist[__builtin_popcount(mask)]++;
    if (n++ < 12) {
      printf("xcc %d se %d sh %d cu %2d:", std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first),
             std::get<3>(kv.first));
      for (auto& p : kv.second) printf("  wg %3d simds %d%d%d%d", p.first, p.second[0], p.second[1], p.second[2], p.second[3]);
      printf("\n");
    }
    if (kv.second.size() >= 2) {
      bool all = true;
      for (auto& p : kv.second) all &= p.second[0] == kv.second[0].second[0];
      same_simd_all += all;
    }
  }
  // co-resident workgroups per CU: the most intervals [start, end) of one CU that overlap at one instant
  int max_per_cu = 0, late = 0;
  unsigned long long first = ~0ull;
  for (int b = 0; b < G; ++b) first = tm[2 * b] < first ? tm[2 * b] : first;
  for (int b = 0; b < G; ++b) late += tm[2 * b] > first + 10000;  // started > 100 us after the first
  for (auto& kv : cu) {
    for (auto& p : kv.second) {
      int c = 0;
      for (auto& q : kv.second) c += tm[2 * q.first] <= tm[2 * p.first] && tm[2 * p.first] < tm[2 * q.first + 1];
      max_per_cu = c > max_per_cu ? c : max_per_cu;
    }
  }
  printf("max co-resident workgroups on one CU %d; workgroups starting > 100 us late %d\n", max_per_cu, late);
  printf("CUs used %zu; CUs by distinct wave-0 SIMDs: 1:%d 2:%d 3:%d 4:%d; CUs with >=2 WGs all wave-0 on one SIMD: %d\n",
         cu.size(), hist[1], hist[2], hist[3], hist[4], same_simd_all);
  return 0;
}
