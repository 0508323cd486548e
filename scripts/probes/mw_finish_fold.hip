// Reproducer (compile-only): k_mw_finish with the size check folded in behind `if (msize)`, the shape of
// copycat_amd/csrc/map_wide.hip before commit bd13b1f split it into k_mw_size.  Question: on the msize == nullptr
// path of the clear / Delete case, does the ISA still define the register holding `slot` before dropped[slot] +=?
#include <hip/hip_runtime.h>
#include <cstdint>
enum { C_PRES = 0, C_USED, C_NULLS, C_MATCH, C_BN, C_BM, C_IN, C_IM, C_CAP, C_N };
constexpr uint32_t kErrMapSize = 32u;
#define OP_CONTAINSVALUE 61
#define OP_ISEMPTY 70
#define OP_SIZE 71
#define OP_CLEAR 72
#define OP_DELETE 1
__global__ void k_mw_finish_folded(uint32_t slot, uint32_t op, uint64_t row, const unsigned long long* __restrict__ ctl,
                                   uint32_t* __restrict__ peak_lo, unsigned long long* __restrict__ dropped,
                                   uint8_t* __restrict__ out_status, uint64_t* __restrict__ out_value,
                                   uint32_t* __restrict__ msize, uint32_t* __restrict__ err) {
  if (threadIdx.x != 0) return;
  const uint64_t pres = ctl[C_PRES];
  if (msize) {  // exact tracking: the tracked size must be what the table holds; clear / Delete empty the map
    if (msize[slot] != pres) atomicOr(err, kErrMapSize);
    if (op == OP_CLEAR || op == OP_DELETE) msize[slot] = 0;
  }
  uint32_t st = 0;
  uint64_t v = 0;
  switch (op) {
    case OP_SIZE:
      st = 2u << 4;
      v = (uint64_t)(int64_t)(int32_t)(uint32_t)pres;
      break;
    case OP_ISEMPTY:
      st = 3u << 4;
      v = pres == 0;
      break;
    case OP_CONTAINSVALUE: {
      const uint64_t nulls = ctl[C_NULLS], match = ctl[C_MATCH];
      bool npe;
      if (nulls == 0 || match == 0) npe = nulls != 0;
      else {
        const uint64_t bn = ctl[C_BN], bm = ctl[C_BM];
        npe = bn != bm ? bn < bm : ctl[C_IN] < ctl[C_IM];
      }
      st = npe ? 5u : (3u << 4);
      v = npe ? 0 : match != 0;
      break;
    }
    default:  // clear / Delete: every entry is dropped; the keys they held count toward the peak bound
      dropped[slot] += ctl[C_USED];
      break;
  }
  if (pres > peak_lo[slot]) peak_lo[slot] = (uint32_t)min(pres, (uint64_t)0xFFFFFFFFu);
  out_status[row] = (uint8_t)st;
  out_value[row] = v;
}
