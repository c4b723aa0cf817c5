// Host/device parameter block of the fused decode-layer skinny GEMMs (csrc/skinny.hip):
// residual add + RMSNorm split across the producing projection (RES) and the consuming one (NIN).
#pragma once
#include <cstdint>

namespace dla {

struct KsFuse {
  const uint16_t* res;     // RES: residual stream [M, N], row stride ldr
  int64_t ldr;
  float* ssq_out;        // RES: [16][gridDim.x] per-(row, workgroup) sums of squares
  const float* ssq_in;   // NIN: [16][nbp] partial sums of squares of x's rows (nbp <= 512)
  int nbp;
  float eps;             // NIN: RMSNorm epsilon (the norm weight is folded into W by the caller)
  const float* wscale;   // F8 weights: per weight-row dequantisation scale (y[:, n] *= wscale[n])
  int straight;          // 1: branch-free ring (ks_body): every slot refill issued unconditionally
};

}  // namespace dla
