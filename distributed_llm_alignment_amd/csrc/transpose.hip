// bf16 matrix transpose out[c, r] = in[r, c] (LDS-tiled, 16-byte global accesses).
//
// Used to keep a transposed copy W^T of every trainable weight so the backward input-gradient
// GEMM dX = dY W runs as dX = dY (W^T)^T — the TN layout hipBLASLt runs at the forward GEMMs'
// rate on gfx950 (1.43-1.52 vs 1.22-1.36 PF/s measured for Llama-3-8B shapes,
// tools/gemm_layout_probe.py). Refreshed once per optimizer step: 2 x 16 GB of HBM traffic for
// an 8B model, a few ms at ~5 TB/s.
//
// Tile 64 x 64: 256 threads; each thread loads 2 x 8 bf16 (two 16-byte row segments) into LDS
// (row pitch 64 + 8 elements: the +16 B skew spreads the column reads over the banks), then
// writes 2 x 8 transposed elements as 16-byte stores.
#include "common.h"

namespace dla {

constexpr int kT = 64, kPad = 8;

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ in,
                                                              int64_t R, int64_t C, int64_t ld_in,
                                                              bf16_t* __restrict__ out,
                                                              int64_t ld_out) {
  __shared__ bf16_t tile[kT][kT + kPad];
  const int64_t r0 = (int64_t)blockIdx.y * kT, c0 = (int64_t)blockIdx.x * kT;
  const int t = threadIdx.x;
  // load: 64 rows x 8 vectors of 8 -> 512 vectors, 2 per thread
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int v = t + k * 256;
    const int rr = v >> 3, cv = (v & 7) * 8;
    const int64_t r = r0 + rr, c = c0 + cv;
    if (r < R && c + 8 <= C) {
      const bf16x8 a = load_bf16x8(in + r * ld_in + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) tile[rr][cv + j] = a[j];
    } else if (r < R) {
      for (int j = 0; j < 8; ++j)
        if (c + j < C) tile[rr][cv + j] = in[r * ld_in + c + j];
    }
  }
  __syncthreads();
  // store: out row = c0 + cc, columns r0 + rv .. +8
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int v = t + k * 256;
    const int cc = v >> 3, rv = (v & 7) * 8;
    const int64_t orow = c0 + cc, ocol = r0 + rv;
    if (orow >= C) continue;
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = tile[rv + j][cc];
    if (ocol + 8 <= R) {
      store_bf16x8(out + orow * ld_out + ocol, o);
    } else {
      for (int j = 0; j < 8; ++j)
        if (ocol + j < R) out[orow * ld_out + ocol + j] = o[j];
    }
  }
}

void launch_transpose_bf16(const bf16_t* in, int64_t R, int64_t C, int64_t ld_in, bf16_t* out,
                           int64_t ld_out, hipStream_t st) {
  if (R == 0 || C == 0) return;
  dim3 grid((unsigned)((C + kT - 1) / kT), (unsigned)((R + kT - 1) / kT));
  transpose_bf16_kernel<<<grid, 256, 0, st>>>(in, R, C, ld_in, out, ld_out);
}

}  // namespace dla
