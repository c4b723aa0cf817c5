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

// Register transpose for R, C multiples of 8 (every activation / weight shape of the models): each
// lane loads an 8 x 8 bf16 block as 8 16-byte row segments, transposes it in registers with
// v_perm_b32 (32 byte-selects, no LDS round trip) and stores 8 16-byte segments. A wave covers a
// 64 x 64 tile; for each of the 8 loads / stores the 8 lanes of a row block touch one full 128-byte
// line. 128 B in flight per lane (4x the LDS kernel) keeps HBM busy.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void transpose_bf16_reg_kernel(const bf16_t* __restrict__ in,
                                                                  int64_t R, int64_t C,
                                                                  int64_t ld_in,
                                                                  bf16_t* __restrict__ out,
                                                                  int64_t ld_out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.y * 64 + (lane >> 3) * 8;
  const int64_t c = (int64_t)blockIdx.x * 256 + w * 64 + (lane & 7) * 8;
  if (r >= R || c >= C) return;  // R, C multiples of 8: blocks are all-in or all-out
  u32x4_t v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(in + (r + i) * ld_in + c));
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t sel = (j & 1) ? 0x07060302u : 0x05040100u;  // high / low bf16 of each dword
    u32x4_t o;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = __builtin_amdgcn_perm(v[2 * k + 1][j >> 1], v[2 * k][j >> 1], sel);
    *reinterpret_cast<u32x4_t*>(out + (c + j) * ld_out + r) = o;
  }
}

void launch_transpose_bf16(const bf16_t* in, int64_t R, int64_t C, int64_t ld_in, bf16_t* out,
                           int64_t ld_out, hipStream_t st) {
  if (R == 0 || C == 0) return;
  if (R % 8 == 0 && C % 8 == 0) {
    dim3 grid((unsigned)((C + 255) / 256), (unsigned)((R + 63) / 64));
    transpose_bf16_reg_kernel<<<grid, 256, 0, st>>>(in, R, C, ld_in, out, ld_out);
    return;
  }
  dim3 grid((unsigned)((C + kT - 1) / kT), (unsigned)((R + kT - 1) / kT));
  transpose_bf16_kernel<<<grid, 256, 0, st>>>(in, R, C, ld_in, out, ld_out);
}

}  // namespace dla
