// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of this package.
//
// Conventions used by every kernel file:
//   * bf16 tensors travel as raw 16-bit words (`bf16_t` = uint16_t); math is fp32.
//   * wave = 64 lanes (never 32); block sizes are multiples of 64.
//   * global loads/stores of bf16 are vectorized to 16 B per lane (8 x bf16).
//   * every launcher takes an explicit hipStream_t (the caller's current torch stream),
//     performs no allocation and no host synchronisation (graph-capture safe).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dla {

using bf16_t = uint16_t;

// 8 x bf16 = 16 bytes: the native global-load width per lane.
typedef uint16_t bf16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
// MFMA operand fragments (bf16 payload in short lanes).
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 hbf16x2 __attribute__((ext_vector_type(2)));

// fp32 -> bf16 round-to-nearest-even, NaN preserving: a plain cast lowers to the gfx950
// hardware v_cvt_pk_bf16_f32 (the integer-rounding form costs ~5 VALU ops per element).
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, static_cast<__bf16>(f));
}

// Pack two fp32 into one dword of two bf16 (lo in bits 0..15): ONE v_cvt_pk_bf16_f32.
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, hbf16x2));
}

// 8 fp32 -> 8 bf16 (16 bytes) with 4 packed conversions.
__device__ __forceinline__ bf16x8 pack_bf16x8(const float* v) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 r = {pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
  return __builtin_bit_cast(bf16x8, r);
}

// out[j] = column j of the 8 x 8 bf16 block held as 8 row vectors v[0..7] (32 v_perm_b32, no LDS):
// the register transpose behind the kernels that write a transposed second output
// (elementwise.hip SwiGLU, logprob.hip log-prob backward, transpose.hip)
__device__ __forceinline__ void tr8_bf16(const bf16x8 (&v)[8], bf16x8 (&out)[8]) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t sel = (j & 1) ? 0x07060302u : 0x05040100u;
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      o[k] = __builtin_amdgcn_perm(__builtin_bit_cast(u32x4, v[2 * k + 1])[j >> 1],
                                   __builtin_bit_cast(u32x4, v[2 * k])[j >> 1], sel);
    out[j] = __builtin_bit_cast(bf16x8, o);
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `scratch` holds NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += scratch[i];
  return r;
}

template <int NT>
__device__ __forceinline__ float block_max(float v, float* scratch) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, scratch[i]);
  return r;
}

__device__ __forceinline__ bf16x8 load_bf16x8(const bf16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}
__device__ __forceinline__ void store_bf16x8(bf16_t* p, bf16x8 v) {
  *reinterpret_cast<bf16x8*>(p) = v;
}

__device__ __forceinline__ float fast_exp(float x) { return __expf(x); }
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
// log(sigmoid(x)) computed stably.
__device__ __forceinline__ float log_sigmoid(float x) {
  return fminf(x, 0.f) - log1pf(__expf(-fabsf(x)));
}

// XCD-aware bijective block remap (8 XCDs, blocks dealt round-robin): consecutive logical tiles
// land on the same XCD so they share its L2. Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int q = nblocks / 8, r = nblocks % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// e4m3 -> bf16, 8 values from two dwords (exact: every e4m3 value is a bf16 value); the per-row
// dequantisation scale is applied to the fp32 sum in the epilogue
__device__ __forceinline__ s16x8 f8x8_to_bf16(uint32_t w0, uint32_t w1) {
  typedef short s16x2v __attribute__((ext_vector_type(2)));
  const s16x2v a = __builtin_bit_cast(s16x2v, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w0, 1.0f, false));
  const s16x2v b = __builtin_bit_cast(s16x2v, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w0, 1.0f, true));
  const s16x2v c = __builtin_bit_cast(s16x2v, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w1, 1.0f, false));
  const s16x2v d = __builtin_bit_cast(s16x2v, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w1, 1.0f, true));
  return s16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}


}  // namespace dla
