// Elementwise activation kernels: fused SwiGLU and tanh-GELU, forward + backward.
//
// Reference: HF LlamaMLP `down(silu(gate(x)) * up(x))` and GPT-2/phi-2 `gelu_new`, reached via
// every model forward in src/training/train_*.py. Eager PyTorch runs silu, mul (and their
// backward) as 3-5 separate HBM passes; here each direction is ONE pass, 16 B per lane.
//
// SwiGLU input is the fused gate_up GEMM output gu[N, 2F] (gate = columns [0,F), up = [F,2F)).
#include "common.h"

#include <cstdlib>

namespace dla {

__device__ __forceinline__ float silu_f(float g) { return g * sigmoidf_(g); }

// d/dg and d/du of silu(g) * u for 8 lanes; shared by both backward kernels so they agree bitwise
__device__ __forceinline__ void swiglu_grad8(const bf16x8& g, const bf16x8& u, const bf16x8& d,
                                             bf16x8& dg, bf16x8& du) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float gf = bf2f(g[j]), uf = bf2f(u[j]), df = bf2f(d[j]);
    const float sg = sigmoidf_(gf);
    du[j] = f2bf(df * (gf * sg));
    dg[j] = f2bf(df * uf * sg * (1.f + gf * (1.f - sg)));
  }
}

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu,
                                                          bf16_t* __restrict__ out, int64_t rows,
                                                          int F) {
  const int fv = F >> 3;
  const int64_t total = rows * fv;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t r = i / fv;
    const int c = static_cast<int>(i - r * fv) * 8;
    const bf16_t* row = gu + r * 2 * F;
    bf16x8 g = load_bf16x8(row + c), u = load_bf16x8(row + F + c), o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(silu_f(bf2f(g[j])) * bf2f(u[j]));
    store_bf16x8(out + r * F + c, o);
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ gu,
                                                          const bf16_t* __restrict__ dout,
                                                          bf16_t* __restrict__ dgu, int64_t rows,
                                                          int F) {
  const int fv = F >> 3;
  const int64_t total = rows * fv;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t r = i / fv;
    const int c = static_cast<int>(i - r * fv) * 8;
    const bf16_t* row = gu + r * 2 * F;
    bf16x8 g = load_bf16x8(row + c), u = load_bf16x8(row + F + c);
    bf16x8 d = load_bf16x8(dout + r * F + c), dg, du;
    swiglu_grad8(g, u, d, dg, du);
    store_bf16x8(dgu + r * 2 * F + c, dg);
    store_bf16x8(dgu + r * 2 * F + F + c, du);
  }
}

// ---------------------------------------------------------------------------------------------
// SwiGLU with a transposed second output, for the fused MLP autograd node (ops.swiglu_mlp).
// The weight-gradient GEMMs run in the TN layout on transposed activations (ops/linear.py), so
// the MLP backward needs m^T (down_proj) and dgu^T (gate|up proj): producing them here, from the
// values already in registers, costs one extra write instead of a separate transpose pass
// (read + write). 64 x 64 tiles: 256 threads, each owns 2 rows x 8 columns; the transposed copy
// goes through a padded LDS tile (16-byte row stores on both sides).
constexpr int kTT = 64, kTPad = 8;

__global__ __launch_bounds__(256) void swiglu_fwd_t_kernel(const bf16_t* __restrict__ gu,
                                                            bf16_t* __restrict__ out,
                                                            bf16_t* __restrict__ outT,
                                                            int64_t rows, int F) {
  __shared__ bf16_t tile[kTT][kTT + kTPad];
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * kTT;
  const int c0 = blockIdx.x * kTT;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int v = t + 256 * k;
    const int rr = v >> 3, cv = (v & 7) * 8;
    const int64_t r = r0 + rr;
    bf16x8 o = {};
    if (r < rows) {  // F % 64 == 0 is checked on the host
      const bf16_t* row = gu + r * 2 * F;
      const bf16x8 g = load_bf16x8(row + c0 + cv), u = load_bf16x8(row + F + c0 + cv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(silu_f(bf2f(g[j])) * bf2f(u[j]));
      store_bf16x8(out + r * F + c0 + cv, o);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[rr][cv + j] = o[j];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // outT[c0 + cc][r0 + rv .. +8]
    const int v = t + 256 * k;
    const int cc = v >> 3, rv = (v & 7) * 8;
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = tile[rv + j][cc];
    const int64_t oc = r0 + rv;
    bf16_t* dst = outT + static_cast<int64_t>(c0 + cc) * rows + oc;
    if (oc + 8 <= rows) {
      store_bf16x8(dst, o);
    } else {
      for (int j = 0; j < 8; ++j)
        if (oc + j < rows) dst[j] = o[j];
    }
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_t_kernel(const bf16_t* __restrict__ gu,
                                                            const bf16_t* __restrict__ dout,
                                                            bf16_t* __restrict__ dgu,
                                                            bf16_t* __restrict__ dguT,
                                                            int64_t rows, int F) {
  __shared__ bf16_t tg[kTT][kTT + kTPad];
  __shared__ bf16_t tu[kTT][kTT + kTPad];
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * kTT;
  const int c0 = blockIdx.x * kTT;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int v = t + 256 * k;
    const int rr = v >> 3, cv = (v & 7) * 8;
    const int64_t r = r0 + rr;
    bf16x8 dg = {}, du = {};
    if (r < rows) {
      const bf16_t* row = gu + r * 2 * F;
      const bf16x8 g = load_bf16x8(row + c0 + cv), u = load_bf16x8(row + F + c0 + cv);
      const bf16x8 d = load_bf16x8(dout + r * F + c0 + cv);
      swiglu_grad8(g, u, d, dg, du);
      store_bf16x8(dgu + r * 2 * F + c0 + cv, dg);
      store_bf16x8(dgu + r * 2 * F + F + c0 + cv, du);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      tg[rr][cv + j] = dg[j];
      tu[rr][cv + j] = du[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // dguT[c0 + cc] (gate rows) and dguT[F + c0 + cc] (up rows)
    const int v = t + 256 * k;
    const int cc = v >> 3, rv = (v & 7) * 8;
    bf16x8 a, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = tg[rv + j][cc];
      b[j] = tu[rv + j][cc];
    }
    const int64_t oc = r0 + rv;
    bf16_t* da = dguT + static_cast<int64_t>(c0 + cc) * rows + oc;
    bf16_t* db = dguT + static_cast<int64_t>(F + c0 + cc) * rows + oc;
    if (oc + 8 <= rows) {
      store_bf16x8(da, a);
      store_bf16x8(db, b);
    } else {
      for (int j = 0; j < 8; ++j)
        if (oc + j < rows) {
          da[j] = a[j];
          db[j] = b[j];
        }
    }
  }
}

// Register-transpose forms (csrc/transpose.hip transpose_bf16_reg_kernel): each lane owns an
// 8 x 8 block, loads its 8 row segments of every operand (16 B each; the 8 lanes of a row block
// cover one 128-byte line), computes the SAME per-element math as the LDS-tiled kernels above
// (bitwise equal), stores the row-major outputs as row segments and the transposed outputs after
// a v_perm_b32 8 x 8 transpose as 16-byte column segments. No LDS round trip and 256-384 B of
// loads in flight per lane. A wave covers 64 rows x 64 columns; grid (ceil(F / 256), rows / 64);
// rows % 8 == 0 and F % 8 == 0 (checked by the launcher; other shapes take the LDS kernels).
__global__ __launch_bounds__(256) void swiglu_fwd_t_reg_kernel(const bf16_t* __restrict__ gu,
                                                                bf16_t* __restrict__ out,
                                                                bf16_t* __restrict__ outT,
                                                                int64_t rows, int F) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r = static_cast<int64_t>(blockIdx.y) * 64 + (lane >> 3) * 8;
  const int c = blockIdx.x * 256 + w * 64 + (lane & 7) * 8;
  if (r >= rows || c >= F) return;
  bf16x8 g[8], u[8], o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bf16_t* row = gu + (r + i) * 2 * F;
    g[i] = load_bf16x8(row + c);
    u[i] = load_bf16x8(row + F + c);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) o[i][j] = f2bf(silu_f(bf2f(g[i][j])) * bf2f(u[i][j]));
    store_bf16x8(out + (r + i) * F + c, o[i]);
  }
  bf16x8 t[8];
  tr8_bf16(o, t);
#pragma unroll
  for (int j = 0; j < 8; ++j) store_bf16x8(outT + static_cast<int64_t>(c + j) * rows + r, t[j]);
}

__global__ __launch_bounds__(256) void swiglu_bwd_t_reg_kernel(const bf16_t* __restrict__ gu,
                                                                const bf16_t* __restrict__ dout,
                                                                bf16_t* __restrict__ dgu,
                                                                bf16_t* __restrict__ dguT,
                                                                int64_t rows, int F) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r = static_cast<int64_t>(blockIdx.y) * 64 + (lane >> 3) * 8;
  const int c = blockIdx.x * 256 + w * 64 + (lane & 7) * 8;
  if (r >= rows || c >= F) return;
  bf16x8 dg[8], du[8];
  {
    bf16x8 g[8], u[8], d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bf16_t* row = gu + (r + i) * 2 * F;
      g[i] = load_bf16x8(row + c);
      u[i] = load_bf16x8(row + F + c);
      d[i] = load_bf16x8(dout + (r + i) * F + c);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      swiglu_grad8(g[i], u[i], d[i], dg[i], du[i]);
      store_bf16x8(dgu + (r + i) * 2 * F + c, dg[i]);
      store_bf16x8(dgu + (r + i) * 2 * F + F + c, du[i]);
    }
  }
  bf16x8 t[8];
  tr8_bf16(dg, t);
#pragma unroll
  for (int j = 0; j < 8; ++j) store_bf16x8(dguT + static_cast<int64_t>(c + j) * rows + r, t[j]);
  tr8_bf16(du, t);
#pragma unroll
  for (int j = 0; j < 8; ++j) store_bf16x8(dguT + static_cast<int64_t>(F + c + j) * rows + r, t[j]);
}

// The register-transpose form wherever its 8 x 8 blocks tile the shape (207 -> 181.5 us forward,
// 343 -> 305 us backward at the DPO shape, bitwise equal); the LDS-tiled kernels serve the rest
static bool swiglu_t_reg(int64_t rows, int F) { return rows % 8 == 0 && F % 8 == 0; }

// gelu_new (tanh approximation), as used by GPT-2 and phi-2.
__device__ __forceinline__ float gelu_tanh(float x, float* dgdx) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float inner = k0 * (x + k1 * x * x * x);
  const float t = tanhf(inner);
  if (dgdx) *dgdx = 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
  return 0.5f * x * (1.f + t);
}

__global__ __launch_bounds__(256) void gelu_fwd_kernel(const bf16_t* __restrict__ x,
                                                        bf16_t* __restrict__ y, int64_t nvec) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < nvec; i += static_cast<int64_t>(gridDim.x) * 256) {
    bf16x8 a = load_bf16x8(x + i * 8), o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(gelu_tanh(bf2f(a[j]), nullptr));
    store_bf16x8(y + i * 8, o);
  }
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const bf16_t* __restrict__ x,
                                                        const bf16_t* __restrict__ dy,
                                                        bf16_t* __restrict__ dx, int64_t nvec) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < nvec; i += static_cast<int64_t>(gridDim.x) * 256) {
    bf16x8 a = load_bf16x8(x + i * 8), d = load_bf16x8(dy + i * 8), o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float der;
      gelu_tanh(bf2f(a[j]), &der);
      o[j] = f2bf(bf2f(d[j]) * der);
    }
    store_bf16x8(dx + i * 8, o);
  }
}

static inline unsigned grid_for(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g > 256 * 8) g = 256 * 8;  // 8 blocks per CU, grid-stride the rest
  return static_cast<unsigned>(g < 1 ? 1 : g);
}

void launch_swiglu_fwd(const bf16_t* gu, bf16_t* out, int64_t rows, int F, hipStream_t st) {
  swiglu_fwd_kernel<<<grid_for(rows * (F / 8)), 256, 0, st>>>(gu, out, rows, F);
}
void launch_swiglu_bwd(const bf16_t* gu, const bf16_t* dout, bf16_t* dgu, int64_t rows, int F,
                       hipStream_t st) {
  swiglu_bwd_kernel<<<grid_for(rows * (F / 8)), 256, 0, st>>>(gu, dout, dgu, rows, F);
}
void launch_swiglu_fwd_t(const bf16_t* gu, bf16_t* out, bf16_t* outT, int64_t rows, int F,
                         hipStream_t st) {
  if (rows == 0) return;
  if (swiglu_t_reg(rows, F)) {
    const dim3 g((F + 255) / 256, static_cast<unsigned>((rows + 63) / 64));
    swiglu_fwd_t_reg_kernel<<<g, 256, 0, st>>>(gu, out, outT, rows, F);
    return;
  }
  const dim3 grid(F / kTT, static_cast<unsigned>((rows + kTT - 1) / kTT));
  swiglu_fwd_t_kernel<<<grid, 256, 0, st>>>(gu, out, outT, rows, F);
}
void launch_swiglu_bwd_t(const bf16_t* gu, const bf16_t* dout, bf16_t* dgu, bf16_t* dguT,
                         int64_t rows, int F, hipStream_t st) {
  if (rows == 0) return;
  if (swiglu_t_reg(rows, F)) {
    const dim3 g((F + 255) / 256, static_cast<unsigned>((rows + 63) / 64));
    swiglu_bwd_t_reg_kernel<<<g, 256, 0, st>>>(gu, dout, dgu, dguT, rows, F);
    return;
  }
  const dim3 grid(F / kTT, static_cast<unsigned>((rows + kTT - 1) / kTT));
  swiglu_bwd_t_kernel<<<grid, 256, 0, st>>>(gu, dout, dgu, dguT, rows, F);
}
void launch_gelu_fwd(const bf16_t* x, bf16_t* y, int64_t n, hipStream_t st) {
  gelu_fwd_kernel<<<grid_for(n / 8), 256, 0, st>>>(x, y, n / 8);
}
void launch_gelu_bwd(const bf16_t* x, const bf16_t* dy, bf16_t* dx, int64_t n, hipStream_t st) {
  gelu_bwd_kernel<<<grid_for(n / 8), 256, 0, st>>>(x, dy, dx, n / 8);
}

}  // namespace dla
