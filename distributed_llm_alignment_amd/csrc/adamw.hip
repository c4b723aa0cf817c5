// Fused AdamW over flat parameter shards + global grad-norm / clip.
//
// Reference: torch.optim.AdamW (src/training/train_dpo.py:73-77, train_sft.py:89-94, ...) and
// accelerator.clip_grad_norm_ (src/training/utils.py:121-123). Eager torch runs these as
// per-tensor foreach launches plus a host-visible norm. Here parameters, grads and states live
// in ONE flat buffer each (or one contiguous shard of it under ZeRO), so the whole optimizer is
// one streaming pass: 16 B loads per lane, fp32 master + fp32 moments, bf16 params written back.
// The clip coefficient is produced and consumed ON DEVICE (no .item() sync per step).
//
// Update (torch AdamW semantics, decoupled weight decay):
//   p <- p * (1 - lr*wd)
//   m <- b1*m + (1-b1)*g ; v <- b2*v + (1-b2)*g^2
//   p <- p - (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
#include "common.h"

namespace dla {

template <bool GRAD_BF16, bool HAS_MASTER>
__global__ __launch_bounds__(256) void adamw_kernel(bf16_t* __restrict__ p, float* __restrict__ master,
                                                     const void* __restrict__ gptr,
                                                     float* __restrict__ m, float* __restrict__ v,
                                                     int64_t nvec, float lr, float b1, float b2,
                                                     float eps, float wd, float step_size,
                                                     float inv_sqrt_bc2,
                                                     const float* __restrict__ clip,
                                                     float grad_scale) {
  const float gs = grad_scale * (clip ? clip[0] : 1.f);
  const float decay = 1.f - lr * wd;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < nvec; i += static_cast<int64_t>(gridDim.x) * 256) {
    float g[8], w[8];
    if constexpr (GRAD_BF16) {
      bf16x8 gv = load_bf16x8(reinterpret_cast<const bf16_t*>(gptr) + i * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = bf2f(gv[j]) * gs;
    } else {
      const f32x4* gp = reinterpret_cast<const f32x4*>(gptr) + i * 2;
      f32x4 a = gp[0], b = gp[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        g[j] = a[j] * gs;
        g[4 + j] = b[j] * gs;
      }
    }
    if constexpr (HAS_MASTER) {
      f32x4 a = reinterpret_cast<f32x4*>(master)[i * 2], b = reinterpret_cast<f32x4*>(master)[i * 2 + 1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        w[j] = a[j];
        w[4 + j] = b[j];
      }
    } else {
      bf16x8 pv = load_bf16x8(p + i * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = bf2f(pv[j]);
    }
    f32x4 m0 = reinterpret_cast<f32x4*>(m)[i * 2], m1 = reinterpret_cast<f32x4*>(m)[i * 2 + 1];
    f32x4 v0 = reinterpret_cast<f32x4*>(v)[i * 2], v1 = reinterpret_cast<f32x4*>(v)[i * 2 + 1];
    float mm[8] = {m0[0], m0[1], m0[2], m0[3], m1[0], m1[1], m1[2], m1[3]};
    float vv[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    bf16x8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      w[j] *= decay;
      mm[j] = b1 * mm[j] + (1.f - b1) * g[j];
      vv[j] = b2 * vv[j] + (1.f - b2) * g[j] * g[j];
      w[j] -= step_size * mm[j] / (sqrtf(vv[j]) * inv_sqrt_bc2 + eps);
      out[j] = f2bf(w[j]);
    }
    reinterpret_cast<f32x4*>(m)[i * 2] = f32x4{mm[0], mm[1], mm[2], mm[3]};
    reinterpret_cast<f32x4*>(m)[i * 2 + 1] = f32x4{mm[4], mm[5], mm[6], mm[7]};
    reinterpret_cast<f32x4*>(v)[i * 2] = f32x4{vv[0], vv[1], vv[2], vv[3]};
    reinterpret_cast<f32x4*>(v)[i * 2 + 1] = f32x4{vv[4], vv[5], vv[6], vv[7]};
    if constexpr (HAS_MASTER) {
      reinterpret_cast<f32x4*>(master)[i * 2] = f32x4{w[0], w[1], w[2], w[3]};
      reinterpret_cast<f32x4*>(master)[i * 2 + 1] = f32x4{w[4], w[5], w[6], w[7]};
    }
    if (p) store_bf16x8(p + i * 8, out);
  }
}

// Stage 1: per-block partial sums of g^2 (fixed grid -> deterministic).
template <bool GRAD_BF16>
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const void* __restrict__ gptr,
                                                             int64_t nvec,
                                                             float* __restrict__ partial) {
  __shared__ float scratch[4];
  float acc = 0.f;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < nvec; i += static_cast<int64_t>(gridDim.x) * 256) {
    if constexpr (GRAD_BF16) {
      bf16x8 gv = load_bf16x8(reinterpret_cast<const bf16_t*>(gptr) + i * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = bf2f(gv[j]);
        acc += x * x;
      }
    } else {
      const f32x4* gp = reinterpret_cast<const f32x4*>(gptr) + i * 2;
      f32x4 a = gp[0], b = gp[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc += a[j] * a[j] + b[j] * b[j];
    }
  }
  acc = block_sum<256>(acc, scratch);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

// Stage 2: out[0] (+)= sum(partial) in fixed order.
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ partial, int n,
                                                            float* __restrict__ out, int accumulate) {
  __shared__ float scratch[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) acc += partial[i];
  acc = block_sum<256>(acc, scratch);
  if (threadIdx.x == 0) out[0] = accumulate ? out[0] + acc : acc;
}

// norm = sqrt(sumsq); coef = min(1, max_norm / (norm + 1e-6))  (torch clip_grad_norm_)
__global__ void clip_coef_kernel(const float* __restrict__ sumsq, float max_norm,
                                 float* __restrict__ norm_out, float* __restrict__ coef_out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const float n = sqrtf(sumsq[0]);
    norm_out[0] = n;
    coef_out[0] = max_norm > 0.f ? fminf(1.f, max_norm / (n + 1e-6f)) : 1.f;
  }
}

static inline unsigned stream_grid(int64_t nvec) {
  int64_t g = (nvec + 255) / 256;
  if (g > 256 * 4) g = 256 * 4;
  return static_cast<unsigned>(g < 1 ? 1 : g);
}

int sumsq_grid(int64_t n) { return static_cast<int>(stream_grid(n / 8)); }

void launch_adamw(bf16_t* p, float* master, const void* g, bool grad_bf16, float* m, float* v,
                  int64_t n, float lr, float b1, float b2, float eps, float wd, int step,
                  const float* clip, float grad_scale, hipStream_t st) {
  if (n == 0) return;
  const float bc1 = 1.f - powf(b1, static_cast<float>(step));
  const float bc2 = 1.f - powf(b2, static_cast<float>(step));
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = 1.f / sqrtf(bc2);
  const int64_t nvec = n / 8;
  const unsigned grid = stream_grid(nvec);
#define DLA_ADAMW(GB, HM)                                                                      \
  adamw_kernel<GB, HM><<<grid, 256, 0, st>>>(p, master, g, m, v, nvec, lr, b1, b2, eps, wd,   \
                                             step_size, inv_sqrt_bc2, clip, grad_scale)
  if (grad_bf16) {
    if (master) DLA_ADAMW(true, true); else DLA_ADAMW(true, false);
  } else {
    if (master) DLA_ADAMW(false, true); else DLA_ADAMW(false, false);
  }
#undef DLA_ADAMW
}

void launch_grad_sumsq(const void* g, bool grad_bf16, int64_t n, float* partial, float* out,
                       bool accumulate, hipStream_t st) {
  const unsigned grid = stream_grid(n / 8);
  if (grad_bf16) sumsq_partial_kernel<true><<<grid, 256, 0, st>>>(g, n / 8, partial);
  else sumsq_partial_kernel<false><<<grid, 256, 0, st>>>(g, n / 8, partial);
  sum_partials_kernel<<<1, 256, 0, st>>>(partial, static_cast<int>(grid), out, accumulate ? 1 : 0);
}

void launch_clip_coef(const float* sumsq, float max_norm, float* norm, float* coef, hipStream_t st) {
  clip_coef_kernel<<<1, 64, 0, st>>>(sumsq, max_norm, norm, coef);
}

}  // namespace dla
