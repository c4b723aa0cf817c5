// Reward head: pooling + dropout + Linear(H, 1) in one pass per sequence (SURVEY K13 + K21).
//
// Reference: src/models/reward_model.py:38-64 -- `scorer = Sequential(Dropout(p), Linear(H, 1))`
// applied to the last-token (or masked-mean) hidden state; eager PyTorch runs an index/gather,
// a dropout kernel (mask tensor materialised), a GEMV and a bias add, and the backward a dense
// [B, T, H] zero tensor plus an index_put.
//
// Forward (one 256-thread workgroup per sequence): pooled row (last valid token, or the masked
// mean over T), dropout from a counter-based hash of (seed, row, column) -- the backward
// regenerates the same mask instead of storing it --, dot with the scorer weight (block
// reduction), + bias. The dropped pooled row is kept (fp32 [B, H]) for the weight gradient.
// Backward: writes dHidden only where the pooling read (the last token, or the valid positions
// for mean), scaled by the regenerated mask; rows are zero elsewhere (one memset).
#include "common.h"
#include "reward_head.h"

namespace dla {

// keep-mask of element (row, col): splitmix64-style hash of (seed, row, col) compared with p
__device__ __forceinline__ bool rh_keep(uint64_t seed, int row, int col, float p) {
  if (p <= 0.f) return true;
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (static_cast<uint64_t>(row) * 0x100000001B3ull +
                                                static_cast<uint64_t>(col) + 1ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const float u = static_cast<float>(z >> 40) * (1.0f / 16777216.0f);  // [0, 1)
  return u >= p;
}



__global__ __launch_bounds__(256) void reward_head_fwd_kernel(RHParams p) {
  __shared__ float red[4];
  const int b = blockIdx.x;
  const bf16_t* hb = p.hidden + b * p.sb;
  float cnt = 1.f;
  if (p.mask) {
    float c = 0.f;
    for (int t = threadIdx.x; t < p.T; t += 256) c += p.mask[static_cast<int64_t>(b) * p.T + t];
    c = block_sum<256>(c, red);
    cnt = fmaxf(c, 1.f);
  }
  const float scale = p.p > 0.f ? 1.f / (1.f - p.p) : 1.f;
  float dot = 0.f;
  for (int c0 = threadIdx.x * 8; c0 < p.H; c0 += 256 * 8) {
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (p.mask) {
      for (int t = 0; t < p.T; ++t) {
        const float m = p.mask[static_cast<int64_t>(b) * p.T + t];
        if (m != 0.f) {
          const bf16x8 x = load_bf16x8(hb + t * p.st + c0);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += bf2f(x[j]) * m;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(v[j] / cnt));  // the reference pools in bf16
    } else {
      const bf16x8 x = load_bf16x8(hb + static_cast<int64_t>(p.last[b]) * p.st + c0);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(x[j]);
    }
    const bf16x8 wv = load_bf16x8(p.w + c0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = rh_keep(p.seed, b, c0 + j, p.p) ? v[j] * scale : 0.f;
      p.pooled[static_cast<int64_t>(b) * p.H + c0 + j] = d;
      dot += d * bf2f(wv[j]);
    }
  }
  dot = block_sum<256>(dot, red);
  if (threadIdx.x == 0) p.score[b] = dot + (p.bias ? bf2f(p.bias[0]) : 0.f);
}

__global__ __launch_bounds__(256) void reward_head_bwd_kernel(RHParams p) {
  __shared__ float red[4];
  const int b = blockIdx.x;
  const float ds = p.dscore[b];
  const float scale = p.p > 0.f ? 1.f / (1.f - p.p) : 1.f;
  float cnt = 1.f;
  if (p.mask) {
    float c = 0.f;
    for (int t = threadIdx.x; t < p.T; t += 256) c += p.mask[static_cast<int64_t>(b) * p.T + t];
    c = block_sum<256>(c, red);
    cnt = fmaxf(c, 1.f);
  }
  bf16_t* db = p.dhidden + static_cast<int64_t>(b) * p.T * p.H;
  for (int c0 = threadIdx.x * 8; c0 < p.H; c0 += 256 * 8) {
    const bf16x8 wv = load_bf16x8(p.w + c0);
    float g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = rh_keep(p.seed, b, c0 + j, p.p) ? ds * bf2f(wv[j]) * scale : 0.f;
    if (p.mask) {
      for (int t = 0; t < p.T; ++t) {
        const float m = p.mask[static_cast<int64_t>(b) * p.T + t];
        if (m != 0.f) {
          float o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = g[j] * m / cnt;
          store_bf16x8(db + static_cast<int64_t>(t) * p.H + c0, pack_bf16x8(o));
        }
      }
    } else {
      store_bf16x8(db + static_cast<int64_t>(p.last[b]) * p.H + c0, pack_bf16x8(g));
    }
  }
}

void launch_reward_head_fwd(const RHParams& p, hipStream_t st) {
  reward_head_fwd_kernel<<<p.B, 256, 0, st>>>(p);
}
void launch_reward_head_bwd(const RHParams& p, hipStream_t st) {
  reward_head_bwd_kernel<<<p.B, 256, 0, st>>>(p);
}

}  // namespace dla
