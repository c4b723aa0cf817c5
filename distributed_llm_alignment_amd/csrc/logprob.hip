// Vocabulary-row reductions on bf16 logits.
//
// Reference semantics:
//   * `compute_logprobs` (src/training/train_dpo.py:31-39) and `sequence_logprob`
//     (src/training/train_rlhf.py:50-58): log_softmax -> gather(target) per token.
//   * HF ForCausalLMLoss (train_sft.py:145-146): token NLL with ignore_index=-100.
//   * Ensemble KL distillation (train_distill.py:127-144): sum_v p_bar (log p_bar - log q).
// The eager reference materialises fp32 log_softmax over [B,T,V] (1+ GB per micro-batch at
// V=128256). Here one 256-thread block streams a bf16 logits row once (16 B per lane,
// online max/sum in fp32), emitting only per-row scalars; the backward rewrites the SAME
// buffer in place as bf16 dlogits, which feeds the dH / dW GEMMs directly.
#include "common.h"

namespace dla {

// online (max, sum-exp) pair merge
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

template <bool VEC>
__device__ __forceinline__ void row_lse(const bf16_t* __restrict__ row, int V, float& m_out,
                                        float& s_out) {
  __shared__ float sm[4], ss[4];
  float m = -INFINITY, s = 0.f;
  if constexpr (VEC) {
    const int nv = V >> 3;
    for (int i = threadIdx.x; i < nv; i += 256) {
      bf16x8 a = load_bf16x8(row + i * 8);
      float x[8];
      float lm = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        x[j] = bf2f(a[j]);
        lm = fmaxf(lm, x[j]);
      }
      if (lm > m) {
        s *= __expf(m - lm);
        m = lm;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(x[j] - m);
    }
  } else {
    for (int i = threadIdx.x; i < V; i += 256) {
      const float x = bf2f(row[i]);
      if (x > m) {
        s *= __expf(m - x);
        m = x;
      }
      s += __expf(x - m);
    }
  }
  // wave merge
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_merge(m, s, m2, s2);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm[w] = m;
    ss[w] = s;
  }
  __syncthreads();
  m = sm[0];
  s = ss[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) lse_merge(m, s, sm[i], ss[i]);
  m_out = m;
  s_out = s;
}

// logp[r] = logits[r, tgt[r] - off] - lse[r] when this vocab shard [off, off+V) owns the
// target; rows with tgt < 0 (ignored) or a target owned by another shard -> logp 0. lse (of the
// local shard) is always written. off = 0, V = full vocab for the unsharded LM head.
template <bool VEC>
__global__ __launch_bounds__(256) void logprob_fwd_kernel(const bf16_t* __restrict__ logits,
                                                           int64_t ld, int V, int64_t off,
                                                           const int64_t* __restrict__ tgt,
                                                           float* __restrict__ logp,
                                                           float* __restrict__ lse_out) {
  const int64_t r = blockIdx.x;
  const bf16_t* row = logits + r * ld;
  float m, s;
  row_lse<VEC>(row, V, m, s);
  if (threadIdx.x == 0) {
    const float lse = m + __logf(s);
    lse_out[r] = lse;
    const int64_t t = tgt[r] - off;
    logp[r] = (tgt[r] >= 0 && t >= 0 && t < V) ? bf2f(row[t]) - lse : 0.f;
  }
}

// In place: logits[r, v] <- g[r] * (1[v == tgt - off] - exp(logits - lse)), g = dL/dlogp[r];
// lse is the GLOBAL (all-shard) log-sum-exp. Ignored rows (tgt < 0) -> 0.
template <bool VEC>
__global__ __launch_bounds__(256) void logprob_bwd_kernel(bf16_t* __restrict__ logits, int64_t ld,
                                                           int V, int64_t off,
                                                           const int64_t* __restrict__ tgt,
                                                           const float* __restrict__ lse_in,
                                                           const float* __restrict__ g) {
  const int64_t r = blockIdx.x;
  bf16_t* row = logits + r * ld;
  const int64_t t = tgt[r] - off;
  const float gr = tgt[r] >= 0 ? g[r] : 0.f;
  const float lse = lse_in[r];
  if constexpr (VEC) {
    const int nv = V >> 3;
    for (int i = threadIdx.x; i < nv; i += 256) {
      bf16x8 a = load_bf16x8(row + i * 8), o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int v = i * 8 + j;
        const float p = __expf(bf2f(a[j]) - lse);
        o[j] = f2bf(gr * ((v == t ? 1.f : 0.f) - p));
      }
      store_bf16x8(row + i * 8, o);
    }
  } else {
    for (int v = threadIdx.x; v < V; v += 256) {
      const float p = __expf(bf2f(row[v]) - lse);
      row[v] = f2bf(gr * ((v == t ? 1.f : 0.f) - p));
    }
  }
}

// The same gradient with a transposed second output (the LM head's TN weight-gradient operand):
// dlogits written in place AND dlogitsT [V, rows] (ld = rows), from one read of the logits, in
// place of the in-place kernel + a separate transpose pass (which reads and writes the [rows, V]
// gradient once more: 815 us per Llama-3-8B DPO micro-batch, profiles/r6_*). Each lane owns an
// 8 x 8 block (8 rows x 8 vocab columns) and transposes it in registers (tr8_bf16); a wave covers
// 64 rows x 64 columns; grid (ceil(V / 256), rows / 64); rows % 8 == 0, V % 8 == 0, ld % 8 == 0.
__global__ __launch_bounds__(256) void logprob_bwd_t_kernel(bf16_t* __restrict__ logits, int64_t ld, int V,
                                                             int64_t off, const int64_t* __restrict__ tgt,
                                                             const float* __restrict__ lse_in,
                                                             const float* __restrict__ g,
                                                             bf16_t* __restrict__ outT, int64_t rows) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r = static_cast<int64_t>(blockIdx.y) * 64 + (lane >> 3) * 8;
  const int c = blockIdx.x * 256 + w * 64 + (lane & 7) * 8;
  if (r >= rows || c >= V) return;
  bf16x8 a[8], o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = load_bf16x8(logits + (r + i) * ld + c);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t t = tgt[r + i] - off;
    const float gr = tgt[r + i] >= 0 ? g[r + i] : 0.f;
    const float lse = lse_in[r + i];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float p = __expf(bf2f(a[i][j]) - lse);
      o[i][j] = f2bf(gr * ((c + j == t ? 1.f : 0.f) - p));
    }
    store_bf16x8(logits + (r + i) * ld + c, o[i]);
  }
  bf16x8 tt[8];
  tr8_bf16(o, tt);
#pragma unroll
  for (int j = 0; j < 8; ++j) store_bf16x8(outT + static_cast<int64_t>(c + j) * rows + r, tt[j]);
}

// Ensemble forward-KL distillation, one row per block:
//   p_bar = mean_k softmax(teacher_k), q = softmax(student)
//   kl[r] = sum_v p_bar (log p_bar - log q)
//   (optionally, in place) student_logits[r,:] <- g[r] * (q - p_bar)   (d kl / d z_student)
// Teacher rows are read with their own precomputed lse (t_lse[k, r]).
template <bool WRITE_GRAD>
__global__ __launch_bounds__(256) void ensemble_kl_kernel(bf16_t* __restrict__ s_logits,
                                                           const bf16_t* __restrict__ t_logits,
                                                           int64_t ld, int64_t t_stride, int K,
                                                           int V, const float* __restrict__ s_lse,
                                                           const float* __restrict__ t_lse,
                                                           int64_t rows, const float* __restrict__ g,
                                                           float* __restrict__ kl_out) {
  __shared__ float red[4];
  const int64_t r = blockIdx.x;
  bf16_t* srow = s_logits + r * ld;
  const float sl = s_lse[r];
  const float gr = WRITE_GRAD ? g[r] : 0.f;
  float acc = 0.f;
  for (int v = threadIdx.x; v < V; v += 256) {
    float pbar = 0.f;
    for (int k = 0; k < K; ++k)
      pbar += __expf(bf2f(t_logits[k * t_stride + r * ld + v]) - t_lse[k * rows + r]);
    pbar /= K;
    const float lq = bf2f(srow[v]) - sl;
    if (pbar > 0.f) acc += pbar * (__logf(pbar) - lq);
    if constexpr (WRITE_GRAD) srow[v] = f2bf(gr * (__expf(lq) - pbar));
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) kl_out[r] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void row_lse_kernel(const bf16_t* __restrict__ logits, int64_t ld,
                                                       int V, float* __restrict__ lse_out) {
  const int64_t r = blockIdx.x;
  float m, s;
  row_lse<false>(logits + r * ld, V, m, s);
  if (threadIdx.x == 0) lse_out[r] = m + __logf(s);
}

// ----------------------------------------------------------------------------------------------
void launch_logprob_fwd(const bf16_t* logits, int64_t ld, int V, int64_t off, int64_t rows,
                        const int64_t* tgt, float* logp, float* lse, hipStream_t st) {
  if (rows == 0) return;
  const bool vec = (V % 8 == 0) && (ld % 8 == 0);
  if (vec) logprob_fwd_kernel<true><<<rows, 256, 0, st>>>(logits, ld, V, off, tgt, logp, lse);
  else logprob_fwd_kernel<false><<<rows, 256, 0, st>>>(logits, ld, V, off, tgt, logp, lse);
}

void launch_logprob_bwd(bf16_t* logits, int64_t ld, int V, int64_t off, int64_t rows,
                        const int64_t* tgt, const float* lse, const float* g, hipStream_t st) {
  if (rows == 0) return;
  const bool vec = (V % 8 == 0) && (ld % 8 == 0);
  if (vec) logprob_bwd_kernel<true><<<rows, 256, 0, st>>>(logits, ld, V, off, tgt, lse, g);
  else logprob_bwd_kernel<false><<<rows, 256, 0, st>>>(logits, ld, V, off, tgt, lse, g);
}

bool launch_logprob_bwd_t(bf16_t* logits, int64_t ld, int V, int64_t rows, int64_t off, const int64_t* tgt,
                          const float* lse, const float* g, bf16_t* outT, hipStream_t st) {
  if (rows % 8 != 0 || V % 8 != 0 || ld % 8 != 0) return false;
  if (rows == 0) return true;
  const dim3 grid((V + 255) / 256, static_cast<unsigned>((rows + 63) / 64));
  logprob_bwd_t_kernel<<<grid, 256, 0, st>>>(logits, ld, V, off, tgt, lse, g, outT, rows);
  return true;
}

void launch_row_lse(const bf16_t* logits, int64_t ld, int V, int64_t rows, float* lse,
                    hipStream_t st) {
  if (rows == 0) return;
  row_lse_kernel<<<rows, 256, 0, st>>>(logits, ld, V, lse);
}

void launch_ensemble_kl(bf16_t* s_logits, const bf16_t* t_logits, int64_t ld, int64_t t_stride,
                        int K, int V, const float* s_lse, const float* t_lse, int64_t rows,
                        const float* g, float* kl, bool write_grad, hipStream_t st) {
  if (rows == 0) return;
  if (write_grad)
    ensemble_kl_kernel<true><<<rows, 256, 0, st>>>(s_logits, t_logits, ld, t_stride, K, V, s_lse,
                                                   t_lse, rows, g, kl);
  else
    ensemble_kl_kernel<false><<<rows, 256, 0, st>>>(s_logits, t_logits, ld, t_stride, K, V, s_lse,
                                                    t_lse, rows, g, kl);
}

}  // namespace dla
