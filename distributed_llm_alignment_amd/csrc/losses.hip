// Sequence-level objective kernels (SURVEY K11 reduction, K12, K14, K15).
//
//   seq_reduce      : masked per-sequence sum / count of token log-probs
//                     (the `(gathered * mask).sum(1) / mask.sum(1).clamp(min=1)` tail of
//                      src/training/train_dpo.py:38 and train_rlhf.py:57)
//   dpo_loss        : -logsigmoid(beta*((pc-pr)-(rc-rr))).mean()   train_dpo.py:42-44
//                     + fused backward coefficients, rewards, margin and accuracy outputs
//   pairwise_loss   : -logsigmoid(sc - sr).mean()                   src/models/reward_model.py:67-68
//   kl_penalty_pg   : kl = lp - lr; r' = r - c*kl; A = r' - mean(r'); loss = -mean(A*lp)
//                                                                   train_rlhf.py:149-153
//   gae / ppo_policy_loss / ppo_value_loss : token-level actor-critic PPO (below)
// Batch dimensions here are small (pairs per micro-batch), so each loss is a single
// 256-thread block; the point is fusing fwd+bwd+metrics into one launch with no host sync.
#include "common.h"

namespace dla {

// one block per sequence: out_sum[s] = sum_t lp[s,t]*m[s,t]; out_cnt[s] = sum_t m[s,t]
__global__ __launch_bounds__(256) void seq_reduce_kernel(const float* __restrict__ lp,
                                                          const float* __restrict__ mask, int T,
                                                          float* __restrict__ out_sum,
                                                          float* __restrict__ out_cnt) {
  __shared__ float scratch[4];
  const int64_t s = blockIdx.x;
  float a = 0.f, c = 0.f;
  for (int t = threadIdx.x; t < T; t += 256) {
    const float m = mask[s * T + t];
    a += lp[s * T + t] * m;
    c += m;
  }
  a = block_sum<256>(a, scratch);
  c = block_sum<256>(c, scratch);
  if (threadIdx.x == 0) {
    out_sum[s] = a;
    out_cnt[s] = c;
  }
}

// g_tok[s,t] = coef[s] * mask[s,t] / (mean ? max(cnt[s],1) : 1)
__global__ __launch_bounds__(256) void seq_expand_grad_kernel(const float* __restrict__ coef,
                                                               const float* __restrict__ mask,
                                                               const float* __restrict__ cnt,
                                                               int T, int S, bool mean,
                                                               float* __restrict__ g) {
  const int64_t n = static_cast<int64_t>(S) * T;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t s = i / T;
    const float d = mean ? fmaxf(cnt[s], 1.f) : 1.f;
    g[i] = coef[s] * mask[i] / d;
  }
}

// pol/ref: [2B] seq log-probs, chosen = [0,B), rejected = [B,2B).
// outputs: loss[0]; metrics[0..3] = (mean chosen reward, mean rejected reward, accuracy, margin)
// dpol[2B] = dloss/dpol (already includes 1/B), rewards_out[2B] = beta*(pol-ref).
__global__ __launch_bounds__(256) void dpo_loss_kernel(const float* __restrict__ pol,
                                                        const float* __restrict__ ref, int B,
                                                        float beta, float label_smoothing,
                                                        float* __restrict__ loss,
                                                        float* __restrict__ dpol,
                                                        float* __restrict__ rewards_out,
                                                        float* __restrict__ metrics) {
  __shared__ float scratch[4];
  float l = 0.f, rc = 0.f, rr = 0.f, acc = 0.f, mg = 0.f;
  for (int i = threadIdx.x; i < B; i += 256) {
    const float c_r = beta * (pol[i] - ref[i]);
    const float r_r = beta * (pol[B + i] - ref[B + i]);
    const float z = c_r - r_r;  // beta * ((pc - pr) - (rc - rr))
    // loss = -(1-ls)*logsig(z) - ls*logsig(-z)
    l += -(1.f - label_smoothing) * log_sigmoid(z) - label_smoothing * log_sigmoid(-z);
    // dloss/dz = -(1-ls)*sig(-z) + ls*sig(z)
    const float dz = (-(1.f - label_smoothing) * sigmoidf_(-z) + label_smoothing * sigmoidf_(z)) / B;
    dpol[i] = dz * beta;
    dpol[B + i] = -dz * beta;
    rewards_out[i] = c_r;
    rewards_out[B + i] = r_r;
    rc += c_r;
    rr += r_r;
    acc += (c_r > r_r) ? 1.f : 0.f;
    mg += z;
  }
  l = block_sum<256>(l, scratch);
  rc = block_sum<256>(rc, scratch);
  rr = block_sum<256>(rr, scratch);
  acc = block_sum<256>(acc, scratch);
  mg = block_sum<256>(mg, scratch);
  if (threadIdx.x == 0) {
    loss[0] = l / B;
    metrics[0] = rc / B;
    metrics[1] = rr / B;
    metrics[2] = acc / B;
    metrics[3] = mg / B;
  }
}

// scores: [2B] (chosen, rejected). loss = -mean logsig(sc - sr); dscores; metrics = accuracy.
__global__ __launch_bounds__(256) void pairwise_loss_kernel(const float* __restrict__ sc,
                                                             const float* __restrict__ sr, int B,
                                                             float* __restrict__ loss,
                                                             float* __restrict__ dsc,
                                                             float* __restrict__ dsr,
                                                             float* __restrict__ acc_out) {
  __shared__ float scratch[4];
  float l = 0.f, acc = 0.f;
  for (int i = threadIdx.x; i < B; i += 256) {
    const float z = sc[i] - sr[i];
    l += -log_sigmoid(z);
    const float dz = -sigmoidf_(-z) / B;
    dsc[i] = dz;
    dsr[i] = -dz;
    acc += z > 0.f ? 1.f : 0.f;
  }
  l = block_sum<256>(l, scratch);
  acc = block_sum<256>(acc, scratch);
  if (threadIdx.x == 0) {
    loss[0] = l / B;
    acc_out[0] = acc / B;
  }
}

// REINFORCE with KL-shaped reward and mean baseline (train_rlhf.py:149-153).
// out: loss[0], kl_mean[0]; dlp[n] = dloss/dlp = -A[i]/n (A is stop-gradient).
__global__ __launch_bounds__(256) void kl_penalty_pg_kernel(const float* __restrict__ lp,
                                                             const float* __restrict__ lr,
                                                             const float* __restrict__ reward,
                                                             int n, float kl_coef,
                                                             float* __restrict__ loss,
                                                             float* __restrict__ kl_mean,
                                                             float* __restrict__ dlp,
                                                             float* __restrict__ adv_out) {
  __shared__ float scratch[4];
  float rsum = 0.f, ksum = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float kl = lp[i] - lr[i];
    rsum += reward[i] - kl_coef * kl;
    ksum += kl;
  }
  rsum = block_sum<256>(rsum, scratch);
  ksum = block_sum<256>(ksum, scratch);
  const float rmean = rsum / n;
  float l = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float kl = lp[i] - lr[i];
    const float a = reward[i] - kl_coef * kl - rmean;
    adv_out[i] = a;
    dlp[i] = -a / n;
    l += -a * lp[i];
  }
  l = block_sum<256>(l, scratch);
  if (threadIdx.x == 0) {
    loss[0] = l / n;
    kl_mean[0] = ksum / n;
  }
}

// ==============================================================================================
// PPO (actor-critic) token objectives: the north-star "PPO RLHF (actor + critic + reward)"
// configuration. The reference's train_rlhf.py:149-153 is the sequence-level REINFORCE special
// case above (kl_penalty_pg); these run over [S, T] token grids.
// ==============================================================================================

// Generalised advantage estimation, one wave per sequence:
//   A_t = m_t * (delta_t + gamma*lam*m_{t+1} * A_{t+1}),  delta_t = r_t + gamma*m_{t+1}*V_{t+1} - V_t
// is the affine reverse recurrence x_t = a_t + c_t x_{t+1}. Lane l owns the contiguous segment
// [l*L, (l+1)*L) (L = ceil(T/64)): pass 1 composes the segment's map x_{t0} = A + C x_{t1}, a
// log2(64)-step shuffle scan composes the maps of lanes l..63 (so every lane learns the x
// entering its segment from the right), pass 2 re-walks the segment writing A_t and the
// returns R_t = A_t + V_t. No serial 1-thread-per-sequence loop over T.
__global__ __launch_bounds__(64) void gae_kernel(const float* __restrict__ r, const float* __restrict__ v,
                                                 const float* __restrict__ m, int T, float gamma,
                                                 float lam, float* __restrict__ adv,
                                                 float* __restrict__ ret) {
  const int lane = threadIdx.x;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const int L = (T + 63) / 64;
  const int t0 = min(T, lane * L), t1 = min(T, t0 + L);
  auto coef = [&](int t, float& a, float& c) {
    const float mt = m[base + t];
    const float mn = t + 1 < T ? m[base + t + 1] : 0.f;
    const float vn = t + 1 < T ? v[base + t + 1] : 0.f;
    a = mt * (r[base + t] + gamma * mn * vn - v[base + t]);
    c = mt * gamma * lam * mn;
  };
  float A = 0.f, C = 1.f;  // identity map for an empty segment
  for (int t = t1 - 1; t >= t0; --t) {
    float a, c;
    coef(t, a, c);
    A = a + c * A;
    C = c * C;
  }
  // (SA, SC): composition of the maps of lanes l .. min(63, l + 2^k - 1)
  float SA = A, SC = C;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float na = __shfl_down(SA, off, 64), nc = __shfl_down(SC, off, 64);
    if (lane + off < 64) {
      SA = SA + SC * na;
      SC = SC * nc;
    }
  }
  float x = __shfl_down(SA, 1, 64);  // x entering this segment from the right (x_T = 0)
  if (lane == 63) x = 0.f;
  for (int t = t1 - 1; t >= t0; --t) {
    float a, c;
    coef(t, a, c);
    x = a + c * x;
    adv[base + t] = x;
    ret[base + t] = x + v[base + t];
  }
}

// Clipped surrogate over masked tokens (fwd + bwd in one launch):
//   rho = exp(lp - lp_old); loss = sum m * max(-A rho, -A clip(rho, 1-eps, 1+eps)) / sum m
//   dlp = m * (-A rho if the unclipped branch is the max else 0) / sum m
//   metrics: [0] clip fraction, [1] approx KL  mean((rho - 1) - log rho), [2] token count
__global__ __launch_bounds__(1024) void ppo_policy_loss_kernel(
    const float* __restrict__ lp, const float* __restrict__ old, const float* __restrict__ adv,
    const float* __restrict__ m, int64_t n, float eps, float* __restrict__ loss,
    float* __restrict__ dlp, float* __restrict__ metrics) {
  __shared__ float scratch[16];
  float cnt = 0.f, l = 0.f, cf = 0.f, kl = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 1024) {
    const float mi = m[i];
    const float d = lp[i] - old[i];
    const float rho = __expf(d), a = adv[i];
    const float l1 = -a * rho, l2 = -a * fminf(fmaxf(rho, 1.f - eps), 1.f + eps);
    l += mi * fmaxf(l1, l2);
    cnt += mi;
    cf += mi * (fabsf(rho - 1.f) > eps ? 1.f : 0.f);
    kl += mi * ((rho - 1.f) - d);
  }
  cnt = block_sum<1024>(cnt, scratch);
  l = block_sum<1024>(l, scratch);
  cf = block_sum<1024>(cf, scratch);
  kl = block_sum<1024>(kl, scratch);
  const float inv = 1.f / fmaxf(cnt, 1.f);
  for (int64_t i = threadIdx.x; i < n; i += 1024) {
    const float d = lp[i] - old[i];
    const float rho = __expf(d), a = adv[i];
    const float l1 = -a * rho, l2 = -a * fminf(fmaxf(rho, 1.f - eps), 1.f + eps);
    dlp[i] = l1 >= l2 ? m[i] * l1 * inv : 0.f;
  }
  if (threadIdx.x == 0) {
    loss[0] = l * inv;
    metrics[0] = cf * inv;
    metrics[1] = kl * inv;
    metrics[2] = cnt;
  }
}

// Clipped value loss: 0.5 * sum m * max((V - R)^2, (Vc - R)^2) / sum m,
// Vc = V_old + clamp(V - V_old, -c, c); dV through whichever branch is the max.
__global__ __launch_bounds__(1024) void ppo_value_loss_kernel(
    const float* __restrict__ val, const float* __restrict__ old, const float* __restrict__ ret,
    const float* __restrict__ m, int64_t n, float clip, float* __restrict__ loss,
    float* __restrict__ dval) {
  __shared__ float scratch[16];
  float cnt = 0.f, l = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 1024) {
    const float mi = m[i], v = val[i], o = old[i], R = ret[i];
    const float vc = o + fminf(fmaxf(v - o, -clip), clip);
    l += mi * 0.5f * fmaxf((v - R) * (v - R), (vc - R) * (vc - R));
    cnt += mi;
  }
  cnt = block_sum<1024>(cnt, scratch);
  l = block_sum<1024>(l, scratch);
  const float inv = 1.f / fmaxf(cnt, 1.f);
  for (int64_t i = threadIdx.x; i < n; i += 1024) {
    const float mi = m[i], v = val[i], o = old[i], R = ret[i];
    const float dv = v - o;
    const float vc = o + fminf(fmaxf(dv, -clip), clip);
    const float u1 = (v - R) * (v - R), u2 = (vc - R) * (vc - R);
    const float g = u1 >= u2 ? (v - R) : (fabsf(dv) <= clip ? (vc - R) : 0.f);
    dval[i] = mi * g * inv;
  }
  if (threadIdx.x == 0) loss[0] = l * inv;
}

// ----------------------------------------------------------------------------------------------
void launch_gae(const float* r, const float* v, const float* m, int S, int T, float gamma,
                float lam, float* adv, float* ret, hipStream_t st) {
  if (S == 0 || T == 0) return;
  gae_kernel<<<S, 64, 0, st>>>(r, v, m, T, gamma, lam, adv, ret);
}
void launch_ppo_policy_loss(const float* lp, const float* old, const float* adv, const float* m,
                            int64_t n, float eps, float* loss, float* dlp, float* metrics,
                            hipStream_t st) {
  ppo_policy_loss_kernel<<<1, 1024, 0, st>>>(lp, old, adv, m, n, eps, loss, dlp, metrics);
}
void launch_ppo_value_loss(const float* val, const float* old, const float* ret, const float* m,
                           int64_t n, float clip, float* loss, float* dval, hipStream_t st) {
  ppo_value_loss_kernel<<<1, 1024, 0, st>>>(val, old, ret, m, n, clip, loss, dval);
}

// ----------------------------------------------------------------------------------------------
void launch_seq_reduce(const float* lp, const float* mask, int S, int T, float* sum, float* cnt,
                       hipStream_t st) {
  if (S == 0) return;
  seq_reduce_kernel<<<S, 256, 0, st>>>(lp, mask, T, sum, cnt);
}
void launch_seq_expand_grad(const float* coef, const float* mask, const float* cnt, int S, int T,
                            bool mean, float* g, hipStream_t st) {
  const int64_t n = static_cast<int64_t>(S) * T;
  if (n == 0) return;
  int64_t grid = (n + 255) / 256;
  if (grid > 2048) grid = 2048;
  seq_expand_grad_kernel<<<static_cast<unsigned>(grid), 256, 0, st>>>(coef, mask, cnt, T, S, mean, g);
}
void launch_dpo_loss(const float* pol, const float* ref, int B, float beta, float ls, float* loss,
                     float* dpol, float* rewards, float* metrics, hipStream_t st) {
  dpo_loss_kernel<<<1, 256, 0, st>>>(pol, ref, B, beta, ls, loss, dpol, rewards, metrics);
}
void launch_pairwise_loss(const float* sc, const float* sr, int B, float* loss, float* dsc,
                          float* dsr, float* acc, hipStream_t st) {
  pairwise_loss_kernel<<<1, 256, 0, st>>>(sc, sr, B, loss, dsc, dsr, acc);
}
void launch_kl_penalty_pg(const float* lp, const float* lr, const float* reward, int n,
                          float kl_coef, float* loss, float* kl_mean, float* dlp, float* adv,
                          hipStream_t st) {
  kl_penalty_pg_kernel<<<1, 256, 0, st>>>(lp, lr, reward, n, kl_coef, loss, kl_mean, dlp, adv);
}

}  // namespace dla
