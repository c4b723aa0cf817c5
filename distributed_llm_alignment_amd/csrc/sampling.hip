// Fused next-token sampler: temperature, top-k, top-p (nucleus) and the categorical draw in one
// kernel per decode step (HF `generate` semantics used by the reference's rollouts,
// teacher generation and eval: train_rlhf.py:123-124, generate_teacher_data.py:72-79,
// eval_alignment.py:68-79).
//
// One 1024-thread block per row streams the (bf16) logits row, which stays L2-resident across
// the passes (V = 128256 -> 256 KB):
//   1. max / argmax (greedy rows stop here);
//   2. top-k threshold: bisection on the logit value, counting tokens >= mid;
//   3. top-p threshold on the renormalised top-k mass: bisection on the value so that the kept
//      set is the smallest prefix (descending) whose mass reaches top_p (HF TopPLogitsWarper);
//   4. draw u ~ U(0, kept mass) with Philox4x32-10 keyed by (seed, row, step counter) and locate
//      the token with a block prefix scan over contiguous per-thread vocab segments.
// No sort, no [B, V] temporaries, no host sync; the step counter lives in device memory so a
// captured hipGraph draws fresh numbers on every replay.
#include "common.h"

namespace dla {

constexpr int kSampNT = 1024;

__device__ __forceinline__ void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                             uint32_t k0, uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
  const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
  const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
  c1 = (uint32_t)p1;
  c3 = (uint32_t)p0;
  c0 = n0;
  c2 = n2;
}

__device__ float philox_uniform(uint64_t seed, uint64_t a, uint64_t b) {
  uint32_t c0 = (uint32_t)a, c1 = (uint32_t)(a >> 32), c2 = (uint32_t)b, c3 = (uint32_t)(b >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return (c0 >> 8) * (1.0f / 16777216.0f);  // [0, 1)
}

template <typename T>
__device__ __forceinline__ float ld(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, int64_t i) { return bf2f(p[i]); }
template <>
__device__ __forceinline__ float ld<float>(const float* p, int64_t i) { return p[i]; }

__device__ __forceinline__ float bsum(float v, float* sc) { return block_sum<kSampNT>(v, sc); }
__device__ __forceinline__ float bmax(float v, float* sc) { return block_max<kSampNT>(v, sc); }

template <typename T>
__global__ __launch_bounds__(kSampNT) void sample_kernel(const T* __restrict__ logits, int64_t ld_,
                                                          int V, float inv_temp, int top_k,
                                                          float top_p, bool greedy,
                                                          const int64_t* __restrict__ rng,
                                                          int64_t* __restrict__ out) {
  __shared__ float sc[kSampNT / 64];
  __shared__ float seg[kSampNT];
  __shared__ int ans;
  const int64_t r = blockIdx.x;
  const T* row = logits + r * ld_;
  const int tid = threadIdx.x;
  // 1. max / argmax (first index on ties)
  float m = -INFINITY;
  int am = 0x7fffffff;
  for (int v = tid; v < V; v += kSampNT) {
    const float x = ld(row, v);
    if (x > m) {
      m = x;
      am = v;
    }
  }
  const float gmax = bmax(m, sc);
  int cand = (m == gmax) ? am : 0x7fffffff;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
  __shared__ int amin[kSampNT / 64];
  if ((tid & 63) == 0) amin[tid >> 6] = cand;
  __syncthreads();
  if (greedy || inv_temp <= 0.f) {
    if (tid == 0) {
      int a = amin[0];
      for (int i = 1; i < kSampNT / 64; ++i) a = min(a, amin[i]);
      out[r] = a;
    }
    return;
  }
  // work in scaled-logit space z = (x - max) * inv_temp (<= 0); weight e(z) = exp(z)
  // 2. top-k threshold: largest tau with count(z >= tau) >= k
  float tau_lo = -INFINITY;
  if (top_k > 0 && top_k < V) {
    float lo = -80.f, hi = 0.f;  // exp(-80) ~ 0: below is irrelevant mass
    for (int it = 0; it < 24; ++it) {
      const float mid = 0.5f * (lo + hi);
      float c = 0.f;
      for (int v = tid; v < V; v += kSampNT) c += ((ld(row, v) - gmax) * inv_temp >= mid) ? 1.f : 0.f;
      c = bsum(c, sc);
      if (c >= (float)top_k) lo = mid;
      else hi = mid;
    }
    tau_lo = lo;
  }
  // 3. top-p threshold on the renormalised top-k mass
  float tau = tau_lo;
  if (top_p < 1.f) {
    float z_tot = 0.f;
    for (int v = tid; v < V; v += kSampNT) {
      const float z = (ld(row, v) - gmax) * inv_temp;
      z_tot += z >= tau_lo ? __expf(z) : 0.f;
    }
    z_tot = bsum(z_tot, sc);
    const float target = top_p * z_tot;
    float lo = fmaxf(tau_lo, -80.f), hi = 0.f;  // mass(z >= hi=0) >= exp(0) > 0
    for (int it = 0; it < 24; ++it) {
      const float mid = 0.5f * (lo + hi);
      float s = 0.f;
      for (int v = tid; v < V; v += kSampNT) {
        const float z = (ld(row, v) - gmax) * inv_temp;
        s += z >= mid ? __expf(z) : 0.f;
      }
      s = bsum(s, sc);
      if (s >= target) lo = mid;
      else hi = mid;
    }
    tau = fmaxf(tau_lo, lo);
  }
  // 4. categorical draw over {z >= tau}: contiguous segment per thread, block scan
  const int per = (V + kSampNT - 1) / kSampNT;
  const int s0 = tid * per, s1 = min(V, s0 + per);
  float mine = 0.f;
  for (int v = s0; v < s1; ++v) {
    const float z = (ld(row, v) - gmax) * inv_temp;
    mine += z >= tau ? __expf(z) : 0.f;
  }
  seg[tid] = mine;
  if (tid == 0) ans = -1;
  __syncthreads();
  // inclusive scan (Hillis-Steele) over 1024 partial masses
  for (int o = 1; o < kSampNT; o <<= 1) {
    const float add = tid >= o ? seg[tid - o] : 0.f;
    __syncthreads();
    seg[tid] += add;
    __syncthreads();
  }
  const float total = seg[kSampNT - 1];
  const float u = philox_uniform((uint64_t)rng[0], (uint64_t)r, (uint64_t)rng[1]) * total;
  const float before = tid > 0 ? seg[tid - 1] : 0.f;
  if (mine > 0.f && u >= before && u < seg[tid]) {
    float acc = before;
    int pick = -1;
    for (int v = s0; v < s1; ++v) {
      const float z = (ld(row, v) - gmax) * inv_temp;
      if (z >= tau) {
        acc += __expf(z);
        pick = v;
        if (u < acc) break;
      }
    }
    ans = pick;
  }
  __syncthreads();
  if (tid == 0) {
    int a = ans;
    if (a < 0) {  // u landed on a rounding gap at the very top: take the argmax
      a = amin[0];
      for (int i = 1; i < kSampNT / 64; ++i) a = min(a, amin[i]);
    }
    out[r] = a;
  }
}

void launch_sample(const void* logits, bool is_bf16, int64_t ld_, int64_t rows, int V,
                   float inv_temp, int top_k, float top_p, bool greedy, const int64_t* rng,
                   int64_t* out, hipStream_t st) {
  if (rows == 0) return;
  if (is_bf16)
    sample_kernel<bf16_t><<<rows, kSampNT, 0, st>>>(static_cast<const bf16_t*>(logits), ld_, V,
                                                     inv_temp, top_k, top_p, greedy, rng, out);
  else
    sample_kernel<float><<<rows, kSampNT, 0, st>>>(static_cast<const float*>(logits), ld_, V,
                                                    inv_temp, top_k, top_p, greedy, rng, out);
}

}  // namespace dla
