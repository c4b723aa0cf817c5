// Fused next-token sampler: temperature, top-k, top-p (nucleus) and the categorical draw in one
// kernel per decode step (HF `generate` semantics used by the reference's rollouts,
// teacher generation and eval: train_rlhf.py:123-124, generate_teacher_data.py:72-79,
// eval_alignment.py:68-79).
//
// One 1024-thread block per row streams the (bf16) logits row, which stays L2-resident across
// the passes (V = 128256 -> 256 KB). Work in z = (x - max) / T:
//   1. max / argmax (greedy rows stop here);
//   2. thresholds by two-level LDS histograms instead of a sort: 2048 coarse bins over
//      z in [-64, 0] (counts + exp-masses, LDS atomics), a block suffix scan locates the bin
//      holding the k-th largest value (top-k) / the nucleus edge (top-p on the renormalised
//      top-k mass, HF TopKLogitsWarper -> TopPLogitsWarper order); a second 2048-bin histogram
//      inside that bin pins the threshold to 64/2048^2 ~ 1.5e-5 in z (2-5 passes per row);
//   3. draw u ~ U(0, kept mass) with Philox4x32-10 keyed by (seed, row, step counter) and locate
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

// 8 consecutive logits as fp32 (one 16-byte load for bf16, two for fp32); rows are 16-B aligned
// and V % 8 == 0 (checked on the host, scalar fallback otherwise)
template <typename T>
__device__ __forceinline__ void ld8(const T* p, int64_t i8, float* x);
template <>
__device__ __forceinline__ void ld8<bf16_t>(const bf16_t* p, int64_t i8, float* x) {
  const bf16x8 a = load_bf16x8(p + i8 * 8);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = bf2f(a[j]);
}
template <>
__device__ __forceinline__ void ld8<float>(const float* p, int64_t i8, float* x) {
  const f32x4 a = reinterpret_cast<const f32x4*>(p + i8 * 8)[0];
  const f32x4 b = reinterpret_cast<const f32x4*>(p + i8 * 8)[1];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    x[j] = a[j];
    x[4 + j] = b[j];
  }
}

// visit every logit of the row: fn(index, value); vectorised when VEC
template <bool VEC, typename T, typename F>
__device__ __forceinline__ void for_each_logit(const T* row, int V, F&& fn) {
  if constexpr (VEC) {
    for (int i = threadIdx.x; i < V / 8; i += kSampNT) {
      float x[8];
      ld8(row, i, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) fn(i * 8 + j, x[j]);
    }
  } else {
    for (int v = threadIdx.x; v < V; v += kSampNT) fn(v, ld(row, v));
  }
}

constexpr int kBins = 2048;    // histogram bins per refinement level
constexpr float kRange = 64.f;  // z = (x - max)/T in [-64, 0]; below: e^-64 relative mass, dropped

// In-place SUFFIX sums (from the top bin down) of c[kBins] / m[kBins] in LDS; 2 bins per thread.
__device__ void suffix_scan(int* c, float* m, int* tc, float* tm) {
  const int t = threadIdx.x;
  const int b0 = kBins - 2 - 2 * t;  // thread t owns bins b0, b0+1 (t = 0 owns the top pair)
  int lc = c[b0] + c[b0 + 1];
  float lm = m[b0] + m[b0 + 1];
  tc[t] = lc;
  tm[t] = lm;
  __syncthreads();
  for (int o = 1; o < kSampNT; o <<= 1) {  // inclusive prefix over t == suffix over bins
    const int ac = t >= o ? tc[t - o] : 0;
    const float am = t >= o ? tm[t - o] : 0.f;
    __syncthreads();
    tc[t] += ac;
    tm[t] += am;
    __syncthreads();
  }
  const int ec = tc[t] - lc;  // mass strictly above this thread's pair
  const float em = tm[t] - lm;
  const int c1 = c[b0 + 1];
  const float m1 = m[b0 + 1];
  __syncthreads();
  c[b0 + 1] = ec + c1;
  m[b0 + 1] = em + m1;
  c[b0] = ec + lc;
  m[b0] = em + lm;
  __syncthreads();
}

// Histogram of the row's z over [lo, lo + w) into kBins bins (counts + exp masses), optionally
// restricted to z >= floor_z.
template <bool VEC, typename T>
__device__ void histogram(const T* row, int V, float gmax, float inv_t, float lo, float w,
                          float floor_z, int* c, float* m) {
  for (int i = threadIdx.x; i < kBins; i += kSampNT) {
    c[i] = 0;
    m[i] = 0.f;
  }
  __syncthreads();
  const float sc = kBins / w;
  const float hi = lo + w;
  const bool top = hi >= 0.f;  // the top bin also holds z == 0 (the max itself)
  for_each_logit<VEC>(row, V, [&](int, float xv) {
    const float z = (xv - gmax) * inv_t;
    if (z >= lo && (z < hi || (top && z <= 0.f)) && z >= floor_z) {
      const int b = min(kBins - 1, (int)((z - lo) * sc));
      atomicAdd(&c[b], 1);
      atomicAdd(&m[b], __expf(z));
    }
  });
  __syncthreads();
}

// Largest bin b whose suffix value reaches `need` (suffix arrays are non-increasing in b).
__device__ int find_bin_count(const int* sc, int need, int* out) {
  if (threadIdx.x == 0) *out = 0;
  __syncthreads();
  for (int b = threadIdx.x; b < kBins; b += kSampNT)
    if (sc[b] >= need && (b == kBins - 1 || sc[b + 1] < need)) *out = b;
  __syncthreads();
  return *out;
}
__device__ int find_bin_mass(const float* sm, float need, int* out) {
  if (threadIdx.x == 0) *out = 0;
  __syncthreads();
  for (int b = threadIdx.x; b < kBins; b += kSampNT)
    if (sm[b] >= need && (b == kBins - 1 || sm[b + 1] < need)) *out = b;
  __syncthreads();
  return *out;
}

template <typename T, bool VEC>
__global__ __launch_bounds__(kSampNT) void sample_kernel(const T* __restrict__ logits, int64_t ld_,
                                                          int V, float inv_temp, int top_k,
                                                          float top_p, bool greedy,
                                                          const int64_t* __restrict__ rng,
                                                          int64_t* __restrict__ out) {
  __shared__ float sc[kSampNT / 64];
  __shared__ int amin[kSampNT / 64];
  __shared__ int hc[kBins];
  __shared__ float hm[kBins];
  __shared__ int tc[kSampNT];
  __shared__ float tm[kSampNT];
  __shared__ int sel;
  __shared__ int ans;
  const int64_t r = blockIdx.x;
  const T* row = logits + r * ld_;
  const int tid = threadIdx.x;
  // 1. max / argmax (first index on ties)
  float m = -INFINITY;
  int am = 0x7fffffff;
  for_each_logit<VEC>(row, V, [&](int v, float x) {
    if (x > m) {
      m = x;
      am = v;
    }
  });
  const float gmax = block_max<kSampNT>(m, sc);
  int cand = (m == gmax) ? am : 0x7fffffff;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
  if ((tid & 63) == 0) amin[tid >> 6] = cand;
  __syncthreads();
  int argmax = amin[0];
  for (int i = 1; i < kSampNT / 64; ++i) argmax = min(argmax, amin[i]);
  if (greedy || inv_temp <= 0.f) {
    if (tid == 0) out[r] = argmax;
    return;
  }
  const float W = kRange / kBins;  // coarse bin width
  float tau = -kRange;             // keep z >= tau
  const bool need_k = top_k > 0 && top_k < V, need_p = top_p < 1.f;
  if (need_k || need_p) {
    // 2. coarse histogram over [-64, 0]
    histogram<VEC>(row, V, gmax, inv_temp, -kRange, kRange, -INFINITY, hc, hm);
    suffix_scan(hc, hm, tc, tm);
    float total = hm[0];
    int kbin = 0;
    int above_c = 0;
    float above_m = 0.f;
    if (need_k) {
      kbin = find_bin_count(hc, top_k, &sel);
      above_c = kbin + 1 < kBins ? hc[kbin + 1] : 0;
      above_m = kbin + 1 < kBins ? hm[kbin + 1] : 0.f;
    }
    // coarse suffix masses must survive the fine pass: stash the one needed later
    float pbin_need = 0.f;
    int pbin = 0;
    if (need_k) {
      // 3. refine the top-k threshold inside bin kbin
      const float lo = -kRange + kbin * W;
      __syncthreads();
      // keep the coarse suffix mass of bins >= kbin+1 for the top-p search below
      histogram<VEC>(row, V, gmax, inv_temp, lo, W, -INFINITY, hc, hm);
      suffix_scan(hc, hm, tc, tm);
      const int sb = find_bin_count(hc, top_k - above_c, &sel);
      tau = lo + sb * (W / kBins);
      total = above_m + hm[sb];
      if (need_p) {
        const float target = top_p * total;
        if (above_m < target) {  // the nucleus edge lies inside this same coarse bin
          const int sp = find_bin_mass(hm, target - above_m, &sel);
          tau = fmaxf(tau, lo + sp * (W / kBins));
          pbin = -1;  // done
        } else {
          pbin = 1;  // edge is in a higher coarse bin: needs the coarse suffix again
          pbin_need = target;
        }
      }
    } else {
      pbin = 2;  // no top-k floor: the coarse suffix sums above are already the right ones
      pbin_need = top_p * total;
    }
    if (need_p && pbin >= 1) {
      if (pbin == 1) {  // coarse pass restricted to z >= tau (the top-k floor)
        __syncthreads();
        histogram<VEC>(row, V, gmax, inv_temp, -kRange, kRange, tau, hc, hm);
        suffix_scan(hc, hm, tc, tm);
      }
      const int cb = find_bin_mass(hm, pbin_need, &sel);
      const float above = cb + 1 < kBins ? hm[cb + 1] : 0.f;
      const float lo = -kRange + cb * W;
      __syncthreads();
      histogram<VEC>(row, V, gmax, inv_temp, lo, W, tau, hc, hm);
      suffix_scan(hc, hm, tc, tm);
      const int sp = find_bin_mass(hm, pbin_need - above, &sel);
      tau = fmaxf(tau, lo + sp * (W / kBins));
    }
  }
  // 4. categorical draw over {z >= tau}: contiguous segment per thread, block scan
  // contiguous per-thread segments, in 8-element vectors when VEC
  const int per = VEC ? ((V / 8 + kSampNT - 1) / kSampNT) * 8 : (V + kSampNT - 1) / kSampNT;
  const int s0 = min(V, tid * per), s1 = min(V, s0 + per);
  float mine = 0.f;
  if constexpr (VEC) {
    for (int v = s0; v < s1; v += 8) {
      float x[8];
      ld8(row, v / 8, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float z = (x[j] - gmax) * inv_temp;
        mine += z >= tau ? __expf(z) : 0.f;
      }
    }
  } else {
    for (int v = s0; v < s1; ++v) {
      const float z = (ld(row, v) - gmax) * inv_temp;
      mine += z >= tau ? __expf(z) : 0.f;
    }
  }
  tm[tid] = mine;
  if (tid == 0) ans = -1;
  __syncthreads();
  for (int o = 1; o < kSampNT; o <<= 1) {
    const float add = tid >= o ? tm[tid - o] : 0.f;
    __syncthreads();
    tm[tid] += add;
    __syncthreads();
  }
  const float total = tm[kSampNT - 1];
  const float u = philox_uniform((uint64_t)rng[0], (uint64_t)r, (uint64_t)rng[1]) * total;
  const float before = tid > 0 ? tm[tid - 1] : 0.f;
  if (mine > 0.f && u >= before && u < tm[tid]) {
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
  if (tid == 0) out[r] = ans >= 0 ? ans : argmax;  // u on a rounding gap at the top: argmax
}

void launch_sample(const void* logits, bool is_bf16, int64_t ld_, int64_t rows, int V,
                   float inv_temp, int top_k, float top_p, bool greedy, const int64_t* rng,
                   int64_t* out, hipStream_t st) {
  if (rows == 0) return;
  const bool vec = V % 8 == 0 && ld_ % 8 == 0 &&
                   reinterpret_cast<uintptr_t>(logits) % 16 == 0;
#define DLA_SAMPLE(T, VV)                                                                         \
  sample_kernel<T, VV><<<rows, kSampNT, 0, st>>>(static_cast<const T*>(logits), ld_, V, inv_temp, \
                                                 top_k, top_p, greedy, rng, out)
  if (is_bf16) {
    if (vec) DLA_SAMPLE(bf16_t, true);
    else DLA_SAMPLE(bf16_t, false);
  } else {
    if (vec) DLA_SAMPLE(float, true);
    else DLA_SAMPLE(float, false);
  }
#undef DLA_SAMPLE
}

}  // namespace dla
