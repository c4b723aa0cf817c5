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
// Bin masses are summed as 2^-40 fixed-point integers (each exp(z) <= 1 rounded once), so the
// histogram -- and with it every threshold and the sampled token -- does not depend on the order
// in which the lanes' atomics land (a float LDS atomicAdd sum does, in its last bits).
constexpr float kHistFix = 1099511627776.0f;  // 2^40

template <bool VEC, typename T>
__device__ void histogram(const T* row, int V, float gmax, float inv_t, float lo, float w,
                          float floor_z, int* c, float* m) {
  __shared__ unsigned long long mfix[kBins];
  for (int i = threadIdx.x; i < kBins; i += kSampNT) {
    c[i] = 0;
    mfix[i] = 0ull;
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
      atomicAdd(&mfix[b], static_cast<unsigned long long>(__expf(z) * kHistFix));
    }
  });
  __syncthreads();
  for (int i = threadIdx.x; i < kBins; i += kSampNT)
    m[i] = static_cast<float>(static_cast<double>(mfix[i]) * (1.0 / 1099511627776.0));
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

// ---------------------------------------------------------------------------------------------
// Row-split sampler (plain / top-k / top-p draws) for large vocabularies. The single-block kernel above keeps
// 8 of 256 CUs busy at B = 8 and spends ~90 us per histogram pass. Here every row is cut into G
// chunks (G = 32 for V = 128256 -> B * 32 workgroups) and each pass is a separate launch:
//   max     (B x G)  chunk max / argmax -> partials
//   hist    (B x G)  chunk histogram in LDS over the pass's [lo, lo + w), z >= floor; occupied
//                    bins added to the row histogram with global integer atomics (masses in
//                    2^-40 fixed point, so the sums do not depend on workgroup order)
//   resolve (B)      read + re-zero the row histogram, suffix scan, the same bin searches as
//                    sample_kernel; writes the next pass's window / tau
//   mass    (B x G)  kept mass of each chunk (z >= tau)
//   pick    (B)      u ~ U(0, total) with the same Philox stream, chunk by prefix, token by a
//                    block scan inside the chunk
// Launch count is fixed by (top_k > 0, top_p < 1), so the sequence is hipGraph-capturable; rows
// whose thresholds settle early skip the remaining passes on the device.
constexpr int kSplitNT = 256;
constexpr int kSplitG = 32;  // chunks per row (compile-time: the merge loops fully unroll)

struct SplitState {  // per row, lives in the workspace between launches
  float tau, lo, w, floor_z, above_m, target;
  int phase, above_c;
};
enum : int { kDone = 0, kKCoarse = 1, kKFine = 2, kPCoarse = 3, kPFine = 4 };

struct SplitWs {
  float* pmax;        // [B, G]
  int* parg;          // [B, G]
  int* hc;                 // [B, kBins] row histogram counts (global atomics)
  unsigned long long* hm;  // [B, kBins] row histogram masses, 2^-40 fixed point
  SplitState* state;  // [B]
  float* cmass;       // [B, G]
};

constexpr double kFix = 1099511627776.0;  // 2^40: integer mass sums are order-independent

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

__host__ __device__ inline SplitWs split_ws(void* base, int64_t B, int G) {
  char* p = static_cast<char*>(base);
  SplitWs w;
  const size_t bg = size_t(B) * G;
  w.pmax = reinterpret_cast<float*>(p); p += align256(bg * 4);
  w.parg = reinterpret_cast<int*>(p); p += align256(bg * 4);
  w.hc = reinterpret_cast<int*>(p); p += align256(size_t(B) * kBins * 4);
  w.hm = reinterpret_cast<unsigned long long*>(p); p += align256(size_t(B) * kBins * 8);
  w.state = reinterpret_cast<SplitState*>(p); p += align256(size_t(B) * sizeof(SplitState));
  w.cmass = reinterpret_cast<float*>(p); p += align256(bg * 4);
  return w;
}
inline size_t split_ws_bytes(int64_t B, int G) {
  const size_t bg = size_t(B) * G;
  return align256(bg * 4) * 3 + align256(size_t(B) * kBins * 4) + align256(size_t(B) * kBins * 8) +
         align256(size_t(B) * sizeof(SplitState));
}

// chunk g of a row, in 8-element vectors: [v0, v1)
__device__ __forceinline__ void chunk_range(int V, int G, int g, int& v0, int& v1) {
  const int nv = V / 8, cv = (nv + G - 1) / G;
  v0 = min(nv, g * cv);
  v1 = min(nv, v0 + cv);
}

// row max (first index on ties) from the G chunk partials; every lane gets the result
__device__ __forceinline__ void row_max(const float* pmax, const int* parg, int G, float& gmax,
                                        int& argmax) {
  float m[kSplitG];
  int a[kSplitG];
#pragma unroll
  for (int g = 0; g < kSplitG; ++g) {  // all loads in flight before the compare chain
    m[g] = pmax[g];
    a[g] = parg[g];
  }
  gmax = -INFINITY;
  argmax = 0x7fffffff;
#pragma unroll
  for (int g = 0; g < kSplitG; ++g)  // chunks are in index order: strict > keeps the first index
    if (m[g] > gmax) {
      gmax = m[g];
      argmax = a[g];
    }
}

template <typename T>
__global__ __launch_bounds__(kSplitNT) void split_max_kernel(const T* __restrict__ logits,
                                                             int64_t ld_, int V, int G, SplitWs ws) {
  __shared__ float sm[kSplitNT / 64];
  __shared__ int sa[kSplitNT / 64];
  const int r = blockIdx.y, g = blockIdx.x, tid = threadIdx.x;
  for (int i = g * (kBins / kSplitG) + tid; i < (g + 1) * (kBins / kSplitG); i += kSplitNT) {
    ws.hc[int64_t(r) * kBins + i] = 0;  // the first histogram pass accumulates into zeros
    ws.hm[int64_t(r) * kBins + i] = 0ull;
  }
  const T* row = logits + int64_t(r) * ld_;
  int v0, v1;
  chunk_range(V, G, g, v0, v1);
  float m = -INFINITY;
  int am = 0x7fffffff;
  for (int i = v0 + tid; i < v1; i += kSplitNT) {
    float x[8];
    ld8(row, i, x);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (x[j] > m) {
        m = x[j];
        am = i * 8 + j;
      }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > m || (om == m && oa < am)) {
      m = om;
      am = oa;
    }
  }
  if ((tid & 63) == 0) {
    sm[tid >> 6] = m;
    sa[tid >> 6] = am;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < kSplitNT / 64; ++w)
      if (sm[w] > m || (sm[w] == m && sa[w] < am)) {
        m = sm[w];
        am = sa[w];
      }
    ws.pmax[r * G + g] = m;
    ws.parg[r * G + g] = am;
  }
}

template <typename T>
__global__ __launch_bounds__(kSplitNT) void split_hist_kernel(const T* __restrict__ logits,
                                                              int64_t ld_, int V, int G,
                                                              float inv_t, bool first, SplitWs ws) {
  __shared__ int c[kBins];
  __shared__ unsigned long long m[kBins];  // 2^-40 fixed point: order-independent sums
  const int r = blockIdx.y, g = blockIdx.x, tid = threadIdx.x;
  float lo = -kRange, w = kRange, floor_z = -INFINITY;
  if (!first) {
    const SplitState s = ws.state[r];
    if (s.phase == kDone) return;
    lo = s.lo;
    w = s.w;
    floor_z = s.floor_z;
  }
  float gmax;
  int argmax;
  row_max(ws.pmax + r * G, ws.parg + r * G, G, gmax, argmax);
  for (int i = tid; i < kBins; i += kSplitNT) {
    c[i] = 0;
    m[i] = 0ull;
  }
  __syncthreads();
  const T* row = logits + int64_t(r) * ld_;
  int v0, v1;
  chunk_range(V, G, g, v0, v1);
  const float sc = kBins / w, hi = lo + w;
  const bool top = hi >= 0.f;
  for (int i = v0 + tid; i < v1; i += kSplitNT) {
    float x[8];
    ld8(row, i, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float z = (x[j] - gmax) * inv_t;
      if (z >= lo && (z < hi || (top && z <= 0.f)) && z >= floor_z) {
        const int b = min(kBins - 1, (int)((z - lo) * sc));
        atomicAdd(&c[b], 1);
        atomicAdd(&m[b], static_cast<unsigned long long>(__expf(z) * kHistFix));
      }
    }
  }
  __syncthreads();
  int* oc = ws.hc + int64_t(r) * kBins;
  unsigned long long* om = ws.hm + int64_t(r) * kBins;
  for (int i = tid; i < kBins; i += kSplitNT)
    if (c[i] > 0) {  // only occupied bins: few atomics for concentrated rows
      atomicAdd(oc + i, c[i]);
      atomicAdd(om + i, m[i]);  // same 2^-40 scale as kFix
    }
}

__global__ __launch_bounds__(kSampNT) void split_resolve_kernel(int G, int top_k, float top_p,
                                                                bool need_p, int first_phase,
                                                                SplitWs ws) {
  __shared__ int hc[kBins];
  __shared__ float hm[kBins];
  __shared__ int tc[kSampNT];
  __shared__ float tm[kSampNT];
  __shared__ int sel;
  const int r = blockIdx.x, tid = threadIdx.x;
  SplitState s;
  if (first_phase != kDone) {  // first pass: fresh state
    s.tau = -kRange;
    s.lo = -kRange;
    s.w = kRange;
    s.floor_z = -INFINITY;
    s.above_m = 0.f;
    s.target = 0.f;
    s.above_c = 0;
    s.phase = first_phase;
  } else {
    s = ws.state[r];
    if (s.phase == kDone) return;
  }
  for (int b = tid; b < kBins; b += kSampNT) {  // read the row histogram, re-zero it for the next pass
    hc[b] = ws.hc[int64_t(r) * kBins + b];
    hm[b] = (float)((double)ws.hm[int64_t(r) * kBins + b] * (1.0 / kFix));
    ws.hc[int64_t(r) * kBins + b] = 0;
    ws.hm[int64_t(r) * kBins + b] = 0ull;
  }
  __syncthreads();
  suffix_scan(hc, hm, tc, tm);
  const float W = kRange / kBins;
  if (s.phase == kKCoarse) {
    const int kbin = find_bin_count(hc, top_k, &sel);
    s.above_c = kbin + 1 < kBins ? hc[kbin + 1] : 0;
    s.above_m = kbin + 1 < kBins ? hm[kbin + 1] : 0.f;
    s.lo = -kRange + kbin * W;
    s.w = W;
    s.floor_z = -INFINITY;
    s.phase = kKFine;
  } else if (s.phase == kKFine) {
    const int sb = find_bin_count(hc, top_k - s.above_c, &sel);
    s.tau = s.lo + sb * (W / kBins);
    const float total = s.above_m + hm[sb];
    s.phase = kDone;
    if (need_p) {
      const float target = top_p * total;
      if (s.above_m < target) {  // nucleus edge inside this same coarse bin
        const int sp = find_bin_mass(hm, target - s.above_m, &sel);
        s.tau = fmaxf(s.tau, s.lo + sp * (W / kBins));
      } else {  // edge in a higher coarse bin: coarse pass again above the top-k floor
        s.target = target;
        s.lo = -kRange;
        s.w = kRange;
        s.floor_z = s.tau;
        s.phase = kPCoarse;
      }
    }
  } else if (s.phase == kPCoarse) {
    if (first_phase == kPCoarse) s.target = top_p * hm[0];  // no top-k: total = whole row
    const int cb = find_bin_mass(hm, s.target, &sel);
    s.above_m = cb + 1 < kBins ? hm[cb + 1] : 0.f;
    s.lo = -kRange + cb * W;
    s.w = W;
    s.floor_z = s.tau;
    s.phase = kPFine;
  } else {  // kPFine
    const int sp = find_bin_mass(hm, s.target - s.above_m, &sel);
    s.tau = fmaxf(s.tau, s.lo + sp * (W / kBins));
    s.phase = kDone;
  }
  __syncthreads();
  if (tid == 0) ws.state[r] = s;
}

template <typename T>
__global__ __launch_bounds__(kSplitNT) void split_mass_kernel(const T* __restrict__ logits,
                                                              int64_t ld_, int V, int G,
                                                              float inv_t, bool has_tau,
                                                              SplitWs ws) {
  __shared__ float red[kSplitNT / 64];
  const int r = blockIdx.y, g = blockIdx.x, tid = threadIdx.x;
  float gmax;
  int argmax;
  row_max(ws.pmax + r * G, ws.parg + r * G, G, gmax, argmax);
  const float tau = has_tau ? ws.state[r].tau : -kRange;
  const T* row = logits + int64_t(r) * ld_;
  int v0, v1;
  chunk_range(V, G, g, v0, v1);
  float acc = 0.f;
  for (int i = v0 + tid; i < v1; i += kSplitNT) {
    float x[8];
    ld8(row, i, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float z = (x[j] - gmax) * inv_t;
      acc += z >= tau ? __expf(z) : 0.f;
    }
  }
  const float tot = block_sum<kSplitNT>(acc, red);
  if (tid == 0) ws.cmass[r * G + g] = tot;
}

template <typename T>
__global__ __launch_bounds__(kSplitNT) void split_pick_kernel(const T* __restrict__ logits,
                                                              int64_t ld_, int V, int G,
                                                              float inv_t, bool has_tau,
                                                              const int64_t* __restrict__ rng,
                                                              SplitWs ws,
                                                              int64_t* __restrict__ out) {
  __shared__ float tm[kSplitNT];
  __shared__ int ans;
  const int r = blockIdx.x, tid = threadIdx.x;
  float gmax;
  int argmax;
  row_max(ws.pmax + r * G, ws.parg + r * G, G, gmax, argmax);
  const float tau = has_tau ? ws.state[r].tau : -kRange;
  float cms[kSplitG];
  float total = 0.f;
#pragma unroll
  for (int g = 0; g < kSplitG; ++g) {
    cms[g] = ws.cmass[r * kSplitG + g];
    total += cms[g];
  }
  const float u = philox_uniform((uint64_t)rng[0], (uint64_t)r, (uint64_t)rng[1]) * total;
  // chunk holding u (every lane walks the G partials in the same order)
  int cg = -1;
  float base = 0.f, acc = 0.f;
#pragma unroll
  for (int g = 0; g < kSplitG; ++g) {
    const float cm = cms[g];
    if (cm > 0.f) {
      if (u < acc + cm) {
        cg = g;
        base = acc;
        break;
      }
      cg = g;  // u on a rounding gap past the last chunk: fall into the last non-empty one
      base = acc;
    }
    acc += cm;
  }
  if (tid == 0) ans = -1;
  const T* row = logits + int64_t(r) * ld_;
  float mine = 0.f;
  int s0 = 0, s1 = 0;
  if (cg >= 0) {
    int v0, v1;
    chunk_range(V, G, cg, v0, v1);
    const int n = (v1 - v0) * 8, per = (n + kSplitNT - 1) / kSplitNT;
    s0 = min(n, tid * per) + v0 * 8;
    s1 = min(n, tid * per + per) + v0 * 8;
    for (int v = s0; v < s1; ++v) {
      const float z = (ld(row, v) - gmax) * inv_t;
      mine += z >= tau ? __expf(z) : 0.f;
    }
  }
  tm[tid] = mine;
  __syncthreads();
  for (int o = 1; o < kSplitNT; o <<= 1) {
    const float add = tid >= o ? tm[tid - o] : 0.f;
    __syncthreads();
    tm[tid] += add;
    __syncthreads();
  }
  const float before = base + (tid > 0 ? tm[tid - 1] : 0.f);
  if (mine > 0.f && u >= before && u < base + tm[tid]) {
    float a = before;
    int pick = -1;
    for (int v = s0; v < s1; ++v) {
      const float z = (ld(row, v) - gmax) * inv_t;
      if (z >= tau) {
        a += __expf(z);
        pick = v;
        if (u < a) break;
      }
    }
    ans = pick;
  }
  __syncthreads();
  if (tid == 0) out[r] = ans >= 0 ? ans : argmax;  // u on a rounding gap: argmax
}

static bool split_enabled() {
  static const bool on = [] {
    const char* e = getenv("DLA_SAMPLER_SPLIT");
    return !(e && e[0] == '0');
  }();
  return on;
}

// chunks per row for the split sampler, 0 = use the single-block kernel
int sample_split_chunks(const void* logits, int64_t ld_, int64_t rows, int V, float inv_temp,
                        int top_k, float top_p, bool greedy) {
  const bool vec = V % 8 == 0 && ld_ % 8 == 0 && reinterpret_cast<uintptr_t>(logits) % 16 == 0;
  if (!split_enabled() || !vec || greedy || inv_temp <= 0.f || V < 32768 || rows > 65535)
    return 0;
  return kSplitG;
}
size_t sample_workspace_bytes(int64_t rows, int G) { return G > 0 ? split_ws_bytes(rows, G) : 0; }

template <typename T>
static void launch_split(const T* lg, int64_t ld_, int64_t rows, int V, int G, float inv_t,
                         int top_k, float top_p, const int64_t* rng, int64_t* out, void* wsp,
                         hipStream_t st) {
  const SplitWs ws = split_ws(wsp, rows, G);
  const dim3 grid(G, rows);
  const bool need_k = top_k > 0 && top_k < V, need_p = top_p < 1.f;
  split_max_kernel<T><<<grid, kSplitNT, 0, st>>>(lg, ld_, V, G, ws);
  const int passes = (need_k ? 2 : 0) + (need_p ? 2 : 0);
  for (int p = 0; p < passes; ++p) {
    split_hist_kernel<T><<<grid, kSplitNT, 0, st>>>(lg, ld_, V, G, inv_t, p == 0, ws);
    const int first_phase = p == 0 ? (need_k ? kKCoarse : kPCoarse) : kDone;
    split_resolve_kernel<<<rows, kSampNT, 0, st>>>(G, top_k, top_p, need_p, first_phase, ws);
  }
  split_mass_kernel<T><<<grid, kSplitNT, 0, st>>>(lg, ld_, V, G, inv_t, passes > 0, ws);
  split_pick_kernel<T><<<rows, kSplitNT, 0, st>>>(lg, ld_, V, G, inv_t, passes > 0, rng, ws, out);
}

void launch_sample_split(const void* logits, bool is_bf16, int64_t ld_, int64_t rows, int V,
                         int G, float inv_temp, int top_k, float top_p, const int64_t* rng,
                         int64_t* out, void* ws, hipStream_t st) {
  if (rows == 0) return;
  if (is_bf16)
    launch_split(static_cast<const bf16_t*>(logits), ld_, rows, V, G, inv_temp, top_k, top_p, rng,
                 out, ws, st);
  else
    launch_split(static_cast<const float*>(logits), ld_, rows, V, G, inv_temp, top_k, top_p, rng,
                 out, ws, st);
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
