// Skinny GEMM for the decode path: y[M, N] = x[M, K] @ W[N, K]^T with M <= 16 rows (the
// sampling batch), bf16 in/out, fp32 accumulate. Optionally the input is the fused gate|up GEMM
// output gu[M, 2K] and the kernel applies SwiGLU (silu(g) * u, rounded to bf16 exactly as the
// standalone swiglu kernel does) while staging it, so the MLP's down projection reads gu directly.
//
// Reference: every autoregressive step of HF `generate` in src/training/train_rlhf.py:115-121 and
// src/training/generate_teacher_data.py:60-80 runs these projections with a handful of rows.
//
// Why a hand-written kernel: at M <= 16 a GEMM is a weight stream (Llama-3-8B decode reads
// ~16 GB of weights per token) and the library's tiles for it ran at 2.2-4.9 TB/s on MI355X
// (profiles/r1_decode_v2_kernel_stats.md). The layout here is built for that stream:
//   * the workgroup stages its K-slice of x in LDS once (rows >= M are never read: those lanes
//     feed zeros to the MFMA);
//   * each wave owns 16 weight rows and walks its K-slice with 16-byte loads, 8 k-steps
//     (8 x 16 B per lane) in flight ahead of the MFMAs (v_mfma_f32_16x16x32_bf16: B fragment =
//     16 weight rows x 32 k, exactly what one 16-byte load per lane delivers);
//   * split-K over workgroups fills the 256 CUs for N = 4096; partial tiles go to an fp32
//     workspace and the last-arriving workgroup of a column (device-scope counter, reset by
//     that workgroup: no memset, graph-capture safe) sums them in a FIXED order: deterministic.
#include "common.h"

namespace dla {

namespace {

constexpr int kSkWaves = 4;           // waves per workgroup; each owns 16 output columns
constexpr int kSkCols = 16 * kSkWaves;  // output columns (weight rows) per workgroup
constexpr int kSkUnroll = 8;          // k-steps (32 each) of weight loads in flight per wave
constexpr int kSkChunk = 32 * kSkUnroll;

__device__ __forceinline__ f32x4 mfma16(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float silu_sk(float g) { return g * sigmoidf_(g); }

}  // namespace

// grid: (ceil(N / 64), S). LDS: M x (kc + 8) bf16 (row pad of 16 B keeps the 16-row fragment
// reads on distinct banks).
template <bool SWIGLU>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(
    const bf16_t* __restrict__ x, int64_t ldx, const bf16_t* __restrict__ W, int64_t ldw,
    bf16_t* __restrict__ y, int64_t ldy, float* __restrict__ ws, unsigned* __restrict__ counters,
    int M, int N, int K, int kc) {
  extern __shared__ __attribute__((aligned(16))) bf16_t xs[];
  const int S = gridDim.y;
  const int s = blockIdx.y;
  const int k0 = s * kc;
  const int klen = min(kc, K - k0);
  const int ldl = kc + 8;

  // ---- stage x[:, k0:k0+klen] (or swiglu(gu) of it) into LDS, 16 B per thread-step
  const int vecs = klen >> 3;
  for (int i = threadIdx.x; i < M * vecs; i += blockDim.x) {
    const int m = i / vecs, c = (i - m * vecs) << 3;
    bf16x8 v;
    if constexpr (SWIGLU) {
      const bf16x8 g = load_bf16x8(x + m * ldx + k0 + c);
      const bf16x8 u = load_bf16x8(x + m * ldx + K + k0 + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = f2bf(silu_sk(bf2f(g[j])) * bf2f(u[j]));
    } else {
      v = load_bf16x8(x + m * ldx + k0 + c);
    }
    store_bf16x8(xs + m * ldl + c, v);
  }
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = blockIdx.x * kSkCols + wave * 16;
  const int r = lane & 15, q = lane >> 4;  // fragment row (m for A, n for B), k quarter
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (n0 < N) {
    const bf16_t* wrow = W + static_cast<int64_t>(n0 + r) * ldw + k0 + q * 8;
    const bf16_t* xrow = xs + r * ldl + q * 8;
    const bool arow = r < M;
    s16x8 b[kSkUnroll];
#pragma unroll
    for (int u = 0; u < kSkUnroll; ++u)
      b[u] = __builtin_bit_cast(s16x8, load_bf16x8(wrow + u * 32));
    for (int kk = 0; kk < klen; kk += kSkChunk) {
      s16x8 nb[kSkUnroll];
      const bool more = kk + kSkChunk < klen;
      if (more) {
#pragma unroll
        for (int u = 0; u < kSkUnroll; ++u)
          nb[u] = __builtin_bit_cast(s16x8, load_bf16x8(wrow + kk + kSkChunk + u * 32));
      }
#pragma unroll
      for (int u = 0; u < kSkUnroll; ++u) {
        s16x8 a = {0, 0, 0, 0, 0, 0, 0, 0};
        if (arow) a = __builtin_bit_cast(s16x8, load_bf16x8(xrow + kk + u * 32));
        acc = mfma16(a, b[u], acc);
      }
      if (more) {
#pragma unroll
        for (int u = 0; u < kSkUnroll; ++u) b[u] = nb[u];
      }
    }
  }

  // ---- epilogue. Lane holds C[m = 4q + i][n = n0 + r], i = 0..3.
  const int n = n0 + r;
  if (S == 1) {
    if (n < N) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = 4 * q + i;
        if (m < M) y[m * ldy + n] = f2bf(acc[i]);
      }
    }
    return;
  }
  // split-K: partial tile -> ws[s][m][n]; the last workgroup of this column block reduces
  if (n < N) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = 4 * q + i;
      if (m < M) ws[(static_cast<int64_t>(s) * M + m) * N + n] = acc[i];
    }
  }
  __threadfence();
  __syncthreads();
  __shared__ unsigned last;
  if (threadIdx.x == 0) {
    const unsigned prev = atomicAdd(&counters[blockIdx.x], 1u);
    last = (prev == static_cast<unsigned>(S - 1));
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  // reduce this block's 64 columns x M rows in split order (fixed -> deterministic)
  const int nb0 = blockIdx.x * kSkCols;
  for (int i = threadIdx.x; i < M * kSkCols; i += blockDim.x) {
    const int m = i / kSkCols, nn = nb0 + (i - m * kSkCols);
    if (nn >= N) continue;
    float t = 0.f;
    for (int ss = 0; ss < S; ++ss)
      t += __hip_atomic_load(ws + (static_cast<int64_t>(ss) * M + m) * N + nn, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    y[m * ldy + nn] = f2bf(t);
  }
  if (threadIdx.x == 0) counters[blockIdx.x] = 0u;  // re-arm for the next launch
}

int skinny_splits(int M, int N, int K) {
  // smallest split count (K-slices a multiple of kSkChunk) that gives >= 512 workgroups, with the
  // x slice within 64 KB of LDS (two workgroups per CU)
  const int nb = (N + kSkCols - 1) / kSkCols;
  const int chunks = K / kSkChunk;
  int best = chunks;
  for (int s = 1; s <= chunks; ++s) {
    if (chunks % s) continue;
    const int kc = K / s;
    if (static_cast<int64_t>(M) * (kc + 8) * 2 > 65536) continue;
    best = s;
    if (static_cast<int64_t>(nb) * s >= 512) break;
  }
  return best;
}

size_t skinny_lds_bytes(int M, int kc) { return static_cast<size_t>(M) * (kc + 8) * sizeof(bf16_t); }

void launch_skinny_gemm(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                        int64_t ldy, float* ws, unsigned* counters, int M, int N, int K, int S,
                        bool swiglu, hipStream_t st) {
  const int kc = K / S;
  dim3 grid((N + kSkCols - 1) / kSkCols, S);
  const size_t lds = skinny_lds_bytes(M, kc);
  if (swiglu)
    skinny_gemm_kernel<true><<<grid, 64 * kSkWaves, lds, st>>>(x, ldx, W, ldw, y, ldy, ws,
                                                                counters, M, N, K, kc);
  else
    skinny_gemm_kernel<false><<<grid, 64 * kSkWaves, lds, st>>>(x, ldx, W, ldw, y, ldy, ws,
                                                                 counters, M, N, K, kc);
}

}  // namespace dla
