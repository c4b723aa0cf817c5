// Skinny GEMM for the decode path: y[M, N] = x[M, K] @ W[N, K]^T with M <= 16 rows (the
// sampling batch), bf16 in/out, fp32 accumulate. Optionally the input is the fused gate|up GEMM
// output gu[M, 2K] and the kernel applies SwiGLU (silu(g) * u, rounded to bf16 exactly as the
// standalone swiglu kernel does) while staging it, so the MLP's down projection reads gu directly.
//
// Reference: every autoregressive step of HF `generate` in src/training/train_rlhf.py:115-121 and
// src/training/generate_teacher_data.py:60-80 runs these projections with a handful of rows.
//
// Why a hand-written kernel: at M <= 16 a GEMM is a weight stream (Llama-3-8B decode reads
// ~16 GB of weights per token) and the library's tiles for it ran at 2.2-4.9 TB/s in a real
// decode step on MI355X. The layout here is built for that stream (measured results and the
// split-K caveat: profiles/r1_decode_skinny.md):
//   * the workgroup stages its K-slice of x in LDS once (rows >= M are never read: those lanes
//     feed zeros to the MFMA);
//   * each wave owns 16 weight rows and walks its K-slice with 16-byte loads, 8 k-steps
//     (8 x 16 B per lane) in flight ahead of the MFMAs (v_mfma_f32_16x16x32_bf16: B fragment =
//     16 weight rows x 32 k, exactly what one 16-byte load per lane delivers);
//   * split-K over workgroups fills the 256 CUs for N = 4096; partial tiles go to an fp32
//     workspace and the last-arriving workgroup of a column (agent-scope release/acquire +
//     ticket counter, re-armed by that workgroup: no memset, graph-capture safe) sums them in a
//     FIXED order: deterministic.
#include "common.h"
#include "skinny_params.h"
#include "skinny_ks.h"

#include <cstdlib>

namespace dla {

namespace {

constexpr int kSkWaves = 8;           // waves per workgroup; each owns 16 output columns
constexpr int kSkCols = 16 * kSkWaves;  // output columns (weight rows) per workgroup
constexpr int kSkUnroll = 8;          // k-steps (32 each) of weight loads in flight per wave
constexpr int kSkChunk = 32 * kSkUnroll;

// Non-temporal loads on the TILED decode weight streams (each byte read once per step by one CU):
// 3.54 vs 3.70 ms/token at B=8 (profiles/r3_decode_tiled.md). On the row-major layout nt lost
// (4.31 vs 4.19 ms/token: the weights rotated past the Infinity Cache), so the row-major kernels
// use default-policy loads. (Its DLA_DECODE_NT A/B switch was removed in round 6.)
static bool decode_nt() { return true; }

}  // namespace

// grid: (ceil(N / 128), S), 8 waves. LDS: M x (kc + 8) bf16 (row pad of 16 B keeps the 16-row fragment
// reads on distinct banks).
// GLU_OUT (decode gate|up projection): W is [gate; up] (2F rows) and the output is
// m = silu(gate) * up [M, F]. Block b's waves 0-3 take gate rows [64b, 64b + 64), waves 4-7 the
// matching up rows F + [64b, 64b + 64); the tile is exchanged through LDS and SwiGLU applied in
// the epilogue (after the same bf16 rounding of gate/up as the unfused path): no gu round trip,
// no separate swiglu launch.
// (A NORM variant that formed s = x + res and RMSNorm(s) inside this kernel's staging measured
// 4.39 vs 4.28 ms/token -- 224 workgroups each re-deriving the row norm -- and was removed.)

// Decode-layer fusion of the residual add + RMSNorm across two launches (no norm launch):
//   RES (producer, the o / down projections): the epilogue writes the new residual stream
//       s = bf16(bf16(x W^T) + res) instead of the projection, plus per-(row, workgroup) partial
//       sums of s^2 over the workgroup's 16 columns (fixed order) into ssq_out [16][gridDim.x];
//   NIN (consumer, the qkv / gate|up projections of the next sublayer): RMSNorm(s) W^T =
//       rstd[m] * (s (W o w)^T) -- the per-row rsqrt(mean(s^2) + eps) factors out of the GEMM and
//       the norm weight w is folded into a cached copy of W (ops/decode.py). So the consumer is a
//       plain GEMM on s whose epilogue scales row m by rstd[m], computed from the producer's
//       partials (prefetched at kernel start, reduced in fixed order at the end): the weight
//       stream starts at once, and no per-element normalisation is needed.
// Deterministic (eager == graph); the rounding differs from the separate-norm path (h is never
// rounded to bf16; W o w is), so the two agree to bf16 accuracy, not bitwise.

template <bool SWIGLU, bool GLU_OUT = false, bool NTW = false, bool NPRE = false, bool TW = false>
__global__ __launch_bounds__(64 * kSkWaves) void skinny_gemm_kernel(
    const bf16_t* __restrict__ x, int64_t ldx, const bf16_t* __restrict__ W, int64_t ldw,
    bf16_t* __restrict__ y, int64_t ldy, float* __restrict__ ws, unsigned* __restrict__ counters,
    int M, int N, int K, int kc, KsFuse fz = KsFuse{}) {
  extern __shared__ __attribute__((aligned(16))) bf16_t xs[];
  // NPRE: per-row rstd from the producer's partial sums (see KsFuse)
  __shared__ __attribute__((aligned(16))) float rstd_p[16];
  const int S = gridDim.y;
  const int s = blockIdx.y;
  const int k0 = s * kc;
  const int klen = min(kc, K - k0);
  const int ldl = kc + 8;

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int F = N >> 1;
  const int n0 = GLU_OUT ? (wave < 4 ? 0 : F) + blockIdx.x * 64 + (wave & 3) * 16
                         : blockIdx.x * kSkCols + wave * 16;
  const int r = lane & 15, q = lane >> 4;  // fragment row (m for A, n for B), k quarter
  const bool active = n0 < N;
  // TW: W in the tiled layout [N/16, K/32, 4, 16, 8] (skinny64.hip): wp(k) = k-offset k of this lane
  const bf16_t* wrow = TW ? W + static_cast<int64_t>(active ? n0 >> 4 : 0) * 16 * K + (k0 >> 5) * 512 + lane * 8
                          : W + static_cast<int64_t>(active ? n0 + r : 0) * ldw + k0 + q * 8;
  auto wp = [&](int kk) { return TW ? wrow + (kk >> 5) * 512 : wrow + kk; };

  // the first two weight chunks are in flight before x is staged (independent of LDS)
  const int nchunks = klen / kSkChunk;
  s16x8 b0[kSkUnroll], b1[kSkUnroll];
  if (active) {
#pragma unroll
    for (int u = 0; u < kSkUnroll; ++u) b0[u] = load_w<NTW>(wp(u * 32));
    if (nchunks > 1) {
#pragma unroll
      for (int u = 0; u < kSkUnroll; ++u) b1[u] = load_w<NTW>(wp(kSkChunk + u * 32));
    }
  }

  KsPart part{};
  if constexpr (NPRE) part = ks_part_load(fz, M, wave, lane);  // reduced in the epilogue
  // ---- stage x[:, k0:k0+klen] (or swiglu(gu) of it) into LDS: 8 independent 16-byte loads per
  // thread per pass (all issued before the first LDS store, so the pass costs one latency)
  const int vecs = klen >> 3;
  const int total = M * vecs;
  constexpr int NT = 64 * kSkWaves;
  for (int base = 0; base < total; base += 8 * NT) {
    bf16x8 v[8];
    if constexpr (SWIGLU) {
      bf16x8 gg[8], uu[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = base + j * NT + threadIdx.x;
        if (i < total) {
          const int m = i / vecs, c = (i - m * vecs) << 3;
          gg[j] = load_bf16x8(x + m * ldx + k0 + c);
          uu[j] = load_bf16x8(x + m * ldx + K + k0 + c);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[j][e] = f2bf(silu_sk(bf2f(gg[j][e])) * bf2f(uu[j][e]));
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = base + j * NT + threadIdx.x;
        if (i < total) {
          const int m = i / vecs, c = (i - m * vecs) << 3;
          v[j] = load_bf16x8(x + m * ldx + k0 + c);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = base + j * NT + threadIdx.x;
      if (i < total) {
        const int m = i / vecs, c = (i - m * vecs) << 3;
        store_bf16x8(xs + m * ldl + c, v[j]);
      }
    }
  }
  __syncthreads();

  // ---- main loop: ping-pong register buffers, the next chunk's 8 loads stay in flight while
  // the current chunk's 8 MFMAs run (no wait on the newest loads until they are consumed)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (active) {
    const bf16_t* xrow = xs + r * ldl + q * 8;
    const bool arow = r < M;
    auto compute = [&](const s16x8* b, int kk) {
#pragma unroll
      for (int u = 0; u < kSkUnroll; ++u) {
        s16x8 a = {0, 0, 0, 0, 0, 0, 0, 0};
        if (arow) a = __builtin_bit_cast(s16x8, load_bf16x8(xrow + kk + u * 32));
        acc = mfma16(a, b[u], acc);
      }
    };
    // two register sets in a ring: compute chunk c while chunk c+1 is in flight, then refill
    for (int c = 0; c < nchunks; c += 2) {
      compute(b0, c * kSkChunk);
      if (c + 2 < nchunks) {
#pragma unroll
        for (int u = 0; u < kSkUnroll; ++u)
          b0[u] = load_w<NTW>(wp((c + 2) * kSkChunk + u * 32));
      }
      if (c + 1 < nchunks) {
        compute(b1, (c + 1) * kSkChunk);
        if (c + 3 < nchunks) {
#pragma unroll
          for (int u = 0; u < kSkUnroll; ++u)
            b1[u] = load_w<NTW>(wp((c + 3) * kSkChunk + u * 32));
        }
      }
    }
  }

  // ---- epilogue. Lane holds C[m = 4q + i][n = n0 + r], i = 0..3.
  const int n = n0 + r;
  if constexpr (GLU_OUT) {
    __shared__ float glu[2][16][64];  // [gate|up][m][column within the block]
    const int half = wave >> 2, col = (wave & 3) * 16 + r;
    if constexpr (NPRE) {  // RMSNorm row factor of the folded-weight GEMM (see KsFuse)
      ks_rstd(part, fz, M, K, wave, lane, rstd_p);
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] *= (4 * q + i < M) ? rstd_p[4 * q + i] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) glu[half][4 * q + i][col] = bf2f(f2bf(acc[i]));
    __syncthreads();
    for (int i = threadIdx.x; i < M * 64; i += blockDim.x) {
      const int m = i >> 6, c = i & 63, nn = blockIdx.x * 64 + c;
      if (nn < F) y[m * ldy + nn] = f2bf(silu_sk(glu[0][m][c]) * glu[1][m][c]);
    }
    return;
  }
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
  // split-K: partial tile -> fp32 slab ws[s][m][n] (plain stores); then one agent-scope release
  // + ticket per workgroup, and one acquire in the last arriver, which sums the S slabs of its 64
  // columns in split order (fixed -> deterministic) with plain loads
  if (n < N) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = 4 * q + i;
      if (m < M) ws[(static_cast<int64_t>(s) * M + m) * N + n] = acc[i];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave's slab stores are complete; the x image in LDS is dead
  unsigned* flag = reinterpret_cast<unsigned*>(xs);
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(&counters[blockIdx.x], 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = (prev == static_cast<unsigned>(S - 1)) ? 1u : 0u;
  }
  __syncthreads();
  if (flag[0] == 0u) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    counters[blockIdx.x] = 0u;  // re-arm for the next launch (kernel boundary orders it)
  }
  __syncthreads();
  const int nb0 = blockIdx.x * kSkCols;
  for (int i = threadIdx.x; i < M * kSkCols; i += blockDim.x) {
    const int m = i / kSkCols, nn = nb0 + (i - m * kSkCols);
    if (nn >= N) continue;
    const float* p = ws + static_cast<int64_t>(m) * N + nn;
    const int64_t slab = static_cast<int64_t>(M) * N;
    float t = 0.f;
    for (int ss = 0; ss < S; ++ss) t += p[ss * slab];
    y[m * ldy + nn] = f2bf(t);
  }
}

int skinny_splits(int M, int N, int K) {
  // Column blocks >= 128 (8 waves each: >= 4 waves per CU): no split (an in-kernel split-K combine costs each
  // workgroup an agent-scope release, measured 1.5-2x slower at 900-4000 workgroups). Otherwise
  // the smallest split count (K-slices a multiple of kSkChunk) giving >= `target` workgroups
  // (DLA_SKINNY_WG, default 256: one 8-wave workgroup per CU).
  static const int target = [] {
    const char* e = getenv("DLA_SKINNY_WG");
    return e ? atoi(e) : 256;
  }();
  const int nb = (N + kSkCols - 1) / kSkCols;
  if (nb >= 128) return 1;
  const int chunks = K / kSkChunk;
  int best = chunks;
  for (int s = 1; s <= chunks; ++s) {
    if (chunks % s) continue;
    const int kc = K / s;
    if (static_cast<int64_t>(M) * (kc + 8) * 2 > 65536) continue;
    best = s;
    if (static_cast<int64_t>(nb) * s >= target) break;
  }
  return best;
}

size_t skinny_lds_bytes(int M, int kc) { return static_cast<size_t>(M) * (kc + 8) * sizeof(bf16_t); }

template <bool NT>
void launch_skinny_gemm_t(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                          int64_t ldy, float* ws, unsigned* counters, int M, int N, int K, int S,
                          bool swiglu, bool glu_out, hipStream_t st) {
  const int kc = K / S;
  dim3 grid((N + kSkCols - 1) / kSkCols, S);
  const size_t lds = skinny_lds_bytes(M, kc);
  static bool attr_set = [] {  // S = 1 at K = 4096 stages up to 16 x 4104 bf16 (> 64 KB default)
    hipFuncSetAttribute(reinterpret_cast<const void*>(&skinny_gemm_kernel<false, false, NT>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&skinny_gemm_kernel<true, false, NT>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    // the GLU variant also holds an 8 KB static exchange tile: dynamic + static <= 160 KB
    hipFuncSetAttribute(reinterpret_cast<const void*>(&skinny_gemm_kernel<false, true, NT>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024);
    (void)hipGetLastError();  // never leave a sticky error for the caller's next launch check
    return true;
  }();
  (void)attr_set;
  if (glu_out) {  // N = 2F weight rows -> F outputs, 64 per block, never split
    dim3 g2(N / 2 / 64, 1);
    skinny_gemm_kernel<false, true, NT><<<g2, 64 * kSkWaves, skinny_lds_bytes(M, K), st>>>(
        x, ldx, W, ldw, y, ldy, ws, counters, M, N, K, K);
    return;
  }
  if (swiglu)
    skinny_gemm_kernel<true, false, NT><<<grid, 64 * kSkWaves, lds, st>>>(
        x, ldx, W, ldw, y, ldy, ws, counters, M, N, K, kc);
  else
    skinny_gemm_kernel<false, false, NT><<<grid, 64 * kSkWaves, lds, st>>>(
        x, ldx, W, ldw, y, ldy, ws, counters, M, N, K, kc);
}

void launch_skinny_gemm(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                        int64_t ldy, float* ws, unsigned* counters, int M, int N, int K, int S,
                        bool swiglu, bool glu_out, hipStream_t st) {
  launch_skinny_gemm_t<false>(x, ldx, W, ldw, y, ldy, ws, counters, M, N, K, S, swiglu, glu_out, st);
}

// Narrow outputs (N <= ~16K: qkv, o, down at Llama-3-8B): ONE workgroup per 16 output columns,
// its 8 waves split K among themselves (wave w: k in [w K/8, (w+1) K/8)) and reduce their
// 16 x 16 accumulators through LDS. No cross-workgroup combine (whose agent-scope release made
// the split-K form slow inside a real decode step), 8 waves per CU for N = 4096. x is read as
// MFMA A fragments straight from global memory (tiny, L2-resident), in the same two-set ring as
// the weights.
// GLU (decode gate|up with the SwiGLU epilogue, W = [gate; up], 2F rows -> m [M, F]): the
// workgroup owns 16 features; waves 0-3 take the gate rows, waves 4-7 the matching up rows, each
// over a quarter of K (F / 16 workgroups).
// MT = row tiles of 16 (M <= 16 MT): every weight fragment feeds MT MFMAs, one per 16 rows of x
// (larger decode batches, e.g. the reference's 64 rollouts per RLHF step on one GPU); UNR k-steps
// per ring slot (4 at MT = 1; 2 above, which keeps the x fragments at ~110 VGPRs for MT = 4, four
// waves per SIMD).
template <int DEPTH, bool NT, bool GLU, int MT = 1, int UNR = kKsUnroll, bool RES = false, bool NIN = false,
          bool TW = false, bool F8 = false>
__global__ __launch_bounds__(512) void skinny_ksplit_kernel(
    const bf16_t* __restrict__ x, int64_t ldx, const bf16_t* __restrict__ W, int64_t ldw,
    bf16_t* __restrict__ y, int64_t ldy, int M, int N, int K, KsFuse fz = KsFuse{}) {
  ks_body<DEPTH, NT, GLU, MT, UNR, RES, NIN, TW, false, F8>(blockIdx.x, gridDim.x, x, ldx, W, ldw, y, ldy, M,
                                                             N, K, fz);
}

// fused decode-layer launches (KsFuse): the residual-producing projection and the
// norm-consuming qkv projection on the in-workgroup split-K kernel, the gate|up GLU on the LDS
// kernel. M <= 16.
// ks_body's branch-free ring (KsFuse::straight) on every shape it covers; its A/B switch went
// in round 6 (3.557 / 3.554 vs 3.581 / 3.569 ms/token at B = 8, profiles/r5_decode_fp8.md)
static int ks_straight() { return 1; }

template <bool TW, bool NT, bool F8 = false>
static void launch_ks_fused_t(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                              int64_t ldy, int M, int N, int K, const KsFuse& fz, bool res, bool nin,
                              hipStream_t st) {
  static const int deep_k = [] {
    const char* e = getenv("DLA_SKINNY_DEEP_K");
    return e ? atoi(e) : 8192;
  }();
  const int nb = N / 16;
  const bool deep = K >= deep_k;
  KsFuse f = fz;
  f.straight = ks_straight();
#define DLA_KSF(D, R, NI) skinny_ksplit_kernel<D, NT, false, 1, kKsUnroll, R, NI, TW, F8><<<nb, 512, 0, st>>>(x, ldx, W, ldw, y, ldy, M, N, K, f)
  if (res && nin) {
    if (deep) DLA_KSF(4, true, true); else DLA_KSF(2, true, true);
  } else if (res) {
    if (deep) DLA_KSF(4, true, false); else DLA_KSF(2, true, false);
  } else if (nin) {
    if (deep) DLA_KSF(4, false, true); else DLA_KSF(2, false, true);
  } else {
    if (deep) DLA_KSF(4, false, false); else DLA_KSF(2, false, false);
  }
#undef DLA_KSF
}

// tiled: W in the tiled layout (ldw unused)
void launch_skinny_ks_fused(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                            int64_t ldy, int M, int N, int K, const KsFuse& fz, bool res, bool nin,
                            bool tiled, hipStream_t st) {
  // DLA_DECODE_NT=1: non-temporal weight loads on the tiled stream (A/B)
  if (tiled && decode_nt()) launch_ks_fused_t<true, true>(x, ldx, W, ldw, y, ldy, M, N, K, fz, res, nin, st);
  else if (tiled) launch_ks_fused_t<true, false>(x, ldx, W, ldw, y, ldy, M, N, K, fz, res, nin, st);
  else launch_ks_fused_t<false, false>(x, ldx, W, ldw, y, ldy, M, N, K, fz, res, nin, st);
}

// fp8 weights (e4m3 tiled copy + per-row scales in fz.wscale, ks_body F8): the o / down / qkv
// projections of the decode layer at half the weight bytes. The ring keeps the bf16 kernel's
// chunk count in flight, i.e. half its bytes: a 4-deep ring everywhere.
void launch_skinny_ks_fused_f8(const bf16_t* x, int64_t ldx, const uint8_t* W8, bf16_t* y, int64_t ldy,
                               int M, int N, int K, const KsFuse& fz, bool res, bool nin, hipStream_t st) {
  const bf16_t* W = reinterpret_cast<const bf16_t*>(W8);
  const int nb = N / 16;
  // DLA_KS_F8_DEPTH (2 or 4): ring depth. Graph decode, Llama-3-8B B=8, same box: 2.62 ms/token
  // at depth 2 vs 2.73 at 4 (fewer VGPRs, more resident waves beat more bytes in flight per wave)
  static const int depth = [] {
    const char* e = getenv("DLA_KS_F8_DEPTH");
    return (e && atoi(e) == 4) ? 4 : 2;
  }();
  KsFuse f = fz;
  f.straight = ks_straight();
#define DLA_KSF8(D, NTV, R, NI) skinny_ksplit_kernel<D, NTV, false, 1, kKsUnroll, R, NI, true, true><<<nb, 512, 0, st>>>(x, ldx, W, K, y, ldy, M, N, K, f)
#define DLA_KSF8_NT(D)                           \
  if (decode_nt()) {                             \
    if (res && nin) DLA_KSF8(D, true, true, true);   \
    else if (res) DLA_KSF8(D, true, true, false);    \
    else if (nin) DLA_KSF8(D, true, false, true);    \
    else DLA_KSF8(D, true, false, false);            \
  } else {                                       \
    if (res && nin) DLA_KSF8(D, false, true, true);  \
    else if (res) DLA_KSF8(D, false, true, false);   \
    else if (nin) DLA_KSF8(D, false, false, true);   \
    else DLA_KSF8(D, false, false, false);           \
  }
  if (depth == 2) {
    DLA_KSF8_NT(2)
  } else {
    DLA_KSF8_NT(4)
  }
#undef DLA_KSF8_NT
#undef DLA_KSF8
}

template <bool TW, bool NT>
static void launch_glu_normin_t(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                                int64_t ldy, int M, int N, int K, const KsFuse& fz, hipStream_t st) {
  static bool attr_set = [] {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&skinny_gemm_kernel<false, true, NT, true, TW>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    (void)hipGetLastError();
    return true;
  }();
  (void)attr_set;
  dim3 g2(N / 2 / 64, 1);
  skinny_gemm_kernel<false, true, NT, true, TW><<<g2, 64 * kSkWaves, skinny_lds_bytes(M, K), st>>>(
      x, ldx, W, ldw, y, ldy, nullptr, nullptr, M, N, K, K, fz);
}

void launch_skinny_glu_normin(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                              int64_t ldy, int M, int N, int K, const KsFuse& fz, bool tiled,
                              hipStream_t st) {
  if (tiled && decode_nt()) launch_glu_normin_t<true, true>(x, ldx, W, ldw, y, ldy, M, N, K, fz, st);
  else if (tiled) launch_glu_normin_t<true, false>(x, ldx, W, ldw, y, ldy, M, N, K, fz, st);
  else launch_glu_normin_t<false, false>(x, ldx, W, ldw, y, ldy, M, N, K, fz, st);
}

// Decode gate|up (M <= 16) over an INTERLEAVED tiled weight (ops/decode.py `glu_weight`): tile t
// (16 rows) holds gate rows 8t .. 8t+7 (r < 8) and the matching up rows F + 8t .. (r >= 8), the RMSNorm
// weight folded in. One wave per tile, so a lane's gate and up sums meet by one lane swap
// (lane ^ 8) -- no LDS exchange -- and the workgroup size is free: 7 waves give exactly 256
// workgroups at Llama-3-8B (F = 14336: 1792 tiles), where the 8-wave gate|up kernel
// (skinny_gemm_kernel GLU_OUT) runs 224 and leaves 32 CUs idle. Same K order, rstd and bf16
// rounding as that kernel: bitwise the same output.
// F8: Wt is the e4m3 interleaved tiled copy [2F/16, K/64, 64, 16 B] (ks_body F8 layout) and
// fz.wscale the per-row scales in the same interleaved row order; one 1-KB wave load feeds two
// k-steps, so a ring slot of kSkUnroll k-steps is kSkUnroll / 2 loads.
template <int DEPTH, bool F8 = false>
__global__ __launch_bounds__(512) void skinny_glu_il_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                           const bf16_t* __restrict__ Wt,
                                                           bf16_t* __restrict__ y, int64_t ldy, int M,
                                                           int ntiles, int K, KsFuse fz) {
  extern __shared__ __attribute__((aligned(16))) bf16_t xs[];
  __shared__ float rstd_s[16];
  const int nwv = blockDim.x >> 6;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int t = blockIdx.x * nwv + wave;
  const bool active = t < ntiles;
  const int ldl = K + 8;
  const bf16_t* wrow = Wt + static_cast<int64_t>(active ? t : 0) * 16 * K + lane * 8;
  const uint8_t* wrow8 = reinterpret_cast<const uint8_t*>(Wt) + static_cast<int64_t>(active ? t : 0) * 16 * K +
                         lane * 16;
  constexpr int UB = F8 ? kSkUnroll / 2 : kSkUnroll;  // wave loads per ring slot
  const int nchunks = K / kSkChunk;
  // DEPTH chunks of kSkUnroll k-steps in flight (a ring of register sets)
  s16x8 b[DEPTH][F8 ? 1 : kSkUnroll];
  ks_u32x4 b8[DEPTH][F8 ? UB : 1];
  auto wload = [&](int j, int c) {
    if constexpr (F8) {
#pragma unroll
      for (int u = 0; u < UB; ++u) b8[j][u] = *reinterpret_cast<const ks_u32x4*>(wrow8 + (c * UB + u) * 1024);
    } else {
#pragma unroll
      for (int u = 0; u < kSkUnroll; ++u)
        b[j][u] = __builtin_bit_cast(s16x8, load_bf16x8(wrow + (c * kSkUnroll + u) * 512));
    }
  };
  if (active) {
#pragma unroll
    for (int j = 0; j < DEPTH; ++j)
      if (j < nchunks) wload(j, j);
  }
  // this wave's rows' norm partials (rows wave, wave + nwv, ...: 4 cover M <= 16 at >= 4 waves),
  // reduced after the main loop
  float pv[4][8];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int m = wave + rr * nwv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = lane + 64 * j;
      pv[rr][j] = (m < M && i < fz.nbp) ? fz.ssq_in[m * fz.nbp + i] : 0.f;
    }
  }
  // stage x [M, K] into LDS, 4 independent 16-byte loads per thread per pass
  const int vecs = K >> 3, total = M * vecs, nthr = blockDim.x;
  for (int base = 0; base < total; base += 4 * nthr) {
    bf16x8 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = base + j * nthr + threadIdx.x;
      if (i < total) {
        const int m = i / vecs, c = (i - m * vecs) << 3;
        v[j] = load_bf16x8(x + m * ldx + c);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = base + j * nthr + threadIdx.x;
      if (i < total) {
        const int m = i / vecs, c = (i - m * vecs) << 3;
        store_bf16x8(xs + m * ldl + c, v[j]);
      }
    }
  }
  __syncthreads();
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (active) {
    const bf16_t* xrow = xs + r * ldl + q * 8;
    const bool arow = r < M;
    auto compute = [&](int j, int kk) {
#pragma unroll
      for (int u = 0; u < kSkUnroll; ++u) {
        s16x8 a = {0, 0, 0, 0, 0, 0, 0, 0};
        if (arow) a = __builtin_bit_cast(s16x8, load_bf16x8(xrow + kk + u * 32));
        s16x8 bu;
        if constexpr (F8) {
          const ks_u32x4 wv = b8[j][u >> 1];
          bu = (u & 1) ? f8x8_to_bf16(wv[2], wv[3]) : f8x8_to_bf16(wv[0], wv[1]);
        } else {
          bu = b[j][u];
        }
        acc = mfma16(a, bu, acc);
      }
    };
    for (int c0 = 0; c0 < nchunks; c0 += DEPTH) {
#pragma unroll
      for (int j = 0; j < DEPTH; ++j) {
        const int c = c0 + j;
        if (c < nchunks) {
          compute(j, c * kSkChunk);
          if (c + DEPTH < nchunks) wload(j, c + DEPTH);
        }
      }
    }
  }
  // rstd per row: in-lane sum in order, then the butterfly (as ks_rstd)
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int m = wave + rr * nwv;
    float tt = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) tt += pv[rr][j];
    tt = wave_sum(tt);
    if (lane == 0 && m < M && m < 16) rstd_s[m] = rsqrtf(tt / static_cast<float>(K) + fz.eps);
  }
  __syncthreads();
  if (!active) return;
  // lane holds C[m = 4q + i][row r of the tile]: gate (r < 8) and up (r >= 8) of feature 8t + (r & 7)
  const float wsc = F8 ? fz.wscale[16 * t + r] : 1.f;  // this lane's weight row (interleaved order)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = 4 * q + i;
    const float v = bf2f(f2bf((F8 ? acc[i] * wsc : acc[i]) * (m < M ? rstd_s[m] : 0.f)));
    const float o = __shfl_xor(v, 8, 64);
    if (r < 8 && m < M) y[m * ldy + 8 * t + r] = f2bf(silu_sk(v) * o);
  }
}

// gate|up over the interleaved tiled weight (2F rows -> [M, F]); waves per workgroup: the largest
// of 8..4 dividing the tile count with >= 256 workgroups, else 8
template <int DEPTH, bool F8 = false>
static void launch_glu_il_d(const bf16_t* x, int64_t ldx, const bf16_t* Wt, bf16_t* y, int64_t ldy, int M,
                            int ntiles, int K, const KsFuse& fz, int w, hipStream_t st) {
  static bool attr_set = [] {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&skinny_glu_il_kernel<DEPTH, F8>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    (void)hipGetLastError();
    return true;
  }();
  (void)attr_set;
  skinny_glu_il_kernel<DEPTH, F8><<<(ntiles + w - 1) / w, 64 * w, skinny_lds_bytes(M, K), st>>>(
      x, ldx, Wt, y, ldy, M, ntiles, K, fz);
}

// fp8 gate|up (interleaved e4m3 tiled copy, fz.wscale): the ring keeps 4 slots of half-size loads
void launch_skinny_glu_il_f8(const bf16_t* x, int64_t ldx, const uint8_t* Wt8, bf16_t* y, int64_t ldy,
                             int M, int N, int K, const KsFuse& fz, hipStream_t st) {
  const int ntiles = N / 16;
  int w = 8;
  for (int c : {8, 7, 6, 5, 4}) {
    if (ntiles % c == 0 && ntiles / c >= 256) { w = c; break; }
  }
  // DLA_GLU_IL_F8_DEPTH (2, 3 or 4): ring depth; same A/B: 2.712 / 2.710 / 2.729 ms/token
  static const int depth = [] {
    const char* e = getenv("DLA_GLU_IL_F8_DEPTH");
    const int d = e ? atoi(e) : 3;
    return d < 2 ? 2 : (d > 4 ? 4 : d);
  }();
  const bf16_t* W = reinterpret_cast<const bf16_t*>(Wt8);
  if (depth == 2) launch_glu_il_d<2, true>(x, ldx, W, y, ldy, M, ntiles, K, fz, w, st);
  else if (depth == 3) launch_glu_il_d<3, true>(x, ldx, W, y, ldy, M, ntiles, K, fz, w, st);
  else launch_glu_il_d<4, true>(x, ldx, W, y, ldy, M, ntiles, K, fz, w, st);
}

void launch_skinny_glu_il(const bf16_t* x, int64_t ldx, const bf16_t* Wt, bf16_t* y, int64_t ldy, int M,
                          int N, int K, const KsFuse& fz, hipStream_t st) {
  // DLA_GLU_IL_DEPTH (2, 3 or 4) and DLA_GLU_IL_WAVES (0 = auto) for A/B runs
  static const int depth = [] {
    const char* e = getenv("DLA_GLU_IL_DEPTH");
    const int d = e ? atoi(e) : 2;
    return d < 2 ? 2 : (d > 4 ? 4 : d);
  }();
  static const int waves = [] {
    const char* e = getenv("DLA_GLU_IL_WAVES");
    const int v = e ? atoi(e) : 0;
    return (v >= 1 && v <= 8) ? v : 0;
  }();
  const int ntiles = N / 16;
  int w = 8;
  for (int c : {8, 7, 6, 5, 4}) {
    if (ntiles % c == 0 && ntiles / c >= 256) { w = c; break; }
  }
  if (waves > 0 && M <= 4 * waves) w = waves;  // the rstd waves cover 4 rows each
  if (depth == 4) launch_glu_il_d<4>(x, ldx, Wt, y, ldy, M, ntiles, K, fz, w, st);
  else if (depth == 3) launch_glu_il_d<3>(x, ldx, Wt, y, ldy, M, ntiles, K, fz, w, st);
  else launch_glu_il_d<2>(x, ldx, Wt, y, ldy, M, ntiles, K, fz, w, st);
}

bool skinny_use_ksplit(int N, int K) {
  return (N + kSkCols - 1) / kSkCols < 128 && (K % (8 * kKsChunk)) == 0 && N % 16 == 0;
}

bool skinny_glu_ks_ok(int N, int K) { return (K % (4 * kKsChunk)) == 0 && N % 32 == 0; }

template <bool NT, bool GLU>
static void launch_ks(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                      int64_t ldy, int M, int N, int K, int nb, hipStream_t st) {
  // M <= 16: a 2-deep ring (84 VGPRs: 5-6 waves per SIMD, every qkv block resident in one round);
  // a 4-deep ring (152 VGPRs) measured slower at qkv (16.0 vs 14.8 us in a decode step)
  // long K (the 14336-deep down projection: 14 ring slots per wave, one workgroup per CU) keeps
  // a 4-deep ring in flight (DLA_SKINNY_DEEP_K, default 8192: K at or above it)
  static const int deep_k = [] {
    const char* e = getenv("DLA_SKINNY_DEEP_K");
    return e ? atoi(e) : 8192;
  }();
  if (M <= 16 && !GLU && K >= deep_k)
    skinny_ksplit_kernel<4, NT, GLU, 1><<<nb, 512, 0, st>>>(x, ldx, W, ldw, y, ldy, M, N, K);
  else if (M <= 16)
    skinny_ksplit_kernel<2, NT, GLU, 1><<<nb, 512, 0, st>>>(x, ldx, W, ldw, y, ldy, M, N, K);
  else if (M <= 32)
    skinny_ksplit_kernel<2, NT, GLU, 2, 2><<<nb, 512, 0, st>>>(x, ldx, W, ldw, y, ldy, M, N, K);
  else
    skinny_ksplit_kernel<2, NT, GLU, 4, 2><<<nb, 512, 0, st>>>(x, ldx, W, ldw, y, ldy, M, N, K);
}

void launch_skinny_ksplit(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                          int64_t ldy, int M, int N, int K, hipStream_t st) {
  launch_ks<false, false>(x, ldx, W, ldw, y, ldy, M, N, K, N / 16, st);
}

// gate|up (N = 2F weight rows) -> m = silu(gate) * up [M, F], F / 16 workgroups
void launch_skinny_glu_ks(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                          int64_t ldy, int M, int N, int K, hipStream_t st) {
  launch_ks<false, true>(x, ldx, W, ldw, y, ldy, M, N, K, N / 32, st);
}

}  // namespace dla
