// Decode GEMMs at 17..64 rows: y[M, N] = x[M, K] @ W[N, K]^T, bf16 in/out, fp32 accumulate.
//
// Reference: the rollout batch of src/training/train_rlhf.py:115-124 (config/rlhf_config.yaml:
// 64 prompts per step) runs every projection of every generated token at 64 rows.
//
// Why a separate kernel from skinny.hip (M <= 16): there every workgroup holds ALL of x for its
// K-slice in LDS (16 x 4096 bf16 = 128 KB), or re-reads x fragments per 16 output columns from
// L2. At 64 rows x is 512 KB: it does not fit, and per-16-column re-reads cost ~1.7 GB of L2
// traffic per layer (README "Tried": 11.6 vs 6.1 ms/token). hipBLASLt's 64-row tiles run the
// narrow projections at 2.2-3.0 TB/s (profiles/r3_decode.md, B = 64). Layout here:
//   * a workgroup owns 128 output columns (8 waves x 16; GLU: 64 gate + the matching 64 up
//     columns) and a K-slice; x streams through a 2-slot LDS ring in 256-deep chunks shared by
//     the 8 waves (x traffic from L2 = 1/8 of the per-16-column form);
//   * each wave streams its 16 weight rows with 16-byte loads straight into registers (two
//     256-deep ring slots = 16 loads in flight per lane), B fragments of
//     v_mfma_f32_16x16x32_bf16; every weight fragment feeds MT = M/16 MFMAs (one per 16 rows);
//   * narrow outputs split K over workgroups (>= 256 workgroups) into fp32 slabs, reduced in a
//     FIXED order with the decode-layer epilogue (residual add + row sum of squares, or the
//     RMSNorm row factor) by a second small launch (m64_reduce_kernel) -- deterministic,
//     graph-capture safe;
//   * the gate|up projection (wide, no split) applies RMSNorm's row factor and SwiGLU in its
//     own epilogue.
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace dla {

namespace {

constexpr int kM64Waves = 8;
constexpr int kM64Ck = 256;             // k per x chunk and per weight ring slot
constexpr int kM64Steps = kM64Ck / 32;  // MFMA k-steps per chunk
constexpr int kM64Ld = kM64Ck + 8;      // LDS row stride in bf16 (16-byte pad)
constexpr int kM64MaxNbp = 64;          // row-norm partials per row (N / 128 <= 64: H <= 8192)
constexpr int kM64RegNbp = 8;           // partials held in registers (reduce-launch producers: N / 1024)

__device__ __forceinline__ f32x4 mfma16(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// F8 (weight-only fp8 decode, TW + nt only): W is the e4m3 tiled copy [N/16, K/64, 64 lanes, 16 B]
// of csrc/skinny_ks.h F8 (ops/decode.py fp8_tiled_weight): one 16-byte load per lane holds its B
// fragments of two consecutive k-steps, so a 256-deep chunk is 4 loads per lane instead of 8 and
// the stream is half the bytes; e4m3 -> bf16 in registers (exact), the bf16 MFMA unchanged, and
// the per-row scale wsc[n] applied to the fp32 sum before any epilogue.
// Weight layouts: row-major W [N, K], or TW (tiled, ops/decode.py `tiled_weight`):
// Wt[N / 16][K / 32][4][16][8] with Wt[t][kk][q][r][e] = W[16 t + r][32 kk + 8 q + e], i.e. the
// 16-byte pieces in the order lane (r = lane & 15, q = lane >> 4) of an MFMA B fragment reads them:
// one weight load instruction is 1 KB contiguous and a wave's 256-deep chunk 8 KB, instead of 16
// rows x 64 B at an 8 KB (K = 4096) stride.
}  // namespace

// grid (N / 16 NW [GLU: F / 8 NW], S), 64 NW threads. LDS: 2 x 16 MT x kM64Ld bf16.
// GLU: W = [gate; up] (2F rows), output m = silu(rstd * g) * (rstd * u) [M, F] where rstd comes
// from ssq_in (the producer's row partial sums, [M][nbp]) when NIN, else 1; gate / up are
// rounded to bf16 before SwiGLU exactly as the unfused GEMM + swiglu pair.
// Otherwise S == 1 writes y = bf16(x W^T); S > 1 writes fp32 slab ws[s][m][n].
template <int MT, bool GLU, bool NIN, bool TW, int DEPTH, int NW = kM64Waves, bool NTL = false, bool F8 = false>
__global__ __launch_bounds__(64 * NW) void m64_gemm_kernel(
    const bf16_t* __restrict__ x, int64_t ldx, const bf16_t* __restrict__ W, int64_t ldw,
    bf16_t* __restrict__ y, int64_t ldy, float* __restrict__ ws, int M, int N, int K, int kc,
    const float* __restrict__ ssq_in, int nbp, float eps, const float* __restrict__ wsc) {
  static_assert(!F8 || (TW && NTL), "fp8 weights: tiled layout, nt stream");
  extern __shared__ __attribute__((aligned(16))) bf16_t xs[];
  __shared__ float rstd_s[64];
  constexpr int RB = 16 * MT * kM64Ld;  // one ring slot
  constexpr int NTH = 64 * NW;
  constexpr int XPASS = 16 * MT * 32 / NTH;  // x staging passes (32 threads per 256-deep row)
  constexpr int FPW = 8 * NW;                // GLU: features per workgroup
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
  const int F = N >> 1;
  const int n0 = GLU ? (wave < NW / 2 ? 0 : F) + blockIdx.x * FPW + (wave % (NW / 2)) * 16
                     : blockIdx.x * (16 * NW) + wave * 16;
  const int s = blockIdx.y;
  const int k0 = s * kc;
  const int nch = kc / kM64Ck;
  const bf16_t* wrow = TW ? W + static_cast<int64_t>(n0 >> 4) * 16 * K + (k0 >> 5) * 512 + lane * 8
                         : W + static_cast<int64_t>(n0 + r) * ldw + k0 + q * 8;
  const uint8_t* wrow8 = reinterpret_cast<const uint8_t*>(W) + static_cast<int64_t>(n0 >> 4) * 16 * K +
                         (k0 >> 6) * 1024 + lane * 16;

  // NIN: this row's producer partials (thread m < M holds row m); up to kM64RegNbp are loaded
  // here, ahead of the first chunk, and summed once those loads land
  float pv[kM64RegNbp];
  if constexpr (NIN) {
#pragma unroll
    for (int j = 0; j < kM64RegNbp; ++j)
      pv[j] = (tid < M && j < nbp && nbp <= kM64RegNbp) ? ssq_in[tid * nbp + j] : 0.f;
  }

  // Pipeline: chunk j = x(j) (this thread's 16-byte pieces of 16 MT rows, into register set
  // j % DEPTH) followed by W(j) (8 loads per lane into ring slot j % DEPTH) -- ALWAYS in that
  // issue order, because s_waitcnt vmcnt is in-order: storing x(c + 1) into LDS waits only for
  // loads older than it, so W(c + 1) stays in flight (loading x after W made every step wait a
  // full HBM round trip for the next weight chunk). DEPTH chunks are in flight; x rows >= M are
  // zeros so the A fragments need no row test.
  const int xm = tid >> 5, xc = (tid & 31) * 8;
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  constexpr int KS8 = kM64Steps / 2;  // fp8: 16-byte weight loads per lane per chunk
  bf16x8 xr[DEPTH][XPASS];
  s16x8 b[DEPTH][F8 ? 1 : kM64Steps];
  u32x4v b8[DEPTH][F8 ? KS8 : 1];
  auto issue = [&](auto J, int c) {
    constexpr int j = decltype(J)::value;
#pragma unroll
    for (int t = 0; t < XPASS; ++t) {
      const int m = xm + (NTH / 32) * t;
      xr[j][t] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (m < M) xr[j][t] = load_bf16x8(x + static_cast<int64_t>(m) * ldx + k0 + c * kM64Ck + xc);
    }
    if constexpr (F8) {
#pragma unroll
      for (int u = 0; u < KS8; ++u)
        b8[j][u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(wrow8 + (c * KS8 + u) * 1024));
      return;
    }
#pragma unroll
    for (int u = 0; u < kM64Steps; ++u)
      b[j][u] = NTL ? __builtin_bit_cast(s16x8, __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(
                          TW ? wrow + (c * kM64Steps + u) * 512 : wrow + c * kM64Ck + u * 32)))
                    : __builtin_bit_cast(s16x8, load_bf16x8(TW ? wrow + (c * kM64Steps + u) * 512 : wrow + c * kM64Ck + u * 32));
  };
  auto xstore = [&](auto J, int slot) {
    constexpr int j = decltype(J)::value;
#pragma unroll
    for (int t = 0; t < XPASS; ++t) store_bf16x8(xs + slot * RB + (xm + (NTH / 32) * t) * kM64Ld + xc, xr[j][t]);
  };
  issue(std::integral_constant<int, 0>{}, 0);
  if (1 < nch) issue(std::integral_constant<int, 1>{}, 1);
  if constexpr (DEPTH > 2) {
    if (2 < nch) issue(std::integral_constant<int, 2>{}, 2);
  }
  if constexpr (DEPTH > 3) {
    if (3 < nch) issue(std::integral_constant<int, 3>{}, 3);
  }
  // NIN: the row's partials summed now, in order (their loads are older than the chunk loads, so
  // this waits only for them), one register live through the loop; the in-kernel-combine
  // producers' N / 128 partials (> kM64RegNbp) are summed by a plain loop
  float rsum = 0.f;
  if constexpr (NIN) {
    if (nbp <= kM64RegNbp) {
#pragma unroll
      for (int j = 0; j < kM64RegNbp; ++j) rsum += pv[j];
    } else if (tid < M) {
      for (int j = 0; j < nbp; ++j) rsum += ssq_in[tid * nbp + j];
    }
    asm volatile("" : "+v"(rsum));
  }
  xstore(std::integral_constant<int, 0>{}, 0);
  __syncthreads();

  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int aoff = r * kM64Ld + q * 8;
  auto step = [&](auto J, int c) {
    constexpr int j = decltype(J)::value;
    const bf16_t* xb = xs + (c & 1) * RB + aoff;
#pragma unroll
    for (int u = 0; u < kM64Steps; ++u) {
      s16x8 bu;
      if constexpr (F8) {
        const u32x4v wv = b8[j][u >> 1];
        bu = (u & 1) ? f8x8_to_bf16(wv[2], wv[3]) : f8x8_to_bf16(wv[0], wv[1]);
      } else {
        bu = b[j][u];
      }
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const s16x8 a = __builtin_bit_cast(s16x8, *reinterpret_cast<const bf16x8*>(xb + t * 16 * kM64Ld + u * 32));
        acc[t] = mfma16(a, bu, acc[t]);
      }
    }
    if (c + 1 < nch) xstore(std::integral_constant<int, (j + 1) % DEPTH>{}, (c + 1) & 1);
    __syncthreads();
    if (c + DEPTH < nch) issue(J, c + DEPTH);
  };
  for (int c = 0; c < nch; c += DEPTH) {
    step(std::integral_constant<int, 0>{}, c);
    if (c + 1 < nch) step(std::integral_constant<int, 1>{}, c + 1);
    if constexpr (DEPTH > 2) {
      if (c + 2 < nch) step(std::integral_constant<int, 2>{}, c + 2);
    }
    if constexpr (DEPTH > 3) {
      if (c + 3 < nch) step(std::integral_constant<int, 3>{}, c + 3);
    }
  }

  // lane holds C[m = 16 t + 4 q + i][n = n0 + r]
  if constexpr (F8) {
    const float sc = wsc[n0 + r];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] *= sc;
  }
  if constexpr (GLU) {
    if constexpr (NIN) {
      if (tid < M) rstd_s[tid] = rsqrtf(rsum / static_cast<float>(K) + eps);
    }
    // the ring is dead after the loop's last barrier: exchange the gate / up tiles through it
    float* glu = reinterpret_cast<float*>(xs);  // [2][64][FPW]
    const int half = wave / (NW / 2), col = (wave % (NW / 2)) * 16 + r;
    __syncthreads();
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = 16 * t + 4 * q + i;
        float v = acc[t][i];
        if constexpr (NIN) v *= m < M ? rstd_s[m] : 0.f;
        glu[(half * 64 + m) * FPW + col] = bf2f(f2bf(v));
      }
    __syncthreads();
    // 8 consecutive features of one row per thread, one 16-byte store
    for (int e = tid; e < M * (FPW / 8); e += NTH) {
      const int m = e / (FPW / 8), c8 = (e % (FPW / 8)) * 8;
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float g = glu[m * FPW + c8 + j], u = glu[(64 + m) * FPW + c8 + j];
        o[j] = g / (1.f + __expf(-g)) * u;
      }
      store_bf16x8(y + static_cast<int64_t>(m) * ldy + blockIdx.x * FPW + c8, pack_bf16x8(o));
    }
    return;
  }
  const int n = n0 + r;
  if (gridDim.y == 1) {
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = 16 * t + 4 * q + i;
        if (m < M) y[static_cast<int64_t>(m) * ldy + n] = f2bf(acc[t][i]);
      }
    return;
  }
  float* slab = ws + static_cast<int64_t>(s) * M * N;
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = 16 * t + 4 * q + i;
      if (m < M) slab[static_cast<int64_t>(m) * N + n] = acc[t][i];
    }
}

// Split-K reduce + decode-layer epilogue. grid (ceil(N / 1024), M), 256 threads x 4 columns.
//   MODE 0: y = bf16(sum_s ws[s])
//   MODE 1 (NIN): y = bf16(rstd[m] * sum), rstd = rsqrt(sum_j ssq_in[m][j] / N_norm + eps)
//   MODE 2 (RES): y = s = bf16(bf16(sum) + res) and ssq_out[m][blockIdx.x] = sum over the
//                 block's 1024 columns of s^2 (fixed order) -- the next NIN consumer's partials
template <int MODE, int S>
__global__ __launch_bounds__(256) void m64_reduce_kernel(const float* __restrict__ ws, int M,
                                                         int N, bf16_t* __restrict__ y, int64_t ldy,
                                                         const bf16_t* __restrict__ res, int64_t ldr,
                                                         const float* __restrict__ ssq_in, int nbp,
                                                         int knorm, float eps, float* __restrict__ ssq_out) {
  __shared__ float red[4];
  const int m = blockIdx.y;
  const int n = blockIdx.x * 1024 + threadIdx.x * 4;
  const float* p = ws + static_cast<int64_t>(m) * N + n;
  const int64_t slab = static_cast<int64_t>(M) * N;
  const bool live = n < N;  // N % 128 == 0: a thread's 4 columns are all in or all out
  // all S slab loads in flight at once (compile-time count), summed in split order
  f32x4 v[S];
  if (live) {
#pragma unroll
    for (int s = 0; s < S; ++s) v[s] = *reinterpret_cast<const f32x4*>(p + s * slab);
  }
  f32x4 t = {0.f, 0.f, 0.f, 0.f};
  if (live) {
#pragma unroll
    for (int s = 0; s < S; ++s) t += v[s];
  }
  if constexpr (MODE == 1) {
    float a = 0.f;
    for (int j = 0; j < nbp; ++j) a += ssq_in[m * nbp + j];
    t *= rsqrtf(a / static_cast<float>(knorm) + eps);
  }
  bf16x4 o;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (!live) break;
    if constexpr (MODE == 2) {
      const float v = bf2f(f2bf(bf2f(f2bf(t[i])) + bf2f(res[static_cast<int64_t>(m) * ldr + n + i])));
      o[i] = f2bf(v);
      ss += v * v;
    } else {
      o[i] = f2bf(t[i]);
    }
  }
  if (live) *reinterpret_cast<bf16x4*>(y + static_cast<int64_t>(m) * ldy + n) = o;
  if constexpr (MODE == 2) {
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    if (threadIdx.x == 0) ssq_out[m * gridDim.x + blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
  }
}

// Split-K count: the most splits that keep the grid within one workgroup per CU. A grid of 1.5
// workgroups per CU (the qkv projection at Llama-3-8B: 48 column blocks x 8 splits = 384) leaves
// half the CUs streaming twice the bytes of the rest; 48 x 4 = 192 workgroups ran the same GEMM +
// reduce in 21.4 vs 26.9 us (B = 64, a round-4 probe since removed). DLA_M64_WG=n (A/B) restores the
// round-3 rule: the fewest splits whose grid reaches n workgroups.
int m64_splits(int N, int K) {
  static const int target = [] {
    const char* e = getenv("DLA_M64_WG");
    return e ? atoi(e) : 0;
  }();
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    (void)hipGetLastError();
    return n;
  }();
  const int nb = N / (16 * kM64Waves);
  const int chunks = K / kM64Ck;
  // split counts the reduce kernel is instantiated for
  if (target > 0) {
    for (int s : {1, 2, 4, 7, 8, 14, 16}) {
      if (chunks % s) continue;
      if (nb * s >= target) return s;
    }
    for (int s : {16, 14, 8, 7, 4, 2}) if (chunks % s == 0) return s;
    return 1;
  }
  // (a grid of fewer column blocks than CUs always splits at least once, as the round-3 rule did:
  // the residual / norm epilogues live in the reduce launch)
  int best = 1;
  for (int s : {2, 4, 7, 8, 14, 16})
    if (chunks % s == 0 && (nb * s <= cus || (best == 1 && nb < cus))) best = s;
  return best;
}

bool m64_shape_ok(int N, int K, bool glu) {
  return K % kM64Ck == 0 && N % 128 == 0;
}

size_t m64_lds_bytes(int M) {
  const int mt = M <= 32 ? 2 : 4;
  return static_cast<size_t>(2 * 16 * mt * kM64Ld) * sizeof(bf16_t);
}

template <int MT, bool GLU, bool NIN, bool TW, int NW, bool NTL, int DEPTH = 2, bool F8 = false>
static void m64_launch_w(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                         int64_t ldy, float* ws, int M, int N, int K, int S, const float* ssq_in,
                         int nbp, float eps, hipStream_t st, const float* wsc = nullptr) {
  const size_t lds = static_cast<size_t>(2 * 16 * MT * kM64Ld) * sizeof(bf16_t);
  static bool attr = [] {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&m64_gemm_kernel<MT, GLU, NIN, TW, DEPTH, NW, NTL, F8>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    (void)hipGetLastError();
    return true;
  }();
  (void)attr;
  dim3 grid(GLU ? N / 2 / (8 * NW) : N / (16 * NW), S);
  m64_gemm_kernel<MT, GLU, NIN, TW, DEPTH, NW, NTL, F8><<<grid, 64 * NW, lds, st>>>(
      x, ldx, W, ldw, y, ldy, ws, M, N, K, K / S, ssq_in, nbp, eps, wsc);
}

// NW = 8 waves per workgroup (gate|up: 64 features per workgroup). 4 waves (448 gate|up
// workgroups at Llama-3-8B, two per CU) measured 55.0 vs 53.2 us: README "Tried".
template <int MT, bool GLU, bool NIN, bool TW>
static void m64_launch(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                       int64_t ldy, float* ws, int M, int N, int K, int S, const float* ssq_in,
                       int nbp, float eps, hipStream_t st) {
  // non-temporal loads on the tiled weight stream (see skinny.hip decode_nt)
  constexpr bool nt = true;
  // two weight chunks in flight per wave on the tiled nt stream (3 or 4 measured 5.10 / 5.27 vs
  // 5.01 ms/token at B = 64: more bytes in flight only lengthen the queues; removed)
  if constexpr (TW) {
    if (nt) {
      m64_launch_w<MT, GLU, NIN, TW, kM64Waves, true>(x, ldx, W, ldw, y, ldy, ws, M, N, K, S, ssq_in, nbp, eps, st);
      return;
    }
  }
  m64_launch_w<MT, GLU, NIN, TW, kM64Waves, false>(x, ldx, W, ldw, y, ldy, ws, M, N, K, S, ssq_in, nbp, eps, st);
}

// fp8 weights (tiled, nt): DLA_M64_F8_DEPTH = weight chunks in flight per wave (2, 3 or 4; a chunk
// is half the bf16 bytes, so the same bytes in flight take twice the chunks)
template <int MT, bool GLU, bool NIN>
static void m64_launch_f8(const bf16_t* x, int64_t ldx, const uint8_t* W8, bf16_t* y, int64_t ldy, float* ws,
                          int M, int N, int K, int S, const float* ssq_in, int nbp, float eps,
                          const float* wsc, hipStream_t st) {
  static const int depth = [] {
    const char* e = getenv("DLA_M64_F8_DEPTH");
    const int d = e ? atoi(e) : 3;
    return d >= 2 && d <= 4 ? d : 3;
  }();
  const bf16_t* W = reinterpret_cast<const bf16_t*>(W8);
  if (depth == 2)
    m64_launch_w<MT, GLU, NIN, true, kM64Waves, true, 2, true>(x, ldx, W, 0, y, ldy, ws, M, N, K, S, ssq_in, nbp, eps, st, wsc);
  else if (depth == 4)
    m64_launch_w<MT, GLU, NIN, true, kM64Waves, true, 4, true>(x, ldx, W, 0, y, ldy, ws, M, N, K, S, ssq_in, nbp, eps, st, wsc);
  else
    m64_launch_w<MT, GLU, NIN, true, kM64Waves, true, 3, true>(x, ldx, W, 0, y, ldy, ws, M, N, K, S, ssq_in, nbp, eps, st, wsc);
}

template <int MT>
static void m64_dispatch_f8(const bf16_t* x, int64_t ldx, const uint8_t* W8, bf16_t* y, int64_t ldy, float* ws,
                            int M, int N, int K, int S, bool glu, const float* ssq_in, int nbp, float eps,
                            const float* wsc, hipStream_t st) {
  if (glu && ssq_in)
    m64_launch_f8<MT, true, true>(x, ldx, W8, y, ldy, ws, M, N, K, 1, ssq_in, nbp, eps, wsc, st);
  else if (glu)
    m64_launch_f8<MT, true, false>(x, ldx, W8, y, ldy, ws, M, N, K, 1, nullptr, 0, 0.f, wsc, st);
  else
    m64_launch_f8<MT, false, false>(x, ldx, W8, y, ldy, ws, M, N, K, S, nullptr, 0, 0.f, wsc, st);
}

// fp8 form of launch_m64_gemm: W8 the e4m3 tiled copy, wsc its per-row scales
void launch_m64_gemm_f8(const bf16_t* x, int64_t ldx, const uint8_t* W8, bf16_t* y, int64_t ldy, float* ws,
                        int M, int N, int K, int S, bool glu, const float* ssq_in, int nbp, float eps,
                        const float* wsc, hipStream_t st) {
  if (M <= 32) m64_dispatch_f8<2>(x, ldx, W8, y, ldy, ws, M, N, K, S, glu, ssq_in, nbp, eps, wsc, st);
  else m64_dispatch_f8<4>(x, ldx, W8, y, ldy, ws, M, N, K, S, glu, ssq_in, nbp, eps, wsc, st);
}

template <int MT, bool TW>
static void m64_dispatch(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                         int64_t ldy, float* ws, int M, int N, int K, int S, bool glu,
                         const float* ssq_in, int nbp, float eps, hipStream_t st) {
  if (glu && ssq_in)
    m64_launch<MT, true, true, TW>(x, ldx, W, ldw, y, ldy, ws, M, N, K, 1, ssq_in, nbp, eps, st);
  else if (glu)
    m64_launch<MT, true, false, TW>(x, ldx, W, ldw, y, ldy, ws, M, N, K, 1, nullptr, 0, 0.f, st);
  else
    m64_launch<MT, false, false, TW>(x, ldx, W, ldw, y, ldy, ws, M, N, K, S, nullptr, 0, 0.f, st);
}

// GEMM (S > 1: fp32 slabs into ws) -- the reduce is a separate launch (launch_m64_reduce).
// tiled: W is the tiled layout (ldw unused).
void launch_m64_gemm(const bf16_t* x, int64_t ldx, const bf16_t* W, int64_t ldw, bf16_t* y,
                     int64_t ldy, float* ws, int M, int N, int K, int S, bool glu,
                     const float* ssq_in, int nbp, float eps, bool tiled, hipStream_t st) {
  if (M <= 32) {
    if (tiled) m64_dispatch<2, true>(x, ldx, W, ldw, y, ldy, ws, M, N, K, S, glu, ssq_in, nbp, eps, st);
    else m64_dispatch<2, false>(x, ldx, W, ldw, y, ldy, ws, M, N, K, S, glu, ssq_in, nbp, eps, st);
  } else {
    if (tiled) m64_dispatch<4, true>(x, ldx, W, ldw, y, ldy, ws, M, N, K, S, glu, ssq_in, nbp, eps, st);
    else m64_dispatch<4, false>(x, ldx, W, ldw, y, ldy, ws, M, N, K, S, glu, ssq_in, nbp, eps, st);
  }
}

template <int MODE>
static void m64_reduce_s(const float* ws, int S, int M, int N, bf16_t* y, int64_t ldy, const bf16_t* res,
                         int64_t ldr, const float* ssq_in, int nbp, int knorm, float eps, float* ssq_out,
                         hipStream_t st) {
  dim3 grid((N + 1023) / 1024, M);
#define DLA_M64R(SS) \
  m64_reduce_kernel<MODE, SS><<<grid, 256, 0, st>>>(ws, M, N, y, ldy, res, ldr, ssq_in, nbp, knorm, eps, ssq_out)
  switch (S) {
    case 2: DLA_M64R(2); break;
    case 4: DLA_M64R(4); break;
    case 7: DLA_M64R(7); break;
    case 8: DLA_M64R(8); break;
    case 14: DLA_M64R(14); break;
    case 16: DLA_M64R(16); break;
    default: DLA_M64R(1); break;  // S == 1 never reaches the reduce (checked by the caller)
  }
#undef DLA_M64R
}

void launch_m64_reduce(const float* ws, int S, int M, int N, bf16_t* y, int64_t ldy, const bf16_t* res,
                       int64_t ldr, const float* ssq_in, int nbp, int knorm, float eps, float* ssq_out,
                       hipStream_t st) {
  if (res)
    m64_reduce_s<2>(ws, S, M, N, y, ldy, res, ldr, nullptr, 0, 0, 0.f, ssq_out, st);
  else if (ssq_in)
    m64_reduce_s<1>(ws, S, M, N, y, ldy, nullptr, 0, ssq_in, nbp, knorm, eps, nullptr, st);
  else
    m64_reduce_s<0>(ws, S, M, N, y, ldy, nullptr, 0, nullptr, 0, 0, 0.f, nullptr, st);
}

// W [N, K] (row stride ldw) -> the tiled layout [N/16, K/32, 4, 16, 8] (see TW above; glu_il: gate /
// up rows interleaved 8 + 8 per tile, skinny.hip skinny_glu_il_kernel), with nw
// the RMSNorm weight folded in (bf16(W * nw), torch.mul's rounding). One 16-byte output piece per
// thread: a wave writes 1 KB contiguous and reads 16 rows x 64 B. Rebuilt whenever the weights
// moved (every RLHF step): one pass instead of mul + a strided permute copy.
__global__ __launch_bounds__(256) void tile_weight_kernel(const bf16_t* __restrict__ W, int64_t ldw,
                                                          const bf16_t* __restrict__ nw,
                                                          bf16_t* __restrict__ out, int K,
                                                          int64_t total, int glu_f) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= total) return;
  const int lane = static_cast<int>(i & 63);
  const int64_t blk = i >> 6;
  const int kb = K >> 5;
  const int64_t t = blk / kb;
  const int kk = static_cast<int>(blk - t * kb);
  const int col = kk * 32 + (lane >> 4) * 8;
  // glu_f > 0 (gate|up, F = glu_f): tile t row r < 8 is gate row 8t + r, r >= 8 up row F + 8t + r - 8
  const int r = lane & 15;
  const int64_t row = glu_f > 0 ? (r < 8 ? 8 * t + r : glu_f + 8 * t + r - 8) : t * 16 + r;
  bf16x8 v = load_bf16x8(W + row * ldw + col);
  if (nw != nullptr) {
    const bf16x8 g = load_bf16x8(nw + col);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) * bf2f(g[e]));
  }
  store_bf16x8(out + i * 8, v);
}

void launch_tile_weight(const bf16_t* W, int64_t ldw, const bf16_t* nw, bf16_t* out, int N, int K,
                        bool glu_il, hipStream_t st) {
  const int64_t total = static_cast<int64_t>(N) * K / 8;
  tile_weight_kernel<<<static_cast<unsigned>((total + 255) / 256), 256, 0, st>>>(W, ldw, nw, out, K, total,
                                                                                 glu_il ? N / 2 : 0);
}

// Weight-only fp8 decode copy in one pass (ops/decode.py fp8_tiled_weight; refreshed every RLHF
// step): W [N, K] (row stride ldw), nw folded as bf16(W * nw), glu_f > 0 = gate / up rows
// interleaved 8 + 8 per tile (as tile_weight_kernel) -> per-row scale amax / 448 and the e4m3
// tiled layout [N/16, K/64, 64, 16 B] of csrc/skinny_ks.h F8. One 256-thread workgroup per 16-row
// tile: 16 threads per row reduce its amax (the rows then sit in L2 for the second pass), every
// thread then writes whole 16-byte lane pieces (round to nearest even, values pre-clamped to
// +-448 as the torch reference does).
__global__ __launch_bounds__(256) void quant_tile_f8_kernel(const bf16_t* __restrict__ W, int64_t ldw,
                                                            const bf16_t* __restrict__ nw,
                                                            uint8_t* __restrict__ out, float* __restrict__ scale,
                                                            int K, int glu_f) {
  __shared__ float inv_s[16];
  const int t = blockIdx.x, tid = threadIdx.x;
  auto row_of = [&](int r) -> int64_t {
    return glu_f > 0 ? (r < 8 ? 8 * static_cast<int64_t>(t) + r : glu_f + 8 * static_cast<int64_t>(t) + r - 8)
                     : static_cast<int64_t>(t) * 16 + r;
  };
  auto fetch = [&](int64_t row, int col) {
    bf16x8 v = load_bf16x8(W + row * ldw + col);
    if (nw != nullptr) {
      const bf16x8 g = load_bf16x8(nw + col);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) * bf2f(g[e]));
    }
    return v;
  };
  {
    const int r = tid >> 4, sub = tid & 15;
    const int64_t row = row_of(r);
    float am = 0.f;
    for (int c = sub * 8; c < K; c += 128) {
      const bf16x8 v = fetch(row, c);
#pragma unroll
      for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(bf2f(v[e])));
    }
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 16));
    if (sub == 0) {
      const float sc = fmaxf(am / 448.f, 1e-12f);
      scale[16 * static_cast<int64_t>(t) + r] = sc;
      inv_s[r] = sc;
    }
  }
  __syncthreads();
  const int pieces = (K >> 6) * 64;
  uint8_t* otile = out + static_cast<int64_t>(t) * 16 * K;
  for (int p = tid; p < pieces; p += 256) {
    const int kt = p >> 6, lane = p & 63, r = lane & 15, qd = lane >> 4;
    const int64_t row = row_of(r);
    const float sc = inv_s[r];
    const bf16x8 lo = fetch(row, 64 * kt + 8 * qd), hi = fetch(row, 64 * kt + 32 + 8 * qd);
    auto q8 = [&](bf16_t x) { return fminf(fmaxf(bf2f(x) / sc, -448.f), 448.f); };
    uint32_t wv[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bf16x8& v = h ? hi : lo;
      // bytes 4j .. 4j+3 of the piece: e4m3 of elements 4j .. 4j+3 (low half first)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        uint32_t wd = __builtin_amdgcn_cvt_pk_fp8_f32(q8(v[4 * j]), q8(v[4 * j + 1]), 0u, false);
        wd = __builtin_amdgcn_cvt_pk_fp8_f32(q8(v[4 * j + 2]), q8(v[4 * j + 3]), wd, true);
        wv[2 * h + j] = wd;
      }
    }
    *reinterpret_cast<uint4*>(otile + static_cast<int64_t>(p) * 16) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
  }
}

void launch_quant_tile_f8(const bf16_t* W, int64_t ldw, const bf16_t* nw, uint8_t* out, float* scale, int N,
                          int K, bool glu_il, hipStream_t st) {
  quant_tile_f8_kernel<<<N / 16, 256, 0, st>>>(W, ldw, nw, out, scale, K, glu_il ? N / 2 : 0);
}

}  // namespace dla
