// In-workgroup split-K skinny GEMM body (decode projections, M <= 64 rows), shared by the
// standalone csrc/skinny.hip kernels and the fused decode qkv + attention kernel (csrc/decode.hip):
// `bx` is the workgroup's column block, `nblk` the number of such blocks. 512 threads (8 waves).
#pragma once
#include "common.h"
#include "skinny_params.h"

namespace dla {

namespace {

__device__ __forceinline__ float silu_sk(float g) { return g * sigmoidf_(g); }

__device__ __forceinline__ f32x4 mfma16(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Weight-stream load: with NT the 16-byte load carries the non-temporal hint (each weight byte is
// read once per decode step by one CU; MI355X_MICROARCH.md "nt-weights").
template <bool NT>
__device__ __forceinline__ s16x8 load_w(const bf16_t* p) {
  if constexpr (NT)
    return __builtin_bit_cast(s16x8, __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(p)));
  else
    return __builtin_bit_cast(s16x8, load_bf16x8(p));
}

// prefetch (kernel start) of this wave's two rows' partial sums of squares: lane-strided, up to
// 8 values per row (nbp <= 512)
struct KsPart {
  float v[2][8];
};

__device__ __forceinline__ KsPart ks_part_load(const KsFuse& fz, int M, int wave, int lane) {
  KsPart p;
#pragma unroll
  for (int rr = 0; rr < 2; ++rr) {
    const int m = 2 * wave + rr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = lane + 64 * j;
      p.v[rr][j] = (m < M && i < fz.nbp) ? fz.ssq_in[m * fz.nbp + i] : 0.f;
    }
  }
  return p;
}

// rows 2w, 2w+1 per wave: rstd = rsqrt(sum / K + eps) (in-lane sum in order, then butterfly)
__device__ __forceinline__ void ks_rstd(const KsPart& p, const KsFuse& fz, int M, int K, int wave,
                                        int lane, float* rstd_s) {
#pragma unroll
  for (int rr = 0; rr < 2; ++rr) {
    const int m = 2 * wave + rr;
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) t += p.v[rr][j];
    t = wave_sum(t);
    if (lane == 0 && m < M) rstd_s[m] = rsqrtf(t / static_cast<float>(K) + fz.eps);
  }
}

}  // namespace

constexpr int kKsUnroll = 4;  // k-steps per chunk (one 16-byte W and x load per lane each)
constexpr int kKsChunk = 32 * kKsUnroll;

// WT: the plain output is stored write-through (`sc1`, two columns per 4-byte store), for a
// consumer in another workgroup of the same launch that reads it with `sc1` loads after a counter
// hand-off (decode.hip decode_qkv_attn_kernel; MI355X_MICROARCH inter-workgroup visibility, the
// release-free valid form)
typedef uint32_t ks_u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ ks_u32x4 load_w8(const uint8_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const ks_u32x4*>(p));
  else return *reinterpret_cast<const ks_u32x4*>(p);
}

// F8 (decode weight-only fp8, TW only): W points at an e4m3 tiled copy [N/16, K/64, 64 lanes, 16 B]:
// lane r + 16q of k-tile kt holds row r's k = 64kt + 8q + [0, 8) in bytes 0-7 and
// 64kt + 32 + 8q + [0, 8) in bytes 8-15, i.e. its B fragments of two consecutive MFMA k-steps, so
// one 16-byte load feeds two MFMAs and the stream is half the bf16 bytes (ops/decode.py
// fp8_tiled_weight); y[:, n] = wscale[n] * (x . w8[n]).
template <int DEPTH, bool NT, bool GLU, int MT = 1, int UNR = kKsUnroll, bool RES = false, bool NIN = false,
          bool TW = false, bool WT = false, bool F8 = false>
__device__ __forceinline__ void ks_body(
    const int bx, const int nblk, const bf16_t* __restrict__ x, int64_t ldx,
    const bf16_t* __restrict__ W, int64_t ldw, bf16_t* __restrict__ y, int64_t ldy, int M, int N, int K,
    const KsFuse& fz) {
  constexpr int CH = 32 * UNR;  // k per ring slot
  static_assert(!(RES || NIN) || (MT == 1 && !GLU), "fused residual / norm: M <= 16, plain output");
  static_assert(!F8 || (TW && !GLU && !WT && MT == 1 && UNR % 2 == 0), "fp8 weights: tiled, plain rows");
  constexpr int UB = F8 ? UNR / 2 : UNR;  // weight loads per ring slot
  __shared__ float red[8][4 * MT][64];
  __shared__ float rstd_s[16];
  __shared__ float sqs[16][16];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int n0 = GLU ? (wave < 4 ? 0 : N >> 1) + bx * 16 : bx * 16;
  // per-wave K slice (multiple of kKsChunk, checked on the host)
  const int kw = GLU ? K >> 2 : K >> 3;
  const int k0 = (GLU ? (wave & 3) : wave) * kw;
  const int nchunks = kw / CH;
  // TW: tiled weight layout (see skinny_gemm_kernel)
  const bf16_t* wrow = TW ? W + static_cast<int64_t>(n0 >> 4) * 16 * K + (k0 >> 5) * 512 + lane * 8
                          : W + static_cast<int64_t>(n0 + r) * ldw + k0 + q * 8;
  const uint8_t* wrow8 = reinterpret_cast<const uint8_t*>(W) + static_cast<int64_t>(n0 >> 4) * 16 * K +
                         (k0 >> 6) * 1024 + lane * 16;
  bool arow[MT];
  const bf16_t* xrow[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    arow[t] = 16 * t + r < M;
    xrow[t] = x + static_cast<int64_t>(arow[t] ? 16 * t + r : 0) * ldx + k0 + q * 8;
  }
  // DEPTH chunks (W and x fragments) in flight: a ring of register sets, refilled as consumed
  s16x8 b[DEPTH][F8 ? 1 : UNR], a[DEPTH][UNR][MT];
  ks_u32x4 b8[DEPTH][F8 ? UB : 1];
  auto load = [&](int j, int c) {
    if constexpr (F8) {
#pragma unroll
      for (int u = 0; u < UB; ++u) b8[j][u] = load_w8<NT>(wrow8 + (c * UB + u) * 1024);
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u) b[j][u] = load_w<NT>(TW ? wrow + (c * UNR + u) * 512 : wrow + c * CH + u * 32);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        a[j][u][t] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
        if (arow[t]) a[j][u][t] = __builtin_bit_cast(s16x8, load_bf16x8(xrow[t] + c * CH + u * 32));
      }
  };
  // fz.straight: the same ring with no load inside a branch. hipcc counts outstanding loads per
  // path; a refill under `if (c + DEPTH < nchunks)` or an x load under `if (arow)` made it wait
  // vmcnt(0) -- the whole ring -- before every chunk's MFMAs. Here x rows past M load row 0 and are
  // masked to zero by AND, and the loop runs as a steady part whose refills are always in range
  // plus a tail without loads (nchunks a multiple of DEPTH; other shapes keep the form below).
  auto load_nb = [&](int j, int c) {
    if constexpr (F8) {
#pragma unroll
      for (int u = 0; u < UB; ++u) b8[j][u] = load_w8<NT>(wrow8 + (c * UB + u) * 1024);
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u) b[j][u] = load_w<NT>(TW ? wrow + (c * UNR + u) * 512 : wrow + c * CH + u * 32);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const ks_u32x4 v = __builtin_bit_cast(ks_u32x4, load_bf16x8(xrow[t] + c * CH + u * 32));
        const uint32_t keep = arow[t] ? 0xffffffffu : 0u;
        a[j][u][t] = __builtin_bit_cast(s16x8, ks_u32x4{v[0] & keep, v[1] & keep, v[2] & keep, v[3] & keep});
      }
  };
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int j) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      s16x8 bu;
      if constexpr (F8) {
        const ks_u32x4 wv = b8[j][u >> 1];
        bu = (u & 1) ? f8x8_to_bf16(wv[2], wv[3]) : f8x8_to_bf16(wv[0], wv[1]);
      } else {
        bu = b[j][u];
      }
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[t] = mfma16(a[j][u][t], bu, acc[t]);
    }
  };
  const bool sl = fz.straight != 0 && nchunks >= DEPTH && nchunks % DEPTH == 0;  // kernel-uniform
  KsPart part{};
  if (sl) {
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) load_nb(j, j);
    if constexpr (NIN) part = ks_part_load(fz, M, wave, lane);  // reduced in the epilogue
    for (int c0 = 0; c0 + DEPTH < nchunks; c0 += DEPTH) {
#pragma unroll
      for (int j = 0; j < DEPTH; ++j) {
        compute(j);
        load_nb(j, c0 + DEPTH + j);
      }
    }
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) compute(j);
  } else {
#pragma unroll
    for (int j = 0; j < DEPTH; ++j)
      if (j < nchunks) load(j, j);
    if constexpr (NIN) part = ks_part_load(fz, M, wave, lane);  // reduced in the epilogue
  }
  for (int c0 = 0; c0 < (sl ? 0 : nchunks); c0 += DEPTH) {
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) {
      const int c = c0 + j;
      if (c < nchunks) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          s16x8 bu;
          if constexpr (F8) {
            const ks_u32x4 wv = b8[j][u >> 1];
            bu = (u & 1) ? f8x8_to_bf16(wv[2], wv[3]) : f8x8_to_bf16(wv[0], wv[1]);
          } else {
            bu = b[j][u];
          }
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[t] = mfma16(a[j][u][t], bu, acc[t]);
        }
        if (c + DEPTH < nchunks) load(j, c + DEPTH);
      }
    }
  }
  // lane holds C[m = 16 t + 4q + i][n = n0 + r]; sum the waves' tiles in wave order (deterministic)
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][4 * t + i][lane] = acc[t][i];
  if constexpr (NIN) ks_rstd(part, fz, M, K, wave, lane, rstd_s);
  __syncthreads();
  if constexpr (WT && !GLU && !RES) {
    static_assert(MT == 1, "write-through epilogue: one row tile");
    if (threadIdx.x < 128) {
      const int e = threadIdx.x;
      const int ti = e >> 5, l = (e & 31) * 2;  // columns l, l + 1 of row group ti
      const int m = 4 * (l >> 4) + ti, n = bx * 16 + (l & 15);
      float t0 = 0.f, t1 = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        t0 += red[w][ti][l];
        t1 += red[w][ti][l + 1];
      }
      if constexpr (NIN) {
        const float rs = m < M ? rstd_s[m] : 0.f;
        t0 *= rs;
        t1 *= rs;
      }
      if (m < M) {
        const uint32_t pk = static_cast<uint32_t>(f2bf(t0)) | (static_cast<uint32_t>(f2bf(t1)) << 16);
        __hip_atomic_store(reinterpret_cast<uint32_t*>(y + m * ldy + n), pk, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  for (int e = threadIdx.x; e < 256 * MT; e += 512) {
    const int ti = e >> 6, l = e & 63;  // ti = 4 t + i
    const int m = 16 * (ti >> 2) + 4 * (l >> 4) + (ti & 3), n = bx * 16 + (l & 15);
    if constexpr (GLU) {
      float g = 0.f, u = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) g += red[w][ti][l];
#pragma unroll
      for (int w = 4; w < 8; ++w) u += red[w][ti][l];
      // gate / up rounded to bf16 first, exactly as the unfused GEMM + swiglu pair
      g = bf2f(f2bf(g));
      u = bf2f(f2bf(u));
      if (m < M) y[m * ldy + n] = f2bf(silu_sk(g) * u);
    } else {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) t += red[w][ti][l];
      if constexpr (F8) t *= fz.wscale[n];
      if constexpr (NIN) t *= m < M ? rstd_s[m] : 0.f;
      if constexpr (RES) {
        if (m < M) {
          const float sv = bf2f(f2bf(bf2f(f2bf(t)) + bf2f(static_cast<bf16_t>(fz.res[m * fz.ldr + n]))));
          y[m * ldy + n] = f2bf(sv);
          sqs[m][l & 15] = sv * sv;
        }
      } else {
        if (m < M) y[m * ldy + n] = f2bf(t);
      }
    }
  }
  if constexpr (RES) {  // per-row partial sum of squares over this workgroup's 16 columns
    __syncthreads();
    if (threadIdx.x < M) {
      float t = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) t += sqs[threadIdx.x][c];
      fz.ssq_out[threadIdx.x * nblk + bx] = t;
    }
  }
}

}  // namespace dla
