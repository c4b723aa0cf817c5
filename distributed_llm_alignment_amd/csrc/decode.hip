// Single-token decode attention over a KV cache (RLHF rollouts, teacher generation,
// eval — reference src/training/train_rlhf.py:123-124 / generate_teacher_data.py:72-79 via HF
// `generate`).
//
// Decode is bandwidth bound: each step streams the whole KV cache once. Design:
//   * split-KV (flash-decoding): grid = (splits, Hkv, B); a block owns one KV head, ALL its
//     G = Hq/Hkv query heads (GQA: the K/V rows are read once, not G times) and a 256-key chunk;
//   * phase 1: one thread per key — the K row (D bf16) is streamed with 16-byte loads, q comes
//     from LDS as a broadcast, G dot products per thread;
//   * phase 2: lanes over the head dim (coalesced 256-byte V rows), 4 waves over 64-key quarters,
//     probabilities from LDS;
//   * partial (m, l, o) per split in fp32, merged by `decode_combine_kernel`.
// Lengths are DEVICE values (kv_len scalar, per-row kv_start for left padding), so the same
// launch replays inside a captured hipGraph while the cache grows; splits beyond kv_len exit.
#include "common.h"

namespace dla {

constexpr int kDecChunk = 256;

template <int D, int G>
__global__ __launch_bounds__(256) void decode_attn_kernel(
    const bf16_t* __restrict__ q, int64_t q_sb, int64_t q_sh,     // q [B, Hq, D]
    const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,  // [B, Tmax, Hkv, D]
    int64_t c_sb, int64_t c_st, int64_t c_sh, const int* __restrict__ kv_len,
    const int* __restrict__ kv_start, int window, float scale_log2, int nsplit,
    float* __restrict__ part_o,  // [B, Hq, nsplit, D]
    float* __restrict__ part_ml, // [B, Hq, nsplit, 2]
    int Hq) {
  __shared__ float qs[G][D];
  __shared__ float ps[G][kDecChunk];
  __shared__ float red[G][4];
  __shared__ float acc_s[4][G][D];
  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int len = kv_len[0];
  int lo = kv_start ? kv_start[b] : 0;
  if (window > 0) lo = max(lo, len - window);
  const int k0 = max(split * kDecChunk, lo), k1 = min((split + 1) * kDecChunk, len);
  const int64_t pbase = ((int64_t)b * Hq + (int64_t)hk * G) * nsplit + split;
  if (k0 >= k1) {  // empty split (beyond the current length or fully masked)
    if (tid < G) {
      part_ml[(pbase + (int64_t)tid * nsplit) * 2 + 0] = -INFINITY;
      part_ml[(pbase + (int64_t)tid * nsplit) * 2 + 1] = 0.f;
    }
    return;
  }
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    qs[g][d] = bf2f(q[(int64_t)b * q_sb + (int64_t)(hk * G + g) * q_sh + d]) * scale_log2;
  }
  __syncthreads();
  // ---- phase 1: scores (log2 domain), thread per key
  const int key = split * kDecChunk + tid;
  float s[G];
#pragma unroll
  for (int g = 0; g < G; ++g) s[g] = -INFINITY;
  if (key >= k0 && key < k1) {
    const bf16_t* krow = kc + (int64_t)b * c_sb + (int64_t)key * c_st + (int64_t)hk * c_sh;
#pragma unroll
    for (int g = 0; g < G; ++g) s[g] = 0.f;
#pragma unroll 4
    for (int d8 = 0; d8 < D / 8; ++d8) {
      const bf16x8 kv = load_bf16x8(krow + d8 * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float kf = bf2f(kv[j]);
#pragma unroll
        for (int g = 0; g < G; ++g) s[g] += qs[g][d8 * 8 + j] * kf;
      }
    }
  }
  // block max per head
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float m = wave_max(s[g]);
    if (lane == 0) red[g][wv] = m;
  }
  __syncthreads();
  float mg[G];
#pragma unroll
  for (int g = 0; g < G; ++g) mg[g] = fmaxf(fmaxf(red[g][0], red[g][1]), fmaxf(red[g][2], red[g][3]));
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float p = (key >= k0 && key < k1) ? __builtin_amdgcn_exp2f(s[g] - mg[g]) : 0.f;
    ps[g][tid] = p;
    const float l = wave_sum(p);
    if (lane == 0) red[g][wv] = l;
  }
  __syncthreads();
  // ---- phase 2: o[g][d] = sum_key p[g][key] * v[key][d]; wave wv covers keys [64 wv, 64 wv + 64)
  constexpr int DPT = D / 64;  // dims per lane
  float o[G][DPT];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < DPT; ++j) o[g][j] = 0.f;
  const int kb = split * kDecChunk + wv * 64;
  const int ka = max(kb, k0), ke = min(kb + 64, k1);
  for (int kk = ka; kk < ke; ++kk) {
    const bf16_t* vrow = vc + (int64_t)b * c_sb + (int64_t)kk * c_st + (int64_t)hk * c_sh + lane * DPT;
    float vf[DPT];
    if constexpr (DPT == 2) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(vrow);
      vf[0] = bf2f(w & 0xffff);
      vf[1] = bf2f(w >> 16);
    } else {
      vf[0] = bf2f(vrow[0]);
    }
    const int pi = kk - split * kDecChunk;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float p = ps[g][pi];
#pragma unroll
      for (int j = 0; j < DPT; ++j) o[g][j] += p * vf[j];
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < DPT; ++j) acc_s[wv][g][lane * DPT + j] = o[g][j];
  __syncthreads();
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    const float v = acc_s[0][g][d] + acc_s[1][g][d] + acc_s[2][g][d] + acc_s[3][g][d];
    part_o[(pbase + (int64_t)g * nsplit) * D + d] = v;
  }
  if (tid < G) {
    part_ml[(pbase + (int64_t)tid * nsplit) * 2 + 0] = mg[tid];
    part_ml[(pbase + (int64_t)tid * nsplit) * 2 + 1] = red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3];
  }
}

// one block per (b, h): merge the splits (log2-domain running max)
template <int D>
__global__ __launch_bounds__(64) void decode_combine_kernel(const float* __restrict__ part_o,
                                                             const float* __restrict__ part_ml,
                                                             int nsplit, bf16_t* __restrict__ out,
                                                             int64_t o_sb, int64_t o_sh, int Hq) {
  const int bh = blockIdx.x;
  const int b = bh / Hq, h = bh % Hq;
  const float* ml = part_ml + (int64_t)bh * nsplit * 2;
  float m = -INFINITY;
  for (int s = 0; s < nsplit; ++s) m = fmaxf(m, ml[2 * s]);
  constexpr int DPT = D / 64;
  float acc[DPT] = {};
  float l = 0.f;
  if (m != -INFINITY) {
    for (int s = 0; s < nsplit; ++s) {
      const float ms = ml[2 * s];
      if (ms == -INFINITY) continue;
      const float c = __builtin_amdgcn_exp2f(ms - m);
      l += c * ml[2 * s + 1];
#pragma unroll
      for (int j = 0; j < DPT; ++j)
        acc[j] += c * part_o[((int64_t)bh * nsplit + s) * D + threadIdx.x * DPT + j];
    }
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
  for (int j = 0; j < DPT; ++j)
    out[(int64_t)b * o_sb + (int64_t)h * o_sh + threadIdx.x * DPT + j] = f2bf(acc[j] * inv);
}

template <int D>
static void launch_decode_d(const bf16_t* q, int64_t q_sb, int64_t q_sh, const bf16_t* kc,
                            const bf16_t* vc, int64_t c_sb, int64_t c_st, int64_t c_sh,
                            const int* kv_len, const int* kv_start, int window, float scale_log2,
                            int B, int Hq, int Hkv, int Tmax, float* part_o, float* part_ml,
                            bf16_t* out, int64_t o_sb, int64_t o_sh, hipStream_t st) {
  const int G = Hq / Hkv;
  const int nsplit = (Tmax + kDecChunk - 1) / kDecChunk;
  dim3 grid(nsplit, Hkv, B);
#define DLA_DEC(GG)                                                                              \
  decode_attn_kernel<D, GG><<<grid, 256, 0, st>>>(q, q_sb, q_sh, kc, vc, c_sb, c_st, c_sh,      \
                                                   kv_len, kv_start, window, scale_log2, nsplit, \
                                                   part_o, part_ml, Hq)
  switch (G) {
    case 1: DLA_DEC(1); break;
    case 2: DLA_DEC(2); break;
    case 4: DLA_DEC(4); break;
    case 8: DLA_DEC(8); break;
    default: break;  // validated on the host
  }
#undef DLA_DEC
  decode_combine_kernel<D><<<B * Hq, 64, 0, st>>>(part_o, part_ml, nsplit, out, o_sb, o_sh, Hq);
}

int decode_num_splits(int Tmax) { return (Tmax + kDecChunk - 1) / kDecChunk; }

void launch_decode_attn(const bf16_t* q, int64_t q_sb, int64_t q_sh, const bf16_t* kc,
                        const bf16_t* vc, int64_t c_sb, int64_t c_st, int64_t c_sh,
                        const int* kv_len, const int* kv_start, int window, float scale_log2, int B,
                        int Hq, int Hkv, int D, int Tmax, float* part_o, float* part_ml,
                        bf16_t* out, int64_t o_sb, int64_t o_sh, hipStream_t st) {
  if (D == 128)
    launch_decode_d<128>(q, q_sb, q_sh, kc, vc, c_sb, c_st, c_sh, kv_len, kv_start, window,
                         scale_log2, B, Hq, Hkv, Tmax, part_o, part_ml, out, o_sb, o_sh, st);
  else
    launch_decode_d<64>(q, q_sb, q_sh, kc, vc, c_sb, c_st, c_sh, kv_len, kv_start, window,
                        scale_log2, B, Hq, Hkv, Tmax, part_o, part_ml, out, o_sb, o_sh, st);
}

}  // namespace dla
