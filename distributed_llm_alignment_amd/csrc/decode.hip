// Single-token decode attention over a KV cache (RLHF rollouts, teacher generation,
// eval — reference src/training/train_rlhf.py:123-124 / generate_teacher_data.py:72-79 via HF
// `generate`).
//
// Decode is bandwidth bound: each step streams the whole KV cache once. Design:
//   * split-KV (flash-decoding): grid = (splits, Hkv, B); a block owns one KV head, ALL its
//     G = Hq/Hkv query heads (GQA: the K/V rows are read once, not G times) and a 128-key chunk;
//   * rows are read cooperatively: D/8 lanes x 16 B per K/V row (one 256-byte row per 16 lanes
//     for D = 128, 4 rows per wave instruction, fully coalesced); each lane keeps its 8-dim slice
//     of the G query vectors in registers; dot products reduce across the row's lanes by
//     shuffles; P.V accumulates per lane and reduces across row groups, then across waves;
//   * partial (m, l, o) per split in fp32, merged by `decode_combine_kernel`.
// Lengths are DEVICE values (kv_len scalar, per-row kv_start for left padding), so the same
// launch replays inside a captured hipGraph while the cache grows; splits beyond kv_len exit.
#include <algorithm>

#include "common.h"

namespace dla {

constexpr int kDecChunk = 128;  // keys per block (4 waves x 32)

// Lanes cooperate on rows: LPK = D/8 lanes x 16 B cover one K/V row (coalesced 256-byte rows
// for D = 128), KPI = 64/LPK rows per wave instruction.
// Fused decode-step prologue (ROPE = true): instead of a separate rope + cache-write launch, the
// kernel reads the raw qkv row of the newest token: every block rotates its G query heads while
// filling `qs`; the newest key's K/V (rotated k, plain v) come from registers rather than the
// cache, and the block whose split holds that key writes them into the cache slot for the next
// steps. Rounding matches rope_cache_kernel + the unfused kernel (q and k rounded to bf16 after
// the rotation), so fused and unfused decode agree bitwise.
struct DecRope {
  const bf16_t* qkv;  // [B, (Hq + 2 Hkv) * D] rows of the newest token
  int64_t ld;
  const float* cos_t;  // [P, rot/2]
  const float* sin_t;
  const int* pos;      // [B] rope position of the newest token
  const int64_t* slot; // cache slot of the newest token (== kv_len - 1)
  int rot;
  int Hkv;
};

// 8 rotated dims [d0, d0 + 8) of one head (rotate-half over the first `rot` dims), rounded to bf16
__device__ __forceinline__ bf16x8 dec_rope8(const bf16_t* src, int d0, int rot, const float* cs,
                                            const float* sn) {
  const bf16x8 x = load_bf16x8(src + d0);
  if (d0 >= rot) return x;
  const int half = rot >> 1;
  const bool lo = d0 < half;
  const bf16x8 y = load_bf16x8(src + (lo ? d0 + half : d0 - half));
  const int c0 = lo ? d0 : d0 - half;
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float c = cs[c0 + j], s = sn[c0 + j], a = bf2f(x[j]), bb = bf2f(y[j]);
    o[j] = f2bf(lo ? a * c - bb * s : a * c + bb * s);
  }
  return o;
}

template <int D, int G, bool ROPE>
__global__ __launch_bounds__(256) void decode_attn_kernel(
    const bf16_t* __restrict__ q, int64_t q_sb, int64_t q_sh,     // q [B, Hq, D]
    bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,              // [B, Tmax, Hkv, D]
    int64_t c_sb, int64_t c_st, int64_t c_sh, const int* __restrict__ kv_len,
    const int* __restrict__ kv_start, int window, float scale_log2, int nsplit,
    float* __restrict__ part_o,  // [B, Hq, nsplit, D]
    float* __restrict__ part_ml, // [B, Hq, nsplit, 2]
    int Hq, DecRope rp) {
  constexpr int LPK = D / 8, KPI = 64 / LPK, KPW = kDecChunk / 4;
  __shared__ float qs[G][D];
  __shared__ float ps[G][kDecChunk];
  __shared__ float red[G][4];
  __shared__ float acc_s[4][G][D];
  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int len = kv_len[0];
  // fused prologue: the newest token's K / V slice of this lane (dims dl .. dl + 7)
  bf16x8 knew = {}, vnew = {};
  int newest = -1;
  if constexpr (ROPE) {
    newest = static_cast<int>(rp.slot[0]);
    const int dl0 = (lane % LPK) * 8;
    const bf16_t* row = rp.qkv + (int64_t)b * rp.ld;
    const int half = rp.rot >> 1;
    const float* cs = rp.cos_t + (int64_t)rp.pos[b] * half;
    const float* sn = rp.sin_t + (int64_t)rp.pos[b] * half;
    knew = dec_rope8(row + (int64_t)(Hq + hk) * D, dl0, rp.rot, cs, sn);
    vnew = load_bf16x8(row + (int64_t)(Hq + rp.Hkv + hk) * D + dl0);
    if (split == newest / kDecChunk && wv == 0 && lane < LPK) {  // cache write for later steps
      store_bf16x8(kc + (int64_t)b * c_sb + (int64_t)newest * c_st + (int64_t)hk * c_sh + dl0, knew);
      store_bf16x8(vc + (int64_t)b * c_sb + (int64_t)newest * c_st + (int64_t)hk * c_sh + dl0, vnew);
    }
  }
  int lo = kv_start ? kv_start[b] : 0;
  if (window > 0) lo = max(lo, len - window);
  const int base = split * kDecChunk;
  const int k0 = max(base, lo), k1 = min(base + kDecChunk, len);
  const int64_t pbase = ((int64_t)b * Hq + (int64_t)hk * G) * nsplit + split;
  if (k0 >= k1) {  // empty split (beyond the current length or fully masked)
    if (tid < G) {
      part_ml[(pbase + (int64_t)tid * nsplit) * 2 + 0] = -INFINITY;
      part_ml[(pbase + (int64_t)tid * nsplit) * 2 + 1] = 0.f;
    }
    return;
  }
  if constexpr (ROPE) {
    const bf16_t* row = rp.qkv + (int64_t)b * rp.ld;
    const int half = rp.rot >> 1;
    const float* cs = rp.cos_t + (int64_t)rp.pos[b] * half;
    const float* sn = rp.sin_t + (int64_t)rp.pos[b] * half;
    for (int i = tid; i < G * (D / 8); i += 256) {
      const int g = i / (D / 8), d0 = (i % (D / 8)) * 8;
      const bf16x8 qv = dec_rope8(row + (int64_t)(hk * G + g) * D, d0, rp.rot, cs, sn);
#pragma unroll
      for (int j = 0; j < 8; ++j) qs[g][d0 + j] = bf2f(qv[j]) * scale_log2;
    }
  } else {
    for (int i = tid; i < G * D; i += 256) {
      const int g = i / D, d = i % D;
      qs[g][d] = bf2f(q[(int64_t)b * q_sb + (int64_t)(hk * G + g) * q_sh + d]) * scale_log2;
    }
  }
  __syncthreads();
  const int sub = lane / LPK, dl = (lane % LPK) * 8;
  const bf16_t* kbase = kc + (int64_t)b * c_sb + (int64_t)hk * c_sh + dl;
  const bf16_t* vbase = vc + (int64_t)b * c_sb + (int64_t)hk * c_sh + dl;
  float qr[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) qr[g][j] = qs[g][dl + j];
  // ---- phase 1: scores (log2 domain). All of the wave's K rows are loaded up front
  // (unconditional loads at clamped keys, so the NIT 16-byte loads issue back to back and the
  // wave has them all in flight), then consumed.
  constexpr int NIT = KPW / KPI;
  bf16x8 kvr[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int key = min(max(base + wv * KPW + it * KPI + sub, k0), k1 - 1);
    kvr[it] = load_bf16x8(kbase + (int64_t)key * c_st);
    if constexpr (ROPE) {
      if (key == newest) kvr[it] = knew;
    }
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int kl = wv * KPW + it * KPI + sub;  // key within the chunk
    const int key = base + kl;
    const bool ok = key >= k0 && key < k1;
    float s[G];
#pragma unroll
    for (int g = 0; g < G; ++g) s[g] = 0.f;
    {
      const bf16x8 kv = kvr[it];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float kf = bf2f(kv[j]);
#pragma unroll
        for (int g = 0; g < G; ++g) s[g] += qr[g][j] * kf;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int o = 1; o < LPK; o <<= 1) s[g] += __shfl_xor(s[g], o, 64);
    }
    if ((lane % LPK) == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) ps[g][kl] = ok ? s[g] : -INFINITY;
    }
  }
  __syncthreads();
  // ---- softmax over the chunk: thread t < 128 owns key t for every head
  float mg[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float v = tid < kDecChunk ? ps[g][tid] : -INFINITY;
    const float m = wave_max(v);
    if (lane == 0) red[g][wv] = m;
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g) mg[g] = fmaxf(fmaxf(red[g][0], red[g][1]), fmaxf(red[g][2], red[g][3]));
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float p = 0.f;
    if (tid < kDecChunk) {
      const float sv = ps[g][tid];
      p = sv == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(sv - mg[g]);
      ps[g][tid] = p;
    }
    const float l = wave_sum(p);
    if (lane == 0) red[g][wv] = l;
  }
  __syncthreads();
  // ---- phase 2: o[g][d] = sum_key p[g][key] v[key][d]; wave wv owns keys [wv*KPW, wv*KPW+KPW)
  float o[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) o[g][j] = 0.f;
  bf16x8 vvr[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int key = min(max(base + wv * KPW + it * KPI + sub, k0), k1 - 1);
    vvr[it] = load_bf16x8(vbase + (int64_t)key * c_st);
    if constexpr (ROPE) {
      if (key == newest) vvr[it] = vnew;
    }
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int kl = wv * KPW + it * KPI + sub;  // p = 0 outside [k0, k1) (set above)
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float p = ps[g][kl];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[g][j] += p * bf2f(vvr[it][j]);
    }
  }
  // reduce the KPI key sub-groups of the wave (lanes sharing dl)
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int off = LPK; off < 64; off <<= 1) o[g][j] += __shfl_xor(o[g][j], off, 64);
  if (sub == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc_s[wv][g][dl + j] = o[g][j];
  }
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

// Decode-step prologue: rotate q (-> q_out [B, Hq, D]) and k of the newest token and write k and
// v straight into the cache slot `*slot` (device value), replacing rope + two index_copy
// launches. qkv [B, (Hq + 2 Hkv) * D] rows; same rotate-half math as rope.hip.
__global__ __launch_bounds__(256) void rope_cache_kernel(
    const bf16_t* __restrict__ qkv, int64_t ld, bf16_t* __restrict__ q_out,
    bf16_t* __restrict__ kc, bf16_t* __restrict__ vc, int64_t c_sb, int64_t c_st, int64_t c_sh,
    const int64_t* __restrict__ slot, const float* __restrict__ cos_t,
    const float* __restrict__ sin_t, const int* __restrict__ pos, int B, int Hq, int Hkv, int D,
    int rot) {
  const int dv = D >> 3, heads = Hq + 2 * Hkv, half = rot >> 1, hv = half >> 3;
  const int64_t total = (int64_t)B * heads * dv;
  const int64_t t_slot = slot[0];
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int v = (int)(i % dv);
    const int h = (int)((i / dv) % heads);
    const int b = (int)(i / ((int64_t)dv * heads));
    const bf16_t* s = qkv + (int64_t)b * ld + (int64_t)h * D;
    bf16_t* d;
    if (h < Hq) d = q_out + ((int64_t)b * Hq + h) * D;
    else if (h < Hq + Hkv) d = kc + (int64_t)b * c_sb + t_slot * c_st + (int64_t)(h - Hq) * c_sh;
    else d = vc + (int64_t)b * c_sb + t_slot * c_st + (int64_t)(h - Hq - Hkv) * c_sh;
    if (h < Hq + Hkv && v < hv) {
      const int p = pos[b];
      const float* cp = cos_t + (int64_t)p * half + v * 8;
      const float* sp = sin_t + (int64_t)p * half + v * 8;
      bf16x8 lo = load_bf16x8(s + v * 8), hi = load_bf16x8(s + half + v * 8), olo, ohi;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = cp[j], sn = sp[j], a = bf2f(lo[j]), bb = bf2f(hi[j]);
        olo[j] = f2bf(a * c - bb * sn);
        ohi[j] = f2bf(bb * c + a * sn);
      }
      store_bf16x8(d + v * 8, olo);
      store_bf16x8(d + half + v * 8, ohi);
    } else if (h >= Hq + Hkv || v >= 2 * hv) {
      store_bf16x8(d + v * 8, load_bf16x8(s + v * 8));
    }
  }
}

void launch_rope_cache(const bf16_t* qkv, int64_t ld, bf16_t* q_out, bf16_t* kc, bf16_t* vc,
                       int64_t c_sb, int64_t c_st, int64_t c_sh, const int64_t* slot,
                       const float* cos_t, const float* sin_t, const int* pos, int B, int Hq,
                       int Hkv, int D, int rot, hipStream_t st) {
  const int64_t work = (int64_t)B * (Hq + 2 * Hkv) * (D / 8);
  const int grid = (int)std::min<int64_t>((work + 255) / 256, 1024);
  rope_cache_kernel<<<grid, 256, 0, st>>>(qkv, ld, q_out, kc, vc, c_sb, c_st, c_sh, slot, cos_t,
                                          sin_t, pos, B, Hq, Hkv, D, rot);
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
static void launch_decode_d(const bf16_t* q, int64_t q_sb, int64_t q_sh, bf16_t* kc,
                            bf16_t* vc, int64_t c_sb, int64_t c_st, int64_t c_sh,
                            const int* kv_len, const int* kv_start, int window, float scale_log2,
                            int B, int Hq, int Hkv, int Tmax, float* part_o, float* part_ml,
                            bf16_t* out, int64_t o_sb, int64_t o_sh, const DecRope* rp,
                            hipStream_t st) {
  const int G = Hq / Hkv;
  const int nsplit = (Tmax + kDecChunk - 1) / kDecChunk;
  dim3 grid(nsplit, Hkv, B);
  const DecRope r0 = rp ? *rp : DecRope{};
#define DLA_DEC(GG)                                                                              \
  if (rp)                                                                                        \
    decode_attn_kernel<D, GG, true><<<grid, 256, 0, st>>>(q, q_sb, q_sh, kc, vc, c_sb, c_st,    \
                                                          c_sh, kv_len, kv_start, window,       \
                                                          scale_log2, nsplit, part_o, part_ml,  \
                                                          Hq, r0);                              \
  else                                                                                           \
    decode_attn_kernel<D, GG, false><<<grid, 256, 0, st>>>(q, q_sb, q_sh, kc, vc, c_sb, c_st,   \
                                                           c_sh, kv_len, kv_start, window,      \
                                                           scale_log2, nsplit, part_o, part_ml, \
                                                           Hq, r0)
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

void launch_decode_attn(const bf16_t* q, int64_t q_sb, int64_t q_sh, bf16_t* kc,
                        bf16_t* vc, int64_t c_sb, int64_t c_st, int64_t c_sh,
                        const int* kv_len, const int* kv_start, int window, float scale_log2, int B,
                        int Hq, int Hkv, int D, int Tmax, float* part_o, float* part_ml,
                        bf16_t* out, int64_t o_sb, int64_t o_sh, hipStream_t st) {
  if (D == 128)
    launch_decode_d<128>(q, q_sb, q_sh, kc, vc, c_sb, c_st, c_sh, kv_len, kv_start, window,
                         scale_log2, B, Hq, Hkv, Tmax, part_o, part_ml, out, o_sb, o_sh, nullptr, st);
  else
    launch_decode_d<64>(q, q_sb, q_sh, kc, vc, c_sb, c_st, c_sh, kv_len, kv_start, window,
                        scale_log2, B, Hq, Hkv, Tmax, part_o, part_ml, out, o_sb, o_sh, nullptr, st);
}

// rope + cache write of the newest token fused into the decode attention (see DecRope)
void launch_decode_attn_rope(const bf16_t* qkv, int64_t ld, const float* cos_t, const float* sin_t,
                             const int* pos, const int64_t* slot, int rot, bf16_t* kc, bf16_t* vc,
                             int64_t c_sb, int64_t c_st, int64_t c_sh, const int* kv_len,
                             const int* kv_start, int window, float scale_log2, int B, int Hq,
                             int Hkv, int D, int Tmax, float* part_o, float* part_ml, bf16_t* out,
                             int64_t o_sb, int64_t o_sh, hipStream_t st) {
  const DecRope rp{qkv, ld, cos_t, sin_t, pos, slot, rot, Hkv};
  if (D == 128)
    launch_decode_d<128>(nullptr, 0, 0, kc, vc, c_sb, c_st, c_sh, kv_len, kv_start, window,
                         scale_log2, B, Hq, Hkv, Tmax, part_o, part_ml, out, o_sb, o_sh, &rp, st);
  else
    launch_decode_d<64>(nullptr, 0, 0, kc, vc, c_sb, c_st, c_sh, kv_len, kv_start, window,
                        scale_log2, B, Hq, Hkv, Tmax, part_o, part_ml, out, o_sb, o_sh, &rp, st);
}

}  // namespace dla
