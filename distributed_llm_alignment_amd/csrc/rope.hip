// Rotary position embedding, rotate-half convention with optional partial rotary
// (phi-2 rotates the first 32 of 80 dims). Reference: HF `apply_rotary_pos_emb`, reached through
// every attention forward of src/models/base_model.py:30-34 models.
//
// Forward reads the fused QKV GEMM output qkv[B*T, (Hq+2*Hkv)*D] (row stride ld) and writes
// rotated q[B*T, Hq, D] and k[B*T, Hkv, D] contiguous for the attention kernel; v is consumed
// in place by attention (no copy). Backward reads dq/dk (rotated space) and writes the
// un-rotated gradient straight into the q/k column slices of the fused dqkv buffer, so the
// QKV weight-gradient GEMM consumes one buffer with no cat/split copies.
//
// cos/sin come from a host-precomputed fp32 table [max_pos, rot/2] (Appendix B: no on-device
// trig). A thread handles 8 rotary pairs (16 B of the low half + 16 B of the high half).
#include "common.h"

namespace dla {

template <bool BWD>
__global__ __launch_bounds__(256) void rope_kernel(
    const bf16_t* __restrict__ q_src, const bf16_t* __restrict__ k_src, int64_t q_src_ld,
    int64_t k_src_ld, bf16_t* __restrict__ q_dst, bf16_t* __restrict__ k_dst, int64_t q_dst_ld,
    int64_t k_dst_ld, const float* __restrict__ cos_t, const float* __restrict__ sin_t,
    const int* __restrict__ pos, int64_t tokens, int T, int pos_offset, int Hq, int Hkv, int D,
    int rot) {
  // work item = (token, head, item): items [0, hv) rotate one pair of 8-column chunks (v, v + hv),
  // items [hv, dv - hv) copy one pass-through chunk (partial rotary). No idle lanes: an item per
  // vec8 of the head would leave the hv high-half chunks' threads with nothing to do.
  const int dv = D >> 3;
  const int heads = Hq + Hkv;
  const int half = rot >> 1;
  const int hv = half >> 3;  // rotary pairs handled per head, in vec8 units
  const int per = dv - hv;   // items per head
  const int64_t total = tokens * heads * per;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int it = static_cast<int>(i % per);
    const int v = it < hv ? it : it + hv;  // rotary pair v, or pass-through chunk v >= 2 hv
    const int64_t th = i / per;
    const int h = static_cast<int>(th % heads);
    const int64_t tok = th / heads;
    const bool isq = h < Hq;
    const int64_t hoff = static_cast<int64_t>(isq ? h : h - Hq) * D;
    const bf16_t* s = (isq ? q_src + tok * q_src_ld : k_src + tok * k_src_ld) + hoff;
    bf16_t* d = (isq ? q_dst + tok * q_dst_ld : k_dst + tok * k_dst_ld) + hoff;
    if (v < hv) {
      const int p = pos ? pos[tok] : static_cast<int>(tok % T) + pos_offset;
      const float* cp = cos_t + static_cast<int64_t>(p) * half + v * 8;
      const float* sp = sin_t + static_cast<int64_t>(p) * half + v * 8;
      bf16x8 lo = load_bf16x8(s + v * 8), hi = load_bf16x8(s + half + v * 8), olo, ohi;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = cp[j], sn = sp[j];
        const float a = bf2f(lo[j]), b = bf2f(hi[j]);
        if constexpr (!BWD) {
          olo[j] = f2bf(a * c - b * sn);
          ohi[j] = f2bf(b * c + a * sn);
        } else {
          olo[j] = f2bf(a * c + b * sn);
          ohi[j] = f2bf(b * c - a * sn);
        }
      }
      store_bf16x8(d + v * 8, olo);
      store_bf16x8(d + half + v * 8, ohi);
    } else if (v >= 2 * hv) {
      store_bf16x8(d + v * 8, load_bf16x8(s + v * 8));  // pass-through (partial rotary)
    }
  }
}

static inline unsigned rope_grid(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g > 2048) g = 2048;
  return static_cast<unsigned>(g < 1 ? 1 : g);
}

void launch_rope_fwd(const bf16_t* qkv, int64_t ld, bf16_t* q, bf16_t* k, const float* cos_t,
                     const float* sin_t, const int* pos, int64_t tokens, int T, int pos_offset,
                     int Hq, int Hkv, int D, int rot, hipStream_t st) {
  const int64_t work = tokens * (Hq + Hkv) * (D / 8 - rot / 16);
  rope_kernel<false><<<rope_grid(work), 256, 0, st>>>(
      qkv, qkv + static_cast<int64_t>(Hq) * D, ld, ld, q, k, static_cast<int64_t>(Hq) * D,
      static_cast<int64_t>(Hkv) * D, cos_t, sin_t, pos, tokens, T, pos_offset, Hq, Hkv, D, rot);
}

// dq [tokens, Hq*D], dk [tokens, Hkv*D] contiguous -> dqkv q/k column slices (row stride ld).
void launch_rope_bwd(const bf16_t* dq_rot, const bf16_t* dk_rot, bf16_t* dqkv, int64_t ld,
                     const float* cos_t, const float* sin_t, const int* pos, int64_t tokens,
                     int T, int pos_offset, int Hq, int Hkv, int D, int rot, hipStream_t st) {
  const int64_t work = tokens * (Hq + Hkv) * (D / 8 - rot / 16);
  rope_kernel<true><<<rope_grid(work), 256, 0, st>>>(
      dq_rot, dk_rot, static_cast<int64_t>(Hq) * D, static_cast<int64_t>(Hkv) * D, dqkv,
      dqkv + static_cast<int64_t>(Hq) * D, ld, ld, cos_t, sin_t, pos, tokens, T, pos_offset, Hq,
      Hkv, D, rot);
}

}  // namespace dla
