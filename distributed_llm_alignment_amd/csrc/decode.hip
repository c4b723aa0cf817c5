// Single-token decode attention over a KV cache (RLHF rollouts, teacher generation,
// eval — reference src/training/train_rlhf.py:123-124 / generate_teacher_data.py:72-79 via HF
// `generate`).
//
// Decode is bandwidth bound: each step streams the whole KV cache once. Design:
//   * split-KV (flash-decoding): grid = (splits, Hkv, B); a block owns one KV head, ALL its
//     G = Hq/Hkv query heads (GQA: the K/V rows are read once, not G times) and a 128-key chunk;
//   * each wave takes 32 keys of the chunk: S^T = K q^T on MFMA (K rows as A fragments), a
//     wave-local softmax, P.V on the VALU over V rows read coalesced (D/8 lanes x 16 B per row);
//     the 4 waves merge once at the end (see decode_attn_kernel);
//   * partial (m, l, o) per split in fp32, merged by `decode_combine_kernel`.
// Lengths are DEVICE values (kv_len scalar, per-row kv_start for left padding), so the same
// launch replays inside a captured hipGraph while the cache grows; splits beyond kv_len exit.
#include <algorithm>
#include <cstdlib>

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

// Element offset of 16-byte chunk `ch` of key row `row` in a wave's [32 keys][D] bf16 V image;
// the XOR keeps the ds_read_b64_tr_b16 column reads of the P.V MFMA spread over banks (cdna
// guide T10 layout (b)).
template <int D>
__device__ __forceinline__ int dec_swz(int row, int ch) {
  constexpr int NCH = D / 8;
  const int f = (((row & 3) << 2) | ((row >> 2) & 3)) & (NCH - 1);
  return row * D + ((ch ^ f) << 3);
}

typedef __attribute__((address_space(3))) s16x4 dec_lds_s16x4;

// ds_read_b64_tr_b16 of 4 key rows x 16 columns, column-major per 16-lane group: lane 4q + p of
// the group addresses row r0 + q, columns c0 + 4p .. +3; lane i receives column c0 + i of the 4
// rows (row q in element q). Every lane of the wave must execute it (EXEC all ones).
template <int D>
__device__ __forceinline__ s16x4 dec_tr_read(const bf16_t* img, int r0, int c0, int lane) {
  const int i = lane & 15, q = i >> 2, pp = i & 3;
  const int ch = (c0 >> 3) + (pp >> 1), sub = (pp & 1) * 4;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((dec_lds_s16x4*)(img + dec_swz<D>(r0 + q, ch) + sub));
}

// The four waves of a block work independently until one final merge.
//   * every load is issued up front, one memory round trip: the wave's 32 K rows as MFMA A
//     fragments (lane = key, 16 B of its row per k-step), its 32 V rows in the coalesced row
//     layout, and q as the B fragment (lane = query head);
//   * S^T = K q^T with v_mfma_f32_16x16x32_bf16 (no cross-lane dot-product reductions); the
//     lane holding (head g, 8 keys) runs a wave-local online softmax with 2 cross-lane steps;
//   * P^T goes to the V row layout through a wave-private LDS slice, P.V on the VALU, and the 4
//     waves' (m, l, o) are merged after the block's single barrier.
// The previous version (one block-wide softmax: 6 barriers, the V loads behind the scores):
// 17.3 -> 16.4 us per layer in a Llama-3-8B B=8 decode step. Neither the grid order (kv head
// fastest) nor a head-major cache layout changed the time (tools/decode_attn_bench.py).
// P.V on MFMA: the exponentiated scores stay in the S^T accumulator layout (lane = head g,
// keys {4kg .. 4kg+3, 16+4kg .. 16+4kg+3}), which IS the A operand of v_mfma_f32_16x16x32_bf16
// once packed to bf16 (k permuted the same way on both operands); V goes through a wave-private
// swizzled LDS image and comes back as the B operand by ds_read_b64_tr_b16 (cdna guide T10). The
// (The VALU P.V form it replaced -- P through LDS, 8 x G FMAs per key and lane -- was deleted in
// round 6; git history has it.)
template <int D, int G, bool ROPE>
__global__ __launch_bounds__(256, 3) void decode_attn_kernel(
    const bf16_t* __restrict__ q, int64_t q_sb, int64_t q_sh,     // q [B, Hq, D]
    bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,              // [B, Tmax, Hkv, D]
    int64_t c_sb, int64_t c_st, int64_t c_sh, const int* __restrict__ kv_len,
    const int* __restrict__ kv_start, int window, float scale_log2, int nsplit,
    float* __restrict__ part_o,  // [B, Hq, nsplit, D]
    float* __restrict__ part_ml, // [B, Hq, nsplit, 2]
    int Hq, DecRope rp, int Tcap) {
  constexpr int LPK = D / 8, KPI = 64 / LPK, KPW = kDecChunk / 4, NIT = KPW / KPI;
  constexpr int KST = D / 32;  // MFMA k-steps over the head dim
  static_assert(G <= 16 && KPW == 32, "decode tile geometry");
  __shared__ __attribute__((aligned(16))) bf16_t vimg[4][KPW * D];
  __shared__ float acc_s[4][G][D];
  __shared__ float mls[4][G][2];
  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int len = kv_len[0];
  // the row's first visible key, loaded together with kv_len ahead of the newest-token prologue
  // (one scalar round trip before the bulk K / V loads; measured neutral vs after the prologue)
  int lo = kv_start ? kv_start[b] : 0;
  const int sub = lane / LPK, dl = (lane % LPK) * 8;  // V row layout
  const int r16 = lane & 15, kg = lane >> 4;           // MFMA fragment layout
  bf16x8 vnew = {};
  int newest = -1;
  const bf16_t* qrow = nullptr;
  const float *cs = nullptr, *sn = nullptr;
  if constexpr (ROPE) {
    newest = static_cast<int>(rp.slot[0]);
    qrow = rp.qkv + (int64_t)b * rp.ld;
    const int half = rp.rot >> 1;
    cs = rp.cos_t + (int64_t)rp.pos[b] * half;
    sn = rp.sin_t + (int64_t)rp.pos[b] * half;
    vnew = load_bf16x8(qrow + (int64_t)(Hq + rp.Hkv + hk) * D + dl);
    if (split == newest / kDecChunk && wv == 0 && lane < LPK) {  // cache write for later steps
      const bf16x8 knew = dec_rope8(qrow + (int64_t)(Hq + hk) * D, dl, rp.rot, cs, sn);
      store_bf16x8(kc + (int64_t)b * c_sb + (int64_t)newest * c_st + (int64_t)hk * c_sh + dl, knew);
      store_bf16x8(vc + (int64_t)b * c_sb + (int64_t)newest * c_st + (int64_t)hk * c_sh + dl, vnew);
    }
  }
  const int base = split * kDecChunk;
  const int kw0 = base + wv * KPW;  // this wave's first key
  const bf16_t* kb0 = kc + (int64_t)b * c_sb + (int64_t)hk * c_sh;
  const bf16_t* vb0 = vc + (int64_t)b * c_sb + (int64_t)hk * c_sh + dl;
  // ---- all loads up front. K rows are clamped only into the cache capacity, so they leave at
  // kernel start without waiting for kv_len / kv_start (rows outside [k0, k1) are masked out of
  // the scores: whatever they hold is discarded); V rows are clamped into [k0, k1) (a masked
  // key's weight is 0 and its row must be finite). The newest key's rotated K / raw V (a
  // dependent chain through pos -> cos / sin) replace their registers only afterwards.
  s16x8 kf[2][KST];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int kcl = min(kw0 + 16 * t + r16, Tcap - 1);
#pragma unroll
    for (int s = 0; s < KST; ++s)
      kf[t][s] = __builtin_bit_cast(s16x8, load_bf16x8(kb0 + (int64_t)kcl * c_st + 32 * s + 8 * kg));
  }
  if (window > 0) lo = max(lo, len - window);
  const int k0 = max(base, lo), k1 = min(base + kDecChunk, len);
  const int64_t pbase = ((int64_t)b * Hq + (int64_t)hk * G) * nsplit + split;
  if (k0 >= k1) {  // empty split (beyond the current length or fully masked)
    if (tid < G) {
      part_ml[(pbase + (int64_t)tid * nsplit) * 2 + 0] = -INFINITY;
      part_ml[(pbase + (int64_t)tid * nsplit) * 2 + 1] = 0.f;
    }
    return;
  }
  bf16x8 vvr[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int key = min(max(kw0 + it * KPI + sub, k0), k1 - 1);
    vvr[it] = load_bf16x8(vb0 + (int64_t)key * c_st);
  }
  if constexpr (ROPE) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (min(kw0 + 16 * t + r16, Tcap - 1) == newest) {
#pragma unroll
        for (int s = 0; s < KST; ++s)
          kf[t][s] = __builtin_bit_cast(s16x8, dec_rope8(qrow + (int64_t)(Hq + hk) * D, 32 * s + 8 * kg, rp.rot, cs, sn));
      }
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it)
      if (min(max(kw0 + it * KPI + sub, k0), k1 - 1) == newest) vvr[it] = vnew;
  }
  s16x8 qf[KST];
#pragma unroll
  for (int s = 0; s < KST; ++s) {
    qf[s] = s16x8{};
    if (r16 < G) {
      if constexpr (ROPE)
        qf[s] = __builtin_bit_cast(s16x8, dec_rope8(qrow + (int64_t)(hk * G + r16) * D, 32 * s + 8 * kg, rp.rot, cs, sn));
      else
        qf[s] = __builtin_bit_cast(s16x8, load_bf16x8(q + (int64_t)b * q_sb + (int64_t)(hk * G + r16) * q_sh + 32 * s + 8 * kg));
    }
  }
  // ---- S^T[key][g]: lane holds keys kw0 + 16t + 4kg + i (i < 4) of head g = r16
  f32x4 sacc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    sacc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KST; ++s) sacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[t][s], qf[s], sacc[t], 0, 0, 0);
  }
  float sc[2][4];
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int key = kw0 + 16 * t + 4 * kg + i;
      sc[t][i] = (key >= k0 && key < k1) ? sacc[t][i] * scale_log2 : -INFINITY;
      m = fmaxf(m, sc[t][i]);
    }
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  const float muse = m == -INFINITY ? 0.f : m;
  float l = 0.f;
  // V rows -> this wave's LDS image (row = key within the wave, swizzled 16-byte chunks)
  bf16_t* vw = &vimg[wv][0];
#pragma unroll
  for (int it = 0; it < NIT; ++it)
    store_bf16x8(vw + dec_swz<D>(it * KPI + sub, dl >> 3), vvr[it]);
  float pf[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p = __builtin_amdgcn_exp2f(sc[t][i] - muse);  // exp2(-inf) = 0 for masked keys
      l += p;
      pf[t][i] = r16 < G ? p : 0.f;
    }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  // A operand: k-slot e < 4 <-> key 4kg + e, e >= 4 <-> key 16 + 4kg + e - 4
  const float pv8[8] = {pf[0][0], pf[0][1], pf[0][2], pf[0][3], pf[1][0], pf[1][1], pf[1][2], pf[1][3]};
  const s16x8 pa = __builtin_bit_cast(s16x8, pack_bf16x8(pv8));
  // wave-private image: this wave's LDS writes complete before its transposed reads
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  f32x4 oacc[D / 16];
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    const s16x4 v0 = dec_tr_read<D>(vw, 4 * kg, 16 * dt, lane);
    const s16x4 v1 = dec_tr_read<D>(vw, 16 + 4 * kg, 16 * dt, lane);
    const s16x8 vb = s16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    oacc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  }
  // lane (d = 16 dt + r16, heads 4kg + i) -> this wave's partial O
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (4 * kg + i < G) acc_s[wv][4 * kg + i][16 * dt + r16] = oacc[dt][i];
  if (kg == 0 && r16 < G) {
    mls[wv][r16][0] = m;
    mls[wv][r16][1] = l;
  }
  __syncthreads();
  // ---- merge the 4 waves (fixed order) into this split's partial
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    float mm = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) mm = fmaxf(mm, mls[w][g][0]);
    float v = 0.f, ll = 0.f;
    if (mm != -INFINITY) {
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float mw = mls[w][g][0];
        const float c = mw == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw - mm);
        v += c * acc_s[w][g][d];
        ll += c * mls[w][g][1];
      }
    }
    part_o[(pbase + (int64_t)g * nsplit) * D + d] = v;
    if (d == 0) {
      part_ml[(pbase + (int64_t)g * nsplit) * 2 + 0] = mm;
      part_ml[(pbase + (int64_t)g * nsplit) * 2 + 1] = ll;
    }
  }
}

// In-kernel split combine (decode_attn_loop_kernel with `cnt`): every block publishes its
// partial (m, l, o) with write-through (sc1) stores, waits for them (vmcnt(0) in every wave), and
// one lane adds to the (b, kv head) arrival counter; the block whose add returns nsplit - 1 re-arms
// the counter, takes ONE agent-scope acquire and merges the nsplit partials into the normalised
// bf16 output -- the decode_combine_kernel launch and its kernel boundary are gone. No block waits
// on another (no polling), so a late or empty split cannot stall the grid. Hand-off form:
// MI355X_MICROARCH "Valid forms" (sc1 stores + drained vmcnt + agent atomic; consumer acquire).
__device__ __forceinline__ void dec_pub(float* p, float v, bool wt) {
  if (wt) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

constexpr int kDecMaxFuse = 8;  // most splits the in-kernel combine merges

template <int D, int G>
__device__ __forceinline__ void dec_arrive_combine(int* __restrict__ cnt, const float* part_o,
                                                   const float* part_ml, int64_t pbase0, int nsplit,
                                                   bf16_t* __restrict__ out, int64_t o_base,
                                                   int64_t o_sh) {
  __shared__ int last_s;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == nsplit - 1;
    if (last) {
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    last_s = last;
  }
  __syncthreads();
  if (!last_s) return;
  // same merge as decode_combine_kernel (log2-domain running max, splits in ascending order),
  // every load of the (<= kDecMaxFuse) splits issued before any use: one round trip after the acquire
  constexpr int EPT = (G * D + 255) / 256;
  float mv[EPT][kDecMaxFuse], lv[EPT][kDecMaxFuse], ov[EPT][kDecMaxFuse];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int i = threadIdx.x + 256 * e;
    const int g = min(i, G * D - 1) / D, d = i % D;
    const float* ml = part_ml + (pbase0 + (int64_t)g * nsplit) * 2;
    const float* po = part_o + (pbase0 + (int64_t)g * nsplit) * D + d;
#pragma unroll
    for (int s = 0; s < kDecMaxFuse; ++s) {
      if (s < nsplit) {
        mv[e][s] = ml[2 * s];
        lv[e][s] = ml[2 * s + 1];
        ov[e][s] = po[(int64_t)s * D];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int i = threadIdx.x + 256 * e;
    if (i >= G * D) break;
    const int g = i / D, d = i % D;
    float m = -INFINITY;
#pragma unroll
    for (int s = 0; s < kDecMaxFuse; ++s)
      if (s < nsplit) m = fmaxf(m, mv[e][s]);
    float acc = 0.f, l = 0.f;
    if (m != -INFINITY) {
#pragma unroll
      for (int s = 0; s < kDecMaxFuse; ++s) {
        if (s < nsplit) {
          const float c = mv[e][s] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mv[e][s] - m);
          l += c * lv[e][s];
          acc += c == 0.f ? 0.f : c * ov[e][s];  // an empty split never wrote its o row
        }
      }
    }
    const float inv = l > 0.f ? 1.f / l : 0.f;
    out[o_base + (int64_t)g * o_sh + d] = f2bf(acc * inv);
  }
}

// Multi-chunk form (the default): grid (nsplit, Hkv, B) with each block looping over `cpb`
// consecutive 128-key chunks of its (b, kv head), chunk c + 2's K / V loads in flight while chunk
// c is computed (a 2-slot register ring), and a per-wave online softmax across the chunks. The
// host picks cpb so the grid fits in ~one round of resident blocks: at B = 64 (the reference's
// RLHF rollout batch) the one-chunk-per-block grid ran 2560 blocks in ~3.3 rounds, each block
// paying its own dependent round trips (scalars -> K/V -> merge); here 512 blocks stream ~4.5
// chunks each and the per-block prologue / merge is paid once. Numerics: the same masked
// exp2-domain softmax and P.V MFMA as decode_attn_kernel, with the running max rescale
// applied between chunks; partials (m, l, o) per split as before.
__device__ __forceinline__ void dec_glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// The loop kernel's body: a block streams chunks [cbeg, cend) of one (split, kv head, sequence)
// through a 2-deep K / V ring.
template <int D, int G, bool ROPE>
__device__ __forceinline__ void dec_loop_body(
    const int split, const int hk, const int b, const int Hkv_grid,
    const bf16_t* __restrict__ q, int64_t q_sb, int64_t q_sh,
    bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
    int64_t c_sb, int64_t c_st, int64_t c_sh, const int* __restrict__ kv_len,
    const int* __restrict__ kv_start, int window, float scale_log2, int nsplit, int cpb,
    float* __restrict__ part_o, float* __restrict__ part_ml, int Hq, const DecRope& rp,
    bf16_t* __restrict__ out, int64_t o_sb, int64_t o_sh, int* __restrict__ cnt, int Tcap) {
  // out != nullptr, cnt == nullptr (one split per sequence): the block writes the normalised bf16
  // output itself; out and cnt (nsplit > 1): partials + in-kernel combine (dec_arrive_combine).
  // Either way the combine launch is skipped.
  constexpr int LPK = D / 8, KPI = 64 / LPK, KPW = kDecChunk / 4, NIT = KPW / KPI;
  constexpr int KST = D / 32;
  static_assert(G <= 16 && KPW == 32, "decode tile geometry");
  static_assert(G * D * 4 <= KPW * D * 2, "acc_s aliases one V image slot");
  // per wave: 2 V image slots (LDS-DMA ring), the first re-used for the wave's partial O
  constexpr int RD = 2;
  __shared__ __attribute__((aligned(16))) bf16_t vimg[4][RD][KPW * D];
  __shared__ float mls[4][G][2];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int len = kv_len[0];
  int lo = kv_start ? kv_start[b] : 0;
  const int sub = lane / LPK, dl = (lane % LPK) * 8;
  const int r16 = lane & 15, kg = lane >> 4;
  int newest = -1;
  // this block's q heads, k and v of the newest token: a row of the qkv projection
  const bf16_t *qh = nullptr, *kh = nullptr, *vh = nullptr;
  const float *cs = nullptr, *sn = nullptr;
  const int cfirst = split * cpb;
  auto cache_write = [&]() {  // the newest key's rotated K / raw V into its cache slot
    if constexpr (ROPE) {
      const int cn = newest / kDecChunk;
      if (cn >= cfirst && cn < cfirst + cpb && wv == 0 && lane < LPK) {
        const bf16x8 vnew = load_bf16x8(vh + dl);
        const bf16x8 knew = dec_rope8(kh, dl, rp.rot, cs, sn);
        store_bf16x8(kc + (int64_t)b * c_sb + (int64_t)newest * c_st + (int64_t)hk * c_sh + dl, knew);
        store_bf16x8(vc + (int64_t)b * c_sb + (int64_t)newest * c_st + (int64_t)hk * c_sh + dl, vnew);
      }
    }
  };
  if constexpr (ROPE) {
    newest = static_cast<int>(rp.slot[0]);
    const bf16_t* qrow = rp.qkv + (int64_t)b * rp.ld;
    qh = qrow + (int64_t)(hk * G) * D;
    kh = qrow + (int64_t)(Hq + hk) * D;
    vh = qrow + (int64_t)(Hq + rp.Hkv + hk) * D;
    const int half = rp.rot >> 1;
    cs = rp.cos_t + (int64_t)rp.pos[b] * half;
    sn = rp.sin_t + (int64_t)rp.pos[b] * half;
    cache_write();
  }
  const bf16_t* kb0 = kc + (int64_t)b * c_sb + (int64_t)hk * c_sh;
  const bf16_t* vb0 = vc + (int64_t)b * c_sb + (int64_t)hk * c_sh;
  // 2-slot ring: K as MFMA A fragments in registers, V by LDS-DMA straight into the wave's
  // swizzled image (lane-linear destination, the swizzle applied on the per-lane SOURCE chunk:
  // image row it * KPI + sub, position dl / 8 holds logical chunk (dl / 8) ^ f(row)). K rows are
  // clamped only into the chunk and the cache capacity (no kv_len / kv_start dependence: the
  // first chunk's K loads leave at kernel start, beside the scalar length loads; rows outside
  // the visible range are masked out of the scores, so whatever they hold is discarded); V rows
  // are clamped into the visible range (a masked key's weight is 0 and its V row must be finite).
  s16x8 kf[RD][2][KST];
  auto loadK = [&](auto J, int c) {
    constexpr int j = decltype(J)::value;
    const int kw0 = c * kDecChunk + wv * KPW;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int kcl = min(kw0 + 16 * t + r16, Tcap - 1);
#pragma unroll
      for (int s = 0; s < KST; ++s)
        kf[j][t][s] = __builtin_bit_cast(s16x8, load_bf16x8(kb0 + (int64_t)kcl * c_st + 32 * s + 8 * kg));
    }
  };
  loadK(std::integral_constant<int, 0>{}, cfirst);  // speculative: the split's first chunk
  if (window > 0) lo = max(lo, len - window);
  // chunks [cbeg, cend) of this split that hold visible keys
  const int cbeg = max(cfirst, lo / kDecChunk);
  const int cend = min(cfirst + cpb, (len + kDecChunk - 1) / kDecChunk);
  const int64_t pbase = ((int64_t)b * Hq + (int64_t)hk * G) * nsplit + split;
  const bool fuse = cnt != nullptr;
  int* const cslot = fuse ? cnt + (int64_t)b * Hkv_grid + hk : nullptr;
  const int64_t pbase0 = ((int64_t)b * Hq + (int64_t)hk * G) * nsplit;
  const int64_t obase = (int64_t)b * o_sb + (int64_t)hk * G * o_sh;
  if (cbeg >= cend || max(cbeg * kDecChunk, lo) >= len) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the speculative K loads
    if (out != nullptr && !fuse) {  // no visible key: zeros, as the combine writes for an all-empty row
      for (int i = tid; i < G * D; i += 256)
        out[(int64_t)b * o_sb + (int64_t)(hk * G + i / D) * o_sh + i % D] = 0;
      return;
    }
    if (tid < G) {
      dec_pub(&part_ml[(pbase + (int64_t)tid * nsplit) * 2 + 0], -INFINITY, fuse);
      dec_pub(&part_ml[(pbase + (int64_t)tid * nsplit) * 2 + 1], 0.f, fuse);
    }
    if (fuse) dec_arrive_combine<D, G>(cslot, part_o, part_ml, pbase0, nsplit, out, obase, o_sh);
    return;
  }
  // q fragments first, the oldest loads: S of chunk 0 waits for them and K(0) only
  s16x8 qf[KST];
#pragma unroll
  for (int s = 0; s < KST; ++s) {
    qf[s] = s16x8{};
    if (r16 < G) {
      if constexpr (ROPE)
        qf[s] = __builtin_bit_cast(s16x8, dec_rope8(qh + (int64_t)r16 * D, 32 * s + 8 * kg, rp.rot, cs, sn));
      else
        qf[s] = __builtin_bit_cast(s16x8, load_bf16x8(q + (int64_t)b * q_sb + (int64_t)(hk * G + r16) * q_sh + 32 * s + 8 * kg));
    }
  }
  auto loadV = [&](auto J, int c) {
    constexpr int j = decltype(J)::value;
    const int base = c * kDecChunk, k0 = max(base, lo), k1 = min(base + kDecChunk, len);
    const int kw0 = base + wv * KPW;
    bf16_t* img = &vimg[wv][j][0];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int row = it * KPI + sub;
      const int key = min(max(kw0 + row, k0), k1 - 1);
      const int ch = (dec_swz<D>(row, dl >> 3) - row * D) >> 3;  // position dl/8 <-> chunk ch
      dec_glds16(vb0 + (int64_t)key * c_st + ch * 8, img + it * 512);
    }
  };
  auto load = [&](auto J, int c) {  // issue order per chunk: K then V
    loadK(J, c);
    loadV(J, c);
  };
  float m_run = -INFINITY, l_run = 0.f;
  f32x4 oacc[D / 16];
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) oacc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto step = [&](auto J, int c) {
    constexpr int j = decltype(J)::value;
    const int base = c * kDecChunk, k0 = max(base, lo), k1 = min(base + kDecChunk, len);
    const int kw0 = base + wv * KPW;
    const bool newest_here = ROPE && newest >= kw0 && newest < kw0 + KPW;
    if constexpr (ROPE) {  // the newest key's K comes from registers (its cache row is being written)
      if (newest_here) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if (min(kw0 + 16 * t + r16, Tcap - 1) == newest) {
#pragma unroll
            for (int s = 0; s < KST; ++s)
              kf[j][t][s] = __builtin_bit_cast(s16x8, dec_rope8(kh, 32 * s + 8 * kg, rp.rot, cs, sn));
          }
        }
      }
    }
    f32x4 sacc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sacc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KST; ++s) sacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[j][t][s], qf[s], sacc[t], 0, 0, 0);
    }
    float sc[2][4];
    float mc = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kw0 + 16 * t + 4 * kg + i;
        sc[t][i] = (key >= k0 && key < k1) ? sacc[t][i] * scale_log2 : -INFINITY;
        mc = fmaxf(mc, sc[t][i]);
      }
    mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
    mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
    const float mnew = fmaxf(m_run, mc);
    const float alpha = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_run - mnew);
    const float muse = mnew == -INFINITY ? 0.f : mnew;
    float pf[2][4], ls = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = __builtin_amdgcn_exp2f(sc[t][i] - muse);
        ls += p;
        pf[t][i] = r16 < G ? p : 0.f;
      }
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = mnew;
    const float pv8[8] = {pf[0][0], pf[0][1], pf[0][2], pf[0][3], pf[1][0], pf[1][1], pf[1][2], pf[1][3]};
    const s16x8 pa = __builtin_bit_cast(s16x8, pack_bf16x8(pv8));
    float ai[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ai[i] = __shfl(alpha, 4 * kg + i, 64);
    // V(c) has landed once every VMEM op but the next chunk's (2 KST K loads + NIT V pieces,
    // issued after it) is done; the compiler does not see the DMA -> LDS dependence
    // (chunks issued after c: min(RD - 1, cend - 1 - c); the refill of c + RD comes after this)
    constexpr int PER = 2 * KST + NIT;
    const int nlater = min(RD - 1, cend - 1 - c);
    if (nlater == 1) {
      if constexpr (PER == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if constexpr (PER == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bf16_t* vw = &vimg[wv][j][0];
    if constexpr (ROPE) {
      // Every image row whose clamped key is the newest one -- its own row, and the rows past
      // the visible range that loadV clamped onto it (a wave beyond kv_len has only those) --
      // takes the V row from the qkv row: the cache slot is written by this launch, so the DMA
      // read stale or never-written bytes there, and a NaN in a masked row still poisons P.V.
      if (newest >= k0 && newest < k1) {
        const bf16x8 vn = load_bf16x8(vh + dl);
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
          const int row = it * KPI + sub;
          if (min(max(kw0 + row, k0), k1 - 1) == newest) store_bf16x8(vw + dec_swz<D>(row, dl >> 3), vn);
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) {
      const s16x4 v0 = dec_tr_read<D>(vw, 4 * kg, 16 * dt, lane);
      const s16x4 v1 = dec_tr_read<D>(vw, 16 + 4 * kg, 16 * dt, lane);
      const s16x8 vb = s16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      f32x4 o = oacc[dt];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] *= ai[i];
      oacc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o, 0, 0, 0);
    }
    if (c + RD < cend) {
      // WAR: this slot's transposed reads are complete before the DMA refill is issued
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      load(J, c + RD);
    }
  };
  if (cbeg != cfirst) loadK(std::integral_constant<int, 0>{}, cbeg);  // left padding: the guess was wrong
  loadV(std::integral_constant<int, 0>{}, cbeg);
  if (cbeg + 1 < cend) load(std::integral_constant<int, 1>{}, cbeg + 1);
  for (int c = cbeg; c < cend; c += RD) {
    step(std::integral_constant<int, 0>{}, c);
    if (c + 1 < cend) step(std::integral_constant<int, 1>{}, c + 1);
  }
  // this wave's partial O into its own (dead) first image slot
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  float* acc_w = reinterpret_cast<float*>(&vimg[wv][0][0]);
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (4 * kg + i < G) acc_w[(4 * kg + i) * D + 16 * dt + r16] = oacc[dt][i];
  if (kg == 0 && r16 < G) {
    mls[wv][r16][0] = m_run;
    mls[wv][r16][1] = l_run;
  }
  __syncthreads();
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    float mm = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) mm = fmaxf(mm, mls[w][g][0]);
    float v = 0.f, ll = 0.f;
    if (mm != -INFINITY) {
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float mw = mls[w][g][0];
        const float cc = mw == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw - mm);
        v += cc * reinterpret_cast<const float*>(&vimg[w][0][0])[g * D + d];
        ll += cc * mls[w][g][1];
      }
    }
    if (out != nullptr && !fuse) {
      out[(int64_t)b * o_sb + (int64_t)(hk * G + g) * o_sh + d] = f2bf(ll > 0.f ? v * (1.f / ll) : 0.f);
      continue;
    }
    dec_pub(&part_o[(pbase + (int64_t)g * nsplit) * D + d], v, fuse);
    if (d == 0) {
      dec_pub(&part_ml[(pbase + (int64_t)g * nsplit) * 2 + 0], mm, fuse);
      dec_pub(&part_ml[(pbase + (int64_t)g * nsplit) * 2 + 1], ll, fuse);
    }
  }
  if (fuse) dec_arrive_combine<D, G>(cslot, part_o, part_ml, pbase0, nsplit, out, obase, o_sh);
}

template <int D, int G, bool ROPE>
__global__ __launch_bounds__(256, 2) void decode_attn_loop_kernel(
    const bf16_t* __restrict__ q, int64_t q_sb, int64_t q_sh,
    bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
    int64_t c_sb, int64_t c_st, int64_t c_sh, const int* __restrict__ kv_len,
    const int* __restrict__ kv_start, int window, float scale_log2, int nsplit, int cpb,
    float* __restrict__ part_o, float* __restrict__ part_ml, int Hq, DecRope rp,
    bf16_t* __restrict__ out, int64_t o_sb, int64_t o_sh, int* __restrict__ cnt, int Tcap) {
  dec_loop_body<D, G, ROPE>(blockIdx.x, blockIdx.y, blockIdx.z, gridDim.y, q, q_sb, q_sh, kc, vc, c_sb, c_st,
                            c_sh, kv_len, kv_start, window, scale_log2, nsplit, cpb, part_o, part_ml, Hq, rp,
                            out, o_sb, o_sh, cnt, Tcap);
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

// one 64-thread block per (b, h): merge the splits (log2-domain running max). The split
// statistics are read in parallel (one split per lane, 64 at a time) and the per-split weights
// go through LDS, so the output pass issues its part_o loads 8 splits at a time instead of one
// dependent load chain per split (which made this launch grow by ~0.5 us per split).
template <int D>
__global__ __launch_bounds__(64) void decode_combine_kernel(const float* __restrict__ part_o,
                                                             const float* __restrict__ part_ml,
                                                             int nsplit, bf16_t* __restrict__ out,
                                                             int64_t o_sb, int64_t o_sh, int Hq) {
  __shared__ float wsp[64];
  const int bh = blockIdx.x, lane = threadIdx.x;
  const int b = bh / Hq, h = bh % Hq;
  const float* ml = part_ml + (int64_t)bh * nsplit * 2;
  const float* po = part_o + (int64_t)bh * nsplit * D;
  float m = -INFINITY;
  for (int s = lane; s < nsplit; s += 64) m = fmaxf(m, ml[2 * s]);
  m = wave_max(m);
  constexpr int DPT = D / 64;
  float acc[DPT] = {};
  float l = 0.f;
  if (m != -INFINITY) {
    for (int s0 = 0; s0 < nsplit; s0 += 64) {
      const int s = s0 + lane;
      float c = 0.f;
      if (s < nsplit) {
        const float ms = ml[2 * s];
        c = ms == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ms - m);
        l += c * ml[2 * s + 1];
      }
      wsp[lane] = c;
      __syncthreads();
      const int n = min(64, nsplit - s0);
      int j = 0;
      for (; j + 8 <= n; j += 8) {
        float v[8][DPT];
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int t = 0; t < DPT; ++t) v[u][t] = po[(int64_t)(s0 + j + u) * D + lane * DPT + t];
        // an empty split never wrote its part_o row (uninitialised memory): weight 0 selects 0
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float w = wsp[j + u];
#pragma unroll
          for (int t = 0; t < DPT; ++t) acc[t] += w == 0.f ? 0.f : w * v[u][t];
        }
      }
      for (; j < n; ++j) {
        const float w = wsp[j];
#pragma unroll
        for (int t = 0; t < DPT; ++t)
          acc[t] += w == 0.f ? 0.f : w * po[(int64_t)(s0 + j) * D + lane * DPT + t];
      }
      __syncthreads();
    }
    l = wave_sum(l);
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
  for (int j = 0; j < DPT; ++j)
    out[(int64_t)b * o_sb + (int64_t)h * o_sh + lane * DPT + j] = f2bf(acc[j] * inv);
}

static int decode_cpb(int Tmax, int B, int Hkv);
int decode_num_splits(int Tmax, int B, int Hkv);

template <int D>
static void launch_decode_d(const bf16_t* q, int64_t q_sb, int64_t q_sh, bf16_t* kc,
                            bf16_t* vc, int64_t c_sb, int64_t c_st, int64_t c_sh,
                            const int* kv_len, const int* kv_start, int window, float scale_log2,
                            int B, int Hq, int Hkv, int Tmax, float* part_o, float* part_ml,
                            bf16_t* out, int64_t o_sb, int64_t o_sh, const DecRope* rp,
                            int* cnt, hipStream_t st) {
  const int G = Hq / Hkv;
  const int cpb = decode_cpb(Tmax, B, Hkv);
  const int nsplit = decode_num_splits(Tmax, B, Hkv);
  dim3 grid(nsplit, Hkv, B);
  const DecRope r0 = rp ? *rp : DecRope{};
  if (cpb > 0) {
    // one split per sequence, or the in-kernel combine (arrival counters given): no combine launch
    int* const cn = (nsplit > 1 && nsplit <= kDecMaxFuse) ? cnt : nullptr;
    bf16_t* fin = (nsplit == 1 || cn != nullptr) ? out : nullptr;
#define DLA_DECL(GG)                                                                                    \
  if (rp)                                                                                               \
    decode_attn_loop_kernel<D, GG, true><<<grid, 256, 0, st>>>(q, q_sb, q_sh, kc, vc, c_sb, c_st, c_sh, \
                                                               kv_len, kv_start, window, scale_log2,    \
                                                               nsplit, cpb, part_o, part_ml, Hq, r0,    \
                                                               fin, o_sb, o_sh, cn, Tmax);              \
  else                                                                                                  \
    decode_attn_loop_kernel<D, GG, false><<<grid, 256, 0, st>>>(q, q_sb, q_sh, kc, vc, c_sb, c_st, c_sh, \
                                                                kv_len, kv_start, window, scale_log2,   \
                                                                nsplit, cpb, part_o, part_ml, Hq, r0,   \
                                                                fin, o_sb, o_sh, cn, Tmax)
    switch (G) {
      case 1: DLA_DECL(1); break;
      case 2: DLA_DECL(2); break;
      case 4: DLA_DECL(4); break;
      case 8: DLA_DECL(8); break;
      default: break;
    }
#undef DLA_DECL
    if (fin == nullptr)
      decode_combine_kernel<D><<<B * Hq, 64, 0, st>>>(part_o, part_ml, nsplit, out, o_sb, o_sh, Hq);
    return;
  }
#define DLA_DEC(GG)                                                                              \
  if (rp)                                                                                        \
    decode_attn_kernel<D, GG, true><<<grid, 256, 0, st>>>(q, q_sb, q_sh, kc, vc, c_sb, c_st,     \
                                                              c_sh, kv_len, kv_start, window,    \
                                                              scale_log2, nsplit, part_o,        \
                                                              part_ml, Hq, r0, Tmax);            \
  else                                                                                           \
    decode_attn_kernel<D, GG, false><<<grid, 256, 0, st>>>(q, q_sb, q_sh, kc, vc, c_sb,          \
                                                               c_st, c_sh, kv_len, kv_start,     \
                                                               window, scale_log2, nsplit,       \
                                                               part_o, part_ml, Hq, r0, Tmax)
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

// DLA_DECODE_LOOP=0: one 128-key chunk per block (decode_attn_kernel); otherwise blocks loop over
// chunks so that B x Hkv x splits stays near DLA_DECODE_BLOCKS (default 256; same-box graph decode:
// B = 8 / 1152 keys 3 chunks per block 3.98-4.00 vs 4.02 ms/token one-chunk, 2 chunks 4.03-4.06,
// 9 chunks (no combine) 4.25; B = 64 / ~576 keys: one split per sequence)
static int decode_cpb(int Tmax, int B, int Hkv) {
  // read per call (cheap next to a launch) so a test can force the loop kernel at small shapes
  const char* e = getenv("DLA_DECODE_LOOP");
  const char* tb = getenv("DLA_DECODE_BLOCKS");
  const int target = (e != nullptr && atoi(e) == 0) ? 0 : (tb ? atoi(tb) : 256);
  const int nch = (Tmax + kDecChunk - 1) / kDecChunk;
  if (target <= 0) return 0;
  const int64_t blocks = static_cast<int64_t>(B) * Hkv * nch;
  const int cpb = static_cast<int>((blocks + target - 1) / target);
  // Below DLA_DECODE_LOOP_MIN chunks per block the one-chunk kernel (3 blocks per CU) + the combine
  // launch. Round 3 measured that faster under 3 chunks (B = 8, 1152 keys: 4.05 vs 4.12 ms/token);
  // with the in-kernel combine the loop kernel now wins at 2 chunks and at 1 chunk whenever the
  // splits fit the fused combine (B = 8, 512 + 256 tokens: 3.466-3.473 at 2, 3.485-3.497 at 1 vs
  // 3.542-3.548 ms/token, same box, tools/gpu_passes.py r6-decode-combine)
  const char* mn = getenv("DLA_DECODE_LOOP_MIN");
  const int min_cpb = mn ? atoi(mn) : 2;
  if (cpb < min_cpb) return (mn == nullptr && cpb == 1 && nch <= kDecMaxFuse) ? 1 : 0;
  return std::min(cpb, nch);
}

int decode_num_splits(int Tmax, int B, int Hkv) {
  const int nch = (Tmax + kDecChunk - 1) / kDecChunk;
  const int cpb = decode_cpb(Tmax, B, Hkv);
  return cpb == 0 ? nch : (nch + cpb - 1) / cpb;
}

void launch_decode_attn(const bf16_t* q, int64_t q_sb, int64_t q_sh, bf16_t* kc,
                        bf16_t* vc, int64_t c_sb, int64_t c_st, int64_t c_sh,
                        const int* kv_len, const int* kv_start, int window, float scale_log2, int B,
                        int Hq, int Hkv, int D, int Tmax, float* part_o, float* part_ml,
                        bf16_t* out, int64_t o_sb, int64_t o_sh, int* cnt, hipStream_t st) {
  if (D == 128)
    launch_decode_d<128>(q, q_sb, q_sh, kc, vc, c_sb, c_st, c_sh, kv_len, kv_start, window,
                         scale_log2, B, Hq, Hkv, Tmax, part_o, part_ml, out, o_sb, o_sh, nullptr, cnt, st);
  else
    launch_decode_d<64>(q, q_sb, q_sh, kc, vc, c_sb, c_st, c_sh, kv_len, kv_start, window,
                        scale_log2, B, Hq, Hkv, Tmax, part_o, part_ml, out, o_sb, o_sh, nullptr, cnt, st);
}

// rope + cache write of the newest token fused into the decode attention (see DecRope)
void launch_decode_attn_rope(const bf16_t* qkv, int64_t ld, const float* cos_t, const float* sin_t,
                             const int* pos, const int64_t* slot, int rot, bf16_t* kc, bf16_t* vc,
                             int64_t c_sb, int64_t c_st, int64_t c_sh, const int* kv_len,
                             const int* kv_start, int window, float scale_log2, int B, int Hq,
                             int Hkv, int D, int Tmax, float* part_o, float* part_ml, bf16_t* out,
                             int64_t o_sb, int64_t o_sh, int* cnt, hipStream_t st) {
  const DecRope rp{qkv, ld, cos_t, sin_t, pos, slot, rot, Hkv};
  if (D == 128)
    launch_decode_d<128>(nullptr, 0, 0, kc, vc, c_sb, c_st, c_sh, kv_len, kv_start, window,
                         scale_log2, B, Hq, Hkv, Tmax, part_o, part_ml, out, o_sb, o_sh, &rp, cnt, st);
  else
    launch_decode_d<64>(nullptr, 0, 0, kc, vc, c_sb, c_st, c_sh, kv_len, kv_start, window,
                        scale_log2, B, Hq, Hkv, Tmax, part_o, part_ml, out, o_sb, o_sh, &rp, cnt, st);
}

}  // namespace dla
