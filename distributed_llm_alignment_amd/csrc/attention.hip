// Flash attention forward + backward for gfx950, MFMA 32x32x16 bf16.
//
// Replaces the HF SDPA path used by every policy/ref/reward forward of the reference
// (src/training/train_dpo.py:31-39 -> HF attention): causal, GQA, optional
// sliding window, per-batch key ranges [kv_start, kv_end) for left/right padding, head_dim
// 64 / 128. Scores never touch HBM; the forward stores only O and a per-row log2-domain
// LSE, the backward recomputes P from it (FA2 scheme).
//
// Forward (workgroup = 8 waves, two per SIMD = 256 queries of one (batch, q head); wave w owns
// query rows 32w..32w+31; KV tile = 64 keys; cdna guide Appendix B "Fused attention prefill"):
//   * "swapped" scores S^T = K Q^T: the query sits on the MFMA column (lane), keys on the
//     16 accumulator registers, so each lane owns whole score columns -> the row max / sum is
//     in-register + one xor-32 shuffle, and the alpha rescale of O^T is a per-lane scalar.
//   * Q lives in registers for the whole kernel (B operand, 8 x 16 B per lane at D=128),
//     pre-scaled by softmax_scale*log2(e) so the scores come out in the exp2 domain.
//   * P^T feeds the PV MFMA straight from the accumulator (cdna guide §3 "accumulator tile as
//     the next MFMA's operand"); V^T fragments come from ds_read_b64_tr_b16 transposed LDS reads.
//   * K/V tiles are double-buffered in LDS and register-staged one tile ahead (the global loads
//     of tile t+2 are issued right after tile t+1's LDS write: async-STAGE split), so a tile
//     costs one barrier; all 256 queries of the workgroup share each K/V tile.
//   * XOR-swizzled LDS image usable both for row (ds_read_b128) and transposed reads.
//   * query blocks are the slowest grid dimension, heaviest causal blocks first (LPT order).
//   * HP query heads of one GQA group share a workgroup (and so every K/V tile in LDS): the
//     per-head query block shrinks to 256 / HP rows, which narrows the causal diagonal band where
//     part of the waves idle (see fwd_dispatch).
//   * widened store tail (T21): O leaves as 8 x 16 B per lane after a permlane32 swap instead
//     of 16 x 8 B (the per-lane row stores are issue-bound): 141 -> 121 us causal T = 1024,
//     190 -> 170 us non-causal (tools/attn_bench.py --ab, one box).
// Backward: see attn_bwd_kernel.
#include <cstdlib>
#include <stdexcept>
#include <type_traits>
#include "common.h"

#include <cstring>
#include "attn_params.h"

namespace dla {

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// LDS row width (elements) of head dim D: a multiple of 32 (the 32-column MFMA output tiles).
// D = 80 (phi-2) uses 96-wide images: the 16 pad columns are zero, so Q.K^T runs over exactly
// D/16 = 5 k-steps and only the P.V / dK / dV column tiles carry the 96/80 pad.
template <int D>
constexpr int attn_dp() { return (D + 31) / 32 * 32; }

// Element offset of 16-byte chunk `ch` of row `row` in a [rows][W] bf16 LDS image. The XOR
// keeps both ds_read_b128 row reads and ds_read_b64_tr_b16 column reads spread over banks
// (cdna guide T10 "one image for row reads AND transposed reads", layout (b)). Rows of a
// non-power-of-two chunk count (W = 96: 12 chunks) XOR inside aligned groups of 4 chunks.
template <int W>
__device__ __forceinline__ int swz(int row, int ch) {
  constexpr int NCH = W / 8;
  constexpr int MASK = (NCH & (NCH - 1)) == 0 ? NCH - 1 : 3;
  const int f = (((row & 3) << 2) | ((row >> 2) & 3)) & MASK;
  return row * W + ((ch ^ f) << 3);
}

// dS^T image [keys][32 queries] bf16 (64-B rows): 8-byte unit c4 of row `row`, XOR-swizzled
// with row bits 1..3. ds_write_b64 banks 16-lane groups over 32 banks: 16 consecutive key rows
// (one unit each) cover (row parity, unit ^ (row>>1)&7) = all 16 bank pairs. The transposed dQ
// reads stay conflict-free: attn_bwd_kernel's 32-lane groups read rows r..r+3 (x 8 units), and
// attn_bwd8_kernel's read rows r..r+3 with units 4t..4t+3 beside rows r+8..r+11, whose XOR
// differs in bit 2 and so moves them to the other four units. (Row bits 2..4 left the latter
// 2-way conflicted on every read: SQ_LDS_BANK_CONFLICT 1.3e7 per call at B8 T1024.)
__device__ __forceinline__ int ds_swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int ds_off(int row, int c4) { return row * 32 + ((c4 ^ ds_swz(row)) << 2); }

__device__ __forceinline__ s16x4 tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}

__device__ __forceinline__ s16x8 cat4(s16x4 a, s16x4 b) {
  return s16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ s16x8 pack8(const f32x16& x, int base) {
  u32x4 r = {pack2bf(x[base], x[base + 1]), pack2bf(x[base + 2], x[base + 3]),
             pack2bf(x[base + 4], x[base + 5]), pack2bf(x[base + 6], x[base + 7])};
  return __builtin_bit_cast(s16x8, r);
}

__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

// RoPE on load (full rotary, rotate-half): rotates the 16-byte chunk `ch` (of NCH per row) of
// token `t` of a sequence (position pos_t[pidx], or t without a position table). Column d < D/2 pairs with d + D/2, i.e. chunk ch ^ NCH/2,
// which the staging layouts below always hold in lane ^ NCH/2 of the same wave: one xor-shuffle
// per dword fetches it. Every lane must call this (the shuffle); `valid` = the row exists.
template <int NCH>
__device__ __forceinline__ bf16x8 rope_rot_chunk(bf16x8 v, int ch, bool valid, int64_t pidx, int t,
                                                 const float* __restrict__ cos_t,
                                                 const float* __restrict__ sin_t,
                                                 const int* __restrict__ pos_t) {
  const u32x4 w = __builtin_bit_cast(u32x4, v);
  u32x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = __shfl_xor(w[i], NCH / 2, 64);
  if (!valid) return v;
  const bf16x8 partner = __builtin_bit_cast(bf16x8, o);
  const bool lo = ch < NCH / 2;
  const int d0 = (lo ? ch : ch - NCH / 2) * 8;
  const int pos = pos_t ? pos_t[pidx] : t;
  const float* cp = cos_t + static_cast<int64_t>(pos) * (NCH * 4) + d0;
  const float* sp = sin_t + static_cast<int64_t>(pos) * (NCH * 4) + d0;
  const f32x4 c0 = *reinterpret_cast<const f32x4*>(cp), c1 = *reinterpret_cast<const f32x4*>(cp + 4);
  const f32x4 s0 = *reinterpret_cast<const f32x4*>(sp), s1 = *reinterpret_cast<const f32x4*>(sp + 4);
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float c = j < 4 ? c0[j] : c1[j - 4], s = j < 4 ? s0[j] : s1[j - 4];
    const float a = bf2f(v[j]), q = bf2f(partner[j]);
    r[j] = lo ? a * c - q * s : a * c + q * s;
  }
  return pack_bf16x8(r);
}

// Deferred-max threshold (cdna guide T13, log2 units): the running max is only raised when a
// tile's max exceeds it by more than this, so most tiles skip the O rescale. P <= 2^8.
constexpr float kRescaleThr = 8.0f;

__device__ __forceinline__ f32x16 mfma32(s16x8 a, s16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// max / sum of x over lanes l and l ^ 32 by one v_permlane32_swap (VALU) instead of a
// ds_bpermute round trip through LDS (cdna guide T12): with both operands x, every lane gets
// {its own x, its partner's x} in some order, so the max is exact and the sum bitwise equal to
// x + partner.
__device__ __forceinline__ float xhalf_max(float x) {
  const uint32_t u = __float_as_uint(x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float x) {
  const uint32_t u = __float_as_uint(x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// transposed 8-row fragment for the 32x32x16 A operand whose k index follows the accumulator
// row permutation: elements 0..3 <- rows r0..r0+3, 4..7 <- rows r0+8..r0+11 (column c0 + lane).
template <int D>
__device__ __forceinline__ s16x8 tr_frag_perm(const bf16_t* img, int r0, int c0, int lane) {
  const int i = lane & 15, qq = i >> 2, pp = i & 3;
  const int ch = (c0 >> 3) + (pp >> 1), sub = (pp & 1) * 4;
  const s16x4 a = tr_read(img + swz<D>(r0 + qq, ch) + sub);
  const s16x4 b = tr_read(img + swz<D>(r0 + 8 + qq, ch) + sub);
  return cat4(a, b);
}

// transposed fragment with natural k order: elements 0..7 <- rows r0..r0+7 (column c0 + lane).
template <int D>
__device__ __forceinline__ s16x8 tr_frag_nat(const bf16_t* img, int r0, int c0, int lane) {
  const int i = lane & 15, qq = i >> 2, pp = i & 3;
  const int ch = (c0 >> 3) + (pp >> 1), sub = (pp & 1) * 4;
  const s16x4 a = tr_read(img + swz<D>(r0 + qq, ch) + sub);
  const s16x4 b = tr_read(img + swz<D>(r0 + 4 + qq, ch) + sub);
  return cat4(a, b);
}

// Partial-rotary backward (phi-2: rot = 32 at D = 80): in the dK^T accumulator tile 0 (lane =
// key, register i = column d = (i&3) + 8(i>>2) + 4h), column d < 16 pairs with d + 16 =
// register i + 8 of the same lane; un-rotate (lo = a c + b s, hi = b c - a s) with
// cp / sp = cos / sin + pos * 16 + 4h.
__device__ __forceinline__ f32x16 unrotate_tile0_rot32(f32x16 x, const float* cp, const float* sp) {
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const f32x4 c4 = *reinterpret_cast<const f32x4*>(cp + 8 * g);
    const f32x4 s4 = *reinterpret_cast<const f32x4*>(sp + 8 * g);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = x[4 * g + e], bb = x[4 * g + e + 8];
      x[4 * g + e] = a * c4[e] + bb * s4[e];
      x[4 * g + e + 8] = bb * c4[e] - a * s4[e];
    }
  }
  return x;
}

// ==============================================================================================
// forward
// ==============================================================================================
constexpr int kFwdKeys = 64;      // keys per K/V tile

// Logical block of item i of persistent workgroup g of G: a snake over the workgroups (causal:
// heaviest-first blocks, equal tile sums). Returns nblk past the end (monotone: once past, every
// later item is past too). (An XCD-grouped block order measured 5 % slower causal at T 1024: removed.)
__device__ __forceinline__ int fwd_persist_logical(int i, int g, int G, int nblk) {
  const int idx = (i & 1) ? (i + 1) * G - 1 - g : i * G + g;
  return idx < nblk ? idx : nblk;
}

// NW waves per workgroup, 32 queries each (NT = 64 NW threads). HP query heads of one GQA group
// per workgroup (HP = 2: waves 0..NW/2-1 take head 2p, the rest head 2p+1): every K/V tile staged
// in LDS still feeds 32 NW query rows, but a head's query block is only BQ = 32 NW / HP rows, so
// the causal diagonal (whose tiles run with part of the waves idle) is HP times narrower.
template <int D, bool CAUSAL, int NW, int HP, bool MSUB = false>
__global__ __launch_bounds__(64 * NW) void attn_fwd_kernel(AttnParams p) {
  constexpr int NT = 64 * NW, BQ = 32 * NW / HP, BK = kFwdKeys;
  constexpr int WPH = NW / HP;  // waves per head
  constexpr int DP = attn_dp<D>();  // LDS row width (D + zero pad to the 32-column tiles)
  constexpr int NCH = DP / 8;       // 16-B chunks per LDS row
  constexpr int NCHL = D / 8;       // of which loaded from memory
  constexpr int KS = D / 16;
  constexpr int DT = DP / 32;
  constexpr int CPT = (BK * NCH + NT - 1) / NT;  // 16-B chunks per thread per K (or V) tile
  constexpr bool CPT_EXACT = (BK * NCH) % NT == 0;
  static_assert(CPT >= 1, "K/V tile smaller than the workgroup");
  __shared__ __attribute__((aligned(16))) bf16_t Kb[2][BK * DP];
  __shared__ __attribute__((aligned(16))) bf16_t Vb[2][BK * DP];

  // readfirstlane: the wave index is wave-uniform, so everything derived from it (key / query
  // ranges, activity and mask flags) stays in SGPRs and its branches are scalar
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int nqb = (p.Tq + BQ - 1) / BQ;
  const int nhb = p.Hq / HP;  // head blocks
  const int nbh = nhb * p.B;
  const int bid = blockIdx.x;
  // query block slowest (causal: heaviest first)
  const int qb = CAUSAL ? nqb - 1 - bid / nbh : bid / nbh;
  const int rest = bid % nbh;
  const int hq = (rest % nhb) * HP + w / WPH, b = rest / nhb;
  const int hk = hq / (p.Hq / p.Hkv);  // the same for the HP heads (host: group % HP == 0)
  const int q0 = qb * BQ + (w % WPH) * 32;
  const int qi = q0 + l32;

  const bf16_t* qp = p.q + b * p.q_sb + static_cast<int64_t>(hq) * p.q_sh;
  const bf16_t* kp = p.k + b * p.k_sb + static_cast<int64_t>(hk) * p.k_sh;
  const bf16_t* vp = p.v + b * p.v_sb + static_cast<int64_t>(hk) * p.v_sh;

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x16{};
  float m = -INFINITY, lsum = 0.f;

  const int kbeg = p.kv_start ? p.kv_start[b] : 0;
  const int kend = p.kv_end ? p.kv_end[b] : p.Tk;
  const int blk_qmax = min(p.Tq, qb * BQ + BQ) - 1;
  int kmax = kend;
  if (CAUSAL) kmax = min(kmax, blk_qmax + p.causal_off + 1);
  int kmin = kbeg;
  if (CAUSAL && p.window > 0) kmin = max(kmin, qb * BQ + p.causal_off - p.window + 1);
  // packed sequences: query i sees keys >= seg_start[i]; seg_start is non-decreasing in i, so
  // the block's first query bounds the key range from below and each wave's first / last query
  // bound its activity / masking (wseg_* are 0 without segments: no effect)
  const int* ss = p.seg_start ? p.seg_start + static_cast<int64_t>(b) * p.Tq : nullptr;
  int wseg_lo = 0, wseg_hi = 0, qseg = 0;
  if (ss) {
    kmin = max(kmin, ss[qb * BQ]);
    wseg_lo = __builtin_amdgcn_readfirstlane(ss[min(q0, p.Tq - 1)]);
    wseg_hi = __builtin_amdgcn_readfirstlane(ss[min(q0 + 31, p.Tq - 1)]);
    qseg = ss[min(qi, p.Tq - 1)];
  }
  const int tile0 = (max(kmin, 0) / BK) * BK;
  const int ntiles = kmax > tile0 ? (kmax - tile0 + BK - 1) / BK : 0;

  bf16x8 kreg[CPT], vreg[CPT];
  // whole tiles load from a wave-uniform (SGPR) tile base + a per-lane 32-bit byte offset fixed for
  // the kernel, with no per-chunk key test; the last, partial tile keeps the guarded form
  const bool ofs32 =
      p.fwd_sgpr != 0 && static_cast<int64_t>(BK) * (p.k_st > p.v_st ? p.k_st : p.v_st) * 2 < (1ll << 31);
  uint32_t kofs[CPT], vofs[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int ci = tid + NT * c;
    const int row = ci / NCH, ch = ci % NCH;
    kofs[c] = static_cast<uint32_t>((row * p.k_st + ch * 8) * 2);
    vofs[c] = static_cast<uint32_t>((row * p.v_st + ch * 8) * 2);
  }
  auto gload = [&](int kt) {
    if (ofs32 && kt + BK <= p.Tk && NCHL == NCH && CPT_EXACT) {  // wave-uniform
      const char* kb = reinterpret_cast<const char*>(kp + static_cast<int64_t>(kt) * p.k_st);
      const char* vb = reinterpret_cast<const char*>(vp + static_cast<int64_t>(kt) * p.v_st);
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        kreg[c] = load_bf16x8(reinterpret_cast<const bf16_t*>(kb + kofs[c]));
        vreg[c] = load_bf16x8(reinterpret_cast<const bf16_t*>(vb + vofs[c]));
      }
      return;
    }
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int ci = tid + NT * c;
      const int row = ci / NCH, ch = ci % NCH;
      const int key = kt + row;
      if (key < p.Tk && ch < NCHL && (CPT_EXACT || ci < BK * NCH)) {
        kreg[c] = load_bf16x8(kp + key * p.k_st + ch * 8);
        vreg[c] = load_bf16x8(vp + key * p.v_st + ch * 8);
      } else {
        kreg[c] = bf16x8{};
        vreg[c] = bf16x8{};
      }
    }
  };
  const bool rope = p.rope_cos != nullptr;  // kernel-uniform
  auto lwrite = [&](int buf, int kt) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int ci = tid + NT * c;
      if (!CPT_EXACT && ci >= BK * NCH) continue;
      const int row = ci / NCH, ch = ci % NCH;
      bf16x8 kv = kreg[c];
      if constexpr (DP == D) {  // RoPE on load: full rotary only (the host checks rot == D)
        if (rope && p.rope_k)
          kv = rope_rot_chunk<NCH>(kv, ch, kt + row < p.Tk, static_cast<int64_t>(b) * p.Tk + kt + row,
                                   kt + row, p.rope_cos, p.rope_sin, p.rope_pos);
      }
      store_bf16x8(&Kb[buf][swz<DP>(row, ch)], kv);
      store_bf16x8(&Vb[buf][swz<DP>(row, ch)], vreg[c]);
    }
  };

  // Q fragments stay in registers, pre-scaled by softmax_scale*log2(e) so the scores come
  // out of the MFMA already in the exp2 domain (no per-score multiply).
  // Prologue load order (p.fwd_pro, default): Q rows, [RoPE: position, then its cos / sin rows],
  // then the K/V tile-0 rows, then the Q math. vmcnt is in-order, so the Q math waits for Q (and
  // cos / sin) only and runs under the K/V flight: one fewer dependent HBM round trip per block.
  // (K/V issued AHEAD of Q measured -2.5 % .. +3 %: the Q math then waited for K/V too.) Each
  // variant is one straight-line copy (a template lambda per (early, rope) pair): a control-flow
  // merge between the loads and the math would make the compiler's waits conservative (vmcnt(0)).
  // Rows past Tq / Tk are clamped into range and zeroed (Q) or masked (K/V: their scores are
  // masked because need_mask covers kt + BK > kend, and their P is 0).
  s16x8 qf[KS];
  auto prologue = [&](auto early_c, auto rope_c) {
    constexpr bool EARLY = decltype(early_c)::value;
    constexpr bool ROPE = decltype(rope_c)::value && DP == D;
    float qv[KS][8];
    {
      const int qc = min(qi, p.Tq - 1);
      // RoPE: the row's position is loaded FIRST, so its round trip overlaps the Q loads' instead
      // of queueing behind them (vmcnt is in-order); the cos / sin rows it addresses follow
      int pv = 0;
      if constexpr (ROPE) {
        // branch-free position: a valid dummy address when there is no position table
        const int* pp = p.rope_pos ? p.rope_pos + static_cast<int64_t>(b) * p.Tq + qc
                                   : reinterpret_cast<const int*>(qp);
        pv = *pp;
      }
      bf16x8 qraw[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) qraw[s] = load_bf16x8(qp + qc * p.q_st + 16 * s + 8 * h);
      f32x4 rc[ROPE ? KS : 1], rs[ROPE ? KS : 1];  // cos / sin of columns 16s + 8h + [0, 8), s < KS/2
      if constexpr (ROPE) {
        const int pos = p.rope_pos ? pv : qc;
        const float* cp = p.rope_cos + static_cast<int64_t>(pos) * (D / 2) + 8 * h;
        const float* sp = p.rope_sin + static_cast<int64_t>(pos) * (D / 2) + 8 * h;
#pragma unroll
        for (int s = 0; s < KS / 2; ++s) {
          rc[2 * s] = *reinterpret_cast<const f32x4*>(cp + 16 * s);
          rc[2 * s + 1] = *reinterpret_cast<const f32x4*>(cp + 16 * s + 4);
          rs[2 * s] = *reinterpret_cast<const f32x4*>(sp + 16 * s);
          rs[2 * s + 1] = *reinterpret_cast<const f32x4*>(sp + 16 * s + 4);
        }
      }
      if constexpr (EARLY) {
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
          const int ci = tid + NT * c;
          const int key = max(min(tile0 + ci / NCH, p.Tk - 1), 0), ch = ci % NCH;
          kreg[c] = load_bf16x8(kp + key * p.k_st + ch * 8);
          vreg[c] = load_bf16x8(vp + key * p.v_st + ch * 8);
        }
      }
      const bool qin = qi < p.Tq;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
#pragma unroll
        for (int j = 0; j < 8; ++j) qv[s][j] = qin ? bf2f(qraw[s][j]) : 0.f;
      }
      if constexpr (ROPE) {
        // RoPE on load: fragment s (columns 16s + 8h + j) pairs with fragment s + KS/2 (+ D/2)
#pragma unroll
        for (int s = 0; s < KS / 2; ++s) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float c = j < 4 ? rc[2 * s][j] : rc[2 * s + 1][j - 4];
            const float sn = j < 4 ? rs[2 * s][j] : rs[2 * s + 1][j - 4];
            const float a = qv[s][j], bb = qv[s + KS / 2][j];
            qv[s][j] = a * c - bb * sn;
            qv[s + KS / 2][j] = bb * c + a * sn;
          }
        }
      }
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = qv[s][j] * p.scale2;
      qf[s] = __builtin_bit_cast(s16x8, pack_bf16x8(t));
    }
    // the rotated (unscaled) Q rows for the backward; the HP heads' waves write disjoint rows
    if (ROPE && p.q_rot != nullptr && qi < p.Tq) {
      bf16_t* qo = p.q_rot + b * p.qr_sb + qi * p.qr_st + static_cast<int64_t>(hq) * p.qr_sh + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) store_bf16x8(qo + 16 * s, pack_bf16x8(qv[s]));
    }
    if (ntiles > 0) {
      if constexpr (!EARLY) gload(tile0);
      lwrite(0, tile0);
      if (ntiles > 1) gload(tile0 + BK);
    }
  };
  {
    using T_ = std::true_type;
    using F_ = std::false_type;
    if (p.fwd_pro != 0 && NCHL == NCH && CPT_EXACT) {
      if (rope) prologue(T_{}, T_{});
      else prologue(T_{}, F_{});
    } else {
      if (rope) prologue(F_{}, T_{});
      else prologue(F_{}, F_{});
    }
  }
  __syncthreads();
  if (p.fwd_prio == 2 && w >= NW / 2) __builtin_amdgcn_s_setprio(1);  // (MI355X_MICROARCH §Two waves item 4)
  // p.fwd_msub: the running max leaves the scores inside the MFMA chain instead of by 32 v_sub per
  // tile. m is kept exactly representable as hi + lo (two bf16); one extra MFMA per tile,
  // ones[key][k 0..1] x (-hi, -lo)[k 0..1][query], yields the tile of -m that the first Q.K^T step
  // of both key halves takes as its C input, so the chain ends at S - m (the same row constant
  // every score of the row gets, so P, l, O and the LSE stay consistent; only the fp32 rounding
  // order of the subtraction moves). Rescales (rare: deferred max) subtract the change by VALU.
  constexpr bool msub_on = MSUB;  // (a runtime switch keeping both paths spilled: 380 B scratch)
  const s16x8 ones = __builtin_bit_cast(s16x8, u32x4{h ? 0u : 0x3F803F80u, 0u, 0u, 0u});
  s16x8 mfrag = s16x8{};  // B operand: (-hi, -lo) of this lane's query row in k slots 0, 1
  float msub = 0.f;       // the value the chain subtracts (m, or 0 while m is -inf)
  // the loop body runs as two copies (buffer 0 / buffer 1) so every LDS read address is a per-lane
  // base plus an immediate: no per-tile buffer select in the VALU stream
  auto step = [&](auto bufc, int t) {
    constexpr int BUF = decltype(bufc)::value;
    const int kt = tile0 + t * BK;
    const bf16_t* Ks = Kb[BUF];
    const bf16_t* Vs = Vb[BUF];
    bool active = q0 < p.Tq && kt + BK > wseg_lo;
    if (CAUSAL) {
      active = active && (kt <= q0 + 31 + p.causal_off);
      if (p.window > 0) active = active && (kt + BK - 1 > q0 + p.causal_off - p.window);
    }
    if (active) {  // wave-uniform
      f32x16 sacc[2];
      if (p.fwd_prio == 1) __builtin_amdgcn_s_setprio(1);
      if (msub_on) {
        const f32x16 negm = mfma32(ones, mfrag, f32x16{});
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          sacc[st] = mfma32(*reinterpret_cast<const s16x8*>(Ks + swz<DP>(32 * st + l32, h)), qf[0], negm);
#pragma unroll
          for (int s = 1; s < KS; ++s) {
            const s16x8 a = *reinterpret_cast<const s16x8*>(Ks + swz<DP>(32 * st + l32, 2 * s + h));
            sacc[st] = mfma32(a, qf[s], sacc[st]);
          }
        }
      } else {
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          sacc[st] = f32x16{};
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const s16x8 a = *reinterpret_cast<const s16x8*>(Ks + swz<DP>(32 * st + l32, 2 * s + h));
            sacc[st] = mfma32(a, qf[s], sacc[st]);
          }
        }
      }
      if (p.fwd_prio == 1) __builtin_amdgcn_s_setprio(0);
      // mask only tiles that touch a boundary (kv range, causal diagonal, window edge)
      bool need_mask = kt < kbeg || kt + BK > kend || kt < wseg_hi;
      if (CAUSAL) {
        need_mask = need_mask || (kt + BK - 1 > q0 + p.causal_off);
        if (p.window > 0) need_mask = need_mask || (kt <= q0 + 31 + p.causal_off - p.window);
      }
      if (need_mask) {
        // key = base + r with r = 32st + (i&3) + 8(i>>2) a compile-time constant per register:
        // the visible keys of this lane's query are r in [lo, hi), tested as one unsigned
        // compare per score
        const int base = kt + 4 * h;
        int lo = max(kbeg, qseg) - base, hi = kend - base;
        if (CAUSAL) {
          hi = min(hi, qi + p.causal_off + 1 - base);
          if (p.window > 0) lo = max(lo, qi + p.causal_off - p.window + 1 - base);
        }
        const unsigned span = hi > lo ? static_cast<unsigned>(hi - lo) : 0u;
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int r = 32 * st + (i & 3) + 8 * (i >> 2);
            sacc[st][i] = static_cast<unsigned>(r - lo) < span ? sacc[st][i] : -INFINITY;
          }
        }
      }
      float mloc = -INFINITY;
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int i = 0; i < 16; ++i) mloc = fmaxf(mloc, sacc[st][i]);
      mloc = xhalf_max(mloc);
      float lpart[2] = {0.f, 0.f};  // two independent add chains (the row sum was one 32-add chain)
      if (msub_on) {
        // the scores are S - msub; deferred max as below, on the true scale mloc + msub
        if (!__all(mloc + msub <= m + kRescaleThr)) {
          const float mnew = fmaxf(m, mloc + msub);
          float mq = -INFINITY, hi = 0.f, lo = 0.f;
          if (mnew != -INFINITY) {  // m as hi + lo (two bf16), exact in fp32
            hi = bf2f(f2bf(mnew));
            lo = bf2f(f2bf(mnew - hi));
            mq = hi + lo;
          }
          const float alpha = ex2(m - (mq == -INFINITY ? 0.f : mq));
          const float nsub = mq == -INFINITY ? 0.f : mq;
          const float d = nsub - msub;
          m = mq;
          msub = nsub;
          mfrag = __builtin_bit_cast(s16x8, u32x4{h ? 0u : pack2bf(-hi, -lo), 0u, 0u, 0u});
          lsum *= alpha;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
#pragma unroll
          for (int st = 0; st < 2; ++st) sacc[st] -= d;
        }
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float pv = ex2(sacc[st][i]);
            sacc[st][i] = pv;
            lpart[st] += pv;
          }
        }
      } else {
        // deferred max: rescale O only when some row's max grew by more than kRescaleThr (the
        // previous tile's P.V is complete, and this tile's P is exponentiated after the decision)
        if (!__all(mloc <= m + kRescaleThr)) {
          const float mnew = fmaxf(m, mloc);
          const float alpha = ex2(m - (mnew == -INFINITY ? 0.f : mnew));
          m = mnew;
          lsum *= alpha;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
        }
        const float muse = m == -INFINITY ? 0.f : m;
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float pv = ex2(sacc[st][i] - muse);
            sacc[st][i] = pv;
            lpart[st] += pv;
          }
        }
      }
      lsum += lpart[0] + lpart[1];
      s16x8 pf[2][2];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        pf[st][0] = pack8(sacc[st], 0);
        pf[st][1] = pack8(sacc[st], 8);
      }
      if (p.fwd_prio == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int c0 = 32 * dt + 16 * ((lane >> 4) & 1);
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const s16x8 a = tr_frag_perm<DP>(Vs, 32 * st + 16 * s + 4 * h, c0, lane);
            o[dt] = mfma32(a, pf[st][s], o[dt]);
          }
        }
      }
      if (p.fwd_prio == 1) __builtin_amdgcn_s_setprio(0);
    }
    if (t + 1 < ntiles) {  // stage tile t+1 into the other buffer, prefetch tile t+2
      lwrite(BUF ^ 1, kt + BK);
      if (t + 2 < ntiles) gload(kt + 2 * BK);
    }
    __syncthreads();
  };
  for (int t = 0; t < ntiles; t += 2) {
    step(std::integral_constant<int, 0>{}, t);
    if (t + 1 < ntiles) step(std::integral_constant<int, 1>{}, t + 1);
  }

  lsum = xhalf_sum(lsum);
  if constexpr (DP == D && D == 128) {
    if (p.fwd_ostage != 0) {
      // O through LDS, stored as whole rows (cdna guide §5.6, pwg4x64 notes: per-lane 16-B stores
      // at a row stride touch 32-64 lines per instruction). The loop ended on a barrier, so the K/V
      // buffers are free: wave w stages its 32 x 128 tile (8 KB) there, chunk-swizzled by row
      // (both the 16-B writes and the row reads are bank-conflict free), then each store
      // instruction writes 4 contiguous 256-B rows.
      const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
      bf16_t* ost = (w < 4 ? &Kb[0][0] : &Vb[0][0]) + (w & 3) * (32 * 128);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
        for (int g4 = 0; g4 < 4; g4 += 2) {
          uint2 a, c;
          a.x = pack2bf(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv);
          a.y = pack2bf(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
          c.x = pack2bf(o[dt][4 * g4 + 4] * inv, o[dt][4 * g4 + 5] * inv);
          c.y = pack2bf(o[dt][4 * g4 + 6] * inv, o[dt][4 * g4 + 7] * inv);
          const auto rx = __builtin_amdgcn_permlane32_swap(a.x, c.x, false, false);
          const auto ry = __builtin_amdgcn_permlane32_swap(a.y, c.y, false, false);
          const int ch = 4 * dt + g4 + h;  // 16-B chunk of the row
          *reinterpret_cast<uint4*>(ost + l32 * 128 + ((ch ^ (l32 & 15)) << 3)) =
              make_uint4(rx[0], ry[0], rx[1], ry[1]);
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes done
      __builtin_amdgcn_wave_barrier();
      const int rr = lane >> 4, cc = lane & 15;
      bf16_t* obase = p.o + b * p.o_sb + static_cast<int64_t>(hq) * p.o_sh;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = 4 * i + rr;
        const uint4 v = *reinterpret_cast<const uint4*>(ost + r * 128 + ((cc ^ (r & 15)) << 3));
        if (q0 + r < p.Tq) *reinterpret_cast<uint4*>(obase + (q0 + r) * p.o_st + cc * 8) = v;
      }
      if (qi < p.Tq && h == 0) {
        p.lse2[(static_cast<int64_t>(b) * p.Hq + hq) * p.Tq + qi] = lsum > 0.f ? m + __log2f(lsum) : INFINITY;
      }
      return;
    }
  }
  if (qi < p.Tq) {
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16_t* op = p.o + b * p.o_sb + qi * p.o_st + static_cast<int64_t>(hq) * p.o_sh;
    // widened store tail (cdna guide T21): lane half h holds columns 8k + 4h .. +3 of each 8-column
    // group k; one v_permlane32_swap per dword pairs groups k, k+1 so that each lane owns 8
    // contiguous columns (8k + 8h ..) and stores 16 B: 8 x dwordx4 per lane instead of 16 x dwordx2
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; g4 += 2) {
        uint2 a, c;
        a.x = pack2bf(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv);
        a.y = pack2bf(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
        c.x = pack2bf(o[dt][4 * g4 + 4] * inv, o[dt][4 * g4 + 5] * inv);
        c.y = pack2bf(o[dt][4 * g4 + 6] * inv, o[dt][4 * g4 + 7] * inv);
        const auto rx = __builtin_amdgcn_permlane32_swap(a.x, c.x, false, false);
        const auto ry = __builtin_amdgcn_permlane32_swap(a.y, c.y, false, false);
        const int d = 32 * dt + 8 * g4 + 8 * h;
        if (d < D) *reinterpret_cast<uint4*>(op + d) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
      }
    }
    if (h == 0) {
      p.lse2[(static_cast<int64_t>(b) * p.Hq + hq) * p.Tq + qi] =
          lsum > 0.f ? m + __log2f(lsum) : INFINITY;
    }
  }
}

// ----------------------------------------------------------------------------------------------
// persistent forward
// ----------------------------------------------------------------------------------------------
// attn_fwd_kernel pays a fixed cost per query block that the tile loop never hides: the Q rows
// and the first K/V tile are fetched with every CU doing the same at once, and the O store tail
// is issue-bound. Fitting t = blocks_per_CU x (c0 + tiles x c1) over T = 256..4096 at B*T = 8192
// (tools/attn_fwd_sweep.py, graph-timed) gives c0 = 11.7 us against c1 = 1.87 us per 64-key tile:
// at causal T = 1024 (8.5 tiles per block on average) ~45 % of the kernel is that seam.
// This variant runs one workgroup per CU over a snake-ordered list of the same blocks (causal:
// heaviest first, so the per-workgroup tile sums come out equal) and streams across the seams:
//   * the next block's first K/V tile is register-staged during the current block's second-last
//     tile (the same async-STAGE pipeline as inside a block);
//   * its Q rows arrive by LDS-DMA (global_load_lds, lane-linear into a per-wave chunk-major
//     [D/8][32 rows][8] image, conflict-free ds_read_b128 at the seam) issued at the top of the
//     current block's last tile, so only the last tile's compute separates issue and use;
//   * the seam reads the new Q, issues the next tile's loads, and only then stores the finished
//     block's O / LSE, so the store tail drains under the next block's first tile.
// The tile math (swapped scores, deferred max, P from the accumulator, tr-read V, T21 stores) is
// attn_fwd_kernel's; outputs are bitwise equal to it (tests/test_kernels_gpu.py).
template <int D, bool CAUSAL, int NW, int HP>
__global__ __launch_bounds__(64 * NW) void attn_fwd_persist_kernel(AttnParams p, int nblk) {
  constexpr int NT = 64 * NW, BQ = 32 * NW / HP, BK = kFwdKeys;
  constexpr int WPH = NW / HP;
  constexpr int DP = attn_dp<D>();
  constexpr int NCH = DP / 8;
  constexpr int NCHL = D / 8;
  constexpr int KS = D / 16;
  constexpr int DT = DP / 32;
  constexpr int CPT = (BK * NCH + NT - 1) / NT;
  constexpr bool CPT_EXACT = (BK * NCH) % NT == 0;
  constexpr int KVE = BK * DP;   // elements of one K or V tile image
  constexpr int QWE = 32 * D;    // elements of one wave's Q image
  static_assert(CPT >= 1, "K/V tile smaller than the workgroup");
  // ONE LDS array (a second __shared__ object beside an LDS-DMA target can make hipcc drain
  // vmcnt before every ds_read: cdna guide §5 'Projection GEMM at M = 256' item 4(a))
  __shared__ __attribute__((aligned(16))) bf16_t lds[4 * KVE + NW * QWE];

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int nqb = (p.Tq + BQ - 1) / BQ;
  const int nhb = p.Hq / HP;
  const int nbh = nhb * p.B;
  const int G = gridDim.x, g = blockIdx.x;
  bf16_t* Qw = lds + 4 * KVE + w * QWE;

  struct Blk {  // wave-uniform description of one query block (this wave's 32 rows of it)
    bool valid;
    int b, hq, hk, q0, kbeg, kend, ntiles, tile0, wseg_lo, wseg_hi;
  };
  auto make_blk = [&](int i) -> Blk {
    Blk c{};
    const int blk = fwd_persist_logical(i, g, G, nblk);
    c.valid = blk < nblk;
    if (!c.valid) return c;
    const int qb = CAUSAL ? nqb - 1 - blk / nbh : blk / nbh;
    const int rest = blk % nbh;
    c.hq = (rest % nhb) * HP + w / WPH;
    c.b = rest / nhb;
    c.hk = c.hq / (p.Hq / p.Hkv);
    c.q0 = qb * BQ + (w % WPH) * 32;
    c.kbeg = p.kv_start ? p.kv_start[c.b] : 0;
    c.kend = p.kv_end ? p.kv_end[c.b] : p.Tk;
    const int blk_qmax = min(p.Tq, qb * BQ + BQ) - 1;
    int kmax = c.kend;
    if (CAUSAL) kmax = min(kmax, blk_qmax + p.causal_off + 1);
    int kmin = c.kbeg;
    if (CAUSAL && p.window > 0) kmin = max(kmin, qb * BQ + p.causal_off - p.window + 1);
    c.wseg_lo = c.wseg_hi = 0;
    if (p.seg_start) {
      const int* ss = p.seg_start + static_cast<int64_t>(c.b) * p.Tq;
      kmin = max(kmin, ss[qb * BQ]);
      c.wseg_lo = __builtin_amdgcn_readfirstlane(ss[min(c.q0, p.Tq - 1)]);
      c.wseg_hi = __builtin_amdgcn_readfirstlane(ss[min(c.q0 + 31, p.Tq - 1)]);
    }
    c.tile0 = (max(kmin, 0) / BK) * BK;
    c.ntiles = kmax > c.tile0 ? (kmax - c.tile0 + BK - 1) / BK : 0;
    return c;
  };

  bf16x8 kreg[CPT], vreg[CPT];
  // (the SGPR-base / 32-bit offset form of attn_fwd_kernel's loads spills here: 256 VGPRs)
  auto gload = [&](const Blk& c, int kt) {
    const bf16_t* kp = p.k + c.b * p.k_sb + static_cast<int64_t>(c.hk) * p.k_sh;
    const bf16_t* vp = p.v + c.b * p.v_sb + static_cast<int64_t>(c.hk) * p.v_sh;
#pragma unroll
    for (int cc = 0; cc < CPT; ++cc) {
      const int ci = tid + NT * cc;
      const int row = ci / NCH, ch = ci % NCH;
      const int key = kt + row;
      if (key < p.Tk && ch < NCHL && (CPT_EXACT || ci < BK * NCH)) {
        kreg[cc] = load_bf16x8(kp + key * p.k_st + ch * 8);
        vreg[cc] = load_bf16x8(vp + key * p.v_st + ch * 8);
      } else {
        kreg[cc] = bf16x8{};
        vreg[cc] = bf16x8{};
      }
    }
  };
  const bool rope = p.rope_cos != nullptr;
  auto lwrite = [&](const Blk& c, int buf, int kt) {
    bf16_t* Kb = lds + buf * KVE;
    bf16_t* Vb = lds + (2 + buf) * KVE;
#pragma unroll
    for (int cc = 0; cc < CPT; ++cc) {
      const int ci = tid + NT * cc;
      if (!CPT_EXACT && ci >= BK * NCH) continue;
      const int row = ci / NCH, ch = ci % NCH;
      bf16x8 kv = kreg[cc];
      if constexpr (DP == D) {
        if (rope && p.rope_k)
          kv = rope_rot_chunk<NCH>(kv, ch, kt + row < p.Tk, static_cast<int64_t>(c.b) * p.Tk + kt + row,
                                   kt + row, p.rope_cos, p.rope_sin, p.rope_pos);
      }
      store_bf16x8(&Kb[swz<DP>(row, ch)], kv);
      store_bf16x8(&Vb[swz<DP>(row, ch)], vreg[cc]);
    }
  };
  // this wave's 32 Q rows of block c -> Qw by LDS-DMA: instruction j writes 1 KB lane-linear,
  // position j*64 + lane = (chunk 2j + lane/32, row lane%32) of the chunk-major image
  auto q_dma = [&](const Blk& c) {
    const bf16_t* qp = p.q + c.b * p.q_sb + static_cast<int64_t>(c.hq) * p.q_sh;
    const bf16_t* src = qp + static_cast<int64_t>(min(c.q0 + l32, p.Tq - 1)) * p.q_st + 8 * h;
#pragma unroll
    for (int j = 0; j < KS; ++j)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 16 * j),
                                       (__attribute__((address_space(3))) void*)(Qw + j * 512), 16, 0, 0);
  };
  s16x8 qf[KS];
  auto q_read = [&](const Blk& c) {  // after this wave's DMA has landed (vmcnt)
    const int qi = c.q0 + l32;
    float qv[KS][8];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf16x8 raw = *(const __attribute__((address_space(3))) bf16x8*)(Qw + ((2 * s + h) * 32 + l32) * 8);
      if (qi >= p.Tq) raw = bf16x8{};
#pragma unroll
      for (int j = 0; j < 8; ++j) qv[s][j] = bf2f(raw[j]);
    }
    if (DP == D && rope && qi < p.Tq) {
      const int pos = p.rope_pos ? p.rope_pos[static_cast<int64_t>(c.b) * p.Tq + qi] : qi;
      const float* cp = p.rope_cos + static_cast<int64_t>(pos) * (D / 2) + 8 * h;
      const float* sp = p.rope_sin + static_cast<int64_t>(pos) * (D / 2) + 8 * h;
#pragma unroll
      for (int s = 0; s < KS / 2; ++s) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float cs = cp[16 * s + j], sn = sp[16 * s + j];
          const float a = qv[s][j], bb = qv[s + KS / 2][j];
          qv[s][j] = a * cs - bb * sn;
          qv[s + KS / 2][j] = bb * cs + a * sn;
        }
      }
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = qv[s][j] * p.scale2;
      qf[s] = __builtin_bit_cast(s16x8, pack_bf16x8(t));
    }
    if (rope && p.q_rot != nullptr && qi < p.Tq) {
      bf16_t* qo = p.q_rot + c.b * p.qr_sb + qi * p.qr_st + static_cast<int64_t>(c.hq) * p.qr_sh + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) store_bf16x8(qo + 16 * s, pack_bf16x8(qv[s]));
    }
  };

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x16{};
  float m = -INFINITY, lsum = 0.f;

  auto tile = [&](const Blk& c, int kt, int buf) {
    const bf16_t* Ks = lds + buf * KVE;
    const bf16_t* Vs = lds + (2 + buf) * KVE;
    const int qi = c.q0 + l32;
    bool active = c.q0 < p.Tq && kt + BK > c.wseg_lo;
    if (CAUSAL) {
      active = active && (kt <= c.q0 + 31 + p.causal_off);
      if (p.window > 0) active = active && (kt + BK - 1 > c.q0 + p.causal_off - p.window);
    }
    if (!active) return;  // wave-uniform
    f32x16 sacc[2];
    if (p.fwd_prio == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      sacc[st] = f32x16{};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const s16x8 a = *reinterpret_cast<const s16x8*>(Ks + swz<DP>(32 * st + l32, 2 * s + h));
        sacc[st] = mfma32(a, qf[s], sacc[st]);
      }
    }
    if (p.fwd_prio == 1) __builtin_amdgcn_s_setprio(0);
    bool need_mask = kt < c.kbeg || kt + BK > c.kend || kt < c.wseg_hi;
    if (CAUSAL) {
      need_mask = need_mask || (kt + BK - 1 > c.q0 + p.causal_off);
      if (p.window > 0) need_mask = need_mask || (kt <= c.q0 + 31 + p.causal_off - p.window);
    }
    if (need_mask) {
      const int qseg = p.seg_start ? p.seg_start[static_cast<int64_t>(c.b) * p.Tq + min(qi, p.Tq - 1)] : 0;
      const int base = kt + 4 * h;
      int lo = max(c.kbeg, qseg) - base, hi = c.kend - base;
      if (CAUSAL) {
        hi = min(hi, qi + p.causal_off + 1 - base);
        if (p.window > 0) lo = max(lo, qi + p.causal_off - p.window + 1 - base);
      }
      const unsigned span = hi > lo ? static_cast<unsigned>(hi - lo) : 0u;
#pragma unroll
      for (int st = 0; st < 2; ++st) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int r = 32 * st + (i & 3) + 8 * (i >> 2);
          sacc[st][i] = static_cast<unsigned>(r - lo) < span ? sacc[st][i] : -INFINITY;
        }
      }
    }
    float mloc = -INFINITY;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int i = 0; i < 16; ++i) mloc = fmaxf(mloc, sacc[st][i]);
    mloc = xhalf_max(mloc);
    if (!__all(mloc <= m + kRescaleThr)) {
      const float mnew = fmaxf(m, mloc);
      const float alpha = ex2(m - (mnew == -INFINITY ? 0.f : mnew));
      m = mnew;
      lsum *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
    }
    const float muse = m == -INFINITY ? 0.f : m;
    float lpart[2] = {0.f, 0.f};  // two independent add chains (the row sum was one 32-add chain)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pv = ex2(sacc[st][i] - muse);
        sacc[st][i] = pv;
        lpart[st] += pv;
      }
    }
    lsum += lpart[0] + lpart[1];
    s16x8 pf[2][2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      pf[st][0] = pack8(sacc[st], 0);
      pf[st][1] = pack8(sacc[st], 8);
    }
    if (p.fwd_prio == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int c0 = 32 * dt + 16 * ((lane >> 4) & 1);
#pragma unroll
      for (int st = 0; st < 2; ++st) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const s16x8 a = tr_frag_perm<DP>(Vs, 32 * st + 16 * s + 4 * h, c0, lane);
          o[dt] = mfma32(a, pf[st][s], o[dt]);
        }
      }
    }
    if (p.fwd_prio == 1) __builtin_amdgcn_s_setprio(0);
  };

  auto epilogue = [&](const Blk& c) {
    const int qi = c.q0 + l32;
    const float ls = xhalf_sum(lsum);
    if (qi < p.Tq) {
      const float inv = ls > 0.f ? 1.f / ls : 0.f;
      bf16_t* op = p.o + c.b * p.o_sb + qi * p.o_st + static_cast<int64_t>(c.hq) * p.o_sh;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
        for (int g4 = 0; g4 < 4; g4 += 2) {
          uint2 a, cc;
          a.x = pack2bf(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv);
          a.y = pack2bf(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
          cc.x = pack2bf(o[dt][4 * g4 + 4] * inv, o[dt][4 * g4 + 5] * inv);
          cc.y = pack2bf(o[dt][4 * g4 + 6] * inv, o[dt][4 * g4 + 7] * inv);
          const auto rx = __builtin_amdgcn_permlane32_swap(a.x, cc.x, false, false);
          const auto ry = __builtin_amdgcn_permlane32_swap(a.y, cc.y, false, false);
          const int d = 32 * dt + 8 * g4 + 8 * h;
          if (d < D) *reinterpret_cast<uint4*>(op + d) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
        }
      }
      if (h == 0)
        p.lse2[(static_cast<int64_t>(c.b) * p.Hq + c.hq) * p.Tq + qi] = ls > 0.f ? m + __log2f(ls) : INFINITY;
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] = f32x16{};
    m = -INFINITY;
    lsum = 0.f;
  };

  int wb = 0, rb = 0;      // LDS buffer of the next tile written / computed
  bool staged = false;     // kreg / vreg hold the first tile of the block after `cur`
  // enter block y (its first tile staged or not), z = the block after it
  auto enter = [&](const Blk& y, const Blk& z) {
    if (y.ntiles > 0) {
      if (!staged) gload(y, y.tile0);
      lwrite(y, wb, y.tile0);
      wb ^= 1;
    }
    staged = false;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's Q DMA has landed
    q_read(y);
    if (y.ntiles > 1) {
      gload(y, y.tile0 + BK);
    } else if (z.valid && z.ntiles > 0) {
      gload(z, z.tile0);
      staged = true;
    }
    if (y.ntiles == 0 && z.valid) q_dma(z);  // no last tile to issue it from
  };

  // debug stamps, 100 MHz clock: per (workgroup, item < 8) tiles start / tiles done / seam
  // entered (next Q read, next loads issued) / epilogue issued
  auto stamp = [&](int item, int k) {
    if (p.stamps != nullptr && tid == 0 && item < 8)
      p.stamps[(static_cast<int64_t>(g) * 8 + item) * 4 + k] = __builtin_amdgcn_s_memrealtime();
  };
  int it = 0;
  Blk cur = make_blk(0);
  if (!cur.valid) return;  // workgroup-uniform (the host launches at most nblk workgroups)
  Blk nxt = make_blk(1);
  q_dma(cur);
  enter(cur, nxt);
  __syncthreads();
  for (;;) {
    stamp(it, 0);
    for (int t = 0; t < cur.ntiles; ++t) {
      const int kt = cur.tile0 + t * BK;
      const bool last = t + 1 == cur.ntiles;
      if (last && nxt.valid) q_dma(nxt);
      tile(cur, kt, rb);
      rb ^= 1;
      if (!last) {
        lwrite(cur, wb, kt + BK);
        wb ^= 1;
        if (t + 2 < cur.ntiles) {
          gload(cur, kt + 2 * BK);
        } else if (nxt.valid && nxt.ntiles > 0) {
          gload(nxt, nxt.tile0);
          staged = true;
        }
        __syncthreads();
      }
    }
    stamp(it, 1);
    ++it;
    const Blk z = nxt.valid ? make_blk(it + 1) : Blk{};
    if (nxt.valid) enter(nxt, z);
    stamp(it - 1, 2);
    epilogue(cur);
    stamp(it - 1, 3);
    if (!nxt.valid) break;
    cur = nxt;
    nxt = z;
    __syncthreads();
  }
}

// ==============================================================================================
// backward preprocessing: delta[b,h,t] = sum_d dO * O   (one wave per (b, t, h) row)
// ==============================================================================================
__global__ __launch_bounds__(256) void attn_bwd_delta_kernel(const bf16_t* __restrict__ o,
                                                              const bf16_t* __restrict__ dout,
                                                              int64_t o_sb, int64_t o_st,
                                                              int64_t o_sh, int64_t do_sb,
                                                              int64_t do_st, int64_t do_sh,
                                                              int B, int H, int T, int D,
                                                              float* __restrict__ delta) {
  // delta[row] = <O[row], dO[row]>: D/8 lanes x 16-B loads per row (16 lanes at D = 128),
  // 64 / (D/8) rows per wave, shuffle reduction inside the lane group. (Four rows per lane group
  // measured bitwise equal and slower inside the DPO step, 30.1 vs 27.3 us: removed.)
  constexpr int kDeltaRows = 1;
  const int lpr = D <= 64 ? 8 : 16;  // lanes per row (power of two; D = 80: 10 of 16 load)
  const int lane = threadIdx.x & 63;
  const int64_t row0 = ((blockIdx.x * 4ll + (threadIdx.x >> 6)) * (64 / lpr) + lane / lpr) * kDeltaRows;
  const int c = (lane % lpr) * 8;
  const int64_t nrows = static_cast<int64_t>(B) * H * T;
  bf16x8 a[kDeltaRows], g[kDeltaRows];
#pragma unroll
  for (int k = 0; k < kDeltaRows; ++k) {
    const int64_t row = row0 + k;
    a[k] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    g[k] = a[k];
    if (row < nrows && c < D) {
      const int t = static_cast<int>(row % T);
      const int64_t bh = row / T;
      const int hh = static_cast<int>(bh % H), b = static_cast<int>(bh / H);
      a[k] = load_bf16x8(o + b * o_sb + t * o_st + hh * o_sh + c);
      g[k] = load_bf16x8(dout + b * do_sb + t * do_st + hh * do_sh + c);
    }
  }
#pragma unroll
  for (int k = 0; k < kDeltaRows; ++k) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += bf2f(a[k][j]) * bf2f(g[k][j]);
    for (int off = 1; off < lpr; off <<= 1) acc += __shfl_xor(acc, off, 64);
    if (row0 + k < nrows && (lane % lpr) == 0) delta[row0 + k] = acc;
  }
}

// ==============================================================================================
// backward main kernel
// ==============================================================================================
// Query tiles [qt0, qend) swept by the workgroup that owns keys [k0, k0 + 256): every query
// that can see one of its keys. Shared by the main kernel and the dQ reduce pass (which must
// know exactly which slab rows a key block wrote).
template <bool CAUSAL>
__device__ __forceinline__ void bwd_q_range(int k0, int Tq, int causal_off, int window, int& qt0,
                                            int& qend) {
  int qlo = 0, qhi = Tq;
  if (CAUSAL) {
    qlo = max(0, k0 - causal_off);
    if (window > 0) qhi = min(qhi, k0 + kAttnBwdKeys - 1 - causal_off + window);
  }
  qt0 = (qlo / kAttnBwdQRows) * kAttnBwdQRows;
  qend = max(qhi, qt0);
}

// Workgroup = 4 waves, ONE per SIMD (the 512-register budget holds the accumulators) = 256 keys
// of one (batch, kv head) and Hq/Hkv/hsplit of its query heads. Wave w owns keys
// k0 + 64w .. +63 as two 32-key sub-tiles and keeps dK^T / dV^T of all 64 in accumulators (256
// registers at D = 128) for the whole sweep over (head, 32-query tile), so dK/dV need no
// cross-workgroup sum (cdna guide Appendix B "Attention backward"). Per query tile:
//   phase A, per sub-tile: S = Q K^T and dP = dO V^T with the key on the lane (K, V rows of the
//     wave's keys and the Q / dO tile from LDS); p = exp2(scale2*S - lse2), dS = p (dP - delta)
//     with the row constants read straight from L2 while the MFMA chains run; dV^T += dO^T P
//     and dK^T += Q^T dS from transposed LDS reads (P and dS are already the B operands);
//     dS^T -> LDS.
//   barrier
//   phase B: the next Q / dO tile (register-prefetched one tile ahead) is staged into LDS, and
//     wave w computes dQ[32 q][32w .. 32w+31] = scale * dS K over all 256 keys and stores it
//     into this key block's fp32 slab row. Plain stores, no atomics: the reduce pass sums the
//     <= ceil(Tk/256) slabs of each row in key-block order, so dQ is deterministic and the
//     chip-wide float-atomic rate is no floor (it was for the earlier 128-key atomic version).
//   barrier
// LDS at D = 128: K 64 KB + V 64 KB + Q 8 KB + dO 8 KB + dS 16 KB = the full 160 KB.
// Every LDS read address is one of ~26 lane offsets computed once plus a wave-uniform or
// compile-time row offset (the swizzles are periodic): with one address register per unrolled
// read the kernel spilled, the dK/dV accumulators holding the whole AGPR file.
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void attn_bwd_kernel(AttnBwdParams p) {
  constexpr int BKV = kAttnBwdKeys, BQ = kAttnBwdQRows;
  constexpr int DP = attn_dp<D>();  // LDS row width (zero-padded to the 32-column tiles)
  constexpr int NCH = DP / 8;
  constexpr int NCHL = D / 8;       // chunks loaded from memory
  constexpr int KS = D / 16;
  constexpr int DT = DP / 32;
  constexpr int QCPT = (BQ * NCH + 255) / 256;  // 16-B chunks per thread per [32][DP] tile
  constexpr bool Q_EXACT = (BQ * NCH) % 256 == 0;
  static_assert(QCPT >= 1 && BKV == 256 && BQ == 32, "tile geometry");
  __shared__ __attribute__((aligned(16))) bf16_t Ks[BKV * DP];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[BKV * DP];
  __shared__ __attribute__((aligned(16))) bf16_t Qs[BQ * DP];
  __shared__ __attribute__((aligned(16))) bf16_t dOs[BQ * DP];
  __shared__ __attribute__((aligned(16))) bf16_t dSs[BKV * BQ];

  // readfirstlane: the wave index is wave-uniform, so everything derived from it (key / query
  // ranges, activity and mask flags) stays in SGPRs and its branches are scalar
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int group = p.Hq / p.Hkv;
  const int hpb = group / p.hsplit;  // query heads per workgroup
  const int nrest = p.Hkv * p.B * p.hsplit;
  const int kb = static_cast<int>(blockIdx.x) / nrest;  // key blocks outermost: heaviest first
  int rest = static_cast<int>(blockIdx.x) - kb * nrest;
  const int sidx = rest % p.hsplit;
  rest /= p.hsplit;
  const int hk = rest % p.Hkv, b = rest / p.Hkv;
  const int k0 = kb * BKV;
  const int kw = k0 + 64 * w;  // this wave's first key
  const int kbeg = p.kv_start ? p.kv_start[b] : 0;
  const int kend = p.kv_end ? p.kv_end[b] : p.Tk;

  // kernel-uniform: k arrives un-rotated (q comes pre-rotated: the forward's q_rot output)
  const bool rope_in = p.rope_inputs != 0;
  {  // K and V blocks -> LDS (rows past Tk zeroed; K rotated on the way with RoPE on load)
    const bf16_t* kp = p.k + b * p.k_sb + static_cast<int64_t>(hk) * p.k_sh;
    const bf16_t* vp = p.v + b * p.v_sb + static_cast<int64_t>(hk) * p.v_sh;
#pragma unroll 4
    for (int c = 0; c < BKV * NCH / 256; ++c) {
      const int ci = tid + 256 * c;
      const int row = ci / NCH, ch = ci % NCH;
      const int key = k0 + row;
      const bool in = key < p.Tk && ch < NCHL;
      bf16x8 kv = in ? load_bf16x8(kp + key * p.k_st + ch * 8) : bf16x8{};
      if constexpr (DP == D) {
        if (rope_in)
          kv = rope_rot_chunk<NCH>(kv, ch, in, static_cast<int64_t>(b) * p.Tk + key, key, p.rope_cos,
                                   p.rope_sin, p.rope_pos);
      }
      store_bf16x8(Ks + swz<DP>(row, ch), kv);
      store_bf16x8(Vs + swz<DP>(row, ch), in ? load_bf16x8(vp + key * p.v_st + ch * 8) : bf16x8{});
    }
  }

  int qt0, qend;
  bwd_q_range<CAUSAL>(k0, p.Tq, p.causal_off, p.window, qt0, qend);
  const int nqt = (qend - qt0 + BQ - 1) / BQ;
  const bool block_has_keys = k0 < kend && k0 + BKV > kbeg;
  const int n_iter = block_has_keys ? hpb * nqt : 0;
  const int hq0 = hk * group + sidx * hpb;

  // register prefetch of the next (head, q-tile)'s Q and dO rows
  bf16x8 qreg[QCPT], dreg[QCPT];
  auto prefetch = [&](int it) {
    const int hq = hq0 + it / nqt;
    const int qt = qt0 + (it % nqt) * BQ;
    const bf16_t* qp = p.q + b * p.q_sb + static_cast<int64_t>(hq) * p.q_sh;
    const bf16_t* dop = p.dout + b * p.do_sb + static_cast<int64_t>(hq) * p.do_sh;
#pragma unroll
    for (int c = 0; c < QCPT; ++c) {
      const int ci = tid + 256 * c;
      const int row = ci / NCH, ch = ci % NCH;
      if ((!Q_EXACT && ci >= BQ * NCH) || ch >= NCHL) {  // pad columns (D = 80): zero
        qreg[c] = bf16x8{};
        dreg[c] = bf16x8{};
      } else if (qt + BQ <= p.Tq) {  // full tile (wave-uniform)
        qreg[c] = load_bf16x8(qp + (qt + row) * p.q_st + ch * 8);
        dreg[c] = load_bf16x8(dop + (qt + row) * p.do_st + ch * 8);
      } else {  // rows past Tq: loaded clamped (unpredicated), zeroed
        const int qq = min(qt + row, p.Tq - 1);
        const bf16x8 a = load_bf16x8(qp + qq * p.q_st + ch * 8);
        const bf16x8 g = load_bf16x8(dop + qq * p.do_st + ch * 8);
        const bool in = qt + row < p.Tq;
        qreg[c] = in ? a : bf16x8{};
        dreg[c] = in ? g : bf16x8{};
      }
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int c = 0; c < QCPT; ++c) {
      const int ci = tid + 256 * c;
      if (!Q_EXACT && ci >= BQ * NCH) continue;
      const int row = ci / NCH, ch = ci % NCH;
      store_bf16x8(Qs + swz<DP>(row, ch), qreg[c]);
      store_bf16x8(dOs + swz<DP>(row, ch), dreg[c]);
    }
  };

  // Lane-dependent LDS offsets (elements), computed once. swz is periodic in 16 rows and ds_off
  // in 32 rows, so every read below is one of these + a wave-uniform / compile-time row offset.
  const int i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3, half16 = (lane >> 4) & 1;
  int roff[KS];  // row reads: row l32 (+16k), chunk 2s + h
#pragma unroll
  for (int s = 0; s < KS; ++s) roff[s] = swz<DP>(l32, 2 * s + h);
  int toff[DT][2];  // tr_frag_perm: rows 4h + qq and 4h + 8 + qq (+16k), columns 32dt + 16*half16
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const int ch = 4 * dt + 2 * half16 + (pp >> 1), sub = (pp & 1) * 4;
    toff[dt][0] = swz<DP>(4 * h + qq, ch) + sub;
    toff[dt][1] = swz<DP>(4 * h + 8 + qq, ch) + sub;
  }
  int noff[2];  // phase B K reads (tr_frag_nat): rows 8h + qq and 8h + 4 + qq (+16s), dt = w
  {
    const int ch = 4 * (w % DT) + 2 * half16 + (pp >> 1), sub = (pp & 1) * 4;
    noff[0] = swz<DP>(8 * h + qq, ch) + sub;
    noff[1] = swz<DP>(8 * h + 4 + qq, ch) + sub;
  }
  int doff[2][2];  // phase B dS^T reads: rows 16*par + 8h + qq (+4) (+32k), query unit colc4
  {
    const int colc4 = (16 * half16 + 4 * pp) >> 2;
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      doff[par][0] = ds_off(16 * par + 8 * h + qq, colc4);
      doff[par][1] = ds_off(16 * par + 8 * h + 4 + qq, colc4);
    }
  }
  int woff[4];  // dS^T writes: row l32 (+32k), 8-byte units 2g + h
#pragma unroll
  for (int g = 0; g < 4; ++g) woff[g] = ds_off(l32, 2 * g + h);

  // packed sequences: key kj is seen only by queries < seg_end[kj] (non-decreasing in kj); per
  // sub-tile j: this lane's bound and the wave-uniform bounds of its first / last key
  const int* se = p.seg_end ? p.seg_end + static_cast<int64_t>(b) * p.Tk : nullptr;
  int kse[2], kse_lo[2], kse_hi[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    kse[j] = kse_lo[j] = kse_hi[j] = 0x7fffffff;
    if (se) {
      const int kj0 = kw + 32 * j;
      kse[j] = se[min(kj0 + l32, p.Tk - 1)];
      kse_lo[j] = __builtin_amdgcn_readfirstlane(se[min(kj0, p.Tk - 1)]);
      kse_hi[j] = __builtin_amdgcn_readfirstlane(se[min(kj0 + 31, p.Tk - 1)]);
    }
  }

  f32x16 dk[2][DT], dv[2][DT];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      dk[j][dt] = f32x16{};
      dv[j][dt] = f32x16{};
    }
  }

  // Row constants (log2-domain LSE, delta) of this lane's 16 accumulator rows
  // r = (i&3) + 8(i>>2) + 4h = four runs of 4 consecutive rows: 4 + 4 dwordx4 loads, issued in
  // phase B of the previous tile so that no memory wait sits in front of the MFMA chains (one
  // dword load per row, issued at the top of the tile, cost a full round trip per tile).
  f32x4 lr4[4], dl4[4];
  const bool rows_vec = (p.Tq & 3) == 0;
  auto load_rows = [&](int it) {
    const int hq = hq0 + it / nqt;
    const int qt = qt0 + (it % nqt) * BQ;
    const int64_t rb = (static_cast<int64_t>(b) * p.Hq + hq) * p.Tq;
    if (rows_vec && qt + BQ <= p.Tq) {  // full tile (wave-uniform), 16-B aligned runs
      const float* lp = p.lse2 + rb + qt + 4 * h;
      const float* dp = p.delta + rb + qt + 4 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        lr4[g] = *reinterpret_cast<const f32x4*>(lp + 8 * g);
        dl4[g] = *reinterpret_cast<const f32x4*>(dp + 8 * g);
      }
    } else {  // partial tile / odd Tq: clamped unpredicated loads, rows past Tq masked (p = 0)
      const int rlim = p.Tq - qt - 4 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 8 * g + e;
          const int64_t ri = rb + min(qt + 4 * h + r, p.Tq - 1);
          const float a = p.lse2[ri], c = p.delta[ri];
          lr4[g][e] = r < rlim ? a : INFINITY;
          dl4[g][e] = r < rlim ? c : 0.f;
        }
      }
    }
  };

  if (n_iter > 0) {
    prefetch(0);
    stage();
    load_rows(0);
    if (n_iter > 1) prefetch(1);
  }
  __syncthreads();

  for (int it = 0; it < n_iter; ++it) {
    const int hq = hq0 + it / nqt;
    const int qt = qt0 + (it % nqt) * BQ;

    // which of the two 32-key sub-tiles see a query of the tile, which need masks (wave-uniform)
    bool act[2], need_mask[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kj0 = kw + 32 * j;
      act[j] = kj0 < kend && kj0 + 32 > kbeg && qt < kse_hi[j];
      need_mask[j] = kj0 < kbeg || kj0 + 32 > kend || qt + BQ > p.Tq || qt + BQ > kse_lo[j];
      if (CAUSAL) {
        act[j] = act[j] && kj0 <= qt + BQ - 1 + p.causal_off;
        need_mask[j] = need_mask[j] || (kj0 + 31 > qt + p.causal_off);
        if (p.window > 0) {
          act[j] = act[j] && (kj0 + 31 > qt + p.causal_off - p.window);
          need_mask[j] = need_mask[j] || (kj0 <= qt + BQ - 1 + p.causal_off - p.window);
        }
      }
    }

    // ---------------------------------------------------------------- phase A
    // per sub-tile: S = Q K^T and dP = dO V^T (key on the lane), two MFMA chains; every
    // fragment is read one k-step ahead and sched_barriers pin that order: at one wave per
    // SIMD, a read the compiler sinks onto its MFMA stalls the matrix pipe for the whole LDS
    // latency. Then P and dS (zero for an inactive sub-tile), packed as the bf16 B operands of
    // the dV / dK products. (Both sub-tiles' chains at once need 64 accumulators on top of the
    // 256 dK / dV ones: the compiler then spills.)
    s16x8 pb0[2], pb1[2], sb0[2], sb1[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      pb0[j] = pb1[j] = sb0[j] = sb1[j] = s16x8{};
      if (act[j]) {
        f32x16 sacc = f32x16{}, dpacc = f32x16{};
        const bf16_t* Kj = Ks + (64 * w + 32 * j) * DP;
        const bf16_t* Vj = Vs + (64 * w + 32 * j) * DP;
        s16x8 fa[2], fb[2], fc[2], fd[2];
        auto ld_sdp = [&](int s, int sl) {
          fa[sl] = *reinterpret_cast<const s16x8*>(Qs + roff[s]);
          fb[sl] = *reinterpret_cast<const s16x8*>(Kj + roff[s]);
          fc[sl] = *reinterpret_cast<const s16x8*>(dOs + roff[s]);
          fd[sl] = *reinterpret_cast<const s16x8*>(Vj + roff[s]);
        };
        ld_sdp(0, 0);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          if (s + 1 < KS) ld_sdp(s + 1, (s + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);
          sacc = mfma32(fa[s & 1], fb[s & 1], sacc);
          dpacc = mfma32(fc[s & 1], fd[s & 1], dpacc);
          __builtin_amdgcn_sched_barrier(0);
        }
        // masking is branch-free per lane: key kj vs query qt + rr + 4h, visible iff rr in
        // [lo, hi), one unsigned compare per element
        const int kj = kw + 32 * j + l32;
        int lo = 0, hi = min(p.Tq, kse[j]) - qt - 4 * h;
        if (kj < kbeg || kj >= kend) hi = 0;
        if (CAUSAL) {
          const int dlt = kj - qt - p.causal_off - 4 * h;  // visible iff rr >= dlt
          lo = max(lo, dlt);
          if (p.window > 0) hi = min(hi, dlt + p.window);
        }
        const unsigned span = hi > lo ? static_cast<unsigned>(hi - lo) : 0u;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int rr = (i & 3) + 8 * (i >> 2);
          float pv = ex2(fmaf(sacc[i], p.scale2, -lr4[i >> 2][i & 3]));
          if (need_mask[j]) pv = static_cast<unsigned>(rr - lo) < span ? pv : 0.f;
          sacc[i] = pv;
          dpacc[i] = pv * (dpacc[i] - dl4[i >> 2][i & 3]);
        }
        pb0[j] = pack8(sacc, 0);
        pb1[j] = pack8(sacc, 8);
        sb0[j] = pack8(dpacc, 0);
        sb1[j] = pack8(dpacc, 8);
      }
    }

    // transposed dO / Q fragments of column tile dt (A operands of dV^T += dO^T P and
    // dK^T += Q^T dS, k = query in the accumulator's permuted row order), shared by both
    // sub-tiles
    s16x8 ta[2], tb[2], tc[2], td[2];
    auto ld_kv = [&](int dt, int sl) {
      ta[sl] = cat4(tr_read(dOs + toff[dt][0]), tr_read(dOs + toff[dt][1]));
      tb[sl] = cat4(tr_read(dOs + 16 * DP + toff[dt][0]), tr_read(dOs + 16 * DP + toff[dt][1]));
      tc[sl] = cat4(tr_read(Qs + toff[dt][0]), tr_read(Qs + toff[dt][1]));
      td[sl] = cat4(tr_read(Qs + 16 * DP + toff[dt][0]), tr_read(Qs + 16 * DP + toff[dt][1]));
    };
    ld_kv(0, 0);
    __builtin_amdgcn_sched_barrier(0);

    // dV^T += dO^T P ; dK^T += Q^T dS for both sub-tiles; the four transposed fragments of
    // column tile dt+1 are read while tile dt's eight MFMAs run. The MFMAs run unconditionally
    // (zero P / dS when inactive): accumulators updated under a branch get phi copies, which
    // for 256 accumulator registers means spilling every iteration.
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      if (dt + 1 < DT) ld_kv(dt + 1, (dt + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        dv[j][dt] = mfma32(ta[dt & 1], pb0[j], dv[j][dt]);
        dv[j][dt] = mfma32(tb[dt & 1], pb1[j], dv[j][dt]);
        dk[j][dt] = mfma32(tc[dt & 1], sb0[j], dk[j][dt]);
        dk[j][dt] = mfma32(td[dt & 1], sb1[j], dk[j][dt]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // dS^T rows -> [key][32 queries] image: accumulator rows 4g..4g+3 are queries 8g + 4h + 0..3,
    // i.e. 8-byte unit 2g + h of the key's row
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const u32x4 ds0 = __builtin_bit_cast(u32x4, sb0[j]), ds1 = __builtin_bit_cast(u32x4, sb1[j]);
      bf16_t* dSw = dSs + (64 * w + 32 * j) * 32;
      *reinterpret_cast<uint2*>(dSw + woff[0]) = make_uint2(ds0[0], ds0[1]);
      *reinterpret_cast<uint2*>(dSw + woff[1]) = make_uint2(ds0[2], ds0[3]);
      *reinterpret_cast<uint2*>(dSw + woff[2]) = make_uint2(ds1[0], ds1[1]);
      *reinterpret_cast<uint2*>(dSw + woff[3]) = make_uint2(ds1[2], ds1[3]);
    }
    __syncthreads();  // dS visible; every wave is done reading this Q / dO tile

    // ---------------------------------------------------------------- phase B
    if (it + 1 < n_iter) {  // stage the next tile, prefetch the one after it + next row constants
      stage();
      if (it + 2 < n_iter) prefetch(it + 2);
      load_rows(it + 1);
    }
    if (w < DT) {  // dQ partial; D = 64: waves 2, 3 have no column slice (D = 80: wave 3)
      const int dt = w;
      f32x16 acc = f32x16{};
      s16x8 qa[2], qb[2];
      auto ld_dq = [&](int s, int sl) {  // A = dS (rows 16s + 8h..), B = K (rows 16s + 8h..)
        const bf16_t* dsr = dSs + (s >> 1) * 32 * 32;
        qa[sl] = cat4(tr_read(dsr + doff[s & 1][0]), tr_read(dsr + doff[s & 1][1]));
        qb[sl] = cat4(tr_read(Ks + 16 * s * DP + noff[0]), tr_read(Ks + 16 * s * DP + noff[1]));
      };
      ld_dq(0, 0);
#pragma unroll
      for (int s = 0; s < BKV / 16; ++s) {
        if (s + 1 < BKV / 16) ld_dq(s + 1, (s + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
        acc = mfma32(qa[s & 1], qb[s & 1], acc);
        __builtin_amdgcn_sched_barrier(0);
      }
      // lane holds column d = 32dt + l32, rows q = qt + (i&3) + 8(i>>2) + 4h (128-B row segments)
      // (slab rows are padded to a multiple of 32: every store is in bounds, none predicated)
      const int64_t rs = static_cast<int64_t>(p.Hq) * D;
      float* sp = p.dq_slab + ((static_cast<int64_t>(kb) * p.B + b) * p.slab_rows + qt) * rs +
                  static_cast<int64_t>(hq) * D + 32 * dt + l32;
      if (32 * dt + l32 < D) {  // (the pad columns of D = 80 are not stored)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int r = (i & 3) + 8 * (i >> 2) + 4 * h;
          sp[r * rs] = acc[i] * p.scale;
        }
      }
    }
    __syncthreads();  // next Q / dO tile visible; every wave is done reading dS
  }

  // dK (scaled) and dV: lane = key, registers = d rows (i&3) + 8(i>>2) + 4h of column tile dt
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int kj = kw + 32 * j + l32;
    if (kj >= p.Tk) continue;
    if (p.hsplit == 1) {
      bf16_t* dkp = p.dk + b * p.dk_sb + kj * p.dk_st + static_cast<int64_t>(hk) * p.dk_sh;
      bf16_t* dvp = p.dv + b * p.dv_sb + kj * p.dv_st + static_cast<int64_t>(hk) * p.dv_sh;
      // widened stores (T21, as the forward's O): permlane32_swap pairs 8-column groups so
      // each lane writes 16 contiguous bytes
      auto store_row = [&](bf16_t* dst, f32x16 x, float sc, int dt) {
#pragma unroll
        for (int g4 = 0; g4 < 4; g4 += 2) {
          const uint32_t a0 = pack2bf(x[4 * g4] * sc, x[4 * g4 + 1] * sc);
          const uint32_t a1 = pack2bf(x[4 * g4 + 2] * sc, x[4 * g4 + 3] * sc);
          const uint32_t c0 = pack2bf(x[4 * g4 + 4] * sc, x[4 * g4 + 5] * sc);
          const uint32_t c1 = pack2bf(x[4 * g4 + 6] * sc, x[4 * g4 + 7] * sc);
          const auto r0 = __builtin_amdgcn_permlane32_swap(a0, c0, false, false);
          const auto r1 = __builtin_amdgcn_permlane32_swap(a1, c1, false, false);
          if (32 * dt + 8 * g4 + 8 * h < D)
            *reinterpret_cast<uint4*>(dst + 32 * dt + 8 * g4 + 8 * h) = make_uint4(r0[0], r1[0], r0[1], r1[1]);
        }
      };
      if (D == 80 && p.rope_cos != nullptr) {  // partial rotary (rot = 32): column tile 0 only
        const int pos = p.rope_pos ? p.rope_pos[static_cast<int64_t>(b) * p.Tk + kj] : kj;
        store_row(dkp, unrotate_tile0_rot32(dk[j][0], p.rope_cos + static_cast<int64_t>(pos) * 16 + 4 * h,
                                            p.rope_sin + static_cast<int64_t>(pos) * 16 + 4 * h),
                  p.scale, 0);
#pragma unroll
        for (int dt = 1; dt < DT; ++dt) store_row(dkp, dk[j][dt], p.scale, dt);
      } else if (DP == D && p.rope_cos != nullptr) {
        // fused RoPE backward: column d < D/2 pairs with d + D/2 = the same register of column
        // tile dt + DT/2 in this lane (un-rotation: lo = a c + b s, hi = b c - a s), applied to
        // register copies on the way out (writing the accumulators back spilled in the loop)
        const int pos = p.rope_pos ? p.rope_pos[static_cast<int64_t>(b) * p.Tk + kj] : kj;
        const float* cp = p.rope_cos + static_cast<int64_t>(pos) * (D / 2) + 4 * h;
        const float* sp = p.rope_sin + static_cast<int64_t>(pos) * (D / 2) + 4 * h;
#pragma unroll
        for (int dt = 0; dt < DT / 2; ++dt) {
          f32x16 lo = dk[j][dt], hi = dk[j][dt + DT / 2];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 c4 = *reinterpret_cast<const f32x4*>(cp + 32 * dt + 8 * g);
            const f32x4 s4 = *reinterpret_cast<const f32x4*>(sp + 32 * dt + 8 * g);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float a = lo[4 * g + e], bb = hi[4 * g + e];
              lo[4 * g + e] = a * c4[e] + bb * s4[e];
              hi[4 * g + e] = bb * c4[e] - a * s4[e];
            }
          }
          store_row(dkp, lo, p.scale, dt);
          store_row(dkp, hi, p.scale, dt + DT / 2);
        }
      } else {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) store_row(dkp, dk[j][dt], p.scale, dt);
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) store_row(dvp, dv[j][dt], 1.f, dt);
    } else {  // fp32 partials of this head subset, summed by attn_dkv_reduce_kernel
      const int64_t off = ((static_cast<int64_t>(sidx) * p.B + b) * p.Tk + kj) * p.Hkv * D +
                          static_cast<int64_t>(hk) * D;
      float* dkp = p.dk_part + off;
      float* dvp = p.dv_part + off;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d = 32 * dt + 8 * g4 + 4 * h;
          if (d >= D) continue;
          *reinterpret_cast<f32x4*>(dkp + d) = f32x4{dk[j][dt][4 * g4], dk[j][dt][4 * g4 + 1],
                                                     dk[j][dt][4 * g4 + 2], dk[j][dt][4 * g4 + 3]};
          *reinterpret_cast<f32x4*>(dvp + d) = f32x4{dv[j][dt][4 * g4], dv[j][dt][4 * g4 + 1],
                                                     dv[j][dt][4 * g4 + 2], dv[j][dt][4 * g4 + 3]};
        }
      }
    }
  }
}

// ----------------------------------------------------------------------------------------------
// backward, 8-wave variant (two waves per SIMD)
// ----------------------------------------------------------------------------------------------
// Same workgroup geometry, LDS images, slab and partial outputs as attn_bwd_kernel (256 keys per
// workgroup, 32-query tiles, 160 KB LDS), but 8 waves of ONE 32-key sub-tile each: dK^T / dV^T of
// a wave are 128 accumulators at D = 128, so two waves fit one SIMD's register file and each
// hides the other's LDS / memory latency (attn_bwd_kernel, one wave per SIMD, exposes it: ~25 %
// MFMA busy). To fit 256 registers:
//   * the row constants (LSE, delta) are loaded straight into the score / dP accumulators, which
//     then start at -lse2/scale2 and -delta (S - lse and dP - delta come out of the MFMA chains);
//   * fragment reads are single-buffered: the other wave of the SIMD fills the gaps;
//   * dQ uses 16x16x32 MFMAs over 16-column slices of d (wave w: columns 16w..16w+15, both
//     16-query halves), so a wave holds 8 dQ accumulators.
// Causal sub-tiles that see no query of a tile skip all their MFMAs (wave-uniform branch).
// Phase timestamps for one workgroup (tools/attn_bwd_probe.hip builds with DLA_BWD_TRACE; the
// extension never defines it): s_memtime per (wave, tile, point), vector-stored by lane 0.
#ifdef DLA_BWD_TRACE
__device__ long long g_bwd_trace[8 * 64 * 8];
#define BWD_TS(k)                                                                         \
  do {                                                                                    \
    if (blockIdx.x == DLA_BWD_TRACE && lane == 0 && it < 64)                              \
      g_bwd_trace[(w * 64 + it) * 8 + (k)] = static_cast<long long>(__builtin_amdgcn_s_memtime()); \
  } while (0)
#else
#define BWD_TS(k) \
  do {            \
  } while (0)
#endif

template <int D, bool CAUSAL>
__global__ __launch_bounds__(512) void attn_bwd8_kernel(AttnBwdParams p) {
  constexpr int BKV = kAttnBwdKeys, BQ = kAttnBwdQRows, NT = 512;
  constexpr int DP = attn_dp<D>();
  constexpr int NCH = DP / 8;
  constexpr int NCHL = D / 8;
  constexpr int KS = D / 16;
  constexpr int DT = DP / 32;
  constexpr int NDS = D / 16;  // 16-column dQ slices: 8 (D = 128), 5 (80), 4 (64)
  constexpr bool Q_EXACT = BQ * NCH == NT;
  static_assert(BQ * NCH <= NT && (BKV * NCH) % NT == 0 && BKV == 256 && BQ == 32, "tile geometry");
  // one array, small images first: Q / dO / dS addresses stay inside the 16-bit ds_read
  // immediate of one base register (Q and dO reads share an address VGPR, +8 KB)
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * BQ * DP + BKV * BQ + 2 * BKV * DP];
  bf16_t* const Qs = lds;
  bf16_t* const dOs = lds + BQ * DP;
  bf16_t* const dSs = lds + 2 * BQ * DP;
  bf16_t* const Ks = dSs + BKV * BQ;
  bf16_t* const Vs = Ks + BKV * DP;

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int group = p.Hq / p.Hkv;
  const int hpb = group / p.hsplit;
  const int nrest = p.Hkv * p.B * p.hsplit;
  const int kb = static_cast<int>(blockIdx.x) / nrest;
  int rest = static_cast<int>(blockIdx.x) - kb * nrest;
  const int sidx = rest % p.hsplit;
  rest /= p.hsplit;
  const int hk = rest % p.Hkv, b = rest / p.Hkv;
  const int k0 = kb * BKV;
  const int kw = k0 + 32 * w;  // this wave's 32 keys
  const int kbeg = p.kv_start ? p.kv_start[b] : 0;
  const int kend = p.kv_end ? p.kv_end[b] : p.Tk;

  const bool rope_in = p.rope_inputs != 0;
  {  // K and V blocks -> LDS (as attn_bwd_kernel; 16 consecutive lanes hold one row)
    const bf16_t* kp = p.k + b * p.k_sb + static_cast<int64_t>(hk) * p.k_sh;
    const bf16_t* vp = p.v + b * p.v_sb + static_cast<int64_t>(hk) * p.v_sh;
#pragma unroll 2
    for (int c = 0; c < BKV * NCH / NT; ++c) {
      const int ci = tid + NT * c;
      const int row = ci / NCH, ch = ci % NCH;
      const int key = k0 + row;
      const bool in = key < p.Tk && ch < NCHL;
      bf16x8 kv = in ? load_bf16x8(kp + key * p.k_st + ch * 8) : bf16x8{};
      if constexpr (DP == D) {
        if (rope_in)
          kv = rope_rot_chunk<NCH>(kv, ch, in, static_cast<int64_t>(b) * p.Tk + key, key, p.rope_cos,
                                   p.rope_sin, p.rope_pos);
      }
      store_bf16x8(Ks + swz<DP>(row, ch), kv);
      store_bf16x8(Vs + swz<DP>(row, ch), in ? load_bf16x8(vp + key * p.v_st + ch * 8) : bf16x8{});
    }
  }

  int qt0, qend;
  bwd_q_range<CAUSAL>(k0, p.Tq, p.causal_off, p.window, qt0, qend);
  const int nqt = (qend - qt0 + BQ - 1) / BQ;
  const bool block_has_keys = k0 < kend && k0 + BKV > kbeg;
  const int n_iter = block_has_keys ? hpb * nqt : 0;
  const int hq0 = hk * group + sidx * hpb;

  // register prefetch of the next (head, q-tile)'s Q and dO rows: one 16-B chunk per thread.
  // Global addresses in the loop are a wave-uniform (SGPR) base + a 32-bit lane byte offset
  // (SGPR-base addressing): per-lane 64-bit pointers cost two registers each and spilled.
  const int qrow = tid / NCH, qch = tid % NCH;
  const bool qslot = (Q_EXACT || tid < BQ * NCH) && qch < NCHL;
  const uint32_t qlo = static_cast<uint32_t>(qrow * p.q_st + qch * 8) * 2u;
  const uint32_t dlo = static_cast<uint32_t>(qrow * p.do_st + qch * 8) * 2u;
  bf16x8 qreg, dreg;
  auto gld = [](const bf16_t* base, uint32_t off) {
    return load_bf16x8(reinterpret_cast<const bf16_t*>(reinterpret_cast<const char*>(base) + off));
  };
  // (head, q-tile) of a tile index, advanced incrementally (no per-tile integer division):
  // heads outer, tiles inner
  const int qtend = qt0 + nqt * BQ;
  auto advance = [&](int& hq, int& qt) {
    qt += BQ;
    if (qt >= qtend) {
      qt = qt0;
      ++hq;
    }
  };
  auto prefetch = [&](int hq, int qt) {
    const bf16_t* qp = p.q + b * p.q_sb + static_cast<int64_t>(hq) * p.q_sh;
    const bf16_t* dop = p.dout + b * p.do_sb + static_cast<int64_t>(hq) * p.do_sh;
    if (!qslot) {
      qreg = bf16x8{};
      dreg = bf16x8{};
    } else if (qt + BQ <= p.Tq) {
      qreg = gld(qp + static_cast<int64_t>(qt) * p.q_st, qlo);
      dreg = gld(dop + static_cast<int64_t>(qt) * p.do_st, dlo);
    } else {
      const int qq = min(qt + qrow, p.Tq - 1);
      const bf16x8 a = load_bf16x8(qp + qq * p.q_st + qch * 8);
      const bf16x8 g = load_bf16x8(dop + qq * p.do_st + qch * 8);
      const bool in = qt + qrow < p.Tq;
      qreg = in ? a : bf16x8{};
      dreg = in ? g : bf16x8{};
    }
  };
  auto stage = [&]() {
    if (Q_EXACT || tid < BQ * NCH) {
      store_bf16x8(Qs + swz<DP>(qrow, qch), qreg);
      store_bf16x8(dOs + swz<DP>(qrow, qch), dreg);
    }
  };

  const int i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3, half16 = (lane >> 4) & 1, g4l = lane >> 4;
  // Lane constants of the LDS addresses. Every swizzled address is base + ((k ^ x) << 3) with a
  // compile-time k (the chunk index minus the bits the XOR never touches), so a handful of
  // bases replace one address register per (image, k-step); they are made opaque at the top of
  // every tile (asm barrier) so the derived addresses are formed next to their reads instead of
  // being hoisted out of the loop (which costs a register each and spilled).
  constexpr int FMASK = (NCH & (NCH - 1)) == 0 ? NCH - 1 : 3;  // as swz<DP>
  auto swzf = [](int row) { return (((row & 3) << 2) | ((row >> 2) & 3)) & FMASK; };
  // row reads (row l32, chunk 2s + h): swz<DP>(l32, 2s + h) = rq + ((2s ^ rx) << 3)
  int rq = l32 * DP, rx = h ^ swzf(l32);
  // transposed Q / dO reads (rows 4h + qq, 4h + 8 + qq; chunk 4dt + c1, c1 < 4)
  const int c1 = 2 * half16 + (pp >> 1);
  int tq0 = (4 * h + qq) * DP + (pp & 1) * 4, tx0 = c1 ^ swzf(4 * h + qq);
  int tq1 = (4 * h + 8 + qq) * DP + (pp & 1) * 4, tx1 = c1 ^ swzf(4 * h + 8 + qq);
  // dS^T writes: ds_off(l32, 2g + h) = wq + ((2g ^ wx) << 2)
  int wq = l32 * 32, wx = h ^ ds_swz(l32);
  // phase B (16x16x32 dQ): A = dS rows (keys) 8*g4l + qq (+4) of query columns 16t + i16,
  // B = K rows 8*g4l + qq (+4) of d columns 16*slice + i16; both + 32 keys per k-step
  constexpr int DQT = NDS == 4 ? 1 : 2;  // query halves per wave (D = 64: 8 waves x 1 half)
  const int dslice = NDS == 4 ? (w & 3) : w;
  const int dthalf = NDS == 4 ? (w >> 2) : 0;
  int qoff[DQT][2], koff[2];
#pragma unroll
  for (int t = 0; t < DQT; ++t) {
    const int tt = NDS == 4 ? dthalf : t;
    qoff[t][0] = ds_off(8 * g4l + qq, 4 * tt + pp);
    qoff[t][1] = ds_off(8 * g4l + 4 + qq, 4 * tt + pp);
  }
  {
    const int ch = 2 * dslice + (pp >> 1), sub = (pp & 1) * 4;
    koff[0] = swz<DP>(8 * g4l + qq, ch) + sub;
    koff[1] = swz<DP>(8 * g4l + 4 + qq, ch) + sub;
  }

  const int* se = p.seg_end ? p.seg_end + static_cast<int64_t>(b) * p.Tk : nullptr;
  int kse = 0x7fffffff, kse_lo = 0x7fffffff, kse_hi = 0x7fffffff;
  if (se) {
    kse = se[min(kw + l32, p.Tk - 1)];
    kse_lo = __builtin_amdgcn_readfirstlane(se[min(kw, p.Tk - 1)]);
    kse_hi = __builtin_amdgcn_readfirstlane(se[min(kw + 31, p.Tk - 1)]);
  }

  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    dk[dt] = f32x16{};
    dv[dt] = f32x16{};
  }

  // Row constants enter through the MFMA chains: one extra k-step per chain whose A fragment
  // holds this lane's query row's -lse2/scale2 (resp. -delta) split into bf16 hi + lo in k slots
  // 0, 1 (lanes h = 0; zero elsewhere) against a B fragment of ones in the same slots, so the
  // fp32 accumulators come out as S - lse2/scale2 and dP - delta. Per tile a wave loads 2
  // dwords per lane (its own query row) instead of the 16 + 16 accumulator-row constants
  // (8 dwordx4 loads per lane of data every lane holds 32-fold: the texture path, not the
  // bytes, cost ~900 cycles per tile) and spends no VALU on accumulator initialisation.
  float rlse = 0.f, rdel = 0.f;  // next tile's values for query row qt + l32
  auto load_rows = [&](int hq, int qt) {
    const int64_t rb = (static_cast<int64_t>(b) * p.Hq + hq) * p.Tq;
    const int r = min(qt + l32, p.Tq - 1);
    rlse = p.lse2[rb + r];
    rdel = p.delta[rb + r];
  };
  const s16x8 ones = __builtin_bit_cast(s16x8, u32x4{h ? 0u : 0x3F803F80u, 0u, 0u, 0u});
  const float inv_s2 = 1.f / p.scale2;

  int hq = hq0, qt = qt0;        // tile it
  int hq_r = hq0, qt_r = qt0;    // tile it + 1 (row constants)
  int hq_p = hq0, qt_p = qt0;    // tile it + 2 (Q / dO prefetch)
  if (n_iter > 0) {
    prefetch(hq_p, qt_p);
    stage();
    load_rows(hq_r, qt_r);
    advance(hq_p, qt_p);
    if (n_iter > 1) prefetch(hq_p, qt_p);
    advance(hq_p, qt_p);
  }
  __syncthreads();

  // static priority for the second-dispatched half (waves 4-7 share SIMDs with 0-3 and lose
  // every VALU arbitration by age otherwise; MI355X_MICROARCH "Two waves per SIMD" item 4)
  // (per-MFMA-cluster s_setprio flips on top measured as noise: the clusters are already pinned
  // by sched_barriers; removed)
  if (w >= 4) __builtin_amdgcn_s_setprio(1);
  for (int it = 0; it < n_iter; ++it) {
    advance(hq_r, qt_r);
    asm volatile("" : "+v"(rq), "+v"(rx), "+v"(tq0), "+v"(tx0), "+v"(tq1), "+v"(tx1), "+v"(wq), "+v"(wx));
    auto roff = [&](int s) { return rq + (((2 * s) ^ rx) << 3); };
    auto toff = [&](int dt, int r) { return r ? tq1 + (((4 * dt) ^ tx1) << 3) : tq0 + (((4 * dt) ^ tx0) << 3); };
    BWD_TS(0);

    bool act = kw < kend && kw + 32 > kbeg && qt < kse_hi;
    bool need_mask = kw < kbeg || kw + 32 > kend || qt + BQ > p.Tq || qt + BQ > kse_lo;
    if (CAUSAL) {
      act = act && kw <= qt + BQ - 1 + p.causal_off;
      need_mask = need_mask || (kw + 31 > qt + p.causal_off);
      if (p.window > 0) {
        act = act && (kw + 31 > qt + p.causal_off - p.window);
        need_mask = need_mask || (kw <= qt + BQ - 1 + p.causal_off - p.window);
      }
    }

    // ---------------------------------------------------------------- phase A
    s16x8 sb0 = s16x8{}, sb1 = s16x8{};
    if (act) {
      f32x16 sacc = f32x16{}, dpacc = f32x16{};
      const bf16_t* Kw = Ks + 32 * w * DP;
      const bf16_t* Vw = Vs + 32 * w * DP;
      // S chain, then dP chain: fragments one k-step ahead, the order pinned by sched_barriers
      // (left free, the scheduler hoists all KS steps' reads and spills; both chains at once
      // need twice the fragment registers)
      s16x8 fa[2], fb[2];
      auto chain = [&](const bf16_t* A, const bf16_t* Bm, f32x16& acc) {
        fa[0] = *reinterpret_cast<const s16x8*>(A + roff(0));
        fb[0] = *reinterpret_cast<const s16x8*>(Bm + roff(0));
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          if (s + 1 < KS) {
            fa[(s + 1) & 1] = *reinterpret_cast<const s16x8*>(A + roff(s + 1));
            fb[(s + 1) & 1] = *reinterpret_cast<const s16x8*>(Bm + roff(s + 1));
          }
          __builtin_amdgcn_sched_barrier(0);
          acc = mfma32(fa[s & 1], fb[s & 1], acc);
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      chain(Qs, Kw, sacc);
      chain(dOs, Vw, dpacc);
      {  // + the row-constant k-step (last: its loads get the whole chains as slack)
        const bool rv = qt + l32 < p.Tq;
        float x = -rlse * inv_s2;
        x = (rv && __builtin_isfinite(x)) ? x : -1e30f;  // rows past Tq / without keys: p = 0
        const float y = rv ? -rdel : 0.f;
        const float xh = bf2f(static_cast<bf16_t>(pack2bf(x, 0.f) & 0xffffu));
        const float yh = bf2f(static_cast<bf16_t>(pack2bf(y, 0.f) & 0xffffu));
        const s16x8 ax = __builtin_bit_cast(s16x8, u32x4{h ? 0u : pack2bf(x, x - xh), 0u, 0u, 0u});
        const s16x8 ay = __builtin_bit_cast(s16x8, u32x4{h ? 0u : pack2bf(y, y - yh), 0u, 0u, 0u});
        sacc = mfma32(ax, ones, sacc);
        dpacc = mfma32(ay, ones, dpacc);
      }
      BWD_TS(1);
      const int kj = kw + l32;
      int lo = 0, hi = min(p.Tq, kse) - qt - 4 * h;
      if (kj < kbeg || kj >= kend) hi = 0;
      if (CAUSAL) {
        const int dlt = kj - qt - p.causal_off - 4 * h;
        lo = max(lo, dlt);
        if (p.window > 0) hi = min(hi, dlt + p.window);
      }
      const unsigned span = hi > lo ? static_cast<unsigned>(hi - lo) : 0u;
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[i] = ex2(sacc[i] * p.scale2);
      // the mask as its own wave-uniform branch: fused into the exp loop, the compiler
      // if-converted it and every tile paid 16 compares + 16 selects + the bound arithmetic
      // (bwd +2-3 % causal, same box, bitwise: gpurun_out/r5/bwdms)
      if (need_mask) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int rr = (i & 3) + 8 * (i >> 2);
          sacc[i] = static_cast<unsigned>(rr - lo) < span ? sacc[i] : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) dpacc[i] = sacc[i] * dpacc[i];
      const s16x8 pb0 = pack8(sacc, 0), pb1 = pack8(sacc, 8);
      sb0 = pack8(dpacc, 0);
      sb1 = pack8(dpacc, 8);
      BWD_TS(2);
      // dV^T += dO^T P ; dK^T += Q^T dS (transposed fragments of column tile dt+1 read while
      // tile dt's four MFMAs run)
      s16x8 ta[2], tb[2], tc[2], td[2];
      auto ld_kv = [&](int dt, int sl) {
        const int o0 = toff(dt, 0), o1 = toff(dt, 1);
        ta[sl] = cat4(tr_read(dOs + o0), tr_read(dOs + o1));
        tb[sl] = cat4(tr_read(dOs + 16 * DP + o0), tr_read(dOs + 16 * DP + o1));
        tc[sl] = cat4(tr_read(Qs + o0), tr_read(Qs + o1));
        td[sl] = cat4(tr_read(Qs + 16 * DP + o0), tr_read(Qs + 16 * DP + o1));
      };
      ld_kv(0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        if (dt + 1 < DT) ld_kv(dt + 1, (dt + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
        // alternating accumulators: no MFMA waits on the one just issued
        dv[dt] = mfma32(ta[dt & 1], pb0, dv[dt]);
        dk[dt] = mfma32(tc[dt & 1], sb0, dk[dt]);
        dv[dt] = mfma32(tb[dt & 1], pb1, dv[dt]);
        dk[dt] = mfma32(td[dt & 1], sb1, dk[dt]);
        __builtin_amdgcn_sched_barrier(0);
      }
      BWD_TS(3);
    }
    {  // dS^T rows -> [key][32 queries] image (zero for an inactive sub-tile)
      const u32x4 ds0 = __builtin_bit_cast(u32x4, sb0), ds1 = __builtin_bit_cast(u32x4, sb1);
      bf16_t* dSw = dSs + 32 * w * 32;
      *reinterpret_cast<uint2*>(dSw + wq + ((0 ^ wx) << 2)) = make_uint2(ds0[0], ds0[1]);
      *reinterpret_cast<uint2*>(dSw + wq + ((2 ^ wx) << 2)) = make_uint2(ds0[2], ds0[3]);
      *reinterpret_cast<uint2*>(dSw + wq + ((4 ^ wx) << 2)) = make_uint2(ds1[0], ds1[1]);
      *reinterpret_cast<uint2*>(dSw + wq + ((6 ^ wx) << 2)) = make_uint2(ds1[2], ds1[3]);
    }
    BWD_TS(4);
    __syncthreads();
    BWD_TS(5);

    // ---------------------------------------------------------------- phase B
    if (it + 1 < n_iter) {
      stage();
      if (it + 2 < n_iter) prefetch(hq_p, qt_p);
      load_rows(hq_r, qt_r);
    }
    BWD_TS(6);
    if (w < NDS || NDS == 4) {
      f32x4 acc[DQT];
#pragma unroll
      for (int t = 0; t < DQT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      // fragments two k-steps ahead (phase B has the registers: the score accumulators are dead)
      constexpr int NB = 3, NKS = BKV / 32;
      s16x8 kf[NB], af[NB][DQT];
      auto ld_dq = [&](int ks, int sl) {
        kf[sl] = cat4(tr_read(Ks + 32 * ks * DP + koff[0]), tr_read(Ks + 32 * ks * DP + koff[1]));
#pragma unroll
        for (int t = 0; t < DQT; ++t)
          af[sl][t] = cat4(tr_read(dSs + 32 * ks * 32 + qoff[t][0]), tr_read(dSs + 32 * ks * 32 + qoff[t][1]));
      };
      ld_dq(0, 0);
      ld_dq(1, 1);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        if (ks + 2 < NKS) ld_dq(ks + 2, (ks + 2) % NB);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < DQT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks % NB][t], kf[ks % NB], acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      // lane holds d = 16*slice + i16 of query rows 16t + 4*g4l + e (64-B row segments)
      const int64_t rs = static_cast<int64_t>(p.Hq) * D;
      const int64_t sbase = ((static_cast<int64_t>(kb) * p.B + b) * p.slab_rows + qt) * rs +
                            static_cast<int64_t>(hq) * D + 16 * dslice;
      const uint32_t so = static_cast<uint32_t>(4 * g4l * rs + i16);
      if (p.dq_slab16 != nullptr) {  // bf16 partials (32-B row segments)
        bf16_t* sp = p.dq_slab16 + sbase;
#pragma unroll
        for (int t = 0; t < DQT; ++t) {
          const int tt = NDS == 4 ? dthalf : t;
#pragma unroll
          for (int e = 0; e < 4; ++e) sp[(16 * tt + e) * rs + so] = f2bf(acc[t][e] * p.scale);
        }
      } else {
        char* sp = reinterpret_cast<char*>(p.dq_slab + sbase);
#pragma unroll
        for (int t = 0; t < DQT; ++t) {
          const int tt = NDS == 4 ? dthalf : t;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            *reinterpret_cast<float*>(sp + ((16 * tt + e) * rs + so) * 4u) = acc[t][e] * p.scale;
        }
      }
    }
    BWD_TS(7);
    __syncthreads();
    advance(hq, qt);
    advance(hq_p, qt_p);
  }

  const int kj = kw + l32;
  if (kj >= p.Tk) return;
  if (p.hsplit == 1) {
    bf16_t* dkp = p.dk + b * p.dk_sb + kj * p.dk_st + static_cast<int64_t>(hk) * p.dk_sh;
    bf16_t* dvp = p.dv + b * p.dv_sb + kj * p.dv_st + static_cast<int64_t>(hk) * p.dv_sh;
    auto store_row = [&](bf16_t* dst, f32x16 x, float sc, int dt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; g4 += 2) {
        const uint32_t a0 = pack2bf(x[4 * g4] * sc, x[4 * g4 + 1] * sc);
        const uint32_t a1 = pack2bf(x[4 * g4 + 2] * sc, x[4 * g4 + 3] * sc);
        const uint32_t c0 = pack2bf(x[4 * g4 + 4] * sc, x[4 * g4 + 5] * sc);
        const uint32_t c1 = pack2bf(x[4 * g4 + 6] * sc, x[4 * g4 + 7] * sc);
        const auto r0 = __builtin_amdgcn_permlane32_swap(a0, c0, false, false);
        const auto r1 = __builtin_amdgcn_permlane32_swap(a1, c1, false, false);
        if (32 * dt + 8 * g4 + 8 * h < D)
          *reinterpret_cast<uint4*>(dst + 32 * dt + 8 * g4 + 8 * h) = make_uint4(r0[0], r1[0], r0[1], r1[1]);
      }
    };
    if (D == 80 && p.rope_cos != nullptr) {  // partial rotary (rot = 32): column tile 0 only
      const int pos = p.rope_pos ? p.rope_pos[static_cast<int64_t>(b) * p.Tk + kj] : kj;
      store_row(dkp, unrotate_tile0_rot32(dk[0], p.rope_cos + static_cast<int64_t>(pos) * 16 + 4 * h,
                                          p.rope_sin + static_cast<int64_t>(pos) * 16 + 4 * h),
                p.scale, 0);
#pragma unroll
      for (int dt = 1; dt < DT; ++dt) store_row(dkp, dk[dt], p.scale, dt);
    } else if (DP == D && p.rope_cos != nullptr) {
      const int pos = p.rope_pos ? p.rope_pos[static_cast<int64_t>(b) * p.Tk + kj] : kj;
      const float* cp = p.rope_cos + static_cast<int64_t>(pos) * (D / 2) + 4 * h;
      const float* sp = p.rope_sin + static_cast<int64_t>(pos) * (D / 2) + 4 * h;
#pragma unroll
      for (int dt = 0; dt < DT / 2; ++dt) {
        f32x16 lo = dk[dt], hi = dk[dt + DT / 2];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 c4 = *reinterpret_cast<const f32x4*>(cp + 32 * dt + 8 * g);
          const f32x4 s4 = *reinterpret_cast<const f32x4*>(sp + 32 * dt + 8 * g);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float a = lo[4 * g + e], bb = hi[4 * g + e];
            lo[4 * g + e] = a * c4[e] + bb * s4[e];
            hi[4 * g + e] = bb * c4[e] - a * s4[e];
          }
        }
        store_row(dkp, lo, p.scale, dt);
        store_row(dkp, hi, p.scale, dt + DT / 2);
      }
    } else {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) store_row(dkp, dk[dt], p.scale, dt);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) store_row(dvp, dv[dt], 1.f, dt);
  } else if (p.dk_part16 != nullptr) {  // bf16 partials: each rounded once, summed in fp32
    const int64_t off = ((static_cast<int64_t>(sidx) * p.B + b) * p.Tk + kj) * p.Hkv * D +
                        static_cast<int64_t>(hk) * D;
    bf16_t* dkp = p.dk_part16 + off;
    bf16_t* dvp = p.dv_part16 + off;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * dt + 8 * g4 + 4 * h;
        if (d >= D) continue;
        *reinterpret_cast<uint2*>(dkp + d) = make_uint2(pack2bf(dk[dt][4 * g4], dk[dt][4 * g4 + 1]),
                                                        pack2bf(dk[dt][4 * g4 + 2], dk[dt][4 * g4 + 3]));
        *reinterpret_cast<uint2*>(dvp + d) = make_uint2(pack2bf(dv[dt][4 * g4], dv[dt][4 * g4 + 1]),
                                                        pack2bf(dv[dt][4 * g4 + 2], dv[dt][4 * g4 + 3]));
      }
    }
  } else {
    const int64_t off = ((static_cast<int64_t>(sidx) * p.B + b) * p.Tk + kj) * p.Hkv * D +
                        static_cast<int64_t>(hk) * D;
    float* dkp = p.dk_part + off;
    float* dvp = p.dv_part + off;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * dt + 8 * g4 + 4 * h;
        if (d >= D) continue;
        *reinterpret_cast<f32x4*>(dkp + d) = f32x4{dk[dt][4 * g4], dk[dt][4 * g4 + 1], dk[dt][4 * g4 + 2], dk[dt][4 * g4 + 3]};
        *reinterpret_cast<f32x4*>(dvp + d) = f32x4{dv[dt][4 * g4], dv[dt][4 * g4 + 1], dv[dt][4 * g4 + 2], dv[dt][4 * g4 + 3]};
      }
    }
  }
}

// Sum of the 8-column chunk at `src` over key blocks [lo, hi) of the slab (fixed kb order, 4
// blocks' loads in flight at a time: bitwise the same as one at a time).
__device__ __forceinline__ void slab_sum8(const float* src, int64_t slab_stride, int lo, int hi,
                                          f32x4& a0, f32x4& a1) {
  a0 = f32x4{0.f, 0.f, 0.f, 0.f};
  a1 = a0;
  int kb = lo;
  for (; kb + 4 <= hi; kb += 4) {
    f32x4 x[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4* sv = reinterpret_cast<const f32x4*>(src + (kb + u) * slab_stride);
      x[u][0] = __builtin_nontemporal_load(sv);
      x[u][1] = __builtin_nontemporal_load(sv + 1);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a0 += x[u][0];
      a1 += x[u][1];
    }
  }
  for (; kb < hi; ++kb) {
    const f32x4* sv = reinterpret_cast<const f32x4*>(src + kb * slab_stride);
    a0 += __builtin_nontemporal_load(sv);
    a1 += __builtin_nontemporal_load(sv + 1);
  }
}

// bf16 slabs: the same sum over the key blocks (fp32 accumulation in kb order)
__device__ __forceinline__ void slab_sum8(const bf16_t* src, int64_t slab_stride, int lo, int hi,
                                          f32x4& a0, f32x4& a1) {
  a0 = f32x4{0.f, 0.f, 0.f, 0.f};
  a1 = a0;
  int kb = lo;
  for (; kb + 4 <= hi; kb += 4) {
    bf16x8 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      x[u] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(src + (kb + u) * slab_stride));
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a0 += f32x4{bf2f(x[u][0]), bf2f(x[u][1]), bf2f(x[u][2]), bf2f(x[u][3])};
      a1 += f32x4{bf2f(x[u][4]), bf2f(x[u][5]), bf2f(x[u][6]), bf2f(x[u][7])};
    }
  }
  for (; kb < hi; ++kb) {
    const bf16x8 x = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(src + kb * slab_stride));
    a0 += f32x4{bf2f(x[0]), bf2f(x[1]), bf2f(x[2]), bf2f(x[3])};
    a1 += f32x4{bf2f(x[4]), bf2f(x[5]), bf2f(x[6]), bf2f(x[7])};
  }
}

// un-rotate one pair of 8-column chunks (d and d + D/2) with the position's cos/sin
__device__ __forceinline__ void rope_unrotate8(const float* cp, const float* sp, float (&lo)[8],
                                               float (&hi)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float c = cp[j], s = sp[j], a = lo[j], b = hi[j];
    lo[j] = a * c + b * s;
    hi[j] = b * c - a * s;
  }
}

// dQ[b, t, h, :] = sum over the key blocks whose workgroups swept row t (fixed kb order)
// -> bf16 into a strided destination. One thread per 8 columns, or with the fused RoPE backward
// (rcos != null) per pair of 8-column chunks d, d + D/2.
template <bool CAUSAL, typename ST = float>
__global__ __launch_bounds__(256) void attn_dq_reduce_kernel(
    const ST* __restrict__ slab, int nkb, int B, int Tq, int slab_rows, int Hq, int D,
    int causal_off, int window, const int* __restrict__ kv_start, const int* __restrict__ kv_end,
    int Tk, bf16_t* __restrict__ dst, int64_t d_sb, int64_t d_st, int64_t d_sh,
    const float* __restrict__ rcos, const float* __restrict__ rsin, const int* __restrict__ rpos,
    int rot) {
  // work items per row: without RoPE one per 8 columns; with it one per rotary chunk pair
  // (c, c + rot/16) plus one per 8 columns past the rotary dims (partial rotary, D = 80)
  const int hv = rot / 16;
  const int cv = rcos ? hv + (D - rot) / 8 : D / 8;
  const int64_t total = static_cast<int64_t>(B) * Tq * Hq * cv;
  const int64_t rs = static_cast<int64_t>(Hq) * D;
  const int64_t slab_stride = static_cast<int64_t>(B) * slab_rows * rs;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int c = static_cast<int>(i % cv);
    int64_t r = i / cv;
    const int hq = static_cast<int>(r % Hq);
    r /= Hq;
    const int t = static_cast<int>(r % Tq);
    const int b = static_cast<int>(r / Tq);
    const int kbeg = kv_start ? kv_start[b] : 0;
    const int kend = kv_end ? kv_end[b] : Tk;
    const bool pair = rcos && c < hv;
    const int col = (rcos && !pair) ? rot + (c - hv) * 8 : c * 8;
    const ST* src = slab + (static_cast<int64_t>(b) * slab_rows + t) * rs + static_cast<int64_t>(hq) * D + col;
    // the key blocks that wrote row t form one contiguous range [lo, hi) (kv range: an
    // interval; causal: a prefix; window: a suffix): find it with ALU only, then sum the slabs
    // in kb order with 4 blocks' loads in flight at a time (same order as one at a time: the
    // sum is bitwise unchanged)
    int lo = nkb, hi = 0;
    for (int kb = 0; kb < nkb; ++kb) {
      const int k0 = kb * kAttnBwdKeys;
      int qt0, qend;
      bwd_q_range<CAUSAL>(k0, Tq, causal_off, window, qt0, qend);
      if (k0 >= kend || k0 + kAttnBwdKeys <= kbeg || t < qt0 || t >= qend) continue;
      lo = min(lo, kb);
      hi = kb + 1;
    }
    f32x4 a0, a1;
    slab_sum8(src, slab_stride, lo, hi, a0, a1);
    float v[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    bf16_t* out = dst + b * d_sb + t * d_st + hq * d_sh + col;
    if (pair) {
      f32x4 b0, b1;
      slab_sum8(src + hv * 8, slab_stride, lo, hi, b0, b1);
      float w[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      const int pos = rpos ? rpos[static_cast<int64_t>(b) * Tq + t] : t;
      rope_unrotate8(rcos + static_cast<int64_t>(pos) * (rot / 2) + c * 8,
                     rsin + static_cast<int64_t>(pos) * (rot / 2) + c * 8, v, w);
      store_bf16x8(out + hv * 8, pack_bf16x8(w));
    }
    store_bf16x8(out, pack_bf16x8(v));
  }
}

// dK = scale * sum_s dk_part[s], dV = sum_s dv_part[s] -> bf16 strided (head-split workgroups).
// With the fused RoPE backward (rcos != null) a work item is the chunk pair d, d + D/2.
__device__ __forceinline__ void part_sum8(const float* p, int64_t pstride, int hs, f32x4& a0, f32x4& a1) {
  a0 = f32x4{0.f, 0.f, 0.f, 0.f};
  a1 = a0;
  for (int s = 0; s < hs; ++s) {
    const f32x4* v = reinterpret_cast<const f32x4*>(p + s * pstride);
    a0 += v[0];
    a1 += v[1];
  }
}

__device__ __forceinline__ void part_sum8(const bf16_t* p, int64_t pstride, int hs, f32x4& a0, f32x4& a1) {
  a0 = f32x4{0.f, 0.f, 0.f, 0.f};
  a1 = a0;
  for (int s = 0; s < hs; ++s) {
    const bf16x8 x = load_bf16x8(p + s * pstride);
    a0 += f32x4{bf2f(x[0]), bf2f(x[1]), bf2f(x[2]), bf2f(x[3])};
    a1 += f32x4{bf2f(x[4]), bf2f(x[5]), bf2f(x[6]), bf2f(x[7])};
  }
}

template <typename PT>
__global__ __launch_bounds__(256) void attn_dkv_reduce_kernel(
    const PT* __restrict__ dkp, const PT* __restrict__ dvp, int hs, int B, int Tk, int Hkv,
    int D, float scale, bf16_t* __restrict__ dk, int64_t dk_sb, int64_t dk_st, int64_t dk_sh,
    bf16_t* __restrict__ dv, int64_t dv_sb, int64_t dv_st, int64_t dv_sh,
    const float* __restrict__ rcos, const float* __restrict__ rsin, const int* __restrict__ rpos,
    int rot) {
  const int hv = rot / 16;  // work items as attn_dq_reduce_kernel
  const int cv = rcos ? hv + (D - rot) / 8 : D / 8;
  const int64_t total = static_cast<int64_t>(B) * Tk * Hkv * cv;
  const int64_t pstride = static_cast<int64_t>(B) * Tk * Hkv * D;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int c = static_cast<int>(i % cv);
    int64_t r = i / cv;
    const int hk = static_cast<int>(r % Hkv);
    r /= Hkv;
    const int t = static_cast<int>(r % Tk);
    const int b = static_cast<int>(r / Tk);
    const bool pair = rcos && c < hv;
    const int col = (rcos && !pair) ? rot + (c - hv) * 8 : c * 8;
    const int64_t off = ((static_cast<int64_t>(b) * Tk + t) * Hkv + hk) * D + col;
    f32x4 k0, k1, v0, v1;
    part_sum8(dkp + off, pstride, hs, k0, k1);
    part_sum8(dvp + off, pstride, hs, v0, v1);
    float kf[8] = {k0[0] * scale, k0[1] * scale, k0[2] * scale, k0[3] * scale,
                   k1[0] * scale, k1[1] * scale, k1[2] * scale, k1[3] * scale};
    const float vf[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    bf16_t* kout = dk + b * dk_sb + t * dk_st + hk * dk_sh + col;
    bf16_t* vout = dv + b * dv_sb + t * dv_st + hk * dv_sh + col;
    if (pair) {  // partner chunk c + rot/16: dV copied through, dK un-rotated with its pair
      part_sum8(dkp + off + hv * 8, pstride, hs, k0, k1);
      part_sum8(dvp + off + hv * 8, pstride, hs, v0, v1);
      float kw[8] = {k0[0] * scale, k0[1] * scale, k0[2] * scale, k0[3] * scale,
                     k1[0] * scale, k1[1] * scale, k1[2] * scale, k1[3] * scale};
      const float vw[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      const int pos = rpos ? rpos[static_cast<int64_t>(b) * Tk + t] : t;
      rope_unrotate8(rcos + static_cast<int64_t>(pos) * (rot / 2) + c * 8,
                     rsin + static_cast<int64_t>(pos) * (rot / 2) + c * 8, kf, kw);
      store_bf16x8(kout + hv * 8, pack_bf16x8(kw));
      store_bf16x8(vout + hv * 8, pack_bf16x8(vw));
    }
    store_bf16x8(kout, pack_bf16x8(kf));
    store_bf16x8(vout, pack_bf16x8(vf));
  }
}

// ----------------------------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------------------------
static inline unsigned stream_grid(int64_t work) {
  // grid-stride cap of the reduce passes: 1024 / 8192 / 32768 measured as noise against 2048
  constexpr int64_t cap = 2048;
  int64_t g = (work + 255) / 256;
  if (g > cap) g = cap;
  return static_cast<unsigned>(g < 1 ? 1 : g);
}

// Forward: 8 waves (256 queries) per workgroup. A 4-wave / 128-query variant (two independent
// workgroups per CU, unaligned barriers) measured 31-35 % slower at T = 1024 and 4096.
// HP GQA heads per workgroup: 4 (64-query blocks, 2 waves per head) when the group size allows
// it, else 2, else 1; DLA_ATTN_FWD_HP=1|2|4 caps it for A/B runs. Same-box A/B (B8 T1024 Hq32
// Hkv8 D128, tools/gpu_attn_env_ab.sh): causal 140-148 / 131-133 / 124-129 us for HP 1 / 2 / 4,
// non-causal 217 -> 205-209 us, T = 4096 unchanged (366-379 us).
// Persistent forward (attn_fwd_persist_kernel): DLA_ATTN_FWD_PERSIST=1 always, =0 never, unset =
// for key ranges of at most 512 (<= 8 tiles per block), where it measured faster: graph-timed,
// B*T = 8192, Hq 32 / Hkv 8 / D 128 (profiles/r5_attention_fwd.md) causal 240 -> 290-318 TF/s
// at T 256 and 413 -> 469-472 at T 512, equal at 1024, 5 % slower at 2048-4096. Read per call so
// one process can A/B both (tools/attn_fwd_sweep.py --cfg, tests/test_kernels_gpu.py).
static bool fwd_persist(int Tk) {
  const char* e = std::getenv("DLA_ATTN_FWD_PERSIST");
  if (e == nullptr || *e == '\0') return Tk <= 512;
  return std::atoi(e) != 0;
}

static int device_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

struct AttnFwdSwitches {
  int prio, sgpr, pro, ostage, msub;
};

// Read from the environment once per process; tests flip a switch through attn_fwd_set_switch
// (torch.ops.dla.attn_fwd_switch) instead of re-reading the environment on every launch.
static AttnFwdSwitches& attn_fwd_switches() {
  static AttnFwdSwitches sw = [] {
    auto env = [](const char* name, int dflt) {
      const char* e = std::getenv(name);
      return e ? std::atoi(e) : dflt;
    };
    return AttnFwdSwitches{env("DLA_ATTN_FWD_PRIO", 1), env("DLA_ATTN_FWD_SGPR", 1), env("DLA_ATTN_FWD_PRO", 1),
                           env("DLA_ATTN_FWD_OSTAGE", 1), env("DLA_ATTN_FWD_MSUB", 1)};
  }();
  return sw;
}

// Set one switch ("prio", "sgpr", "pro", "ostage", "msub"); returns its previous value, or
// -1 for an unknown name (nothing changed).
int attn_fwd_set_switch(const char* name, int value) {
  AttnFwdSwitches& sw = attn_fwd_switches();
  int* f = nullptr;
  if (!std::strcmp(name, "prio")) f = &sw.prio;
  else if (!std::strcmp(name, "sgpr")) f = &sw.sgpr;
  else if (!std::strcmp(name, "pro")) f = &sw.pro;
  else if (!std::strcmp(name, "ostage")) f = &sw.ostage;
  else if (!std::strcmp(name, "msub")) f = &sw.msub;
  if (f == nullptr) return -1;
  const int prev = *f;
  *f = value;
  return prev;
}

template <int D, int HP>
static void fwd_launch(const AttnParams& p0, bool causal, hipStream_t st) {
  constexpr int NW = 8, BQ = 32 * NW / HP;
  AttnParams p = p0;
  {
    // The forward's structure switches, read ONCE per process (attn_fwd_switches; every switch
    // defaults to its measured winner, the others exist for same-binary A/B runs):
    //   prio 1: s_setprio 1 around each MFMA chain, so the matrix chain of one wave issues ahead
    //     of its SIMD partner's softmax VALU (cdna guide T5). Same box, graph-timed, B*T 8192:
    //     causal T1024 654 vs 613 TF/s, T4096 937 vs 897; non-causal +4-6 %. 2 (static priority
    //     for waves 4-7) measured +0-7 % and below 1 everywhere; 0 = off.
    //   msub (D = 128): same box, graph-timed, interleaved: causal T1024 701 vs 668 TF/s, T2048
    //     898 vs 865, non-causal +3-7 % (gpurun_out/r5/attn13); outputs within one bf16 ulp
    const AttnFwdSwitches& sw = attn_fwd_switches();
    p.fwd_prio = sw.prio;
    p.fwd_sgpr = sw.sgpr;
    p.fwd_pro = sw.pro;
    p.fwd_ostage = sw.ostage;
    p.fwd_msub = sw.msub;
  }
  const int nqb = (p.Tq + BQ - 1) / BQ;
  const int64_t nblk = static_cast<int64_t>(nqb) * (p.Hq / HP) * p.B;
  if (fwd_persist(p.Tk) && nblk < (int64_t(1) << 30)) {
    // one 8-wave workgroup per CU (230 VGPRs: two waves per SIMD), never more than the blocks
    const int grid = static_cast<int>(std::min<int64_t>(nblk, device_cus()));
    if (causal) attn_fwd_persist_kernel<D, true, NW, HP><<<grid, 64 * NW, 0, st>>>(p, static_cast<int>(nblk));
    else attn_fwd_persist_kernel<D, false, NW, HP><<<grid, 64 * NW, 0, st>>>(p, static_cast<int>(nblk));
    return;
  }
  const dim3 grid(static_cast<unsigned>(nblk));
  if constexpr (D == 128) {
    if (p.fwd_msub) {
      if (causal) attn_fwd_kernel<D, true, NW, HP, true><<<grid, 64 * NW, 0, st>>>(p);
      else attn_fwd_kernel<D, false, NW, HP, true><<<grid, 64 * NW, 0, st>>>(p);
      return;
    }
  }
  if (causal) attn_fwd_kernel<D, true, NW, HP><<<grid, 64 * NW, 0, st>>>(p);
  else attn_fwd_kernel<D, false, NW, HP><<<grid, 64 * NW, 0, st>>>(p);
}

template <int D>
static void fwd_dispatch(const AttnParams& p, bool causal, hipStream_t st) {
  static const int forced = [] {
    const char* e = std::getenv("DLA_ATTN_FWD_HP");
    return e ? std::atoi(e) : 0;
  }();
  const int group = p.Hq / p.Hkv;
  const int want = forced > 0 ? forced : 4;
  if (want >= 4 && group % 4 == 0) fwd_launch<D, 4>(p, causal, st);
  else if (want >= 2 && group % 2 == 0) fwd_launch<D, 2>(p, causal, st);
  else fwd_launch<D, 1>(p, causal, st);
}

void launch_attn_fwd(const AttnParams& p, int D, bool causal, hipStream_t st) {
  if (p.B == 0 || p.Tq == 0) return;
  switch (D) {
    case 64: fwd_dispatch<64>(p, causal, st); break;
    case 80: fwd_dispatch<80>(p, causal, st); break;
    case 128: fwd_dispatch<128>(p, causal, st); break;
    default: throw std::invalid_argument("attn_fwd: head_dim must be 64, 80 or 128");
  }
}

void launch_attn_bwd_delta(const bf16_t* o, const bf16_t* dout, int64_t o_sb, int64_t o_st,
                           int64_t o_sh, int64_t do_sb, int64_t do_st, int64_t do_sh, int B,
                           int H, int T, int D, float* delta, hipStream_t st) {
  const int64_t rows = static_cast<int64_t>(B) * H * T;
  if (rows == 0) return;
  const int64_t rows_per_block = 4 * (64 / (D <= 64 ? 8 : 16));  // as attn_bwd_delta_kernel
  const unsigned nb = static_cast<unsigned>((rows + rows_per_block - 1) / rows_per_block);
  attn_bwd_delta_kernel<<<nb, 256, 0, st>>>(o, dout, o_sb, o_st, o_sh, do_sb, do_st, do_sh, B, H, T, D, delta);
}

// Backward main kernel: attn_bwd8_kernel (8 waves, default) or attn_bwd_kernel
// (DLA_ATTN_BWD_WAVES=4). Same-box A/B, B8 T1024 Hq32 Hkv8 D128 causal, all backward passes:
// 489 -> 410 us; non-causal 624 -> 549 us (profiles/r3_attention_bwd.md). Read per call (not
// cached) so one process can A/B both.
static int attn_bwd_waves() {
  const char* e = std::getenv("DLA_ATTN_BWD_WAVES");
  return (e && std::atoi(e) == 4) ? 4 : 8;
}

// bf16 dQ slabs (8-wave kernel; DLA_ATTN_DQ_BF16=0 keeps fp32). Read per call, like the wave count.
bool attn_dq_slab_bf16() {
  const char* e = std::getenv("DLA_ATTN_DQ_BF16");
  return attn_bwd_waves() == 8 && !(e && std::atoi(e) == 0);
}

// bf16 dK / dV head-split partials (8-wave kernel; DLA_ATTN_DKV_BF16=0 keeps fp32), read per call
bool attn_dkv_part_bf16() {
  const char* e = std::getenv("DLA_ATTN_DKV_BF16");
  return attn_bwd_waves() == 8 && !(e && std::atoi(e) == 0);
}

template <int D>
static void bwd_dispatch(const AttnBwdParams& p_in, bool causal, hipStream_t st) {
  const AttnBwdParams& p = p_in;
  const int nkb = (p.Tk + kAttnBwdKeys - 1) / kAttnBwdKeys;
  const dim3 grid(nkb * p.Hkv * p.B * p.hsplit);
  if (attn_bwd_waves() == 8) {
    if (causal) attn_bwd8_kernel<D, true><<<grid, 512, 0, st>>>(p);
    else attn_bwd8_kernel<D, false><<<grid, 512, 0, st>>>(p);
    return;
  }
  if (causal) attn_bwd_kernel<D, true><<<grid, 256, 0, st>>>(p);
  else attn_bwd_kernel<D, false><<<grid, 256, 0, st>>>(p);
}

void launch_attn_bwd(const AttnBwdParams& p, int D, bool causal, hipStream_t st) {
  if (p.B == 0 || p.Tq == 0 || p.Tk == 0) return;
  switch (D) {
    case 64: bwd_dispatch<64>(p, causal, st); break;
    case 80: bwd_dispatch<80>(p, causal, st); break;
    case 128: bwd_dispatch<128>(p, causal, st); break;
    default: throw std::invalid_argument("attn_bwd: head_dim must be 64, 80 or 128");
  }
}

void launch_attn_dq_reduce(const float* slab, int nkb, int B, int Tq, int slab_rows, int Hq, int D,
                           bool causal, int causal_off, int window, const int* kv_start,
                           const int* kv_end, int Tk, bf16_t* dst, int64_t d_sb, int64_t d_st,
                           int64_t d_sh, const float* rcos, const float* rsin, const int* rpos,
                           int rot, hipStream_t st, const bf16_t* slab16) {
  const int64_t work = static_cast<int64_t>(B) * Tq * Hq * (rcos ? rot / 16 + (D - rot) / 8 : D / 8);
  if (work == 0) return;
  if (slab16 != nullptr) {
    if (causal)
      attn_dq_reduce_kernel<true, bf16_t><<<stream_grid(work), 256, 0, st>>>(
          slab16, nkb, B, Tq, slab_rows, Hq, D, causal_off, window, kv_start, kv_end, Tk, dst, d_sb, d_st, d_sh,
          rcos, rsin, rpos, rot);
    else
      attn_dq_reduce_kernel<false, bf16_t><<<stream_grid(work), 256, 0, st>>>(
          slab16, nkb, B, Tq, slab_rows, Hq, D, causal_off, window, kv_start, kv_end, Tk, dst, d_sb, d_st, d_sh,
          rcos, rsin, rpos, rot);
    return;
  }
  if (causal)
    attn_dq_reduce_kernel<true><<<stream_grid(work), 256, 0, st>>>(
        slab, nkb, B, Tq, slab_rows, Hq, D, causal_off, window, kv_start, kv_end, Tk, dst, d_sb, d_st, d_sh,
        rcos, rsin, rpos, rot);
  else
    attn_dq_reduce_kernel<false><<<stream_grid(work), 256, 0, st>>>(
        slab, nkb, B, Tq, slab_rows, Hq, D, causal_off, window, kv_start, kv_end, Tk, dst, d_sb, d_st, d_sh,
        rcos, rsin, rpos, rot);
}

void launch_attn_dkv_reduce(const float* dkp, const float* dvp, int hs, int B, int Tk, int Hkv,
                            int D, float scale, bf16_t* dk, int64_t dk_sb, int64_t dk_st,
                            int64_t dk_sh, bf16_t* dv, int64_t dv_sb, int64_t dv_st,
                            int64_t dv_sh, const float* rcos, const float* rsin, const int* rpos,
                            int rot, hipStream_t st, const bf16_t* dkp16, const bf16_t* dvp16) {
  const int64_t work = static_cast<int64_t>(B) * Tk * Hkv * (rcos ? rot / 16 + (D - rot) / 8 : D / 8);
  if (work == 0) return;
  if (dkp16 != nullptr) {
    attn_dkv_reduce_kernel<bf16_t><<<stream_grid(work), 256, 0, st>>>(
        dkp16, dvp16, hs, B, Tk, Hkv, D, scale, dk, dk_sb, dk_st, dk_sh, dv, dv_sb, dv_st, dv_sh, rcos, rsin,
        rpos, rot);
    return;
  }
  attn_dkv_reduce_kernel<float><<<stream_grid(work), 256, 0, st>>>(dkp, dvp, hs, B, Tk, Hkv, D, scale, dk,
                                                                   dk_sb, dk_st, dk_sh, dv, dv_sb, dv_st,
                                                                   dv_sh, rcos, rsin, rpos, rot);
}

}  // namespace dla
