// Flash attention forward + backward for gfx950, MFMA 32x32x16 bf16.
//
// Replaces the HF SDPA path used by every policy/ref/reward forward of the reference
// (src/training/train_dpo.py:31-39 -> HF attention): causal, GQA, optional
// sliding window, per-batch key ranges [kv_start, kv_end) for left/right padding, head_dim
// 64 / 128. Scores never touch HBM; the forward stores only O and a per-row log2-domain
// LSE, the backward recomputes P from it (FA2 scheme).
//
// Forward structure (block = 4 waves = 128 queries of one (batch, q-head); KV tile = 64 keys):
//   * "swapped" scores S^T = K Q^T: the query sits on the MFMA column (lane), keys on the
//     16 accumulator registers, so each lane owns whole score columns -> the row max / sum is
//     in-register + one xor-32 shuffle, and the alpha rescale of O^T is a per-lane scalar.
//   * Q lives in registers for the whole kernel (B operand, 8 x 16 B per lane at D=128).
//   * P^T feeds the PV MFMA straight from the accumulator (cdna guide §3 "accumulator tile as
//     the next MFMA's operand"); V^T fragments come from ds_read_b64_tr_b16 transposed LDS reads.
//   * K/V tiles are register-staged (global loads for tile t+1 issued before computing tile t,
//     LDS write after the barrier: async-STAGE split), XOR-swizzled LDS image usable both for
//     row (ds_read_b128) and transposed reads.
// Backward structure (block = 4 waves = 128 keys of one (batch, kv-head); wave owns 32 keys):
//   * loops over every q head of the GQA group x 32-query tiles; dK^T/dV^T for the wave's keys
//     stay in accumulators for the whole sweep -> no cross-block reduction for dK/dV.
//   * "key on the lane": S and dP are computed with keys on the lane, so P and dS are already
//     the B operands of dV^T += dO^T P and dK^T += Q^T dS.
//   * dS crosses LDS once (as a [key][query] image) for dQ += dS K, summed over the block's
//     128 keys by MFMA, then added to an fp32 dQ accumulator with 128-B-segment atomics.
#include "common.h"
#include "attn_params.h"

namespace dla {

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// Element offset of 16-byte chunk `ch` of row `row` in a [rows][D] bf16 LDS image. The XOR
// keeps both ds_read_b128 row reads and ds_read_b64_tr_b16 column reads spread over banks
// (cdna guide T10 "one image for row reads AND transposed reads", layout (b)).
template <int D>
__device__ __forceinline__ int swz(int row, int ch) {
  constexpr int NCH = D / 8;
  static_assert((NCH & (NCH - 1)) == 0, "power-of-two chunks per row");
  const int f = (((row & 3) << 2) | ((row >> 2) & 3)) & (NCH - 1);
  return row * D + ((ch ^ f) << 3);
}

// dS^T image [128 keys][32 queries] bf16 (64-B rows): 8-byte unit c4 of row `row`, XOR-swizzled
// with row bits 2..4 so the 32 key rows written by a half-wave land on 32 distinct bank pairs
// (unswizzled: 16-bank row stride -> 8-way conflicts; the swizzle is a per-row permutation, so
// the ds_read_b64_tr_b16 reads of the dQ MFMA stay conflict-free).
__device__ __forceinline__ int ds_off(int row, int c4) { return row * 32 + ((c4 ^ ((row >> 2) & 7)) << 2); }

__device__ __forceinline__ s16x4 tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}

__device__ __forceinline__ s16x8 cat4(s16x4 a, s16x4 b) {
  return s16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

__device__ __forceinline__ s16x8 pack8(const f32x16& x, int base) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 r = {pack2bf(x[base], x[base + 1]), pack2bf(x[base + 2], x[base + 3]),
             pack2bf(x[base + 4], x[base + 5]), pack2bf(x[base + 6], x[base + 7])};
  return __builtin_bit_cast(s16x8, r);
}

__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

// Deferred-max threshold (cdna guide T13, log2 units): the running max is only raised when a
// tile's max exceeds it by more than this, so most tiles skip the O rescale. P <= 2^8.
constexpr float kRescaleThr = 8.0f;

__device__ __forceinline__ f32x16 mfma32(s16x8 a, s16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
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

// ==============================================================================================
// forward
// ==============================================================================================
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AttnParams p) {
  constexpr int BQ = 128, BK = 64;
  constexpr int NCH = D / 8;
  constexpr int KS = D / 16;
  constexpr int DT = D / 32;
  constexpr int CPT = BK * NCH / 256;  // 16-B chunks per thread per K (or V) tile
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * BK * D];
  bf16_t* Ks = smem;
  bf16_t* Vs = smem + BK * D;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int nqb = (p.Tq + BQ - 1) / BQ;
  const int bid = blockIdx.x;
  const int qb = CAUSAL ? nqb - 1 - (bid % nqb) : bid % nqb;  // heaviest causal blocks first
  const int rest = bid / nqb;
  const int hq = rest % p.Hq, b = rest / p.Hq;
  const int hk = hq / (p.Hq / p.Hkv);
  const int q0 = qb * BQ + w * 32;
  const int qi = q0 + l32;

  const bf16_t* qp = p.q + b * p.q_sb + static_cast<int64_t>(hq) * p.q_sh;
  const bf16_t* kp = p.k + b * p.k_sb + static_cast<int64_t>(hk) * p.k_sh;
  const bf16_t* vp = p.v + b * p.v_sb + static_cast<int64_t>(hk) * p.v_sh;

  // Q fragments stay in registers, pre-scaled by softmax_scale*log2(e) so the scores come
  // out of the MFMA already in the exp2 domain (no per-score multiply).
  s16x8 qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (qi < p.Tq) {
      const bf16x8 raw = load_bf16x8(qp + qi * p.q_st + 16 * s + 8 * h);
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = bf2f(raw[j]) * p.scale2;
      qf[s] = __builtin_bit_cast(s16x8, pack_bf16x8(t));
    } else {
      qf[s] = s16x8{};
    }
  }

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
  const int tile0 = (max(kmin, 0) / BK) * BK;

  bf16x8 kreg[CPT], vreg[CPT];
  auto gload = [&](int kt) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int ci = tid + 256 * c;
      const int row = ci / NCH, ch = ci % NCH;
      const int key = kt + row;
      if (key < p.Tk) {
        kreg[c] = load_bf16x8(kp + key * p.k_st + ch * 8);
        vreg[c] = load_bf16x8(vp + key * p.v_st + ch * 8);
      } else {
        kreg[c] = bf16x8{};
        vreg[c] = bf16x8{};
      }
    }
  };
  auto lwrite = [&]() {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int ci = tid + 256 * c;
      const int row = ci / NCH, ch = ci % NCH;
      store_bf16x8(Ks + swz<D>(row, ch), kreg[c]);
      store_bf16x8(Vs + swz<D>(row, ch), vreg[c]);
    }
  };

  if (tile0 < kmax) gload(tile0);
  for (int kt = tile0; kt < kmax; kt += BK) {
    __syncthreads();
    lwrite();
    __syncthreads();
    if (kt + BK < kmax) gload(kt + BK);

    bool active = q0 < p.Tq;
    if (CAUSAL) {
      active = active && (kt <= q0 + 31 + p.causal_off);
      if (p.window > 0) active = active && (kt + BK - 1 > q0 + p.causal_off - p.window);
    }
    if (!active) continue;  // wave-uniform

    f32x16 sacc[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      sacc[st] = f32x16{};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const s16x8 a = *reinterpret_cast<const s16x8*>(Ks + swz<D>(32 * st + l32, 2 * s + h));
        sacc[st] = mfma32(a, qf[s], sacc[st]);
      }
    }
    // mask only tiles that touch a boundary (kv range, causal diagonal, window edge)
    bool need_mask = kt < kbeg || kt + BK > kend;
    if (CAUSAL) {
      need_mask = need_mask || (kt + BK - 1 > q0 + p.causal_off);
      if (p.window > 0) need_mask = need_mask || (kt <= q0 + 31 + p.causal_off - p.window);
    }
    if (need_mask) {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kt + 32 * st + (i & 3) + 8 * (i >> 2) + 4 * h;
          bool ok = key >= kbeg && key < kend;
          if (CAUSAL) {
            ok = ok && key <= qi + p.causal_off;
            if (p.window > 0) ok = ok && key > qi + p.causal_off - p.window;
          }
          sacc[st][i] = ok ? sacc[st][i] : -INFINITY;
        }
      }
    }
    float mloc = -INFINITY;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int i = 0; i < 16; ++i) mloc = fmaxf(mloc, sacc[st][i]);
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    // deferred max: rescale O only when some row's max grew by more than kRescaleThr
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
        lsum += pv;
      }
    }
    s16x8 pf[2][2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      pf[st][0] = pack8(sacc[st], 0);
      pf[st][1] = pack8(sacc[st], 8);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int c0 = 32 * dt + 16 * ((lane >> 4) & 1);
#pragma unroll
      for (int st = 0; st < 2; ++st) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const s16x8 a = tr_frag_perm<D>(Vs, 32 * st + 16 * s + 4 * h, c0, lane);
          o[dt] = mfma32(a, pf[st][s], o[dt]);
        }
      }
    }
  }

  lsum += __shfl_xor(lsum, 32, 64);
  if (qi < p.Tq) {
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16_t* op = p.o + b * p.o_sb + qi * p.o_st + static_cast<int64_t>(hq) * p.o_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * dt + 8 * g4 + 4 * h;
        uint2 pk;
        pk.x = pack2bf(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv);
        pk.y = pack2bf(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(op + d) = pk;
      }
    }
    if (h == 0) {
      p.lse2[(static_cast<int64_t>(b) * p.Hq + hq) * p.Tq + qi] =
          lsum > 0.f ? m + __log2f(lsum) : INFINITY;
    }
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
  // 64 / (D/8) rows per wave, shuffle reduction inside the lane group
  const int lpr = D >> 3;  // lanes per row (power of two: 8 or 16)
  const int lane = threadIdx.x & 63;
  const int64_t row = (blockIdx.x * 4ll + (threadIdx.x >> 6)) * (64 / lpr) + lane / lpr;
  const int c = (lane % lpr) * 8;
  float acc = 0.f;
  const bool ok = row < static_cast<int64_t>(B) * H * T;
  if (ok) {
    const int t = static_cast<int>(row % T);
    const int64_t bh = row / T;
    const int hh = static_cast<int>(bh % H), b = static_cast<int>(bh / H);
    const bf16x8 a = load_bf16x8(o + b * o_sb + t * o_st + hh * o_sh + c);
    const bf16x8 g = load_bf16x8(dout + b * do_sb + t * do_st + hh * do_sh + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += bf2f(a[j]) * bf2f(g[j]);
  }
  for (int off = 1; off < lpr; off <<= 1) acc += __shfl_xor(acc, off, 64);
  if (ok && (lane % lpr) == 0) delta[row] = acc;
}

// ==============================================================================================
// backward main kernel
// ==============================================================================================
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void attn_bwd_kernel(AttnBwdParams p) {
  constexpr int BKV = 128, BQ = 32;
  constexpr int NCH = D / 8;
  constexpr int KS = D / 16;
  constexpr int DT = D / 32;
  // LDS: K [128][D], V [128][D], Q [32][D], dO [32][D]; dS^T [128][32] aliases Q+dO
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * BKV * D + 2 * BQ * D];
  bf16_t* Ks = smem;
  bf16_t* Vs = smem + BKV * D;
  bf16_t* Qs = smem + 2 * BKV * D;
  bf16_t* dOs = Qs + BQ * D;
  bf16_t* dSs = Qs;  // [128 keys][32 queries], 64-B rows (needs 8 KB = Q+dO region for D>=64)

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int nkb = (p.Tk + BKV - 1) / BKV;
  const int bid = blockIdx.x;
  const int kb = bid % nkb;
  const int rest = bid / nkb;
  const int hk = rest % p.Hkv, b = rest / p.Hkv;
  const int group = p.Hq / p.Hkv;
  const int k0 = kb * BKV;
  const int kw = k0 + 32 * w;  // this wave's first key
  const int kj = kw + l32;     // key on this lane

  const int kbeg = p.kv_start ? p.kv_start[b] : 0;
  const int kend = p.kv_end ? p.kv_end[b] : p.Tk;

  // stage K, V tiles (zero rows past Tk)
  {
    const bf16_t* kp = p.k + b * p.k_sb + static_cast<int64_t>(hk) * p.k_sh;
    const bf16_t* vp = p.v + b * p.v_sb + static_cast<int64_t>(hk) * p.v_sh;
    for (int ci = tid; ci < BKV * NCH; ci += 256) {
      const int row = ci / NCH, ch = ci % NCH;
      const int key = k0 + row;
      bf16x8 kv = key < p.Tk ? load_bf16x8(kp + key * p.k_st + ch * 8) : bf16x8{};
      bf16x8 vv = key < p.Tk ? load_bf16x8(vp + key * p.v_st + ch * 8) : bf16x8{};
      store_bf16x8(Ks + swz<D>(row, ch), kv);
      store_bf16x8(Vs + swz<D>(row, ch), vv);
    }
  }

  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    dk[dt] = f32x16{};
    dv[dt] = f32x16{};
  }

  // query range that can see any key of this block
  int qlo = 0, qhi = p.Tq;  // [qlo, qhi)
  if (CAUSAL) {
    qlo = max(0, k0 - p.causal_off);
    if (p.window > 0) qhi = min(qhi, k0 + BKV - 1 - p.causal_off + p.window);
  }
  const bool block_has_keys = k0 < kend && k0 + BKV > kbeg;
  const int qt0 = (qlo / BQ) * BQ;

  constexpr int QCPT = BQ * NCH / 256;  // chunks per thread for a [32][D] tile (D=128 -> 2)
  __shared__ float rowc[2][BQ];           // per-query lse2 / delta of the current tile
  const int nqt = qhi > qt0 ? (qhi - qt0 + BQ - 1) / BQ : 0;
  const int n_iter = block_has_keys ? group * nqt : 0;
  const int64_t dq_st = static_cast<int64_t>(p.Hq) * D;

  // register prefetch of the NEXT (head, q-tile) while the current one is computed (T14)
  bf16x8 qreg[QCPT], dreg[QCPT];
  float rreg = 0.f;
  auto prefetch = [&](int it) {
    const int hq = hk * group + it / nqt;
    const int qt = qt0 + (it % nqt) * BQ;
    const bf16_t* qp = p.q + b * p.q_sb + static_cast<int64_t>(hq) * p.q_sh;
    const bf16_t* dop = p.dout + b * p.do_sb + static_cast<int64_t>(hq) * p.do_sh;
#pragma unroll
    for (int c = 0; c < QCPT; ++c) {
      const int ci = tid + 256 * c;
      const int row = ci / NCH, ch = ci % NCH;
      const int qq = qt + row;
      qreg[c] = qq < p.Tq ? load_bf16x8(qp + qq * p.q_st + ch * 8) : bf16x8{};
      dreg[c] = qq < p.Tq ? load_bf16x8(dop + qq * p.do_st + ch * 8) : bf16x8{};
    }
    if (tid < 2 * BQ) {
      const int qq = qt + (tid & (BQ - 1));
      const float* src = (tid < BQ ? p.lse2 : p.delta) + (static_cast<int64_t>(b) * p.Hq + hq) * p.Tq;
      rreg = qq < p.Tq ? src[qq] : 0.f;
    }
  };
  if (n_iter > 0) prefetch(0);

  for (int it = 0; it < n_iter; ++it) {
    const int hq = hk * group + it / nqt;
    const int qt = qt0 + (it % nqt) * BQ;
    float* dqp = p.dq + (static_cast<int64_t>(b) * p.Tq) * p.Hq * D + static_cast<int64_t>(hq) * D;
    __syncthreads();  // previous iteration finished with Qs/dOs/dSs/rowc
#pragma unroll
    for (int c = 0; c < QCPT; ++c) {
      const int ci = tid + 256 * c;
      const int row = ci / NCH, ch = ci % NCH;
      store_bf16x8(Qs + swz<D>(row, ch), qreg[c]);
      store_bf16x8(dOs + swz<D>(row, ch), dreg[c]);
    }
    if (tid < 2 * BQ) rowc[tid / BQ][tid & (BQ - 1)] = rreg;
    __syncthreads();
    if (it + 1 < n_iter) prefetch(it + 1);

    // does this wave's key slice see any query of the tile? (wave-uniform)
    bool wave_active = kw < kend && kw + 32 > kbeg;
    bool need_mask = kw < kbeg || kw + 32 > kend || qt + BQ > p.Tq;
    if (CAUSAL) {
      wave_active = wave_active && kw <= qt + BQ - 1 + p.causal_off;
      need_mask = need_mask || (kw + 31 > qt + p.causal_off);
      if (p.window > 0) {
        wave_active = wave_active && (kw + 31 > qt + p.causal_off - p.window);
        need_mask = need_mask || (kw <= qt + BQ - 1 + p.causal_off - p.window);
      }
    }
    f32x16 sacc = f32x16{}, dpacc = f32x16{};
    if (wave_active) {
      // row constants of this lane's 16 accumulator rows r = (i&3) + 8(i>>2) + 4h: 4 x 16-B LDS
      // reads each for lse2 / delta, issued ahead of the MFMA chain so their latency hides
      float lr[16], dl[16];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(&rowc[0][8 * j + 4 * h]);
        const f32x4 c = *reinterpret_cast<const f32x4*>(&rowc[1][8 * j + 4 * h]);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          lr[4 * j + t] = a[t];
          dl[4 * j + t] = c[t];
        }
      }
      // S (rows = queries, cols = this wave's keys) and dP = dO V^T; operand fragments are
      // double-buffered one k-step ahead so no MFMA waits on its own LDS read
      s16x8 fa[2], fb[2], fc[2], fd[2];
      auto ld_sdp = [&](int ks, int sl) {
        fa[sl] = *reinterpret_cast<const s16x8*>(Qs + swz<D>(l32, 2 * ks + h));
        fb[sl] = *reinterpret_cast<const s16x8*>(Ks + swz<D>(32 * w + l32, 2 * ks + h));
        fc[sl] = *reinterpret_cast<const s16x8*>(dOs + swz<D>(l32, 2 * ks + h));
        fd[sl] = *reinterpret_cast<const s16x8*>(Vs + swz<D>(32 * w + l32, 2 * ks + h));
      };
      ld_sdp(0, 0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) ld_sdp(ks + 1, (ks + 1) & 1);
        sacc = mfma32(fa[ks & 1], fb[ks & 1], sacc);
        dpacc = mfma32(fc[ks & 1], fd[ks & 1], dpacc);
      }
      // P and dS; masking is branch-free: per lane, key kj vs query qt + rr + 4h
      const int dlt = kj - qt - p.causal_off - 4 * h;  // causal: visible iff rr >= dlt
      const int rlim = p.Tq - qt - 4 * h;              // rr < rlim
      const bool lane_ok = kj >= kbeg && kj < kend;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int rr = (i & 3) + 8 * (i >> 2);
        float pv = ex2(fmaf(sacc[i], p.scale2, -lr[i]));
        if (need_mask) {
          bool ok = lane_ok && rr < rlim;
          if (CAUSAL) {
            ok = ok && rr >= dlt;
            if (p.window > 0) ok = ok && rr < dlt + p.window;
          }
          pv = ok ? pv : 0.f;
        }
        sacc[i] = pv;
        dpacc[i] = pv * (dpacc[i] - dl[i]);
      }
      const s16x8 pb0 = pack8(sacc, 0), pb1 = pack8(sacc, 8);
      const s16x8 sb0 = pack8(dpacc, 0), sb1 = pack8(dpacc, 8);
      // dV^T += dO^T P ; dK^T += Q^T dS   (k = query, permuted accumulator-row order); the four
      // transposed fragments of tile dt+1 are read while tile dt's MFMAs run
      s16x8 ta[2], tb[2], tc[2], td[2];
      auto ld_kv = [&](int dt, int sl) {
        const int c0 = 32 * dt + 16 * ((lane >> 4) & 1);
        ta[sl] = tr_frag_perm<D>(dOs, 4 * h, c0, lane);
        tb[sl] = tr_frag_perm<D>(dOs, 16 + 4 * h, c0, lane);
        tc[sl] = tr_frag_perm<D>(Qs, 4 * h, c0, lane);
        td[sl] = tr_frag_perm<D>(Qs, 16 + 4 * h, c0, lane);
      };
      ld_kv(0, 0);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        if (dt + 1 < DT) ld_kv(dt + 1, (dt + 1) & 1);
        dv[dt] = mfma32(ta[dt & 1], pb0, dv[dt]);
        dv[dt] = mfma32(tb[dt & 1], pb1, dv[dt]);
        dk[dt] = mfma32(tc[dt & 1], sb0, dk[dt]);
        dk[dt] = mfma32(td[dt & 1], sb1, dk[dt]);
      }
    }
    __syncthreads();  // everyone done reading Qs/dOs
    // dS^T image [key 0..127][query 0..31], 64-B rows: lane writes its key row,
    // 4 groups of 4 consecutive queries (8 B each).
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int row = 32 * w + l32;
      uint2 pk;
      pk.x = pack2bf(dpacc[4 * g4 + 0], dpacc[4 * g4 + 1]);
      pk.y = pack2bf(dpacc[4 * g4 + 2], dpacc[4 * g4 + 3]);
      *reinterpret_cast<uint2*>(dSs + ds_off(row, 2 * g4 + h)) = pk;
    }
    __syncthreads();
    // dQ[q][d] for d in this wave's slices: sum over 128 keys. A = dS (q rows, keys k) via
    // transposed reads of dS^T; B = K (keys, d cols) via transposed reads of K.
    for (int dt = w; dt < DT; dt += 4) {
      f32x16 dqacc = f32x16{};
      const int i16 = lane & 15, qq2 = i16 >> 2, pp = i16 & 3;
      const int colc4 = (16 * ((lane >> 4) & 1) + 4 * pp) >> 2;  // query column block (8-B unit)
      s16x8 qa[2], qb[2];
      auto ld_dq = [&](int ks, int sl) {
        const int r0 = 16 * ks + 8 * h;
        qa[sl] = cat4(tr_read(dSs + ds_off(r0 + qq2, colc4)), tr_read(dSs + ds_off(r0 + 4 + qq2, colc4)));
        qb[sl] = tr_frag_nat<D>(Ks, r0, 32 * dt + 16 * ((lane >> 4) & 1), lane);
      };
      ld_dq(0, 0);
#pragma unroll
      for (int ks = 0; ks < BKV / 16; ++ks) {
        if (ks + 1 < BKV / 16) ld_dq(ks + 1, (ks + 1) & 1);
        dqacc = mfma32(qa[ks & 1], qb[ks & 1], dqacc);
      }
      // accumulate: lane holds d = 32dt + l32 (col), rows q = qt + (i&3) + 8(i>>2) + 4h.
      // Buffer atomics: the per-row offset is a scalar (soffset), one VGPR holds the lane part,
      // and the descriptor's num_records ends at the last valid query row of this tile, so the
      // hardware drops rows >= Tq (no per-element compares, no 64-bit address per element).
      {
        const int nrow = p.Tq - qt;  // > 0
        float* base = dqp + static_cast<int64_t>(qt) * dq_st;
        const int nrec = ((nrow - 1) * static_cast<int>(dq_st) + D) * 4;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, nrec, 0x00020000);
        const int voff = ((4 * h) * static_cast<int>(dq_st) + 32 * dt + l32) * 4;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int soff = ((i & 3) + 8 * (i >> 2)) * static_cast<int>(dq_st) * 4;
          __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(dqacc[i] * p.scale, rs, voff, soff, 0);
        }
      }
    }
  }

  // write dK (scaled) and dV: lane = key kj, regs = d rows (i&3) + 8(i>>2) + 4h of tile dt
  if (kj < p.Tk) {
    bf16_t* dkp = p.dk + b * p.dk_sb + kj * p.dk_st + static_cast<int64_t>(hk) * p.dk_sh;
    bf16_t* dvp = p.dv + b * p.dv_sb + kj * p.dv_st + static_cast<int64_t>(hk) * p.dv_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * dt + 8 * g4 + 4 * h;
        uint2 a, c;
        a.x = pack2bf(dk[dt][4 * g4] * p.scale, dk[dt][4 * g4 + 1] * p.scale);
        a.y = pack2bf(dk[dt][4 * g4 + 2] * p.scale, dk[dt][4 * g4 + 3] * p.scale);
        c.x = pack2bf(dv[dt][4 * g4], dv[dt][4 * g4 + 1]);
        c.y = pack2bf(dv[dt][4 * g4 + 2], dv[dt][4 * g4 + 3]);
        *reinterpret_cast<uint2*>(dkp + d) = a;
        *reinterpret_cast<uint2*>(dvp + d) = c;
      }
    }
  }
}

// fp32 dQ accumulator [rows, D] -> bf16 (strided destination)
__global__ __launch_bounds__(256) void f32_to_bf16_rows_kernel(const float* __restrict__ src,
                                                                int64_t rows, int cols,
                                                                bf16_t* __restrict__ dst,
                                                                int64_t dst_ld) {
  const int cv = cols / 8;
  const int64_t total = rows * cv;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t r = i / cv;
    const int c = static_cast<int>(i - r * cv) * 8;
    const f32x4* s = reinterpret_cast<const f32x4*>(src + r * cols + c);
    f32x4 a = s[0], bb = s[1];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = f2bf(a[j]);
      o[4 + j] = f2bf(bb[j]);
    }
    store_bf16x8(dst + r * dst_ld + c, o);
  }
}

// ----------------------------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------------------------
template <int D>
static void fwd_dispatch(const AttnParams& p, bool causal, hipStream_t st) {
  const int nqb = (p.Tq + 127) / 128;
  const dim3 grid(nqb * p.Hq * p.B);
  if (causal) attn_fwd_kernel<D, true><<<grid, 256, 0, st>>>(p);
  else attn_fwd_kernel<D, false><<<grid, 256, 0, st>>>(p);
}

void launch_attn_fwd(const AttnParams& p, int D, bool causal, hipStream_t st) {
  if (p.B == 0 || p.Tq == 0) return;
  switch (D) {
    case 64: fwd_dispatch<64>(p, causal, st); break;
    default: fwd_dispatch<128>(p, causal, st); break;
  }
}

void launch_attn_bwd_delta(const bf16_t* o, const bf16_t* dout, int64_t o_sb, int64_t o_st,
                           int64_t o_sh, int64_t do_sb, int64_t do_st, int64_t do_sh, int B,
                           int H, int T, int D, float* delta, hipStream_t st) {
  const int64_t rows = static_cast<int64_t>(B) * H * T;
  if (rows == 0) return;
  const int64_t rows_per_block = 4 * (64 / (D / 8));
  attn_bwd_delta_kernel<<<static_cast<unsigned>((rows + rows_per_block - 1) / rows_per_block), 256, 0, st>>>(
      o, dout, o_sb, o_st, o_sh, do_sb, do_st, do_sh, B, H, T, D, delta);
}

template <int D>
static void bwd_dispatch(const AttnBwdParams& p, bool causal, hipStream_t st) {
  const int nkb = (p.Tk + 127) / 128;
  const dim3 grid(nkb * p.Hkv * p.B);
  if (causal) attn_bwd_kernel<D, true><<<grid, 256, 0, st>>>(p);
  else attn_bwd_kernel<D, false><<<grid, 256, 0, st>>>(p);
}

void launch_attn_bwd(const AttnBwdParams& p, int D, bool causal, hipStream_t st) {
  if (p.B == 0 || p.Tq == 0) return;
  switch (D) {
    case 64: bwd_dispatch<64>(p, causal, st); break;
    default: bwd_dispatch<128>(p, causal, st); break;
  }
}

void launch_f32_to_bf16_rows(const float* src, int64_t rows, int cols, bf16_t* dst,
                             int64_t dst_ld, hipStream_t st) {
  const int64_t work = rows * (cols / 8);
  if (work == 0) return;
  int64_t g = (work + 255) / 256;
  if (g > 2048) g = 2048;
  f32_to_bf16_rows_kernel<<<static_cast<unsigned>(g), 256, 0, st>>>(src, rows, cols, dst, dst_ld);
}

}  // namespace dla
