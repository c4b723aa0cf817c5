// Device-driven grouped GEMM for the MoE experts (SURVEY K24 grouped GEMM, K25 fp8 MFMA forward).
//
// Reference semantics: HF MixtralSparseMoeBlock (transformers/models/mixtral/modeling_mixtral.py
// :96-128) runs one pair of nn.Linear per expert on a boolean-masked token subset, reached from
// src/training/train_dpo.py via the Mixtral north-star config. Here ONE launch covers every
// expert: the per-expert row ranges are read from a device array `offs[G+1]` (exclusive prefix
// of the routing counts), so there is no host sync, no per-expert launch loop, and the whole MoE
// layer is hipGraph-capturable.
//
// Three problem shapes share one kernel body:
//   MVAR (forward / input-gradient): C[rows of g, N] = A[rows of g, K] . B_g(n, k)
//        A = expert-sorted activations (k contiguous); B_g = expert weight, either [N, K]
//        (k contiguous: forward) or [K, N] (n contiguous: input gradient dX = dY . W_g).
//   KVAR (weight gradient): C_g[M, N] (+)= sum over the rows r of group g of A[r, m] B[r, n]
//        (dW_g = dY_g^T X_g): the reduction length is the group's row count.
// Tiles: 256 x 256 outputs per workgroup of 8 waves (2 x 4, 128 x 64 per wave), K step 64 bf16
// (128 fp8) = 128 bytes per row. Each operand tile is copied global -> LDS by
// global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip) into a lane-linear image whose XOR
// swizzle is applied on the per-lane SOURCE address (cdna guide §5.4 rule 21):
//   * k-contiguous operands: image [256 rows][128 B], read as MFMA fragments by ds_read_b128;
//     chunk swizzle f(row>>1) chosen so both the bf16 (16x16x32) and the fp8 (16x16x128)
//     fragment reads are bank-conflict free for the ds_read_b128 lane groups;
//   * m/n-contiguous operands: image [64 k-rows][512 B], read by ds_read_b64_tr_b16 (hardware
//     transpose, cdna guide T10); swizzle (k&3 | (k>>3&1)<<2) << 1 keeps each half-wave's eight
//     k-rows on distinct 32-byte bank slots.
// Two LDS buffers, one barrier per K step: the DMA of tile t+1 is issued before the MFMAs of tile
// t and drained (vmcnt(0)) at the barrier that ends the step (cdna guide §5 "glds vs register
// staging": 256² tile, 2 buffers, BK=64).
// MFMA: v_mfma_f32_16x16x32_bf16 (bf16), or the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4
// with unit E8M0 block scales for e4m3 operands (2x the bf16 rate; the row-wise fp8 scales are
// applied in the epilogue).
// Epilogues (staged through LDS so stores are 16 B per lane along rows):
//   STORE        bf16 or fp32 C, optional accumulate (beta = 1, the weight-gradient buffer);
//   SWIGLU_FWD   the gate|up projection: a workgroup owns gate columns [f0, f0+128) AND the
//                matching up columns, so it writes gu (kept for backward) and a = silu(g) * u
//                directly: no separate SwiGLU pass;
//   SWIGLU_BWD   the down projection's input gradient da, fused with the SwiGLU backward: reads
//                gu, writes dgu = [da * u * silu'(g), da * silu(g)] and the recomputed a (the
//                B operand of the down-weight gradient).
// Rows/columns past the problem edge are clamped on load and masked on store; reduction tails
// read a zero page (no out-of-bounds access in any lane).
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "common.h"
#include "gg_params.h"

namespace dla {

namespace {

constexpr int kGgThreads = 512;
constexpr int kGgNGroup = 4;  // N tiles per L2 tile group (MVAR)
constexpr int kGgTileBytes = 256 * 128;            // one operand tile: 256 rows x 128 B
constexpr int kGgBufBytes = 2 * kGgTileBytes;      // A + B
constexpr int kGgEpiStride = 68;                   // fp32 epilogue row stride (bank-spread)
constexpr int kGgEpiWaveFloats = 64 * kGgEpiStride;
constexpr int kGgSmem = (2 * kGgBufBytes > 8 * kGgEpiWaveFloats * 4) ? 2 * kGgBufBytes
                                                                      : 8 * kGgEpiWaveFloats * 4;

enum { kMVar = 0, kKVar = 1 };
enum { kEpiStore = 0, kEpiSwigluFwd = 1, kEpiSwigluBwd = 2 };

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __attribute__((aligned(16))) uint8_t g_gg_zero[1024];  // zero page for reduction tails

// K-contiguous image: chunk swizzle of row r (table over row pairs, see header)
__device__ __forceinline__ int gg_fsw(int r) { return (0x32765410 >> (((r >> 1) & 7) << 2)) & 7; }
__device__ __forceinline__ int gg_koff(int r, int c) { return r * 128 + ((c ^ gg_fsw(r)) << 4); }
// MN-contiguous image: chunk swizzle of k-row k
__device__ __forceinline__ int gg_hsw(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }
__device__ __forceinline__ int gg_moff(int k, int c) { return k * 512 + ((c ^ gg_hsw(k)) << 4); }

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

__device__ __forceinline__ s16x4 gg_tr(const uint8_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}

// The same read as inline asm: hipcc treats every ds_read_tr builtin as aliasing the LDS-DMA
// writes in flight and waits vmcnt(0) before it, which would drain the counted pipeline of the
// 4-phase schedule. Its results are waited for by hand (lgkmcnt(0) + sched_barrier before use).
__device__ __forceinline__ s16x4 gg_tr_asm(const uint8_t* p) {
  s16x4 r;
  const uint32_t a = static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) uint8_t*)(p)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

__device__ __forceinline__ float gg_sig(float x) { return 1.f / (1.f + __expf(-x)); }

template <int I, int N, class Fn>
__device__ __forceinline__ void gg_static_for(Fn&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    gg_static_for<I + 1, N>(f);
  }
}

__device__ __forceinline__ void gg_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

}  // namespace



// SCHED (K-step schedule; A/B-selected on hardware, tools/grouped_gemm_bench.py):
//   0: the next tile's 8 DMA pieces issued in one burst ahead of the MFMAs, fragments read per
//      MFMA group; 1: burst DMA, fragments of the next group prefetched in registers;
//   2: DMA pieces interleaved between MFMA groups, fragments prefetched;
//   3: ping-pong phases: a K step is 4 phases of 16 MFMA-equivalents per wave; the waves of
//      the second M half (one per SIMD) run one barrier behind the first, so on every SIMD one
//      wave's MFMA cluster overlaps the other wave's LDS fragment reads and DMA issue (the
//      wave-group stagger of the cdna guide's 8-phase template). Next-tile DMA pieces go out
//      in phases 1-2 (>= 2 barriers after the last read of that buffer: WAR-safe), each wave
//      retires its own with vmcnt(0) in phase 3, one barrier before the tile's first read.
//   4: (bf16, the default) counted 4-phase step: quarter tiles staged 2-6 phases ahead into
//      whichever buffer slot is free, a counted vmcnt per phase, never vmcnt(0) in the loop
//      (see the SCH == 4 loop). Mixtral expert block, same box: gate|up + SwiGLU forward 1205
//      vs 1092 TF/s (schedule 0), down forward 1192 vs 1002, up dgrad 1110 vs 821 (schedule 3),
//      down dgrad + SwiGLU backward 922 vs 768, weight gradients 813-936 vs 689-835.
template <int MODE, bool BK, bool FP8, int EPI, bool OUTF32, int SCHED>
__global__ __launch_bounds__(kGgThreads) void grouped_gemm_kernel(GGParams p) {
  // the ping-pong schedule needs more registers than the fp8 fragments leave: fp8 uses 1; the
  // counted 4-phase schedule (4) is built for the bf16 k-contiguous forward only, others use 0
  constexpr bool PH4 = SCHED == 4 && !FP8;
  constexpr int SCH = PH4 ? 4 : SCHED == 4 ? 0 : (SCHED == 3 && FP8) ? 1 : SCHED;
  __shared__ __attribute__((aligned(16))) uint8_t smem[kGgSmem];
  constexpr int ESZ = FP8 ? 1 : 2;  // operand element size
  constexpr int KT = 128 / ESZ;     // reduction elements per K step
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;

  // ---------------------------------------------------------------- tile -> (group, m, n)
  const int nblk = gridDim.x;
  const int L = xcd_remap(blockIdx.x, nblk);
  int g = 0, mt = 0, nt = 0;
  int row0 = 0, row_end = 0, Kg = p.K;
  if constexpr (MODE == kMVar) {
    // L2-aware order: consecutive logical tiles (the ~32 a workgroup's XCD runs at once) form
    // 8 M tiles x kGgNGroup N tiles, so every activation panel and every weight panel fetched
    // into that XCD's L2 is shared by several resident workgroups.
    const int per = p.tiles_m * kGgNGroup;
    const int ng = L / per, r = L % per;
    nt = ng * kGgNGroup + r % kGgNGroup;
    if (nt >= p.tiles_n) return;
    int t = r / kGgNGroup;
    bool found = false;
    for (int gg = 0; gg < p.G; ++gg) {
      const int a = p.offs[gg], b = p.offs[gg + 1];
      const int tg = (b - a + 255) >> 8;
      if (t < tg) {
        g = gg;
        row0 = a + t * 256;
        row_end = b;
        found = true;
        break;
      }
      t -= tg;
    }
    if (!found) return;
    mt = 0;
  } else {
    // per group: L2 tile groups of 8 M tiles x kGgNGroup N tiles (as MVAR)
    const int ngr = (p.tiles_n + kGgNGroup - 1) / kGgNGroup;
    const int per = p.tiles_m * ngr * kGgNGroup;
    g = L / per;
    const int rem = L % per;
    const int ng = rem / (p.tiles_m * kGgNGroup), r = rem % (p.tiles_m * kGgNGroup);
    mt = r / kGgNGroup;
    nt = ng * kGgNGroup + r % kGgNGroup;
    if (nt >= p.tiles_n) return;
    row0 = p.offs[g];
    Kg = p.offs[g + 1] - row0;
    if (Kg == 0 && p.accumulate) return;
  }

  // ---------------------------------------------------------------- per-lane DMA sources
  // Each wave issues 4 pieces (1 KiB each) of the A tile and 4 of the B tile per K step.
  const uint8_t* srcA[4];
  const uint8_t* srcB[4];
  int cA[4], cB[4];  // K-contig: logical chunk; MN-contig: k-row within the tile
  int pA[4], pB[4];  // 1-KiB piece (8 image rows) each source fills; wave-uniform
  const int64_t Kbytes = static_cast<int64_t>(p.K) * ESZ;
  const uint8_t* zp = g_gg_zero + lane * 16;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = 4 * w + i;
    pA[i] = pB[i] = piece;
    if constexpr (SCH == 4) {
      // quarter tiles (see the SCH == 4 loop), source i = 2h + j takes piece q = 2w + j of the
      // 16 pieces of quarter h: k-contiguous A = rows of the waves' first / second 64-row
      // halves, k-contiguous B = rows of their first / second 32-column halves, an
      // mn-contiguous operand = k-rows [0, 32) / [32, 64) (16 KiB contiguous each)
      const int h = i >> 1, q = 2 * w + (i & 1);
      pA[i] = (MODE == kKVar) ? h * 16 + q : (q >> 3) * 16 + h * 8 + (q & 7);
      pB[i] = !BK ? h * 16 + q : (EPI == kEpiSwigluFwd) ? h * 16 + q : (q >> 2) * 8 + h * 4 + (q & 3);
    }
    if constexpr (MODE == kMVar) {
      // A: k-contiguous activation rows of the group (clamped: rows past the group end are
      // loaded from its last row and never stored)
      const int r = pA[i] * 8 + (lane >> 3);
      const int c = (lane & 7) ^ gg_fsw(r);
      const int gr = min(row0 + r, row_end - 1);
      srcA[i] = p.A + static_cast<int64_t>(gr) * p.lda * ESZ;
      cA[i] = c;
      if constexpr (BK) {
        const int r = pB[i] * 8 + (lane >> 3);
        const int c = (lane & 7) ^ gg_fsw(r);
        int n;
        if constexpr (EPI == kEpiSwigluFwd) {
          const int f0 = nt * 128;
          n = r < 128 ? f0 + r : p.F + f0 + (r - 128);
        } else {
          n = min(nt * 256 + r, p.N - 1);
        }
        srcB[i] = p.B + (static_cast<int64_t>(g) * p.sBg + static_cast<int64_t>(n) * p.ldb) * ESZ;
        cB[i] = c;
      } else {
        const int kr = pB[i] * 2 + (lane >> 5);
        const int cc = (lane & 31) ^ gg_hsw(kr);
        const int ch = min(nt * 32 + cc, p.N / 8 - 1);
        srcB[i] = p.B + (static_cast<int64_t>(g) * p.sBg + static_cast<int64_t>(ch) * 8) * ESZ;
        cB[i] = kr;
      }
    } else {
      const int kra = pA[i] * 2 + (lane >> 5), krb = pB[i] * 2 + (lane >> 5);
      const int cha = min(mt * 32 + ((lane & 31) ^ gg_hsw(kra)), p.M / 8 - 1);
      const int chb = min(nt * 32 + ((lane & 31) ^ gg_hsw(krb)), p.N / 8 - 1);
      srcA[i] = p.A + (static_cast<int64_t>(row0) * p.lda + static_cast<int64_t>(cha) * 8) * ESZ;
      srcB[i] = p.B + (static_cast<int64_t>(row0) * p.ldb + static_cast<int64_t>(chb) * 8) * ESZ;
      cA[i] = kra;
      cB[i] = krb;
    }
  }

  // one 1-KiB DMA piece j (0..3: A pieces, 4..7: B pieces) of K tile t into LDS buffer buf
  auto stage_piece = [&](int t, int buf, int j) {
    uint8_t* base = smem + buf * kGgBufBytes + (j >= 4 ? kGgTileBytes : 0);
    const int i = j & 3;
    uint8_t* dst = base + (4 * w + i) * 1024;
    if constexpr (MODE == kMVar) {
      if (j < 4 || BK) {
        const int64_t kb = static_cast<int64_t>(t) * 128 + (j < 4 ? cA[i] : cB[i]) * 16;
        glds16(kb < Kbytes ? (j < 4 ? srcA[i] : srcB[i]) + kb : zp, dst);
      } else {
        const int k = t * KT + cB[i];
        glds16(k < p.K ? srcB[i] + static_cast<int64_t>(k) * p.ldb * ESZ : zp, dst);
      }
    } else {
      const int k = t * KT + cA[i];
      const bool ok = k < Kg;
      if (j < 4) glds16(ok ? srcA[i] + static_cast<int64_t>(k) * p.lda * ESZ : zp, dst);
      else glds16(ok ? srcB[i] + static_cast<int64_t>(k) * p.ldb * ESZ : zp, dst);
    }
  };

  // ---------------------------------------------------------------- fragment readers
  const int fr = lane & 15, fg = lane >> 4;
  // B-tile row of the wave's n-subtile ni
  auto brow = [&](int ni) -> int {
    if constexpr (EPI == kEpiSwigluFwd) return (ni < 2 ? 0 : 128) + wn * 32 + (ni & 1) * 16;
    else return wn * 64 + ni * 16;
  };
  // bf16 fragment of 16 rows [r0, r0+16) at k-step kk from a k-contiguous image
  auto kfrag = [&](const uint8_t* img, int r0, int kk) -> s16x8 {
    const int r = r0 + fr;
    return *reinterpret_cast<const s16x8*>(img + gg_koff(r, kk * 4 + fg));
  };
  // bf16 fragment of 16 columns [c0, c0+16) at k-step kk from an mn-contiguous image
  auto mfrag = [&](const uint8_t* img, int c0, int kk) -> s16x8 {
    const int q = fr >> 2, pp = fr & 3;
    const int ch = (c0 >> 3) + (pp >> 1), sub = (pp & 1) * 8;
    const int k1 = kk * 32 + 8 * fg + q;
    const s16x4 x = gg_tr(img + gg_moff(k1, ch) + sub);
    const s16x4 y = gg_tr(img + gg_moff(k1 + 4, ch) + sub);
    return s16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  };
  auto mfrag_asm = [&](const uint8_t* img, int c0, int kk) -> s16x8 {
    const int q = fr >> 2, pp = fr & 3;
    const int ch = (c0 >> 3) + (pp >> 1), sub = (pp & 1) * 8;
    const int k1 = kk * 32 + 8 * fg + q;
    const s16x4 x = gg_tr_asm(img + gg_moff(k1, ch) + sub);
    const s16x4 y = gg_tr_asm(img + gg_moff(k1 + 4, ch) + sub);
    return s16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  };
  // fp8 fragment (32 k per lane) of 16 rows from a k-contiguous image
  auto kfrag8 = [&](const uint8_t* img, int r0) -> i32x8 {
    const int r = r0 + fr;
    const i32x4 x = *reinterpret_cast<const i32x4*>(img + gg_koff(r, 2 * fg));
    const i32x4 y = *reinterpret_cast<const i32x4*>(img + gg_koff(r, 2 * fg + 1));
    return i32x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // One K step on LDS buffer `buf`, software-pipelined: the A fragment of the next MFMA group
  // and the second k-half's B fragments are read while the current group's MFMAs run, and (PRE)
  // the 8 DMA pieces of the next K tile are issued one every other group instead of in a burst
  // ahead of the MFMAs.
  auto compute = [&](int buf, int tn, auto pre) {
    constexpr bool PRE = decltype(pre)::value && SCH == 2;
    const uint8_t* imA = smem + buf * kGgBufBytes;
    const uint8_t* imB = imA + kGgTileBytes;
    if constexpr (SCH == 0) {
      if constexpr (FP8) {
        i32x8 bfr[4];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) bfr[ni] = kfrag8(imB, brow(ni));
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
          const i32x8 af = kfrag8(imA, wm * 128 + mi * 16);
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bfr[ni], acc[mi][ni], 0,
                                                                           0, 0, 127, 0, 127);
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          s16x8 bfr[4];
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) bfr[ni] = BK ? kfrag(imB, brow(ni), kk) : mfrag(imB, brow(ni), kk);
#pragma unroll
          for (int mi = 0; mi < 8; ++mi) {
            const s16x8 af = (MODE == kMVar) ? kfrag(imA, wm * 128 + mi * 16, kk)
                                             : mfrag(imA, wm * 128 + mi * 16, kk);
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[ni], acc[mi][ni], 0, 0, 0);
          }
        }
      }
    } else if constexpr (FP8) {
      i32x8 bfr[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bfr[ni] = kfrag8(imB, brow(ni));
      i32x8 a = kfrag8(imA, wm * 128);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        i32x8 an = a;
        if (mi < 7) an = kfrag8(imA, wm * 128 + (mi + 1) * 16);
        if constexpr (PRE) stage_piece(tn, buf ^ 1, mi);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, bfr[ni], acc[mi][ni], 0, 0,
                                                                         0, 127, 0, 127);
        a = an;
      }
    } else {
      auto rdA = [&](int mi, int kk) -> s16x8 {
        return (MODE == kMVar) ? kfrag(imA, wm * 128 + mi * 16, kk) : mfrag(imA, wm * 128 + mi * 16, kk);
      };
      auto rdB = [&](int ni, int kk) -> s16x8 {
        return BK ? kfrag(imB, brow(ni), kk) : mfrag(imB, brow(ni), kk);
      };
      s16x8 b0[4], b1[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) b0[ni] = rdB(ni, 0);
      s16x8 a = rdA(0, 0);
#pragma unroll
      for (int sidx = 0; sidx < 16; ++sidx) {
        const int kk = sidx >> 3, mi = sidx & 7;
        s16x8 an = a;
        if (sidx < 15) an = rdA((sidx + 1) & 7, (sidx + 1) >> 3);
        if (sidx >= 4 && sidx < 8) b1[sidx - 4] = rdB(sidx - 4, 1);
        if constexpr (PRE) {
          if ((sidx & 1) == 0) stage_piece(tn, buf ^ 1, sidx >> 1);
        }
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, kk ? b1[ni] : b0[ni], acc[mi][ni], 0, 0, 0);
        a = an;
      }
    }
  };

  // ---------------------------------------------------------------- main loop
  const int nk = (Kg + KT - 1) / KT;
  if constexpr (SCH == 4) {
    // Counted 4-phase K step (cdna guide §5 "256² 8-phase template", T3+T4): each phase runs
    // 16 MFMAs of the wave between two raw barriers, the second wave group (wm = 1) one barrier
    // behind the first. A K tile is staged as 4 quarter tiles QA0 / QA1 / QB0 / QB1 (pieces:
    // see pA / pB), each restaged as soon as its slot is 2 phases past its last read (the WAR
    // distance the staggered groups need), so a quarter is in flight for 2-6 phases; each wave
    // waits a counted vmcnt (never 0 in the loop) before the first barrier of a phase, which
    // retires what the next phase reads (cdna guide: a staged buffer is read one phase after
    // the wait that retires it). Zero page past the last tile. Layouts:
    //   F (forward, both k-contiguous): phases = quadrants (mh, nh) (0,0) (0,1) (1,1) (1,0);
    //     reads QA0+QB0 / QB1 / QA1 / - (QB0 held to phase 3); stages QB1, QA1 of tile t+1,
    //     QA0, QB0 of tile t+2; vmcnt(8).
    //   D (input gradient, B mn-contiguous): phases (kk, mh) (0,0) (0,1) (1,0) (1,1); reads
    //     QA0+QB0 / QA1 / QA0+QB1 / QA1; stages QB1, QA0, QA1 of t+1, QB0 of t+2; vmcnt(4).
    //   W (weight gradient, both mn-contiguous): phases (kk, mh); reads QA0+QB0 / QA0 / QA1+QB1
    //     / QA1; stages QB1, QA1 of t+1, QB0, QA0 of t+2; vmcnt(8).
    if (nk > 0) {
      constexpr int LAY = (MODE == kKVar) ? 2 : BK ? 0 : 1;
      constexpr bool KQA = MODE == kKVar, KQB = !BK;
      const int Klim = (MODE == kMVar) ? p.K : Kg;
      // quarter qi: 0 = QA0, 1 = QB0, 2 = QB1, 3 = QA1
      auto stage_q = [&](int t, int buf, auto QI) {
        constexpr int qi = decltype(QI)::value;
        constexpr bool isA = qi == 0 || qi == 3;
        constexpr int h = (qi == 0 || qi == 1) ? 0 : 1;
        constexpr bool kq = isA ? KQA : KQB;
        uint8_t* base = smem + buf * kGgBufBytes + (isA ? 0 : kGgTileBytes);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int i = h * 2 + j;
          uint8_t* dst = base + (isA ? pA[i] : pB[i]) * 1024;
          const uint8_t* src = isA ? srcA[i] : srcB[i];
          if constexpr (!kq) {
            const int64_t kb = static_cast<int64_t>(t) * 128 + (isA ? cA[i] : cB[i]) * 16;
            glds16(kb < Kbytes ? src + kb : zp, dst);
          } else {
            const int k = t * KT + (isA ? cA[i] : cB[i]);
            glds16(k < Klim ? src + static_cast<int64_t>(k) * (isA ? p.lda : p.ldb) * ESZ : zp, dst);
          }
        }
      };
      using Q0 = std::integral_constant<int, 0>;
      using Q1 = std::integral_constant<int, 1>;
      using Q2 = std::integral_constant<int, 2>;
      using Q3 = std::integral_constant<int, 3>;
      auto vwait = [&]() {
        if constexpr (LAY == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      };
      s16x8 af[2][4], blo[2][2], bhi[2][2], bq[4];
      if constexpr (LAY == 0) {
        stage_q(0, 0, Q0{}); stage_q(0, 0, Q1{}); stage_q(0, 0, Q2{}); stage_q(0, 0, Q3{});
        stage_q(1, 1, Q0{}); stage_q(1, 1, Q1{});
      } else if constexpr (LAY == 1) {
        stage_q(0, 0, Q1{}); stage_q(0, 0, Q2{}); stage_q(0, 0, Q0{}); stage_q(0, 0, Q3{});
        stage_q(1, 1, Q1{});
      } else {
        stage_q(0, 0, Q1{}); stage_q(0, 0, Q0{}); stage_q(0, 0, Q2{}); stage_q(0, 0, Q3{});
        stage_q(1, 1, Q1{}); stage_q(1, 1, Q0{});
      }
      vwait();
      gg_barrier();
      if (wm == 1) gg_barrier();  // second wave group runs one barrier behind
      for (int t = 0; t < nk; ++t) {
        const uint8_t* imA = smem + (t & 1) * kGgBufBytes;
        const uint8_t* imB = imA + kGgTileBytes;
        gg_static_for<0, 4>([&](auto PH) {
          constexpr int ph = decltype(PH)::value;
          if constexpr (LAY == 0) {
            constexpr int mh = ph >> 1;
            if constexpr (ph == 0 || ph == 2) {
#pragma unroll
              for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int i = 0; i < 4; ++i) af[kk][i] = kfrag(imA, wm * 128 + (mh * 4 + i) * 16, kk);
            }
            if constexpr (ph == 0) {
#pragma unroll
              for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int j = 0; j < 2; ++j) blo[kk][j] = kfrag(imB, brow(j), kk);
            }
            if constexpr (ph == 1) {
#pragma unroll
              for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int j = 0; j < 2; ++j) bhi[kk][j] = kfrag(imB, brow(2 + j), kk);
            }
            if constexpr (ph == 0) stage_q(t + 1, (t + 1) & 1, Q2{});
            if constexpr (ph == 1) stage_q(t + 1, (t + 1) & 1, Q3{});
            if constexpr (ph == 2) stage_q(t + 2, t & 1, Q0{});
            if constexpr (ph == 3) stage_q(t + 2, t & 1, Q1{});
          } else {
            constexpr int kk = ph >> 1, mh = ph & 1;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              if constexpr (KQA) af[0][i] = mfrag_asm(imA, wm * 128 + (mh * 4 + i) * 16, kk);
              else af[0][i] = kfrag(imA, wm * 128 + (mh * 4 + i) * 16, kk);
            }
            if constexpr (mh == 0) {
#pragma unroll
              for (int ni = 0; ni < 4; ++ni) bq[ni] = mfrag_asm(imB, brow(ni), kk);
            }
            if constexpr (LAY == 1) {
              if constexpr (ph == 0) stage_q(t + 1, (t + 1) & 1, Q2{});
              if constexpr (ph == 1) stage_q(t + 1, (t + 1) & 1, Q0{});
              if constexpr (ph == 2) stage_q(t + 1, (t + 1) & 1, Q3{});
              if constexpr (ph == 3) stage_q(t + 2, t & 1, Q1{});
            } else {
              if constexpr (ph == 0) stage_q(t + 1, (t + 1) & 1, Q2{});
              if constexpr (ph == 1) stage_q(t + 1, (t + 1) & 1, Q3{});
              if constexpr (ph == 2) stage_q(t + 2, t & 1, Q1{});
              if constexpr (ph == 3) stage_q(t + 2, t & 1, Q0{});
            }
          }
          vwait();
          gg_barrier();
          if constexpr (LAY != 0) {  // the inline-asm transposed reads of this phase
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
          }
          __builtin_amdgcn_s_setprio(1);
          if constexpr (LAY == 0) {
            constexpr int mh = ph >> 1, nh = (ph == 1 || ph == 2) ? 1 : 0;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
              for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                  acc[mh * 4 + i][nh * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                      af[kk][i], nh ? bhi[kk][j] : blo[kk][j], acc[mh * 4 + i][nh * 2 + j], 0, 0, 0);
          } else {
            constexpr int mh = ph & 1;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
              for (int ni = 0; ni < 4; ++ni)
                acc[mh * 4 + i][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bq[ni], acc[mh * 4 + i][ni], 0, 0, 0);
          }
          __builtin_amdgcn_s_setprio(0);
          gg_barrier();
        });
      }
      if (wm == 0) gg_barrier();  // balance the barrier count of the two groups
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else if constexpr (SCH == 3) {
    if (nk > 0) {
      s16x8 af[4], bfv[4];
      i32x8 af8[2], bf8[4];
      auto read_phase = [&](auto PH, int t) {
        constexpr int ph = decltype(PH)::value;
        const int buf = t & 1;
        const uint8_t* imA = smem + buf * kGgBufBytes;
        const uint8_t* imB = imA + kGgTileBytes;
        if constexpr (FP8) {
          if constexpr (ph == 0) {
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) bf8[ni] = kfrag8(imB, brow(ni));
          }
#pragma unroll
          for (int i = 0; i < 2; ++i) af8[i] = kfrag8(imA, wm * 128 + (ph * 2 + i) * 16);
        } else {
          constexpr int kk = ph >> 1, half = ph & 1;
          if constexpr (half == 0) {
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) bfv[ni] = BK ? kfrag(imB, brow(ni), kk) : mfrag(imB, brow(ni), kk);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
            af[i] = (MODE == kMVar) ? kfrag(imA, wm * 128 + (half * 4 + i) * 16, kk)
                                    : mfrag(imA, wm * 128 + (half * 4 + i) * 16, kk);
        }
        if constexpr (ph == 1 || ph == 2) {
          if (t + 1 < nk) {
#pragma unroll
            for (int j = 0; j < 4; ++j) stage_piece(t + 1, buf ^ 1, (ph - 1) * 4 + j);
          }
        }
        if constexpr (ph == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      };
      auto mfma_phase = [&](auto PH) {
        constexpr int ph = decltype(PH)::value;
        __builtin_amdgcn_s_setprio(1);
        if constexpr (FP8) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
              acc[ph * 2 + i][ni] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                  af8[i], bf8[ni], acc[ph * 2 + i][ni], 0, 0, 0, 127, 0, 127);
        } else {
          constexpr int half = ph & 1;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
              acc[half * 4 + i][ni] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfv[ni], acc[half * 4 + i][ni], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
      };
#pragma unroll
      for (int j = 0; j < 8; ++j) stage_piece(0, 0, j);
      __syncthreads();
      if (wm == 1) gg_barrier();  // second wave group runs one barrier behind
      read_phase(std::integral_constant<int, 0>{}, 0);
      for (int t = 0; t < nk; ++t) {
        gg_static_for<0, 4>([&](auto PH) {
          constexpr int ph = decltype(PH)::value;
          gg_barrier();
          mfma_phase(PH);
          gg_barrier();
          if constexpr (ph < 3) {
            read_phase(std::integral_constant<int, ph + 1>{}, t);
          } else {
            if (t + 1 < nk) read_phase(std::integral_constant<int, 0>{}, t + 1);
          }
        });
      }
      if (wm == 0) gg_barrier();  // balance the barrier count of the two groups
      __syncthreads();
    }
  } else if (nk > 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) stage_piece(0, 0, j);
    __syncthreads();
    for (int t = 0; t + 1 < nk; ++t) {
      if constexpr (SCH != 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) stage_piece(t + 1, (t + 1) & 1, j);
      }
      compute(t & 1, t + 1, std::true_type{});
      __syncthreads();  // drains this step's DMA (vmcnt(0)) and retires every wave's reads of buf
    }
    compute((nk - 1) & 1, 0, std::false_type{});
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  const float* sbg = FP8 ? p.sb + g * p.sSg : nullptr;
  float* ep = reinterpret_cast<float*>(smem) + w * kGgEpiWaveFloats;
  int mbase, nbase, mlim;
  if constexpr (MODE == kMVar) {
    mbase = row0 + wm * 128;
    mlim = row_end;
    nbase = (EPI == kEpiSwigluFwd ? nt * 128 + wn * 32 : nt * 256 + wn * 64);
  } else {
    mbase = mt * 256 + wm * 128;
    mlim = p.M;
    nbase = nt * 256 + wn * 64;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int mm = 0; mm < 4; ++mm)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          ep[(mm * 16 + fg * 4 + i) * kGgEpiStride + ni * 16 + fr] = acc[h * 4 + mm][ni][i];
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes done
    __builtin_amdgcn_wave_barrier();
    if constexpr (EPI == kEpiSwigluFwd) {
      // 64 rows x 4 units of 8 gate columns (+ the matching 8 up columns)
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int u = it * 64 + lane;
        const int r = u >> 2, cu = u & 3;
        const int grow = mbase + h * 64 + r;
        if (grow < mlim) {
          const float* e = ep + r * kGgEpiStride + cu * 8;
          const int f = nbase + cu * 8;
          float gv[8], uv[8], av[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            gv[j] = e[j];
            uv[j] = e[32 + j];
          }
          if constexpr (FP8) {
            const float s = p.sa[grow];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              gv[j] *= s * sbg[f + j];
              uv[j] *= s * sbg[p.F + f + j];
            }
          }
          const bf16x8 gb = pack_bf16x8(gv), ub = pack_bf16x8(uv);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float gf = bf2f(gb[j]), uf = bf2f(ub[j]);
            av[j] = gf * gg_sig(gf) * uf;
          }
          bf16_t* gu = reinterpret_cast<bf16_t*>(p.C) + static_cast<int64_t>(grow) * p.ldc;
          store_bf16x8(gu + f, gb);
          store_bf16x8(gu + p.F + f, ub);
          store_bf16x8(p.out2 + static_cast<int64_t>(grow) * p.ld_out2 + f, pack_bf16x8(av));
        }
      }
    } else if constexpr (OUTF32) {
      // 64 rows x 16 units of 4 fp32 columns
#pragma unroll 4
      for (int it = 0; it < 16; ++it) {
        const int u = it * 64 + lane;
        const int r = u >> 4, cu = u & 15;
        const int grow = mbase + h * 64 + r;
        const int gcol = nbase + cu * 4;
        if (grow < mlim && gcol < p.N) {
          f32x4 v = *reinterpret_cast<const f32x4*>(ep + r * kGgEpiStride + cu * 4);
          float* c = reinterpret_cast<float*>(p.C) + static_cast<int64_t>(g) * p.sCg +
                     static_cast<int64_t>(grow) * p.ldc + gcol;
          if (p.accumulate) v += *reinterpret_cast<const f32x4*>(c);
          *reinterpret_cast<f32x4*>(c) = v;
        }
      }
    } else {
      // 64 rows x 8 units of 8 bf16 columns
#pragma unroll 4
      for (int it = 0; it < 8; ++it) {
        const int u = it * 64 + lane;
        const int r = u >> 3, cu = u & 7;
        const int grow = mbase + h * 64 + r;
        const int gcol = nbase + cu * 8;
        if (grow < mlim && gcol < p.N) {
          const float* e = ep + r * kGgEpiStride + cu * 8;
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = e[j];
          if constexpr (FP8) {
            const float s = p.sa[grow];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] *= s * sbg[gcol + j];
          }
          if constexpr (EPI == kEpiSwigluBwd) {
            // v = da (fp32); gu at (grow, gcol) and (grow, F + gcol)
            const bf16_t* gup = p.aux + static_cast<int64_t>(grow) * p.ld_aux;
            const bf16x8 gb = load_bf16x8(gup + gcol), ub = load_bf16x8(gup + p.F + gcol);
            float dgv[8], duv[8], av[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float gf = bf2f(gb[j]), uf = bf2f(ub[j]);
              const float sg = gg_sig(gf);
              const float d = bf2f(f2bf(v[j]));  // da rounded as the unfused path stores it
              duv[j] = d * (gf * sg);
              dgv[j] = d * uf * sg * (1.f + gf * (1.f - sg));
              av[j] = gf * sg * uf;
            }
            bf16_t* dg = reinterpret_cast<bf16_t*>(p.C) + static_cast<int64_t>(grow) * p.ldc;
            store_bf16x8(dg + gcol, pack_bf16x8(dgv));
            store_bf16x8(dg + p.F + gcol, pack_bf16x8(duv));
            store_bf16x8(p.out2 + static_cast<int64_t>(grow) * p.ld_out2 + gcol, pack_bf16x8(av));
          } else {
            bf16_t* c = reinterpret_cast<bf16_t*>(p.C) + static_cast<int64_t>(g) * p.sCg +
                        static_cast<int64_t>(grow) * p.ldc + gcol;
            if (p.accumulate) {
              const bf16x8 old = load_bf16x8(c);
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] += bf2f(old[j]);
            }
            store_bf16x8(c, pack_bf16x8(v));
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------------------------------- host
// Default schedule (measured, tools/grouped_gemm_bench.py, profiles/r5_grouped_gemm.md): the
// counted 4-phase step for every bf16 layout (fp8 keeps the plain 2-phase step). 0-3 stay
// selectable for A/B.
// K-step schedule: DLA_GG_SCHED read once per process (default 4, the counted 4-phase step);
// tests and tools/grouped_gemm_bench.py switch it in-process through gg_set_sched
// (torch.ops.dla.gg_set_sched) instead of an environment read on every launch.
static int& gg_sched_slot() {
  static int v = [] {
    const char* e = std::getenv("DLA_GG_SCHED");
    return e ? std::atoi(e) : 4;
  }();
  return v;
}
static int gg_sched() { return gg_sched_slot(); }

int gg_set_sched(int sched) {
  int& s = gg_sched_slot();
  const int prev = s;
  s = sched < 0 ? 4 : sched;
  return prev;
}

template <int MODE, bool BK, bool FP8, int EPI, bool OUTF32>
static void gg_launch(const GGParams& p, int nblk, hipStream_t st) {
  switch (gg_sched()) {
    case 1:
      hipLaunchKernelGGL((grouped_gemm_kernel<MODE, BK, FP8, EPI, OUTF32, 1>), dim3(nblk), dim3(kGgThreads),
                         0, st, p);
      break;
    case 2:
      hipLaunchKernelGGL((grouped_gemm_kernel<MODE, BK, FP8, EPI, OUTF32, 2>), dim3(nblk), dim3(kGgThreads),
                         0, st, p);
      break;
    case 3:
      hipLaunchKernelGGL((grouped_gemm_kernel<MODE, BK, FP8, EPI, OUTF32, 3>), dim3(nblk), dim3(kGgThreads),
                         0, st, p);
      break;
    case 4:
      hipLaunchKernelGGL((grouped_gemm_kernel<MODE, BK, FP8, EPI, OUTF32, 4>), dim3(nblk), dim3(kGgThreads),
                         0, st, p);
      break;
    default:
      hipLaunchKernelGGL((grouped_gemm_kernel<MODE, BK, FP8, EPI, OUTF32, 0>), dim3(nblk), dim3(kGgThreads),
                         0, st, p);
  }
}

// kind: 0 fwd (A rows . W_g^T), 1 fwd + SwiGLU epilogue, 2 dgrad (dY . W_g), 3 dgrad + SwiGLU
// backward epilogue, 4 wgrad (dW_g (+)= dY_g^T X_g)
void launch_grouped_gemm(GGParams p, int kind, bool fp8, bool out_f32, int64_t total_rows,
                         hipStream_t st) {
  if (kind <= 3) {
    // upper bound on M tiles over all groups: ceil(total/256) + G
    p.tiles_m = static_cast<int>((total_rows + 255) / 256) + p.G;
    p.tiles_n = (kind == 1) ? p.F / 128 : (p.N + 255) / 256;
    const int nblk = p.tiles_m * ((p.tiles_n + kGgNGroup - 1) / kGgNGroup) * kGgNGroup;
    if (nblk == 0) return;
    switch (kind) {
      case 0:
        if (fp8) gg_launch<kMVar, true, true, kEpiStore, false>(p, nblk, st);
        else gg_launch<kMVar, true, false, kEpiStore, false>(p, nblk, st);
        break;
      case 1:
        if (fp8) gg_launch<kMVar, true, true, kEpiSwigluFwd, false>(p, nblk, st);
        else gg_launch<kMVar, true, false, kEpiSwigluFwd, false>(p, nblk, st);
        break;
      case 2:
        gg_launch<kMVar, false, false, kEpiStore, false>(p, nblk, st);
        break;
      default:
        gg_launch<kMVar, false, false, kEpiSwigluBwd, false>(p, nblk, st);
        break;
    }
  } else {
    p.tiles_m = (p.M + 255) / 256;
    p.tiles_n = (p.N + 255) / 256;
    const int nblk = p.G * p.tiles_m * ((p.tiles_n + kGgNGroup - 1) / kGgNGroup) * kGgNGroup;
    if (nblk == 0) return;
    if (out_f32) gg_launch<kKVar, false, false, kEpiStore, true>(p, nblk, st);
    else gg_launch<kKVar, false, false, kEpiStore, false>(p, nblk, st);
  }
}

}  // namespace dla
