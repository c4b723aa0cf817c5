// Persistent decode "layer tail" (B <= 16 rows, Llama-family decoder layer): the o projection,
// the gate|up projection with SwiGLU, the down projection and the NEXT layer's qkv projection as
// ONE launch of one 512-thread workgroup per CU, instead of four dependent launches
// (RLHF rollouts / teacher generation; reference src/training/train_rlhf.py:123-124).
//
// Why: a decode step streams every weight once (473 MB per Llama-3-8B layer at B = 8) and each
// launch of the four-launch chain pays its own ramp (the first HBM round trip with the CU idle)
// and drain (the last workgroups finishing alone) -- ~24 us of the 103 us per layer
// (profiles/r4_decode.md). Here the weights of the NEXT phase do not depend on this phase's
// output, so every workgroup issues its first weight fragments of phase p+1 BEFORE it waits for the
// other workgroups to finish phase p: the HBM stream continues through the phase boundary.
//
// Phases (tiles of 16 output columns; the weights in the tiled layout [N/16, K/32, 4, 16, 8] of
// ops/decode.py, RMSNorm weights folded in):
//   O    s  = x + a Wo^T, row sums of squares of s per tile        8 waves split K per tile
//   GU   m  = SwiGLU(rstd(s) (s * ln2) Wgu^T)                       one wave per tile (interleaved
//                                                                    8 gate + 8 up rows), full K,
//                                                                    s staged in LDS
//   DOWN x' = s + m Wd^T, row sums of squares of x' per tile        8 waves split K per tile
//   QKV  qkv' = rstd(x') (x' * ln1') Wqkv'^T  (next layer; optional) 8 waves split K per tile
// Every phase keeps the arithmetic of the corresponding standalone kernel (csrc/skinny_ks.h
// ks_body: wave w sums k in [w K/8, (w+1) K/8) in order and the 8 partials are added in wave
// order; the GU tile sums k in order, csrc/skinny.hip skinny_glu_il_kernel), so the launch is
// bitwise equal to the four-launch fused decode layer.
//
// Hand-offs inside the launch (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md "Valid
// forms", replicated-counter row): every handed-off value (s, its row partials, m, x', x' row
// partials) is stored write-through (`sc1`, 4-byte pairs); every storing wave drains
// (`s_waitcnt vmcnt(0)`) and the workgroup barrier precedes ONE wave instruction that adds 1 to each
// of the 8 replicas of the phase counter; a consumer polls ONE replica with relaxed `sc1` loads
// (+ s_sleep) and, after a workgroup barrier, reads the handed-off bytes ONLY with `sc1` loads
// (16-byte buffer loads with aux 16, or 4-byte agent-scope atomic loads). Counters are monotonic
// within a generation: decode step k (kv_len = len_first + k - 1) waits for nwg * k arrivals; the
// KV cache zeroes them at every prefill. Every workgroup is resident (one per CU, checked on the
// host), so a wait cannot deadlock; a wait beyond ~2^22 polls sets `err` and proceeds.
#include "common.h"
#include "decode_tail.h"
#include "skinny_ks.h"

namespace dla {

namespace {

constexpr int kTlRep = 8;          // replicas of each phase counter
constexpr int kTlRepStride = 32;   // ints between replicas (one 128-byte line each)
constexpr int kTlUnr = 4;          // k-steps (32) per ring slot
constexpr int kTlChunk = 32 * kTlUnr;

typedef unsigned int tl_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned int tl_gu32;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tl_rsrc(const void* p) {
  // raw buffer, stride 0, num_records bytes (offsets stay < 2 GB), gfx9 dword3
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7FFFFFFF, 0x00020000);
}

// 16-byte `sc1` load (bypasses the CU's L1: device-coherent after the counter hand-off)
__device__ __forceinline__ s16x8 tl_ld16_sc1(__amdgpu_buffer_rsrc_t r, int64_t elem_off) {
  return __builtin_bit_cast(s16x8, __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(elem_off * 2), 0, 16));
}

__device__ __forceinline__ uint32_t tl_ld4_sc1(const void* p) {
  return __hip_atomic_load((const tl_gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void tl_st4_sc1(void* p, uint32_t v) {
  __hip_atomic_store((tl_gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

template <int RO, int RG, int RD, bool NT>
__global__ __launch_bounds__(512) void decode_tail_kernel(TailArgs A) {
  extern __shared__ __attribute__((aligned(16))) bf16_t tl_xs[];  // GU: s [M][H + 8]
  __shared__ float red[8][4][64];
  __shared__ float rstd_s[16];
  __shared__ float sqs[16][16];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int M = A.M, H = A.H;
  const bool arow = r < M;
  const int target = nwg * (A.kv_len[0] - A.len_first[0] + 1);
  // debug stamps (100 MHz constant clock): 0 start, 1 O done, 2 O released, 3 GU done, 4 GU
  // released, 5 DOWN done, 6 DOWN released, 7 end
  auto stamp = [&](int i) {
    if (A.stamps != nullptr && threadIdx.x == 0) A.stamps[bid * 8 + i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  // ------------------------------------------------------------------ hand-off
  auto arrive = [&](int j) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its sc1 stores drained
    __syncthreads();
    if (threadIdx.x < kTlRep)
      __hip_atomic_fetch_add((tl_gu32*)(A.cnt + (j * kTlRep + threadIdx.x) * kTlRepStride), 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  };
  auto wait = [&](int j) {
    if (threadIdx.x == 0) {
      const int* rep = A.cnt + (j * kTlRep + bid % kTlRep) * kTlRepStride;
      int spins = 0;
      while (static_cast<int>(tl_ld4_sc1(rep)) < target) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1 << 22)) {
          tl_st4_sc1(A.err, 1u);
          break;
        }
      }
    }
    __syncthreads();
  };

  // ------------------------------------------------------------------ weight streams
  // W fragment row of (tile bx, this wave) in the tiled layout: k-step s (32 k) at + s * 512
  auto wrow_of = [&](const bf16_t* W, int bx, int K) {
    const int k0 = wave * (K >> 3);
    return W + static_cast<int64_t>(bx) * 16 * K + (k0 >> 5) * 512 + lane * 8;
  };
  // LDS-DMA prefetch of a wave's first P k-steps into its LDS image (1 KB per k-step, lane-linear:
  // lane l's 16 bytes land at +16 l, exactly where the consumer's ds_read_b128 reads them). Issued
  // right after a phase's arrival, BEFORE the wait: the weight stream keeps HBM busy while the
  // other workgroups finish the phase.
  auto pf_issue = [&](const bf16_t* wrow, bf16_t* pf, int P) {
    for (int s = 0; s < P; ++s)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(wrow + s * 512),
                                       (__attribute__((address_space(3))) void*)(pf + s * 512), 16, 0,
                                       NT ? 2 : 0);
  };
  // the prefetched images are written behind the compiler's back: every wave waits for its own
  // LDS-DMA (vmcnt counts it) before its first ds_read of them
  auto pf_landed = [&]() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
  // (explicit address spaces: a select between an LDS and a global pointer would become ONE flat
  // load without the nt hint)
  auto wfrag = [&](const bf16_t* wrow, const bf16_t* pf, int P, int s) -> s16x8 {
    if (s < P) return *(const __attribute__((address_space(3))) s16x8*)(pf + s * 512 + lane * 8);
    const __attribute__((address_space(1))) bf16x8* g = (const __attribute__((address_space(1))) bf16x8*)(wrow + s * 512);
    if constexpr (NT) return __builtin_bit_cast(s16x8, __builtin_nontemporal_load(g));
    else return __builtin_bit_cast(s16x8, *g);
  };

  // ------------------------------------------------------------------ K-split tile body
  // one 16-column tile: the 8 waves split K, wave w sums its k-steps in order (a ring of RK
  // k-steps of W and x fragments in flight; the first P k-steps of W come from the LDS image);
  // x rows from `xg` (SC1: produced inside this launch); partial of this wave -> red[wave]
  auto ks_tile = [&](auto rk_c, auto sc1_c, const bf16_t* wrow, const bf16_t* pf, int P, int K, const bf16_t* xg,
                     int64_t ldxg) {
    constexpr int RK = decltype(rk_c)::value;
    constexpr bool SC1 = decltype(sc1_c)::value;
    const int kw = K >> 3, k0 = wave * kw, nks = kw >> 5;
    const __amdgpu_buffer_rsrc_t xr = tl_rsrc(xg);
    const int64_t xoff = static_cast<int64_t>(arow ? r : 0) * ldxg + k0 + q * 8;
    s16x8 b[RK], a[RK];
    auto load = [&](int j, int st) {
      b[j] = wfrag(wrow, pf, P, st);
      a[j] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (arow) {
        const int64_t o = xoff + st * 32;
        a[j] = SC1 ? tl_ld16_sc1(xr, o) : __builtin_bit_cast(s16x8, load_bf16x8(xg + o));
      }
    };
#pragma unroll
    for (int j = 0; j < RK; ++j)
      if (j < nks) load(j, j);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < nks; s0 += RK) {
#pragma unroll
      for (int j = 0; j < RK; ++j) {
        const int st = s0 + j;
        if (st < nks) {
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], b[j], acc, 0, 0, 0);
          if (st + RK < nks) load(j, st + RK);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][i][lane] = acc[i];
    __syncthreads();
  };
  // epilogue of a K-split tile: 128 threads, two adjacent columns each (4-byte sc1 stores)
  // RES: y = bf16(bf16(acc) + res), row partials of y^2 over the tile's 16 columns -> ssq[m][bx]
  auto epi_res = [&](int bx, const bf16_t* res, int64_t ldr, bool res_sc1, bf16_t* y, int64_t ldy, float* ssq,
                     int nblk, bool out_sc1) {
    if (threadIdx.x < 128) {
      const int e = threadIdx.x;
      const int ti = e >> 5, l = (e & 31) * 2;
      const int mm = 4 * (l >> 4) + ti, n = bx * 16 + (l & 15);
      float t0 = 0.f, t1 = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        t0 += red[w][ti][l];
        t1 += red[w][ti][l + 1];
      }
      if (mm < M) {
        const uint32_t rp = res_sc1 ? tl_ld4_sc1(res + mm * ldr + n)
                                    : *reinterpret_cast<const uint32_t*>(res + mm * ldr + n);
        const float s0 = bf2f(f2bf(bf2f(f2bf(t0)) + bf2f(static_cast<bf16_t>(rp & 0xffffu))));
        const float s1 = bf2f(f2bf(bf2f(f2bf(t1)) + bf2f(static_cast<bf16_t>(rp >> 16))));
        const uint32_t pk = static_cast<uint32_t>(f2bf(s0)) | (static_cast<uint32_t>(f2bf(s1)) << 16);
        if (out_sc1) tl_st4_sc1(y + mm * ldy + n, pk);
        else *reinterpret_cast<uint32_t*>(y + mm * ldy + n) = pk;
        sqs[mm][l & 15] = s0 * s0;
        sqs[mm][(l & 15) + 1] = s1 * s1;
      }
    }
    __syncthreads();
    if (threadIdx.x < M) {
      float t = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) t += sqs[threadIdx.x][c];
      if (out_sc1) tl_st4_sc1(ssq + threadIdx.x * nblk + bx, __float_as_uint(t));
      else ssq[threadIdx.x * nblk + bx] = t;
    }
  };
  // NIN: y = bf16(acc * rstd[m]) (plain stores: read by the next launch)
  auto epi_nin = [&](int bx, bf16_t* y, int64_t ldy) {
    if (threadIdx.x < 128) {
      const int e = threadIdx.x;
      const int ti = e >> 5, l = (e & 31) * 2;
      const int mm = 4 * (l >> 4) + ti, n = bx * 16 + (l & 15);
      float t0 = 0.f, t1 = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        t0 += red[w][ti][l];
        t1 += red[w][ti][l + 1];
      }
      if (mm < M) {
        const float rs = rstd_s[mm];
        *reinterpret_cast<uint32_t*>(y + mm * ldy + n) =
            static_cast<uint32_t>(f2bf(t0 * rs)) | (static_cast<uint32_t>(f2bf(t1 * rs)) << 16);
      }
    }
    __syncthreads();  // red is rewritten by the next tile
  };
  // rstd per row from [16][nbp] partials handed off in this launch (sc1 loads): the ks_part_load /
  // ks_rstd order (lane-strided in-lane sum, then the butterfly)
  auto rstd_from = [&](const float* ssq, int nbp, int K) {
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int mm = 2 * wave + rr;
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = lane + 64 * j;
        t += (mm < M && i < nbp) ? __uint_as_float(tl_ld4_sc1(ssq + mm * nbp + i)) : 0.f;
      }
      t = wave_sum(t);
      if (lane == 0 && mm < M) rstd_s[mm] = rsqrtf(t / static_cast<float>(K) + A.eps);
    }
  };

  const int nt_h = H >> 4;  // O / DOWN tiles
  // ================================================================== O
  for (int bx = bid; bx < nt_h; bx += nwg) {
    ks_tile(std::integral_constant<int, RO>{}, std::false_type{}, wrow_of(A.Wo, bx, A.Ko), nullptr, 0, A.Ko, A.a,
            A.lda);
    epi_res(bx, A.x, A.ldx, false, A.s, H, A.ssq_s, nt_h, true);
    __syncthreads();
  }
  stamp(1);
  arrive(0);
  // ================================================================== GU
  const int nt_g = A.F >> 3;  // interleaved tiles of 16 rows (8 gate + 8 up)
  const int tpw = (nt_g + nwg - 1) / nwg;
  const int g0 = bid * tpw, g1 = min(nt_g, g0 + tpw);
  const int ss = ((M * (H + 8) * 2 + 15) & ~15) / 2;  // s staging, elements
  {
    const int nks = H >> 5;
    const int PG = min(A.pg, nks);
    bf16_t* pf = tl_xs + ss + wave * PG * 512;
    int t = g0 + wave;
    if (t < g1) pf_issue(A.Wgu + static_cast<int64_t>(t) * 16 * H + lane * 8, pf, PG);  // before the wait
    wait(0);
    stamp(2);
    // stage s [M, H] in LDS (sc1 16-byte loads), rstd per row from the O phase's partials
    const int ldl = H + 8, vecs = H >> 3, total = M * vecs;
    const __amdgpu_buffer_rsrc_t sr = tl_rsrc(A.s);
    for (int i = threadIdx.x; i < total; i += 512) {
      const int mm = i / vecs, c = (i - mm * vecs) << 3;
      *reinterpret_cast<s16x8*>(tl_xs + mm * ldl + c) = tl_ld16_sc1(sr, static_cast<int64_t>(mm) * H + c);
    }
    rstd_from(A.ssq_s, nt_h, H);
    pf_landed();
    __syncthreads();
    const bf16_t* xrow = tl_xs + r * ldl + q * 8;
    constexpr int RK = RG;
    for (int P = PG; t < g1; t += 8, P = 0) {
      const bf16_t* wr = A.Wgu + static_cast<int64_t>(t) * 16 * H + lane * 8;
      s16x8 b[RK];
#pragma unroll
      for (int j = 0; j < RK; ++j)
        if (j < nks) b[j] = wfrag(wr, pf, P, j);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int s0 = 0; s0 < nks; s0 += RK) {
#pragma unroll
        for (int j = 0; j < RK; ++j) {
          const int st = s0 + j;
          if (st < nks) {
            s16x8 av = {0, 0, 0, 0, 0, 0, 0, 0};
            if (arow) av = *(const __attribute__((address_space(3))) s16x8*)(xrow + st * 32);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b[j], acc, 0, 0, 0);
            if (st + RK < nks) b[j] = wfrag(wr, pf, P, st + RK);
          }
        }
      }
      // lane holds C[m = 4q + i][tile row r]: gate (r < 8) / up (r >= 8) of feature 8t + (r & 7)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mm = 4 * q + i;
        const float v = bf2f(f2bf(acc[i] * (mm < M ? rstd_s[mm] : 0.f)));
        const float o = __shfl_xor(v, 8, 64);
        const uint32_t y = f2bf(silu_sk(v) * o);
        const uint32_t yn = __shfl_xor(y, 1, 64);  // the neighbouring feature
        if (r < 8 && (r & 1) == 0 && mm < M) tl_st4_sc1(A.m + mm * A.F + 8 * t + r, y | (yn << 16));
      }
    }
  }
  stamp(3);
  arrive(1);
  // ================================================================== DOWN
  {
    const int PD = min(A.pd, (A.F >> 3) >> 5);
    bf16_t* pf = tl_xs + wave * PD * 512;
    if (bid < nt_h) pf_issue(wrow_of(A.Wd, bid, A.F), pf, PD);  // before the wait
    wait(1);
    stamp(4);
    pf_landed();
    for (int bx = bid, P = PD; bx < nt_h; bx += nwg, P = 0) {
      ks_tile(std::integral_constant<int, RD>{}, std::true_type{}, wrow_of(A.Wd, bx, A.F), pf, P, A.F, A.m, A.F);
      epi_res(bx, A.s, H, true, A.xo, H, A.ssq_x, nt_h, A.Wq != nullptr);
      __syncthreads();
    }
  }
  stamp(5);
  if (A.Wq == nullptr) return;
  arrive(2);
  // ================================================================== QKV (next layer)
  {
    const int nt_q = A.Nq >> 4;
    const int PQ = min(A.pq, (H >> 3) >> 5);
    bf16_t* pf = tl_xs + wave * PQ * 512;
    if (bid < nt_q) pf_issue(wrow_of(A.Wq, bid, H), pf, PQ);  // before the wait
    wait(2);
    stamp(6);
    rstd_from(A.ssq_x, nt_h, H);
    pf_landed();
    __syncthreads();
    for (int bx = bid, P = PQ; bx < nt_q; bx += nwg, P = 0) {
      ks_tile(std::integral_constant<int, RO>{}, std::true_type{}, wrow_of(A.Wq, bx, H), pf, P, H, A.xo, H);
      epi_nin(bx, A.qkv, A.Nq);
    }
  }
  stamp(7);
}

// workgroups resident at once (one per CU expected), per instantiation and LDS size
template <int RO, int RG, int RD, bool NT>
static int tail_capacity(int lds) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_tail_kernel<RO, RG, RD, NT>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, decode_tail_kernel<RO, RG, RD, NT>, 512, lds) !=
      hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return per >= 1 ? cus : 0;  // ONE workgroup per CU: every one resident
}

constexpr int kTlLdsBudget = 144 * 1024;  // dynamic LDS (static ~9.3 KB: red, sqs, rstd)

// false: shape not supported (nothing launched). Fills the prefetch depths (k-steps per wave)
// from the LDS budget: GU next to the s staging, DOWN / QKV alone.
bool launch_decode_tail(const TailArgs& Ain, hipStream_t st) {
  TailArgs A = Ain;
  const int ss = (A.M * (A.H + 8) * 2 + 15) & ~15;
  if (A.M < 1 || A.M > 16 || A.H % 1024 || A.Ko % 1024 || A.F % 1024 || A.Nq % 16 || ss > kTlLdsBudget - 8 * 1024)
    return false;
  static const int pf_env = [] {  // DLA_TAIL_PF=0: no LDS prefetch (A/B)
    const char* e = std::getenv("DLA_TAIL_PF");
    return e ? std::atoi(e) : 1;
  }();
  const int kstep_all = 8 * 1024;  // one k-step of every wave
  A.pg = pf_env ? std::min(A.H / 32, (kTlLdsBudget - ss) / kstep_all) : 0;
  A.pd = pf_env ? std::min(A.F / 256, kTlLdsBudget / kstep_all) : 0;
  A.pq = pf_env ? std::min(A.H / 256, kTlLdsBudget / kstep_all) : 0;
  const int lds = std::max({ss + A.pg * kstep_all, A.pd * kstep_all, A.pq * kstep_all, ss});
  static int cap = -1;
  if (cap < 0) cap = tail_capacity<8, 16, 16, true>(kTlLdsBudget);
  if (cap <= 0) return false;
  decode_tail_kernel<8, 16, 16, true><<<cap, 512, lds, st>>>(A);
  return true;
}

int decode_tail_grid() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return cus;
}

}  // namespace dla
