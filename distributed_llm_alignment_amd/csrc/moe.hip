// Mixture-of-experts routing / permutation kernels (HF Mixtral semantics,
// transformers/models/mixtral/modeling_mixtral.py sparse MoE block: softmax -> top-k ->
// renormalise -> dispatch -> expert SwiGLU -> weighted combine).
//
// Layout: token-slot (t, j) (j < k) is sent to row pos[t, j] of the expert-sorted activation
// matrix xs [N*k, H] (rows of one expert contiguous, experts in order; under expert parallelism
// experts of one destination rank are contiguous too, so the all-to-all payload needs no extra
// copy). Every kernel is a GATHER over that map — no atomics, deterministic:
//   dispatch  : xs[pos[t,j]]  = x[t]                        (forward permute)
//   combine   : out[t]        = sum_j w[t,j] * ys[pos[t,j]]  (forward un-permute + weighting;
//                                                             with w = 1: dispatch backward)
//   combine_bwd: dys[pos[t,j]] = w[t,j] * dout[t],  dw[t,j] = <dout[t], ys[pos[t,j]]>
// Router: the renormalised top-k softmax equals a softmax over the selected logits, so the
// forward needs one pass over E logits per token and the backward touches only k of them.
#include <cstdlib>

#include "common.h"

namespace dla {

constexpr int kMaxK = 8;

// one thread per token; E <= 256 logits read twice from L1/L2 (E * 2 B per token)
__global__ __launch_bounds__(256) void moe_topk_fwd_kernel(const bf16_t* __restrict__ logits,
                                                            int64_t N, int E, int k,
                                                            float* __restrict__ topv,
                                                            int* __restrict__ topi) {
  const int64_t t = blockIdx.x * 256ll + threadIdx.x;
  if (t >= N) return;
  const bf16_t* row = logits + t * E;
  float v[kMaxK];
  int id[kMaxK];
#pragma unroll
  for (int j = 0; j < kMaxK; ++j) {
    v[j] = -INFINITY;
    id[j] = -1;
  }
  for (int e = 0; e < E; ++e) {
    const float x = bf2f(row[e]);
    // insertion into the descending top-k list; ties keep the lower expert index first
    if (x > v[k - 1] || id[k - 1] < 0) {
      int p = k - 1;
      while (p > 0 && (x > v[p - 1] || id[p - 1] < 0)) {
        v[p] = v[p - 1];
        id[p] = id[p - 1];
        --p;
      }
      v[p] = x;
      id[p] = e;
    }
  }
  float s = 0.f;
  float ex[kMaxK];
#pragma unroll
  for (int j = 0; j < kMaxK; ++j) {
    ex[j] = j < k ? __expf(v[j] - v[0]) : 0.f;
    s += ex[j];
  }
  const float inv = 1.f / s;
  for (int j = 0; j < k; ++j) {
    topv[t * k + j] = ex[j] * inv;
    topi[t * k + j] = id[j];
  }
}

// dlogits[t, e] = topv*(g - <g, topv>) on the k selected experts, 0 elsewhere
__global__ __launch_bounds__(256) void moe_topk_bwd_kernel(const float* __restrict__ topv,
                                                            const int* __restrict__ topi,
                                                            const float* __restrict__ g,
                                                            int64_t N, int E, int k,
                                                            bf16_t* __restrict__ dlogits) {
  const int64_t t = blockIdx.x * 256ll + threadIdx.x;
  if (t >= N) return;
  bf16_t* row = dlogits + t * E;
  for (int e = 0; e < E; ++e) row[e] = 0;
  float dot = 0.f;
  for (int j = 0; j < k; ++j) dot += g[t * k + j] * topv[t * k + j];
  for (int j = 0; j < k; ++j) {
    const float p = topv[t * k + j];
    row[topi[t * k + j]] = f2bf(p * (g[t * k + j] - dot));
  }
}

// block per token; 16-byte vectors over H
__global__ __launch_bounds__(256) void moe_dispatch_kernel(const bf16_t* __restrict__ x,
                                                            const int* __restrict__ pos,
                                                            int64_t N, int H, int k,
                                                            bf16_t* __restrict__ xs) {
  const int64_t t = blockIdx.x;
  const bf16_t* src = x + t * H;
  int p[kMaxK];
  for (int j = 0; j < k; ++j) p[j] = pos[t * k + j];
  for (int i = threadIdx.x; i < H / 8; i += 256) {
    const bf16x8 a = load_bf16x8(src + i * 8);
    for (int j = 0; j < k; ++j) store_bf16x8(xs + (int64_t)p[j] * H + i * 8, a);
  }
}

template <bool HAS_W>
__global__ __launch_bounds__(256) void moe_combine_kernel(const bf16_t* __restrict__ ys,
                                                           const int* __restrict__ pos,
                                                           const float* __restrict__ w,
                                                           int64_t N, int H, int k, int64_t R,
                                                           bf16_t* __restrict__ out) {
  // rows p >= R read as zero (dropped slots of a capacity buffer: no appended zero row needed)
  const int64_t t = blockIdx.x;
  int p[kMaxK];
  float wt[kMaxK];
  for (int j = 0; j < k; ++j) {
    p[j] = pos[t * k + j];
    wt[j] = HAS_W ? w[t * k + j] : 1.f;
  }
  for (int i = threadIdx.x; i < H / 8; i += 256) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      if (p[j] >= R) continue;
      const bf16x8 a = load_bf16x8(ys + (int64_t)p[j] * H + i * 8);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += wt[j] * bf2f(a[q]);
    }
    store_bf16x8(out + t * H + i * 8, pack_bf16x8(acc));
  }
}

__global__ __launch_bounds__(256) void moe_combine_bwd_kernel(const bf16_t* __restrict__ dout,
                                                               const bf16_t* __restrict__ ys,
                                                               const int* __restrict__ pos,
                                                               const float* __restrict__ w,
                                                               int64_t N, int H, int k, int64_t R,
                                                               bf16_t* __restrict__ dys,
                                                               float* __restrict__ dw) {
  __shared__ float red[4];
  const int64_t t = blockIdx.x;
  for (int j = 0; j < k; ++j) {
    const int64_t p = pos[t * k + j];
    const float wt = w[t * k + j];
    if (p >= R) {  // a dropped slot (block-uniform): no row, zero weight gradient
      if (threadIdx.x == 0) dw[t * k + j] = 0.f;
      continue;
    }
    float dot = 0.f;
    for (int i = threadIdx.x; i < H / 8; i += 256) {
      const bf16x8 g = load_bf16x8(dout + t * H + i * 8);
      const bf16x8 y = load_bf16x8(ys + p * H + i * 8);
      float o[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float gq = bf2f(g[q]);
        dot += gq * bf2f(y[q]);
        o[q] = wt * gq;
      }
      store_bf16x8(dys + p * H + i * 8, pack_bf16x8(o));
    }
    const float s = block_sum<256>(dot, red);
    if (threadIdx.x == 0) dw[t * k + j] = s;
  }
}

// Row-wise e4m3 quantisation for the fp8 MFMA GEMMs (hipBLASLt row-wise scaled fp8):
// q[r, :] = sat(x[r, :] * 448 / amax_r) as OCP e4m3fn (gfx950 v_cvt_pk_fp8_f32), inv[r] =
// amax_r / 448. One 256-thread block per row: the row is read twice (amax, then convert) and
// stays in L1/L2 between the passes; no intermediate fp32 copy.
__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(const bf16_t* __restrict__ x,
                                                              int64_t ld, int K,
                                                              uint8_t* __restrict__ q,
                                                              float* __restrict__ inv) {
  __shared__ float red[4];
  const int64_t r = blockIdx.x;
  const bf16_t* row = x + r * ld;
  float m = 0.f;
  for (int i = threadIdx.x; i < K / 8; i += 256) {
    const bf16x8 a = load_bf16x8(row + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(bf2f(a[j])));
  }
  m = block_max<256>(m, red);
  const float amax = fmaxf(m, 1e-12f);
  const float sc = 448.f / amax;
  if (threadIdx.x == 0) inv[r] = amax / 448.f;
  uint8_t* qrow = q + r * (int64_t)K;
  for (int i = threadIdx.x; i < K / 8; i += 256) {
    const bf16x8 a = load_bf16x8(row + i * 8);
    uint32_t lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(a[0]) * sc, bf2f(a[1]) * sc, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(a[2]) * sc, bf2f(a[3]) * sc, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(a[4]) * sc, bf2f(a[5]) * sc, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(a[6]) * sc, bf2f(a[7]) * sc, hi, true);
    *reinterpret_cast<uint2*>(qrow + i * 8) = make_uint2(lo, hi);
  }
}

// Single-pass form for rows of <= 256 * 8 * NV elements: the row stays in registers between the
// amax reduction and the conversion (the two-pass kernel above re-reads it), all NV loads of a
// thread in flight at once. Same arithmetic and reduction, so the same bits.
template <int NV>
__global__ __launch_bounds__(256) void quant_fp8_rows_reg_kernel(const bf16_t* __restrict__ x,
                                                                 int64_t ld, int K,
                                                                 uint8_t* __restrict__ q,
                                                                 float* __restrict__ inv) {
  __shared__ float red[4];
  const int64_t r = blockIdx.x;
  const bf16_t* row = x + r * ld;
  const int nv = K / 8;
  bf16x8 a[NV];
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i = threadIdx.x + u * 256;
    if (i < nv) a[u] = load_bf16x8(row + i * 8);
  }
  float m = 0.f;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i = threadIdx.x + u * 256;
    if (i < nv) {
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(bf2f(a[u][j])));
    }
  }
  m = block_max<256>(m, red);
  const float amax = fmaxf(m, 1e-12f);
  const float sc = 448.f / amax;
  if (threadIdx.x == 0) inv[r] = amax / 448.f;
  uint8_t* qrow = q + r * (int64_t)K;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i = threadIdx.x + u * 256;
    if (i < nv) {
      uint32_t lo = 0, hi = 0;
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(a[u][0]) * sc, bf2f(a[u][1]) * sc, lo, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(a[u][2]) * sc, bf2f(a[u][3]) * sc, lo, true);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(a[u][4]) * sc, bf2f(a[u][5]) * sc, hi, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(a[u][6]) * sc, bf2f(a[u][7]) * sc, hi, true);
      *reinterpret_cast<uint2*>(qrow + i * 8) = make_uint2(lo, hi);
    }
  }
}

void launch_quant_fp8_rows(const bf16_t* x, int64_t ld, int64_t rows, int K, uint8_t* q, float* inv,
                           hipStream_t st) {
  if (rows == 0) return;
  // DLA_FP8_QUANT_2PASS=1: the two-pass kernel (A/B)
  static const bool two_pass = [] {
    const char* e = getenv("DLA_FP8_QUANT_2PASS");
    return e != nullptr && e[0] == '1';
  }();
  const int nv = K / 8;
  if (!two_pass && nv <= 256)
    quant_fp8_rows_reg_kernel<1><<<rows, 256, 0, st>>>(x, ld, K, q, inv);
  else if (!two_pass && nv <= 512)
    quant_fp8_rows_reg_kernel<2><<<rows, 256, 0, st>>>(x, ld, K, q, inv);
  else if (!two_pass && nv <= 1024)
    quant_fp8_rows_reg_kernel<4><<<rows, 256, 0, st>>>(x, ld, K, q, inv);
  else if (!two_pass && nv <= 2048)
    quant_fp8_rows_reg_kernel<8><<<rows, 256, 0, st>>>(x, ld, K, q, inv);
  else
    quant_fp8_rows_kernel<<<rows, 256, 0, st>>>(x, ld, K, q, inv);
}

// ----------------------------------------------------------------------------------------------
void launch_moe_topk_fwd(const bf16_t* logits, int64_t N, int E, int k, float* topv, int* topi,
                         hipStream_t st) {
  if (N == 0) return;
  moe_topk_fwd_kernel<<<(N + 255) / 256, 256, 0, st>>>(logits, N, E, k, topv, topi);
}
void launch_moe_topk_bwd(const float* topv, const int* topi, const float* g, int64_t N, int E,
                         int k, bf16_t* dlogits, hipStream_t st) {
  if (N == 0) return;
  moe_topk_bwd_kernel<<<(N + 255) / 256, 256, 0, st>>>(topv, topi, g, N, E, k, dlogits);
}
void launch_moe_dispatch(const bf16_t* x, const int* pos, int64_t N, int H, int k, bf16_t* xs,
                         hipStream_t st) {
  if (N == 0) return;
  moe_dispatch_kernel<<<N, 256, 0, st>>>(x, pos, N, H, k, xs);
}
// ---------------------------------------------------------------------------------------------
// Expert-parallel capacity routing (parallel/expert.py `_route_chunk` / `_expert_order`), each
// as ONE single-workgroup launch instead of ~20 small torch ops (argsort, scatters, cumsums):
// the EP step launched ~160 kernels per layer and pass, most of them these.
//
// ep_route: slot s = (token t, choice j) of expert e = topi[t, j], destination d = e / El.
// Ranks are stable (slot order) within each expert: slots go through in 64-slot batches, one
// ballot per expert per batch; pass 1 counts per (batch, expert) into LDS, a per-expert scan over
// the batches gives each batch's base, pass 2 ranks. Then, as the torch form: the slot's offset
// in its destination's expert-sorted block, kept if < C, its send row d * C + off (else the
// dropped row ep * C), send_src[row] = t (-1 where empty), the rows actually sent per
// (destination, local expert), and the dropped count added to a device counter.
constexpr int kRouteThreads = 1024;
constexpr int kRouteMaxE = 64;
constexpr int kRouteMaxBatches = 256;  // 16384 slots per chunk (host-checked)

template <typename TI>
__global__ __launch_bounds__(kRouteThreads) void ep_route_kernel(
    const TI* __restrict__ topi, int S, int k, int E, int El, int ep, int C,
    int64_t* __restrict__ send_src, int* __restrict__ pos, int* __restrict__ sent,
    int64_t* __restrict__ dropped) {
  __shared__ int bcnt[kRouteMaxBatches][kRouteMaxE];  // (batch, expert) counts -> bases
  __shared__ int ecnt[kRouteMaxE], ecum[kRouteMaxE + 1];
  __shared__ int ndrop;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = kRouteThreads / 64;
  const int nb = (S + 63) / 64;
  for (int i = tid; i < ep * C; i += kRouteThreads) send_src[i] = -1;
  if (tid == 0) ndrop = 0;
  // pass 1: per-batch counts
  for (int b = wv; b < nb; b += nw) {
    const int s = b * 64 + lane;
    const int e = s < S ? static_cast<int>(topi[s]) : -1;
    for (int x = 0; x < E; ++x) {
      const uint64_t m = __ballot(e == x);
      if (lane == 0) bcnt[b][x] = __popcll(m);
    }
  }
  __syncthreads();
  // per-expert exclusive scan over the batches (one thread per expert)
  if (tid < E) {
    int run = 0;
    for (int b = 0; b < nb; ++b) {
      const int c = bcnt[b][tid];
      bcnt[b][tid] = run;
      run += c;
    }
    ecnt[tid] = run;
  }
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int x = 0; x < E; ++x) {
      ecum[x] = run;
      run += ecnt[x];
    }
    ecum[E] = run;
  }
  __syncthreads();
  // sent rows per (destination, local expert): the first C of each destination block in order
  for (int i = tid; i < E; i += kRouteThreads) {
    const int d = i / El;
    const int before = ecum[i] - ecum[d * El];
    sent[i] = min(max(C - before, 0), ecnt[i]);
  }
  // pass 2: ranks -> positions
  for (int b = wv; b < nb; b += nw) {
    const int s = b * 64 + lane;
    const int e = s < S ? static_cast<int>(topi[s]) : -1;
    int rank = 0;
    for (int x = 0; x < E; ++x) {
      const uint64_t m = __ballot(e == x);
      if (e == x) rank = bcnt[b][x] + __popcll(m & ((1ull << lane) - 1ull));
    }
    if (s < S) {
      const int d = e / El;
      const int off = ecum[e] + rank - ecum[d * El];
      int p;
      if (off < C) {
        p = d * C + off;
        send_src[p] = s / k;
      } else {
        p = ep * C;
        atomicAdd(&ndrop, 1);
      }
      pos[s] = p;
    }
  }
  __syncthreads();
  if (tid == 0 && ndrop > 0) dropped[0] += ndrop;
}

// ep_expert_order (receiver): rc [ep, El] rows received per (source, local expert), each source's
// block local-expert sorted. Row j < C of source s: its local expert e (first with j < the
// inclusive prefix of rc[s]), its index in that run, and its expert-major position q = (rows of
// experts < e over all sources) + (rows of expert e from sources < s) + index. Outputs
// xe_src[q] = s * C + j (-1 where no row), inv[s * C + j] = q (-1 past the source's rows), and
// the grouped-GEMM offsets offs[El + 1].
__global__ __launch_bounds__(kRouteThreads) void ep_expert_order_kernel(
    const int* __restrict__ rc, int ep, int El, int C, int64_t* __restrict__ xe_src,
    int64_t* __restrict__ inv, int* __restrict__ offs) {
  __shared__ int cum_s[64][kRouteMaxE + 1];  // per source: exclusive prefix over local experts
  __shared__ int start_es[kRouteMaxE][64];   // expert-major start of (e, s)
  __shared__ int tot_s[64];
  const int tid = threadIdx.x;
  for (int i = tid; i < ep * C; i += kRouteThreads) xe_src[i] = -1;
  if (tid < ep) {
    int run = 0;
    for (int e = 0; e < El; ++e) {
      cum_s[tid][e] = run;
      run += rc[tid * El + e];
    }
    cum_s[tid][El] = run;
    tot_s[tid] = run;
  }
  if (tid == 0) {
    int run = 0;
    offs[0] = 0;
    for (int e = 0; e < El; ++e) {
      for (int s2 = 0; s2 < ep; ++s2) {
        start_es[e][s2] = run;
        run += rc[s2 * El + e];
      }
      offs[e + 1] = run;
    }
  }
  __syncthreads();
  for (int i = tid; i < ep * C; i += kRouteThreads) {
    const int s2 = i / C, j = i % C;
    if (j >= tot_s[s2]) {
      inv[i] = -1;
      continue;
    }
    int e = 0;
    while (e + 1 < El && j >= cum_s[s2][e + 1]) ++e;
    const int q = start_es[e][s2] + (j - cum_s[s2][e]);
    inv[i] = q;
    xe_src[q] = i;
  }
}

void launch_ep_route(const void* topi, bool i64, int S, int k, int E, int El, int ep, int C,
                     int64_t* send_src, int* pos, int* sent, int64_t* dropped, hipStream_t st) {
  if (i64)
    ep_route_kernel<int64_t><<<1, kRouteThreads, 0, st>>>(static_cast<const int64_t*>(topi), S, k, E, El, ep,
                                                          C, send_src, pos, sent, dropped);
  else
    ep_route_kernel<int><<<1, kRouteThreads, 0, st>>>(static_cast<const int*>(topi), S, k, E, El, ep, C,
                                                      send_src, pos, sent, dropped);
}

void launch_ep_expert_order(const int* rc, int ep, int El, int C, int64_t* xe_src, int64_t* inv, int* offs,
                            hipStream_t st) {
  ep_expert_order_kernel<<<1, kRouteThreads, 0, st>>>(rc, ep, El, C, xe_src, inv, offs);
}

// Row gather with holes (parallel/expert.py `_gather_rows`): out[i] = idx[i] >= 0 ? x[idx[i]] : 0,
// and its adjoint for an idx injective on its valid entries: dx[idx[i]] = g[i] (dx pre-zeroed).
// One launch each instead of clamp + index_select + where (+ index_add in the backward).
__global__ __launch_bounds__(256) void gather_rows_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                          const int64_t* __restrict__ idx, int H,
                                                          bf16_t* __restrict__ out) {
  const int64_t r = blockIdx.x;
  const int64_t i = idx[r];
  for (int c = threadIdx.x; c < H / 8; c += 256) {
    const bf16x8 v = i >= 0 ? load_bf16x8(x + i * ldx + c * 8) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    store_bf16x8(out + r * H + c * 8, v);
  }
}

__global__ __launch_bounds__(256) void scatter_rows_kernel(const bf16_t* __restrict__ g,
                                                           const int64_t* __restrict__ idx, int H,
                                                           bf16_t* __restrict__ dx) {
  const int64_t r = blockIdx.x;
  const int64_t i = idx[r];
  if (i < 0) return;
  for (int c = threadIdx.x; c < H / 8; c += 256) store_bf16x8(dx + i * H + c * 8, load_bf16x8(g + r * H + c * 8));
}

void launch_gather_rows(const bf16_t* x, int64_t ldx, const int64_t* idx, int64_t n, int H, bf16_t* out,
                        hipStream_t st) {
  if (n == 0) return;
  gather_rows_kernel<<<n, 256, 0, st>>>(x, ldx, idx, H, out);
}

void launch_scatter_rows(const bf16_t* g, const int64_t* idx, int64_t n, int H, bf16_t* dx, hipStream_t st) {
  if (n == 0) return;
  scatter_rows_kernel<<<n, 256, 0, st>>>(g, idx, H, dx);
}

// zero rows [*from, R) of a [R, C] bf16 tensor (C % 8 == 0), the row bound read on the device:
// the unwritten padding rows of a capacity buffer before a GEMM reduces over them
__global__ __launch_bounds__(256) void zero_rows_from_kernel(bf16_t* __restrict__ x, int64_t R, int C,
                                                             int64_t ld, const int* __restrict__ from) {
  const int64_t r0 = from[0];
  const int64_t per_row = C / 8;
  const int64_t n = (R - r0) * per_row;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t r = r0 + i / per_row, c = (i % per_row) * 8;
    store_bf16x8(x + r * ld + c, bf16x8{0, 0, 0, 0, 0, 0, 0, 0});
  }
}

void launch_zero_rows_from(bf16_t* x, int64_t R, int C, int64_t ld, const int* from, hipStream_t st) {
  if (R == 0 || C == 0) return;
  zero_rows_from_kernel<<<1024, 256, 0, st>>>(x, R, C, ld, from);
}

void launch_moe_combine(const bf16_t* ys, const int* pos, const float* w, int64_t N, int H, int k,
                        int64_t R, bf16_t* out, hipStream_t st) {
  if (N == 0) return;
  if (w) moe_combine_kernel<true><<<N, 256, 0, st>>>(ys, pos, w, N, H, k, R, out);
  else moe_combine_kernel<false><<<N, 256, 0, st>>>(ys, pos, w, N, H, k, R, out);
}
void launch_moe_combine_bwd(const bf16_t* dout, const bf16_t* ys, const int* pos, const float* w,
                            int64_t N, int H, int k, int64_t R, bf16_t* dys, float* dw, hipStream_t st) {
  if (N == 0) return;
  moe_combine_bwd_kernel<<<N, 256, 0, st>>>(dout, ys, pos, w, N, H, k, R, dys, dw);
}

}  // namespace dla
