// Fused (residual-add +) RMSNorm / LayerNorm forward and backward for gfx950.
//
// Replaces HF LlamaRMSNorm / nn.LayerNorm: reference call sites are every decoder
// layer of the HF model reached from src/training/train_dpo.py:31-39 / train_sft.py:145.
//
// Layout: rows x H, bf16 I/O, fp32 math. One wave (64 lanes) owns a row; each lane holds NC
// 16-byte chunks (8 bf16) of the row in registers, so the row is read exactly once per pass.
// Residual fusion: s = bf16(x + r) is written out (the new residual stream) and normalised,
// saving a separate elementwise pass in both directions.
#include <stdexcept>
#include "common.h"

namespace dla {

template <int NC, bool RMS, bool HAS_RES, bool HAS_BIAS>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const bf16_t* __restrict__ x,
                                                        const bf16_t* __restrict__ res,
                                                        bf16_t* __restrict__ sum_out,
                                                        const bf16_t* __restrict__ w,
                                                        const bf16_t* __restrict__ b,
                                                        bf16_t* __restrict__ y,
                                                        float* __restrict__ rstd_out,
                                                        float* __restrict__ mean_out, int rows,
                                                        int H, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = H >> 3;
  const size_t base = static_cast<size_t>(row) * H;
  float v[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int vi = c * 64 + lane;
    if (vi < nvec) {
      bf16x8 a = load_bf16x8(x + base + vi * 8);
      if constexpr (HAS_RES) {
        bf16x8 r = load_bf16x8(res + base + vi * 8);
        bf16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] = f2bf(bf2f(a[j]) + bf2f(r[j]));
          v[c][j] = bf2f(s[j]);
        }
        store_bf16x8(sum_out + base + vi * 8, s);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = bf2f(a[j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
  float mean = 0.f;
  if constexpr (!RMS) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[c][j];
    mean = wave_sum(s) / H;
  }
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int vi = c * 64 + lane;
    if (vi < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[c][j] - mean;
        ss += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / H + eps);
  if (lane == 0) {
    rstd_out[row] = rstd;
    if constexpr (!RMS) mean_out[row] = mean;
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int vi = c * 64 + lane;
    if (vi < nvec) {
      bf16x8 wv = load_bf16x8(w + vi * 8);
      bf16x8 bv;
      if constexpr (HAS_BIAS) bv = load_bf16x8(b + vi * 8);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = (v[c][j] - mean) * rstd * bf2f(wv[j]);
        if constexpr (HAS_BIAS) t += bf2f(bv[j]);
        o[j] = f2bf(t);
      }
      store_bf16x8(y + base + vi * 8, o);
    }
  }
}

// Few-row variant (decode: rows = batch): one block per row, one 16-byte chunk per thread
// (blockDim = H/8 rounded to a wave multiple, <= 1024), so a row costs one load round trip
// instead of NC sequential chunks on a single wave.
template <bool RMS, bool HAS_RES, bool HAS_BIAS>
__global__ __launch_bounds__(1024) void norm_fwd_row_kernel(const bf16_t* __restrict__ x,
                                                             const bf16_t* __restrict__ res,
                                                             bf16_t* __restrict__ sum_out,
                                                             const bf16_t* __restrict__ w,
                                                             const bf16_t* __restrict__ b,
                                                             bf16_t* __restrict__ y,
                                                             float* __restrict__ rstd_out,
                                                             float* __restrict__ mean_out, int H,
                                                             float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x, t = threadIdx.x, nw = blockDim.x >> 6;
  const size_t base = static_cast<size_t>(row) * H;
  const bool on = t < (H >> 3);
  float v[8];
  // weight (and bias) requested together with the row: the reduction below then hides their
  // latency instead of paying a second dependent round trip after it (decode rows: ~5 us/call)
  bf16x8 wv, bv;
  if (on) {
    wv = load_bf16x8(w + t * 8);
    if constexpr (HAS_BIAS) bv = load_bf16x8(b + t * 8);
  }
  if (on) {
    bf16x8 a = load_bf16x8(x + base + t * 8);
    if constexpr (HAS_RES) {
      bf16x8 r = load_bf16x8(res + base + t * 8), sm;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sm[j] = f2bf(bf2f(a[j]) + bf2f(r[j]));
        v[j] = bf2f(sm[j]);
      }
      store_bf16x8(sum_out + base + t * 8, sm);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(a[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
  }
  auto bsum = [&](float q) {
    q = wave_sum(q);
    __syncthreads();
    if ((t & 63) == 0) red[t >> 6] = q;
    __syncthreads();
    float r = 0.f;
    for (int i = 0; i < nw; ++i) r += red[i];
    return r;
  };
  float mean = 0.f;
  if constexpr (!RMS) {
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) q += v[j];
    mean = bsum(q) / H;
  }
  float ss = 0.f;
  if (on) {
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += (v[j] - mean) * (v[j] - mean);
  }
  const float rstd = rsqrtf(bsum(ss) / H + eps);
  if (t == 0) {
    rstd_out[row] = rstd;
    if constexpr (!RMS) mean_out[row] = mean;
  }
  if (on) {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float q = (v[j] - mean) * rstd * bf2f(wv[j]);
      if constexpr (HAS_BIAS) q += bf2f(bv[j]);
      o[j] = f2bf(q);
    }
    store_bf16x8(y + base + t * 8, o);
  }
}

// Backward. One 256-thread block owns a row at a time (grid-stride over rows with a fixed
// grid); each thread owns NC fixed 8-column chunks, so its dw/db partials stay in NC*8
// registers across all rows of the block. One fp32 partial row per block ([grid, H]) is then
// folded by norm_wgrad_reduce_kernel. Row reductions: wave shuffle + 4-entry LDS.
template <int NC, bool RMS, bool HAS_DRES, bool HAS_BIAS>
__global__ __launch_bounds__(256) void norm_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s, const bf16_t* __restrict__ w,
    const float* __restrict__ rstd_in, const float* __restrict__ mean_in,
    const bf16_t* __restrict__ dres, bf16_t* __restrict__ ds, float* __restrict__ dw_part,
    float* __restrict__ db_part, int rows, int H) {
  __shared__ float red[2][4], redg[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nvec = H >> 3;
  float dwa[NC][8], dba[NC][8], wf[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int vi = c * 256 + tid;
    bf16x8 wv = vi < nvec ? load_bf16x8(w + vi * 8) : bf16x8{};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dwa[c][j] = dba[c][j] = 0.f;
      wf[c][j] = bf2f(wv[j]);
    }
  }
  int parity = 0;
  for (int row = blockIdx.x; row < rows; row += gridDim.x, parity ^= 1) {
    const size_t base = static_cast<size_t>(row) * H;
    const float rstd = rstd_in[row];
    const float mean = RMS ? 0.f : mean_in[row];
    float xh[NC][8], g[NC][8];
    float sum_g = 0.f, sum_gx = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int vi = c * 256 + tid;
      if (vi < nvec) {
        bf16x8 dv = load_bf16x8(dy + base + vi * 8);
        bf16x8 sv = load_bf16x8(s + base + vi * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = bf2f(dv[j]);
          xh[c][j] = (bf2f(sv[j]) - mean) * rstd;
          g[c][j] = d * wf[c][j];
          dwa[c][j] += d * xh[c][j];
          if constexpr (HAS_BIAS) dba[c][j] += d;
          sum_g += g[c][j];
          sum_gx += g[c][j] * xh[c][j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) xh[c][j] = g[c][j] = 0.f;
      }
    }
    // block reduction; double-buffered slots (parity) make one barrier per row sufficient.
    sum_gx = wave_sum(sum_gx);
    if constexpr (!RMS) sum_g = wave_sum(sum_g);
    if (lane == 0) {
      red[parity][wid] = sum_gx;
      if constexpr (!RMS) redg[parity][wid] = sum_g;
    }
    __syncthreads();
    sum_gx = (red[parity][0] + red[parity][1] + red[parity][2] + red[parity][3]) / H;
    if constexpr (!RMS) sum_g = (redg[parity][0] + redg[parity][1] + redg[parity][2] + redg[parity][3]) / H;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int vi = c * 256 + tid;
      if (vi < nvec) {
        bf16x8 rv;
        if constexpr (HAS_DRES) rv = load_bf16x8(dres + base + vi * 8);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = g[c][j] - xh[c][j] * sum_gx;
          if constexpr (!RMS) t -= sum_g;
          t *= rstd;
          if constexpr (HAS_DRES) t += bf2f(rv[j]);
          o[j] = f2bf(t);
        }
        store_bf16x8(ds + base + vi * 8, o);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int vi = c * 256 + tid;
    if (vi < nvec) {
      float* o = dw_part + static_cast<size_t>(blockIdx.x) * H + vi * 8;
      *reinterpret_cast<f32x4*>(o) = f32x4{dwa[c][0], dwa[c][1], dwa[c][2], dwa[c][3]};
      *reinterpret_cast<f32x4*>(o + 4) = f32x4{dwa[c][4], dwa[c][5], dwa[c][6], dwa[c][7]};
      if constexpr (HAS_BIAS) {
        float* ob = db_part + static_cast<size_t>(blockIdx.x) * H + vi * 8;
        *reinterpret_cast<f32x4*>(ob) = f32x4{dba[c][0], dba[c][1], dba[c][2], dba[c][3]};
        *reinterpret_cast<f32x4*>(ob + 4) = f32x4{dba[c][4], dba[c][5], dba[c][6], dba[c][7]};
      }
    }
  }
}

// Two-stage fold of the [nparts, H] fp32 partials: stage 1 = grid (H/256 column tiles x
// kSplit row splits), one column per thread (coalesced 1 KiB rows), independent loads
// unrolled; stage 2 folds the kSplit rows and rounds to bf16. Both stages are fully
// parallel (the first version walked 768 rows per thread on 16 blocks: 181 us -> ~10 us).
constexpr int kSplit = 16;

__global__ __launch_bounds__(256) void norm_wgrad_stage1_kernel(const float* __restrict__ part,
                                                                 int nparts, int H,
                                                                 float* __restrict__ out2) {
  const int h = blockIdx.x * 256 + threadIdx.x;
  if (h >= H) return;
  const int per = (nparts + kSplit - 1) / kSplit;
  const int r0 = blockIdx.y * per, r1 = min(nparts, r0 + per);
  float acc = 0.f;
#pragma unroll 8
  for (int r = r0; r < r1; ++r) acc += part[static_cast<size_t>(r) * H + h];
  out2[static_cast<size_t>(blockIdx.y) * H + h] = acc;
}

__global__ __launch_bounds__(256) void norm_wgrad_stage2_kernel(const float* __restrict__ out2, int H,
                                                                 bf16_t* __restrict__ out) {
  const int h = blockIdx.x * 256 + threadIdx.x;
  if (h >= H) return;
  float acc = 0.f;
#pragma unroll
  for (int r = 0; r < kSplit; ++r) acc += out2[static_cast<size_t>(r) * H + h];
  out[h] = f2bf(acc);
}

static void wgrad_reduce(const float* part, int nparts, int H, bf16_t* out, float* scratch,
                         hipStream_t st) {
  const dim3 g1((H + 255) / 256, kSplit), g2((H + 255) / 256);
  norm_wgrad_stage1_kernel<<<g1, 256, 0, st>>>(part, nparts, H, scratch);
  norm_wgrad_stage2_kernel<<<g2, 256, 0, st>>>(scratch, H, out);
}

// ----------------------------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------------------------
template <bool RMS, bool HAS_RES, bool HAS_BIAS>
static void launch_fwd_nc(int nc, dim3 grid, hipStream_t st, const bf16_t* x, const bf16_t* r,
                          bf16_t* so, const bf16_t* w, const bf16_t* b, bf16_t* y, float* rstd,
                          float* mean, int rows, int H, float eps) {
#define DLA_NORM_FWD(NC)                                                                 \
  norm_fwd_kernel<NC, RMS, HAS_RES, HAS_BIAS>                                            \
      <<<grid, 256, 0, st>>>(x, r, so, w, b, y, rstd, mean, rows, H, eps)
  switch (nc) {
    case 1: DLA_NORM_FWD(1); break;
    case 2: DLA_NORM_FWD(2); break;
    case 4: DLA_NORM_FWD(4); break;
    case 8: DLA_NORM_FWD(8); break;
    default: DLA_NORM_FWD(16); break;
  }
#undef DLA_NORM_FWD
}

static int chunks_for(int H, int threads) {
  const int need = (H / 8 + threads - 1) / threads;
  return need <= 1 ? 1 : need <= 2 ? 2 : need <= 4 ? 4 : need <= 8 ? 8 : 16;
}

void launch_norm_fwd(const bf16_t* x, const bf16_t* res, bf16_t* sum_out, const bf16_t* w,
                     const bf16_t* b, bf16_t* y, float* rstd, float* mean, int rows, int H,
                     float eps, bool rms, hipStream_t st) {
  const bool hr = res != nullptr, hb = b != nullptr;
  if (rows < 512 && H <= 8192) {  // few rows (decode): block per row
    const int nt = ((H / 8 + 63) / 64) * 64;
#define DLA_NORM_ROW(R, HR, HB) \
  norm_fwd_row_kernel<R, HR, HB><<<rows, nt, 0, st>>>(x, res, sum_out, w, b, y, rstd, mean, H, eps)
    if (rms) {
      if (hr) DLA_NORM_ROW(true, true, false);
      else DLA_NORM_ROW(true, false, false);
    } else if (hr) {
      if (hb) DLA_NORM_ROW(false, true, true);
      else DLA_NORM_ROW(false, true, false);
    } else {
      if (hb) DLA_NORM_ROW(false, false, true);
      else DLA_NORM_ROW(false, false, false);
    }
#undef DLA_NORM_ROW
    return;
  }
  // wave-per-row: 64 lanes x NC(<=16) x 8 columns covers H <= 8192 (binding enforces it)
  if (H > 64 * 16 * 8) throw std::invalid_argument("norm_fwd: hidden size > 8192");
  const int nc = chunks_for(H, 64);
  dim3 grid((rows + 3) / 4);
  if (rms) {
    if (hr) launch_fwd_nc<true, true, false>(nc, grid, st, x, res, sum_out, w, b, y, rstd, mean, rows, H, eps);
    else launch_fwd_nc<true, false, false>(nc, grid, st, x, res, sum_out, w, b, y, rstd, mean, rows, H, eps);
  } else {
    if (hr) {
      if (hb) launch_fwd_nc<false, true, true>(nc, grid, st, x, res, sum_out, w, b, y, rstd, mean, rows, H, eps);
      else launch_fwd_nc<false, true, false>(nc, grid, st, x, res, sum_out, w, b, y, rstd, mean, rows, H, eps);
    } else {
      if (hb) launch_fwd_nc<false, false, true>(nc, grid, st, x, res, sum_out, w, b, y, rstd, mean, rows, H, eps);
      else launch_fwd_nc<false, false, false>(nc, grid, st, x, res, sum_out, w, b, y, rstd, mean, rows, H, eps);
    }
  }
}

int norm_bwd_grid(int rows) { return rows < 768 ? rows : 768; }
int norm_wgrad_scratch_rows() { return kSplit; }

template <bool RMS, bool HAS_DRES, bool HAS_BIAS>
static void launch_bwd_t(int nc, int grid, hipStream_t st, const bf16_t* dy, const bf16_t* s,
                         const bf16_t* w, const float* rstd, const float* mean,
                         const bf16_t* dres, bf16_t* ds, float* dwp, float* dbp, int rows,
                         int H) {
#define DLA_NORM_BWD(NC)                                                                     \
  norm_bwd_kernel<NC, RMS, HAS_DRES, HAS_BIAS>                                               \
      <<<grid, 256, 0, st>>>(dy, s, w, rstd, mean, dres, ds, dwp, dbp, rows, H)
  switch (nc) {
    case 1: DLA_NORM_BWD(1); break;
    case 2: DLA_NORM_BWD(2); break;
    case 4: DLA_NORM_BWD(4); break;
    case 8: DLA_NORM_BWD(8); break;
    default: DLA_NORM_BWD(16); break;
  }
#undef DLA_NORM_BWD
}

void launch_norm_bwd(const bf16_t* dy, const bf16_t* s, const bf16_t* w, const float* rstd,
                     const float* mean, const bf16_t* dres, bf16_t* ds, float* dw_part,
                     float* db_part, bf16_t* dw, bf16_t* db, int rows, int H, bool rms,
                     hipStream_t st) {
  const int nc = chunks_for(H, 256);
  const int grid = norm_bwd_grid(rows);
  const bool hd = dres != nullptr, hb = db != nullptr;
  if (rms) {
    if (hd) launch_bwd_t<true, true, false>(nc, grid, st, dy, s, w, rstd, mean, dres, ds, dw_part, db_part, rows, H);
    else launch_bwd_t<true, false, false>(nc, grid, st, dy, s, w, rstd, mean, dres, ds, dw_part, db_part, rows, H);
  } else {
    if (hd) {
      if (hb) launch_bwd_t<false, true, true>(nc, grid, st, dy, s, w, rstd, mean, dres, ds, dw_part, db_part, rows, H);
      else launch_bwd_t<false, true, false>(nc, grid, st, dy, s, w, rstd, mean, dres, ds, dw_part, db_part, rows, H);
    } else {
      if (hb) launch_bwd_t<false, false, true>(nc, grid, st, dy, s, w, rstd, mean, dres, ds, dw_part, db_part, rows, H);
      else launch_bwd_t<false, false, false>(nc, grid, st, dy, s, w, rstd, mean, dres, ds, dw_part, db_part, rows, H);
    }
  }
  // stage-1 scratch = kSplit extra rows allocated after the `grid` partial rows
  wgrad_reduce(dw_part, grid, H, dw, dw_part + static_cast<size_t>(grid) * H, st);
  if (hb) wgrad_reduce(db_part, grid, H, db, db_part + static_cast<size_t>(grid) * H, st);
}

}  // namespace dla
