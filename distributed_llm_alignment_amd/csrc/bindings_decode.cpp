// torch.ops.dla decode-path ops: split-KV decode attention (decode.hip) and the fused sampler
// (sampling.hip). Host-side validation only; both are graph-capture safe (device-side lengths
// and RNG counter, outputs from the caching allocator, no host sync).
#include <ATen/ATen.h>
#include <torch/library.h>

#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "bind_util.h"
#include "skinny_params.h"

namespace dla {

void launch_decode_attn(const bf16_t*, int64_t, int64_t, bf16_t*, bf16_t*, int64_t,
                        int64_t, int64_t, const int*, const int*, int, float, int, int, int, int,
                        int, float*, float*, bf16_t*, int64_t, int64_t, int*, hipStream_t);
void launch_decode_attn_rope(const bf16_t*, int64_t, const float*, const float*, const int*,
                             const int64_t*, int, bf16_t*, bf16_t*, int64_t, int64_t, int64_t,
                             const int*, const int*, int, float, int, int, int, int, int, float*,
                             float*, bf16_t*, int64_t, int64_t, int*, hipStream_t);
int decode_num_splits(int Tmax, int B, int Hkv);
void launch_rope_cache(const bf16_t*, int64_t, bf16_t*, bf16_t*, bf16_t*, int64_t, int64_t,
                       int64_t, const int64_t*, const float*, const float*, const int*, int, int,
                       int, int, int, hipStream_t);
void launch_sample(const void*, bool, int64_t, int64_t, int, float, int, float, bool,
                   const int64_t*, int64_t*, hipStream_t);
int sample_split_chunks(const void*, int64_t, int64_t, int, float, int, float, bool);
size_t sample_workspace_bytes(int64_t, int);
void launch_sample_split(const void*, bool, int64_t, int64_t, int, int, float, int, float,
                         const int64_t*, int64_t*, void*, hipStream_t);

int skinny_splits(int M, int N, int K);
bool skinny_use_ksplit(int N, int K);
void launch_skinny_ksplit(const bf16_t*, int64_t, const bf16_t*, int64_t, bf16_t*, int64_t, int,
                          int, int, hipStream_t);
void launch_skinny_gemm(const bf16_t*, int64_t, const bf16_t*, int64_t, bf16_t*, int64_t, float*,
                        unsigned*, int, int, int, int, bool, bool, hipStream_t);
bool skinny_glu_ks_ok(int N, int K);
void launch_skinny_glu_ks(const bf16_t*, int64_t, const bf16_t*, int64_t, bf16_t*, int64_t, int,
                          int, int, hipStream_t);

void launch_skinny_ks_fused(const bf16_t*, int64_t, const bf16_t*, int64_t, bf16_t*, int64_t, int,
                            int, int, const KsFuse&, bool, bool, bool, hipStream_t);
void launch_skinny_glu_normin(const bf16_t*, int64_t, const bf16_t*, int64_t, bf16_t*, int64_t, int,
                              int, int, const KsFuse&, bool, hipStream_t);

int m64_splits(int N, int K);
void launch_tile_weight(const bf16_t*, int64_t, const bf16_t*, bf16_t*, int, int, bool, hipStream_t);
void launch_quant_tile_f8(const bf16_t*, int64_t, const bf16_t*, uint8_t*, float*, int, int, bool, hipStream_t);
void launch_skinny_glu_il(const bf16_t*, int64_t, const bf16_t*, bf16_t*, int64_t, int, int, int,
                          const KsFuse&, hipStream_t);
void launch_skinny_ks_fused_f8(const bf16_t*, int64_t, const uint8_t*, bf16_t*, int64_t, int, int, int,
                               const KsFuse&, bool, bool, hipStream_t);
void launch_skinny_glu_il_f8(const bf16_t*, int64_t, const uint8_t*, bf16_t*, int64_t, int, int, int,
                             const KsFuse&, hipStream_t);
bool m64_shape_ok(int N, int K, bool glu);
void launch_m64_gemm(const bf16_t*, int64_t, const bf16_t*, int64_t, bf16_t*, int64_t, float*, int,
                     int, int, int, bool, const float*, int, float, bool, hipStream_t);
void launch_m64_reduce(const float*, int, int, int, bf16_t*, int64_t, const bf16_t*, int64_t,
                       const float*, int, int, float, float*, hipStream_t);
void launch_m64_gemm_f8(const bf16_t*, int64_t, const uint8_t*, bf16_t*, int64_t, float*, int, int, int, int,
                        bool, const float*, int, float, const float*, hipStream_t);

// Decode projection at 17..64 rows (skinny64.hip), the same fused-layer contract as
// skinny_fused below with row-norm partials per (row, 1024 columns):
//   * plain: y = x w^T;
//   * res given: (s = bf16(bf16(x w^T) + res), ssq [M, ceil(N / 1024)]);
//   * ssq_in given ([M, nbp], nbp <= 8): y = rstd[m] * (x w^T), w with the norm weight folded in;
//     with `glu` the gate|up projection + SwiGLU epilogue (w = [gate; up], output [M, F]).
std::tuple<at::Tensor, at::Tensor> skinny64(const at::Tensor& x, const at::Tensor& w,
                                            const c10::optional<at::Tensor>& res,
                                            const c10::optional<at::Tensor>& ssq_in, double eps,
                                            bool glu) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  // w: [N, K] row-major, or the tiled layout [N / 16, K / 32, 4, 16, 8] (skinny64.hip TW)
  const bool tiled = w.dim() == 5;
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 &&
                  (tiled ? (w.size(2) == 4 && w.size(3) == 16 && w.size(4) == 8 && w.is_contiguous())
                         : (w.dim() == 2 && w.stride(1) == 1 && w.stride(0) % 8 == 0)),
              "x [M, K] / w [N, K] (unit inner stride, 16-byte aligned rows) or tiled [N/16, K/32, 4, 16, 8]");
  const int64_t M = x.size(0), N = tiled ? w.size(0) * 16 : w.size(0), K = tiled ? w.size(1) * 32 : w.size(1);
  TORCH_CHECK(M >= 1 && M <= 64 && x.size(1) == K, "skinny64: 1 <= M <= 64, x [M, K]");
  TORCH_CHECK(N < (1ll << 30) && K < (1ll << 30), "shape too large");
  TORCH_CHECK(m64_shape_ok((int)N, (int)K, glu),
              "skinny64: K % 256 == 0 and N % 128 == 0");
  check_aligned16(x, "x");
  check_aligned16(w, "w");
  same_device(x, w);
  const float* sq = nullptr;
  int nbp = 0;
  if (ssq_in.has_value()) {
    const at::Tensor& t = *ssq_in;
    check_cuda(t, "ssq_in");
    TORCH_CHECK(t.scalar_type() == at::kFloat && t.dim() == 2 && t.size(0) == M && t.is_contiguous() &&
                    t.size(1) >= 1 && t.size(1) <= 64,
                "ssq_in fp32 [M, nbp <= 64] contiguous");
    same_device(x, t);
    sq = t.data_ptr<float>();
    nbp = static_cast<int>(t.size(1));
  }
  TORCH_CHECK(!(res.has_value() && (sq || glu)), "skinny64: residual output takes a plain input");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto st = cur_stream(x);
  if (glu) {
    auto m = at::empty({M, N / 2}, x.options());
    launch_m64_gemm(cbp(x), x.stride(0), cbp(w), tiled ? K : w.stride(0), bp(m), m.stride(0), nullptr,
                    (int)M, (int)N, (int)K, 1, true, sq, nbp, static_cast<float>(eps), tiled, st);
    return {m, at::Tensor()};
  }
  const int S = m64_splits((int)N, (int)K);
  TORCH_CHECK(S > 1 || !(sq || res.has_value()),
              "skinny64: the residual / normalised-input epilogue needs a split-K shape");
  auto y = at::empty({M, N}, x.options());
  at::Tensor ws;
  if (S > 1) ws = at::empty({S, M, N}, x.options().dtype(at::kFloat));
  const bf16_t* rp = nullptr;
  int64_t ldr = 0;
  at::Tensor ssq;
  if (res.has_value()) {
    const at::Tensor& r = *res;
    check_bf16(r, "res");
    TORCH_CHECK(r.dim() == 2 && r.size(0) == M && r.size(1) == N && r.stride(1) == 1, "res [M, N]");
    same_device(x, r);
    rp = cbp(r);
    ldr = r.stride(0);
    // row partials per 1024 columns (written by the reduce launch)
    ssq = at::empty({M, (N + 1023) / 1024}, x.options().dtype(at::kFloat));
  }
  float* sqo = ssq.defined() ? ssq.data_ptr<float>() : nullptr;
  launch_m64_gemm(cbp(x), x.stride(0), cbp(w), tiled ? K : w.stride(0), bp(y), y.stride(0),
                  S > 1 ? ws.data_ptr<float>() : nullptr, (int)M, (int)N, (int)K, S, false, sq, nbp,
                  static_cast<float>(eps), tiled, st);
  if (S > 1)
    launch_m64_reduce(ws.data_ptr<float>(), S, (int)M, (int)N, bp(y), y.stride(0), rp, ldr, sq, nbp,
                      (int)K, static_cast<float>(eps), sqo, st);
  return {y, ssq};
}

// out <- w [N, K] in the tiled decode layout [N/16, K/32, 4, 16, 8] (nw given: bf16(w * nw), the
// RMSNorm weight folded into the input columns)
void tile_weight(const at::Tensor& w, const c10::optional<at::Tensor>& nw, at::Tensor& out, bool glu_il) {
  check_bf16(w, "w");
  check_bf16(out, "out");
  TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1 && w.stride(0) % 8 == 0, "w [N, K], unit inner stride");
  const int64_t N = w.size(0), K = w.size(1);
  TORCH_CHECK(N % 16 == 0 && K % 32 == 0 && N < (1ll << 30) && K < (1ll << 30), "N % 16 == 0, K % 32 == 0");
  TORCH_CHECK(!glu_il || N % 32 == 0, "glu_il: N = 2F, F % 16 == 0");
  TORCH_CHECK(out.dim() == 5 && out.size(0) == N / 16 && out.size(1) == K / 32 && out.size(2) == 4 &&
                  out.size(3) == 16 && out.size(4) == 8 && out.is_contiguous(),
              "out [N/16, K/32, 4, 16, 8] contiguous");
  check_aligned16(w, "w");
  check_aligned16(out, "out");
  same_device(w, out);
  const bf16_t* np = nullptr;
  if (nw.has_value()) {
    check_bf16(*nw, "nw");
    TORCH_CHECK(nw->dim() == 1 && nw->size(0) == K && nw->is_contiguous(), "nw [K]");
    check_aligned16(*nw, "nw");
    same_device(w, *nw);
    np = cbp(*nw);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(w.device());
  launch_tile_weight(cbp(w), w.stride(0), np, bp(out), (int)N, (int)K, glu_il, cur_stream(w));
}

// w [N, K] bf16 (+ nw folded, glu_il interleave) -> out8 uint8 [N/16, K/64, 64, 16] e4m3 tiled
// and scale fp32 [N] (per tiled row), in place (a captured decode graph keeps reading them)
void quant_tile_f8(const at::Tensor& w, const c10::optional<at::Tensor>& nw, at::Tensor& out8, at::Tensor& scale,
                   bool glu_il) {
  check_bf16(w, "w");
  TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1 && w.stride(0) % 8 == 0, "w [N, K], unit inner stride");
  const int64_t N = w.size(0), K = w.size(1);
  TORCH_CHECK(N % 32 == 0 && K % 64 == 0 && N < (1ll << 30) && K < (1ll << 30), "N % 32 == 0, K % 64 == 0");
  check_cuda(out8, "out8");
  TORCH_CHECK(out8.scalar_type() == at::kByte && out8.is_contiguous() && out8.numel() == N * K,
              "out8 uint8 contiguous, N * K bytes");
  check_cuda(scale, "scale");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.is_contiguous() && scale.numel() == N, "scale fp32 [N]");
  check_aligned16(w, "w");
  check_aligned16(out8, "out8");
  same_device(w, out8);
  same_device(w, scale);
  const bf16_t* np = nullptr;
  if (nw.has_value() && nw->defined()) {
    check_bf16(*nw, "nw");
    TORCH_CHECK(nw->dim() == 1 && nw->size(0) == K && nw->is_contiguous(), "nw [K] contiguous");
    same_device(w, *nw);
    np = cbp(*nw);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(w.device());
  launch_quant_tile_f8(cbp(w), w.stride(0), np, out8.data_ptr<uint8_t>(), scale.data_ptr<float>(), (int)N, (int)K,
                       glu_il, cur_stream(w));
}

// Decode gate|up + SwiGLU at M <= 16 over the interleaved tiled weight (tile_weight glu_il, norm
// folded) from the producer's row-norm partials: [M, F] = silu(rstd * g) * (rstd * u)
at::Tensor skinny_glu_il(const at::Tensor& x, const at::Tensor& wt, const at::Tensor& ssq_in, double eps) {
  check_bf16(x, "x");
  check_bf16(wt, "wt");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "x [M, K]");
  TORCH_CHECK(wt.dim() == 5 && wt.size(2) == 4 && wt.size(3) == 16 && wt.size(4) == 8 && wt.is_contiguous(),
              "wt [2F/16, K/32, 4, 16, 8] contiguous");
  const int64_t M = x.size(0), N = wt.size(0) * 16, K = wt.size(1) * 32;
  TORCH_CHECK(M >= 1 && M <= 16 && x.size(1) == K, "skinny_glu_il: 1 <= M <= 16, x [M, K]");
  TORCH_CHECK(K % 512 == 0 && N < (1ll << 30) && K < (1ll << 30) && M * (K + 8) * 2 <= 148 * 1024,
              "K % 512 == 0, x fits LDS");
  check_cuda(ssq_in, "ssq_in");
  TORCH_CHECK(ssq_in.scalar_type() == at::kFloat && ssq_in.dim() == 2 && ssq_in.size(0) == 16 &&
                  ssq_in.is_contiguous() && ssq_in.size(1) >= 1 && ssq_in.size(1) <= 512,
              "ssq_in fp32 [16, nbp <= 512] contiguous");
  check_aligned16(x, "x");
  check_aligned16(wt, "wt");
  same_device(x, wt);
  same_device(x, ssq_in);
  KsFuse fz{};
  fz.ssq_in = ssq_in.data_ptr<float>();
  fz.nbp = static_cast<int>(ssq_in.size(1));
  fz.eps = static_cast<float>(eps);
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto m = at::empty({M, N / 2}, x.options());
  launch_skinny_glu_il(cbp(x), x.stride(0), cbp(wt), bp(m), m.stride(0), (int)M, (int)N, (int)K, fz,
                       cur_stream(x));
  return m;
}

// fp8 weight-only decode projections (ops/decode.py fp8_tiled_weight): w8 = e4m3 tiled copy
// [N/16, K/64, 64, 16] (uint8 storage), wscale [N] fp32 per weight row; otherwise skinny_fused /
// skinny_glu_il (res: o / down producing the residual; ssq_in: qkv / gate|up on a normalised input).
static void check_w8(const at::Tensor& w8, const at::Tensor& wscale, const at::Tensor& x, int64_t* N,
                     int64_t* K) {
  check_cuda(w8, "w8");
  TORCH_CHECK(w8.scalar_type() == at::kByte && w8.dim() == 4 && w8.size(2) == 64 && w8.size(3) == 16 &&
                  w8.is_contiguous(),
              "w8 uint8 [N/16, K/64, 64, 16] contiguous");
  *N = w8.size(0) * 16;
  *K = w8.size(1) * 64;
  check_cuda(wscale, "wscale");
  TORCH_CHECK(wscale.scalar_type() == at::kFloat && wscale.dim() == 1 && wscale.size(0) == *N &&
                  wscale.is_contiguous(),
              "wscale fp32 [N] contiguous");
  check_aligned16(w8, "w8");
  same_device(x, w8);
  same_device(x, wscale);
}

static void check_ssq(const at::Tensor& sq, const at::Tensor& x, KsFuse* fz, double eps) {
  check_cuda(sq, "ssq_in");
  TORCH_CHECK(sq.scalar_type() == at::kFloat && sq.dim() == 2 && sq.size(0) == 16 && sq.is_contiguous() &&
                  sq.size(1) >= 1 && sq.size(1) <= 512,
              "ssq_in fp32 [16, nbp <= 512] contiguous");
  same_device(x, sq);
  fz->ssq_in = sq.data_ptr<float>();
  fz->nbp = static_cast<int>(sq.size(1));
  fz->eps = static_cast<float>(eps);
}

std::tuple<at::Tensor, at::Tensor> skinny_fused_f8(const at::Tensor& x, const at::Tensor& w8,
                                                   const at::Tensor& wscale,
                                                   const c10::optional<at::Tensor>& res,
                                                   const c10::optional<at::Tensor>& ssq_in, double eps) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "x [M, K], 16-byte aligned rows");
  int64_t N = 0, K = 0;
  check_w8(w8, wscale, x, &N, &K);
  const int64_t M = x.size(0);
  TORCH_CHECK(M >= 1 && M <= 16 && x.size(1) == K, "fp8 skinny: 1 <= M <= 16, x [M, K]");
  // (a plain projection -- the LM head -- may be any width: one workgroup per 16 columns)
  const bool plain = !res.has_value() && !ssq_in.has_value();
  TORCH_CHECK(N < (1ll << 30) && K < (1ll << 30) &&
                  (plain ? (N % 16 == 0 && K % 1024 == 0) : skinny_use_ksplit((int)N, (int)K)),
              "fp8 skinny: N % 16 == 0, K % 1024 == 0 (fused forms: N < 16384)");
  check_aligned16(x, "x");
  KsFuse fz{};
  fz.wscale = wscale.data_ptr<float>();
  const bool nin = ssq_in.has_value();
  if (nin) check_ssq(*ssq_in, x, &fz, eps);
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto y = at::empty({M, N}, x.options());
  at::Tensor ssq;
  if (res.has_value()) {
    const at::Tensor& r = *res;
    check_bf16(r, "res");
    TORCH_CHECK(r.dim() == 2 && r.size(0) == M && r.size(1) == N && r.stride(1) == 1, "res [M, N]");
    same_device(x, r);
    fz.res = cbp(r);
    fz.ldr = r.stride(0);
    ssq = at::empty({16, N / 16}, x.options().dtype(at::kFloat));
    fz.ssq_out = ssq.data_ptr<float>();
  }
  launch_skinny_ks_fused_f8(cbp(x), x.stride(0), w8.data_ptr<uint8_t>(), bp(y), y.stride(0), (int)M, (int)N,
                            (int)K, fz, res.has_value(), nin, cur_stream(x));
  return {y, ssq};
}

// fp8 form of skinny64 (17..64 rows, csrc/skinny64.hip F8): w8 the e4m3 tiled copy
// [N/16, K/64, 64, 16] with per-row scales `wscale` (ops/decode.py fp8_tiled_weight; gate|up: the
// plain [gate; up] row order, norm weight folded in). Same epilogue contract as skinny64.
std::tuple<at::Tensor, at::Tensor> skinny64_f8(const at::Tensor& x, const at::Tensor& w8, const at::Tensor& wscale,
                                               const c10::optional<at::Tensor>& res,
                                               const c10::optional<at::Tensor>& ssq_in, double eps, bool glu) {
  check_bf16(x, "x");
  int64_t N = 0, K = 0;
  check_w8(w8, wscale, x, &N, &K);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "x [M, K], unit inner stride");
  const int64_t M = x.size(0);
  TORCH_CHECK(M >= 1 && M <= 64 && x.size(1) == K, "fp8 skinny64: 1 <= M <= 64, x [M, K]");
  TORCH_CHECK(N < (1ll << 30) && K < (1ll << 30) && m64_shape_ok((int)N, (int)K, glu),
              "fp8 skinny64: K % 256 == 0 and N % 128 == 0");
  check_aligned16(x, "x");
  const float* sq = nullptr;
  int nbp = 0;
  if (ssq_in.has_value()) {
    const at::Tensor& t = *ssq_in;
    check_cuda(t, "ssq_in");
    TORCH_CHECK(t.scalar_type() == at::kFloat && t.dim() == 2 && t.size(0) == M && t.is_contiguous() &&
                    t.size(1) >= 1 && t.size(1) <= 64,
                "ssq_in fp32 [M, nbp <= 64] contiguous");
    same_device(x, t);
    sq = t.data_ptr<float>();
    nbp = static_cast<int>(t.size(1));
  }
  TORCH_CHECK(!(res.has_value() && (sq || glu)), "fp8 skinny64: residual output takes a plain input");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto st = cur_stream(x);
  const uint8_t* wp = w8.data_ptr<uint8_t>();
  const float* wsc = wscale.data_ptr<float>();
  if (glu) {
    auto m = at::empty({M, N / 2}, x.options());
    launch_m64_gemm_f8(cbp(x), x.stride(0), wp, bp(m), m.stride(0), nullptr, (int)M, (int)N, (int)K, 1, true, sq,
                       nbp, static_cast<float>(eps), wsc, st);
    return {m, at::Tensor()};
  }
  const int S = m64_splits((int)N, (int)K);
  TORCH_CHECK(S > 1 || !(sq || res.has_value()),
              "fp8 skinny64: the residual / normalised-input epilogue needs a split-K shape");
  auto y = at::empty({M, N}, x.options());
  at::Tensor ws;
  if (S > 1) ws = at::empty({S, M, N}, x.options().dtype(at::kFloat));
  const bf16_t* rp = nullptr;
  int64_t ldr = 0;
  at::Tensor ssq;
  if (res.has_value()) {
    const at::Tensor& r = *res;
    check_bf16(r, "res");
    TORCH_CHECK(r.dim() == 2 && r.size(0) == M && r.size(1) == N && r.stride(1) == 1, "res [M, N]");
    same_device(x, r);
    rp = cbp(r);
    ldr = r.stride(0);
    ssq = at::empty({M, (N + 1023) / 1024}, x.options().dtype(at::kFloat));
  }
  float* sqo = ssq.defined() ? ssq.data_ptr<float>() : nullptr;
  launch_m64_gemm_f8(cbp(x), x.stride(0), wp, bp(y), y.stride(0), S > 1 ? ws.data_ptr<float>() : nullptr, (int)M,
                     (int)N, (int)K, S, false, sq, nbp, static_cast<float>(eps), wsc, st);
  if (S > 1)
    launch_m64_reduce(ws.data_ptr<float>(), S, (int)M, (int)N, bp(y), y.stride(0), rp, ldr, sq, nbp, (int)K,
                      static_cast<float>(eps), sqo, st);
  return {y, ssq};
}

at::Tensor skinny_glu_il_f8(const at::Tensor& x, const at::Tensor& w8, const at::Tensor& wscale,
                            const at::Tensor& ssq_in, double eps) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "x [M, K]");
  int64_t N = 0, K = 0;
  check_w8(w8, wscale, x, &N, &K);
  const int64_t M = x.size(0);
  TORCH_CHECK(M >= 1 && M <= 16 && x.size(1) == K, "fp8 glu: 1 <= M <= 16, x [M, K]");
  TORCH_CHECK(K % 512 == 0 && N % 32 == 0 && N < (1ll << 30) && K < (1ll << 30) &&
                  M * (K + 8) * 2 <= 148 * 1024,
              "fp8 glu: K % 512 == 0, 2F % 32 == 0, x fits LDS");
  check_aligned16(x, "x");
  KsFuse fz{};
  fz.wscale = wscale.data_ptr<float>();
  check_ssq(ssq_in, x, &fz, eps);
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto m = at::empty({M, N / 2}, x.options());
  launch_skinny_glu_il_f8(cbp(x), x.stride(0), w8.data_ptr<uint8_t>(), bp(m), m.stride(0), (int)M, (int)N,
                          (int)K, fz, cur_stream(x));
  return m;
}

// Fused decode-layer projection (M <= 16, skinny.hip KsFuse):
//   * res given: returns (s = bf16(bf16(x w^T) + res) [M, N], ssq [16, N/16] fp32 partial sums of
//     s^2 per (row, 16-column workgroup)) -- the o / down projection producing the residual;
//   * ssq_in given: x is a residual stream s and w a weight with the RMSNorm weight folded in
//     (w o norm_w, ops/decode.py): returns rstd[m] * (s w^T), rstd = rsqrt(sum(ssq_in[m]) / K +
//     eps) -- RMSNorm(s) @ W^T without a norm launch: the qkv projection, or with `glu` the
//     gate|up projection with the SwiGLU epilogue (w = [gate; up], output [M, F]).
std::tuple<at::Tensor, at::Tensor> skinny_fused(const at::Tensor& x, const at::Tensor& w,
                                                const c10::optional<at::Tensor>& res,
                                                const c10::optional<at::Tensor>& ssq_in, double eps,
                                                bool glu) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  // w: [N, K] row-major, or the tiled layout [N / 16, K / 32, 4, 16, 8] (skinny64.hip TW)
  const bool tiled = w.dim() == 5;
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 &&
                  (tiled ? (w.size(2) == 4 && w.size(3) == 16 && w.size(4) == 8 && w.is_contiguous())
                         : (w.dim() == 2 && w.stride(1) == 1 && w.stride(0) % 8 == 0)),
              "x [M, K] / w [N, K] (unit inner stride, 16-byte aligned rows) or tiled [N/16, K/32, 4, 16, 8]");
  const int64_t M = x.size(0), N = tiled ? w.size(0) * 16 : w.size(0), K = tiled ? w.size(1) * 32 : w.size(1);
  TORCH_CHECK(M >= 1 && M <= 16 && x.size(1) == K, "fused skinny: 1 <= M <= 16, x [M, K]");
  TORCH_CHECK(N < (1ll << 30) && K < (1ll << 30), "shape too large");
  check_aligned16(x, "x");
  check_aligned16(w, "w");
  same_device(x, w);
  const bool nin = ssq_in.has_value();
  KsFuse fz{};
  if (nin) {
    const at::Tensor& sq = *ssq_in;
    check_cuda(sq, "ssq_in");
    TORCH_CHECK(sq.scalar_type() == at::kFloat && sq.dim() == 2 && sq.size(0) == 16 && sq.is_contiguous() &&
                    sq.size(1) >= 1 && sq.size(1) <= 512,
                "ssq_in fp32 [16, nbp <= 512] contiguous");
    same_device(x, sq);
    fz.ssq_in = sq.data_ptr<float>();
    fz.nbp = static_cast<int>(sq.size(1));
    fz.eps = static_cast<float>(eps);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  if (glu) {
    TORCH_CHECK(nin && !res.has_value(), "glu: normalised input, no residual");
    TORCH_CHECK(N % 128 == 0 && M * (K + 8) * 2 <= 148 * 1024, "glu: 2F % 128 == 0, x fits LDS");
    auto m = at::empty({M, N / 2}, x.options());
    launch_skinny_glu_normin(cbp(x), x.stride(0), cbp(w), tiled ? K : w.stride(0), bp(m), m.stride(0),
                             (int)M, (int)N, (int)K, fz, tiled, cur_stream(x));
    return {m, at::Tensor()};
  }
  TORCH_CHECK(skinny_use_ksplit((int)N, (int)K), "fused skinny: N < 16384, N % 16 == 0, K % 1024 == 0");
  auto y = at::empty({M, N}, x.options());
  at::Tensor ssq;
  if (res.has_value()) {
    const at::Tensor& r = *res;
    check_bf16(r, "res");
    TORCH_CHECK(r.dim() == 2 && r.size(0) == M && r.size(1) == N && r.stride(1) == 1, "res [M, N]");
    same_device(x, r);
    fz.res = cbp(r);
    fz.ldr = r.stride(0);
    ssq = at::empty({16, N / 16}, x.options().dtype(at::kFloat));
    fz.ssq_out = ssq.data_ptr<float>();
  }
  launch_skinny_ks_fused(cbp(x), x.stride(0), cbp(w), tiled ? K : w.stride(0), bp(y), y.stride(0),
                         (int)M, (int)N, (int)K, fz, res.has_value(), nin, tiled, cur_stream(x));
  return {y, ssq};
}

// Decode gate|up with the SwiGLU epilogue on the in-workgroup split-K kernel: w = [gate; up]
// (2F rows) -> m = silu(x gate^T) * (x up^T) [M, F], one workgroup per 16 features.
at::Tensor skinny_glu_ks(const at::Tensor& x, const at::Tensor& w) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.stride(1) == 1 && w.stride(1) == 1,
              "x [M, K] / w [2F, K] with unit inner stride");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(M >= 1 && M <= 64, "skinny GLU: 1 <= M <= 64");
  TORCH_CHECK(x.size(1) == K, "x width must be K");
  TORCH_CHECK(N < (1ll << 30) && K < (1ll << 30) && skinny_glu_ks_ok((int)N, (int)K),
              "skinny GLU: K % 512 == 0 and 2F % 32 == 0");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "16-byte aligned rows");
  check_aligned16(x, "x");
  check_aligned16(w, "w");
  same_device(x, w);
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto m = at::empty({M, N / 2}, x.options());
  launch_skinny_glu_ks(cbp(x), x.stride(0), cbp(w), w.stride(0), bp(m), m.stride(0), (int)M,
                       (int)N, (int)K, cur_stream(x));
  return m;
}


// y[M, N] = x[M, K] @ w[N, K]^T for M <= 16 (decode). With `swiglu`, x is the fused gate|up
// output gu[M, 2K] and the kernel applies silu(g) * u while staging it. `counters` (int32,
// zero-initialised once, re-armed by the kernel) holds one split-K arrival counter per 128
// output columns.
at::Tensor skinny_gemm(const at::Tensor& x, const at::Tensor& w, at::Tensor& counters, bool swiglu,
                       bool glu_out) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_i32(counters, "counters");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.stride(1) == 1 && w.stride(1) == 1,
              "x [M, K] / w [N, K] with unit inner stride");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  // 17..64 rows: only the in-workgroup split-K kernel (narrow N, no fused swiglu input)
  TORCH_CHECK(M >= 1 && (M <= 16 || (M <= 64 && !swiglu && !glu_out && skinny_use_ksplit((int)N, (int)K))),
              "skinny GEMM: 1 <= M <= 16 (<= 64 on the split-K path: N < 16384, K % 1024 == 0)");
  TORCH_CHECK(x.size(1) == (swiglu ? 2 * K : K), "x width must be K (2K with swiglu)");
  TORCH_CHECK(K % 256 == 0 && N % 16 == 0, "skinny GEMM: K % 256 == 0 and N % 16 == 0");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "16-byte aligned rows");
  TORCH_CHECK(N < (1ll << 30) && K < (1ll << 30), "shape too large");
  check_aligned16(x, "x");
  check_aligned16(w, "w");
  same_device(x, w);
  same_device(x, counters);
  const int64_t nb = (N + 127) / 128;
  TORCH_CHECK(counters.is_contiguous() && counters.numel() >= nb, "counters: one per 128 columns");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  if (glu_out) {  // w = [gate; up] (2F rows) -> silu(x gate^T) * (x up^T) [M, F]
    TORCH_CHECK(!swiglu && N % 128 == 0, "glu_out: 2F rows with F % 64 == 0, no swiglu input");
    TORCH_CHECK(M * (K + 8) * 2 <= 152 * 1024, "skinny GEMM: x exceeds LDS");
    auto m = at::empty({M, N / 2}, x.options());
    launch_skinny_gemm(cbp(x), x.stride(0), cbp(w), w.stride(0), bp(m), m.stride(0), nullptr,
                       reinterpret_cast<unsigned*>(counters.data_ptr<int>()), (int)M, (int)N,
                       (int)K, 1, false, true, cur_stream(x));
    return m;
  }
  auto y = at::empty({M, N}, x.options());
  if (!swiglu && skinny_use_ksplit((int)N, (int)K)) {  // narrow N: in-workgroup split-K
    launch_skinny_ksplit(cbp(x), x.stride(0), cbp(w), w.stride(0), bp(y), y.stride(0), (int)M,
                         (int)N, (int)K, cur_stream(x));
    return y;
  }
  const int S = skinny_splits((int)M, (int)N, (int)K);
  TORCH_CHECK(M * (K / S + 8) * 2 <= 160 * 1024, "skinny GEMM: x slice exceeds LDS");
  at::Tensor ws;
  if (S > 1) ws = at::empty({S, M, N}, x.options().dtype(at::kFloat));
  launch_skinny_gemm(cbp(x), x.stride(0), cbp(w), w.stride(0), bp(y), y.stride(0),
                     S > 1 ? ws.data_ptr<float>() : nullptr,
                     reinterpret_cast<unsigned*>(counters.data_ptr<int>()), (int)M, (int)N, (int)K,
                     S, swiglu, false, cur_stream(x));
  return y;
}

// Per-device arrival counters of the in-kernel split combine (decode.hip dec_arrive_combine):
// zeroed once here, re-armed to 0 by the block that combines. Created only outside a stream
// capture (generation runs an eager decode step before capturing); nullptr -> the combine launch.
// One buffer per device: two decode attention kernels must not run concurrently on one device.
// DLA_DECODE_FUSED_COMBINE=0 keeps the separate combine launch.
constexpr int64_t kDecCounters = 4096;
static int* decode_counters(const at::Tensor& like, int64_t n) {
  static const bool on = [] {
    const char* e = std::getenv("DLA_DECODE_FUSED_COMBINE");
    return !(e != nullptr && std::atoi(e) == 0);
  }();
  if (!on || n > kDecCounters) return nullptr;
  static auto* bufs = new std::map<int, at::Tensor>();  // never destroyed (outlives the allocator)
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  const int dev = like.get_device();
  auto it = bufs->find(dev);
  if (it != bufs->end()) return it->second.data_ptr<int>();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(cur_stream(like), &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
    return nullptr;
  auto t = at::zeros({kDecCounters}, like.options().dtype(at::kInt));
  bufs->emplace(dev, t);
  return t.data_ptr<int>();
}

at::Tensor decode_attn(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                       const at::Tensor& kv_len, const c10::optional<at::Tensor>& kv_start,
                       int64_t window, double scale) {
  check_bf16(q, "q");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  check_i32(kv_len, "kv_len");
  TORCH_CHECK(q.dim() == 3 && k_cache.dim() == 4 && v_cache.sizes() == k_cache.sizes(),
              "q [B, Hq, D], caches [B, Tmax, Hkv, D]");
  const int64_t B = q.size(0), Hq = q.size(1), D = q.size(2);
  const int64_t Tmax = k_cache.size(1), Hkv = k_cache.size(2);
  TORCH_CHECK(k_cache.size(0) == B && k_cache.size(3) == D, "cache batch / head dim");
  TORCH_CHECK(D == 64 || D == 128, "decode attention supports head_dim 64 or 128");
  TORCH_CHECK(Hq % Hkv == 0, "Hq % Hkv");
  const int64_t G = Hq / Hkv;
  TORCH_CHECK(G == 1 || G == 2 || G == 4 || G == 8, "GQA group size must be 1, 2, 4 or 8");
  TORCH_CHECK(q.stride(2) == 1 && k_cache.stride(3) == 1 && v_cache.stride(3) == 1,
              "head dim must be contiguous");
  TORCH_CHECK(k_cache.strides() == v_cache.strides(), "k/v caches must share strides");
  TORCH_CHECK(q.stride(1) % 8 == 0 && k_cache.stride(1) % 8 == 0 && k_cache.stride(2) % 8 == 0 &&
                  k_cache.stride(0) % 8 == 0,
              "16-byte aligned rows");
  check_aligned16(k_cache, "k_cache");
  check_aligned16(v_cache, "v_cache");
  TORCH_CHECK(kv_len.numel() >= 1, "kv_len");
  const int* ks = nullptr;
  if (kv_start && kv_start->defined()) {
    check_i32(*kv_start, "kv_start");
    TORCH_CHECK(kv_start->numel() == B && kv_start->is_contiguous(), "kv_start [B]");
    ks = kv_start->data_ptr<int>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  const int nsplit = decode_num_splits(static_cast<int>(Tmax), static_cast<int>(B), static_cast<int>(Hkv));
  auto fopt = q.options().dtype(at::kFloat);
  auto part_o = at::empty({B, Hq, nsplit, D}, fopt);
  auto part_ml = at::empty({B, Hq, nsplit, 2}, fopt);
  auto out = at::empty({B, Hq, D}, q.options());
  launch_decode_attn(cbp(q), q.stride(0), q.stride(1), bp(k_cache), bp(v_cache),
                     k_cache.stride(0), k_cache.stride(1), k_cache.stride(2),
                     kv_len.data_ptr<int>(), ks, static_cast<int>(window),
                     static_cast<float>(scale * 1.4426950408889634), (int)B, (int)Hq, (int)Hkv,
                     (int)D, (int)Tmax, part_o.data_ptr<float>(), part_ml.data_ptr<float>(),
                     bp(out), out.stride(0), out.stride(1), decode_counters(q, B * Hkv), cur_stream(q));
  return out;
}

// qkv [B, 1, (Hq + 2 Hkv) D] of the newest token -> rotated q [B, Hq, D]; k/v written into
// k_cache/v_cache [B, Tmax, Hkv, D] at row `slot` (int64 [1] on device).
at::Tensor rope_cache_write(const at::Tensor& qkv, const at::Tensor& cos, const at::Tensor& sin,
                            const at::Tensor& pos, at::Tensor& k_cache, at::Tensor& v_cache,
                            const at::Tensor& slot, int64_t Hq, int64_t Hkv, int64_t D, int64_t rot) {
  check_bf16(qkv, "qkv");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  check_f32(cos, "cos");
  check_f32(sin, "sin");
  check_i32(pos, "pos");
  check_cuda(slot, "slot");
  TORCH_CHECK(slot.scalar_type() == at::kLong && slot.numel() >= 1, "slot int64");
  const int64_t B = qkv.size(0);
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(1) == 1 && qkv.size(2) == (Hq + 2 * Hkv) * D &&
                  qkv.stride(2) == 1 && qkv.stride(0) % 8 == 0,
              "qkv [B, 1, (Hq+2Hkv)D] with 16-byte aligned rows");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(0) == B && k_cache.size(2) == Hkv &&
                  k_cache.size(3) == D && k_cache.sizes() == v_cache.sizes() &&
                  k_cache.strides() == v_cache.strides() && k_cache.stride(3) == 1,
              "caches [B, Tmax, Hkv, D]");
  TORCH_CHECK(D % 8 == 0 && rot % 16 == 0 && rot <= D, "D % 8, rot % 16");
  TORCH_CHECK(cos.is_contiguous() && sin.is_contiguous() && cos.size(-1) == rot / 2, "rope tables");
  TORCH_CHECK(pos.numel() == B && pos.is_contiguous(), "pos [B]");
  check_aligned16(qkv, "qkv");
  check_aligned16(k_cache, "k_cache");
  check_aligned16(v_cache, "v_cache");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  auto q = at::empty({B, Hq, D}, qkv.options());
  launch_rope_cache(cbp(qkv), qkv.stride(0), bp(q), bp(k_cache), bp(v_cache), k_cache.stride(0),
                    k_cache.stride(1), k_cache.stride(2), slot.data_ptr<int64_t>(),
                    cos.data_ptr<float>(), sin.data_ptr<float>(), pos.data_ptr<int>(), (int)B,
                    (int)Hq, (int)Hkv, (int)D, (int)rot, cur_stream(qkv));
  return q;
}

// One decode step's attention with the rope + cache write of the newest token fused in (one
// launch pair instead of rope_cache_write + decode_attn): qkv [B, 1, (Hq + 2 Hkv) D] raw row,
// caches [B, Tmax, Hkv, D] (row `slot` is written), kv_len = slot + 1 (device).
at::Tensor decode_attn_rope(const at::Tensor& qkv, const at::Tensor& cos, const at::Tensor& sin,
                            const at::Tensor& pos, at::Tensor& k_cache, at::Tensor& v_cache,
                            const at::Tensor& slot, const at::Tensor& kv_len,
                            const c10::optional<at::Tensor>& kv_start, int64_t window, double scale,
                            int64_t Hq, int64_t Hkv, int64_t D, int64_t rot) {
  check_bf16(qkv, "qkv");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  check_f32(cos, "cos");
  check_f32(sin, "sin");
  check_i32(pos, "pos");
  check_i32(kv_len, "kv_len");
  check_cuda(slot, "slot");
  TORCH_CHECK(slot.scalar_type() == at::kLong && slot.numel() >= 1, "slot int64");
  const int64_t B = qkv.size(0);
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(1) == 1 && qkv.size(2) == (Hq + 2 * Hkv) * D &&
                  qkv.stride(2) == 1 && qkv.stride(0) % 8 == 0,
              "qkv [B, 1, (Hq+2Hkv)D] with 16-byte aligned rows");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(0) == B && k_cache.size(2) == Hkv &&
                  k_cache.size(3) == D && k_cache.sizes() == v_cache.sizes() &&
                  k_cache.strides() == v_cache.strides() && k_cache.stride(3) == 1,
              "caches [B, Tmax, Hkv, D]");
  TORCH_CHECK(D == 64 || D == 128, "decode attention supports head_dim 64 or 128");
  TORCH_CHECK(Hq % Hkv == 0, "Hq % Hkv");
  const int64_t G = Hq / Hkv;
  TORCH_CHECK(G == 1 || G == 2 || G == 4 || G == 8, "GQA group size must be 1, 2, 4 or 8");
  TORCH_CHECK(rot % 16 == 0 && rot <= D && rot > 0, "rot % 16 == 0, 0 < rot <= D");
  TORCH_CHECK(cos.is_contiguous() && sin.is_contiguous() && cos.size(-1) == rot / 2, "rope tables");
  TORCH_CHECK(pos.numel() == B && pos.is_contiguous(), "pos [B]");
  TORCH_CHECK(k_cache.stride(1) % 8 == 0 && k_cache.stride(2) % 8 == 0 && k_cache.stride(0) % 8 == 0,
              "16-byte aligned cache rows");
  check_aligned16(qkv, "qkv");
  check_aligned16(k_cache, "k_cache");
  check_aligned16(v_cache, "v_cache");
  const int* ks = nullptr;
  if (kv_start && kv_start->defined()) {
    check_i32(*kv_start, "kv_start");
    TORCH_CHECK(kv_start->numel() == B && kv_start->is_contiguous(), "kv_start [B]");
    ks = kv_start->data_ptr<int>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  const int64_t Tmax = k_cache.size(1);
  const int nsplit = decode_num_splits(static_cast<int>(Tmax), static_cast<int>(B), static_cast<int>(Hkv));
  auto fopt = qkv.options().dtype(at::kFloat);
  auto part_o = at::empty({B, Hq, nsplit, D}, fopt);
  auto part_ml = at::empty({B, Hq, nsplit, 2}, fopt);
  auto out = at::empty({B, Hq, D}, qkv.options());
  launch_decode_attn_rope(cbp(qkv), qkv.stride(0), cos.data_ptr<float>(), sin.data_ptr<float>(),
                          pos.data_ptr<int>(), slot.data_ptr<int64_t>(), (int)rot, bp(k_cache),
                          bp(v_cache), k_cache.stride(0), k_cache.stride(1), k_cache.stride(2),
                          kv_len.data_ptr<int>(), ks, static_cast<int>(window),
                          static_cast<float>(scale * 1.4426950408889634), (int)B, (int)Hq, (int)Hkv,
                          (int)D, (int)Tmax, part_o.data_ptr<float>(), part_ml.data_ptr<float>(),
                          bp(out), out.stride(0), out.stride(1), decode_counters(qkv, B * Hkv),
                          cur_stream(qkv));
  return out;
}

at::Tensor sample_tokens(const at::Tensor& logits, double temperature, int64_t top_k,
                         double top_p, bool greedy, const at::Tensor& rng) {
  check_cuda(logits, "logits");
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat,
              "logits must be bf16 or fp32");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits [B, V] with unit vocab stride");
  check_cuda(rng, "rng");
  TORCH_CHECK(rng.scalar_type() == at::kLong && rng.numel() >= 2, "rng int64 [seed, counter]");
  TORCH_CHECK(top_p > 0.0 && top_p <= 1.0, "top_p in (0, 1]");
  const int64_t B = logits.size(0), V = logits.size(1);
  TORCH_CHECK(V < (1ll << 31), "vocab too large");
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  auto out = at::empty({B}, logits.options().dtype(at::kLong));
  const float inv_t = temperature > 0.0 ? static_cast<float>(1.0 / temperature) : 0.f;
  const bool is_bf16 = logits.scalar_type() == at::kBFloat16;
  const int G = sample_split_chunks(logits.data_ptr(), logits.stride(0), B, (int)V, inv_t,
                                    (int)top_k, static_cast<float>(top_p), greedy);
  if (G > 0) {  // top-k / top-p on a large vocabulary: row-split multi-launch sampler
    auto ws = at::empty({(int64_t)sample_workspace_bytes(B, G)}, logits.options().dtype(at::kByte));
    launch_sample_split(logits.data_ptr(), is_bf16, logits.stride(0), B, (int)V, G, inv_t,
                        (int)top_k, static_cast<float>(top_p), rng.data_ptr<int64_t>(),
                        out.data_ptr<int64_t>(), ws.data_ptr(), cur_stream(logits));
    return out;
  }
  launch_sample(logits.data_ptr(), is_bf16, logits.stride(0), B, (int)V, inv_t, (int)top_k,
                static_cast<float>(top_p), greedy, rng.data_ptr<int64_t>(),
                out.data_ptr<int64_t>(), cur_stream(logits));
  return out;
}

}  // namespace dla

TORCH_LIBRARY_FRAGMENT(dla, m) {
  m.def("decode_attn(Tensor q, Tensor k_cache, Tensor v_cache, Tensor kv_len, Tensor? kv_start, int window, float scale) -> Tensor");
  m.def("rope_cache_write(Tensor qkv, Tensor cos, Tensor sin, Tensor pos, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor slot, int Hq, int Hkv, int D, int rot) -> Tensor");
  m.def("decode_attn_rope(Tensor qkv, Tensor cos, Tensor sin, Tensor pos, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor slot, Tensor kv_len, Tensor? kv_start, int window, float scale, int Hq, int Hkv, int D, int rot) -> Tensor");
  m.def("sample_tokens(Tensor logits, float temperature, int top_k, float top_p, bool greedy, Tensor rng) -> Tensor");
  m.def("skinny_gemm(Tensor x, Tensor w, Tensor(a!) counters, bool swiglu, bool glu_out=False) -> Tensor");
  m.def("skinny_glu_ks(Tensor x, Tensor w) -> Tensor");
  m.def("skinny_fused(Tensor x, Tensor w, Tensor? res, Tensor? ssq_in, float eps, bool glu) -> (Tensor, Tensor)");
  m.def("skinny64(Tensor x, Tensor w, Tensor? res, Tensor? ssq_in, float eps, bool glu) -> (Tensor, Tensor)");
  m.def("skinny64_f8(Tensor x, Tensor w8, Tensor wscale, Tensor? res, Tensor? ssq_in, float eps, bool glu) -> (Tensor, Tensor)");
  m.def("tile_weight(Tensor w, Tensor? nw, Tensor(a!) out, bool glu_il=False) -> ()");
  m.def("quant_tile_f8(Tensor w, Tensor? nw, Tensor(a!) out8, Tensor(b!) scale, bool glu_il=False) -> ()");
  m.def("skinny_glu_il(Tensor x, Tensor wt, Tensor ssq_in, float eps) -> Tensor");
  m.def("skinny_fused_f8(Tensor x, Tensor w8, Tensor wscale, Tensor? res, Tensor? ssq_in, float eps) -> (Tensor, Tensor)");
  m.def("skinny_glu_il_f8(Tensor x, Tensor w8, Tensor wscale, Tensor ssq_in, float eps) -> Tensor");
}

TORCH_LIBRARY_IMPL(dla, CUDA, m) {
  m.impl("decode_attn", &dla::decode_attn);
  m.impl("sample_tokens", &dla::sample_tokens);
  m.impl("rope_cache_write", &dla::rope_cache_write);
  m.impl("decode_attn_rope", &dla::decode_attn_rope);
  m.impl("skinny_gemm", &dla::skinny_gemm);
  m.impl("skinny_glu_ks", &dla::skinny_glu_ks);
  m.impl("skinny_fused", &dla::skinny_fused);
  m.impl("skinny64", &dla::skinny64);
  m.impl("skinny64_f8", &dla::skinny64_f8);
  m.impl("tile_weight", &dla::tile_weight);
  m.impl("quant_tile_f8", &dla::quant_tile_f8);
  m.impl("skinny_glu_il", &dla::skinny_glu_il);
  m.impl("skinny_fused_f8", &dla::skinny_fused_f8);
  m.impl("skinny_glu_il_f8", &dla::skinny_glu_il_f8);
}
