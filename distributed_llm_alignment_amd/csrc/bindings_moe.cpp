// torch.ops.dla MoE routing / permutation ops (kernels in moe.hip). Host-side validation only.
#include <ATen/ATen.h>
#include <torch/library.h>

#include <tuple>

#include "bind_util.h"
#include "gg_params.h"
#include "reward_head.h"

namespace dla {

void launch_moe_topk_fwd(const bf16_t*, int64_t, int, int, float*, int*, hipStream_t);
void launch_moe_topk_bwd(const float*, const int*, const float*, int64_t, int, int, bf16_t*,
                         hipStream_t);
void launch_moe_dispatch(const bf16_t*, const int*, int64_t, int, int, bf16_t*, hipStream_t);
void launch_moe_combine(const bf16_t*, const int*, const float*, int64_t, int, int, int64_t, bf16_t*,
                        hipStream_t);
void launch_zero_rows_from(bf16_t*, int64_t, int, int64_t, const int*, hipStream_t);
void launch_ep_route(const void*, bool, int, int, int, int, int, int, int64_t*, int*, int*, int64_t*,
                     hipStream_t);
void launch_ep_expert_order(const int*, int, int, int, int64_t*, int64_t*, int*, hipStream_t);
void launch_gather_rows(const bf16_t*, int64_t, const int64_t*, int64_t, int, bf16_t*, hipStream_t);
void launch_scatter_rows(const bf16_t*, const int64_t*, int64_t, int, bf16_t*, hipStream_t);
void launch_moe_combine_bwd(const bf16_t*, const bf16_t*, const int*, const float*, int64_t, int,
                            int, int64_t, bf16_t*, float*, hipStream_t);

void launch_quant_fp8_rows(const bf16_t*, int64_t, int64_t, int, uint8_t*, float*, hipStream_t);
void launch_embed_fwd(const bf16_t*, int64_t, const int64_t*, int64_t, int, int64_t, bf16_t*, int*, hipStream_t);
void launch_embed_bwd(const int64_t*, const int64_t*, const bf16_t*, int64_t, int, int64_t, float*, void*,
                      bool, int64_t, hipStream_t);

static RHParams rh_params(const at::Tensor& hidden, const c10::optional<at::Tensor>& last,
                          const c10::optional<at::Tensor>& mask, const at::Tensor& w,
                          const c10::optional<at::Tensor>& bias, double p, int64_t seed) {
  check_bf16(hidden, "hidden");
  check_bf16(w, "w");
  TORCH_CHECK(hidden.dim() == 3 && hidden.stride(2) == 1 && hidden.stride(1) % 8 == 0 &&
                  hidden.stride(0) % 8 == 0 && hidden.size(2) % 8 == 0,
              "hidden [B, T, H], H % 8 == 0, 16-byte aligned rows");
  check_aligned16(hidden, "hidden");
  const int64_t B = hidden.size(0), T = hidden.size(1), H = hidden.size(2);
  TORCH_CHECK(w.numel() == H && w.is_contiguous(), "w [H] (Linear(H, 1).weight)");
  check_aligned16(w, "w");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout p in [0, 1)");
  RHParams r{};
  r.hidden = cbp(hidden);
  r.sb = hidden.stride(0);
  r.st = hidden.stride(1);
  if (mask && mask->defined()) {
    check_f32(*mask, "mask");
    TORCH_CHECK(mask->dim() == 2 && mask->size(0) == B && mask->size(1) == T && mask->is_contiguous(),
                "mask [B, T] fp32");
    r.mask = mask->data_ptr<float>();
  } else {
    TORCH_CHECK(last && last->defined(), "last_token pooling needs `last`");
    check_i32(*last, "last");
    TORCH_CHECK(last->numel() == B && last->is_contiguous(), "last [B] int32");
    r.last = last->data_ptr<int>();
  }
  r.w = cbp(w);
  if (bias && bias->defined()) {
    check_bf16(*bias, "bias");
    r.bias = cbp(*bias);
  }
  r.B = (int)B;
  r.T = (int)T;
  r.H = (int)H;
  r.p = static_cast<float>(p);
  r.seed = static_cast<uint64_t>(seed);
  return r;
}

// pooled (last valid token via `last`, or masked mean via `mask`) -> dropout -> . w + bias:
// returns (score fp32 [B], dropped pooled rows fp32 [B, H])
std::tuple<at::Tensor, at::Tensor> reward_head_fwd(const at::Tensor& hidden,
                                                   const c10::optional<at::Tensor>& last,
                                                   const c10::optional<at::Tensor>& mask,
                                                   const at::Tensor& w,
                                                   const c10::optional<at::Tensor>& bias, double p,
                                                   int64_t seed) {
  RHParams r = rh_params(hidden, last, mask, w, bias, p, seed);
  c10::hip::HIPGuardMasqueradingAsCUDA g(hidden.device());
  auto score = at::empty({hidden.size(0)}, hidden.options().dtype(at::kFloat));
  auto pooled = at::empty({hidden.size(0), hidden.size(2)}, hidden.options().dtype(at::kFloat));
  r.score = score.data_ptr<float>();
  r.pooled = pooled.data_ptr<float>();
  launch_reward_head_fwd(r, cur_stream(hidden));
  return {score, pooled};
}

// dHidden [B, T, H] (zero except the pooled positions), same mask regenerated from `seed`
at::Tensor reward_head_bwd(const at::Tensor& dscore, const at::Tensor& hidden,
                           const c10::optional<at::Tensor>& last, const c10::optional<at::Tensor>& mask,
                           const at::Tensor& w, double p, int64_t seed) {
  RHParams r = rh_params(hidden, last, mask, w, c10::nullopt, p, seed);
  check_f32(dscore, "dscore");
  TORCH_CHECK(dscore.numel() == hidden.size(0) && dscore.is_contiguous(), "dscore [B]");
  c10::hip::HIPGuardMasqueradingAsCUDA g(hidden.device());
  auto dh = at::zeros({hidden.size(0), hidden.size(1), hidden.size(2)}, hidden.options());
  r.dscore = dscore.data_ptr<float>();
  r.dhidden = bp(dh);
  launch_reward_head_bwd(r, cur_stream(hidden));
  return dh;
}

// token embedding gather: out[n] = w[ids[n]] (ids int64 [N], w [V, H] bf16). An id outside
// [0, V) gives a zero row and sets bad[0] = 1 (int32 [1], sticky, checked by the caller at its
// next host sync): no device assert, no host sync here.
at::Tensor embed_fwd(const at::Tensor& w, const at::Tensor& ids, at::Tensor bad) {
  check_bf16(w, "w");
  check_cuda(ids, "ids");
  check_i32(bad, "bad");
  TORCH_CHECK(bad.numel() >= 1 && bad.device() == w.device(), "bad: int32 [1] on the table's device");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.dim() == 1 && ids.is_contiguous(), "ids int64 [N]");
  TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1 && w.stride(0) % 8 == 0 && w.size(1) % 8 == 0,
              "w [V, H], H % 8 == 0, 16-byte aligned rows");
  check_aligned16(w, "w");
  c10::hip::HIPGuardMasqueradingAsCUDA g(w.device());
  auto out = at::empty({ids.size(0), w.size(1)}, w.options());
  launch_embed_fwd(cbp(w), w.stride(0), ids.data_ptr<int64_t>(), ids.size(0), (int)w.size(1),
                   w.size(0), bp(out), bad.data_ptr<int>(), cur_stream(w));
  return out;
}

// grad[sid[j]] += dy[perm[j]] for the sorted ids (deterministic run sums, no atomics), in place
// into grad [V, H] (bf16 or fp32: the engine's main-grad view)
void embed_bwd(const at::Tensor& sid, const at::Tensor& perm, const at::Tensor& dy, at::Tensor grad) {
  check_cuda(sid, "sid");
  check_cuda(perm, "perm");
  check_bf16(dy, "dy");
  check_cuda(grad, "grad");
  TORCH_CHECK(sid.scalar_type() == at::kLong && perm.scalar_type() == at::kLong && sid.dim() == 1 &&
                  sid.sizes() == perm.sizes() && sid.is_contiguous() && perm.is_contiguous(),
              "sid / perm int64 [N]");
  TORCH_CHECK(grad.scalar_type() == at::kBFloat16 || grad.scalar_type() == at::kFloat, "grad bf16 / fp32");
  TORCH_CHECK(dy.dim() == 2 && dy.is_contiguous() && dy.size(0) == sid.size(0) && dy.size(1) % 8 == 0,
              "dy [N, H] contiguous, H % 8 == 0");
  TORCH_CHECK(grad.dim() == 2 && grad.size(1) == dy.size(1) && grad.stride(1) == 1 && grad.stride(0) % 8 == 0,
              "grad [V, H] with 16-byte aligned rows");
  check_aligned16(dy, "dy");
  check_aligned16(grad, "grad");
  c10::hip::HIPGuardMasqueradingAsCUDA g(dy.device());
  const int64_t N = sid.size(0);
  auto scratch = at::empty({N, dy.size(1)}, dy.options().dtype(at::kFloat));
  launch_embed_bwd(sid.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), cbp(dy), N, (int)dy.size(1),
                   grad.size(0), scratch.data_ptr<float>(), grad.data_ptr(), grad.scalar_type() == at::kFloat,
                   grad.stride(0), cur_stream(dy));
}



static void check_offs(const at::Tensor& offs, int64_t G) {
  check_i32(offs, "offs");
  TORCH_CHECK(offs.dim() == 1 && offs.is_contiguous() && offs.size(0) == G + 1,
              "offs must be contiguous int32 [G + 1]");
}

static bool gg_is_fp8(const at::Tensor& t) { return t.scalar_type() == at::kFloat8_e4m3fn; }

static void check_operand(const at::Tensor& t, const char* name, bool fp8) {
  check_cuda(t, name);
  TORCH_CHECK(fp8 ? gg_is_fp8(t) : t.scalar_type() == at::kBFloat16, name,
              fp8 ? " must be float8_e4m3fn" : " must be bfloat16");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  check_aligned16(t, name);
}

// Rows of A are the expert-sorted token rows; offs[g]..offs[g+1] are expert g's rows (device
// array, never read on the host). The kernel trusts 0 = offs[0] <= ... <= offs[G] = rows.
static GGParams gg_base(const at::Tensor& a, const at::Tensor& offs) {
  GGParams p{};
  p.A = reinterpret_cast<const uint8_t*>(a.data_ptr());
  p.offs = offs.data_ptr<int>();
  p.G = static_cast<int>(offs.size(0) - 1);
  return p;
}

// y[M, N] = x[M, K] . w[g]^T per expert row range; fp8: x/w e4m3 with row scales sx [M, 1],
// sw [G, N, 1]
at::Tensor gg_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& offs,
                  const c10::optional<at::Tensor>& sx, const c10::optional<at::Tensor>& sw) {
  const bool fp8 = gg_is_fp8(x);
  check_operand(x, "x", fp8);
  check_operand(w, "w", fp8);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 3 && w.size(2) == x.size(1), "x [M, K], w [G, N, K]");
  const int64_t M = x.size(0), K = x.size(1), G = w.size(0), N = w.size(1);
  check_offs(offs, G);
  TORCH_CHECK(K % (fp8 ? 16 : 8) == 0 && N % 8 == 0 && N < (1 << 30) && K < (1 << 30),
              "K % 8 (bf16) / 16 (fp8) == 0 and N % 8 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(x.device());
  auto y = at::empty({M, N}, x.options().dtype(at::kBFloat16));
  if (M == 0) return y;
  GGParams p = gg_base(x, offs);
  p.B = reinterpret_cast<const uint8_t*>(w.data_ptr());
  p.C = y.data_ptr();
  p.lda = K; p.ldb = K; p.ldc = N; p.sBg = N * K;
  p.N = (int)N; p.K = (int)K;
  if (fp8) {
    TORCH_CHECK(sx && sw && sx->numel() == M && sw->numel() == G * N, "fp8 needs sx [M, 1] and sw [G, N, 1]");
    check_f32(*sx, "sx"); check_f32(*sw, "sw");
    TORCH_CHECK(sx->is_contiguous() && sw->is_contiguous(), "scales contiguous");
    p.sa = sx->data_ptr<float>(); p.sb = sw->data_ptr<float>(); p.sSg = N;
  }
  launch_grouped_gemm(p, 0, fp8, false, M, cur_stream(x));
  return y;
}

// gate|up projection with the SwiGLU epilogue: w_up [G, 2F, K] = [gate; up] -> (gu [M, 2F], a [M, F])
std::tuple<at::Tensor, at::Tensor> gg_fwd_swiglu(const at::Tensor& x, const at::Tensor& w,
                                                 const at::Tensor& offs,
                                                 const c10::optional<at::Tensor>& sx,
                                                 const c10::optional<at::Tensor>& sw) {
  const bool fp8 = gg_is_fp8(x);
  check_operand(x, "x", fp8);
  check_operand(w, "w_up", fp8);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 3 && w.size(2) == x.size(1) && w.size(1) % 2 == 0,
              "x [M, K], w_up [G, 2F, K]");
  const int64_t M = x.size(0), K = x.size(1), G = w.size(0), F = w.size(1) / 2;
  check_offs(offs, G);
  TORCH_CHECK(F % 128 == 0 && K % (fp8 ? 16 : 8) == 0, "F % 128 == 0, K % 8 (bf16) / 16 (fp8) == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(x.device());
  auto gu = at::empty({M, 2 * F}, x.options().dtype(at::kBFloat16));
  auto a = at::empty({M, F}, x.options().dtype(at::kBFloat16));
  if (M == 0) return {gu, a};
  GGParams p = gg_base(x, offs);
  p.B = reinterpret_cast<const uint8_t*>(w.data_ptr());
  p.C = gu.data_ptr();
  p.lda = K; p.ldb = K; p.ldc = 2 * F; p.sBg = 2 * F * K;
  p.N = (int)F; p.K = (int)K; p.F = (int)F;
  p.out2 = bp(a); p.ld_out2 = F;
  if (fp8) {
    TORCH_CHECK(sx && sw && sx->numel() == M && sw->numel() == G * 2 * F, "fp8 needs sx [M, 1] and sw [G, 2F, 1]");
    check_f32(*sx, "sx"); check_f32(*sw, "sw");
    TORCH_CHECK(sx->is_contiguous() && sw->is_contiguous(), "scales contiguous");
    p.sa = sx->data_ptr<float>(); p.sb = sw->data_ptr<float>(); p.sSg = 2 * F;
  }
  launch_grouped_gemm(p, 1, fp8, false, M, cur_stream(x));
  return {gu, a};
}

// input gradient: dx[M, K] = dy[M, N] . w[g] (w [G, N, K])
at::Tensor gg_dgrad(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& offs) {
  check_operand(dy, "dy", false);
  check_operand(w, "w", false);
  TORCH_CHECK(dy.dim() == 2 && w.dim() == 3 && w.size(1) == dy.size(1), "dy [M, N], w [G, N, K]");
  const int64_t M = dy.size(0), N = dy.size(1), G = w.size(0), K = w.size(2);
  check_offs(offs, G);
  TORCH_CHECK(K % 8 == 0 && N % 8 == 0, "N % 8 == 0 and K % 8 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(dy.device());
  auto dx = at::empty({M, K}, dy.options());
  if (M == 0) return dx;
  GGParams p = gg_base(dy, offs);
  p.B = reinterpret_cast<const uint8_t*>(w.data_ptr());
  p.C = dx.data_ptr();
  p.lda = N; p.ldb = K; p.ldc = K; p.sBg = N * K;
  p.N = (int)K; p.K = (int)N;
  launch_grouped_gemm(p, 2, false, false, M, cur_stream(dy));
  return dx;
}

// down projection input gradient fused with the SwiGLU backward: da = dy . w_down[g]
// (w_down [G, H, F]) -> (dgu [M, 2F], a [M, F]) from gu [M, 2F]
std::tuple<at::Tensor, at::Tensor> gg_dgrad_swiglu(const at::Tensor& dy, const at::Tensor& w,
                                                   const at::Tensor& offs, const at::Tensor& gu) {
  check_operand(dy, "dy", false);
  check_operand(w, "w_down", false);
  check_operand(gu, "gu", false);
  TORCH_CHECK(dy.dim() == 2 && w.dim() == 3 && w.size(1) == dy.size(1), "dy [M, H], w_down [G, H, F]");
  const int64_t M = dy.size(0), H = dy.size(1), G = w.size(0), F = w.size(2);
  TORCH_CHECK(gu.dim() == 2 && gu.size(0) == M && gu.size(1) == 2 * F, "gu [M, 2F]");
  check_offs(offs, G);
  TORCH_CHECK(F % 8 == 0 && H % 8 == 0, "H % 8 == 0 and F % 8 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(dy.device());
  auto dgu = at::empty({M, 2 * F}, dy.options());
  auto a = at::empty({M, F}, dy.options());
  if (M == 0) return {dgu, a};
  GGParams p = gg_base(dy, offs);
  p.B = reinterpret_cast<const uint8_t*>(w.data_ptr());
  p.C = dgu.data_ptr();
  p.lda = H; p.ldb = F; p.ldc = 2 * F; p.sBg = H * F;
  p.N = (int)F; p.K = (int)H; p.F = (int)F;
  p.aux = cbp(gu); p.ld_aux = 2 * F;
  p.out2 = bp(a); p.ld_out2 = F;
  launch_grouped_gemm(p, 3, false, false, M, cur_stream(dy));
  return {dgu, a};
}

// weight gradient: out[g] (+)= dy[rows of g]^T . x[rows of g]; dy [M, N1], x [M, N2],
// out [G, N1, N2] bf16 or fp32 (the fp32 main-grad buffer)
void gg_wgrad(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& offs, at::Tensor out,
              bool accumulate) {
  check_operand(dy, "dy", false);
  check_operand(x, "x", false);
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "dy [M, N1], x [M, N2]");
  const int64_t N1 = dy.size(1), N2 = x.size(1);
  check_cuda(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "out bf16 or fp32");
  TORCH_CHECK(out.dim() == 3 && out.size(1) == N1 && out.size(2) == N2 && out.is_contiguous(),
              "out [G, N1, N2] contiguous");
  check_aligned16(out, "out");
  const int64_t G = out.size(0);
  check_offs(offs, G);
  TORCH_CHECK(N1 % 8 == 0 && N2 % 8 == 0, "N1 % 8 == 0 and N2 % 8 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(dy.device());
  GGParams p = gg_base(dy, offs);
  p.B = reinterpret_cast<const uint8_t*>(x.data_ptr());
  p.C = out.data_ptr();
  p.lda = N1; p.ldb = N2; p.ldc = N2; p.sCg = N1 * N2;
  p.M = (int)N1; p.N = (int)N2; p.K = 0;
  p.accumulate = accumulate ? 1 : 0;
  launch_grouped_gemm(p, 4, false, out.scalar_type() == at::kFloat, dy.size(0), cur_stream(dy));
}

// x [M, K] bf16 (unit column stride, 16-B aligned rows) -> (q [M, K] float8_e4m3fn, inv_scale [M, 1])
std::tuple<at::Tensor, at::Tensor> quant_fp8_rows(const at::Tensor& x) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 && x.size(1) % 8 == 0,
              "x [M, K], K % 8 == 0, 16-byte aligned rows");
  check_aligned16(x, "x");
  const int64_t M = x.size(0), K = x.size(1);
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto q = at::empty({M, K}, x.options().dtype(at::kFloat8_e4m3fn));
  auto inv = at::empty({M, 1}, x.options().dtype(at::kFloat));
  launch_quant_fp8_rows(cbp(x), x.stride(0), M, (int)K, reinterpret_cast<uint8_t*>(q.data_ptr()),
                        inv.data_ptr<float>(), cur_stream(x));
  return {q, inv};
}

static void check_pos(const at::Tensor& pos, int64_t N, int64_t k) {
  check_i32(pos, "pos");
  TORCH_CHECK(pos.is_contiguous() && pos.dim() == 2 && pos.size(0) == N && pos.size(1) == k,
              "pos must be contiguous [N, k]");
  TORCH_CHECK(k >= 1 && k <= 8, "top-k must be in [1, 8]");
}

// The kernels trust pos[] to index rows of ys / xs: a permutation of [0, N*k) on the exact path
// (ops/moe.py builds it from an argsort), or slots of a capacity-padded buffer (parallel/expert.py)
// whose dropped slots point one past its last row -- the combine kernels read pos >= rows as a
// zero row (no gradient, zero weight gradient); the caller's construction is the bound.
std::tuple<at::Tensor, at::Tensor> moe_topk_fwd(const at::Tensor& logits, int64_t k) {
  check_bf16(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "logits [N, E] contiguous");
  const int64_t N = logits.size(0), E = logits.size(1);
  TORCH_CHECK(E >= 1 && E <= 256 && k >= 1 && k <= 8 && k <= E, "E <= 256, 1 <= k <= min(8, E)");
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  auto topv = at::empty({N, k}, logits.options().dtype(at::kFloat));
  auto topi = at::empty({N, k}, logits.options().dtype(at::kInt));
  launch_moe_topk_fwd(cbp(logits), N, (int)E, (int)k, topv.data_ptr<float>(), topi.data_ptr<int>(),
                      cur_stream(logits));
  return {topv, topi};
}

at::Tensor moe_topk_bwd(const at::Tensor& topv, const at::Tensor& topi, const at::Tensor& grad,
                        int64_t E) {
  check_f32(topv, "topv");
  check_f32(grad, "grad");
  check_i32(topi, "topi");
  TORCH_CHECK(topv.dim() == 2 && topv.sizes() == topi.sizes() && topv.sizes() == grad.sizes() &&
                  topv.is_contiguous() && topi.is_contiguous() && grad.is_contiguous(),
              "topv/topi/grad [N, k] contiguous");
  const int64_t N = topv.size(0), k = topv.size(1);
  TORCH_CHECK(E >= k && E <= 256 && k <= 8, "E/k range");
  c10::hip::HIPGuardMasqueradingAsCUDA g(topv.device());
  auto dl = at::empty({N, E}, topv.options().dtype(at::kBFloat16));
  launch_moe_topk_bwd(topv.data_ptr<float>(), topi.data_ptr<int>(), grad.data_ptr<float>(), N,
                      (int)E, (int)k, bp(dl), cur_stream(topv));
  return dl;
}

at::Tensor moe_dispatch(const at::Tensor& x, const at::Tensor& pos) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.size(1) % 8 == 0, "x [N, H], H % 8 == 0");
  const int64_t N = x.size(0), H = x.size(1), k = pos.size(-1);
  check_pos(pos, N, k);
  check_aligned16(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto xs = at::empty({N * k, H}, x.options());
  launch_moe_dispatch(cbp(x), pos.data_ptr<int>(), N, (int)H, (int)k, bp(xs), cur_stream(x));
  return xs;
}

at::Tensor moe_combine(const at::Tensor& ys, const at::Tensor& pos,
                       const c10::optional<at::Tensor>& w) {
  check_bf16(ys, "ys");
  TORCH_CHECK(ys.dim() == 2 && ys.is_contiguous() && ys.size(1) % 8 == 0, "ys [M, H], H % 8 == 0");
  const int64_t N = pos.size(0), k = pos.size(-1), H = ys.size(1);
  check_pos(pos, N, k);
  TORCH_CHECK(ys.size(0) >= 1, "ys has no rows");  // pos rows index ys (exact: N*k, capacity: any)
  const float* wp = nullptr;
  if (w && w->defined()) {
    check_f32(*w, "w");
    TORCH_CHECK(w->sizes() == pos.sizes() && w->is_contiguous(), "w [N, k]");
    wp = w->data_ptr<float>();
  }
  check_aligned16(ys, "ys");
  c10::hip::HIPGuardMasqueradingAsCUDA g(ys.device());
  auto out = at::empty({N, H}, ys.options());
  launch_moe_combine(cbp(ys), pos.data_ptr<int>(), wp, N, (int)H, (int)k, ys.size(0), bp(out), cur_stream(ys));
  return out;
}

// Expert-parallel capacity routing of one token chunk (parallel/expert.py _route_chunk):
// topi [n, k] int32/int64 -> (send_src [ep*C] int64, pos [n, k] int32, sent [ep, El] int32);
// the dropped-slot count is added to `dropped` (int64 [1] on the device).
std::tuple<at::Tensor, at::Tensor, at::Tensor> ep_route(const at::Tensor& topi, int64_t E, int64_t ep,
                                                        int64_t C, at::Tensor& dropped) {
  check_cuda(topi, "topi");
  TORCH_CHECK(topi.dim() == 2 && topi.is_contiguous() &&
                  (topi.scalar_type() == at::kInt || topi.scalar_type() == at::kLong),
              "topi [n, k] int32/int64 contiguous");
  TORCH_CHECK(dropped.scalar_type() == at::kLong && dropped.numel() >= 1 && dropped.device() == topi.device(),
              "dropped: int64 counter on the device");
  const int64_t n = topi.size(0), k = topi.size(1), S = n * k;
  TORCH_CHECK(E >= 1 && E <= 64 && ep >= 1 && E % ep == 0 && C >= 1, "1 <= E <= 64, ep | E");
  TORCH_CHECK(S <= 256 * 64, "ep_route: at most 16384 slots per chunk");
  c10::hip::HIPGuardMasqueradingAsCUDA g(topi.device());
  auto send_src = at::empty({ep * C}, topi.options().dtype(at::kLong));
  auto pos = at::empty({n, k}, topi.options().dtype(at::kInt));
  auto sent = at::empty({ep, E / ep}, topi.options().dtype(at::kInt));
  launch_ep_route(topi.data_ptr(), topi.scalar_type() == at::kLong, (int)S, (int)k, (int)E, (int)(E / ep),
                  (int)ep, (int)C, send_src.data_ptr<int64_t>(), pos.data_ptr<int>(), sent.data_ptr<int>(),
                  dropped.data_ptr<int64_t>(), cur_stream(topi));
  return {send_src, pos, sent};
}

// Receiver side (_expert_order): rc [ep, El] int32 -> (xe_src [ep*C], inv [ep*C] int64, offs [El+1] int32)
std::tuple<at::Tensor, at::Tensor, at::Tensor> ep_expert_order(const at::Tensor& rc, int64_t C) {
  check_i32(rc, "rc");
  TORCH_CHECK(rc.dim() == 2 && rc.is_contiguous() && rc.size(0) <= 64 && rc.size(1) <= 64 && C >= 1,
              "rc [ep <= 64, El <= 64] contiguous");
  const int64_t ep = rc.size(0), El = rc.size(1);
  c10::hip::HIPGuardMasqueradingAsCUDA g(rc.device());
  auto xe_src = at::empty({ep * C}, rc.options().dtype(at::kLong));
  auto inv = at::empty({ep * C}, rc.options().dtype(at::kLong));
  auto offs = at::empty({El + 1}, rc.options());
  launch_ep_expert_order(rc.data_ptr<int>(), (int)ep, (int)El, (int)C, xe_src.data_ptr<int64_t>(),
                         inv.data_ptr<int64_t>(), offs.data_ptr<int>(), cur_stream(rc));
  return {xe_src, inv, offs};
}

// out[i] = idx[i] >= 0 ? x[idx[i]] : 0 (idx int64 [n], x [R, H] bf16 with unit column stride);
// the caller guarantees idx < R
at::Tensor gather_rows(const at::Tensor& x, const at::Tensor& idx) {
  check_bf16(x, "x");
  check_cuda(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.dim() == 1 && idx.is_contiguous(), "idx int64 [n]");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 && x.size(1) % 8 == 0,
              "x [R, H], H % 8 == 0, 16-byte aligned rows");
  check_aligned16(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto out = at::empty({idx.size(0), x.size(1)}, x.options());
  launch_gather_rows(cbp(x), x.stride(0), idx.data_ptr<int64_t>(), idx.size(0), (int)x.size(1), bp(out),
                     cur_stream(x));
  return out;
}

// dx[idx[i]] = g[i] for idx[i] >= 0 (idx injective on those), other rows of dx zero; dx [R, H]
at::Tensor scatter_rows(const at::Tensor& gr, const at::Tensor& idx, int64_t R) {
  check_bf16(gr, "g");
  check_cuda(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.dim() == 1 && idx.is_contiguous(), "idx int64 [n]");
  TORCH_CHECK(gr.dim() == 2 && gr.is_contiguous() && gr.size(0) == idx.size(0) && gr.size(1) % 8 == 0,
              "g [n, H] contiguous, H % 8 == 0");
  check_aligned16(gr, "g");
  c10::hip::HIPGuardMasqueradingAsCUDA g(gr.device());
  auto dx = at::zeros({R, gr.size(1)}, gr.options());
  launch_scatter_rows(cbp(gr), idx.data_ptr<int64_t>(), idx.size(0), (int)gr.size(1), bp(dx), cur_stream(gr));
  return dx;
}

// x[r] = 0 for r >= from[0] (device scalar: e.g. offs[-1] of a capacity buffer); no host sync
void zero_rows_from(at::Tensor& x, const at::Tensor& from) {
  check_bf16(x, "x");
  check_i32(from, "from");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 && x.size(1) % 8 == 0,
              "x [R, C], C % 8 == 0, 16-byte aligned rows");
  check_aligned16(x, "x");
  TORCH_CHECK(from.numel() >= 1, "from: one int32 on the device");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  launch_zero_rows_from(bp(x), x.size(0), (int)x.size(1), x.stride(0), from.data_ptr<int>(), cur_stream(x));
}

std::tuple<at::Tensor, at::Tensor> moe_combine_bwd(const at::Tensor& dout, const at::Tensor& ys,
                                                   const at::Tensor& pos, const at::Tensor& w,
                                                   bool permutation) {
  check_bf16(dout, "dout");
  check_bf16(ys, "ys");
  check_f32(w, "w");
  const int64_t N = pos.size(0), k = pos.size(-1), H = ys.size(1);
  check_pos(pos, N, k);
  TORCH_CHECK(dout.dim() == 2 && dout.size(0) == N && dout.size(1) == H && dout.is_contiguous(),
              "dout [N, H]");
  TORCH_CHECK(ys.dim() == 2 && ys.size(0) >= 1 && ys.is_contiguous() && H % 8 == 0, "ys [R, H]");
  TORCH_CHECK(w.sizes() == pos.sizes() && w.is_contiguous(), "w [N, k]");
  check_aligned16(ys, "ys");
  check_aligned16(dout, "dout");
  c10::hip::HIPGuardMasqueradingAsCUDA g(ys.device());
  // `permutation` (the caller's promise: pos maps the N*k slots one-to-one onto the rows of ys,
  // the dropless dispatch): every row is written. Otherwise (capacity buffer, possibly with
  // ep*C == N*k by coincidence): rows no slot reads get a zero gradient and the appended zero row
  // shared by the dropped slots receives racing writes whose gradient is discarded
  TORCH_CHECK(!permutation || ys.size(0) == N * k, "permutation: ys must have N*k rows");
  auto dys = permutation ? at::empty_like(ys) : at::zeros_like(ys);
  auto dw = at::empty({N, k}, w.options());
  launch_moe_combine_bwd(cbp(dout), cbp(ys), pos.data_ptr<int>(), w.data_ptr<float>(), N, (int)H,
                         (int)k, ys.size(0), bp(dys), dw.data_ptr<float>(), cur_stream(ys));
  return {dys, dw};
}

}  // namespace dla

namespace dla {
int gg_set_sched(int sched);
// the grouped GEMM's K-step schedule for the rest of the process (-1: the default); returns the
// previous one
int64_t gg_set_sched_op(int64_t sched) { return gg_set_sched(static_cast<int>(sched)); }
}  // namespace dla

TORCH_LIBRARY_FRAGMENT(dla, m) {
  m.def("gg_set_sched(int sched) -> int", &dla::gg_set_sched_op);
  m.def("moe_topk_fwd(Tensor logits, int k) -> (Tensor, Tensor)");
  m.def("quant_fp8_rows(Tensor x) -> (Tensor, Tensor)");
  m.def("embed_fwd(Tensor w, Tensor ids, Tensor(a!) bad) -> Tensor");
  m.def("reward_head_fwd(Tensor hidden, Tensor? last, Tensor? mask, Tensor w, Tensor? bias, float p, int seed) -> (Tensor, Tensor)");
  m.def("reward_head_bwd(Tensor dscore, Tensor hidden, Tensor? last, Tensor? mask, Tensor w, float p, int seed) -> Tensor");
  m.def("embed_bwd(Tensor sid, Tensor perm, Tensor dy, Tensor(a!) grad) -> ()");
  m.def("moe_topk_bwd(Tensor topv, Tensor topi, Tensor grad, int E) -> Tensor");
  m.def("moe_dispatch(Tensor x, Tensor pos) -> Tensor");
  m.def("moe_combine(Tensor ys, Tensor pos, Tensor? w) -> Tensor");
  m.def("moe_combine_bwd(Tensor dout, Tensor ys, Tensor pos, Tensor w, bool permutation=False) -> (Tensor, Tensor)");
  m.def("zero_rows_from(Tensor(a!) x, Tensor from) -> ()");
  m.def("ep_route(Tensor topi, int E, int ep, int C, Tensor(a!) dropped) -> (Tensor, Tensor, Tensor)");
  m.def("ep_expert_order(Tensor rc, int C) -> (Tensor, Tensor, Tensor)");
  m.def("gather_rows(Tensor x, Tensor idx) -> Tensor");
  m.def("scatter_rows(Tensor g, Tensor idx, int R) -> Tensor");
  m.def("gg_fwd(Tensor x, Tensor w, Tensor offs, Tensor? sx, Tensor? sw) -> Tensor");
  m.def("gg_fwd_swiglu(Tensor x, Tensor w_up, Tensor offs, Tensor? sx, Tensor? sw) -> (Tensor, Tensor)");
  m.def("gg_dgrad(Tensor dy, Tensor w, Tensor offs) -> Tensor");
  m.def("gg_dgrad_swiglu(Tensor dy, Tensor w_down, Tensor offs, Tensor gu) -> (Tensor, Tensor)");
  m.def("gg_wgrad(Tensor dy, Tensor x, Tensor offs, Tensor(a!) out, bool accumulate) -> ()");
}

TORCH_LIBRARY_IMPL(dla, CUDA, m) {
  m.impl("moe_topk_fwd", &dla::moe_topk_fwd);
  m.impl("quant_fp8_rows", &dla::quant_fp8_rows);
  m.impl("embed_fwd", &dla::embed_fwd);
  m.impl("reward_head_fwd", &dla::reward_head_fwd);
  m.impl("reward_head_bwd", &dla::reward_head_bwd);
  m.impl("embed_bwd", &dla::embed_bwd);
  m.impl("moe_topk_bwd", &dla::moe_topk_bwd);
  m.impl("moe_dispatch", &dla::moe_dispatch);
  m.impl("moe_combine", &dla::moe_combine);
  m.impl("moe_combine_bwd", &dla::moe_combine_bwd);
  m.impl("zero_rows_from", &dla::zero_rows_from);
  m.impl("ep_route", &dla::ep_route);
  m.impl("ep_expert_order", &dla::ep_expert_order);
  m.impl("gather_rows", &dla::gather_rows);
  m.impl("scatter_rows", &dla::scatter_rows);
  m.impl("gg_fwd", &dla::gg_fwd);
  m.impl("gg_fwd_swiglu", &dla::gg_fwd_swiglu);
  m.impl("gg_dgrad", &dla::gg_dgrad);
  m.impl("gg_dgrad_swiglu", &dla::gg_dgrad_swiglu);
  m.impl("gg_wgrad", &dla::gg_wgrad);
}
