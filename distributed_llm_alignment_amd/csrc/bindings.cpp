// Torch custom-op registry for the gfx950 kernels: `torch.ops.dla.*`.
//
// Host side only (compiled by the host C++ compiler): every op validates operand shapes,
// dtypes, strides and devices BEFORE launching (a mis-shaped launch of a hand-written kernel
// can fault the GPU), allocates outputs through the torch caching allocator and launches on
// the caller's current HIP stream. No op synchronises the host.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <tuple>

#include "attn_params.h"
#include "bind_util.h"

namespace dla {

// ---- kernel launchers (defined in *.hip) ----
void launch_norm_fwd(const bf16_t*, const bf16_t*, bf16_t*, const bf16_t*, const bf16_t*, bf16_t*,
                     float*, float*, int, int, float, bool, hipStream_t);
void launch_norm_bwd(const bf16_t*, const bf16_t*, const bf16_t*, const float*, const float*,
                     const bf16_t*, bf16_t*, float*, float*, bf16_t*, bf16_t*, int, int, bool,
                     hipStream_t);
int norm_bwd_grid(int rows);
int norm_wgrad_scratch_rows();
void launch_swiglu_fwd(const bf16_t*, bf16_t*, int64_t, int, hipStream_t);
void launch_swiglu_bwd(const bf16_t*, const bf16_t*, bf16_t*, int64_t, int, hipStream_t);
void launch_swiglu_fwd_t(const bf16_t*, bf16_t*, bf16_t*, int64_t, int, hipStream_t);
void launch_swiglu_bwd_t(const bf16_t*, const bf16_t*, bf16_t*, bf16_t*, int64_t, int, hipStream_t);
void launch_gelu_fwd(const bf16_t*, bf16_t*, int64_t, hipStream_t);
void launch_gelu_bwd(const bf16_t*, const bf16_t*, bf16_t*, int64_t, hipStream_t);
void launch_rope_fwd(const bf16_t*, int64_t, bf16_t*, bf16_t*, const float*, const float*,
                     const int*, int64_t, int, int, int, int, int, int, hipStream_t);
void launch_rope_bwd(const bf16_t*, const bf16_t*, bf16_t*, int64_t, const float*, const float*,
                     const int*, int64_t, int, int, int, int, int, int, hipStream_t);
void launch_logprob_fwd(const bf16_t*, int64_t, int, int64_t, int64_t, const int64_t*, float*,
                        float*, hipStream_t);
void launch_logprob_bwd(bf16_t*, int64_t, int, int64_t, int64_t, const int64_t*, const float*,
                        const float*, hipStream_t);
void launch_row_lse(const bf16_t*, int64_t, int, int64_t, float*, hipStream_t);
bool launch_logprob_bwd_t(bf16_t*, int64_t, int, int64_t, int64_t, const int64_t*, const float*,
                          const float*, bf16_t*, hipStream_t);
void launch_ensemble_kl(bf16_t*, const bf16_t*, int64_t, int64_t, int, int, const float*,
                        const float*, int64_t, const float*, float*, bool, hipStream_t);
void launch_seq_reduce(const float*, const float*, int, int, float*, float*, hipStream_t);
void launch_seq_expand_grad(const float*, const float*, const float*, int, int, bool, float*,
                            hipStream_t);
void launch_dpo_loss(const float*, const float*, int, float, float, float*, float*, float*,
                     float*, hipStream_t);
void launch_pairwise_loss(const float*, const float*, int, float*, float*, float*, float*,
                          hipStream_t);
void launch_kl_penalty_pg(const float*, const float*, const float*, int, float, float*, float*,
                          float*, float*, hipStream_t);
void launch_gae(const float*, const float*, const float*, int, int, float, float, float*, float*,
                hipStream_t);
void launch_ppo_policy_loss(const float*, const float*, const float*, const float*, int64_t, float,
                            float*, float*, float*, hipStream_t);
void launch_ppo_value_loss(const float*, const float*, const float*, const float*, int64_t, float,
                           float*, float*, hipStream_t);
void launch_adamw(bf16_t*, float*, const void*, bool, float*, float*, int64_t, float, float,
                  float, float, float, int, const float*, float, hipStream_t);
void launch_grad_sumsq(const void*, bool, int64_t, float*, float*, bool, hipStream_t);
int sumsq_grid(int64_t n);
void launch_clip_coef(const float*, float, float*, float*, hipStream_t);

void launch_attn_fwd(const AttnParams&, int, bool, hipStream_t);
int attn_fwd_set_switch(const char* name, int value);
void launch_attn_bwd_delta(const bf16_t*, const bf16_t*, int64_t, int64_t, int64_t, int64_t,
                           int64_t, int64_t, int, int, int, int, float*, hipStream_t);
void launch_attn_bwd(const AttnBwdParams&, int, bool, hipStream_t);
bool attn_dkv_part_bf16();
bool attn_dq_slab_bf16();
void launch_attn_dq_reduce(const float*, int, int, int, int, int, int, bool, int, int,
                           const int*, const int*, int, bf16_t*, int64_t, int64_t, int64_t,
                           const float*, const float*, const int*, int, hipStream_t, const bf16_t*);
void launch_attn_dkv_reduce(const float*, const float*, int, int, int, int, int, float, bf16_t*,
                            int64_t, int64_t, int64_t, bf16_t*, int64_t, int64_t, int64_t,
                            const float*, const float*, const int*, int, hipStream_t, const bf16_t*,
                            const bf16_t*);
void launch_transpose_bf16(const bf16_t*, int64_t, int64_t, int64_t, bf16_t*, int64_t, hipStream_t);

// ================================= norms ======================================================
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> norm_fwd(
    const at::Tensor& x, const c10::optional<at::Tensor>& res, const at::Tensor& w,
    const c10::optional<at::Tensor>& b, double eps, bool rms) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  TORCH_CHECK(x.is_contiguous(), "x must be contiguous");
  const int64_t H = x.size(-1);
  // forward kernels cover H <= 8192 (wave per row, 16 x 8 columns per lane)
  TORCH_CHECK(H % 8 == 0 && H <= 8192, "norm_fwd: hidden size must be a multiple of 8 and <= 8192");
  TORCH_CHECK(w.numel() == H && w.is_contiguous(), "w shape");
  const int64_t rows = x.numel() / H;
  TORCH_CHECK(rows < (1ll << 31), "too many rows");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto y = at::empty_like(x);
  at::Tensor so;
  const bf16_t* rptr = nullptr;
  if (res && res->defined()) {
    check_bf16(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous(), "res shape");
    so = at::empty_like(x);
    rptr = cbp(*res);
  }
  const bf16_t* bptr = nullptr;
  if (b && b->defined()) {
    check_bf16(*b, "b");
    TORCH_CHECK(b->numel() == H && b->is_contiguous(), "b shape");
    bptr = cbp(*b);
  }
  auto opt = x.options().dtype(at::kFloat);
  auto rstd = at::empty({rows}, opt);
  auto mean = rms ? at::empty({0}, opt) : at::empty({rows}, opt);
  check_aligned16(x, "x");
  launch_norm_fwd(cbp(x), rptr, so.defined() ? bp(so) : nullptr, cbp(w), bptr, bp(y),
                  rstd.data_ptr<float>(), rms ? nullptr : mean.data_ptr<float>(),
                  static_cast<int>(rows), static_cast<int>(H), static_cast<float>(eps), rms,
                  cur_stream(x));
  return {y, so.defined() ? so : at::empty({0}, x.options()), rstd, mean};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> norm_bwd(const at::Tensor& dy, const at::Tensor& s,
                                                        const at::Tensor& w,
                                                        const at::Tensor& rstd,
                                                        const c10::optional<at::Tensor>& mean,
                                                        const c10::optional<at::Tensor>& dres,
                                                        bool has_bias, bool rms) {
  check_bf16(dy, "dy");
  check_bf16(s, "s");
  check_bf16(w, "w");
  check_f32(rstd, "rstd");
  TORCH_CHECK(dy.is_contiguous() && s.is_contiguous() && dy.sizes() == s.sizes(), "dy/s shape");
  const int64_t H = s.size(-1);
  const int64_t rows = s.numel() / H;
  TORCH_CHECK(H % 8 == 0 && H <= 16384, "hidden size");
  TORCH_CHECK(rstd.numel() == rows, "rstd shape");
  const float* mptr = nullptr;
  if (!rms) {
    TORCH_CHECK(mean && mean->defined() && mean->numel() == rows, "LayerNorm needs mean");
    mptr = mean->data_ptr<float>();
  }
  const bf16_t* dr = nullptr;
  if (dres && dres->defined()) {
    check_bf16(*dres, "dres");
    TORCH_CHECK(dres->sizes() == s.sizes() && dres->is_contiguous(), "dres shape");
    dr = cbp(*dres);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(s.device());
  auto ds = at::empty_like(s);
  const int grid = norm_bwd_grid(static_cast<int>(rows));
  auto fopt = s.options().dtype(at::kFloat);
  const int srows = grid + norm_wgrad_scratch_rows();  // partials + stage-1 scratch
  auto dwp = at::empty({srows, H}, fopt);
  auto dbp = has_bias ? at::empty({srows, H}, fopt) : at::empty({0}, fopt);
  auto dw = at::empty({H}, w.options());
  auto db = has_bias ? at::empty({H}, w.options()) : at::empty({0}, w.options());
  launch_norm_bwd(cbp(dy), cbp(s), cbp(w), rstd.data_ptr<float>(), mptr, dr, bp(ds),
                  dwp.data_ptr<float>(), has_bias ? dbp.data_ptr<float>() : nullptr, bp(dw),
                  has_bias ? bp(db) : nullptr, static_cast<int>(rows), static_cast<int>(H), rms,
                  cur_stream(s));
  return {ds, dw, db};
}

// ================================= activations ================================================
at::Tensor swiglu_fwd(const at::Tensor& gu) {
  check_bf16(gu, "gu");
  TORCH_CHECK(gu.is_contiguous(), "gu contiguous");
  const int64_t two_f = gu.size(-1);
  TORCH_CHECK(two_f % 16 == 0, "2F must be a multiple of 16");
  const int64_t F = two_f / 2, rows = gu.numel() / two_f;
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
  auto out = at::empty(sizes, gu.options());
  launch_swiglu_fwd(cbp(gu), bp(out), rows, static_cast<int>(F), cur_stream(gu));
  return out;
}

at::Tensor swiglu_bwd(const at::Tensor& gu, const at::Tensor& dout) {
  check_bf16(gu, "gu");
  check_bf16(dout, "dout");
  TORCH_CHECK(gu.is_contiguous() && dout.is_contiguous(), "contiguous");
  const int64_t two_f = gu.size(-1), F = two_f / 2, rows = gu.numel() / two_f;
  TORCH_CHECK(two_f % 16 == 0 && dout.numel() == rows * F, "shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
  auto dgu = at::empty_like(gu);
  launch_swiglu_bwd(cbp(gu), cbp(dout), bp(dgu), rows, static_cast<int>(F), cur_stream(gu));
  return dgu;
}

// SwiGLU that also writes the transposed output ([F, rows]) for the TN weight-gradient GEMMs.
std::tuple<at::Tensor, at::Tensor> swiglu_fwd_t(const at::Tensor& gu) {
  check_bf16(gu, "gu");
  TORCH_CHECK(gu.is_contiguous() && gu.dim() == 2, "gu: contiguous [rows, 2F]");
  const int64_t rows = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(gu.size(1) == 2 * F && F % 64 == 0, "F must be a multiple of 64");
  c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
  auto out = at::empty({rows, F}, gu.options());
  auto outT = at::empty({F, rows}, gu.options());
  launch_swiglu_fwd_t(cbp(gu), bp(out), bp(outT), rows, static_cast<int>(F), cur_stream(gu));
  return {out, outT};
}

std::tuple<at::Tensor, at::Tensor> swiglu_bwd_t(const at::Tensor& gu, const at::Tensor& dout) {
  check_bf16(gu, "gu");
  check_bf16(dout, "dout");
  TORCH_CHECK(gu.is_contiguous() && dout.is_contiguous() && gu.dim() == 2, "contiguous 2-D");
  const int64_t rows = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(gu.size(1) == 2 * F && F % 64 == 0 && dout.numel() == rows * F, "shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
  auto dgu = at::empty_like(gu);
  auto dguT = at::empty({2 * F, rows}, gu.options());
  launch_swiglu_bwd_t(cbp(gu), cbp(dout), bp(dgu), bp(dguT), rows, static_cast<int>(F),
                      cur_stream(gu));
  return {dgu, dguT};
}

at::Tensor gelu_fwd(const at::Tensor& x) {
  check_bf16(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.numel() % 8 == 0, "x contiguous, numel % 8");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto y = at::empty_like(x);
  launch_gelu_fwd(cbp(x), bp(y), x.numel(), cur_stream(x));
  return y;
}

at::Tensor gelu_bwd(const at::Tensor& x, const at::Tensor& dy) {
  check_bf16(x, "x");
  check_bf16(dy, "dy");
  TORCH_CHECK(x.is_contiguous() && dy.is_contiguous() && x.numel() == dy.numel() &&
                  x.numel() % 8 == 0,
              "shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto dx = at::empty_like(x);
  launch_gelu_bwd(cbp(x), cbp(dy), bp(dx), x.numel(), cur_stream(x));
  return dx;
}

// ================================= rope =======================================================
static void check_rope_common(const at::Tensor& cos_t, const at::Tensor& sin_t,
                              const c10::optional<at::Tensor>& pos, int64_t tokens, int64_t D,
                              int64_t rot) {
  check_f32(cos_t, "cos");
  check_f32(sin_t, "sin");
  TORCH_CHECK(cos_t.is_contiguous() && sin_t.is_contiguous() && cos_t.dim() == 2 &&
                  cos_t.sizes() == sin_t.sizes() && cos_t.size(1) == rot / 2,
              "cos/sin tables must be [max_pos, rot/2]");
  TORCH_CHECK(D % 8 == 0 && rot % 16 == 0 && rot <= D, "rot must be a multiple of 16 <= D");
  if (pos && pos->defined()) {
    TORCH_CHECK(pos->scalar_type() == at::kInt && pos->is_contiguous() && pos->numel() == tokens,
                "pos must be int32 [tokens]");
  }
}

std::tuple<at::Tensor, at::Tensor> rope_fwd(const at::Tensor& qkv, const at::Tensor& cos_t,
                                            const at::Tensor& sin_t,
                                            const c10::optional<at::Tensor>& pos, int64_t Hq,
                                            int64_t Hkv, int64_t D, int64_t rot, int64_t T,
                                            int64_t pos_offset) {
  check_bf16(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1, "qkv must be [tokens, C] with unit col stride");
  TORCH_CHECK(qkv.size(1) >= (Hq + 2 * Hkv) * D, "qkv width");
  TORCH_CHECK(qkv.stride(0) % 8 == 0, "qkv row stride must be a multiple of 8");
  const int64_t tokens = qkv.size(0);
  TORCH_CHECK(T > 0 && tokens % T == 0, "tokens must be a multiple of T");
  check_rope_common(cos_t, sin_t, pos, tokens, D, rot);
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  auto q = at::empty({tokens, Hq * D}, qkv.options());
  auto k = at::empty({tokens, Hkv * D}, qkv.options());
  launch_rope_fwd(cbp(qkv), qkv.stride(0), bp(q), bp(k), cos_t.data_ptr<float>(),
                  sin_t.data_ptr<float>(),
                  (pos && pos->defined()) ? pos->data_ptr<int>() : nullptr, tokens,
                  static_cast<int>(T), static_cast<int>(pos_offset), static_cast<int>(Hq),
                  static_cast<int>(Hkv), static_cast<int>(D), static_cast<int>(rot),
                  cur_stream(qkv));
  return {q, k};
}

void rope_bwd(const at::Tensor& dq, const at::Tensor& dk, at::Tensor& dqkv,
              const at::Tensor& cos_t, const at::Tensor& sin_t,
              const c10::optional<at::Tensor>& pos, int64_t Hq, int64_t Hkv, int64_t D,
              int64_t rot, int64_t T, int64_t pos_offset) {
  check_bf16(dq, "dq");
  check_bf16(dk, "dk");
  check_bf16(dqkv, "dqkv");
  const int64_t tokens = dqkv.size(0);
  TORCH_CHECK(dq.is_contiguous() && dk.is_contiguous() && dq.numel() == tokens * Hq * D &&
                  dk.numel() == tokens * Hkv * D,
              "dq/dk shape");
  TORCH_CHECK(dqkv.dim() == 2 && dqkv.stride(1) == 1 && dqkv.stride(0) % 8 == 0 &&
                  dqkv.size(1) >= (Hq + 2 * Hkv) * D,
              "dqkv layout");
  TORCH_CHECK(T > 0 && tokens % T == 0, "tokens must be a multiple of T");
  check_rope_common(cos_t, sin_t, pos, tokens, D, rot);
  c10::hip::HIPGuardMasqueradingAsCUDA g(dqkv.device());
  launch_rope_bwd(cbp(dq), cbp(dk), bp(dqkv), dqkv.stride(0), cos_t.data_ptr<float>(),
                  sin_t.data_ptr<float>(),
                  (pos && pos->defined()) ? pos->data_ptr<int>() : nullptr, tokens,
                  static_cast<int>(T), static_cast<int>(pos_offset), static_cast<int>(Hq),
                  static_cast<int>(Hkv), static_cast<int>(D), static_cast<int>(rot),
                  cur_stream(dqkv));
}

// ================================= attention ==================================================
static void check_bthd(const at::Tensor& t, const char* name) {
  check_bf16(t, name);
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1, name, " must be [B, T, H, D] with unit d stride");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0, name,
              " strides must be multiples of 8 elements");
  check_aligned16(t, name);
}

static void check_kv_range(const c10::optional<at::Tensor>& r, int64_t B, const char* name) {
  if (r && r->defined()) {
    TORCH_CHECK(r->scalar_type() == at::kInt && r->is_contiguous() && r->numel() == B && r->is_cuda(),
                name, " must be int32 [B] on GPU");
  }
}

// packed-sequence bounds [2, B, T] int32 (seg_start; seg_end), causal self-attention only
static const int* seg_ptr(const c10::optional<at::Tensor>& segs, int64_t B, int64_t Tq, int64_t Tk,
                          bool causal, int64_t causal_off, const at::Tensor& q, int row) {
  if (!segs || !segs->defined()) return nullptr;
  TORCH_CHECK(segs->scalar_type() == at::kInt && segs->is_contiguous() && segs->dim() == 3 &&
                  segs->size(0) == 2 && segs->size(1) == B && segs->size(2) == Tq,
              "segs must be contiguous int32 [2, B, T]");
  TORCH_CHECK(causal && causal_off == 0 && Tq == Tk, "packed sequences need causal self-attention");
  same_device(q, *segs);
  return segs->data_ptr<int>() + row * B * Tq;
}

// rotary tables for the fused RoPE paths: contiguous fp32 [max_pos, D/2] cos / sin, optional
// int32 [B*T] positions (else position = t); full rotary, self-attention only
static void rope_args(const c10::optional<at::Tensor>& rope_cos, const c10::optional<at::Tensor>& rope_sin,
                      const c10::optional<at::Tensor>& rope_pos, const at::Tensor& q, int64_t B,
                      int64_t Tq, int64_t Tk, int64_t D, int64_t causal_off, const float** cos_p,
                      const float** sin_p, const int** pos_p, int* rot_p = nullptr) {
  *cos_p = *sin_p = nullptr;
  *pos_p = nullptr;
  if (rot_p) *rot_p = 0;
  if (!rope_cos || !rope_cos->defined()) return;
  TORCH_CHECK(rope_sin && rope_sin->defined(), "rope_sin missing");
  // full rotary, or (backward only: rot_p given) phi-2's partial rotary, 32 of D = 80 dims
  const int64_t half = rope_cos->dim() == 2 ? rope_cos->size(1) : -1;
  const bool partial_ok = rot_p != nullptr && D == 80 && half == 16;
  for (const at::Tensor* t : {&*rope_cos, &*rope_sin}) {
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->dim() == 2 &&
                    (t->size(1) == D / 2 || (partial_ok && t->size(1) == 16)),
                "rope cos/sin must be contiguous fp32 [max_pos, head_dim/2] (or [max_pos, 16] at "
                "head_dim 80 in the backward)");
    same_device(q, *t);
  }
  if (rot_p) *rot_p = static_cast<int>(2 * half);
  TORCH_CHECK(Tq == Tk && causal_off == 0, "fused RoPE needs self-attention");
  if (rope_pos && rope_pos->defined()) {
    TORCH_CHECK(rope_pos->scalar_type() == at::kInt && rope_pos->is_contiguous() &&
                    rope_pos->numel() == B * Tq, "rope_pos must be contiguous int32 [B*T]");
    same_device(q, *rope_pos);
    *pos_p = rope_pos->data_ptr<int>();
  } else {
    TORCH_CHECK(Tq <= rope_cos->size(0), "positions exceed the rotary table");
  }
  *cos_p = rope_cos->data_ptr<float>();
  *sin_p = rope_sin->data_ptr<float>();
}

static at::Tensor& attn_stamp_buffer() {
  static at::Tensor buf;
  return buf;
}

at::Tensor attn_stamps(const at::Tensor& like) {
  (void)like;
  return attn_stamp_buffer().defined() ? attn_stamp_buffer().clone() : at::Tensor();
}

std::tuple<at::Tensor, at::Tensor> attn_fwd(const at::Tensor& q, const at::Tensor& k,
                                            const at::Tensor& v, double scale, bool causal,
                                            int64_t causal_off, int64_t window,
                                            const c10::optional<at::Tensor>& kv_start,
                                            const c10::optional<at::Tensor>& kv_end,
                                            const c10::optional<at::Tensor>& segs,
                                            const c10::optional<at::Tensor>& rope_cos,
                                            const c10::optional<at::Tensor>& rope_sin,
                                            const c10::optional<at::Tensor>& rope_pos,
                                            const c10::optional<at::Tensor>& q_rot, bool rope_k) {
  check_bthd(q, "q");
  check_bthd(k, "k");
  check_bthd(v, "v");
  same_device(q, k);
  same_device(q, v);
  const int64_t B = q.size(0), Tq = q.size(1), Hq = q.size(2), D = q.size(3);
  const int64_t Tk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(D == 64 || D == 80 || D == 128, "head_dim must be 64, 80 or 128 (pad others)");
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && k.size(3) == D && v.size(3) == D &&
                  v.size(1) == Tk && v.size(2) == Hkv,
              "k/v shapes");
  TORCH_CHECK(Hkv > 0 && Hq % Hkv == 0, "Hq must be a multiple of Hkv");
  check_kv_range(kv_start, B, "kv_start");
  check_kv_range(kv_end, B, "kv_end");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  auto o = at::empty({B, Tq, Hq, D}, q.options());
  auto lse2 = at::empty({B, Hq, Tq}, q.options().dtype(at::kFloat));
  AttnParams p{};
  p.q = cbp(q);
  p.k = cbp(k);
  p.v = cbp(v);
  p.o = bp(o);
  p.lse2 = lse2.data_ptr<float>();
  p.q_sb = q.stride(0); p.q_st = q.stride(1); p.q_sh = q.stride(2);
  p.k_sb = k.stride(0); p.k_st = k.stride(1); p.k_sh = k.stride(2);
  p.v_sb = v.stride(0); p.v_st = v.stride(1); p.v_sh = v.stride(2);
  p.o_sb = o.stride(0); p.o_st = o.stride(1); p.o_sh = o.stride(2);
  p.B = B; p.Hq = Hq; p.Hkv = Hkv; p.Tq = Tq; p.Tk = Tk;
  p.scale2 = static_cast<float>(scale * 1.4426950408889634);
  p.causal_off = static_cast<int>(causal_off);
  p.window = static_cast<int>(window);
  p.kv_start = (kv_start && kv_start->defined()) ? kv_start->data_ptr<int>() : nullptr;
  p.kv_end = (kv_end && kv_end->defined()) ? kv_end->data_ptr<int>() : nullptr;
  p.seg_start = seg_ptr(segs, B, Tq, Tk, causal, causal_off, q, 0);
  rope_args(rope_cos, rope_sin, rope_pos, q, B, Tq, Tk, D, causal_off, &p.rope_cos, &p.rope_sin,
            &p.rope_pos);
  TORCH_CHECK(p.rope_cos == nullptr || D != 80, "RoPE on load: full-rotary head dims 64 / 128 only");
  p.rope_k = rope_k ? 1 : 0;
  if (q_rot && q_rot->defined()) {
    TORCH_CHECK(p.rope_cos != nullptr, "q_rot needs the rotary tables");
    check_bthd(*q_rot, "q_rot");
    TORCH_CHECK(q_rot->sizes() == q.sizes(), "q_rot shape");
    same_device(q, *q_rot);
    p.q_rot = bp(*q_rot);
    p.qr_sb = q_rot->stride(0); p.qr_st = q_rot->stride(1); p.qr_sh = q_rot->stride(2);
  }
  static const bool stamps = [] {
    const char* e = std::getenv("DLA_ATTN_STAMPS");
    return e != nullptr && std::atoi(e) == 1;
  }();
  if (stamps) {  // debug: read back with attn_stamps()
    auto& buf = attn_stamp_buffer();
    if (!buf.defined() || buf.device() != q.device())
      buf = at::zeros({1024 * 8 * 4}, q.options().dtype(at::kLong));
    p.stamps = reinterpret_cast<unsigned long long*>(buf.data_ptr<int64_t>());
  }
  launch_attn_fwd(p, static_cast<int>(D), causal, cur_stream(q));
  return {o, lse2};
}

static int device_cus(int dev) {
  static int cache[64] = {0};
  if (dev < 0 || dev >= 64) return 256;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// GQA heads of one kv head split across `hs` backward workgroups when the (key block x kv head x
// batch) grid alone would under-fill the chip: causal key blocks carry unequal work (block 0
// sees every query), so target two workgroups per CU there and let the heaviest-first dispatch
// balance them. Partial dK/dV of the splits are summed by a reduce pass.
static int attn_bwd_hsplit(int64_t nkb, int64_t Hkv, int64_t B, int64_t group, bool causal, int cus) {
  const int64_t base = nkb * Hkv * B;
  const int64_t target = causal ? 2 * static_cast<int64_t>(cus) : cus;
  int hs = 1;
  while (base * hs < target && group % (2 * hs) == 0) hs *= 2;
  return hs;
}

// dq / dk / dv are written into the given (possibly strided, e.g. fused-dqkv) bf16 outputs
void attn_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k,
              const at::Tensor& v, const at::Tensor& o, const at::Tensor& lse2, at::Tensor& dq,
              at::Tensor& dk, at::Tensor& dv, double scale, bool causal, int64_t causal_off,
              int64_t window, const c10::optional<at::Tensor>& kv_start,
              const c10::optional<at::Tensor>& kv_end, const c10::optional<at::Tensor>& segs,
              const c10::optional<at::Tensor>& rope_cos, const c10::optional<at::Tensor>& rope_sin,
              const c10::optional<at::Tensor>& rope_pos, bool rope_inputs) {
  check_bthd(dout, "dout");
  check_bthd(q, "q");
  check_bthd(k, "k");
  check_bthd(v, "v");
  check_bthd(o, "o");
  check_bthd(dq, "dq");
  check_bthd(dk, "dk");
  check_bthd(dv, "dv");
  check_f32(lse2, "lse2");
  const int64_t B = q.size(0), Tq = q.size(1), Hq = q.size(2), D = q.size(3);
  const int64_t Tk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(D == 64 || D == 80 || D == 128, "head_dim must be 64, 80 or 128");
  TORCH_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes() && dq.sizes() == q.sizes(),
              "dout/o/dq shape");
  TORCH_CHECK(dk.sizes() == k.sizes() && dv.sizes() == v.sizes(), "dk/dv shape");
  TORCH_CHECK(lse2.is_contiguous() && lse2.numel() == B * Hq * Tq, "lse2 shape");
  TORCH_CHECK(Hkv > 0 && Hq % Hkv == 0, "GQA ratio");
  check_kv_range(kv_start, B, "kv_start");
  check_kv_range(kv_end, B, "kv_end");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  auto st = cur_stream(q);
  auto fopt = q.options().dtype(at::kFloat);
  auto delta = at::empty({B, Hq, Tq}, fopt);
  launch_attn_bwd_delta(cbp(o), cbp(dout), o.stride(0), o.stride(1), o.stride(2),
                        dout.stride(0), dout.stride(1), dout.stride(2), B, Hq, Tq, D,
                        delta.data_ptr<float>(), st);
  const int64_t nkb = (Tk + kAttnBwdKeys - 1) / kAttnBwdKeys;
  // one fp32 dQ partial per key block (no zero fill: the reduce pass reads exactly the rows
  // each key block's workgroups wrote)
  const int64_t slab_rows = (Tq + kAttnBwdQRows - 1) / kAttnBwdQRows * kAttnBwdQRows;
  const bool slab16 = attn_dq_slab_bf16();
  auto slab = at::empty({std::max<int64_t>(nkb, 1), B, slab_rows, Hq, D}, slab16 ? q.options() : fopt);
  const int hs = attn_bwd_hsplit(nkb, Hkv, B, Hq / Hkv, causal, device_cus(q.get_device()));
  at::Tensor dkp, dvp;
  const bool part16 = hs > 1 && attn_dkv_part_bf16();
  if (hs > 1) {
    dkp = at::empty({hs, B, Tk, Hkv, D}, part16 ? q.options() : fopt);
    dvp = at::empty({hs, B, Tk, Hkv, D}, part16 ? q.options() : fopt);
  }
  AttnBwdParams p{};
  p.q = cbp(q); p.k = cbp(k); p.v = cbp(v); p.dout = cbp(dout);
  p.lse2 = lse2.data_ptr<float>(); p.delta = delta.data_ptr<float>();
  p.dq_slab = slab16 ? nullptr : slab.data_ptr<float>();
  p.dq_slab16 = slab16 ? bp(slab) : nullptr;
  p.dk_part = hs > 1 && !part16 ? dkp.data_ptr<float>() : nullptr;
  p.dv_part = hs > 1 && !part16 ? dvp.data_ptr<float>() : nullptr;
  p.dk_part16 = part16 ? bp(dkp) : nullptr;
  p.dv_part16 = part16 ? bp(dvp) : nullptr;
  p.dk = bp(dk); p.dv = bp(dv);
  p.hsplit = hs;
  p.slab_rows = static_cast<int>(slab_rows);
  p.q_sb = q.stride(0); p.q_st = q.stride(1); p.q_sh = q.stride(2);
  p.k_sb = k.stride(0); p.k_st = k.stride(1); p.k_sh = k.stride(2);
  p.v_sb = v.stride(0); p.v_st = v.stride(1); p.v_sh = v.stride(2);
  p.do_sb = dout.stride(0); p.do_st = dout.stride(1); p.do_sh = dout.stride(2);
  p.dk_sb = dk.stride(0); p.dk_st = dk.stride(1); p.dk_sh = dk.stride(2);
  p.dv_sb = dv.stride(0); p.dv_st = dv.stride(1); p.dv_sh = dv.stride(2);
  p.B = B; p.Hq = Hq; p.Hkv = Hkv; p.Tq = Tq; p.Tk = Tk;
  p.scale = static_cast<float>(scale);
  p.scale2 = static_cast<float>(scale * 1.4426950408889634);
  p.causal_off = static_cast<int>(causal_off);
  p.window = static_cast<int>(window);
  p.kv_start = (kv_start && kv_start->defined()) ? kv_start->data_ptr<int>() : nullptr;
  p.kv_end = (kv_end && kv_end->defined()) ? kv_end->data_ptr<int>() : nullptr;
  p.seg_end = seg_ptr(segs, B, Tq, Tk, causal, causal_off, q, 1);
  // fused RoPE backward: dq / dk receive the un-rotated gradients (full rotary only); with
  // rope_inputs q / k are also un-rotated and get rotated as they are staged
  rope_args(rope_cos, rope_sin, rope_pos, q, B, Tq, Tk, D, causal_off, &p.rope_cos, &p.rope_sin,
            &p.rope_pos, &p.rope_rot);
  TORCH_CHECK(!rope_inputs || p.rope_cos != nullptr, "rope_inputs needs the rotary tables");
  TORCH_CHECK(!rope_inputs || p.rope_rot == D, "rope_inputs (RoPE on load): full rotary only");
  p.rope_inputs = rope_inputs ? 1 : 0;
  launch_attn_bwd(p, static_cast<int>(D), causal, st);
  launch_attn_dq_reduce(p.dq_slab, static_cast<int>(nkb), static_cast<int>(B), static_cast<int>(Tq),
                        p.slab_rows, static_cast<int>(Hq), static_cast<int>(D), causal, p.causal_off, p.window,
                        p.kv_start, p.kv_end, static_cast<int>(Tk), bp(dq), dq.stride(0),
                        dq.stride(1), dq.stride(2), p.rope_cos, p.rope_sin, p.rope_pos, p.rope_rot, st,
                        p.dq_slab16);
  if (hs > 1) {
    launch_attn_dkv_reduce(p.dk_part, p.dv_part, hs, static_cast<int>(B), static_cast<int>(Tk),
                           static_cast<int>(Hkv), static_cast<int>(D), p.scale, bp(dk),
                           dk.stride(0), dk.stride(1), dk.stride(2), bp(dv), dv.stride(0),
                           dv.stride(1), dv.stride(2), p.rope_cos, p.rope_sin, p.rope_pos, p.rope_rot, st,
                           p.dk_part16, p.dv_part16);
  }
}

// out [C, R] <- in [R, C]^T (both row-major with unit column stride, 16-byte aligned rows)
void transpose_bf16(const at::Tensor& in, at::Tensor& out) {
  check_bf16(in, "in");
  check_bf16(out, "out");
  TORCH_CHECK(in.dim() == 2 && out.dim() == 2 && in.stride(1) == 1 && out.stride(1) == 1 &&
                  out.size(0) == in.size(1) && out.size(1) == in.size(0),
              "transpose_bf16: in [R, C], out [C, R], unit column stride");
  TORCH_CHECK(in.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "16-byte aligned rows");
  check_aligned16(in, "in");
  check_aligned16(out, "out");
  same_device(in, out);
  c10::hip::HIPGuardMasqueradingAsCUDA g(in.device());
  launch_transpose_bf16(cbp(in), in.size(0), in.size(1), in.stride(0), bp(out), out.stride(0),
                        cur_stream(in));
}

// ================================= vocab reductions ===========================================
static void check_logits(const at::Tensor& logits) {
  check_bf16(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be [N, V] row-major");
}

std::tuple<at::Tensor, at::Tensor> logprob_fwd(const at::Tensor& logits, const at::Tensor& tgt,
                                               int64_t vocab_offset) {
  check_logits(logits);
  TORCH_CHECK(tgt.scalar_type() == at::kLong && tgt.is_contiguous() && tgt.numel() == logits.size(0),
              "targets int64 [N]");
  same_device(logits, tgt);
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  auto opt = logits.options().dtype(at::kFloat);
  auto logp = at::empty({logits.size(0)}, opt);
  auto lse = at::empty({logits.size(0)}, opt);
  launch_logprob_fwd(cbp(logits), logits.stride(0), static_cast<int>(logits.size(1)),
                     vocab_offset, logits.size(0), tgt.data_ptr<int64_t>(), logp.data_ptr<float>(),
                     lse.data_ptr<float>(), cur_stream(logits));
  return {logp, lse};
}

void logprob_bwd(at::Tensor& logits, const at::Tensor& tgt, const at::Tensor& lse,
                 const at::Tensor& grad, int64_t vocab_offset) {
  check_logits(logits);
  check_f32(lse, "lse");
  check_f32(grad, "grad");
  const int64_t N = logits.size(0);
  TORCH_CHECK(tgt.scalar_type() == at::kLong && tgt.numel() == N && tgt.is_contiguous(), "targets");
  TORCH_CHECK(lse.numel() == N && grad.numel() == N && grad.is_contiguous(), "lse/grad shape");
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  launch_logprob_bwd(bp(logits), logits.stride(0), static_cast<int>(logits.size(1)), vocab_offset,
                     N, tgt.data_ptr<int64_t>(), lse.data_ptr<float>(), grad.data_ptr<float>(),
                     cur_stream(logits));
}

// logprob_bwd with the transposed gradient as a second output: logits <- dlogits (in place) and
// returns dlogitsT [V, N] (the LM head's TN weight-gradient operand). An empty tensor when the
// shape is outside the kernel (N, V or the row stride not a multiple of 8): run logprob_bwd.
at::Tensor logprob_bwd_t(at::Tensor& logits, const at::Tensor& tgt, const at::Tensor& lse,
                         const at::Tensor& grad, int64_t vocab_offset) {
  check_logits(logits);
  check_f32(lse, "lse");
  check_f32(grad, "grad");
  const int64_t N = logits.size(0), V = logits.size(1);
  TORCH_CHECK(tgt.scalar_type() == at::kLong && tgt.numel() == N && tgt.is_contiguous(), "targets");
  TORCH_CHECK(lse.numel() == N && grad.numel() == N && grad.is_contiguous() && lse.is_contiguous(),
              "lse/grad shape");
  if (N == 0 || N % 8 != 0 || V % 8 != 0 || logits.stride(0) % 8 != 0) return at::empty({0}, logits.options());
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  auto outT = at::empty({V, N}, logits.options());
  const bool ok = launch_logprob_bwd_t(bp(logits), logits.stride(0), static_cast<int>(V), N, vocab_offset,
                                       tgt.data_ptr<int64_t>(), lse.data_ptr<float>(), grad.data_ptr<float>(),
                                       bp(outT), cur_stream(logits));
  TORCH_CHECK(ok, "logprob_bwd_t: shape");
  return outT;
}

at::Tensor row_lse(const at::Tensor& logits) {
  check_logits(logits);
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  auto lse = at::empty({logits.size(0)}, logits.options().dtype(at::kFloat));
  launch_row_lse(cbp(logits), logits.stride(0), static_cast<int>(logits.size(1)), logits.size(0),
                 lse.data_ptr<float>(), cur_stream(logits));
  return lse;
}

// s_logits [N, V] (overwritten with dKL/dz * g when write_grad), t_logits [K, N, V] contiguous
at::Tensor ensemble_kl(at::Tensor& s_logits, const at::Tensor& t_logits, const at::Tensor& s_lse,
                       const at::Tensor& t_lse, const c10::optional<at::Tensor>& grad,
                       bool write_grad) {
  check_bf16(s_logits, "s_logits");
  check_bf16(t_logits, "t_logits");
  TORCH_CHECK(s_logits.is_contiguous() && t_logits.is_contiguous() && s_logits.dim() == 2 &&
                  t_logits.dim() == 3 && t_logits.size(1) == s_logits.size(0) &&
                  t_logits.size(2) == s_logits.size(1),
              "ensemble_kl shapes (shared vocab required)");
  const int64_t N = s_logits.size(0), K = t_logits.size(0);
  check_f32(s_lse, "s_lse");
  check_f32(t_lse, "t_lse");
  TORCH_CHECK(s_lse.numel() == N && t_lse.numel() == K * N && t_lse.is_contiguous(), "lse shapes");
  const float* gp = nullptr;
  if (write_grad) {
    TORCH_CHECK(grad && grad->defined() && grad->numel() == N, "grad required");
    check_f32(*grad, "grad");
    gp = grad->data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(s_logits.device());
  auto kl = at::empty({N}, s_logits.options().dtype(at::kFloat));
  launch_ensemble_kl(bp(s_logits), cbp(t_logits), s_logits.size(1), N * s_logits.size(1),
                     static_cast<int>(K), static_cast<int>(s_logits.size(1)),
                     s_lse.data_ptr<float>(), t_lse.data_ptr<float>(), N, gp,
                     kl.data_ptr<float>(), write_grad, cur_stream(s_logits));
  return kl;
}

// ================================= sequence objectives ========================================
std::tuple<at::Tensor, at::Tensor> seq_reduce(const at::Tensor& lp, const at::Tensor& mask) {
  check_f32(lp, "lp");
  check_f32(mask, "mask");
  TORCH_CHECK(lp.dim() == 2 && lp.is_contiguous() && mask.sizes() == lp.sizes() && mask.is_contiguous(),
              "lp/mask [S, T]");
  c10::hip::HIPGuardMasqueradingAsCUDA g(lp.device());
  auto sum = at::empty({lp.size(0)}, lp.options());
  auto cnt = at::empty({lp.size(0)}, lp.options());
  launch_seq_reduce(lp.data_ptr<float>(), mask.data_ptr<float>(), static_cast<int>(lp.size(0)),
                    static_cast<int>(lp.size(1)), sum.data_ptr<float>(), cnt.data_ptr<float>(),
                    cur_stream(lp));
  return {sum, cnt};
}

at::Tensor seq_expand_grad(const at::Tensor& coef, const at::Tensor& mask, const at::Tensor& cnt,
                           bool mean) {
  check_f32(coef, "coef");
  check_f32(mask, "mask");
  check_f32(cnt, "cnt");
  TORCH_CHECK(mask.dim() == 2 && mask.is_contiguous() && coef.numel() == mask.size(0) &&
                  cnt.numel() == mask.size(0) && coef.is_contiguous() && cnt.is_contiguous(),
              "shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(mask.device());
  auto out = at::empty_like(mask);
  launch_seq_expand_grad(coef.data_ptr<float>(), mask.data_ptr<float>(), cnt.data_ptr<float>(),
                         static_cast<int>(mask.size(0)), static_cast<int>(mask.size(1)), mean,
                         out.data_ptr<float>(), cur_stream(mask));
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> dpo_loss(const at::Tensor& pol,
                                                                    const at::Tensor& ref,
                                                                    double beta,
                                                                    double label_smoothing) {
  check_f32(pol, "pol");
  check_f32(ref, "ref");
  TORCH_CHECK(pol.is_contiguous() && ref.is_contiguous() && pol.numel() == ref.numel() &&
                  pol.numel() % 2 == 0,
              "pol/ref must be [2B] (chosen then rejected)");
  const int B = static_cast<int>(pol.numel() / 2);
  c10::hip::HIPGuardMasqueradingAsCUDA g(pol.device());
  auto opt = pol.options();
  auto loss = at::empty({}, opt);
  auto dpol = at::empty({2 * B}, opt);
  auto rewards = at::empty({2 * B}, opt);
  auto metrics = at::empty({4}, opt);
  launch_dpo_loss(pol.data_ptr<float>(), ref.data_ptr<float>(), B, static_cast<float>(beta),
                  static_cast<float>(label_smoothing), loss.data_ptr<float>(),
                  dpol.data_ptr<float>(), rewards.data_ptr<float>(), metrics.data_ptr<float>(),
                  cur_stream(pol));
  return {loss, dpol, rewards, metrics};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> pairwise_loss(const at::Tensor& sc,
                                                                         const at::Tensor& sr) {
  check_f32(sc, "sc");
  check_f32(sr, "sr");
  TORCH_CHECK(sc.is_contiguous() && sr.is_contiguous() && sc.numel() == sr.numel(), "shapes");
  const int B = static_cast<int>(sc.numel());
  c10::hip::HIPGuardMasqueradingAsCUDA g(sc.device());
  auto opt = sc.options();
  auto loss = at::empty({}, opt);
  auto dsc = at::empty({B}, opt);
  auto dsr = at::empty({B}, opt);
  auto acc = at::empty({}, opt);
  launch_pairwise_loss(sc.data_ptr<float>(), sr.data_ptr<float>(), B, loss.data_ptr<float>(),
                       dsc.data_ptr<float>(), dsr.data_ptr<float>(), acc.data_ptr<float>(),
                       cur_stream(sc));
  return {loss, dsc, dsr, acc};
}

// ---- PPO (actor-critic) token objectives: [S, T] fp32 grids ----
static void check_grid(const at::Tensor& t, const at::Tensor& like, const char* name) {
  check_f32(t, name);
  TORCH_CHECK(t.is_contiguous() && t.sizes() == like.sizes(), name, " must be a contiguous fp32 grid like the first operand");
}

std::tuple<at::Tensor, at::Tensor> gae(const at::Tensor& rewards, const at::Tensor& values,
                                       const at::Tensor& mask, double gamma, double lam) {
  check_f32(rewards, "rewards");
  TORCH_CHECK(rewards.dim() == 2 && rewards.is_contiguous(), "rewards [S, T] contiguous");
  check_grid(values, rewards, "values");
  check_grid(mask, rewards, "mask");
  c10::hip::HIPGuardMasqueradingAsCUDA g(rewards.device());
  auto adv = at::empty_like(rewards);
  auto ret = at::empty_like(rewards);
  launch_gae(rewards.data_ptr<float>(), values.data_ptr<float>(), mask.data_ptr<float>(),
             static_cast<int>(rewards.size(0)), static_cast<int>(rewards.size(1)),
             static_cast<float>(gamma), static_cast<float>(lam), adv.data_ptr<float>(),
             ret.data_ptr<float>(), cur_stream(rewards));
  return {adv, ret};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> ppo_policy_loss(const at::Tensor& lp,
                                                               const at::Tensor& old,
                                                               const at::Tensor& adv,
                                                               const at::Tensor& mask,
                                                               double eps) {
  check_f32(lp, "lp");
  TORCH_CHECK(lp.is_contiguous(), "lp contiguous");
  check_grid(old, lp, "old");
  check_grid(adv, lp, "adv");
  check_grid(mask, lp, "mask");
  c10::hip::HIPGuardMasqueradingAsCUDA g(lp.device());
  auto opt = lp.options();
  auto loss = at::empty({}, opt);
  auto dlp = at::empty_like(lp);
  auto metrics = at::empty({3}, opt);
  launch_ppo_policy_loss(lp.data_ptr<float>(), old.data_ptr<float>(), adv.data_ptr<float>(),
                         mask.data_ptr<float>(), lp.numel(), static_cast<float>(eps),
                         loss.data_ptr<float>(), dlp.data_ptr<float>(), metrics.data_ptr<float>(),
                         cur_stream(lp));
  return {loss, dlp, metrics};
}

std::tuple<at::Tensor, at::Tensor> ppo_value_loss(const at::Tensor& values, const at::Tensor& old,
                                                  const at::Tensor& returns,
                                                  const at::Tensor& mask, double clip) {
  check_f32(values, "values");
  TORCH_CHECK(values.is_contiguous(), "values contiguous");
  check_grid(old, values, "old");
  check_grid(returns, values, "returns");
  check_grid(mask, values, "mask");
  c10::hip::HIPGuardMasqueradingAsCUDA g(values.device());
  auto loss = at::empty({}, values.options());
  auto dval = at::empty_like(values);
  launch_ppo_value_loss(values.data_ptr<float>(), old.data_ptr<float>(), returns.data_ptr<float>(),
                        mask.data_ptr<float>(), values.numel(), static_cast<float>(clip),
                        loss.data_ptr<float>(), dval.data_ptr<float>(), cur_stream(values));
  return {loss, dval};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> kl_penalty_pg(const at::Tensor& lp,
                                                                         const at::Tensor& lr,
                                                                         const at::Tensor& reward,
                                                                         double kl_coef) {
  check_f32(lp, "lp");
  check_f32(lr, "lr");
  check_f32(reward, "reward");
  TORCH_CHECK(lp.is_contiguous() && lr.is_contiguous() && reward.is_contiguous() &&
                  lp.numel() == lr.numel() && lp.numel() == reward.numel() && lp.numel() > 0,
              "shapes");
  const int n = static_cast<int>(lp.numel());
  c10::hip::HIPGuardMasqueradingAsCUDA g(lp.device());
  auto opt = lp.options();
  auto loss = at::empty({}, opt);
  auto klm = at::empty({}, opt);
  auto dlp = at::empty({n}, opt);
  auto adv = at::empty({n}, opt);
  launch_kl_penalty_pg(lp.data_ptr<float>(), lr.data_ptr<float>(), reward.data_ptr<float>(), n,
                       static_cast<float>(kl_coef), loss.data_ptr<float>(), klm.data_ptr<float>(),
                       dlp.data_ptr<float>(), adv.data_ptr<float>(), cur_stream(lp));
  return {loss, klm, dlp, adv};
}

// ================================= optimizer ==================================================
void adamw_step(const c10::optional<at::Tensor>& param, const c10::optional<at::Tensor>& master,
                const at::Tensor& grad, at::Tensor& m, at::Tensor& v, double lr, double b1,
                double b2, double eps, double wd, int64_t step,
                const c10::optional<at::Tensor>& clip, double grad_scale) {
  const int64_t n = grad.numel();
  TORCH_CHECK(n % 8 == 0, "flat buffers must be padded to a multiple of 8 elements");
  TORCH_CHECK(grad.is_contiguous() && m.is_contiguous() && v.is_contiguous(), "contiguous");
  check_cuda(grad, "grad");
  TORCH_CHECK(grad.scalar_type() == at::kBFloat16 || grad.scalar_type() == at::kFloat,
              "grad must be bf16 or fp32");
  check_f32(m, "m");
  check_f32(v, "v");
  TORCH_CHECK(m.numel() == n && v.numel() == n, "m/v size");
  bf16_t* pp = nullptr;
  float* mp = nullptr;
  if (param && param->defined()) {
    check_bf16(*param, "param");
    TORCH_CHECK(param->is_contiguous() && param->numel() == n, "param size");
    pp = bp(*param);
  }
  if (master && master->defined()) {
    check_f32(*master, "master");
    TORCH_CHECK(master->is_contiguous() && master->numel() == n, "master size");
    mp = master->data_ptr<float>();
  }
  TORCH_CHECK(pp || mp, "need bf16 param or fp32 master");
  const float* cp = nullptr;
  if (clip && clip->defined()) {
    check_f32(*clip, "clip");
    cp = clip->data_ptr<float>();
  }
  TORCH_CHECK(step >= 1, "step must be >= 1");
  c10::hip::HIPGuardMasqueradingAsCUDA g(grad.device());
  launch_adamw(pp, mp, grad.data_ptr(), grad.scalar_type() == at::kBFloat16, m.data_ptr<float>(),
               v.data_ptr<float>(), n, static_cast<float>(lr), static_cast<float>(b1),
               static_cast<float>(b2), static_cast<float>(eps), static_cast<float>(wd),
               static_cast<int>(step), cp, static_cast<float>(grad_scale), cur_stream(grad));
}

void grad_sumsq(const at::Tensor& grad, at::Tensor& out, bool accumulate) {
  check_cuda(grad, "grad");
  check_f32(out, "out");
  TORCH_CHECK(grad.is_contiguous() && grad.numel() % 8 == 0, "grad contiguous, numel % 8");
  TORCH_CHECK(grad.scalar_type() == at::kBFloat16 || grad.scalar_type() == at::kFloat, "dtype");
  TORCH_CHECK(out.numel() >= 1, "out");
  c10::hip::HIPGuardMasqueradingAsCUDA g(grad.device());
  auto partial = at::empty({sumsq_grid(grad.numel())}, out.options());
  launch_grad_sumsq(grad.data_ptr(), grad.scalar_type() == at::kBFloat16, grad.numel(),
                    partial.data_ptr<float>(), out.data_ptr<float>(), accumulate,
                    cur_stream(grad));
}

std::tuple<at::Tensor, at::Tensor> clip_coef(const at::Tensor& sumsq, double max_norm) {
  check_f32(sumsq, "sumsq");
  c10::hip::HIPGuardMasqueradingAsCUDA g(sumsq.device());
  auto norm = at::empty({}, sumsq.options());
  auto coef = at::empty({}, sumsq.options());
  launch_clip_coef(sumsq.data_ptr<float>(), static_cast<float>(max_norm), norm.data_ptr<float>(),
                   coef.data_ptr<float>(), cur_stream(sumsq));
  return {norm, coef};
}

// Flip one attention-forward structure switch for this process (tests / same-binary A/B): the
// launcher reads DLA_ATTN_FWD_{PRIO,SGPR,PRO,OSTAGE,MSUB} once; returns the previous value.
int64_t attn_fwd_switch(c10::string_view name, int64_t value) {
  const std::string n(name.data(), name.size());
  const int prev = attn_fwd_set_switch(n.c_str(), static_cast<int>(value));
  TORCH_CHECK(prev != -1, "attn_fwd_switch: unknown switch ", n);
  return prev;
}

}  // namespace dla

TORCH_LIBRARY(dla, m) {
  m.def("norm_fwd(Tensor x, Tensor? res, Tensor w, Tensor? b, float eps, bool rms) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("norm_bwd(Tensor dy, Tensor s, Tensor w, Tensor rstd, Tensor? mean, Tensor? dres, bool has_bias, bool rms) -> (Tensor, Tensor, Tensor)");
  m.def("swiglu_fwd(Tensor gu) -> Tensor");
  m.def("swiglu_bwd(Tensor gu, Tensor dout) -> Tensor");
  m.def("swiglu_fwd_t(Tensor gu) -> (Tensor, Tensor)");
  m.def("swiglu_bwd_t(Tensor gu, Tensor dout) -> (Tensor, Tensor)");
  m.def("gelu_fwd(Tensor x) -> Tensor");
  m.def("gelu_bwd(Tensor x, Tensor dy) -> Tensor");
  m.def("rope_fwd(Tensor qkv, Tensor cos, Tensor sin, Tensor? pos, int Hq, int Hkv, int D, int rot, int T, int pos_offset) -> (Tensor, Tensor)");
  m.def("rope_bwd(Tensor dq, Tensor dk, Tensor(a!) dqkv, Tensor cos, Tensor sin, Tensor? pos, int Hq, int Hkv, int D, int rot, int T, int pos_offset) -> ()");
  m.def("attn_fwd(Tensor q, Tensor k, Tensor v, float scale, bool causal, int causal_off, int window, Tensor? kv_start, Tensor? kv_end, Tensor? segs=None, Tensor? rope_cos=None, Tensor? rope_sin=None, Tensor? rope_pos=None, Tensor(a!)? q_rot=None, bool rope_k=True) -> (Tensor, Tensor)");
  m.def("attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse2, Tensor(a!) dq, Tensor(b!) dk, Tensor(c!) dv, float scale, bool causal, int causal_off, int window, Tensor? kv_start, Tensor? kv_end, Tensor? segs=None, Tensor? rope_cos=None, Tensor? rope_sin=None, Tensor? rope_pos=None, bool rope_inputs=False) -> ()");
  m.def("attn_stamps(Tensor like) -> Tensor");
  m.def("attn_fwd_switch(str name, int value) -> int", &dla::attn_fwd_switch);
  m.def("transpose_bf16(Tensor input, Tensor(a!) out) -> ()");
  m.def("logprob_fwd(Tensor logits, Tensor targets, int vocab_offset=0) -> (Tensor, Tensor)");
  m.def("logprob_bwd(Tensor(a!) logits, Tensor targets, Tensor lse, Tensor grad, int vocab_offset=0) -> ()");
  m.def("logprob_bwd_t(Tensor(a!) logits, Tensor targets, Tensor lse, Tensor grad, int vocab_offset=0) -> Tensor");
  m.def("row_lse(Tensor logits) -> Tensor");
  m.def("ensemble_kl(Tensor(a!) s_logits, Tensor t_logits, Tensor s_lse, Tensor t_lse, Tensor? grad, bool write_grad) -> Tensor");
  m.def("seq_reduce(Tensor lp, Tensor mask) -> (Tensor, Tensor)");
  m.def("seq_expand_grad(Tensor coef, Tensor mask, Tensor cnt, bool mean) -> Tensor");
  m.def("dpo_loss(Tensor pol, Tensor ref, float beta, float label_smoothing) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("pairwise_loss(Tensor sc, Tensor sr) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("gae(Tensor rewards, Tensor values, Tensor mask, float gamma, float lam) -> (Tensor, Tensor)");
  m.def("ppo_policy_loss(Tensor lp, Tensor old, Tensor adv, Tensor mask, float eps) -> (Tensor, Tensor, Tensor)");
  m.def("ppo_value_loss(Tensor values, Tensor old, Tensor returns, Tensor mask, float clip) -> (Tensor, Tensor)");
  m.def("kl_penalty_pg(Tensor lp, Tensor lr, Tensor reward, float kl_coef) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("adamw_step(Tensor(a!)? param, Tensor(b!)? master, Tensor grad, Tensor(c!) m, Tensor(d!) v, float lr, float b1, float b2, float eps, float wd, int step, Tensor? clip, float grad_scale) -> ()");
  m.def("grad_sumsq(Tensor grad, Tensor(a!) out, bool accumulate) -> ()");
  m.def("clip_coef(Tensor sumsq, float max_norm) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(dla, CUDA, m) {
  m.impl("norm_fwd", &dla::norm_fwd);
  m.impl("norm_bwd", &dla::norm_bwd);
  m.impl("swiglu_fwd", &dla::swiglu_fwd);
  m.impl("swiglu_bwd", &dla::swiglu_bwd);
  m.impl("swiglu_fwd_t", &dla::swiglu_fwd_t);
  m.impl("swiglu_bwd_t", &dla::swiglu_bwd_t);
  m.impl("gelu_fwd", &dla::gelu_fwd);
  m.impl("gelu_bwd", &dla::gelu_bwd);
  m.impl("rope_fwd", &dla::rope_fwd);
  m.impl("rope_bwd", &dla::rope_bwd);
  m.impl("attn_fwd", &dla::attn_fwd);
  m.impl("attn_bwd", &dla::attn_bwd);
  m.impl("attn_stamps", &dla::attn_stamps);
  m.impl("transpose_bf16", &dla::transpose_bf16);
  m.impl("logprob_fwd", &dla::logprob_fwd);
  m.impl("logprob_bwd", &dla::logprob_bwd);
  m.impl("logprob_bwd_t", &dla::logprob_bwd_t);
  m.impl("row_lse", &dla::row_lse);
  m.impl("ensemble_kl", &dla::ensemble_kl);
  m.impl("seq_reduce", &dla::seq_reduce);
  m.impl("seq_expand_grad", &dla::seq_expand_grad);
  m.impl("dpo_loss", &dla::dpo_loss);
  m.impl("pairwise_loss", &dla::pairwise_loss);
  m.impl("kl_penalty_pg", &dla::kl_penalty_pg);
  m.impl("gae", &dla::gae);
  m.impl("ppo_policy_loss", &dla::ppo_policy_loss);
  m.impl("ppo_value_loss", &dla::ppo_value_loss);
  m.impl("adamw_step", &dla::adamw_step);
  m.impl("grad_sumsq", &dla::grad_sumsq);
  m.impl("clip_coef", &dla::clip_coef);
}
