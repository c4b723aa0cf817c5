// torch.ops.dla MoE routing / permutation ops (kernels in moe.hip). Host-side validation only.
#include <ATen/ATen.h>
#include <torch/library.h>

#include <tuple>

#include "bind_util.h"

namespace dla {

void launch_moe_topk_fwd(const bf16_t*, int64_t, int, int, float*, int*, hipStream_t);
void launch_moe_topk_bwd(const float*, const int*, const float*, int64_t, int, int, bf16_t*,
                         hipStream_t);
void launch_moe_dispatch(const bf16_t*, const int*, int64_t, int, int, bf16_t*, hipStream_t);
void launch_moe_combine(const bf16_t*, const int*, const float*, int64_t, int, int, bf16_t*,
                        hipStream_t);
void launch_moe_combine_bwd(const bf16_t*, const bf16_t*, const int*, const float*, int64_t, int,
                            int, bf16_t*, float*, hipStream_t);

void launch_quant_fp8_rows(const bf16_t*, int64_t, int64_t, int, uint8_t*, float*, hipStream_t);

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

// The kernels trust pos[] to be a permutation of [0, N*k): verified cheaply on the device side
// by the caller's construction (ops/moe.py builds it from an argsort); rows are bounds-checked
// here through the output allocation size.
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
  TORCH_CHECK(ys.size(0) == N * k, "ys rows must equal N * k");
  const float* wp = nullptr;
  if (w && w->defined()) {
    check_f32(*w, "w");
    TORCH_CHECK(w->sizes() == pos.sizes() && w->is_contiguous(), "w [N, k]");
    wp = w->data_ptr<float>();
  }
  check_aligned16(ys, "ys");
  c10::hip::HIPGuardMasqueradingAsCUDA g(ys.device());
  auto out = at::empty({N, H}, ys.options());
  launch_moe_combine(cbp(ys), pos.data_ptr<int>(), wp, N, (int)H, (int)k, bp(out), cur_stream(ys));
  return out;
}

std::tuple<at::Tensor, at::Tensor> moe_combine_bwd(const at::Tensor& dout, const at::Tensor& ys,
                                                   const at::Tensor& pos, const at::Tensor& w) {
  check_bf16(dout, "dout");
  check_bf16(ys, "ys");
  check_f32(w, "w");
  const int64_t N = pos.size(0), k = pos.size(-1), H = ys.size(1);
  check_pos(pos, N, k);
  TORCH_CHECK(dout.dim() == 2 && dout.size(0) == N && dout.size(1) == H && dout.is_contiguous(),
              "dout [N, H]");
  TORCH_CHECK(ys.dim() == 2 && ys.size(0) == N * k && ys.is_contiguous() && H % 8 == 0, "ys [N*k, H]");
  TORCH_CHECK(w.sizes() == pos.sizes() && w.is_contiguous(), "w [N, k]");
  check_aligned16(ys, "ys");
  check_aligned16(dout, "dout");
  c10::hip::HIPGuardMasqueradingAsCUDA g(ys.device());
  auto dys = at::empty_like(ys);
  auto dw = at::empty({N, k}, w.options());
  launch_moe_combine_bwd(cbp(dout), cbp(ys), pos.data_ptr<int>(), w.data_ptr<float>(), N, (int)H,
                         (int)k, bp(dys), dw.data_ptr<float>(), cur_stream(ys));
  return {dys, dw};
}

}  // namespace dla

TORCH_LIBRARY_FRAGMENT(dla, m) {
  m.def("moe_topk_fwd(Tensor logits, int k) -> (Tensor, Tensor)");
  m.def("quant_fp8_rows(Tensor x) -> (Tensor, Tensor)");
  m.def("moe_topk_bwd(Tensor topv, Tensor topi, Tensor grad, int E) -> Tensor");
  m.def("moe_dispatch(Tensor x, Tensor pos) -> Tensor");
  m.def("moe_combine(Tensor ys, Tensor pos, Tensor? w) -> Tensor");
  m.def("moe_combine_bwd(Tensor dout, Tensor ys, Tensor pos, Tensor w) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(dla, CUDA, m) {
  m.impl("moe_topk_fwd", &dla::moe_topk_fwd);
  m.impl("quant_fp8_rows", &dla::quant_fp8_rows);
  m.impl("moe_topk_bwd", &dla::moe_topk_bwd);
  m.impl("moe_dispatch", &dla::moe_dispatch);
  m.impl("moe_combine", &dla::moe_combine);
  m.impl("moe_combine_bwd", &dla::moe_combine_bwd);
}
