// Host-side helpers shared by the torch op bindings (bindings*.cpp).
#pragma once
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <cstdint>

namespace dla {
using bf16_t = uint16_t;

// ---- helpers ----
inline hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}
inline bf16_t* bp(const at::Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }
inline const bf16_t* cbp(const at::Tensor& t) {
  return reinterpret_cast<const bf16_t*>(t.data_ptr());
}
inline void check_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}
inline void check_bf16(const at::Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
}
inline void check_f32(const at::Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
}
inline void check_aligned16(const at::Tensor& t, const char* name) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name,
              " must be 16-byte aligned");
}
inline void same_device(const at::Tensor& a, const at::Tensor& b) {
  TORCH_CHECK(a.device() == b.device(), "operands on different devices");
}

inline void check_i32(const at::Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kInt, name, " must be int32");
}

}  // namespace dla
