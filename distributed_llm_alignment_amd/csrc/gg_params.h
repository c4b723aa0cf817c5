// Parameter block of the grouped expert GEMM (grouped_gemm.hip), shared with its torch binding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dla {

struct GGParams {
  const uint8_t* A;
  const uint8_t* B;
  void* C;
  const int* offs;  // [G + 1] exclusive prefix of the group row counts (device)
  int G;
  int64_t lda, ldb, ldc;  // row strides in ELEMENTS of the operand / output dtype
  int64_t sBg, sCg;       // per-group element strides: B (MVAR weights), C (KVAR gradients)
  int M, N, K;            // MVAR: N, K fixed. KVAR: M, N fixed (K = group rows)
  int tiles_m, tiles_n;   // MVAR: tiles_m = max M tiles over all groups (grid upper bound)
  const float* sa;        // fp8: per-row scale of A rows (MVAR)
  const float* sb;        // fp8: per-row scale of B rows (MVAR, k-contiguous B)
  int64_t sSg;            // per-group stride of sb
  const uint16_t* aux;      // SWIGLU_BWD: gu [rows, 2F]
  int64_t ld_aux;
  uint16_t* out2;           // SWIGLU_*: a [rows, F]
  int64_t ld_out2;
  int F;                  // SWIGLU: gate/up split
  int accumulate;         // STORE: C += result
};

// kind: 0 fwd (A rows . W_g^T), 1 fwd + SwiGLU epilogue, 2 dgrad (dY . W_g), 3 dgrad + SwiGLU
// backward epilogue, 4 wgrad (dW_g (+)= dY_g^T X_g)
void launch_grouped_gemm(GGParams p, int kind, bool fp8, bool out_f32, int64_t total_rows,
                         hipStream_t st);

}  // namespace dla
