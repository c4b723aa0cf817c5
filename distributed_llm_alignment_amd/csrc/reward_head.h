// Parameter block of the fused reward head (reward_head.hip), shared with its torch binding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dla {

struct RHParams {
  const uint16_t* hidden;  // [B, T, H]
  int64_t sb, st;        // batch / token strides (elements)
  const int* last;       // [B] last valid position (last_token pooling)
  const float* mask;     // [B, T] validity weights (mean pooling), nullptr for last_token
  const uint16_t* w;       // [H]
  const uint16_t* bias;    // [1] or nullptr
  int B, T, H;
  float p;               // dropout probability (0: eval)
  uint64_t seed;
  float* score;          // [B]
  float* pooled;         // [B, H] dropped pooled rows (fp32)
  const float* dscore;   // [B] (backward)
  uint16_t* dhidden;       // [B, T, H] (backward; zero-filled by the host)
};

void launch_reward_head_fwd(const RHParams& p, hipStream_t st);
void launch_reward_head_bwd(const RHParams& p, hipStream_t st);

}  // namespace dla
