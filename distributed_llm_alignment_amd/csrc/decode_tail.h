// Host/device argument block of the persistent decode layer tail (csrc/decode_tail.hip).
#pragma once
#include <cstdint>

namespace dla {

struct TailArgs {
  const uint16_t* a;        // attention output [M, Ko] (previous launch)
  int64_t lda;
  const uint16_t* x;        // layer input residual [M, H] (previous launch)
  int64_t ldx;
  const uint16_t* Wo;       // tiled [H/16][Ko/32][4][16][8]
  const uint16_t* Wgu;      // interleaved tiled, ln2 folded [2F/16][H/32][4][16][8]
  const uint16_t* Wd;       // tiled [H/16][F/32][4][16][8]
  const uint16_t* Wq;       // tiled, next layer's ln1 folded [Nq/16][H/32][4][16][8]; nullptr: no QKV phase
  uint16_t* s;              // [M, H]  (ld H)
  float* ssq_s;           // [16][H/16]
  uint16_t* m;              // [M, F]  (ld F)
  uint16_t* xo;             // [M, H]  (ld H): the layer output
  float* ssq_x;           // [16][H/16]: its row partials (next layer's norm)
  uint16_t* qkv;            // [M, Nq] (ld Nq)
  int M, H, Ko, F, Nq;
  float eps;
  int* cnt;               // [3][kTlRep][kTlRepStride]
  const int* kv_len;
  const int* len_first;
  int* err;
  int pg, pd, pq;          // LDS-DMA prefetch depth (k-steps per wave) of GU / DOWN / QKV (set by the launcher)
  unsigned long long* stamps;  // debug (DLA_TAIL_STAMPS): [grid][8] s_memrealtime per phase edge
};

bool launch_decode_tail(const TailArgs& A, hipStream_t st);
int decode_tail_grid();

}  // namespace dla
