// Kernel-argument structs shared by attention.hip (device side) and bindings.cpp (host side).
#pragma once
#include <stdint.h>

namespace dla {

using bf16_t = uint16_t;

struct AttnParams {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* o;
  float* lse2;  // [B, Hq, Tq], log2 domain: m2 + log2(l) of scores scaled by scale*log2(e)
  int64_t q_sb, q_st, q_sh;
  int64_t k_sb, k_st, k_sh;
  int64_t v_sb, v_st, v_sh;
  int64_t o_sb, o_st, o_sh;
  int B, Hq, Hkv, Tq, Tk;
  float scale2;     // softmax scale * log2(e)
  int causal_off;   // key j visible to query i iff j <= i + causal_off (causal only)
  int window;       // >0: also require j > i + causal_off - window
  const int* kv_start;  // [B] or null
  const int* kv_end;    // [B] or null
  const int* seg_start;  // [B, Tq] or null: packed sequences, query i sees keys >= seg_start[i]
  // RoPE on load (full rotary, self-attention): q / k are the un-rotated projections; the kernel
  // rotates Q in registers and every K row as it is staged into LDS; null = inputs pre-rotated
  const float* rope_cos;  // [max_pos, D/2] fp32
  const float* rope_sin;
  const int* rope_pos;    // [B * T] token positions, or null: position = t
  int rope_k;             // 1: K rotated as it is staged too; 0: K arrives pre-rotated, Q only
  bf16_t* q_rot;          // optional [B, T, Hq, D] out: the rotated Q (what the backward reads)
  int64_t qr_sb, qr_st, qr_sh;
  // forward structure switches (set once per process by the launcher, attn_fwd_switches)
  int fwd_prio;  // issue priority A/B (DLA_ATTN_FWD_PRIO): 1 = s_setprio 1 around each MFMA chain,
  int fwd_sgpr;   // 1: whole K/V tiles load from an SGPR tile base + 32-bit lane offsets (A/B: DLA_ATTN_FWD_SGPR=0)
  int fwd_pro;    // 1: K/V tile-0 loads issued right after the Q loads (A/B: DLA_ATTN_FWD_PRO=0)
  int fwd_ostage; // 1: O staged through LDS and stored as whole rows (A/B: DLA_ATTN_FWD_OSTAGE=0)
  int fwd_msub;   // 1: running max subtracted inside the Q.K^T MFMA chain (A/B: DLA_ATTN_FWD_MSUB)
                 // 2 = static s_setprio 1 for the second wave of each SIMD (waves 4-7)
  unsigned long long* stamps;  // debug (DLA_ATTN_STAMPS=1): persistent forward seam stamps
};

// Backward geometry: one workgroup per (256-key block, GQA head subset, kv head, batch);
// queries are swept in 32-row tiles.
constexpr int kAttnBwdKeys = 256;
constexpr int kAttnBwdQRows = 32;

struct AttnBwdParams {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  const bf16_t* dout;
  const float* lse2;   // [B, Hq, Tq]
  const float* delta;  // [B, Hq, Tq] = rowsum(dO * O)
  float* dq_slab;      // [nkb, B, slab_rows, Hq, D] fp32: one dQ partial per 256-key block (plain
                       // stores, no atomics), summed in key-block order by the reduce pass
  bf16_t* dq_slab16;   // the same slabs in bf16 (8-wave kernel, DLA_ATTN_DQ_BF16): each partial
                       // rounded once, summed in fp32 by the reduce -- half the slab traffic
  float* dk_part;      // [hsplit, B, Tk, Hkv, D] fp32 partials (hsplit > 1 only)
  float* dv_part;
  bf16_t* dk_part16;   // the same partials in bf16 (8-wave kernel, DLA_ATTN_DKV_BF16): summed in
  bf16_t* dv_part16;   // fp32 by the reduce -- half the partial traffic, as dq_slab16
  bf16_t* dk;          // strided like k (hsplit == 1)
  bf16_t* dv;          // strided like v (hsplit == 1)
  int hsplit;          // GQA group split across workgroups (balances causal key blocks)
  int slab_rows;       // Tq rounded up to a multiple of kAttnBwdQRows (dq_slab row count)
  int64_t q_sb, q_st, q_sh;
  int64_t k_sb, k_st, k_sh;
  int64_t v_sb, v_st, v_sh;
  int64_t do_sb, do_st, do_sh;
  int64_t dk_sb, dk_st, dk_sh;
  int64_t dv_sb, dv_st, dv_sh;
  int B, Hq, Hkv, Tq, Tk;
  float scale;   // softmax scale (natural)
  float scale2;  // scale * log2(e)
  int causal_off;
  int window;
  const int* kv_start;
  const int* kv_end;
  const int* seg_end;  // [B, Tk] or null: packed sequences, key j is seen by queries < seg_end[j]
  // fused RoPE backward (full rotary, rot = D, self-attention Tq = Tk): dQ / dK leave the
  // kernels un-rotated (the transpose of the rotation applied in the forward), written straight
  // into the q / k column slices of the fused dqkv buffer; null = no rotation
  const float* rope_cos;  // [max_pos, D/2] fp32
  const float* rope_sin;
  const int* rope_pos;    // [B * T] token positions, or null: position = t
  int rope_inputs;        // 1: k arrives un-rotated and is rotated as it is staged (q is the
                          // forward's q_rot output)
  int rope_rot;           // rotary dims: D (full), or 32 at D = 80 (phi-2's partial rotary:
                          // only dims [0, 32) rotate, d < 16 pairing with d + 16)
                          // 1 around every MFMA cluster, 2 both
};

}  // namespace dla
