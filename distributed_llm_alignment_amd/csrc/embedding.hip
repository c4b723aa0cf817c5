// Token embedding gather (forward) and deterministic scatter-add (backward) for gfx950 (SURVEY
// K1). Reference: the HF `nn.Embedding` of every model forward (src/training/train_*.py); eager
// PyTorch's backward materialises a dense [V, H] gradient (zero-fill + sort-based segment sum),
// then autograd adds it into `.grad`: two passes over V x H (1 GB at Llama-3's 128256 x 4096)
// per micro-batch for a few thousand touched rows.
//
// Forward: one wave per token row, 16-byte loads/stores (the table row is contiguous).
// Backward: the token ids arrive sorted (with the inverse permutation) from a device sort, so all
// occurrences of a token are adjacent. The wave at the FIRST position of each run sums the run's
// dY rows in sorted order (fixed order: bitwise reproducible, no float atomics) and adds the sum
// into the gradient row in place -- straight into the training engine's flat main-grad buffer
// (bf16 or fp32), so untouched rows cost nothing. The sorted positions are cut into chunks of
// kEmbChunk, one wave each: a run that lies inside one chunk is summed and added by that wave
// directly; a longer run (a frequent token) leaves one fp32 partial per chunk in a scratch slab,
// folded in chunk order by a second pass, so a hot token does not serialise the pass (cdna guide
// Appendix B "Scatter / gather / embedding": split long lists, sum per destination in a fixed order).
#include "common.h"

namespace dla {

constexpr int kEmbChunk = 16;  // sorted positions per backward wave

__global__ __launch_bounds__(256) void embed_fwd_kernel(const bf16_t* __restrict__ w, int64_t ldw,
                                                        const int64_t* __restrict__ ids, int64_t N,
                                                        int H, int64_t V, bf16_t* __restrict__ out,
                                                        int* __restrict__ bad) {
  const int64_t row = blockIdx.x * 4ll + (threadIdx.x >> 6);
  if (row >= N) return;
  const int lane = threadIdx.x & 63;
  const int64_t id = ids[row];
  bf16_t* dst = out + row * static_cast<int64_t>(H);
  if (id < 0 || id >= V) {
    // out-of-range id: never read outside the table. The row is zeros and the sticky error word
    // is set (vector store from lane 0); ops/embedding.py raises on it at the next host sync.
    for (int c = lane * 8; c < H; c += 512) store_bf16x8(dst + c, bf16x8{});
    if (lane == 0) bad[0] = 1;
    return;
  }
  const bf16_t* src = w + id * ldw;
  for (int c = lane * 8; c < H; c += 512) store_bf16x8(dst + c, load_bf16x8(src + c));
}

template <typename G>
__device__ __forceinline__ void emb_add_row(G* g, int c, const float* a) {
  if constexpr (sizeof(G) == 4) {
    f32x4 o0 = *reinterpret_cast<const f32x4*>(g + c), o1 = *reinterpret_cast<const f32x4*>(g + c + 4);
    o0 += f32x4{a[0], a[1], a[2], a[3]};
    o1 += f32x4{a[4], a[5], a[6], a[7]};
    *reinterpret_cast<f32x4*>(g + c) = o0;
    *reinterpret_cast<f32x4*>(g + c + 4) = o1;
  } else {
    const bf16x8 o = load_bf16x8(reinterpret_cast<const bf16_t*>(g) + c);
    float r[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = bf2f(o[e]) + a[e];
    store_bf16x8(reinterpret_cast<bf16_t*>(g) + c, pack_bf16x8(r));
  }
}

// Pass 1: wave per chunk of kEmbChunk sorted positions. Each run piece [p, q) in the chunk is
// summed in order; a run wholly inside the chunk is added into grad here, a piece of a run that
// crosses a chunk boundary goes to scratch[p] (fp32 [H]) for pass 2.
template <typename G>
__global__ __launch_bounds__(256) void embed_bwd_partial_kernel(
    const int64_t* __restrict__ sid, const int64_t* __restrict__ perm, const bf16_t* __restrict__ dy,
    int64_t N, int H, int64_t V, float* __restrict__ scratch, G* __restrict__ grad, int64_t ldg) {
  const int64_t chunk = blockIdx.x * 4ll + (threadIdx.x >> 6);
  const int64_t p0 = chunk * kEmbChunk;
  if (p0 >= N) return;
  const int lane = threadIdx.x & 63;
  const int64_t p1 = p0 + kEmbChunk < N ? p0 + kEmbChunk : N;
  int64_t p = p0;
  while (p < p1) {
    const int64_t id = sid[p];
    int64_t q = p + 1;
    while (q < p1 && sid[q] == id) ++q;
    const bool whole = (p == 0 || sid[p - 1] != id) && (q == N || sid[q] != id);
    if (id < 0 || id >= V) {  // out-of-range ids (flagged by the forward) touch no gradient row
      p = q;
      continue;
    }
    for (int c = lane * 8; c < H; c += 512) {
      float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int64_t j = p; j < q; ++j) {
        const bf16x8 v = load_bf16x8(dy + perm[j] * static_cast<int64_t>(H) + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += bf2f(v[e]);
      }
      if (whole) {
        emb_add_row(grad + id * ldg, c, a);
      } else {
        float* dst = scratch + p * static_cast<int64_t>(H) + c;
        *reinterpret_cast<f32x4*>(dst) = f32x4{a[0], a[1], a[2], a[3]};
        *reinterpret_cast<f32x4*>(dst + 4) = f32x4{a[4], a[5], a[6], a[7]};
      }
    }
    p = q;
  }
}

// Pass 2: wave per run start (sorted position p with sid[p] != sid[p-1]) of a run that crosses a
// chunk boundary: fold its pieces (head p, then each chunk start inside the run, in order) and
// add into grad[id].
template <typename G>
__global__ __launch_bounds__(256) void embed_bwd_fold_kernel(const int64_t* __restrict__ sid,
                                                             int64_t N, int H, int64_t V,
                                                             const float* __restrict__ scratch,
                                                             G* __restrict__ grad, int64_t ldg) {
  const int64_t p = blockIdx.x * 4ll + (threadIdx.x >> 6);
  if (p >= N) return;
  const int64_t id = sid[p];
  if (p > 0 && sid[p - 1] == id) return;  // not a run head
  if (id < 0 || id >= V) return;
  int64_t end = p + 1;
  while (end < N && sid[end] == id) ++end;
  if (p / kEmbChunk == (end - 1) / kEmbChunk) return;  // whole run inside one chunk: pass 1 did it
  const int lane = threadIdx.x & 63;
  for (int c = lane * 8; c < H; c += 512) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int64_t s = p; s < end; s = (s / kEmbChunk + 1) * kEmbChunk) {
      const float* src = scratch + s * static_cast<int64_t>(H) + c;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(src);
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(src + 4);
      a[0] += x0[0]; a[1] += x0[1]; a[2] += x0[2]; a[3] += x0[3];
      a[4] += x1[0]; a[5] += x1[1]; a[6] += x1[2]; a[7] += x1[3];
    }
    emb_add_row(grad + id * ldg, c, a);
  }
}

void launch_embed_fwd(const bf16_t* w, int64_t ldw, const int64_t* ids, int64_t N, int H, int64_t V,
                      bf16_t* out, int* bad, hipStream_t st) {
  if (N == 0) return;
  embed_fwd_kernel<<<static_cast<unsigned>((N + 3) / 4), 256, 0, st>>>(w, ldw, ids, N, H, V, out, bad);
}

void launch_embed_bwd(const int64_t* sid, const int64_t* perm, const bf16_t* dy, int64_t N, int H,
                      int64_t V, float* scratch, void* grad, bool grad_f32, int64_t ldg, hipStream_t st) {
  if (N == 0) return;
  const int64_t chunks = (N + kEmbChunk - 1) / kEmbChunk;
  const unsigned g1 = static_cast<unsigned>((chunks + 3) / 4), g2 = static_cast<unsigned>((N + 3) / 4);
  if (grad_f32) {
    embed_bwd_partial_kernel<float><<<g1, 256, 0, st>>>(sid, perm, dy, N, H, V, scratch, static_cast<float*>(grad), ldg);
    embed_bwd_fold_kernel<float><<<g2, 256, 0, st>>>(sid, N, H, V, scratch, static_cast<float*>(grad), ldg);
  } else {
    embed_bwd_partial_kernel<bf16_t><<<g1, 256, 0, st>>>(sid, perm, dy, N, H, V, scratch, static_cast<bf16_t*>(grad), ldg);
    embed_bwd_fold_kernel<bf16_t><<<g2, 256, 0, st>>>(sid, N, H, V, scratch, static_cast<bf16_t*>(grad), ldg);
  }
}

}  // namespace dla
