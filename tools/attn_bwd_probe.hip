// Standalone timing probe of the attention-backward main kernels (no torch): times
// attn_bwd_kernel (4 waves) / attn_bwd8_kernel (8 waves) on synthetic inputs and, for the 8-wave
// kernel, prints the per-phase cycle breakdown of workgroup 0 (the heaviest causal key block)
// from the DLA_BWD_TRACE s_memtime stamps.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/attn_bwd_probe.hip -o tools/attn_bwd_probe.bin
//   tools/attn_bwd_probe.bin [waves=8] [B=8] [T=1024] [Hq=32] [Hkv=8] [causal=1]
#define DLA_BWD_TRACE 0
#include "../distributed_llm_alignment_amd/csrc/attention.hip"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

using namespace dla;

static uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return static_cast<uint16_t>((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

int main(int argc, char** argv) {
  const int waves = argc > 1 ? std::atoi(argv[1]) : 8;
  const int B = argc > 2 ? std::atoi(argv[2]) : 8;
  const int T = argc > 3 ? std::atoi(argv[3]) : 1024;
  const int Hq = argc > 4 ? std::atoi(argv[4]) : 32;
  const int Hkv = argc > 5 ? std::atoi(argv[5]) : 8;
  const bool causal = argc > 6 ? std::atoi(argv[6]) != 0 : true;
  constexpr int D = 128;
  const size_t nq = static_cast<size_t>(B) * T * Hq * D, nk = static_cast<size_t>(B) * T * Hkv * D;
  std::mt19937 rng(0);
  std::normal_distribution<float> nd(0.f, 1.f);
  auto randbf = [&](size_t n) {
    std::vector<uint16_t> h(n);
    for (auto& x : h) x = f2bf(nd(rng));
    return h;
  };
  auto up = [&](const std::vector<uint16_t>& h) {
    bf16_t* d;
    CK(hipMalloc(&d, h.size() * 2));
    CK(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    return d;
  };
  bf16_t *q = up(randbf(nq)), *k = up(randbf(nk)), *v = up(randbf(nk)), *dO = up(randbf(nq));
  std::vector<float> lse(static_cast<size_t>(B) * Hq * T, 12.f), del(lse.size(), 0.01f);
  float *lse2, *delta;
  CK(hipMalloc(&lse2, lse.size() * 4));
  CK(hipMalloc(&delta, del.size() * 4));
  CK(hipMemcpy(lse2, lse.data(), lse.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(delta, del.data(), del.size() * 4, hipMemcpyHostToDevice));
  const int nkb = (T + kAttnBwdKeys - 1) / kAttnBwdKeys;
  const int slab_rows = (T + kAttnBwdQRows - 1) / kAttnBwdQRows * kAttnBwdQRows;
  int hs = 1;  // as bindings.cpp attn_bwd_hsplit with 256 CUs
  const int group = Hq / Hkv;
  while (static_cast<int64_t>(nkb) * Hkv * B * hs < (causal ? 512 : 256) && group % (2 * hs) == 0) hs *= 2;
  float *slab, *dkp = nullptr, *dvp = nullptr;
  CK(hipMalloc(&slab, static_cast<size_t>(nkb) * B * slab_rows * Hq * D * 4));
  if (hs > 1) {
    CK(hipMalloc(&dkp, hs * nk * 4));
    CK(hipMalloc(&dvp, hs * nk * 4));
  }
  bf16_t *dk, *dv;
  CK(hipMalloc(&dk, nk * 2));
  CK(hipMalloc(&dv, nk * 2));
  AttnBwdParams p{};
  p.q = q; p.k = k; p.v = v; p.dout = dO; p.lse2 = lse2; p.delta = delta; p.dq_slab = slab;
  p.dk_part = dkp; p.dv_part = dvp; p.dk = dk; p.dv = dv; p.hsplit = hs; p.slab_rows = slab_rows;
  p.q_sb = static_cast<int64_t>(T) * Hq * D; p.q_st = Hq * D; p.q_sh = D;
  p.k_sb = static_cast<int64_t>(T) * Hkv * D; p.k_st = Hkv * D; p.k_sh = D;
  p.v_sb = p.k_sb; p.v_st = p.k_st; p.v_sh = D;
  p.do_sb = p.q_sb; p.do_st = p.q_st; p.do_sh = D;
  p.dk_sb = p.k_sb; p.dk_st = p.k_st; p.dk_sh = D;
  p.dv_sb = p.k_sb; p.dv_st = p.k_st; p.dv_sh = D;
  p.B = B; p.Hq = Hq; p.Hkv = Hkv; p.Tq = T; p.Tk = T;
  p.scale = 1.f / std::sqrt(static_cast<float>(D));
  p.scale2 = p.scale * 1.4426950408889634f;
  const dim3 grid(nkb * Hkv * B * hs);
  auto launch = [&]() {
    if (waves == 8) {
      if (causal) attn_bwd8_kernel<D, true><<<grid, 512>>>(p);
      else attn_bwd8_kernel<D, false><<<grid, 512>>>(p);
    } else {
      if (causal) attn_bwd_kernel<D, true><<<grid, 256>>>(p);
      else attn_bwd_kernel<D, false><<<grid, 256>>>(p);
    }
  };
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::printf("[probe] waves=%d B=%d T=%d Hq=%d Hkv=%d causal=%d hsplit=%d grid=%u main kernel %.1f us\n", waves, B,
              T, Hq, Hkv, causal ? 1 : 0, hs, grid.x, 1000.f * ms / iters);
  if (waves == 8) {
    std::vector<long long> tr(8 * 64 * 8, 0);
    CK(hipMemset(slab, 0, 4));
    std::vector<long long> zero(tr.size(), 0);
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_bwd_trace), zero.data(), zero.size() * 8));
    launch();
    CK(hipDeviceSynchronize());
    CK(hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_bwd_trace), tr.size() * 8));
    // per point k: mean over (wave, tile) of t[k] - t[k-1] (k = 0: from the previous tile's 7)
    const char* names[8] = {"bar2->top", "S+dP chains", "exp/mask/pack", "dV/dK mfma", "dS write",
                            "barrier1", "stage+prefetch", "dQ"};
    double sum[8] = {0}, cnt[8] = {0};
    double tile_sum = 0, tile_cnt = 0;
    for (int w = 0; w < 8; ++w) {
      for (int it = 1; it < 64; ++it) {
        const long long* t = &tr[(w * 64 + it) * 8];
        const long long* tp = &tr[(w * 64 + it - 1) * 8];
        if (t[0] == 0 || tp[7] == 0) continue;
        tile_sum += t[0] - tp[0];
        tile_cnt += 1;
        sum[0] += t[0] - tp[7];
        cnt[0] += 1;
        long long prev = t[0];
        for (int kk = 1; kk < 8; ++kk) {
          if (t[kk] == 0) continue;  // inactive sub-tile: points 1..3 absent
          sum[kk] += t[kk] - prev;
          cnt[kk] += 1;
          prev = t[kk];
        }
      }
    }
    std::printf("[probe] workgroup 0: %.0f s_memtime ticks per tile (mean over waves)\n",
                tile_cnt ? tile_sum / tile_cnt : 0.0);
    for (int kk = 0; kk < 8; ++kk)
      std::printf("[probe]   %-16s %8.0f  (n=%.0f)\n", names[kk], cnt[kk] ? sum[kk] / cnt[kk] : 0.0, cnt[kk]);
    for (int w = 0; w < 8; ++w) {
      const long long* t = &tr[(w * 64 + 10) * 8];
      std::printf("[probe]   wave %d tile 10:", w);
      for (int kk = 0; kk < 8; ++kk) std::printf(" %lld", t[kk] ? t[kk] - tr[(0 * 64 + 10) * 8] : -1);
      std::printf("\n");
    }
  }
  return 0;
}
