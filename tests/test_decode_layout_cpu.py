"""Host-side checks of the tiled decode weight layout (ops/decode.py `tiled_weight` /
`folded_weight(tiled=True)`, csrc/skinny64.hip TW): Wt[t][kk][q][r][e] = W[16 t + r][32 kk + 8 q + e],
the order in which lane (r = lane % 16, q = lane // 16) of an MFMA B fragment reads 16-byte pieces."""
import torch

from distributed_llm_alignment_amd.ops import decode


def test_tiled_layout_index_map():
    N, K = 32, 64
    w = torch.arange(N * K, dtype=torch.float32).view(N, K).to(torch.bfloat16)
    t = decode.tiled_weight(w)
    assert t.shape == (N // 16, K // 32, 4, 16, 8)
    wf = w.float()
    for tt in range(N // 16):
        for kk in range(K // 32):
            for q in range(4):
                for r in range(16):
                    assert torch.equal(t[tt, kk, q, r].float(), wf[16 * tt + r, 32 * kk + 8 * q: 32 * kk + 8 * q + 8])
    # a lane's consecutive 32-deep k-steps are 512 elements apart (one 1 KB wave load each)
    flat = t.reshape(-1)
    assert torch.equal(flat[512: 520].float(), wf[0, 32:40])


def test_folded_tiled_weight_refreshes_in_place():
    g = torch.Generator().manual_seed(0)
    w = torch.randn(16, 32, generator=g).to(torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(32, generator=g)).to(torch.bfloat16)
    t = decode.folded_weight(w, nw, tiled=True)
    ref = (w * nw.view(1, -1)).view(1, 16, 1, 4, 8).permute(0, 2, 3, 1, 4)
    assert torch.equal(t, ref)
    ptr = t.data_ptr()
    with torch.no_grad():
        w.mul_(2)  # bumps the version counter: the cache is rebuilt into the same storage
    t2 = decode.folded_weight(w, nw, tiled=True)
    assert t2.data_ptr() == ptr
    assert torch.equal(t2, (w * nw.view(1, -1)).view(1, 16, 1, 4, 8).permute(0, 2, 3, 1, 4))


def test_glu_interleave_row_order():
    F, K = 32, 32
    w = torch.arange(2 * F, dtype=torch.float32).view(-1, 1).expand(2 * F, K).contiguous()
    il = decode._glu_interleave(w)[:, 0].long().tolist()
    # tile t: gate rows 8t .. 8t+7, then up rows F + 8t .. F + 8t + 7
    assert il[:16] == list(range(8)) + list(range(F, F + 8))
    assert il[16:32] == list(range(8, 16)) + list(range(F + 8, F + 16))
    t = decode.folded_weight(w.to(torch.bfloat16), torch.ones(K, dtype=torch.bfloat16), tiled=True, glu_il=True)
    assert t.shape == (2 * F // 16, 1, 4, 16, 8)
    # tile 1, lane r = 9 holds up row F + 8 + 1
    assert float(t[1, 0, 0, 9, 0]) == F + 9
