"""Layout and quantisation of the weight-only fp8 decode copies (ops/decode.py), on CPU: the tiled
byte layout the F8 kernels read (csrc/skinny_ks.h) and the per-row e4m3 scaling."""
import torch

from distributed_llm_alignment_amd.ops import decode


def test_tile_f8_layout_matches_definition():
    N, K = 32, 128
    q = torch.randint(0, 256, (N, K), dtype=torch.uint8)
    t = decode.tile_f8(q)
    assert t.shape == (N // 16, K // 64, 64, 16) and t.is_contiguous()
    for tn in range(N // 16):
        for kt in range(K // 64):
            for lane in range(64):
                r, qd = lane % 16, lane // 16
                row = 16 * tn + r
                lo = q[row, 64 * kt + 8 * qd: 64 * kt + 8 * qd + 8]
                hi = q[row, 64 * kt + 32 + 8 * qd: 64 * kt + 32 + 8 * qd + 8]
                assert torch.equal(t[tn, kt, lane], torch.cat([lo, hi]))


def test_quantize_rows_f8_scales_and_error():
    g = torch.Generator().manual_seed(0)
    w = torch.randn(64, 256, generator=g) * torch.linspace(0.01, 10, 64)[:, None]
    q, sc = decode.quantize_rows_f8(w)
    assert q.dtype == torch.uint8 and sc.shape == (64,)
    deq = q.view(torch.float8_e4m3fn).float() * sc[:, None]
    assert torch.allclose(deq.abs().amax(1), w.abs().amax(1), rtol=1e-6)  # row amax is exact
    rel = (deq - w).norm(dim=1) / w.norm(dim=1)
    assert float(rel.max()) < 0.04  # e4m3: 3 mantissa bits
    z = torch.zeros(16, 64)
    qz, sz = decode.quantize_rows_f8(z)
    assert torch.all(qz.view(torch.float8_e4m3fn).float() == 0) and torch.all(sz > 0)


def test_fp8_context_manager_nests():
    assert not decode.fp8_enabled()
    with decode.fp8_weights(True):
        assert decode.fp8_enabled()
        with decode.fp8_weights(False):
            assert not decode.fp8_enabled()
        assert decode.fp8_enabled()
    assert not decode.fp8_enabled()
