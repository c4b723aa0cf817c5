"""CPU tier: model families, HF key layout round trips, reward model, generation/KV cache."""
import pytest
import torch

from distributed_llm_alignment_amd.models import (ByteTokenizer, RewardModel, build_model, generate,
                                                  get_config, load_causal_lm, save_hf_pretrained)
from distributed_llm_alignment_amd.models.config import PRESETS

TINY = ["tiny-llama", "tiny-mistral", "tiny-mixtral", "tiny-gpt2", "tiny-phi"]


@pytest.mark.parametrize("name", TINY)
def test_forward_backward_all_families(name):
    cfg = get_config(name)
    m = build_model(cfg, device="cpu", seed=0)
    ids = torch.randint(3, cfg.vocab_size, (2, 12))
    lp = m.sequence_logprob(ids, torch.ones_like(ids))
    assert lp.shape == (2,) and torch.isfinite(lp).all()
    lp.sum().backward()
    assert all(p.grad is not None for p in m.parameters() if p.requires_grad)


@pytest.mark.parametrize("name", TINY)
def test_hf_state_dict_roundtrip(name):
    cfg = get_config(name)
    a = build_model(cfg, device="cpu", seed=1)
    b = build_model(cfg, device="cpu", seed=2)
    sd = a.hf_state_dict()
    b.load_hf_state_dict(sd, strict=True)
    for (n1, p1), (n2, p2) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(p1, p2), n1


def test_hf_key_names_llama_layout():
    cfg = get_config("tiny-llama")
    keys = set(build_model(cfg, device="cpu").hf_state_dict())
    for k in ("model.embed_tokens.weight", "model.layers.0.self_attn.q_proj.weight",
              "model.layers.0.self_attn.k_proj.weight", "model.layers.0.self_attn.v_proj.weight",
              "model.layers.0.self_attn.o_proj.weight", "model.layers.0.mlp.gate_proj.weight",
              "model.layers.0.mlp.up_proj.weight", "model.layers.0.mlp.down_proj.weight",
              "model.layers.0.input_layernorm.weight", "model.layers.0.post_attention_layernorm.weight",
              "model.norm.weight", "lm_head.weight"):
        assert k in keys, k


def test_transformers_llama_parity_if_available():
    """Logits parity with HF LlamaForCausalLM (transformers is installed; random tiny config)."""
    transformers = pytest.importorskip("transformers")
    cfg = get_config("tiny-llama")
    hf_cfg = transformers.LlamaConfig(**{k: v for k, v in cfg.to_hf().items()
                                         if k not in ("architectures", "torch_dtype", "model_type")})
    hf = transformers.LlamaForCausalLM(hf_cfg).eval()
    mine = build_model(cfg, device="cpu", seed=0).eval()
    mine.load_hf_state_dict(hf.state_dict(), strict=False)
    ids = torch.randint(3, cfg.vocab_size, (2, 10))
    with torch.no_grad():
        a = hf(ids).logits
        b = mine.logits(mine(ids))
    assert torch.allclose(a, b, atol=2e-4), (a - b).abs().max()


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mistral", "tiny-mixtral", "tiny-gpt2", "tiny-phi"])
def test_transformers_parity_all_families_with_padding(name):
    """Logits parity with the installed transformers model of every family (random tiny config,
    eager attention, a right-padded row): Llama, Mistral (sliding window), Mixtral (top-2 MoE,
    fused or per-expert HF key layout), GPT-2, Phi-2."""
    transformers = pytest.importorskip("transformers")
    cfg = get_config(name)
    d = cfg.to_hf()
    hc = transformers.AutoConfig.for_model(d["model_type"], **{k: v for k, v in d.items() if k not in
                                                               ("architectures", "torch_dtype", "model_type")})
    hc._attn_implementation = "eager"
    torch.manual_seed(0)
    hf = transformers.AutoModelForCausalLM.from_config(hc).eval()
    mine = build_model(cfg, device="cpu", seed=1).eval()
    missing, unexpected = mine.load_hf_state_dict(hf.state_dict(), strict=False)
    assert not missing and not unexpected, (missing, unexpected)
    ids = torch.randint(3, cfg.vocab_size, (2, 24))
    am = torch.ones_like(ids)
    am[1, 18:] = 0
    with torch.no_grad():
        a = hf(ids, attention_mask=am).logits
        b = mine.logits(mine(ids, am))
    m = am.bool()
    assert torch.allclose(a[m], b[m], atol=2e-4), (a - b)[m].abs().max()


def test_padding_invariance_left_and_right():
    cfg = get_config("tiny-llama")
    m = build_model(cfg, device="cpu", seed=0).eval()
    ids = torch.randint(3, cfg.vocab_size, (1, 8))
    base = m.sequence_logprob(ids, torch.ones_like(ids))
    rp = torch.cat([ids, torch.zeros(1, 4, dtype=torch.long)], 1)
    rm = torch.cat([torch.ones(1, 8, dtype=torch.long), torch.zeros(1, 4, dtype=torch.long)], 1)
    assert torch.allclose(m.sequence_logprob(rp, rm), base, atol=1e-5)
    lpd = torch.cat([torch.zeros(1, 4, dtype=torch.long), ids], 1)
    lm = torch.cat([torch.zeros(1, 4, dtype=torch.long), torch.ones(1, 8, dtype=torch.long)], 1)
    # left padding: shifted mask keeps 7 real targets + (pad->first token) is masked out
    assert torch.allclose(m.sequence_logprob(lpd, lm), base, atol=1e-5)


def test_greedy_generation_matches_full_forward():
    cfg = get_config("tiny-llama")
    m = build_model(cfg, device="cpu", seed=0).eval()
    ids = torch.randint(3, cfg.vocab_size, (2, 6))
    mask = torch.ones_like(ids)
    ids[1, :2] = 0
    mask[1, :2] = 0
    out = generate(m, ids, mask, max_new_tokens=5, do_sample=False, eos_token_id=-1)
    assert out.shape == (2, 11)
    # re-derive each greedy token with a full (uncached) forward
    seq = ids.clone()
    fm = mask.clone()
    for _ in range(5):
        h = m(seq, fm)
        nxt = m.logits(h[:, -1]).argmax(-1, keepdim=True)
        seq = torch.cat([seq, nxt], 1)
        fm = torch.cat([fm, torch.ones_like(nxt)], 1)
    assert torch.equal(out, seq)


def test_reward_model_pooling_and_keys():
    cfg = get_config("tiny-llama")
    bb = build_model(cfg, device="cpu", seed=0, headless=True)
    rm = RewardModel(bb, pooling="last_token", dropout=0.0).eval()
    ids = torch.randint(3, cfg.vocab_size, (2, 7))
    mask = torch.ones_like(ids)
    mask[0, 5:] = 0
    s = rm(ids, mask)
    h = bb(ids, mask)
    ref = rm.scorer(h[torch.arange(2), mask.sum(1) - 1]).squeeze(-1)
    assert torch.allclose(s, ref, atol=1e-6)
    sd = rm.hf_state_dict()
    assert "scorer.1.weight" in sd and "scorer.1.bias" in sd
    assert any(k.startswith("backbone.layers.0.") for k in sd)
    rm2 = RewardModel(build_model(cfg, device="cpu", seed=5, headless=True), dropout=0.0).eval()
    rm2.load_hf_state_dict({"module." + k: v for k, v in sd.items()})
    assert torch.allclose(rm2(ids, mask), s, atol=1e-6)


def test_save_and_load_hf_pretrained(tmp_path):
    b = load_causal_lm("tiny-llama", gradient_checkpointing=False, device="cpu")
    save_hf_pretrained(b.model, b.tokenizer, str(tmp_path / "m"))
    c = load_causal_lm(str(tmp_path / "m"), gradient_checkpointing=False, device="cpu")
    ids = torch.randint(3, 500, (1, 9))
    assert torch.allclose(b.model.sequence_logprob(ids), c.model.sequence_logprob(ids))
    assert isinstance(c.tokenizer, ByteTokenizer)


def test_presets_param_counts():
    assert abs(get_config("llama3-8b").num_params() / 8.03e9 - 1) < 0.01
    assert abs(get_config("mistral-7b").num_params() / 7.24e9 - 1) < 0.01
    assert abs(get_config("mixtral-8x7b").num_params() / 46.7e9 - 1) < 0.01
    assert abs(get_config("gpt2").num_params() / 124.4e6 - 1) < 0.01
    assert abs(get_config("llama3-70b").num_params() / 70.6e9 - 1) < 0.01


def test_byte_tokenizer_roundtrip_and_padding():
    t = ByteTokenizer()
    enc = t(["hi", "hello</s>"], padding=True, return_tensors="pt")
    assert enc["input_ids"].shape == (2, 7)
    assert t.decode(enc["input_ids"][1], skip_special_tokens=True) == "hello"
    t.padding_side = "left"
    enc = t(["a", "abc"], padding=True)
    assert enc["attention_mask"][0] == [0, 0, 1, 1]


def test_layer_split_plan_balanced_and_contiguous():
    from distributed_llm_alignment_amd.parallel.layer_split import plan_layer_split

    assert plan_layer_split([1] * 32, 4) == [0] * 8 + [1] * 8 + [2] * 8 + [3] * 8
    p = plan_layer_split([1] * 8, 3, first_extra=2)  # device 0 also holds embed/head
    assert p == sorted(p) and set(p) == {0, 1, 2} and p.count(0) < p.count(2)
    assert plan_layer_split([5, 5], 4) == [0, 1]  # never more devices than layers


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-gpt2"])
def test_layer_split_model_matches_single_device(name):
    """device_map-style layer split (reference base_model.py:33) is numerically the same model:
    forward, backward and cached greedy generation match the one-device model."""
    from distributed_llm_alignment_amd.parallel.layer_split import dispatch_layers

    cfg = get_config(name)
    a = build_model(cfg, device="cpu", seed=0)
    b = build_model(cfg, device="cpu", seed=0)
    devs = dispatch_layers(b, ["cpu", "cpu", "cpu"])
    assert len(devs) == cfg.num_layers and b.layer_devices is devs
    ids = torch.randint(3, cfg.vocab_size, (2, 10))
    mask = torch.ones_like(ids)
    mask[0, :3] = 0
    la, lb = a.sequence_logprob(ids, mask), b.sequence_logprob(ids, mask)
    assert torch.allclose(la, lb)
    la.sum().backward()
    lb.sum().backward()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa.grad, pb.grad)
    ga = generate(a, ids, mask, max_new_tokens=4, do_sample=False, eos_token_id=-1)
    gb = generate(b, ids, mask, max_new_tokens=4, do_sample=False, eos_token_id=-1)
    assert torch.equal(ga, gb)


def test_load_causal_lm_device_map_single_device_is_plain():
    b = load_causal_lm("tiny-llama", gradient_checkpointing=False, device="cpu", device_map="auto")
    assert b.model.layer_devices is None


def test_packed_layout_runs():
    from distributed_llm_alignment_amd.models.transformer import packed_layout

    seg = torch.tensor([[1, 1, 1, 2, 2, 3, 0, 0], [1, 1, 1, 1, 1, 1, 1, 1]])
    pos, segs = packed_layout(seg)
    assert pos.tolist() == [[0, 1, 2, 0, 1, 0, 0, 1], list(range(8))]
    assert segs[0].tolist() == [[0, 0, 0, 3, 3, 5, 6, 6], [0] * 8]
    assert segs[1].tolist() == [[3, 3, 3, 5, 5, 6, 8, 8], [8] * 8]


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mistral"])
def test_packed_rows_match_separate_sequences(name):
    """Block-diagonal packed attention: each packed sequence's hidden states and
    loss equal those of the sequence run on its own."""
    cfg = get_config(name)
    m = build_model(cfg, device="cpu", seed=0)
    lens = [5, 7, 3]
    seqs = [torch.randint(3, cfg.vocab_size, (n,)) for n in lens]
    T = sum(lens) + 2
    ids = torch.zeros(1, T, dtype=torch.long)
    ids[0, : sum(lens)] = torch.cat(seqs)
    seg = torch.zeros(1, T, dtype=torch.long)
    mask = torch.zeros(1, T, dtype=torch.long)
    o = 0
    for j, n in enumerate(lens):
        seg[0, o:o + n] = j + 1
        mask[0, o:o + n] = 1
        o += n
    hp = m(ids, mask, segment_ids=seg)
    o = 0
    for x in seqs:
        hs = m(x.unsqueeze(0))
        assert torch.allclose(hp[0, o:o + len(x)], hs[0], atol=1e-5), name
        o += len(x)
    # loss over the packed row == token-weighted mean of the separate losses
    labels = ids.clone()
    labels[mask == 0] = -100
    o = 0
    for n in lens:
        labels[0, o] = -100
        o += n
    lp = m.causal_lm_loss(ids, labels, mask, segment_ids=seg)
    tot = sum(m.causal_lm_loss(x.unsqueeze(0), x.unsqueeze(0)) * (len(x) - 1) for x in seqs)
    assert torch.allclose(lp, tot / sum(n - 1 for n in lens), atol=1e-5)


def test_packed_dataset_rows():
    from distributed_llm_alignment_amd.data import InstructionDataset, PackedDataset

    tok = ByteTokenizer()
    recs = [{"prompt": "p" * a, "response": "r" * b} for a, b in [(3, 4), (2, 2), (10, 20), (1, 1)]]
    base = InstructionDataset(tok, max_length=32, records=recs)
    ds = PackedDataset(base, 32)
    sizes = [base[i]["input_ids"].numel() for i in range(len(base))]
    assert sum(len(r) for r in ds.rows) == len(base) and all(len(r) >= 1 for r in ds.rows)
    for r in range(len(ds)):
        row = ds[r]
        n = row["input_ids"].numel()
        assert n <= 32 and n == sum(sizes[i] for i in ds.rows[r])
        starts = [0] + list(torch.cumsum(torch.tensor([sizes[i] for i in ds.rows[r]]), 0)[:-1])
        assert all(row["labels"][int(s)] == -100 for s in starts)
        assert row["segment_ids"].max().item() == len(ds.rows[r])
    b = ds.collate([ds[0], ds[len(ds) - 1]])
    assert set(b) == {"input_ids", "attention_mask", "labels", "segment_ids"}


def test_greedy_generation_matches_transformers_generate():
    """Left-padded greedy decoding (KV cache path) == HF `generate(do_sample=False)` — the call
    the reference's RLHF / teacher-generation loops make (train_rlhf.py:115-121)."""
    transformers = pytest.importorskip("transformers")
    from distributed_llm_alignment_amd.models import generate

    cfg = get_config("tiny-llama")
    d = cfg.to_hf()
    hc = transformers.AutoConfig.for_model(d["model_type"], **{k: v for k, v in d.items() if k not in
                                                               ("architectures", "torch_dtype", "model_type")})
    hc._attn_implementation = "eager"
    torch.manual_seed(0)
    hf = transformers.AutoModelForCausalLM.from_config(hc).eval()
    mine = build_model(cfg, device="cpu", seed=1).eval()
    mine.load_hf_state_dict(hf.state_dict(), strict=False)
    g = torch.Generator().manual_seed(4)
    ids = torch.randint(3, cfg.vocab_size, (2, 12), generator=g)
    am = torch.ones_like(ids)
    ids[1, :4] = 0
    am[1, :4] = 0  # left padding, as the reference's generation pads
    ours = generate(mine, ids, am, max_new_tokens=10, do_sample=False, eos_token_id=-1, pad_token_id=0)
    with torch.no_grad():
        theirs = hf.generate(ids, attention_mask=am, max_new_tokens=10, do_sample=False,
                             eos_token_id=None, pad_token_id=0)
    assert torch.equal(ours, theirs), (ours, theirs)


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-phi", "tiny-mixtral"])
@pytest.mark.parametrize("policy", ["full", "mlp", "attention"])
def test_recompute_policies_match_no_recompute(name, policy):
    """Selective activation recompute: re-running the MLP or the attention block in
    backward gives the same loss and gradients as keeping every activation."""
    cfg = get_config(name)
    ids = torch.randint(3, cfg.vocab_size, (2, 16), generator=torch.Generator().manual_seed(1))
    am = torch.ones_like(ids)
    am[1, :3] = 0
    grads = []
    for pol in (None, policy):
        m = build_model(cfg, device="cpu", seed=4).train()
        if pol is not None:
            m.gradient_checkpointing_enable(pol)
        lp = m.sequence_logprob(ids, am)
        lp.sum().backward()
        grads.append([p.grad.clone() for p in m.parameters() if p.requires_grad])
    for a, b in zip(*grads):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_recompute_policy_rejects_unknown():
    m = build_model(get_config("tiny-llama"), device="cpu")
    with pytest.raises(ValueError):
        m.gradient_checkpointing_enable("everything")
