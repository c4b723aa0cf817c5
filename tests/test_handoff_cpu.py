"""Device-side RLHF rollout -> reward hand-off (training/handoff.py): the ids
built on the device equal the reference's decode + re-tokenise path (src/training/train_rlhf.py:
131-147) on the byte-level tokenizer fixture, for left-padded prompts, responses that end in EOS
and padding, special tokens mid-response, and truncation at max_length."""
import torch

from distributed_llm_alignment_amd.models.tokenizer import ByteTokenizer
from distributed_llm_alignment_amd.training.handoff import (RewardHandoff, device_reward_inputs,
                                                            separator_ids, special_token_table,
                                                            tokenizers_match)


def _rollouts(tok, prompts, responses, pad_to):
    tok.padding_side = "left"
    enc = tok(prompts, return_tensors="pt", padding=True)
    tok.padding_side = "right"
    ids, am = enc["input_ids"], enc["attention_mask"]
    rows, masks = [], []
    for r in responses:
        x = tok.encode(r, add_special_tokens=False) + [tok.eos_token_id]
        m = [1] * len(x)
        x += [tok.pad_token_id] * (pad_to - len(x))
        m += [0] * (pad_to - len(m))
        rows.append(x)
        masks.append(m)
    seqs = torch.cat([ids, torch.tensor(rows)], 1)
    gen_mask = torch.cat([am, torch.tensor(masks)], 1)
    return ids, am, seqs, gen_mask


def _text_path(tok, prompts, ids, seqs, max_len):
    resp = tok.batch_decode(seqs[:, ids.shape[1]:], skip_special_tokens=True)
    enc = tok([f"{p}\n\n{r}" for p, r in zip(prompts, resp)], return_tensors="pt", padding=True,
              truncation=True, max_length=max_len)
    return enc["input_ids"], enc["attention_mask"]


def test_device_ids_equal_retokenised_ids():
    tok = ByteTokenizer(vocab_size=300)
    prompts = ["Human: hi", "Human: tell me a longer story please", "Q: ünïcødé?"]
    responses = ["Sure.", "Once upon a time, there was a GPU.", "Ja — natürlich"]
    ids, am, seqs, gmask = _rollouts(tok, prompts, responses, pad_to=48)
    # a special token sampled mid-response is dropped by skip_special_tokens: the same here
    seqs[0, ids.shape[1] + 2] = tok.bos_token_id
    gmask_c = gmask.clone()
    want_ids, want_mask = _text_path(tok, prompts, ids, seqs, 1024)
    got_ids, got_mask = device_reward_inputs(ids, am, seqs, separator_ids(tok),
                                             special_token_table(tok, 300, "cpu"), tok.pad_token_id,
                                             1024, gmask_c)
    W = want_ids.shape[1]
    assert torch.equal(got_mask[:, :W], want_mask) and int(got_mask[:, W:].sum()) == 0
    assert torch.equal(got_ids[:, :W][want_mask.bool()], want_ids[want_mask.bool()])


def test_device_ids_truncate_like_the_tokenizer():
    tok = ByteTokenizer(vocab_size=300)
    prompts = ["abcdefghij", "xy"]
    responses = ["0123456789" * 3, "z"]
    ids, am, seqs, gmask = _rollouts(tok, prompts, responses, pad_to=40)
    for L in (8, 13, 20):
        want_ids, want_mask = _text_path(tok, prompts, ids, seqs, L)
        got_ids, got_mask = device_reward_inputs(ids, am, seqs, separator_ids(tok),
                                                 special_token_table(tok, 300, "cpu"),
                                                 tok.pad_token_id, L, gmask)
        W = want_ids.shape[1]
        assert got_ids.shape[1] <= L
        assert torch.equal(got_mask[:, :W], want_mask)
        assert torch.equal(got_ids[:, :W][want_mask.bool()], want_ids[want_mask.bool()])


def test_handoff_mode_selection():
    a, b = ByteTokenizer(vocab_size=300), ByteTokenizer(vocab_size=300)
    assert tokenizers_match(a, b)
    assert not tokenizers_match(a, ByteTokenizer(vocab_size=300, eos_token_id=1, bos_token_id=2))
    assert RewardHandoff(a, b, 300, "cpu", 64).device_path
    assert not RewardHandoff(a, b, 300, "cpu", 64, "text").device_path
    other = ByteTokenizer(vocab_size=300, offset=4)
    assert not RewardHandoff(a, other, 300, "cpu", 64).device_path
    import pytest

    with pytest.raises(ValueError):
        RewardHandoff(a, other, 300, "cpu", 64, "device")


def test_auto_handoff_revalidates_and_falls_back(monkeypatch):
    """auto mode re-checks the device ids against the text round trip every `validate_every`
    batches (not only the first): a later mismatching batch switches to the text path."""
    import pytest

    tok = ByteTokenizer(vocab_size=300)
    h = RewardHandoff(tok, tok, 300, "cpu", 1024, validate_every=2)
    h._validate = True  # byte tokenizer fixture: force the BPE-style validation on
    prompts, responses = ["Human: hi", "Q: x"], ["Sure.", "ok"]
    ids, am, seqs, gmask = _rollouts(tok, prompts, responses, pad_to=16)
    calls = []
    real_same = RewardHandoff._same
    monkeypatch.setattr(RewardHandoff, "_same",
                        staticmethod(lambda a, b: calls.append(1) or (len(calls) < 2 and real_same(a, b))))
    for _ in range(2):  # batch 0 validated (match), batch 1 not due
        h(prompts, ids, am, seqs, gmask)
        assert h.device_path
    assert len(calls) == 1
    with pytest.warns(UserWarning, match="text path"):
        out = h(prompts, ids, am, seqs, gmask)  # batch 2 validated: mismatch -> text from now on
    assert not h.device_path and h.fallback_reason and len(calls) == 2
    want = _text_path(tok, prompts, ids, seqs, 1024)
    assert torch.equal(out[0], want[0]) and torch.equal(out[1], want[1])


def test_rlhf_micro_bounds_fold_ragged_tail():
    from distributed_llm_alignment_amd.training.train_rlhf import micro_bounds

    assert micro_bounds(16, 8) == [(0, 8), (8, 16)]
    assert micro_bounds(17, 8) == [(0, 8), (8, 17)]  # a 1-rollout micro-batch has zero advantage
    assert micro_bounds(5, 8) == [(0, 5)]
    assert micro_bounds(20, 8) == [(0, 8), (8, 20)]
