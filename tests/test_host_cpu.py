"""Host-side pieces of the training step on CPU: clip-in-optimizer
(mtts/optim.py) against clip_grad_norm_ + the same optimizer.  (The
embedding sums run on the HIP kernel: tests/test_gpu_codec.py.)"""
import pytest
import torch
import torch.nn.functional as F


def test_clip_into_optimizer_equals_clip_grad_norm():
    from mtts.optim import clip_into_optimizer
    torch.manual_seed(0)
    try:
        torch.optim.Adam([torch.zeros(1, requires_grad=True)], fused=True)
    except Exception as e:  # pragma: no cover
        pytest.skip(f"fused Adam unavailable on CPU: {e}")
    ps1 = [torch.randn(7, 5, requires_grad=True), torch.randn(11, requires_grad=True)]
    ps2 = [p.detach().clone().requires_grad_(True) for p in ps1]
    o1 = torch.optim.Adam(ps1, lr=1e-2, fused=True)
    o2 = torch.optim.Adam(ps2, lr=1e-2, fused=True)
    for step in range(3):
        gs = [torch.randn_like(p) * 10 for p in ps1]
        for p, gg in zip(ps1, gs):
            p.grad = gg.clone()
        for p, gg in zip(ps2, gs):
            p.grad = gg.clone()
        n1 = torch.nn.utils.clip_grad_norm_(ps1, 1.0)
        o1.step()
        n2 = clip_into_optimizer(o2, ps2, 1.0)
        o2.step()
        torch.testing.assert_close(n1, n2)
        for a, b in zip(ps1, ps2):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_text_processor_batching():
    """text_encoder.TextProcessor (host side of reference text_encoder.py:212-428)
    with the reference's own phoneme vocabulary (tests/golden/phoneme_vocab.json,
    a data file of the reference): ids, the <UNK> -> padding-id fallback of a
    vocabulary without <UNK>, truncation, padding and the True = pad mask."""
    import json
    import os
    import text_encoder as te
    from conftest import GOLDEN
    path = os.path.join(GOLDEN, "phoneme_vocab.json")
    vocab = json.load(open(path))
    tp = te.TextProcessor(vocab_path=path)
    assert tp.vocab_size == len(vocab) and tp.padding_id == vocab.index("<PAD>")
    assert tp.unk_id == (vocab.index("<UNK>") if "<UNK>" in vocab else tp.padding_id)
    ids, ph = tp.process_text("HH AH0 L OW1 QQQ")
    assert ph == ["HH", "AH0", "L", "OW1", "QQQ"]
    assert ids == [vocab.index("HH"), vocab.index("AH0"), vocab.index("L"), vocab.index("OW1"), tp.unk_id]
    assert tp.ids_to_phonemes(ids[:4]) == ph[:4]
    batch, lengths, mask = tp.batch_process(["HH AH0", "L OW1 HH AH0 L", "OW1"], max_length=4)
    assert lengths == [2, 4, 1] and batch.shape == (3, 4)
    assert batch[0].tolist() == [vocab.index("HH"), vocab.index("AH0"), tp.padding_id, tp.padding_id]
    assert mask.tolist() == [[False, False, True, True], [False] * 4, [False, True, True, True]]
    seqs, lengths, mask = tp.batch_process(["HH", "L OW1"], pad_to_max=False)
    assert [s.tolist() for s in seqs] == [[vocab.index("HH")], [vocab.index("L"), vocab.index("OW1")]] and mask is None
    tab = tp.create_positional_encoding(10, 8)
    assert tab.shape == (10, 8) and float(tab[tp.padding_id].abs().sum()) == 0.0


def test_packed_activation_layout_roundtrip_and_split_rules():
    """Host side of the packed decode operands (csrc/common.h xpk_index): the
    PackedAct image built by pack() holds element (m, k) at
    ((k/32*2 + m/16)*64 + (k/8%4)*16 + m%16)*8 + k%8 and unpacks to the rows;
    gemv_split_ok mirrors the kernel's wave split (K/32 = KS*S, KS <= 8,
    S <= 16; <= 8 with the LayerNorm prologue)."""
    from mtts import ops
    M, K = 20, 96
    x = torch.arange(M * K, dtype=torch.float32).view(M, K).to(torch.bfloat16)
    p = ops.PackedAct.pack(x)
    assert p.data.numel() == 32 * K and p.shape == (M, K)
    flat = p.data
    for m, k in [(0, 0), (5, 7), (19, 95), (16, 32), (3, 40)]:
        idx = (((k >> 5) * 2 + (m >> 4)) * 64 + ((k >> 3) & 3) * 16 + (m & 15)) * 8 + (k & 7)
        assert flat[idx] == x[m, k]
    assert torch.equal(p.unpack(), x)
    assert ops.gemv_split_ok(1024) and ops.gemv_split_ok(2048) and ops.gemv_split_ok(4096)
    assert ops.gemv_split_ok(64) and not ops.gemv_split_ok(96) and not ops.gemv_split_ok(8192)
    assert ops.gemv_split_ok(2048, ln=True) and not ops.gemv_split_ok(4096, ln=True)
