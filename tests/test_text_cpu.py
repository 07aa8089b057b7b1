"""The product's host-side text pieces against the reference text_encoder.py's
own outputs (tests/golden/text_processor.json and text.npz, written by
tests/golden/make_golden.py from /root/reference/text_encoder.py behind a
lib.FastSpeech2 shim).  TextProcessor is integer / string work: bit-exact.
CPU only (no kernels run)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

G2P = {"dict": lambda t: {"ph": t}, "str": lambda t: " ".join(reversed(t.split())), "list": lambda t: t.split()[1:]}


@pytest.fixture(scope="module")
def tp_golden():
    with open(os.path.join(GOLDEN, "text_processor.json"), encoding="utf-8") as f:
        return json.load(f)


def _processor(case):
    import text_encoder as te
    kw = dict(case["kwargs"])
    if case["vocab"] == "file":
        kw["vocab_path"] = os.path.join(GOLDEN, "phoneme_vocab.json")
    return te.TextProcessor(**kw)


@pytest.mark.parametrize("vocab", ["file", "unk_custom_pad", "no_specials"])
def test_text_processor_bit_exact(tp_golden, vocab):
    """ids, lengths and masks of batch_process (max_length None / 3 / 0,
    pad_to_max True / False, an empty text, unknown phonemes -> <UNK> or the
    padding id), process_text through dict / str / list G2P results,
    ids_to_phonemes with out-of-range ids, the empty batch, and the embedding
    factory's padding index (text_encoder.py:212-428)."""
    case = next(c for c in tp_golden["cases"] if c["vocab"] == vocab)
    tp = _processor(case)
    assert (tp.vocab_size, tp.padding_id, tp.unk_id) == (case["vocab_size"], case["padding_id"], case["unk_id"])
    texts = tp_golden["texts"]
    for b in case["batches"]:
        ids, lengths, masks = tp.batch_process(texts, max_length=b["max_length"], pad_to_max=b["pad_to_max"])
        assert lengths == b["lengths"]
        if b["pad_to_max"]:
            assert ids.dtype == torch.int64 and list(ids.shape) == b["ids_shape"]
            assert ids.tolist() == b["ids"]
            assert masks.dtype == torch.bool and masks.tolist() == b["masks"]
        else:
            assert masks is None and [t.tolist() for t in ids] == b["ids"]
            assert all(t.dtype == torch.int64 for t in ids)
    ids, lengths, masks = tp.batch_process([], pad_to_max=True)
    e = case["empty_batch"]
    assert list(ids.shape) == e["ids_shape"] and lengths == e["lengths"] and list(masks.shape) == e["masks_shape"]
    for pc in case["process"]:
        fn = None if pc["g2p"] is None else G2P[pc["g2p"]]
        pids, phs = tp.process_text(pc["text"], g2p_processor=fn, max_length=5)
        assert pids == pc["ids"] and phs == pc["phonemes"], pc
    assert tp.ids_to_phonemes(case["ids_to_phonemes"]["ids"]) == case["ids_to_phonemes"]["phonemes"]
    emb = tp.create_phoneme_embedding(8)
    assert (emb.num_embeddings, emb.embedding_dim, emb.padding_idx) == tuple(case["embedding"][k] for k in
                                                                            ("num", "dim", "padding_idx"))


def test_sinusoid_tables_match_reference(golden):
    """The product's get_sinusoid_encoding_table (TextEncoder.position_enc and
    the eval branch for L > max_seq_len) equals the reference's fp32 table."""
    import text_encoder as te
    g = golden("text.npz")
    tp = te.TextProcessor(vocab_list=["<PAD>", "a"])
    np.testing.assert_allclose(tp.create_positional_encoding(10, 8).numpy(), g["table/pad"], rtol=0, atol=1e-7)
    np.testing.assert_allclose(te.get_sinusoid_encoding_table(60, 64).numpy(), g["table/eval"], rtol=0, atol=1e-7)
    enc_pos = g["enc/sd/position_enc"]
    np.testing.assert_allclose(te.get_sinusoid_encoding_table(enc_pos.shape[1], enc_pos.shape[2], 0)[None].numpy(),
                               enc_pos, rtol=0, atol=1e-7)


def test_text_encoder_state_dict_matches_reference(golden):
    """The product TextEncoder / DurationPredictor carry the reference's
    state_dict keys and shapes (text.npz holds the reference modules' own)."""
    import text_encoder as te
    g = golden("text.npz")
    enc = te.TextEncoder(40, d_model=64, n_layers=2, n_head=2, d_k=32, d_v=32, d_inner=128, max_seq_len=48)
    ref = {k[len("enc/sd/"):]: v.shape for k, v in g.items() if k.startswith("enc/sd/")}
    assert {k: tuple(v.shape) for k, v in enc.state_dict().items()} == {k: tuple(s) for k, s in ref.items()}
    dp = te.DurationPredictor(d_model=64, filter_size=128, kernel_size=3)
    ref = {k[len("dur/sd/"):]: v.shape for k, v in g.items() if k.startswith("dur/sd/")}
    assert {k: tuple(v.shape) for k, v in dp.state_dict().items()} == {k: tuple(s) for k, s in ref.items()}
