"""Text encoder and duration predictor — MI355X-native drop-in for the
reference's text_encoder.py: same class names,
constructor arguments, forward signatures and state_dict keys.

The reference builds these from the un-vendored FastSpeech2 repository
(text_encoder.py:16-18 import ``lib.FastSpeech2``; setup.sh clones
ming024/FastSpeech2, unpinned), which is absent here, so its published
architecture is restated:

* ``get_sinusoid_encoding_table`` (FastSpeech2 transformer/Models.py): angle
  pos / 10000^(2*(i//2)/d), sin on even and cos on odd columns, the
  padding_idx row zeroed;
* ``FFTBlock`` (transformer/Layers.py): self-attention, masked_fill(pad, 0),
  position-wise conv FFN, masked_fill(pad, 0);
* ``MultiHeadAttention`` (transformer/SubLayers.py): w_qs / w_ks / w_vs
  (d_model -> n_head*d_k), softmax(q k^T / sqrt(d_k), keys masked -inf), fc
  back to d_model, dropout, LayerNorm(out + residual);
* ``PositionwiseFeedForward``: Conv1d(d, d_inner, k0, pad (k0-1)/2) -> ReLU ->
  Conv1d(d_inner, d, k1) -> dropout -> LayerNorm(out + residual);
* ``VariancePredictor`` (model/modules.py): [Conv(k, pad (k-1)/2) -> ReLU ->
  LayerNorm -> Dropout] x 2 -> Linear(filter, 1) -> squeeze -> masked_fill.

Arithmetic (fp32, as the reference): the attention core is the HIP MFMA
attention (mtts_attention_*, key_padding_mask = the pad mask, True = pad, as
the reference's slf_attn_mask) on ONE fused q/k/v projection;
LayerNorm(x + residual) is the fused HIP LayerNorm; every nn.Dropout is the
HIP dropout (mtts.dropout, a counter-based mask regenerated in the
backward); the projections and the
convolutions run on the hand-written fp32 MFMA GEMM over windowed rows
(mtts.convgemm, csrc/convgemm.hip): a 'same' Conv1d is a direct implicit-GEMM
convolution over the zero-padded channel-last activation (no unfold copy),
the FFN's ReLU is fused into conv 1's epilogue and its backward into conv 2's
data-gradient epilogue.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from mtts import attn_kernels, ops
from mtts import convgemm as CG
from mtts.dropout import dropout as hip_dropout


def get_sinusoid_encoding_table(n_position, d_hid, padding_idx=None):
    """Sinusoid position table (FastSpeech2 transformer/Models.py)."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    i = np.arange(d_hid)[None, :]
    table = pos / np.power(10000, 2 * (i // 2) / d_hid)
    table[:, 0::2] = np.sin(table[:, 0::2])
    table[:, 1::2] = np.cos(table[:, 1::2])
    if padding_idx is not None:
        table[padding_idx] = 0.0
    return torch.FloatTensor(table)


class EmbeddingFn(torch.autograd.Function):
    """F.embedding(ids, weight, padding_idx) with the weight gradient as one
    fp32 TN GEMM, dW = onehot(ids)^T dy (mtts.convgemm; padding ids land in a
    discarded column), deterministic, instead of torch's sort-based dense
    embedding backward (49 us at B=8 x 128 phonemes)."""

    @staticmethod
    def forward(ctx, ids, weight, padding_idx):
        ctx.save_for_backward(ids)
        ctx.V, ctx.pad = weight.shape[0], padding_idx
        return F.embedding(ids, weight, padding_idx=padding_idx)

    @staticmethod
    def backward(ctx, dy):
        ids, = ctx.saved_tensors
        V, pad = ctx.V, ctx.pad
        d = dy.shape[-1]
        dy2 = dy.reshape(-1, d).contiguous()
        n = dy2.shape[0]
        Vp = (V + 1 + 3) // 4 * 4                 # + one discard column, a multiple of 4
        cols = ids.reshape(-1).long()      # scatter_ takes int64 indices (int32 ids are valid input)
        if pad is not None:
            cols = torch.where(cols == pad, torch.full_like(cols, V), cols)
        onehot = torch.zeros(n, Vp, device=dy.device, dtype=torch.float32)
        onehot.scatter_(1, cols[:, None], 1.0)
        dw = torch.empty(Vp, d, device=dy.device, dtype=torch.float32)
        CG.gemm(CG.TN, Vp, d, n, CG._plain(onehot), CG._plain(dy2), CG._plain(dw))
        return None, dw[:V], None


def _ln(mod, x, res=None):
    y, _ = ops.layer_norm(x, mod.weight, mod.bias, mod.eps, res=res)
    return y


def conv1d_same(x, weight, bias, padding, relu=False):
    """Conv1d over the time axis of channel-last x (B, T, C) with weight
    (O, C, K) and padding (K - 1) / 2 (the reference's 'same' convolutions),
    optionally followed by ReLU: a direct implicit-GEMM convolution
    (mtts.convgemm.conv1d_same)."""
    K = weight.shape[2]
    if 2 * padding != K - 1:
        raise ValueError(f"conv1d_same: padding {padding} with kernel {K} (only 'same' convolutions)")
    return CG.conv1d_same(x, weight, bias, relu=relu)


def linear(x, weight, bias=None):
    return CG.linear(x, weight, bias)


def kc_major(conv: nn.Conv1d) -> nn.Conv1d:
    """Keep a Conv1d weight's storage as [O][K][C] behind its (O, C, K) shape
    (a permuted dense view: state_dict keys, shapes and values unchanged).
    The implicit-GEMM convolution reads the weight as (O, K*C) rows, so its
    forward and weight gradient then need no transposing copies; the fused
    optimizer and the DP buckets follow the parameter's strides."""
    w = conv.weight
    if w.shape[2] > 1 and not w.permute(0, 2, 1).is_contiguous():
        conv.weight = nn.Parameter(w.detach().permute(0, 2, 1).contiguous().permute(0, 2, 1),
                                   requires_grad=w.requires_grad)
    return conv


class Conv(nn.Module):
    """FastSpeech2 model/modules.py Conv: Conv1d on (B, T, C) inputs."""

    def __init__(self, in_channels, out_channels, kernel_size=1, stride=1, padding=0, dilation=1, bias=True,
                 w_init="linear"):
        super().__init__()
        if stride != 1 or dilation != 1:
            raise ValueError("Conv: stride / dilation 1 only (the text encoder's use)")
        self.conv = kc_major(nn.Conv1d(in_channels, out_channels, kernel_size=kernel_size, padding=padding, bias=bias))

    def forward(self, x):
        return conv1d_same(x, self.conv.weight, self.conv.bias, self.conv.padding[0])


def _adjacent(ts):
    """Contiguous tensors laid end to end in one storage, in order."""
    t0 = ts[0]
    off = t0.storage_offset()
    for t in ts:
        if not t.is_contiguous() or t.untyped_storage().data_ptr() != t0.untyped_storage().data_ptr() or \
                t.storage_offset() != off:
            return False
        off += t.numel()
    return True


class PackedRowsFn(torch.autograd.Function):
    """cat(ts) along dim 0 for parameters stored end to end (MultiHeadAttention
    packs w_qs / w_ks / w_vs so): a view of their storage, no copy; the
    gradient comes back as row-slice views."""

    @staticmethod
    def forward(ctx, *ts):
        ctx.rows = [t.shape[0] for t in ts]
        t0 = ts[0]
        shape = (sum(ctx.rows),) + tuple(t0.shape[1:])
        return t0.new_empty(0).set_(t0.untyped_storage(), t0.storage_offset(), shape,
                                    torch.empty(shape, device="meta").stride())

    @staticmethod
    def backward(ctx, g):
        return tuple(g.split(ctx.rows, 0))


def _packed_rows(ts):
    return PackedRowsFn.apply(*ts) if _adjacent(ts) else torch.cat(ts)


class MultiHeadAttention(nn.Module):
    def __init__(self, n_head, d_model, d_k, d_v, dropout=0.1):
        super().__init__()
        if d_k != d_v:
            raise ValueError("MultiHeadAttention: d_k == d_v only (the text encoder's use)")
        self.n_head, self.d_k, self.d_v = n_head, d_k, d_v
        self.w_qs = nn.Linear(d_model, n_head * d_k)
        self.w_ks = nn.Linear(d_model, n_head * d_k)
        self.w_vs = nn.Linear(d_model, n_head * d_v)
        self.layer_norm = nn.LayerNorm(d_model)
        self.fc = nn.Linear(n_head * d_v, d_model)
        self.dropout = nn.Dropout(dropout)
        self._pack()

    def _pack(self):
        """Store the q / k / v weights (and biases) end to end so the fused
        projection reads them in place (state_dict keys and shapes unchanged;
        re-packed after .to() / .cuda(), which move each parameter alone)."""
        lins = (self.w_qs, self.w_ks, self.w_vs)
        for name in ("weight", "bias"):
            ps = [getattr(m, name) for m in lins]
            if _adjacent(ps):
                continue
            packed = torch.cat([p.detach() for p in ps])
            off = 0
            for p in ps:
                p.data = packed[off:off + p.shape[0]]
                off += p.shape[0]

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._pack()
        return out

    def forward(self, q, k, v, mask=None):
        """q/k/v (B, L, d_model); mask (B, L_k) bool, True = pad key.
        Returns (output, None): attention weights are not materialised."""
        residual = q
        # temperature sqrt(d_k) = the kernel's 1/sqrt(head_dim) scale
        if q is k and k is v:   # self-attention (the encoder's use): one fused q/k/v projection
            w = _packed_rows([self.w_qs.weight, self.w_ks.weight, self.w_vs.weight])
            b = _packed_rows([self.w_qs.bias, self.w_ks.bias, self.w_vs.bias])
            o = attn_kernels.attention_qkv(linear(q, w, b), self.n_head, key_padding_mask=mask)
        else:
            qh = linear(q, self.w_qs.weight, self.w_qs.bias)
            kh = linear(k, self.w_ks.weight, self.w_ks.bias)
            vh = linear(v, self.w_vs.weight, self.w_vs.bias)
            o = attn_kernels.attention(qh, kh, vh, self.n_head, key_padding_mask=mask)
        o = hip_dropout(linear(o, self.fc.weight, self.fc.bias), self.dropout.p, self.training)
        return _ln(self.layer_norm, o, res=residual), None


class PositionwiseFeedForward(nn.Module):
    def __init__(self, d_in, d_hid, kernel_size, dropout=0.1):
        super().__init__()
        self.w_1 = kc_major(nn.Conv1d(d_in, d_hid, kernel_size=kernel_size[0], padding=(kernel_size[0] - 1) // 2))
        self.w_2 = kc_major(nn.Conv1d(d_hid, d_in, kernel_size=kernel_size[1], padding=(kernel_size[1] - 1) // 2))
        self.layer_norm = nn.LayerNorm(d_in)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        for c in (self.w_1, self.w_2):
            if 2 * c.padding[0] != c.kernel_size[0] - 1:
                raise ValueError("PositionwiseFeedForward: 'same' convolutions only")
        out = hip_dropout(CG.conv_ffn(x, self.w_1.weight, self.w_1.bias, self.w_2.weight, self.w_2.bias),
                          self.dropout.p, self.training)
        return _ln(self.layer_norm, out, res=x)


class FFTBlock(nn.Module):
    def __init__(self, d_model, n_head, d_k, d_v, d_inner, kernel_size, dropout=0.1):
        super().__init__()
        self.slf_attn = MultiHeadAttention(n_head, d_model, d_k, d_v, dropout=dropout)
        self.pos_ffn = PositionwiseFeedForward(d_model, d_inner, kernel_size, dropout=dropout)

    def forward(self, enc_input, mask=None, slf_attn_mask=None, keep=None):
        """keep (optional): (~mask)[..., None] as bool, expanded to the
        activation's shape, made once by TextEncoder for all its blocks."""
        keypad = mask                      # slf_attn_mask = mask expanded over queries: the key pad mask
        enc_output, attn = self.slf_attn(enc_input, enc_input, enc_input, mask=keypad)
        # masked_fill(mask, 0) as torch.where over the keep mask: one kernel
        # each way instead of a clone + fill; like masked_fill it zeroes the NaN
        # rows a zero-length sequence's all-masked softmax leaves
        if keep is None:
            keep = (~mask).unsqueeze(-1)
        zero = enc_output.new_zeros(())
        enc_output = torch.where(keep, enc_output, zero)
        enc_output = self.pos_ffn(enc_output)
        enc_output = torch.where(keep, enc_output, zero)
        return enc_output, attn


class TextEncoder(nn.Module):
    """Reference text_encoder.py:21-128 (FastSpeech2 Encoder over phonemes)."""

    def __init__(self, vocab_size, d_model=256, n_layers=4, n_head=2, d_k=64, d_v=64, d_inner=1024,
                 kernel_size=(9, 1), dropout=0.1, max_seq_len=3000, padding_idx=0):
        super().__init__()
        n_position = max_seq_len + 1
        self.max_seq_len = max_seq_len
        self.d_model = d_model
        self.padding_idx = padding_idx
        self.phoneme_emb = nn.Embedding(vocab_size, d_model, padding_idx=padding_idx)
        self.position_enc = nn.Parameter(get_sinusoid_encoding_table(n_position, d_model, padding_idx).unsqueeze(0),
                                         requires_grad=False)
        self.layer_stack = nn.ModuleList([FFTBlock(d_model, n_head, d_k, d_v, d_inner, kernel_size, dropout=dropout)
                                          for _ in range(n_layers)])

    def forward(self, phoneme_ids, mask=None, return_attns=False):
        """phoneme_ids (B, L); mask (B, L) bool, True = pad.  -> (B, L, d_model)
        [, list of None per layer when return_attns: weights not materialised].
        mask None means no padding (the reference's FFTBlock would fail on it)."""
        B, L = phoneme_ids.shape
        if mask is None:
            mask = torch.zeros(B, L, dtype=torch.bool, device=phoneme_ids.device)
        w = self.phoneme_emb.weight
        if w.dtype == torch.float32 and w.is_cuda and w.shape[1] % 4 == 0:
            emb = EmbeddingFn.apply(phoneme_ids, w, self.padding_idx)
        else:
            emb = F.embedding(phoneme_ids, w, padding_idx=self.padding_idx)
        if not self.training and L > self.max_seq_len:
            pos = get_sinusoid_encoding_table(L, self.d_model)[:L].to(emb.device, emb.dtype)
        else:
            pos = self.position_enc[0, :L].to(emb.dtype)
        x = emb + pos[None]
        attns = []
        # full-width keep mask: the 8 masking selects per direction then run
        # as vectorised same-shape kernels instead of broadcasting ones
        keep = (~mask).unsqueeze(-1).expand(x.shape).contiguous()
        for layer in self.layer_stack:
            x, a = layer(x, mask=mask, slf_attn_mask=None, keep=keep)
            if return_attns:
                attns.append(a)
        return (x, attns) if return_attns else x


class VariancePredictor(nn.Module):
    """FastSpeech2 model/modules.py VariancePredictor (state_dict keys kept)."""

    def __init__(self, model_config):
        super().__init__()
        from collections import OrderedDict
        self.input_size = model_config["transformer"]["encoder_hidden"]
        self.filter_size = model_config["variance_predictor"]["filter_size"]
        self.kernel = model_config["variance_predictor"]["kernel_size"]
        self.conv_output_size = self.filter_size
        self.dropout = model_config["variance_predictor"]["dropout"]
        self.conv_layer = nn.Sequential(OrderedDict([
            ("conv1d_1", Conv(self.input_size, self.filter_size, kernel_size=self.kernel,
                              padding=(self.kernel - 1) // 2)),
            ("relu_1", nn.ReLU()),
            ("layer_norm_1", nn.LayerNorm(self.filter_size)),
            ("dropout_1", nn.Dropout(self.dropout)),
            ("conv1d_2", Conv(self.filter_size, self.filter_size, kernel_size=self.kernel, padding=1)),
            ("relu_2", nn.ReLU()),
            ("layer_norm_2", nn.LayerNorm(self.filter_size)),
            ("dropout_2", nn.Dropout(self.dropout)),
        ]))
        self.linear_layer = nn.Linear(self.conv_output_size, 1)

    def forward(self, encoder_output, mask):
        cl = self.conv_layer
        c1, c2 = cl.conv1d_1.conv, cl.conv1d_2.conv
        out = conv1d_same(encoder_output, c1.weight, c1.bias, c1.padding[0], relu=True)
        out = hip_dropout(_ln(cl.layer_norm_1, out), cl.dropout_1.p, self.training)
        out = conv1d_same(out, c2.weight, c2.bias, c2.padding[0], relu=True)
        out = hip_dropout(_ln(cl.layer_norm_2, out), cl.dropout_2.p, self.training)
        out = linear(out, self.linear_layer.weight, self.linear_layer.bias).squeeze(-1)
        if mask is not None:
            out = out.masked_fill(mask, 0.0)
        return out


class DurationPredictor(nn.Module):
    """Reference text_encoder.py:131-209."""

    def __init__(self, d_model=256, filter_size=256, kernel_size=3, dropout=0.1):
        super().__init__()
        model_config = {"transformer": {"encoder_hidden": d_model},
                        "variance_predictor": {"filter_size": filter_size, "kernel_size": kernel_size,
                                               "dropout": dropout}}
        self.predictor = VariancePredictor(model_config)

    def forward(self, encoder_output, mask=None):
        return self.predictor(encoder_output, mask)

    def compute_loss(self, log_duration_pred, duration_target, mask=None):
        log_duration_target = torch.log(duration_target.float() + 1e-8)
        loss = F.mse_loss(log_duration_pred, log_duration_target, reduction="none")
        if mask is not None:
            loss = loss.masked_fill(mask, 0.0)
            loss = loss.sum() / (~mask).sum().float()
        else:
            loss = loss.mean()
        return loss


class TextProcessor:
    """Phoneme vocabulary and batching (reference text_encoder.py:212-428; host
    side, no GPU work): vocab from a JSON list or a Python list; unknown
    phonemes map to <UNK>, or to the padding id when the vocabulary has no
    <UNK>; batches padded with the padding id, mask True = pad."""

    def __init__(self, vocab_path=None, vocab_list=None, padding_token="<PAD>", unk_token="<UNK>"):
        import json
        if vocab_path is not None:
            with open(vocab_path, "r", encoding="utf-8") as f:
                vocab_list = json.load(f)
        elif vocab_list is None:
            raise ValueError("Either vocab_path or vocab_list must be provided")
        self.vocab_list = list(vocab_list)
        self.phoneme_to_id = {ph: i for i, ph in enumerate(self.vocab_list)}
        self.id_to_phoneme = {i: ph for ph, i in self.phoneme_to_id.items()}
        self.vocab_size = len(self.vocab_list)
        self.padding_token, self.unk_token = padding_token, unk_token
        self.padding_id = self.phoneme_to_id.get(padding_token, 0)
        self.unk_id = self.phoneme_to_id.get(unk_token, self.padding_id)

    def text_to_phonemes(self, text, g2p_processor=None):
        if g2p_processor is None:
            return text.split()                  # pre-phonemized, space separated
        r = g2p_processor(text)
        if isinstance(r, dict):
            return r.get("ph", "").split()
        return r.split() if isinstance(r, str) else r

    def phonemes_to_ids(self, phonemes):
        return [self.phoneme_to_id.get(ph, self.unk_id) for ph in phonemes]

    def ids_to_phonemes(self, ids):
        return [self.id_to_phoneme.get(i, self.unk_token) for i in ids]

    def process_text(self, text, g2p_processor=None, max_length=None):
        phonemes = self.text_to_phonemes(text, g2p_processor)
        if max_length is not None:
            phonemes = phonemes[:max_length]
        return self.phonemes_to_ids(phonemes), phonemes

    def create_phoneme_embedding(self, embedding_dim, padding_idx=None):
        return nn.Embedding(self.vocab_size, embedding_dim,
                            padding_idx=self.padding_id if padding_idx is None else padding_idx)

    def create_positional_encoding(self, max_length, embedding_dim, padding_idx=None):
        return get_sinusoid_encoding_table(max_length, embedding_dim,
                                           self.padding_id if padding_idx is None else padding_idx)

    def batch_process(self, texts, g2p_processor=None, max_length=None, pad_to_max=True):
        """-> (ids (B, L) LongTensor | list of LongTensors, lengths, mask (B, L) | None)."""
        seqs = [self.process_text(t, g2p_processor, max_length)[0] for t in texts]
        lengths = [len(s) for s in seqs]
        if not pad_to_max:
            return [torch.LongTensor(s) for s in seqs], lengths, None
        L = max(lengths) if lengths else 0
        ids = torch.LongTensor([s + [self.padding_id] * (L - len(s)) for s in seqs])
        mask = torch.arange(L)[None, :] >= torch.tensor(lengths, dtype=torch.long)[:, None] if lengths else \
            torch.zeros(0, 0, dtype=torch.bool)
        return ids, lengths, mask


__all__ = ["TextProcessor", "TextEncoder", "DurationPredictor", "VariancePredictor", "FFTBlock", "MultiHeadAttention",
           "PositionwiseFeedForward", "Conv", "get_sinusoid_encoding_table", "conv1d_same"]
