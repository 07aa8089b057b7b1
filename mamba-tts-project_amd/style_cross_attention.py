"""
Style Cross-Attention Modules — MI355X-native drop-in for the reference's
style_cross_attention.py (same classes, signatures, state_dict keys).

Implements:
1. Style K,V projections from SMSD output                 (reference :16-66)
2. Cross-Attention #1: Text ⊗ Style                        (reference :69-141)
3. Cross-Attention #2: Upsampled ⊗ Style                   (reference :215-286)
4. Length Regulator (phoneme-level → frame-level)          (reference :144-212)

Arithmetic runs on libmtts kernels: fused residual-add + LayerNorm, the
single-key attention shortcut (with the attention-weight dropout as one HIP
mask draw per (batch, query, head)), the FFN on the hand-written NT GEMM with
bias + GELU fused into its epilogue (bf16; the dropout between GELU and the
second linear and the GELU backward in the HIP dropout kernel), the HIP
dropout (mtts.dropout) for every nn.Dropout, and the HIP length regulator
(mtts_length_regulate_*: the reference loops over (b, phoneme) with one
.item() each, :185-196); only the output length needs one device->host read
when max_len is None, as in the reference.

`StyleConditioningPipeline.compute_dtype` (default None: the input's dtype,
fp32 as the reference) casts the pipeline's activations on entry, as the
decoder's compute_dtype does; train_harness runs train.py's dead style branch
in the decoder's bf16.
"""

import torch
import torch.nn as nn
import torch.nn.functional as F

from mtts.attention import CrossAttention
from mtts import ops
from mtts.dropout import dropout as hip_dropout
from mtts.linear import cast_scope, ffn, linear


def _ln(mod, x, res=None):
    y, _ = ops.layer_norm(x, mod.weight, mod.bias, mod.eps, res=res)
    return y


class StyleProjection(nn.Module):
    """Project SMSD style embedding (B, d_style) to single-token K, V (B, 1, d_model)."""

    def __init__(self, d_style, d_model, dropout=0.1):
        super().__init__()
        self.d_style = d_style
        self.d_model = d_model
        self.key_proj = nn.Sequential(nn.Linear(d_style, d_model), nn.LayerNorm(d_model), nn.Dropout(dropout))
        self.value_proj = nn.Sequential(nn.Linear(d_style, d_model), nn.LayerNorm(d_model), nn.Dropout(dropout))

    def _proj(self, seq, x):
        h = linear(x, seq[0].weight, seq[0].bias)
        h = _ln(seq[1], h)
        return hip_dropout(h, seq[2].p, self.training)

    def forward(self, style_emb):
        with cast_scope():   # compute-dtype weight copies valid for this call (mtts.linear)
            K = self._proj(self.key_proj, style_emb)
            V = self._proj(self.value_proj, style_emb)
        return K.unsqueeze(1), V.unsqueeze(1)


class _StyleBlock(nn.Module):
    """Shared body of the two style cross-attention blocks:
    x = LN(x + drop(MHA(x, K, V))); x = LN(x + FFN(x))."""

    def __init__(self, d_model, num_heads=8, dropout=0.1):
        super().__init__()
        self.d_model = d_model
        self.num_heads = num_heads
        self.cross_attn = CrossAttention(embed_dim=d_model, num_heads=num_heads, dropout=dropout, batch_first=True)
        self.norm = nn.LayerNorm(d_model)
        self.dropout = nn.Dropout(dropout)
        self.ffn = nn.Sequential(
            nn.Linear(d_model, d_model * 4),
            nn.GELU(),
            nn.Dropout(dropout),
            nn.Linear(d_model * 4, d_model),
            nn.Dropout(dropout),
        )
        self.ffn_norm = nn.LayerNorm(d_model)

    def _body(self, x, style_K, style_V):
        with cast_scope():   # compute-dtype weight copies valid for this call (mtts.linear)
            return self._body_scoped(x, style_K, style_V)

    def _body_scoped(self, x, style_K, style_V):
        cd = x.dtype
        attn_out, _ = self.cross_attn(query=x, key=style_K.to(cd), value=style_V.to(cd))
        x = _ln(self.norm, hip_dropout(attn_out, self.dropout.p, self.training), res=x)
        f0, f3 = self.ffn[0], self.ffn[3]
        h = ffn(x.contiguous(), f0.weight, f0.bias, f3.weight, f3.bias, p=self.ffn[2].p if self.training else 0.0)
        h = hip_dropout(h, self.ffn[4].p, self.training)
        return _ln(self.ffn_norm, h, res=x)


class StyleTextCrossAttention(_StyleBlock):
    """Cross-Attention #1: text (B, T_text, d) attends to the style token."""

    def forward(self, text_hidden, style_K, style_V, text_mask=None):
        # the reference ignores text_mask here (style is a single token)
        return self._body(text_hidden, style_K, style_V)


class LengthRegulator(nn.Module):
    """Expand phoneme-level features by rounded, clamped durations."""

    def __init__(self):
        super().__init__()

    def forward(self, hidden, durations, max_len=None):
        """hidden (B, T_text, d), durations (B, T_text) -> (expanded (B, T_frame, d),
        output_lengths (B,)), reference :156-198; one HIP kernel for the lengths
        and one for the gather (mtts_length_regulate_*)."""
        return ops.length_regulate(hidden, durations, max_len)

    def forward_with_target(self, hidden, target_durations):
        return self.forward(hidden, target_durations)


class StyleDecoderCrossAttention(_StyleBlock):
    """Cross-Attention #2: upsampled frames attend to the (reused) style token."""

    def forward(self, upsampled_hidden, style_K, style_V, frame_mask=None):
        return self._body(upsampled_hidden, style_K, style_V)


class StyleConditioningPipeline(nn.Module):
    def __init__(self, d_style=256, d_model=512, num_heads=8, dropout=0.1):
        super().__init__()
        self.compute_dtype = None   # None: the input's dtype (see the module docstring)
        self.style_proj = StyleProjection(d_style, d_model, dropout)
        self.cross_attn_1 = StyleTextCrossAttention(d_model, num_heads, dropout)
        self.cross_attn_2 = StyleDecoderCrossAttention(d_model, num_heads, dropout)
        self.length_regulator = LengthRegulator()

    def _gemm_weights(self):
        ws = []
        for m in self.modules():
            if isinstance(m, nn.Linear):
                ws += [m.weight, m.bias]
            elif isinstance(m, CrossAttention):
                ws += [m.in_proj_weight, m.in_proj_bias]
        return [w for w in ws if w is not None]

    def forward(self, text_hidden, style_emb, durations, text_mask=None, max_frame_len=None):
        if self.compute_dtype is not None:
            text_hidden, style_emb = text_hidden.to(self.compute_dtype), style_emb.to(self.compute_dtype)
        # ONE cast scope for the whole pipeline: every GEMM weight cast to the
        # compute dtype in one launch (with the W^T copies the data gradients
        # read), valid for this forward and its backward -- per-block scopes
        # would re-cast each weight at every block entry and again in the
        # backward (mtts.linear.cast_scope)
        with cast_scope(self._gemm_weights(), text_hidden.dtype):
            style_K, style_V = self.style_proj(style_emb)
            styled_text = self.cross_attn_1(text_hidden, style_K, style_V, text_mask)
            upsampled, output_lengths = self.length_regulator(styled_text, durations, max_len=max_frame_len)
            styled_frames = self.cross_attn_2(upsampled, style_K, style_V)
        return styled_frames, output_lengths, style_K, style_V


def test_style_cross_attention():
    """Shape self-test (reference :357-426), on the GPU."""
    dev = "cuda"
    batch_size, T_text, d_style, d_model = 4, 20, 256, 512
    pipeline = StyleConditioningPipeline(d_style=d_style, d_model=d_model, num_heads=8, dropout=0.1).to(dev)
    text_hidden = torch.randn(batch_size, T_text, d_model, device=dev)
    style_emb = torch.randn(batch_size, d_style, device=dev)
    durations = torch.randint(1, 5, (batch_size, T_text), device=dev).float()
    styled_frames, output_lengths, style_K, style_V = pipeline(text_hidden, style_emb, durations)
    assert styled_frames.shape[0] == batch_size
    assert styled_frames.shape[2] == d_model
    assert output_lengths.shape[0] == batch_size
    print("All tests passed!")


if __name__ == "__main__":
    test_style_cross_attention()
