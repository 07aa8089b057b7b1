"""Codec-token plumbing of the training loop around the decoder (SURVEY.md
§8f row 3), mirroring the reference's train.py helpers with the same names,
arguments and semantics:

  codec_ce_loss(logits, targets, pad_id=0)        train.py:31-42
  embed_codec_tokens(tokens_3d, decoder)          train.py:115-131
  flatten_codec_tokens(codec_tokens)              train.py:179-183 (inline there)

FACodec tokens arrive as (B, T, C) with C = 5 streams in the order
[prosody, 3 x residual, content] (data_utils/audio_encoder.py:225-255); the
decoder consumes them quantizer-major, flattened to (B, C*T).  The reference
voice prompt is embedded through the DECODER's own tables (token + position
arange(T_ref).repeat(Q) + quantizer arange(Q).repeat_interleave(T_ref)) --
here one HIP kernel (mtts_embed_sum) with a batch-reduced backward -- and its
pad mask is True where the token is 0 (pad_id 0 is also a valid codebook id,
SURVEY quirk 4).  Note the decoder itself treats text_mask/ref_mask True as
VALID (key_padding_mask = ~mask, mamba_decoder.py:68-70); the reference
passes this True = pad mask anyway (quirk 1) and so do we.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from mtts.embed import embed_codec_layout


def codec_ce_loss(logits: torch.Tensor, targets: torch.Tensor, pad_id: int = 0) -> torch.Tensor:
    """Cross-entropy over flattened codec tokens; logits (B, T, V), targets
    (B, T) long; targets == pad_id are ignored; targets are NOT shifted."""
    B, T, V = logits.shape
    x = logits.reshape(B * T, V)
    if logits.is_cuda and logits.dtype in (torch.float32, torch.bfloat16) and x.stride(1) == 1:
        # csrc/loss.hip (fp32 / bf16 logits, unit column stride): the fp32
        # upcast happens in registers
        from mtts.loss import cross_entropy
        return cross_entropy(x, targets.reshape(B * T), ignore_index=pad_id)
    # any other dtype / layout: F.cross_entropy exactly as train.py:38-42
    return F.cross_entropy(x, targets.reshape(B * T), ignore_index=pad_id)


def flatten_codec_tokens(codec_tokens: torch.Tensor):
    """(B, T, C) codec ids -> (audio_tokens (B, C*T) quantizer-major,
    tokens_3d (B, C, T), pad mask (B, C*T) True where the id is 0)."""
    tokens_3d = codec_tokens.permute(0, 2, 1)
    B = tokens_3d.shape[0]
    audio_tokens = tokens_3d.reshape(B, -1)
    return audio_tokens, tokens_3d, (tokens_3d == 0).reshape(B, -1)


def embed_codec_tokens(tokens_3d: torch.Tensor, decoder):
    """tokens_3d (B, Q, T_ref) long -> (ref_hidden (B, Q*T_ref, d_model) in the
    decoder's compute dtype (fp32 when it has none, as the reference),
    mask (B, Q*T_ref) bool, True = pad)."""
    B, Q, T = tokens_3d.shape
    if T > decoder.pos_embed.num_embeddings:
        raise IndexError(f"T_ref {T} exceeds pos_embed max_len {decoder.pos_embed.num_embeddings}")
    if Q > decoder.quant_embed.num_embeddings:
        raise IndexError(f"{Q} quantizers exceed quant_embed's {decoder.quant_embed.num_embeddings} rows")
    cd = decoder._cd()
    ref_hidden = embed_codec_layout(tokens_3d, decoder.token_embed.weight, decoder.quant_embed.weight,
                                    decoder.pos_embed.weight, cd)
    mask = (tokens_3d == 0).reshape(B, Q * T)
    return ref_hidden, mask
