"""Synthetic-batch harness of the reference's training step (train.py:134-242;
BASELINE configs[4] = C5).

The reference's step needs FACodec (HF Hub weights), BERT (SMSD) and the
VccmTTS tarball, none of which exist offline; everything between those
inputs and the optimizer runs here on the drop-in modules, in the reference's
order and with its semantics:

  codec (B, T, C) -> (B, C, T) -> flatten (B, C*T)              train.py:179-183
  text_encoder(phoneme_ids, mask True = pad)                    :187-188
  loss_smsd = 0 (spk_embs None), style_emb = a fixed synthetic
  z_style in place of smsd(style_prompts) (no_grad)             :190-195
  dur_predictor -> heuristic_durations -> compute_loss           :197-203
  style_pipe(text_hidden, style_emb, exp(log_dur).detach())     :205-210
  (its outputs are dead in train.py: they enter no loss)
  embed_codec_tokens(voice (B, C, T_ref), decoder)              :212-217
  decoder(audio_tokens, text_hidden, z_style, text_mask,
          ref_hidden, ref_mask = voice pad mask)                :219-227
  codec_ce_loss(logits, audio_tokens) (no shift, pad 0)         :228
  w_codec L_codec + w_dur L_dur + w_smsd L_smsd                 :230
  zero_grad; backward; clip_grad_norm_(decoder, 1.0); Adam step :232-235

Adam over all five modules with clipping over the DECODER's parameters only
(train.py:152-159, 234) = FusedClipAdam(decoder, max_grad_norm=1.0) beside
FusedClipAdam(others, no clip): Adam is element-wise, so two optimizers with
the same hyper-parameters are the same update.  With a GradAllReduce (N > 1
ranks, batch data parallel) the gradients of every trainable parameter are
all-reduced before the optimizer.

The module shapes follow build_models (train.py:45-70): d_model 512,
d_style 256, the 80-entry phoneme vocabulary, an 8-layer decoder with 5
quantizers and vocab 10; FACodec's 1024 frames per utterance (audio_encoder
pad/trunc) for both the target and the voice prompt.
"""
from __future__ import annotations

from collections import namedtuple

import torch

import codec_tokens as ct
import mamba_decoder
import style_cross_attention as sca
import text_encoder as te
from mtts import wgrad
from mtts.optim import FusedClipAdam

C5Models = namedtuple("C5Models", "text_encoder dur_predictor style_pipe decoder")

PHONEME_VOCAB = 80      # phoneme_vocab.json (10 specials + ARPAbet), train.py:48-53
CODEC_VOCAB = 10        # train.py:60-66
CODEC_STREAMS = 5       # FACodec: prosody, 3 x residual, content


def heuristic_durations(text_mask: torch.Tensor, target_frames: int) -> torch.Tensor:
    """train.py:84-97 without the per-row Python loop: row b holds
    floor(target_frames / n_b) (at least 1) in its first n_b positions, n_b =
    its non-pad count clamped to >= 1; float32 like torch.zeros_like(mask,
    dtype=torch.float)."""
    B, T = text_mask.shape
    lengths = (~text_mask).sum(dim=1).clamp(min=1)
    per_ph = torch.div(target_frames, lengths, rounding_mode="floor").clamp(min=1)
    pos = torch.arange(T, device=text_mask.device)
    return torch.where(pos[None] < lengths[:, None], per_ph[:, None].to(torch.float), torch.zeros((), device=text_mask.device))


def build_models(device, d_model=512, d_style=256, vocab_size_text=PHONEME_VOCAB, dec_layers=8, dec_heads=8,
                 d_ff=2048, num_quantizers=CODEC_STREAMS, text_layers=4, text_heads=2, text_d_k=64,
                 text_d_inner=1024, dur_filter=256, style_heads=8, dropout=0.1, max_len=8192,
                 compute_dtype=None) -> C5Models:
    """build_models (train.py:45-70) minus SMSD and FACodec (network-only).
    Defaults are train.py's; the keyword arguments shrink it for parity tests.
    `compute_dtype` is the decoder's (bf16 for the benchmark)."""
    enc = te.TextEncoder(vocab_size_text, d_model=d_model, n_layers=text_layers, n_head=text_heads, d_k=text_d_k,
                         d_v=text_d_k, d_inner=text_d_inner, dropout=dropout).to(device)
    dur = te.DurationPredictor(d_model=d_model, filter_size=dur_filter, dropout=dropout).to(device)
    pipe = sca.StyleConditioningPipeline(d_style=d_style, d_model=d_model, num_heads=style_heads,
                                         dropout=dropout).to(device)
    dec = mamba_decoder.MambaTTSDecoder(vocab_size_audio=CODEC_VOCAB, d_model=d_model, n_layers=dec_layers,
                                        n_heads=dec_heads, d_ff=d_ff, d_style=d_style, max_len=max_len,
                                        num_quantizers=num_quantizers).to(device)
    dec.compute_dtype = compute_dtype
    # train.py's style branch is dead (its output enters no loss, :206-210):
    # it runs in the decoder's compute dtype (bf16 for the benchmark: the FFN
    # on the hand-written NT GEMM instead of fp32 vendor GEMMs over ~40 k
    # regulated frames)
    pipe.compute_dtype = compute_dtype
    return C5Models(enc, dur, pipe, dec)


def synthetic_batch(B, device, T_text=128, T_codec=1024, T_ref=1024, n_streams=CODEC_STREAMS, d_style=256,
                    vocab_text=PHONEME_VOCAB, vocab_audio=CODEC_VOCAB, seed=0, min_text_frac=0.6):
    """One batch of the shapes train.py feeds its step: right-padded phoneme
    ids (the first row unpadded) with mask True = pad (TextProcessor.
    batch_process), FACodec-layout target and voice tokens (B, T, C) drawn
    from the codebook (0 is both the pad id and a valid code, quirk 4), and a
    fixed N(0, 1) style vector for z_style."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    lengths = torch.randint(max(1, int(T_text * min_text_frac)), T_text + 1, (B,), generator=g)
    lengths[0] = T_text
    mask = torch.arange(T_text)[None] >= lengths[:, None]
    ids = torch.randint(1, vocab_text, (B, T_text), generator=g).masked_fill(mask, 0)
    codec = torch.randint(0, vocab_audio, (B, T_codec, n_streams), generator=g)
    voice = torch.randint(0, vocab_audio, (B, T_ref, n_streams), generator=g)
    style = torch.randn(B, d_style, generator=g)
    return {"phoneme_ids": ids.to(device), "text_mask": mask.to(device), "codec_tokens": codec.to(device),
            "voice_codec": voice.to(device), "style_emb": style.to(device)}


class TrainStep:
    """One optimisation step of train.py's loop body (train.py:168-241) on the
    drop-in modules.  Call with a batch from `synthetic_batch`; returns the
    loss terms as device scalars (no host sync besides the style pipeline's
    length read, which the reference makes too)."""

    def __init__(self, models: C5Models, lr=1e-4, w_codec=1.0, w_dur=0.1, w_smsd=0.5, grad_allreduce=None,
                 train_mode=True):
        self.m = models
        self.w = (w_codec, w_dur, w_smsd)
        for mod in models:
            mod.train(train_mode)
        dec_params = list(models.decoder.parameters())
        rest = [p for mod in (models.text_encoder, models.dur_predictor, models.style_pipe)
                for p in mod.parameters() if p.requires_grad]
        self.opt_dec = FusedClipAdam(dec_params, lr=lr, max_grad_norm=1.0)   # clip_grad_norm_(decoder, 1.0)
        self.opt_rest = FusedClipAdam(rest, lr=lr)
        self.dp = grad_allreduce
        self.params = dec_params + rest

    def losses(self, batch):
        """Forward of the step: (loss_total, loss_codec, loss_dur, loss_smsd, logits)."""
        enc, dur, pipe, dec = self.m
        codec = batch["codec_tokens"]
        B = codec.shape[0]
        audio_tokens, _, _ = ct.flatten_codec_tokens(codec)                        # :179-183
        ids, text_mask = batch["phoneme_ids"], batch["text_mask"]
        text_hidden = enc(ids, mask=text_mask)                                     # :188
        loss_smsd = torch.zeros((), device=codec.device)                          # :192 (spk_embs None)
        style_emb = batch["style_emb"]                                            # :193-195 (no_grad there)
        log_dur_pred = dur(text_hidden, mask=text_mask)                            # :198
        durations_target = heuristic_durations(text_mask, audio_tokens.shape[1])   # :201
        loss_dur = dur.compute_loss(log_dur_pred, durations_target, mask=text_mask)
        durations_for_lr = torch.exp(log_dur_pred).detach()                       # :203
        styled_frames, frame_lengths, _, _ = pipe(text_hidden, style_emb, durations_for_lr,
                                                  text_mask=text_mask)             # :206-208 (dead branch)
        max_frame = styled_frames.shape[1]
        _ = torch.arange(max_frame, device=codec.device)[None, :].expand(B, -1) >= frame_lengths[:, None]  # :210
        _, voice3, _ = ct.flatten_codec_tokens(batch["voice_codec"])               # :215-216
        ref_hidden, voice_mask = ct.embed_codec_tokens(voice3, dec)                # :217
        logits = dec(audio_tokens, text_hidden=text_hidden, z_style=style_emb, text_mask=text_mask,
                     ref_hidden=ref_hidden, ref_mask=voice_mask)                   # :220-227
        loss_codec = ct.codec_ce_loss(logits, audio_tokens, pad_id=0)              # :228
        w_codec, w_dur, w_smsd = self.w
        total = w_codec * loss_codec + w_dur * loss_dur + w_smsd * loss_smsd       # :230
        return total, loss_codec, loss_dur, loss_smsd, logits

    def backward(self, total):
        if self.dp is not None:
            self.dp.zero_grad()
        else:
            for p in self.params:
                p.grad = None                                                      # optim.zero_grad(), :232
        with wgrad.deferred():      # projection weight gradients grouped per layer (mtts/wgrad.py)
            total.backward()                                                       # :233
        if self.dp is not None:
            self.dp.finish()

    def optimizer_step(self):
        self.opt_dec.step()                                                        # :234-235
        self.opt_rest.step()

    def __call__(self, batch):
        total, lc, ld, ls, _ = self.losses(batch)
        self.backward(total)
        self.optimizer_step()
        return {"loss_total": total.detach(), "codec": lc.detach(), "dur": ld.detach(), "smsd": ls}
