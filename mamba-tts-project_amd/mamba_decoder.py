# mamba_decoder.py — MI355X-native drop-in for whcorkran/mamba-TTS-project's
# mamba_decoder.py.  Same classes, constructor/forward/decode_step signatures
# and state_dict keys (mamba_decoder.py:25-256 of the reference); the
# arithmetic runs on libmtts HIP kernels (mtts/) instead of mamba-ssm CUDA.
"""Mamba-based TTS decoder (drop-in).

- `MambaTTSDecoderLayer(d_model, n_heads, d_ff, d_style)`:
  LN -> Mamba -> +res -> LN -> cross-attn(text) -> +res -> LN -> FiLM -> FFN -> +res
  (reference mamba_decoder.py:50-91).  The two "+res then LN" pairs run as
  one fused HIP kernel (residual add + LayerNorm [+ FiLM]).
- `MambaTTSDecoder(...)`: embeddings, layer stack, `forward` (teacher forced)
  and `decode_step` (one AR step with per-layer states kept in HBM).

Reference quirks reproduced on purpose:
  * key_padding_mask = ~text_mask (True in text_mask = attend);
  * decode_step adds no quant_embed;
  * FiLM is gamma*h + beta with tanh-bounded gamma; GELU is exact (erf);
  * 3D tokens (B, Q, T) with Q > 1 raise RuntimeError (the reference adds
    pos_embed(arange(T)) to Q*T token rows: size mismatch, :169-171).

Precision: set `model.compute_dtype = torch.bfloat16` to run activations and
GEMMs in bf16 (params stay fp32 masters; scan/LN math is fp32 internally).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from mtts.mamba import Mamba
from mtts.attention import CrossAttention, kv_all, kv_all_ok
from mtts import ops
from mtts.linear import BiasGradSlot, cast_scope, ffn, linear
from mtts.decode import DecodeEngine
from mtts.embed import embed_sum


class StyleMLPAll(torch.autograd.Function):
    """All layers' FiLM conditioning tanh(z W_l^T + b_l) at once (reference
    mamba_decoder.py:52-55, 82-84): forward one baddbmm + tanh (fp32 outputs:
    the FiLM LayerNorm kernel reads them as they are, no cast); the
    backward takes the n_layers gamma|beta gradients together (one stack),
    one tanh-backward, one bmm for the weight gradients, one sum for the
    biases and one for z -- instead of ~8 small launches per layer (and no
    zero-filled per-layer slices of a stacked gradient)."""

    @staticmethod
    def forward(ctx, z, cd, *params):
        ws, bs = params[0::2], params[1::2]
        W = torch.stack(ws)                                               # (L, 2d, d_style)
        b = torch.stack(bs)                                               # (L, 2d)
        gb = torch.tanh(torch.baddbmm(b[:, None, :], z[None].expand(len(ws), -1, -1), W.transpose(1, 2)))
        ctx.save_for_backward(z, W, gb)
        return tuple(gb[i] for i in range(len(ws)))

    @staticmethod
    def backward(ctx, *grads):
        z, W, gb = ctx.saved_tensors
        L = W.shape[0]
        g = torch.stack([gi if gi is not None else torch.zeros_like(gb[0]) for gi in grads]).to(gb.dtype)
        dpre = g * (1.0 - gb * gb)                                        # tanh'
        dW = torch.bmm(dpre.transpose(1, 2), z[None].expand(L, -1, -1))   # (L, 2d, d_style)
        db = dpre.sum(1)                                                  # (L, 2d)
        dz = torch.bmm(dpre, W).sum(0) if ctx.needs_input_grad[0] else None
        out = [dz, None]
        for i in range(L):
            out += [dW[i], db[i]]
        return tuple(out)


class MambaTTSDecoderLayer(nn.Module):
    def __init__(self, d_model, n_heads, d_ff, d_style):
        super().__init__()
        self.norm_mamba = nn.LayerNorm(d_model)
        self.mamba = Mamba(d_model)

        self.norm_cross = nn.LayerNorm(d_model)
        self.cross_attn = CrossAttention(embed_dim=d_model, num_heads=n_heads, batch_first=True)

        self.norm_ff = nn.LayerNorm(d_model)
        self.ff = nn.Sequential(
            nn.Linear(d_model, d_ff),
            nn.GELU(),
            nn.Linear(d_ff, d_model),
        )

        self.style_mlp = nn.Sequential(
            nn.Linear(d_style, 2 * d_model),
            nn.Tanh(),
        )

    def forward(self, x, text_hidden, z_style, text_mask=None, mamba_state=None):
        with cast_scope():
            x, ff_out, new_state = self.forward_fused(x, None, text_hidden, z_style, text_mask, mamba_state,
                                                      ff_slot=False)
        return x + ff_out, new_state                                          # :88-89

    def forward_fused(self, x, pending, text_hidden, z_style, text_mask=None, mamba_state=None, kpm=None, gb=None,
                      ff_slot=True, kv=None):
        """Same math as forward(); the input residual `x + pending` and the
        output residual `x + ff_out` are left to the neighbouring fused
        residual+LayerNorm kernels.  `gb` (B, 2d): this layer's
        style_mlp(z_style) when the decoder computed all layers' at once.
        Bias gradients of out_proj (:77) and ff[2] (:88) come from the fused
        residual+LayerNorm backward that consumes those outputs (BiasGradSlot;
        `ff_slot`: ff_out feeds only the next fused LayerNorm, which reads the
        slot attached to it as `_mtts_dbias_slot`).
        `kv`: this layer's K/V projection of text_hidden when the decoder
        ran all layers' at once (mtts.attention.kv_all).
        Returns (x, ff_out, new_state)."""
        T = x.shape[1]
        # 1) (x += pending) ; h = norm_mamba(x) ; Mamba   (mamba_decoder.py:59-64)
        h, xs = ops.layer_norm(x if pending is None else pending, self.norm_mamba.weight, self.norm_mamba.bias,
                               self.norm_mamba.eps, res=None if pending is None else x,
                               colsum_slot=getattr(pending, "_mtts_dbias_slot", None))
        if pending is not None:
            x = xs
        h_mamba, new_state = self.mamba(h, mamba_state)

        # 2) x = x + h_mamba ; h = norm_cross(x)   (fused, :64-67)
        h, x = ops.layer_norm(h_mamba, self.norm_cross.weight, self.norm_cross.bias, self.norm_cross.eps, res=x)
        key_padding_mask = kpm                     # precomputed once per decoder forward
        if key_padding_mask is None and text_mask is not None:
            key_padding_mask = ~text_mask                                   # :68-70 (sic)
        attn_slot = BiasGradSlot()
        attn_out, _ = self.cross_attn(query=h, key=text_hidden, value=text_hidden,
                                      key_padding_mask=key_padding_mask, _dbias_slot=attn_slot, _kv=kv)

        # 3) x = x + attn ; h = gamma * norm_ff(x) + beta   (fused, :78-86);
        # gamma | beta as ONE fp32 (B, 2d) tensor (its gradient written in place)
        if gb is None:
            gb = self.style_mlp(z_style.to(self.style_mlp[0].weight.dtype))
        h, x = ops.layer_norm(attn_out, self.norm_ff.weight, self.norm_ff.bias, self.norm_ff.eps, res=x,
                              rows_per_group=T, film=gb, colsum_slot=attn_slot)
        f0, f2 = self.ff[0], self.ff[2]
        slot = BiasGradSlot() if ff_slot else None
        ff_out = ffn(h, f0.weight, f0.bias, f2.weight, f2.bias, dbias_slot=slot)   # :88 (gelu(ff0) -> ff2)
        if slot is not None:
            ff_out._mtts_dbias_slot = slot
        return x, ff_out, new_state


class MambaTTSDecoder(nn.Module):
    def __init__(
        self,
        vocab_size_audio,
        d_model=512,
        n_layers=8,
        n_heads=8,
        d_ff=2048,
        d_style=256,
        max_len=8192,  # allow flattened multi-quantizer codec sequences
        num_quantizers=1,
    ):
        super().__init__()
        self.vocab_size_audio = vocab_size_audio
        self.token_embed = nn.Embedding(vocab_size_audio, d_model)
        self.pos_embed = nn.Embedding(max_len, d_model)
        self.quant_embed = nn.Embedding(num_quantizers, d_model)

        self.layers = nn.ModuleList([
            MambaTTSDecoderLayer(d_model, n_heads, d_ff, d_style)
            for _ in range(n_layers)
        ])

        self.norm_out = nn.LayerNorm(d_model)
        self.head = nn.Linear(d_model, vocab_size_audio)
        self.compute_dtype = None  # e.g. torch.bfloat16
        # decode_step under torch.no_grad on HIP tensors runs the incremental
        # engine (mtts/decode.py): "graph" (hipGraph replay), "eager", or None
        # for the generic per-module path.
        self.decode_mode = "graph"
        self._engine = None

    def reset_decode_cache(self):
        """Drop cached conditioning K/V, FiLM and graphs (call after editing weights)."""
        self._engine = None

    # -- helpers ----------------------------------------------------------
    def _cd(self):
        return self.compute_dtype if self.compute_dtype is not None else self.token_embed.weight.dtype

    @staticmethod
    def _concat_ref(text_hidden, text_mask, ref_hidden, ref_mask, B, device):
        if ref_hidden is not None:
            assert ref_hidden.dim() == 3 and ref_hidden.shape[0] == B, (
                "ref_hidden must be (B, T_ref, d_model)"
            )
            if ref_mask is None:
                ref_mask = torch.ones(B, ref_hidden.shape[1], dtype=torch.bool, device=device)
            else:
                assert ref_mask.dim() == 2 and ref_mask.shape[0] == B, (
                    "ref_mask must be (B, T_ref) bool"
                )
            text_hidden = torch.cat([ref_hidden.to(text_hidden.dtype), text_hidden], dim=1)
            if text_mask is None:
                text_mask = ref_mask
            else:
                text_mask = torch.cat([ref_mask, text_mask], dim=1)
        return text_hidden, text_mask

    def _tail(self, x, pending=None):
        """norm_out(x [+ pending]) -> head (mamba_decoder.py:184-185)."""
        h, _ = ops.layer_norm(x if pending is None else pending, self.norm_out.weight, self.norm_out.bias,
                              self.norm_out.eps, res=None if pending is None else x,
                              colsum_slot=getattr(pending, "_mtts_dbias_slot", None))
        return linear(h, self.head.weight, self.head.bias)

    def _gemm_weights(self):
        ws = [self.head.weight, self.head.bias]
        for l in self.layers:
            m = l.mamba
            ws += [m.in_proj.weight, m.x_proj.weight, m.dt_proj.weight, m.out_proj.weight,
                   l.cross_attn.in_proj_weight, l.cross_attn.in_proj_bias, l.cross_attn.out_proj.weight,
                   l.cross_attn.out_proj.bias, l.ff[0].weight, l.ff[0].bias, l.ff[2].weight, l.ff[2].bias]
        return [w for w in ws if w is not None]

    def _style_all(self, z_style, cd):
        """Every layer's style_mlp(z_style) = tanh(z W_l^T + b_l) (:52-55, applied
        at :82-84) in ONE batched GEMM over the stacked layer weights (fp32, the
        parameters' dtype, kept fp32 for the FiLM LayerNorm kernel: StyleMLPAll).
        Returns n_layers (B, 2d) tensors, or None when the layers' style MLPs
        differ in shape / dtype."""
        lins = [l.style_mlp[0] for l in self.layers]
        w0 = lins[0].weight
        if (len(lins) < 2 or any(m.weight.shape != w0.shape or m.weight.dtype != w0.dtype or m.bias is None
                                 or m.bias.dtype != w0.dtype for m in lins)):
            return None
        params = [t for m in lins for t in (m.weight, m.bias)]
        return StyleMLPAll.apply(z_style.to(w0.dtype), cd, *params)

    def _run_layers(self, x, text_hidden, z_style, text_mask, states):
        pending = None
        new_states = []
        kpm = None if text_mask is None else ~text_mask                     # :68-70 (sic), once for all layers
        gbs = self._style_all(z_style, x.dtype) if x.shape[1] > 1 else None
        # every layer's K/V projection of the shared text (+ reference) states
        # in one GEMM (mtts.attention.KVAllFn; reference :72-77 per layer)
        attns = [l.cross_attn for l in self.layers]
        kvs = kv_all(text_hidden, attns) if kv_all_ok(text_hidden, attns) else None
        for i, layer in enumerate(self.layers):
            x, pending, st = layer.forward_fused(x, pending, text_hidden, z_style, text_mask,
                                                 None if states is None else states[i], kpm=kpm,
                                                 gb=None if gbs is None else gbs[i],
                                                 kv=None if kvs is None else kvs[i])
            new_states.append(st)
        return x, pending, new_states

    # -- API --------------------------------------------------------------
    def forward(self, audio_tokens, text_hidden, z_style, text_mask=None, ref_hidden=None, ref_mask=None):
        """
        audio_tokens: either
            - (B, T_audio) int codec ids (single quantizer)
            - (B, Q, T_audio) int codec ids (multi-quantizer; flattened internally)
        text_hidden: (B, T_text, d_model) text encoder outputs
        z_style: (B, d_style) style/timbre embedding
        """
        if audio_tokens.dim() == 3:
            B, Q, T = audio_tokens.shape
            audio_tokens = audio_tokens.reshape(B, Q * T)
            quant_ids = torch.arange(Q, device=audio_tokens.device).repeat_interleave(T)   # per position
        elif audio_tokens.dim() == 2:
            B, T = audio_tokens.shape
            quant_ids = torch.zeros(T, device=audio_tokens.device, dtype=torch.long)
        else:
            raise ValueError("audio_tokens must be (B, T) or (B, Q, T)")
        device = audio_tokens.device

        if text_mask is not None:
            assert text_mask.dim() == 2 and text_mask.shape[0] == B, (
                "text_mask must be shape (B, T_text) with dtype=bool"
            )
        cd = self._cd()
        text_hidden = text_hidden.to(cd)
        text_hidden, text_mask = self._concat_ref(text_hidden, text_mask, ref_hidden, ref_mask, B, device)

        # token + position + quantizer embeddings (:167-171), fused backward.
        # The reference embeds positions arange(T) of the UNflattened length,
        # so `tok (B, Q*T, d) + pos (B, T, d)` fails for Q > 1 (quirk 3):
        # raise the same broadcast error instead of computing a result.
        if T > self.pos_embed.num_embeddings:
            raise IndexError("index out of range in self")                    # pos_embed(arange(T)), :169-170
        if audio_tokens.shape[1] != T:
            raise RuntimeError(f"The size of tensor a ({audio_tokens.shape[1]}) must match the size of tensor b "
                               f"({T}) at non-singleton dimension 1")            # tok + pos, :171
        x = embed_sum(audio_tokens, quant_ids, self.token_embed.weight, self.quant_embed.weight,
                      self.pos_embed.weight, cd)

        with cast_scope(self._gemm_weights(), cd):
            x, pending, _ = self._run_layers(x, text_hidden, z_style, text_mask, None)
            return self._tail(x, pending)

    def decode_step(
        self,
        last_token,
        text_hidden,
        z_style,
        mamba_states,
        step_index: int,
        text_mask=None,
        ref_hidden=None,
        ref_mask=None,
    ):
        """Generate logits for a single autoregressive step.

        Args:
            last_token: (B, 1) int tensor containing the most recent audio token.
            text_hidden: (B, T_text, d_model) encoder outputs.
            z_style: (B, d_style) style embedding.
            mamba_states: list of per-layer states (length == n_layers). Each
                entry may be None for the first step.
            step_index: int, absolute position index of this token (0-based).
            text_mask: optional (B, T_text) boolean mask for text padding.

        Returns:
            logits: (B, 1, vocab_size_audio)
            new_states: list of updated per-layer mamba states
        """
        B_local = last_token.shape[0]
        device = last_token.device
        cd = self._cd()
        if self.decode_mode and not torch.is_grad_enabled() and last_token.is_cuda:
            use_graph = self.decode_mode == "graph"
            if self._engine is None or self._engine.use_graph != use_graph:
                self._engine = DecodeEngine(self, use_graph=use_graph)
            return self._engine.step(last_token, text_hidden, z_style, mamba_states, step_index, text_mask,
                                     ref_hidden, ref_mask)

        tok = self.token_embed(last_token)
        pos_id = torch.tensor([step_index], device=device)
        pos = self.pos_embed(pos_id)[None, :, :].expand(B_local, 1, -1)
        x = (tok + pos).to(cd)                                               # no quant_embed (:217-221)

        text_hidden = text_hidden.to(cd)
        text_hidden, text_mask = self._concat_ref(text_hidden, text_mask, ref_hidden, ref_mask, B_local, device)

        with cast_scope(self._gemm_weights(), cd):
            x, pending, new_states = self._run_layers(x, text_hidden, z_style, text_mask, mamba_states)
            return self._tail(x, pending), new_states
