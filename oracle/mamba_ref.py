"""CPU ORACLE — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the timed CPU baseline.  The product
path (mamba-tts-project_amd/) never imports it.

This is a plain-PyTorch (CPU) restatement of the arithmetic on the decoder hot
path of whcorkran/mamba-TTS-project.  The hot-path arithmetic lives in the
third-party ``mamba_ssm`` package, which the reference imports at
``mamba_decoder.py:4`` and constructs with defaults at ``mamba_decoder.py:29``.
It is NOT vendored and NOT pinned (absent from ``environment.yml:1-150``;
``README.md:29`` names it without a version), so this file restates its
published algorithm (mamba-ssm 1.x/2.x ``selective_scan_ref``,
``causal_conv1d_ref``, ``Mamba.step``), and parity is pinned against golden
vectors produced in the build container from
  * transformers' torch-only Mamba v1 (an independent implementation of the
    same math, ``transformers/models/mamba/modeling_mamba.py`` = ``HF``), and
  * the reference ``mamba_decoder.py`` / ``style_cross_attention.py`` imported
    with a ``mamba_ssm`` shim that wraps HF's mixer and honours the documented
    ``out, state = mamba(x[, state])`` contract (``mamba_decoder.py:10-15``).
The text-encoder / duration-predictor restatements (text_encoder_ref,
duration_predictor_ref, duration_loss_ref, sinusoid_table_ref) are pinned
against the reference ``text_encoder.py`` itself, imported behind a
``lib.FastSpeech2`` shim that restates the three FastSpeech2 names it imports
(tests/golden/text.npz).  See tests/golden/make_golden.py.

Layouts follow upstream mamba-ssm: u/delta/z are (B, D, L), B/C are (B, N, L).
Everything runs in the dtype and on the device of the inputs (tests use
float64 for grads; the large-shape parity tests evaluate this same
restatement on the GPU in float64 so that it finishes in seconds).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


# --------------------------------------------------------------------------
# Op-level restatements
# --------------------------------------------------------------------------

def softplus(x: torch.Tensor) -> torch.Tensor:
    """softplus with threshold 20, as torch.nn.functional.softplus and the
    upstream CUDA kernel (``delta <= 20 ? log1p(exp(delta)) : delta``)."""
    return torch.where(x <= 20.0, torch.log1p(torch.exp(torch.clamp(x, max=20.0))), x)


def selective_scan_ref(u, delta, A, B, C, D=None, z=None, delta_bias=None,
                       delta_softplus=False, h0=None, return_last_state=False):
    """Restates [upstream] mamba_ssm/ops/selective_scan_interface.py::selective_scan_ref
    (same math as HF:174-279, recurrent branch HF:248-268).

    u, delta, z : (B, D, L)      A : (D, N)      B, C : (B, N, L)
    D, delta_bias : (D,)         h0 : optional (B, D, N) initial state
      delta   <- softplus(delta + delta_bias)
      h_t      = exp(delta_t * A) * h_{t-1} + delta_t * B_t * u_t
      y_t      = <h_t, C_t> + D * u_t ;  y_t *= silu(z_t)
    Returns out (B, D, L) [, last_state (B, D, N)].
    """
    dt = delta
    if delta_bias is not None:
        dt = dt + delta_bias[None, :, None]
    if delta_softplus:
        dt = softplus(dt)
    Bsz, Dm, L = u.shape
    h = torch.zeros(Bsz, Dm, A.shape[1], dtype=u.dtype, device=u.device) if h0 is None else h0.to(u.dtype)
    ys = []
    for t in range(L):
        dA = torch.exp(dt[:, :, t, None] * A[None])                      # (B, D, N)
        dBu = dt[:, :, t, None] * B[:, None, :, t] * u[:, :, t, None]    # (B, D, N)
        h = dA * h + dBu
        ys.append((h * C[:, None, :, t]).sum(-1))
    y = torch.stack(ys, dim=-1) if L > 0 else torch.zeros_like(u)
    if D is not None:
        y = y + u * D[None, :, None]
    if z is not None:
        y = y * F.silu(z)
    return (y, h) if return_last_state else y


def causal_conv1d_ref(x, weight, bias=None, activation=None, conv_state=None):
    """Restates [upstream] causal_conv1d_ref (fallback HF:81-101): depthwise
    causal conv of width K over L with left context ``conv_state`` (B, D, K)
    (the last K pre-conv inputs; zeros when None), + bias, optional SiLU.

    x : (B, D, L), weight : (D, K).  Returns (out (B, D, L), new_conv_state
    (B, D, K)) where new_conv_state holds the last K inputs of [state ‖ x]
    (mamba-ssm ``Mamba.forward`` prefill: ``F.pad(x, (d_conv - L, 0))``).
    """
    Bsz, Dm, L = x.shape
    K = weight.shape[1]
    prev = torch.zeros(Bsz, Dm, K, dtype=x.dtype, device=x.device) if conv_state is None else conv_state.to(x.dtype)
    full = torch.cat([prev, x], dim=-1)                                  # (B, D, K+L)
    out = torch.zeros_like(x)
    for k in range(K):
        # out[t] += w[k] * full[t + 1 + k]   (full index K+t is x_t)
        out = out + weight[None, :, k, None] * full[:, :, 1 + k: 1 + k + L]
    if bias is not None:
        out = out + bias[None, :, None]
    if activation in ("silu", "swish"):
        out = F.silu(out)
    return out, full[:, :, -K:].clone()


def causal_conv1d_update_ref(x, conv_state, weight, bias=None, activation=None):
    """Restates [upstream] causal_conv1d_update / Mamba.step conv part
    (HF:61-78): roll the window, insert x (B, D), dot with weight, +b, SiLU.
    Returns (out (B, D), new_conv_state)."""
    st = torch.cat([conv_state[:, :, 1:], x[:, :, None]], dim=-1)
    out = (st * weight[None]).sum(-1)
    if bias is not None:
        out = out + bias[None]
    if activation in ("silu", "swish"):
        out = F.silu(out)
    return out, st


def selective_state_update_ref(state, x, dt, A, B, C, D=None, z=None, dt_bias=None, dt_softplus=False):
    """Restates [upstream] ops/triton/selective_state_update.py::selective_state_update_ref
    (HF:128-171).  state (B, D, N), x/dt/z (B, D), B/C (B, N).
    Returns (out (B, D), new_state)."""
    if dt_bias is not None:
        dt = dt + dt_bias[None]
    if dt_softplus:
        dt = softplus(dt)
    dA = torch.exp(dt[..., None] * A[None])
    dBx = dt[..., None] * B[:, None, :] * x[..., None]
    new_state = state * dA + dBx
    out = (new_state * C[:, None, :]).sum(-1)
    if D is not None:
        out = out + x * D[None]
    if z is not None:
        out = out * F.silu(z)
    return out, new_state


def layer_norm_ref(x, w, b, eps=1e-5):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def mha_ref(q_in, kv_in, in_w, in_b, out_w, out_b, n_heads, key_padding_mask=None):
    """Restates torch nn.MultiheadAttention(batch_first=True, dropout=0) as
    used at mamba_decoder.py:32-36,72-77 (query != key path).
    key_padding_mask: (B, S) bool, True = ignore.  Fully masked rows -> NaN
    (PyTorch semantics, reproduced on purpose)."""
    Bsz, T, d = q_in.shape
    S = kv_in.shape[1]
    hd = d // n_heads
    q = q_in @ in_w[:d].T + in_b[:d]
    k = kv_in @ in_w[d:2 * d].T + in_b[d:2 * d]
    v = kv_in @ in_w[2 * d:].T + in_b[2 * d:]
    q = q.view(Bsz, T, n_heads, hd).transpose(1, 2)
    k = k.view(Bsz, S, n_heads, hd).transpose(1, 2)
    v = v.view(Bsz, S, n_heads, hd).transpose(1, 2)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(hd)
    if key_padding_mask is not None:
        s = s.masked_fill(key_padding_mask[:, None, None, :], float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = (p @ v).transpose(1, 2).reshape(Bsz, T, d)
    return o @ out_w.T + out_b


def embed_codec_tokens_ref(tokens_3d, tok_w, pos_w, q_w):
    """Restates train.py:115-131 (embed_codec_tokens): flatten (B, Q, T) ids
    quantizer-major; ref = tok_w[ids] + pos_w[arange(T).repeat(Q)] +
    q_w[arange(Q).repeat_interleave(T)]; mask True where the id is 0."""
    B, Q, T = tokens_3d.shape
    flat = tokens_3d.reshape(B, Q * T)
    quant_ids = torch.arange(Q, device=tokens_3d.device).repeat_interleave(T).unsqueeze(0).expand(B, -1)
    pos_ids = torch.arange(T, device=tokens_3d.device).repeat(Q)
    ref = F.embedding(flat, tok_w) + F.embedding(pos_ids, pos_w)[None].expand(B, -1, -1) + F.embedding(quant_ids, q_w)
    return ref, (tokens_3d == 0).reshape(B, Q * T)


def codec_ce_loss_ref(logits, targets, pad_id=0):
    """Restates train.py:31-42: CE over (B*T, V), ignore_index=pad_id, no shift."""
    B, T, V = logits.shape
    return F.cross_entropy(logits.reshape(B * T, V), targets.reshape(B * T), ignore_index=pad_id)


def sinusoid_table_ref(n_position, d_hid, padding_idx=None):
    """FastSpeech2 transformer/Models.py get_sinusoid_encoding_table (the
    reference's text_encoder.py:16, :74-77), elementwise in float64."""
    t = torch.zeros(n_position, d_hid, dtype=torch.float64)
    for pos in range(n_position):
        for i in range(d_hid):
            a = pos / 10000 ** (2 * (i // 2) / d_hid)
            t[pos, i] = math.sin(a) if i % 2 == 0 else math.cos(a)
    if padding_idx is not None:
        t[padding_idx] = 0.0
    return t


def _conv_ref(x, w, b, pad):
    return F.conv1d(x.transpose(1, 2), w, b, padding=pad).transpose(1, 2)


def text_encoder_ref(p, ids, mask, n_layers, n_head, d_k, kernel=(9, 1), training=True, relu=torch.relu,
                     padding_idx=0):
    """Restates text_encoder.py:87-128 with FastSpeech2's FFTBlock /
    MultiHeadAttention / ScaledDotProductAttention / PositionwiseFeedForward
    (transformer/Layers.py, SubLayers.py, Modules.py; ming024, unpinned):
    x = emb + pos; per layer: attn = softmax(q k^T / sqrt(d_k), pad keys -inf)
    v -> fc -> LN(+res) -> masked_fill(pad, 0) -> conv FFN -> LN(+res) ->
    masked_fill(pad, 0).  Dropout off.  Positions: position_enc[:, :L]
    (padding row 0 zeroed), or -- eval mode with L > max_seq_len
    (text_encoder.py:107-112) -- a fresh fp32 table of L rows with row 0 NOT
    zeroed.  The embedding's padding_idx row receives no gradient
    (nn.Embedding(padding_idx), :69-71).  `relu` (tests): the FFN's activation, e.g. one that applies a
    recorded mask so the comparison follows the kernel's side of the kink."""
    B, L = ids.shape
    n_pos = p["position_enc"].shape[1]
    if not training and L > n_pos - 1:
        pos = sinusoid_table_ref(L, p["position_enc"].shape[2]).float().to(p["phoneme_emb.weight"].dtype)
    else:
        pos = p["position_enc"][0, :L]
    x = F.embedding(ids, p["phoneme_emb.weight"], padding_idx=padding_idx) + pos[None]
    for i in range(n_layers):
        pre = f"layer_stack.{i}."
        res = x
        q = x @ p[pre + "slf_attn.w_qs.weight"].T + p[pre + "slf_attn.w_qs.bias"]
        k = x @ p[pre + "slf_attn.w_ks.weight"].T + p[pre + "slf_attn.w_ks.bias"]
        v = x @ p[pre + "slf_attn.w_vs.weight"].T + p[pre + "slf_attn.w_vs.bias"]
        qh = q.view(B, L, n_head, d_k).transpose(1, 2)
        kh = k.view(B, L, n_head, d_k).transpose(1, 2)
        vh = v.view(B, L, n_head, d_k).transpose(1, 2)
        s = (qh @ kh.transpose(-1, -2)) / math.sqrt(d_k)
        s = s.masked_fill(mask[:, None, None, :], float("-inf"))
        o = (torch.softmax(s, -1) @ vh).transpose(1, 2).reshape(B, L, n_head * d_k)
        o = o @ p[pre + "slf_attn.fc.weight"].T + p[pre + "slf_attn.fc.bias"]
        x = layer_norm_ref(o + res, p[pre + "slf_attn.layer_norm.weight"], p[pre + "slf_attn.layer_norm.bias"])
        x = x.masked_fill(mask[..., None], 0.0)
        res = x
        h = relu(_conv_ref(x, p[pre + "pos_ffn.w_1.weight"], p[pre + "pos_ffn.w_1.bias"], (kernel[0] - 1) // 2))
        h = _conv_ref(h, p[pre + "pos_ffn.w_2.weight"], p[pre + "pos_ffn.w_2.bias"], (kernel[1] - 1) // 2)
        x = layer_norm_ref(h + res, p[pre + "pos_ffn.layer_norm.weight"], p[pre + "pos_ffn.layer_norm.bias"])
        x = x.masked_fill(mask[..., None], 0.0)
    return x


def duration_predictor_ref(p, x, mask, kernel=3, relu=torch.relu):
    """Restates text_encoder.py:131-181 -> FastSpeech2 model/modules.py
    VariancePredictor: [conv(k, pad (k-1)/2) -> relu -> LN] x 2 (the second
    conv's padding is 1) -> linear -> squeeze -> masked_fill(pad, 0)."""
    c = "predictor.conv_layer."
    h = relu(_conv_ref(x, p[c + "conv1d_1.conv.weight"], p[c + "conv1d_1.conv.bias"], (kernel - 1) // 2))
    h = layer_norm_ref(h, p[c + "layer_norm_1.weight"], p[c + "layer_norm_1.bias"])
    h = relu(_conv_ref(h, p[c + "conv1d_2.conv.weight"], p[c + "conv1d_2.conv.bias"], 1))
    h = layer_norm_ref(h, p[c + "layer_norm_2.weight"], p[c + "layer_norm_2.bias"])
    out = (h @ p["predictor.linear_layer.weight"].T + p["predictor.linear_layer.bias"]).squeeze(-1)
    return out.masked_fill(mask, 0.0) if mask is not None else out


def length_regulator_ref(hidden, durations, max_len=None):
    """Restates style_cross_attention.py:156-198 (LengthRegulator.forward):
    durations rounded half-to-even (torch.round) and clamped >= 0; row b of
    the output repeats hidden[b, t] dur[b, t] times, in order, truncated to
    max_len and zero-padded; lengths are the untruncated sums (int64)."""
    Bsz, T, D = hidden.shape
    dur = torch.clamp(torch.round(durations), min=0).long()
    lengths = dur.sum(dim=1)
    if max_len is None:
        max_len = int(lengths.max().item()) if Bsz > 0 else 0
    rows = []
    for b in range(Bsz):
        idx = [t for t in range(T) for _ in range(int(dur[b, t]))][:max_len]
        r = hidden[b, idx] if idx else hidden.new_zeros(0, D)
        rows.append(torch.cat([r, hidden.new_zeros(max_len - len(idx), D)], 0))
    out = torch.stack(rows) if rows else hidden.new_zeros(0, max_len, D)
    return out, lengths


# --------------------------------------------------------------------------
# Module-level restatements (state_dict keys identical to the reference)
# --------------------------------------------------------------------------

def mamba_forward_ref(p: dict, prefix: str, x, state=None, d_state=16, d_conv=4):
    """[upstream] mamba_simple.Mamba.forward / step under the contract of
    mamba_decoder.py:10-15: returns (out (B, L, d), (conv_state (B, di, K),
    ssm_state (B, di, N))).  p: flat dict of tensors keyed like the
    reference state_dict."""
    W_in = p[prefix + "in_proj.weight"]
    di = W_in.shape[0] // 2
    conv_w = p[prefix + "conv1d.weight"].reshape(di, -1)
    conv_b = p[prefix + "conv1d.bias"]
    W_x = p[prefix + "x_proj.weight"]
    W_dt = p[prefix + "dt_proj.weight"]
    b_dt = p[prefix + "dt_proj.bias"]
    A = -torch.exp(p[prefix + "A_log"])
    Dp = p[prefix + "D"]
    W_out = p[prefix + "out_proj.weight"]
    r = W_dt.shape[1]
    N = A.shape[1]

    xz = (x @ W_in.T).transpose(1, 2)                      # (B, 2di, L)
    xs, z = xz[:, :di], xz[:, di:]
    conv_state = None if state is None else state[0]
    h0 = None if state is None else state[1]
    u, new_conv = causal_conv1d_ref(xs, conv_w, conv_b, "silu", conv_state)
    x_dbl = u.transpose(1, 2) @ W_x.T                      # (B, L, r+2N)
    dt, Bm, Cm = torch.split(x_dbl, [r, N, N], dim=-1)
    delta = (dt @ W_dt.T).transpose(1, 2)                  # (B, di, L)
    y, last = selective_scan_ref(u, delta, A, Bm.transpose(1, 2), Cm.transpose(1, 2), Dp, z,
                                 b_dt, True, h0=h0, return_last_state=True)
    out = y.transpose(1, 2) @ W_out.T
    return out, (new_conv, last)


def decoder_layer_ref(p, prefix, x, text_hidden, z_style, text_mask, mamba_state, n_heads):
    """Restates MambaTTSDecoderLayer.forward (mamba_decoder.py:50-91)."""
    h = layer_norm_ref(x, p[prefix + "norm_mamba.weight"], p[prefix + "norm_mamba.bias"])
    hm, new_state = mamba_forward_ref(p, prefix + "mamba.", h, mamba_state)
    x = x + hm
    h = layer_norm_ref(x, p[prefix + "norm_cross.weight"], p[prefix + "norm_cross.bias"])
    kpm = None if text_mask is None else ~text_mask                     # :68-70 (inverted!)
    attn = mha_ref(h, text_hidden, p[prefix + "cross_attn.in_proj_weight"],
                   p[prefix + "cross_attn.in_proj_bias"], p[prefix + "cross_attn.out_proj.weight"],
                   p[prefix + "cross_attn.out_proj.bias"], n_heads, kpm)
    x = x + attn
    h = layer_norm_ref(x, p[prefix + "norm_ff.weight"], p[prefix + "norm_ff.bias"])
    gb = torch.tanh(z_style @ p[prefix + "style_mlp.0.weight"].T + p[prefix + "style_mlp.0.bias"])
    gamma, beta = torch.chunk(gb, 2, dim=-1)
    h = gamma[:, None] * h + beta[:, None]
    f = F.gelu(h @ p[prefix + "ff.0.weight"].T + p[prefix + "ff.0.bias"])
    x = x + (f @ p[prefix + "ff.2.weight"].T + p[prefix + "ff.2.bias"])
    return x, new_state


def _concat_ref(text_hidden, text_mask, ref_hidden, ref_mask):
    """mamba_decoder.py:148-165 / 226-241."""
    if ref_hidden is None:
        return text_hidden, text_mask
    B = ref_hidden.shape[0]
    if ref_mask is None:
        ref_mask = torch.ones(B, ref_hidden.shape[1], dtype=torch.bool, device=ref_hidden.device)
    text_hidden = torch.cat([ref_hidden, text_hidden], dim=1)
    text_mask = ref_mask if text_mask is None else torch.cat([ref_mask, text_mask], dim=1)
    return text_hidden, text_mask


def decoder_forward_ref(p, n_layers, n_heads, audio_tokens, text_hidden, z_style,
                        text_mask=None, ref_hidden=None, ref_mask=None):
    """Restates MambaTTSDecoder.forward (mamba_decoder.py:120-186), 2D tokens."""
    B, T = audio_tokens.shape
    text_hidden, text_mask = _concat_ref(text_hidden, text_mask, ref_hidden, ref_mask)
    if T > p["pos_embed.weight"].shape[0]:
        raise IndexError("index out of range in self")                # pos_embed(arange(T)), :169-170
    x = (p["token_embed.weight"][audio_tokens] + p["pos_embed.weight"][:T][None]
         + p["quant_embed.weight"][torch.zeros_like(audio_tokens)])
    for i in range(n_layers):
        x, _ = decoder_layer_ref(p, f"layers.{i}.", x, text_hidden, z_style, text_mask, None, n_heads)
    x = layer_norm_ref(x, p["norm_out.weight"], p["norm_out.bias"])
    return x @ p["head.weight"].T + p["head.bias"]


def decode_step_ref(p, n_layers, n_heads, last_token, text_hidden, z_style, states, step_index,
                    text_mask=None, ref_hidden=None, ref_mask=None):
    """Restates MambaTTSDecoder.decode_step (mamba_decoder.py:188-256): no
    quant_embed (quirk :217-221), pos = step_index."""
    text_hidden, text_mask = _concat_ref(text_hidden, text_mask, ref_hidden, ref_mask)
    x = p["token_embed.weight"][last_token] + p["pos_embed.weight"][step_index][None, None]
    new_states = []
    for i in range(n_layers):
        st = None if states is None else states[i]
        x, s = decoder_layer_ref(p, f"layers.{i}.", x, text_hidden, z_style, text_mask, st, n_heads)
        new_states.append(s)
    x = layer_norm_ref(x, p["norm_out.weight"], p["norm_out.bias"])
    return x @ p["head.weight"].T + p["head.bias"], new_states


# --------------------------------------------------------------------------
# Style pipeline and the train.py step (SURVEY §8f rows 1-4, configs[4] = C5)
# --------------------------------------------------------------------------

def style_pipeline_ref(p, text_hidden, style_emb, durations, n_heads, max_len=None):
    """Restates StyleConditioningPipeline.forward (style_cross_attention.py:316-354)
    with dropout off: StyleProjection (:49-66: Linear -> LayerNorm, unsqueezed
    to one token), the two cross-attention blocks (:112-141 / :258-286:
    x = LN(x + MHA(x, K, V)); x = LN(x + W2 GELU(W1 x)) ) around the
    LengthRegulator (:156-198).  p keys as the pipeline's state_dict."""
    def proj(pre):
        h = style_emb @ p[pre + ".0.weight"].T + p[pre + ".0.bias"]
        return layer_norm_ref(h, p[pre + ".1.weight"], p[pre + ".1.bias"])[:, None]

    K, V = proj("style_proj.key_proj"), proj("style_proj.value_proj")

    def block(pre, x):
        a = _mha_kv_ref(x, K, V, p[pre + ".cross_attn.in_proj_weight"], p[pre + ".cross_attn.in_proj_bias"],
                        p[pre + ".cross_attn.out_proj.weight"], p[pre + ".cross_attn.out_proj.bias"], n_heads)
        x = layer_norm_ref(x + a, p[pre + ".norm.weight"], p[pre + ".norm.bias"])
        f = F.gelu(x @ p[pre + ".ffn.0.weight"].T + p[pre + ".ffn.0.bias"]) @ p[pre + ".ffn.3.weight"].T \
            + p[pre + ".ffn.3.bias"]
        return layer_norm_ref(x + f, p[pre + ".ffn_norm.weight"], p[pre + ".ffn_norm.bias"])

    styled = block("cross_attn_1", text_hidden)
    up, lengths = length_regulator_ref(styled, durations, max_len)
    return block("cross_attn_2", up), lengths, K, V


def _mha_kv_ref(q_in, k_in, v_in, in_w, in_b, out_w, out_b, n_heads):
    """nn.MultiheadAttention(query, key, value) with distinct key / value inputs."""
    Bsz, T, d = q_in.shape
    S = k_in.shape[1]
    hd = d // n_heads
    q = (q_in @ in_w[:d].T + in_b[:d]).view(Bsz, T, n_heads, hd).transpose(1, 2)
    k = (k_in @ in_w[d:2 * d].T + in_b[d:2 * d]).view(Bsz, S, n_heads, hd).transpose(1, 2)
    v = (v_in @ in_w[2 * d:].T + in_b[2 * d:]).view(Bsz, S, n_heads, hd).transpose(1, 2)
    pr = torch.softmax((q @ k.transpose(-1, -2)) / math.sqrt(hd), dim=-1)
    return (pr @ v).transpose(1, 2).reshape(Bsz, T, d) @ out_w.T + out_b


def heuristic_durations_ref(text_mask, target_frames):
    """Restates train.py:84-97 (the per-row Python loop as written there)."""
    B, T = text_mask.shape
    lengths = (~text_mask).sum(dim=1).clamp(min=1)
    per_ph = torch.div(target_frames, lengths, rounding_mode="floor").clamp(min=1)
    durations = torch.zeros_like(text_mask, dtype=torch.float)
    for b in range(B):
        durations[b, : lengths[b]] = per_ph[b]
    return durations


def duration_loss_ref(log_duration_pred, duration_target, mask=None):
    """Restates DurationPredictor.compute_loss (text_encoder.py:183-209): MSE in
    the log domain, masked mean over non-pad phonemes."""
    log_t = torch.log(duration_target.float() + 1e-8).to(log_duration_pred.dtype)   # target built in fp32 (:196)
    loss = F.mse_loss(log_duration_pred, log_t, reduction="none")
    if mask is not None:
        return loss.masked_fill(mask, 0.0).sum() / (~mask).sum().to(loss.dtype)
    return loss.mean()


def train_step_losses_ref(p_te, p_dur, p_dec, batch, te_cfg, dec_cfg, w_codec=1.0, w_dur=0.1, w_smsd=0.5,
                          relu=torch.relu):
    """Restates the loss of one train.py step (train.py:168-230) on a synthetic
    batch, dropout off, SMSD absent (spk_embs None -> loss_smsd = 0, :192;
    z_style = the batch's fixed style vector in place of smsd(style_prompts)):
    text_encoder -> duration predictor + heuristic-duration loss -> decoder on
    the flattened codec tokens with the voice prompt embedded as reference ->
    codec CE.  The style pipeline's output is dead in train.py (:206-210) and
    enters no loss.  Returns (loss_total, loss_codec, loss_dur, logits,
    text_hidden, log_dur_pred)."""
    codec = batch["codec_tokens"]
    B, T_codec, C = codec.shape
    audio_tokens = codec.permute(0, 2, 1).reshape(B, -1)                          # :181-182
    ids, tmask = batch["phoneme_ids"], batch["text_mask"]
    text_hidden = text_encoder_ref(p_te, ids, tmask, te_cfg["n_layers"], te_cfg["n_head"], te_cfg["d_k"],
                                   te_cfg.get("kernel", (9, 1)), relu=relu)        # :188
    log_dur = duration_predictor_ref(p_dur, text_hidden, tmask, relu=relu)         # :198
    dur_t = heuristic_durations_ref(tmask, audio_tokens.shape[1])                  # :201
    loss_dur = duration_loss_ref(log_dur, dur_t, tmask)                            # :202
    v3 = batch["voice_codec"].permute(0, 2, 1)                                     # :216
    ref_hidden, vmask = embed_codec_tokens_ref(v3, p_dec["token_embed.weight"], p_dec["pos_embed.weight"],
                                               p_dec["quant_embed.weight"])        # :217
    logits = decoder_forward_ref(p_dec, dec_cfg["n_layers"], dec_cfg["n_heads"], audio_tokens, text_hidden,
                                 batch["style_emb"].to(text_hidden.dtype), text_mask=tmask, ref_hidden=ref_hidden,
                                 ref_mask=vmask)                                    # :220-227
    loss_codec = codec_ce_loss_ref(logits, audio_tokens)                           # :228
    loss_smsd = torch.zeros((), dtype=logits.dtype)
    total = w_codec * loss_codec + w_dur * loss_dur + w_smsd * loss_smsd           # :230
    return total, loss_codec, loss_dur, logits, text_hidden, log_dur
