"""Generate the committed golden vectors (tests/golden/*.npz).

RUN ONLY IN THE BUILD CONTAINER (it reads /root/reference, which does not
exist on the GPU box).  The fixtures it writes are plain data (inputs +
expected outputs), loaded with numpy.load(allow_pickle=False).

Sources of truth:
  * op-level vectors: transformers' torch-only Mamba v1 functions
    (``mamba_selective_scan`` HF:174-279, ``causal_conv1d_fn`` HF:81-101,
    ``causal_conv1d_update`` HF:61-78, ``mamba_selective_state_update``
    HF:128-171) — an implementation independent of ours of the same
    mamba-ssm math; evaluated in float64 on float32-representable inputs.
  * module-level vectors: the REFERENCE ``/root/reference/mamba_decoder.py``
    and ``style_cross_attention.py`` themselves, imported with a
    ``mamba_ssm`` shim whose ``Mamba`` subclasses HF ``MambaMixer`` (same
    parameter names/shapes as mamba-ssm) and honours the documented
    ``out, state = mamba(x[, state])`` contract (mamba_decoder.py:10-15).

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import math
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

from transformers import MambaConfig  # noqa: E402
from transformers.models.mamba import modeling_mamba as HF  # noqa: E402


# ---------------------------------------------------------------------------
# mamba_ssm shim (documented contract) over HF's torch path
# ---------------------------------------------------------------------------
class ShimMamba(HF.MambaMixer):
    """Mamba(d_model) with mamba-ssm defaults: d_state=16, d_conv=4, expand=2,
    dt_rank=ceil(d/16), bias=False, conv_bias=True."""

    def __init__(self, d_model, d_state=16, d_conv=4, expand=2):
        cfg = MambaConfig(hidden_size=d_model, state_size=d_state, expand=expand,
                          conv_kernel=d_conv, use_bias=False, use_conv_bias=True,
                          num_hidden_layers=1)
        super().__init__(cfg, layer_idx=0)

    def forward(self, x, state=None):  # noqa: D401
        L = x.shape[1]
        di, K = self.intermediate_size, self.conv_kernel_size
        xz = self.in_proj(x).transpose(1, 2)
        xs, z = xz.chunk(2, dim=1)
        A = -torch.exp(self.A_log)
        w = self.conv1d.weight.squeeze(1)
        if state is None:
            conv_state = nn.functional.pad(xs, (K - L, 0)) if L < K else xs[..., -K:]
            u = HF.causal_conv1d_fn(xs, w, self.conv1d.bias, activation="silu")
            h0 = None
        else:
            conv_state, h0 = state
            assert L == 1, "shim step path is L == 1 (mamba-ssm Mamba.step)"
            conv_state = conv_state.clone()
            u = HF.causal_conv1d_update(xs, conv_state, w, self.conv1d.bias, activation="silu")
        dt, Bm, Cm = torch.split(self.x_proj(u.transpose(1, 2)),
                                 [self.time_step_rank, self.ssm_state_size, self.ssm_state_size], dim=-1)
        delta = self.dt_proj.weight @ dt.transpose(1, 2)
        if h0 is None:
            y, last = HF.mamba_selective_scan(u, delta, A, Bm.transpose(1, 2), Cm.transpose(1, 2),
                                              D=self.D, z=z, delta_bias=self.dt_proj.bias,
                                              delta_softplus=True, return_last_state=True)
        else:
            last = h0.clone()
            y = HF.mamba_selective_state_update(last, u[..., 0], delta[..., 0], A, Bm[:, 0], Cm[:, 0],
                                                self.D, z=z[..., 0], dt_bias=self.dt_proj.bias,
                                                dt_softplus=True).unsqueeze(-1)
        out = self.out_proj(y.transpose(1, 2))
        return out, (conv_state, last)


def import_reference():
    shim = types.ModuleType("mamba_ssm")
    shim.Mamba = ShimMamba
    sys.modules["mamba_ssm"] = shim
    sys.path.insert(0, REF)
    import mamba_decoder  # noqa: F401
    import style_cross_attention  # noqa: F401
    return mamba_decoder, style_cross_attention


# ---------------------------------------------------------------------------
# lib.FastSpeech2 shim: the three names /root/reference/text_encoder.py:16-18
# imports from ming024/FastSpeech2 (cloned unpinned by setup.sh, absent here),
# restated from that repository's published code -- transformer/Models.py
# get_sinusoid_encoding_table, transformer/Layers.py FFTBlock,
# transformer/SubLayers.py MultiHeadAttention + PositionwiseFeedForward,
# transformer/Modules.py ScaledDotProductAttention, model/modules.py
# VariancePredictor + Conv.  Written against torch directly (independent of
# the product's text_encoder.py); the reference's OWN code around them
# (TextEncoder.forward's embedding, position_enc slice and eval branch,
# DurationPredictor.compute_loss, TextProcessor) runs unmodified.
# ---------------------------------------------------------------------------
def fs2_sinusoid_table(n_position, d_hid, padding_idx=None):
    def angle(pos, j):
        return pos / np.power(10000, 2 * (j // 2) / d_hid)

    table = np.array([[angle(p, j) for j in range(d_hid)] for p in range(n_position)])
    table[:, 0::2] = np.sin(table[:, 0::2])
    table[:, 1::2] = np.cos(table[:, 1::2])
    if padding_idx is not None:
        table[padding_idx] = 0.0
    return torch.FloatTensor(table)


class FS2ScaledDotProductAttention(nn.Module):
    def __init__(self, temperature):
        super().__init__()
        self.temperature = temperature
        self.softmax = nn.Softmax(dim=2)

    def forward(self, q, k, v, mask=None):
        attn = torch.bmm(q, k.transpose(1, 2)) / self.temperature
        if mask is not None:
            attn = attn.masked_fill(mask, -np.inf)
        attn = self.softmax(attn)
        return torch.bmm(attn, v), attn


class FS2MultiHeadAttention(nn.Module):
    def __init__(self, n_head, d_model, d_k, d_v, dropout=0.1):
        super().__init__()
        self.n_head, self.d_k, self.d_v = n_head, d_k, d_v
        self.w_qs = nn.Linear(d_model, n_head * d_k)
        self.w_ks = nn.Linear(d_model, n_head * d_k)
        self.w_vs = nn.Linear(d_model, n_head * d_v)
        self.attention = FS2ScaledDotProductAttention(temperature=np.power(d_k, 0.5))
        self.layer_norm = nn.LayerNorm(d_model)
        self.fc = nn.Linear(n_head * d_v, d_model)
        self.dropout = nn.Dropout(dropout)

    def forward(self, q, k, v, mask=None):
        d_k, d_v, n_head = self.d_k, self.d_v, self.n_head
        sz_b, len_q, _ = q.size()
        _, len_k, _ = k.size()
        _, len_v, _ = v.size()
        residual = q
        q = self.w_qs(q).view(sz_b, len_q, n_head, d_k)
        k = self.w_ks(k).view(sz_b, len_k, n_head, d_k)
        v = self.w_vs(v).view(sz_b, len_v, n_head, d_v)
        q = q.permute(2, 0, 1, 3).contiguous().view(-1, len_q, d_k)
        k = k.permute(2, 0, 1, 3).contiguous().view(-1, len_k, d_k)
        v = v.permute(2, 0, 1, 3).contiguous().view(-1, len_v, d_v)
        mask = mask.repeat(n_head, 1, 1)
        output, attn = self.attention(q, k, v, mask=mask)
        output = output.view(n_head, sz_b, len_q, d_v)
        output = output.permute(1, 2, 0, 3).contiguous().view(sz_b, len_q, -1)
        output = self.dropout(self.fc(output))
        return self.layer_norm(output + residual), attn


class FS2PositionwiseFeedForward(nn.Module):
    def __init__(self, d_in, d_hid, kernel_size, dropout=0.1):
        super().__init__()
        self.w_1 = nn.Conv1d(d_in, d_hid, kernel_size=kernel_size[0], padding=(kernel_size[0] - 1) // 2)
        self.w_2 = nn.Conv1d(d_hid, d_in, kernel_size=kernel_size[1], padding=(kernel_size[1] - 1) // 2)
        self.layer_norm = nn.LayerNorm(d_in)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        residual = x
        output = self.w_2(torch.relu(self.w_1(x.transpose(1, 2)))).transpose(1, 2)
        return self.layer_norm(self.dropout(output) + residual)


class FS2FFTBlock(nn.Module):
    def __init__(self, d_model, n_head, d_k, d_v, d_inner, kernel_size, dropout=0.1):
        super().__init__()
        self.slf_attn = FS2MultiHeadAttention(n_head, d_model, d_k, d_v, dropout=dropout)
        self.pos_ffn = FS2PositionwiseFeedForward(d_model, d_inner, kernel_size, dropout=dropout)

    def forward(self, enc_input, mask=None, slf_attn_mask=None):
        enc_output, enc_slf_attn = self.slf_attn(enc_input, enc_input, enc_input, mask=slf_attn_mask)
        enc_output = enc_output.masked_fill(mask.unsqueeze(-1), 0)
        enc_output = self.pos_ffn(enc_output)
        enc_output = enc_output.masked_fill(mask.unsqueeze(-1), 0)
        return enc_output, enc_slf_attn


class FS2Conv(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size=1, stride=1, padding=0, dilation=1, bias=True,
                 w_init="linear"):
        super().__init__()
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size=kernel_size, stride=stride, padding=padding,
                              dilation=dilation, bias=bias)

    def forward(self, x):
        return self.conv(x.contiguous().transpose(1, 2)).contiguous().transpose(1, 2)


class FS2VariancePredictor(nn.Module):
    def __init__(self, model_config):
        super().__init__()
        from collections import OrderedDict
        self.input_size = model_config["transformer"]["encoder_hidden"]
        self.filter_size = model_config["variance_predictor"]["filter_size"]
        self.kernel = model_config["variance_predictor"]["kernel_size"]
        self.conv_output_size = model_config["variance_predictor"]["filter_size"]
        self.dropout = model_config["variance_predictor"]["dropout"]
        self.conv_layer = nn.Sequential(OrderedDict([
            ("conv1d_1", FS2Conv(self.input_size, self.filter_size, kernel_size=self.kernel,
                                 padding=(self.kernel - 1) // 2)),
            ("relu_1", nn.ReLU()),
            ("layer_norm_1", nn.LayerNorm(self.filter_size)),
            ("dropout_1", nn.Dropout(self.dropout)),
            ("conv1d_2", FS2Conv(self.filter_size, self.filter_size, kernel_size=self.kernel, padding=1)),
            ("relu_2", nn.ReLU()),
            ("layer_norm_2", nn.LayerNorm(self.filter_size)),
            ("dropout_2", nn.Dropout(self.dropout)),
        ]))
        self.linear_layer = nn.Linear(self.conv_output_size, 1)

    def forward(self, encoder_output, mask):
        out = self.linear_layer(self.conv_layer(encoder_output)).squeeze(-1)
        if mask is not None:
            out = out.masked_fill(mask, 0.0)
        return out


def import_reference_text_encoder():
    """/root/reference/text_encoder.py itself, behind the lib.FastSpeech2 shim."""
    import importlib.util
    names = {
        "lib": {}, "lib.FastSpeech2": {}, "lib.FastSpeech2.transformer": {}, "lib.FastSpeech2.model": {},
        "lib.FastSpeech2.transformer.Models": {"get_sinusoid_encoding_table": fs2_sinusoid_table},
        "lib.FastSpeech2.transformer.Layers": {"FFTBlock": FS2FFTBlock},
        "lib.FastSpeech2.model.modules": {"VariancePredictor": FS2VariancePredictor},
    }
    for name, attrs in names.items():
        mod = types.ModuleType(name)
        mod.__path__ = []
        for k, v in attrs.items():
            setattr(mod, k, v)
        sys.modules[name] = mod
    spec = importlib.util.spec_from_file_location("ref_text_encoder", os.path.join(REF, "text_encoder.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def f32(t):
    return t.detach().to(torch.float32).cpu().numpy()


def rnd(g, *shape, scale=1.0):
    # float32-representable values, promoted to float64 for evaluation
    return (torch.randn(*shape, generator=g, dtype=torch.float32) * scale).double()


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: np.ascontiguousarray(v) for k, v in arrays.items()})
    print(f"wrote {name}: {os.path.getsize(path) / 1024:.1f} KiB, {len(arrays)} arrays")


# ---------------------------------------------------------------------------
# 1. selective scan (fwd + bwd)
# ---------------------------------------------------------------------------
def gen_scan(name, Bsz, Dm, L, N=16, use_z=True, use_D=True, use_bias=True, softplus=True, seed=0):
    g = torch.Generator().manual_seed(seed)
    u = rnd(g, Bsz, Dm, L)
    delta = rnd(g, Bsz, Dm, L, scale=0.5)
    A = -torch.exp(rnd(g, Dm, N, scale=0.5) + torch.log(torch.arange(1, N + 1, dtype=torch.float64)))
    A = A.float().double()
    Bm = rnd(g, Bsz, N, L)
    Cm = rnd(g, Bsz, N, L)
    D = rnd(g, Dm) if use_D else None
    z = rnd(g, Bsz, Dm, L) if use_z else None
    dt0 = torch.exp(torch.rand(Dm, generator=g) * (math.log(0.1) - math.log(1e-3)) + math.log(1e-3))
    bias = (dt0 + torch.log(-torch.expm1(-dt0))).float().double() if use_bias else None
    if not softplus:
        delta = delta.abs() * 0.2
    ins = dict(u=u, delta=delta, A=A, B=Bm, C=Cm)
    if D is not None:
        ins["D"] = D
    if z is not None:
        ins["z"] = z
    if bias is not None:
        ins["delta_bias"] = bias
    req = {k: v.clone().requires_grad_(True) for k, v in ins.items()}
    out, last = HF.mamba_selective_scan(req["u"], req["delta"], req["A"], req["B"], req["C"],
                                        D=req.get("D"), z=req.get("z"), delta_bias=req.get("delta_bias"),
                                        delta_softplus=softplus, return_last_state=True)
    dout = rnd(g, Bsz, Dm, L)
    (out * dout).sum().backward()
    arrays = {k: f32(v) for k, v in ins.items()}
    arrays.update(out=f32(out), last_state=f32(last), dout=f32(dout),
                  softplus=np.array(int(softplus)))
    for k, v in req.items():
        arrays["d" + k] = f32(v.grad)
    save(name, **arrays)


# ---------------------------------------------------------------------------
# 2. causal conv1d fwd/bwd + update sequence; state-update decode vs full scan
# ---------------------------------------------------------------------------
def gen_conv(seed=1):
    g = torch.Generator().manual_seed(seed)
    Bsz, Dm, L, K = 2, 64, 64, 4
    x = rnd(g, Bsz, Dm, L)
    w = rnd(g, Dm, K, scale=0.5)
    b = rnd(g, Dm, scale=0.5)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    out = HF.causal_conv1d_fn(xr, wr, br, activation="silu")
    dout = rnd(g, Bsz, Dm, L)
    (out * dout).sum().backward()
    # update sequence: 8 steps from a zero window == conv over those 8 steps
    T = 8
    xs = rnd(g, Bsz, Dm, T)
    state = torch.zeros(Bsz, Dm, K, dtype=torch.float64)
    ups = []
    for t in range(T):
        ups.append(HF.causal_conv1d_update(xs[:, :, t:t + 1], state, w, b, activation="silu")[:, :, 0])
    save("conv1d.npz", x=f32(x), w=f32(w), b=f32(b), out=f32(out), dout=f32(dout),
         dx=f32(xr.grad), dw=f32(wr.grad), db=f32(br.grad),
         xs=f32(xs), upd_out=f32(torch.stack(ups, -1)), upd_state=f32(state))


def gen_state_update(seed=2):
    g = torch.Generator().manual_seed(seed)
    Bsz, Dm, T, N = 2, 32, 16, 16
    u = rnd(g, Bsz, Dm, T)
    delta = rnd(g, Bsz, Dm, T, scale=0.5)
    A = (-torch.exp(rnd(g, Dm, N, scale=0.3))).float().double()
    Bm, Cm = rnd(g, Bsz, N, T), rnd(g, Bsz, N, T)
    D, z, bias = rnd(g, Dm), rnd(g, Bsz, Dm, T), rnd(g, Dm, scale=0.2)
    state = torch.zeros(Bsz, Dm, N, dtype=torch.float64)
    outs = []
    for t in range(T):
        outs.append(HF.mamba_selective_state_update(state, u[:, :, t], delta[:, :, t], A, Bm[:, :, t],
                                                    Cm[:, :, t], D, z=z[:, :, t], dt_bias=bias,
                                                    dt_softplus=True))
    full, last = HF.mamba_selective_scan(u, delta, A, Bm, Cm, D=D, z=z, delta_bias=bias,
                                         delta_softplus=True, return_last_state=True)
    save("state_update.npz", u=f32(u), delta=f32(delta), A=f32(A), B=f32(Bm), C=f32(Cm), D=f32(D),
         z=f32(z), delta_bias=f32(bias), step_out=f32(torch.stack(outs, -1)), step_state=f32(state),
         full_out=f32(full), full_state=f32(last))


# ---------------------------------------------------------------------------
# 3./4. decoder layer stack + decode_step through the REFERENCE module
# ---------------------------------------------------------------------------
DEC = dict(vocab_size_audio=10, d_model=64, n_layers=2, n_heads=4, d_ff=128, d_style=16, max_len=256)


def perturb_norms(model, g):
    with torch.no_grad():
        for name, p in model.named_parameters():
            if "norm" in name:
                p.add_(0.1 * torch.randn(p.shape, generator=g, dtype=p.dtype))
            if name.endswith("in_proj_bias") or name.endswith("out_proj.bias") or name.endswith("ff.0.bias"):
                p.add_(0.1 * torch.randn(p.shape, generator=g, dtype=p.dtype))


def gen_decoder(mdec, seed=3):
    torch.manual_seed(seed)
    g = torch.Generator().manual_seed(seed + 100)
    model = mdec.MambaTTSDecoder(**DEC).double()
    perturb_norms(model, g)
    model.train()  # dropout is 0 in the decoder; train() exercises nothing random
    sd = {k: f32(v) for k, v in model.state_dict().items()}
    # round weights to float32 so the float64 evaluation sees the stored values
    model.load_state_dict({k: torch.from_numpy(v).double() for k, v in sd.items()})
    B, T, Tt, Tr = 3, 64, 12, 8
    d = DEC["d_model"]
    tokens = torch.randint(0, 10, (B, T), generator=g)
    text = rnd(g, B, Tt, d)
    zsty = rnd(g, B, DEC["d_style"])
    # text_mask True = VALID for the decoder (quirk: kpm = ~text_mask, mamba_decoder.py:68-70)
    tmask = torch.ones(B, Tt, dtype=torch.bool)
    tmask[0, 9:] = False
    tmask[1, 5:] = False
    ref = rnd(g, B, Tr, d)
    rmask = torch.ones(B, Tr, dtype=torch.bool)
    rmask[2, 3:] = False
    cases = {}
    for tag, kw in [("plain", dict(text_mask=None, ref_hidden=None, ref_mask=None)),
                    ("masked_ref", dict(text_mask=tmask, ref_hidden=ref, ref_mask=rmask))]:
        model.zero_grad()
        th = text.clone().requires_grad_(True)
        zs = zsty.clone().requires_grad_(True)
        rh = kw["ref_hidden"].clone().requires_grad_(True) if kw["ref_hidden"] is not None else None
        logits = model(tokens, th, zs, text_mask=kw["text_mask"], ref_hidden=rh, ref_mask=kw["ref_mask"])
        G = rnd(g, *logits.shape)
        (logits * G).sum().backward()
        c = {f"{tag}/logits": f32(logits), f"{tag}/G": f32(G), f"{tag}/dtext": f32(th.grad),
             f"{tag}/dz": f32(zs.grad)}
        if rh is not None:
            c[f"{tag}/dref"] = f32(rh.grad)
        for n, p in model.named_parameters():
            c[f"{tag}/grad/{n}"] = f32(p.grad)
        cases.update(c)
    # decode_step: 12 AR steps from empty states; same states fed back
    model.eval()
    with torch.no_grad():
        states = [None] * DEC["n_layers"]
        step_logits = []
        for t in range(12):
            lt = tokens[:, t:t + 1]
            lg, states = model.decode_step(lt, text, zsty, states, t, text_mask=tmask,
                                           ref_hidden=ref, ref_mask=rmask)
            step_logits.append(lg)
        cases["decode/logits"] = f32(torch.cat(step_logits, 1))
        for i, (cs, ss) in enumerate(states):
            cases[f"decode/conv_state{i}"] = f32(cs)
            cases[f"decode/ssm_state{i}"] = f32(ss)
    arrays = {f"sd/{k}": v for k, v in sd.items()}
    arrays.update(tokens=tokens.numpy(), text=f32(text), z_style=f32(zsty), text_mask=tmask.numpy(),
                  ref=f32(ref), ref_mask=rmask.numpy(), **cases)
    save("decoder.npz", **arrays)


def gen_style(msca, seed=4):
    torch.manual_seed(seed)
    g = torch.Generator().manual_seed(seed + 100)
    pipe = msca.StyleConditioningPipeline(d_style=16, d_model=64, num_heads=4, dropout=0.1).double()
    perturb_norms(pipe, g)
    pipe.eval()  # dropout off
    sd = {k: f32(v) for k, v in pipe.state_dict().items()}
    pipe.load_state_dict({k: torch.from_numpy(v).double() for k, v in sd.items()})
    B, Tt = 3, 10
    text = rnd(g, B, Tt, 64)
    style = rnd(g, B, 16)
    dur = torch.randint(0, 5, (B, Tt), generator=g).double() + 0.3  # rounding exercised
    dur[1, 4] = -1.0  # clamp >= 0 exercised
    with torch.no_grad():
        frames, lengths, K, V = pipe(text, style, dur)
        frames_cap, lengths_cap, _, _ = pipe(text, style, dur, max_frame_len=7)
    arrays = {f"sd/{k}": v for k, v in sd.items()}
    arrays.update(text=f32(text), style=f32(style), durations=f32(dur), frames=f32(frames),
                  lengths=lengths.numpy(), K=f32(K), V=f32(V), frames_cap=f32(frames_cap),
                  lengths_cap=lengths_cap.numpy())
    save("style.npz", **arrays)


def gen_regulator(msca, seed=7):
    """Reference LengthRegulator (style_cross_attention.py:156-198) alone:
    half-integer durations (round half to even), negatives (clamp), an
    all-zero row, max_len None / shorter / longer than the longest row; the
    hidden gradient of sum(expanded * w) through the reference loop."""
    g = torch.Generator().manual_seed(seed)
    reg = msca.LengthRegulator()
    B, Tt, D = 4, 9, 24
    hidden = rnd(g, B, Tt, D)
    dur = torch.randint(0, 6, (B, Tt), generator=g).double()
    dur[0, :4] = torch.tensor([0.5, 1.5, 2.5, 3.5], dtype=torch.float64)
    dur[1, 2], dur[1, 5] = -2.0, 0.49
    dur[2] = 0.0
    dur[3, 0] = 4.6
    arrays = dict(hidden=f32(hidden), durations=f32(dur))
    for tag, ml in (("none", None), ("short", 6), ("long", 40)):
        h = hidden.clone().requires_grad_(True)
        out, lengths = reg(h, dur, max_len=ml)
        w = rnd(g, *out.shape)
        (out * w).sum().backward()
        arrays.update({f"{tag}/out": f32(out.detach()), f"{tag}/lengths": lengths.numpy(), f"{tag}/w": f32(w),
                       f"{tag}/dhidden": f32(h.grad)})
    save("regulator.npz", **arrays)


# ---------------------------------------------------------------------------
# 5. text encoder / duration predictor / text processor through the REFERENCE
#    text_encoder.py (behind the lib.FastSpeech2 shim)
# ---------------------------------------------------------------------------
TEXT = dict(vocab_size=40, d_model=64, n_layers=2, n_head=2, d_k=32, d_v=32, d_inner=128, kernel_size=(9, 1),
            dropout=0.0, max_seq_len=48, padding_idx=0)
DUR = dict(d_model=64, filter_size=128, kernel_size=3, dropout=0.0)
RELU_MARGIN = 2e-5    # every ReLU pre-activation at least this far from 0 (fp32 rounding cannot flip one)


def _pad_batch(g, lengths, V, L):
    ids = torch.randint(1, V, (len(lengths), L), generator=g)
    mask = torch.arange(L)[None] >= torch.tensor(lengths)[:, None]   # True = pad (text_encoder.py:93)
    ids[mask] = 0
    return ids, mask


def _relu_margin(model, run):
    """min |pre-activation| over every ReLU input the reference computes in run()."""
    pres = []
    hooks = []
    for name, mod in model.named_modules():
        if name.endswith("pos_ffn.w_1") or name.endswith("conv1d_1") or name.endswith("conv1d_2"):
            hooks.append(mod.register_forward_hook(lambda m, i, o: pres.append(o.detach().abs().min().item())))
    try:
        run()
    finally:
        for h in hooks:
            h.remove()
    return min(pres)


def gen_text(mte, seed=11):
    arrays = {}
    for attempt in range(50):
        s = seed + 1000 * attempt
        torch.manual_seed(s)
        g = torch.Generator().manual_seed(s + 1)
        enc = mte.TextEncoder(**TEXT).double()
        perturb_norms(enc, g)
        with torch.no_grad():
            for n, p in enc.named_parameters():
                if n.endswith("bias"):
                    p.copy_(0.1 * torch.randn(p.shape, generator=g, dtype=p.dtype))
        sd = {k: f32(v) for k, v in enc.state_dict().items()}
        enc.load_state_dict({k: torch.from_numpy(v).double() for k, v in sd.items()})
        ids_t, mask_t = _pad_batch(g, [37, 20, 29], TEXT["vocab_size"], 37)
        ids_t[0, 5] = 0          # the padding id inside a valid span: zero embedding row, no gradient
        ids_e, mask_e = _pad_batch(g, [60, 45], TEXT["vocab_size"], 60)   # eval branch: L > max_seq_len
        ids_z, mask_z = _pad_batch(g, [52, 0, 17], TEXT["vocab_size"], 52)  # a zero-length row (forward only)
        enc.train()
        m_train = _relu_margin(enc, lambda: enc(ids_t, mask=mask_t))
        enc.eval()
        m_eval = _relu_margin(enc, lambda: enc(ids_e, mask=mask_e))
        if min(m_train, m_eval) > RELU_MARGIN:
            break
    print(f"text encoder seed {s}: relu margins train {m_train:.2e} eval {m_eval:.2e}")
    arrays.update({f"enc/sd/{k}": v for k, v in sd.items()})
    arrays["enc/seed"] = np.array(s)
    for tag, ids, mask, train in (("train", ids_t, mask_t, True), ("eval", ids_e, mask_e, False)):
        enc.train(train)
        enc.zero_grad()
        out = enc(ids, mask=mask)
        w = rnd(g, *out.shape)
        (out * w).sum().backward()
        arrays.update({f"{tag}/ids": ids.numpy(), f"{tag}/mask": mask.numpy(), f"{tag}/out": f32(out),
                       f"{tag}/w": f32(w)})
        for n, p in enc.named_parameters():
            if p.requires_grad:
                arrays[f"{tag}/grad/{n}"] = f32(p.grad)
    enc.eval()
    with torch.no_grad():
        out_z = enc(ids_z, mask=mask_z)
    assert torch.isfinite(out_z).all()
    arrays.update({"empty/ids": ids_z.numpy(), "empty/mask": mask_z.numpy(), "empty/out": f32(out_z)})

    # DurationPredictor (text_encoder.py:131-209): forward + compute_loss, masked and not
    for attempt in range(50):
        s = seed + 7 + 1000 * attempt
        torch.manual_seed(s)
        g = torch.Generator().manual_seed(s + 1)
        dp = mte.DurationPredictor(**DUR).double()
        perturb_norms(dp, g)
        with torch.no_grad():
            for n, p in dp.named_parameters():
                if n.endswith("bias"):
                    p.copy_(0.1 * torch.randn(p.shape, generator=g, dtype=p.dtype))
        sd = {k: f32(v) for k, v in dp.state_dict().items()}
        dp.load_state_dict({k: torch.from_numpy(v).double() for k, v in sd.items()})
        x = rnd(g, 3, 29, DUR["d_model"])
        _, dmask = _pad_batch(g, [29, 11, 23], 10, 29)
        if _relu_margin(dp, lambda: dp(x, mask=dmask)) > RELU_MARGIN:
            break
    dp.train()
    target = torch.randint(1, 9, (3, 29), generator=g).double()
    target[dmask] = 0.0
    target[0, 3] = 0.0           # a zero duration inside a valid span: log(1e-8)
    xr = x.clone().requires_grad_(True)
    pred = dp(xr, mask=dmask)
    # compute_loss builds its target in float32 (duration_target.float(),
    # text_encoder.py:196) as it runs in train.py on fp32 predictions: the loss
    # stage runs on the fp32-rounded prediction and its gradient is carried back
    # through the float64 predictor
    pred32 = pred.detach().float().requires_grad_(True)
    loss = dp.compute_loss(pred32, target, mask=dmask)
    loss.backward()
    pred.backward(pred32.grad.double())
    with torch.no_grad():
        loss_nomask = dp.compute_loss(dp(x, mask=None).float(), target.clamp(min=1.0))
    arrays.update({f"dur/sd/{k}": v for k, v in sd.items()})
    arrays.update({"dur/x": f32(x), "dur/mask": dmask.numpy(), "dur/target": f32(target), "dur/pred": f32(pred),
                   "dur/loss": f32(loss), "dur/loss_nomask": f32(loss_nomask), "dur/dx": f32(xr.grad)})
    for n, p in dp.named_parameters():
        arrays[f"dur/grad/{n}"] = f32(p.grad)
    # the positional table the reference builds (FastSpeech2's, padding row zeroed) and the eval-branch one
    arrays["table/pad"] = f32(mte.TextProcessor(vocab_list=["<PAD>", "a"]).create_positional_encoding(10, 8))
    arrays["table/eval"] = f32(fs2_sinusoid_table(60, TEXT["d_model"]))
    save("text.npz", **arrays)


G2P = {"dict": lambda t: {"ph": t}, "str": lambda t: " ".join(reversed(t.split())), "list": lambda t: t.split()[1:]}


def gen_text_processor(mte):
    """TextProcessor (text_encoder.py:212-428) on the reference's own
    phoneme_vocab.json and two list vocabularies -> text_processor.json
    (inputs and the reference's outputs; ints, strings and bools only)."""
    import json
    vocabs = {"file": None,
              "unk_custom_pad": ["<UNK>", "AA0", "B", "<SIL>", "K"],
              "no_specials": ["x", "y", "z"]}
    texts = ["HH AH0 L OW1 , W ER1 L D .", "", "K AE1 T QQ S AE1 T", "B IY1 | XX YY ZZ", "  AA0   B  ",
             "x y z w", "<PAD> <UNK> <SIL>"]
    cases = []
    for vname, vlist in vocabs.items():
        kw = {"vocab_path": os.path.join(REF, "phoneme_vocab.json")} if vlist is None else {"vocab_list": vlist}
        if vname == "unk_custom_pad":
            kw["padding_token"] = "<SIL>"
        tp = mte.TextProcessor(**kw)
        case = {"vocab": vname, "kwargs": {k: v for k, v in kw.items() if k != "vocab_path"},
                "vocab_size": tp.vocab_size, "padding_id": tp.padding_id, "unk_id": tp.unk_id, "batches": [],
                "process": [], "ids_to_phonemes": []}
        for max_length in (None, 3, 0):
            for pad in (True, False):
                ids, lengths, masks = tp.batch_process(texts, max_length=max_length, pad_to_max=pad)
                case["batches"].append({
                    "max_length": max_length, "pad_to_max": pad, "lengths": lengths,
                    "ids": ids.tolist() if pad else [t.tolist() for t in ids],
                    "masks": None if masks is None else masks.tolist(),
                    "ids_shape": list(ids.shape) if pad else None})
        ids, lengths, masks = tp.batch_process([], pad_to_max=True)
        case["empty_batch"] = {"ids_shape": list(ids.shape), "lengths": lengths, "masks_shape": list(masks.shape)}
        for gname, fn in list(G2P.items()) + [(None, None)]:
            for t in texts[:4]:
                pids, phs = tp.process_text(t, g2p_processor=fn, max_length=5)
                case["process"].append({"text": t, "g2p": gname, "ids": pids, "phonemes": phs})
        case["ids_to_phonemes"] = {"ids": [0, 1, 2, 4, 77, 78, 79, 500, -1],
                                   "phonemes": tp.ids_to_phonemes([0, 1, 2, 4, 77, 78, 79, 500, -1])}
        emb = tp.create_phoneme_embedding(8)
        case["embedding"] = {"num": emb.num_embeddings, "dim": emb.embedding_dim, "padding_idx": emb.padding_idx}
        cases.append(case)
    path = os.path.join(HERE, "text_processor.json")
    with open(path, "w", encoding="utf-8") as f:
        json.dump({"texts": texts, "cases": cases}, f, ensure_ascii=False, indent=0)
    print(f"wrote text_processor.json: {os.path.getsize(path) / 1024:.1f} KiB")


def main():
    torch.set_num_threads(8)
    if sys.argv[1:] == ["text"]:
        mte = import_reference_text_encoder()
        gen_text(mte)
        gen_text_processor(mte)
        return
    mdec, msca = import_reference()
    if sys.argv[1:] == ["regulator"]:
        gen_regulator(msca)
        return
    gen_scan("scan_full.npz", 2, 64, 256)
    gen_scan("scan_plain.npz", 1, 32, 512, use_z=False, use_D=False, use_bias=False, softplus=False, seed=5)
    gen_scan("scan_short.npz", 3, 16, 3, seed=6)
    gen_conv()
    gen_state_update()
    gen_decoder(mdec)
    gen_style(msca)
    gen_regulator(msca)
    mte = import_reference_text_encoder()
    gen_text(mte)
    gen_text_processor(mte)


if __name__ == "__main__":
    main()
