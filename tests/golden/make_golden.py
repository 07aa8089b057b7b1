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


def main():
    torch.set_num_threads(8)
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


if __name__ == "__main__":
    main()
