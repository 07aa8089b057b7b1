"""Which loss term carries the text-encoder gradient error of the train.py-width
C5 test: te gradients of loss_dur alone and loss_codec alone vs the float64
oracle, the hand-written convolutions vs a torch (F.conv1d / F.linear)
restatement of the same modules.   python tools/dbg/c5w_te_dbg.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
import train_harness as th  # noqa: E402
import text_encoder as te  # noqa: E402
from oracle import mamba_ref as R  # noqa: E402
from test_gpu_c5 import _perturb, _params64  # noqa: E402

DEV = "cuda"


def torch_conv(x, weight, bias, padding, relu=False):
    y = F.conv1d(x.transpose(1, 2), weight, bias, padding=padding).transpose(1, 2)
    return (torch.relu(y) if relu else y).contiguous()


DOUTS = {"all": [], "mha": []}
RET = []
LAST = {}


def ffn_torch(self, x):
    h = torch_conv(x, self.w_1.weight, self.w_1.bias, self.w_1.padding[0], relu=True)
    c = torch_conv(h, self.w_2.weight, self.w_2.bias, self.w_2.padding[0])
    c.register_hook(lambda g: DOUTS["all"].append(g.detach().clone()))
    out = self.dropout(c)
    return te._ln(self.layer_norm, out, res=x)


def mha_sep(self, q, k, v, mask=None):
    residual = q
    qh = F.linear(q, self.w_qs.weight, self.w_qs.bias)
    kh = F.linear(k, self.w_ks.weight, self.w_ks.bias)
    vh = F.linear(v, self.w_vs.weight, self.w_vs.bias)
    from mtts import attn_kernels
    o = attn_kernels.attention(qh, kh, vh, self.n_head, key_padding_mask=mask)
    o = self.dropout(F.linear(o, self.fc.weight, self.fc.bias))
    return te._ln(self.layer_norm, o, res=residual), None


def run(which, use_torch):
    torch.manual_seed(0)
    models = th.build_models(DEV, dec_layers=2, compute_dtype=torch.bfloat16, dropout=0.0)
    _perturb(models, 4)
    step = th.TrainStep(models, lr=1e-3)
    batch = th.synthetic_batch(1, DEV, T_text=64, T_codec=256, T_ref=128, seed=5)
    p_te, p_dur, p_dec = (_params64(m) for m in (models.text_encoder, models.dur_predictor, models.decoder))
    saved = (te.conv1d_same, te.linear, te.PositionwiseFeedForward.forward, te.MultiHeadAttention.forward)
    if use_torch:
        te.conv1d_same = torch_conv
        te.linear = F.linear
    if use_torch in ("ffn", "all"):
        te.PositionwiseFeedForward.forward = ffn_torch
    if use_torch in ("mha", "all"):
        te.MultiHeadAttention.forward = mha_sep
    try:
        total, lc, ld, ls, logits = step.losses(batch)
        for p in step.params:
            p.grad = None
        {"dur": ld, "codec": lc}[which].backward()
    finally:
        te.conv1d_same, te.linear, te.PositionwiseFeedForward.forward, te.MultiHeadAttention.forward = saved
    cb = {k: v.cpu() for k, v in batch.items()}
    cb["style_emb"] = cb["style_emb"].double()
    rt, rc, rd, rlogits, _, _ = R.train_step_losses_ref(p_te, p_dur, p_dec, cb, dict(n_layers=4, n_head=2, d_k=64),
                                                       dict(n_layers=2, n_heads=8))
    {"dur": rd, "codec": rc}[which].backward()
    out = {}
    for k, v in models.text_encoder.named_parameters():
        rg = p_te[k].grad
        if v.grad is None or rg is None or rg.abs().max() < 1e-12:
            continue
        out[k] = ((v.grad.double().cpu() - rg).abs().max() / rg.abs().max()).item()
    return out


def grads(use_torch):
    torch.manual_seed(0)
    models = th.build_models(DEV, dec_layers=2, compute_dtype=torch.bfloat16, dropout=0.0)
    _perturb(models, 4)
    step = th.TrainStep(models, lr=1e-3)
    batch = th.synthetic_batch(1, DEV, T_text=64, T_codec=256, T_ref=128, seed=5)
    saved = (te.conv1d_same, te.linear, te.PositionwiseFeedForward.forward, te.MultiHeadAttention.forward)
    te.conv1d_same, te.linear = torch_conv, F.linear
    te.PositionwiseFeedForward.forward = ffn_torch
    if use_torch == "all":
        te.MultiHeadAttention.forward = mha_sep
    hooks = {}
    try:
        enc = models.text_encoder
        for i, layer in enumerate(enc.layer_stack):
            layer.register_full_backward_hook(lambda m, gi, go, i=i: hooks.__setitem__(i, go[0].detach().clone()))
            layer.pos_ffn.register_forward_hook(lambda m, inp, out, i=i: hooks.__setitem__(f"ffn_in{i}", inp[0].detach().clone()))
            def bh(m, gi, go, i=i):
                hooks[f"ffn_gout{i}"] = go[0].detach().clone()
                hooks[f"ffn_gin{i}"] = gi[0].detach().clone()
            layer.pos_ffn.register_full_backward_hook(bh)
        total, lc, ld, ls, logits = step.losses(batch)
        for p in step.params:
            p.grad = None
        ld.backward()
    finally:
        te.conv1d_same, te.linear, te.PositionwiseFeedForward.forward, te.MultiHeadAttention.forward = saved
    return {k: v.grad.clone() for k, v in models.text_encoder.named_parameters() if v.grad is not None}, hooks


def poison():
    ts = [torch.full((1 << 22,), float("nan"), device=DEV) for _ in range(64)]
    ts += [torch.full((1 << 16,), 1e30, device=DEV) for _ in range(256)]
    del ts


def ref_errs(use_torch, poisoned):
    if poisoned:
        poison()
    e = run("dur", use_torch)
    worst = sorted(e.items(), key=lambda kv: -kv[1])[:3]
    print(f"poison={poisoned} torch={use_torch!s:5s} max err {max(e.values()):.2e}: "
          + ", ".join(f"{k} {v:.1e}" for k, v in worst), flush=True)


def grads2(use_torch):
    torch.manual_seed(0)
    models = th.build_models(DEV, dec_layers=2, compute_dtype=torch.bfloat16, dropout=0.0)
    _perturb(models, 4)
    step = th.TrainStep(models, lr=1e-3)
    batch = th.synthetic_batch(1, DEV, T_text=64, T_codec=256, T_ref=128, seed=5)
    saved = (te.conv1d_same, te.linear, te.PositionwiseFeedForward.forward, te.MultiHeadAttention.forward)
    te.conv1d_same, te.linear = torch_conv, F.linear
    if use_torch in ("ffn", "all"):
        te.PositionwiseFeedForward.forward = ffn_torch
    if use_torch in ("mha", "all"):
        te.MultiHeadAttention.forward = mha_sep
    acts = {}
    try:
        for i, layer in enumerate(models.text_encoder.layer_stack):
            layer.slf_attn.register_forward_hook(lambda m, inp, out, i=i: acts.__setitem__(f"mha{i}", out[0].detach().clone()))
            layer.pos_ffn.register_forward_hook(lambda m, inp, out, i=i: acts.__setitem__(f"ffn{i}", out.detach().clone()))
        total, lc, ld, ls, logits = step.losses(batch)
        for p in step.params:
            p.grad = None
        ld.backward()
    finally:
        te.conv1d_same, te.linear, te.PositionwiseFeedForward.forward, te.MultiHeadAttention.forward = saved
    LAST["m"] = models
    return {k: v.grad.clone() for k, v in models.text_encoder.named_parameters() if v.grad is not None}, acts


from mtts import convgemm as CGm  # noqa: E402
_orig_ffn_bwd = CGm.ConvFFNFn.backward


def _ffn_bwd_check(ctx, dout):
    res = _orig_ffn_bwd(ctx, dout)
    DOUTS["mha"].append(dout.detach().clone())
    RET.append((res[1].data_ptr(), res[1].detach().clone(), res[1].shape, res[1].stride()))
    xp, w1, hp, w2 = ctx.saved_tensors
    B, T, O = dout.shape
    H = w2.shape[1]
    x = xp[:, 4:4 + T]
    d = dout.double()
    dh = (d @ w2.view(O, H).double()) * (hp > 0)
    dw2 = torch.einsum("bto,bth->oh", d, hp.double())
    dw1 = torch.nn.grad.conv1d_weight(x.transpose(1, 2).double(), w1.shape, dh.transpose(1, 2), padding=4)
    dx = torch.nn.grad.conv1d_input(x.transpose(1, 2).shape, w1.double(), dh.transpose(1, 2), padding=4).transpose(1, 2)
    msg = []
    for n, got, ref in zip(("dx", "dw1", "db1", "dw2", "db2"), res, (dx, dw1, dh.sum((0, 1)), dw2.unsqueeze(-1), d.sum((0, 1)))):
        msg.append(f"{n} {((got.double() - ref).abs().max() / ref.abs().max()).item():.1e}")
    print(f"ConvFFN bwd check T{T}: " + ", ".join(msg) + f"; dout max {dout.abs().max().item():.2e} "
          f"contig {dout.is_contiguous()} stride {tuple(dout.stride())} ptr%16 {dout.data_ptr() % 16}", flush=True)
    return res


def _ffn_bwd_torch(ctx, dout):
    res = _orig_ffn_bwd(ctx, dout)
    xp, w1, hp, w2 = ctx.saved_tensors
    T = dout.shape[1]
    with torch.enable_grad():
        x = xp[:, 4:4 + T].detach().clone().requires_grad_(True)
        w1r = w1.detach().clone().requires_grad_(True)
        pre = F.conv1d(x.transpose(1, 2), w1r, None, padding=4).transpose(1, 2)
        b1 = (hp - torch.relu(pre)).detach()     # hp = relu(pre + b1): recover b1 where active
        h = torch.relu(pre + LASTB1[-1])
        y = F.conv1d(h.transpose(1, 2), w2.detach(), None).transpose(1, 2)
        gx, gw1 = torch.autograd.grad(y, (x, w1r), dout)
    near0 = ((pre + LASTB1[-1]).abs() < 1e-4).float().mean().item()
    hdiff = (h - hp).abs().max().item()
    print(f"torch-autograd check: dx {((res[0] - gx).abs().max() / gx.abs().max()).item():.1e} "
          f"dw1 {((res[1] - gw1).abs().max() / gw1.abs().max()).item():.1e}; |pre|<1e-4 frac {near0:.2e}; "
          f"h vs torch h {hdiff:.1e}", flush=True)
    LASTB1.pop()
    return res


LASTB1 = []
_orig_ffn_fwd0 = CGm.ConvFFNFn.forward


def _ffn_fwd_b1(ctx, x, w1, b1, w2, b2):
    LASTB1.append(b1.detach().clone())
    return _orig_ffn_fwd0(ctx, x, w1, b1, w2, b2)


CGm.ConvFFNFn.forward = staticmethod(_ffn_fwd_b1)
CGm.ConvFFNFn.backward = staticmethod(_ffn_bwd_torch)
grads2("mha")
CGm.ConvFFNFn.forward = staticmethod(_orig_ffn_fwd0)
CGm.ConvFFNFn.backward = staticmethod(_orig_ffn_bwd)
