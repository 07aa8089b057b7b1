"""Component-level GPU-vs-oracle diagnostics (prints max errors)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch
from oracle import mamba_ref as R
from mtts import ops
from mtts.mamba import Mamba
from mtts.attention import CrossAttention

torch.manual_seed(0)
dev = "cuda"
def err(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return (a - b).abs().max().item(), b.abs().max().item()

# LN
x = torch.randn(6, 64, device=dev); w = torch.randn(64, device=dev); b = torch.randn(64, device=dev)
y, _ = ops.layer_norm(x, w, b)
print("LN", err(y, R.layer_norm_ref(x.double().cpu(), w.double().cpu(), b.double().cpu())))
# Mamba
m = Mamba(64).to(dev)
p = {"m." + k: v.detach().double().cpu() for k, v in m.state_dict().items()}
xin = torch.randn(2, 40, 64, device=dev)
out, (cs, ss) = m(xin)
ro, (rcs, rss) = R.mamba_forward_ref(p, "m.", xin.double().cpu())
print("mamba out", err(out, ro), "conv_state", err(cs, rcs), "ssm", err(ss, rss))
# conv only on strided view
xz = torch.randn(2, 40, 256, device=dev)
u, _ = ops.conv_fwd(xz[..., :128], m.conv1d.weight, m.conv1d.bias, True)
ru, _ = R.causal_conv1d_ref(xz[..., :128].transpose(1, 2).double().cpu(), m.conv1d.weight.reshape(128, 4).double().cpu(), m.conv1d.bias.double().cpu(), "silu")
print("conv strided", err(u.transpose(1, 2), ru))
# attention
ca = CrossAttention(64, 4).to(dev)
with torch.no_grad():
    ca.in_proj_bias.normal_(); ca.out_proj.bias.normal_()
q = torch.randn(2, 40, 64, device=dev); kv = torch.randn(2, 12, 64, device=dev)
kpm = torch.zeros(2, 12, dtype=torch.bool, device=dev); kpm[0, 7:] = True
o, _ = ca(q, kv, kv, key_padding_mask=kpm)
ro = R.mha_ref(q.double().cpu(), kv.double().cpu(), ca.in_proj_weight.double().cpu(), ca.in_proj_bias.double().cpu(), ca.out_proj.weight.double().cpu(), ca.out_proj.bias.double().cpu(), 4, kpm.cpu())
print("attn", err(o, ro))
# scan with z strided view
B, L, D = 2, 40, 128
u = torch.randn(B, L, D, device=dev); dl = torch.randn(B, L, D, device=dev)
zz = torch.randn(B, L, 2 * D, device=dev)[..., D:]
A = -torch.rand(D, 16, device=dev) - 0.5
xd = torch.randn(B, L, 36, device=dev)
Bm, Cm = xd[..., 4:20], xd[..., 20:]
Dp = torch.randn(D, device=dev); bias = torch.randn(D, device=dev) * 0.1
for P in ("1", "2", "4"):
    os.environ["MTTS_SCAN_P"] = P
    o, l, _ = ops.scan_fwd(u, dl, A, Bm, Cm, Dp, zz, bias, True, want_last=True)
    ro, rl = R.selective_scan_ref(u.transpose(1,2).double().cpu(), dl.transpose(1,2).double().cpu(), A.double().cpu(), Bm.transpose(1,2).double().cpu(), Cm.transpose(1,2).double().cpu(), Dp.double().cpu(), zz.transpose(1,2).double().cpu(), bias.double().cpu(), True, return_last_state=True)
    print("scan P", P, err(o.transpose(1, 2), ro), err(l, rl))
