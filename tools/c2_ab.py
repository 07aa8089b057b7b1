"""C2 training step time of one package tree, for same-box A/Bs between
processes: AB_ROOT=tools/ab/base python tools/c2_ab.py  vs  python tools/c2_ab.py
(the bench's own step: forward, HIP cross-entropy, backward, fused clip+Adam;
2 warmup steps, then 3 windows of 5 steps, median ms per step)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.abspath(os.path.join(os.environ.get("AB_ROOT", ROOT), "mamba-tts-project_amd"))
sys.path[:0] = [ROOT]
import torch  # noqa: E402
import bench  # noqa: E402   (puts this tree's package on sys.path: the tree under test goes in front)
sys.path.insert(0, PKG)
import mamba_decoder  # noqa: E402
assert mamba_decoder.__file__.startswith(PKG), (mamba_decoder.__file__, PKG)
from mtts.loss import cross_entropy  # noqa: E402
from mtts.optim import FusedClipAdam  # noqa: E402
try:   # the deferred grouped weight gradients (round 5); DEFER=0 turns them off, SIDE=1 the side stream on
    from mtts import wgrad as _wg  # noqa: E402
    defer = lambda: _wg.deferred(os.environ.get("DEFER", "1") == "1")  # noqa: E731
    _wg.SIDE_STREAM = os.environ.get("SIDE", "0") == "1"   # product default: off (wgrad.py)
    if hasattr(_wg, "FUSE_BIAS"):
        _wg.FUSE_BIAS = os.environ.get("FUSE", "1") == "1"
except ImportError:
    import contextlib  # noqa: E402
    defer = contextlib.nullcontext

c = dict(bench.C2)
torch.manual_seed(0)
model = mamba_decoder.MambaTTSDecoder(c["vocab"], d_model=c["d_model"], n_layers=c["n_layers"], n_heads=c["n_heads"],
                                      d_ff=c["d_ff"], d_style=c["d_style"]).cuda()
model.compute_dtype = torch.bfloat16
tokens, text, z, mask = bench.make_batch(c, "cuda", 1234)
opt = FusedClipAdam(list(model.parameters()), lr=1e-4, max_grad_norm=1.0)


def step():
    logits = model(tokens, text, z, text_mask=mask)
    loss = cross_entropy(logits.view(-1, c["vocab"]), tokens.view(-1), ignore_index=0)
    opt.zero_grad(set_to_none=True)
    with defer():
        loss.backward()
    opt.step()


for _ in range(2):
    step()
torch.cuda.synchronize()
ts = []
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        step()
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1) / 5)
ts.sort()
print(f"{'base' if 'AB_ROOT' in os.environ else 'new '}{' defer=' + os.environ['DEFER'] if 'DEFER' in os.environ else ''}{' side=' + os.environ['SIDE'] if 'SIDE' in os.environ else ''} C2 step {ts[1]:.2f} ms (windows {', '.join(f'{t:.2f}' for t in ts)})",
      flush=True)
