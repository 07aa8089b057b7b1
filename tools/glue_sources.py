"""Which Python call sites launch the torch glue kernels (fill / copy / cat /
elementwise) of the C2 training step: torch.profiler (with stacks) over one
step after warm-up; GPU time and launch count grouped by kernel family and by
the innermost frame in mtts/ or mamba_decoder.py of the launching op.
python tools/glue_sources.py"""
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402
import bench  # noqa: E402
import mamba_decoder  # noqa: E402
from mtts.optim import FusedClipAdam  # noqa: E402

c = dict(bench.C2)
torch.manual_seed(0)
model = mamba_decoder.MambaTTSDecoder(c["vocab"], d_model=c["d_model"], n_layers=c["n_layers"], n_heads=c["n_heads"],
                                      d_ff=c["d_ff"], d_style=c["d_style"]).cuda()
model.compute_dtype = torch.bfloat16
tokens, text, z, mask = bench.make_batch(c, "cuda", 1234)
opt = FusedClipAdam(list(model.parameters()), lr=1e-4, max_grad_norm=1.0)


def step():
    logits = model(tokens, text, z, text_mask=mask)
    loss = torch.nn.functional.cross_entropy(logits.float().view(-1, 10), tokens.view(-1), ignore_index=0)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    step()
    torch.cuda.synchronize()

GLUE = ("Fill", "copy", "Cat", "elementwise", "reduce_kernel", "index", "fill")
by_site = defaultdict(lambda: [0, 0.0])
for ev in prof.events():
    if ev.device_type != torch.autograd.DeviceType.CPU:
        continue
    kern = [k for k in ev.kernels] if hasattr(ev, "kernels") else []
    if not kern:
        continue
    site = "?"
    for fr in ev.stack or []:
        if "mtts/" in fr or "mamba_decoder.py" in fr or "bench.py" in fr:
            site = fr.split("/")[-1]
            break
    for k in kern:
        if any(g in k.name for g in GLUE):
            key = (ev.name, site)
            by_site[key][0] += 1
            by_site[key][1] += k.duration / 1e3 if hasattr(k, "duration") else 0.0
rows = sorted(by_site.items(), key=lambda kv: -kv[1][1])
for (op, site), (n, us) in rows[:40]:
    print(f"{us:9.1f} us {n:4d}  {op:40s} {site}")
