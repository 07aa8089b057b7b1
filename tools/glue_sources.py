"""Which ops launch the small kernels (fills, copies, casts, column sums,
split-K reduces, ...) of the C2 training step: torch.profiler over one step
after warm-up; every GPU kernel is attributed to its chain of CPU ops (the
autograd Function / module op that issued it and the aten op under it), and
the kernels are grouped by (issuing chain, kernel family) with launch count
and GPU time per step.   python tools/glue_sources.py [--all]"""
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
from mtts import loss as mloss  # noqa: E402
from mtts import wgrad  # noqa: E402

c = dict(bench.C2)
torch.manual_seed(0)
model = mamba_decoder.MambaTTSDecoder(c["vocab"], d_model=c["d_model"], n_layers=c["n_layers"], n_heads=c["n_heads"],
                                      d_ff=c["d_ff"], d_style=c["d_style"]).cuda()
model.compute_dtype = torch.bfloat16
tokens, text, z, mask = bench.make_batch(c, "cuda", 1234)
opt = FusedClipAdam(list(model.parameters()), lr=1e-4, max_grad_norm=1.0)


def step():
    logits = model(tokens, text, z, text_mask=mask)
    loss = mloss.cross_entropy(logits.view(-1, logits.shape[-1]), tokens.view(-1), ignore_index=0)
    opt.zero_grad(set_to_none=True)
    with wgrad.deferred():
        loss.backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    step()
    torch.cuda.synchronize()

BIG = ("gemm_pp_kernel", "gemm_kernel", "scan_", "attn_", "ln_fwd", "ln_bwd", "conv_", "adam_kernel", "Cijk",
       "skinny", "small_k", "sumsq", "cast_multi", "embed", "ce_")
show_all = "--all" in sys.argv


def family(name):
    for f in ("FillFunctor", "copy_kernel", "copyBuffer", "CatArray", "colsum_rows", "colsum_multi", "colsum",
              "split_reduce", "reduce_kernel", "elementwise", "index"):
        if f in name:
            return f
    return name[:60]


groups = defaultdict(lambda: [0, 0.0])
for ev in prof.events():
    if ev.device_type != torch.autograd.DeviceType.CPU:
        continue
    for k in getattr(ev, "kernels", []) or []:
        if not show_all and any(b in k.name for b in BIG):
            continue
        chain = []
        p = ev
        while p is not None and len(chain) < 4:
            chain.append(p.name)
            p = p.cpu_parent
        # the outermost interesting frame: an autograd Function / module op
        fn = next((n for n in reversed(chain) if "Backward" in n or n.startswith("mtts") or "Fn" in n), chain[-1])
        key = (fn, chain[0], family(k.name))
        groups[key][0] += 1
        groups[key][1] += k.duration if hasattr(k, "duration") else 0.0

tot = sum(v[1] for v in groups.values())
print(f"{'us/step':>9} {'n':>4}  {'issuing op':34s} {'aten op':26s} kernel family   (total {tot:.0f} us)")
for (fn, op, fam), (n, us) in sorted(groups.items(), key=lambda kv: -kv[1][1])[:60]:
    print(f"{us:9.1f} {n:4d}  {fn[:34]:34s} {op[:26]:26s} {fam}")
