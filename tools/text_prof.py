"""Where the text-encoder bench leg's time goes: bench.text_bench's step
(TextEncoder + DurationPredictor fwd+bwd, train.py width, B=8, 128 phonemes)
under torch.profiler after warm-up; GPU kernels grouped by name with count and
time per step, plus wall time per step.   python tools/text_prof.py"""
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402
import text_encoder as te  # noqa: E402

if os.environ.get("HALO") == "0":   # explicit zero-padded conv inputs instead of halo row maps (A/B)
    from mtts import convgemm as CG
    CG._halo_ok = lambda C_, p: False
B, T_text, d_model = 8, 128, 512
dev = "cuda"
torch.manual_seed(0)
enc = te.TextEncoder(79, d_model=d_model).to(dev).train()
dur = te.DurationPredictor(d_model=d_model).to(dev).train()
g = torch.Generator(device=dev).manual_seed(9)
ids = torch.randint(1, 79, (B, T_text), device=dev, generator=g)
lens = torch.randint(T_text // 2, T_text + 1, (B,), device=dev, generator=g)
mask = torch.arange(T_text, device=dev)[None] >= lens[:, None]
ids = ids.masked_fill(mask, 0)
target = torch.randint(1, 10, (B, T_text), device=dev, generator=g).float()


params = list(enc.parameters()) + list(dur.parameters())


def step():   # as bench.text_bench: gradients set to None first (zero_grad(set_to_none=True))
    for p in params:
        p.grad = None
    h = enc(ids, mask=mask)
    loss = dur.compute_loss(dur(h, mask=mask), target, mask=mask) + h.square().mean()
    loss.backward()


for _ in range(5):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    step()
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / 20 * 1e3
with profile(activities=[ProfilerActivity.CUDA, ProfilerActivity.CPU]) as prof:
    for _ in range(5):
        step()
    torch.cuda.synchronize()
agg = defaultdict(lambda: [0, 0.0])
for ev in prof.events():
    if ev.device_type == torch.autograd.DeviceType.CUDA and ev.device_time > 0:
        a = agg[ev.name[:90]]
        a[0] += 1
        a[1] += ev.device_time
tot = sum(v[1] for v in agg.values()) / 5
print(f"wall {wall:.3f} ms/step, GPU kernel time {tot / 1e3:.3f} ms/step, "
      f"{sum(v[0] for v in agg.values()) / 5:.0f} kernels/step")
for name, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{us / 5:9.1f} us {n / 5:5.0f}x  {name}")
ops = defaultdict(int)
for ev in prof.events():
    if ev.device_type == torch.autograd.DeviceType.CPU and ev.name.startswith("aten::") and \
            ev.name in ("aten::add", "aten::add_", "aten::copy_", "aten::fill_", "aten::zero_", "aten::where",
                        "aten::masked_fill", "aten::cat", "aten::constant_pad_nd", "aten::mul", "aten::clone"):
        ops[ev.name] += 1
print("aten ops per step:", ", ".join(f"{k} {v / 5:.0f}" for k, v in sorted(ops.items(), key=lambda kv: -kv[1])))
if os.environ.get("STACKS"):   # where the copies / clones / fills come from
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof2:
        step()
        torch.cuda.synchronize()
    for row in prof2.key_averages(group_by_stack_n=6, group_by_input_shape=True):
        if row.key in ("aten::copy_", "aten::clone", "aten::fill_", "aten::add_", "aten::add", "aten::mul"):
            st = [f for f in row.stack if "site-packages" not in f and "dist-packages" not in f][:3]
            print(f"{row.key:12s} x{row.count:3d} {str(row.input_shapes)[:70]:70s} {' <- '.join(st)}")
