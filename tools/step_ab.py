"""In-process A/B of C2 training-step variants (same model, same box):
torch fused Adam + foreach clip vs FusedClipAdam, eager vs hipGraph."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
import mamba_decoder  # noqa: E402
from mtts.optim import FusedClipAdam, clip_into_optimizer  # noqa: E402

c = dict(bench.C2)
torch.manual_seed(0)
model = mamba_decoder.MambaTTSDecoder(c["vocab"], d_model=c["d_model"], n_layers=c["n_layers"], n_heads=c["n_heads"],
                                      d_ff=c["d_ff"], d_style=c["d_style"]).cuda()
model.compute_dtype = torch.bfloat16
params = list(model.parameters())
tokens, text, z, mask = bench.make_batch(c, "cuda", 1234)


def make(kind):
    if kind == "torch":
        opt = torch.optim.Adam(params, lr=1e-4, fused=True)
    else:
        opt = FusedClipAdam(params, lr=1e-4, max_grad_norm=1.0)

    def step():
        logits = model(tokens, text, z, text_mask=mask)
        loss = torch.nn.functional.cross_entropy(logits.float().view(-1, 10), tokens.view(-1), ignore_index=0)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        if kind == "torch":
            clip_into_optimizer(opt, params, 1.0)
        opt.step()
        return loss
    return step, opt


def timeit(run, n=10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        run()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


res = {}
for rnd in range(2):
    for kind in ("torch", "fused"):
        step, opt = make(kind)
        for _ in range(3):
            step()
        res.setdefault(kind + "-eager", []).append(timeit(step))
        if kind == "fused":
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(2):
                    step()
            torch.cuda.current_stream().wait_stream(side)
            opt.zero_grad(set_to_none=True)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            res.setdefault("fused-graph", []).append(timeit(g.replay))
            del g
        del opt
print({k: [round(x, 2) for x in v] for k, v in res.items()})
