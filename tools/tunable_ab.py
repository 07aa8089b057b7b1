"""C2 training step with PyTorch TunableOp (hipBLASLt / rocBLAS solution
search for the GEMMs left on the vendor library) vs the default heuristic
choice: tunes once (results file), then interleaves timed rounds.
python tools/tunable_ab.py OUT.csv"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd")]
import torch  # noqa: E402
import torch.cuda.tunable as TO  # noqa: E402
import bench  # noqa: E402
import mamba_decoder  # noqa: E402
from mtts.optim import FusedClipAdam  # noqa: E402

out = sys.argv[1]
c = dict(bench.C2)
torch.manual_seed(0)
model = mamba_decoder.MambaTTSDecoder(c["vocab"], d_model=c["d_model"], n_layers=c["n_layers"], n_heads=c["n_heads"],
                                      d_ff=c["d_ff"], d_style=c["d_style"]).cuda()
model.compute_dtype = torch.bfloat16
params = list(model.parameters())
tokens, text, z, mask = bench.make_batch(c, "cuda", 1234)
opt = FusedClipAdam(params, lr=1e-4, max_grad_norm=1.0)


def step():
    logits = model(tokens, text, z, text_mask=mask)
    loss = torch.nn.functional.cross_entropy(logits.float().view(-1, 10), tokens.view(-1), ignore_index=0)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()
    return loss


def timeit(n=10):
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


base = timeit()
print("default", round(base, 2), flush=True)
TO.enable(True)
TO.tuning_enable(True)
TO.set_filename(out)
TO.set_max_tuning_duration(int(os.environ.get("TUNE_MS", "30")))
TO.set_max_tuning_iterations(int(os.environ.get("TUNE_IT", "100")))
t0 = time.perf_counter()
step()
torch.cuda.synchronize()
print("tuning pass", round(time.perf_counter() - t0, 1), "s", flush=True)
pass
TO.tuning_enable(False)
res = {"default": [], "tuned": []}
for _ in range(3):
    for kind in res:
        TO.enable(kind == "tuned")
        res[kind].append(timeit())
print({k: [round(x, 2) for x in v] for k, v in res.items()}, flush=True)
