"""Time every C2 GEMM shape (fwd, dgrad, wgrad) through torch (hipBLASLt), bf16,
with the operand layouts the decoder could choose.

  fwd    y = x @ W^T      : W (n, k) row-major ("nt") or W^T stored (k, n) ("nn")
  dgrad  dx = dy @ W      : W (n, k) ("nn") or W^T stored ("nt")
  wgrad  dW = dy^T @ x    : fp32 out; direct, split-K s (bmm + sum), or
                            into a (k, n) result ("tn" swapped operands)
"""
import torch

M = 8 * 2048
d, di, r, N, dff, S = 1024, 2048, 64, 16, 2048, 8 * 128
shapes = {  # name: (m, n, k) for C[m,n] = A[m,k] @ B[k,n]
    "in_proj": (M, 2 * di, d), "x_proj": (M, r + 2 * N, di), "dt_proj": (M, di, r), "out_proj": (M, d, di),
    "q_proj": (M, d, d), "kv_proj": (S, 2 * d, d), "o_proj": (M, d, d), "ff1": (M, dff, d), "ff2": (M, d, dff),
}
count = {"in_proj": 1, "x_proj": 1, "dt_proj": 1, "out_proj": 1, "q_proj": 1, "kv_proj": 1, "o_proj": 1,
         "ff1": 1, "ff2": 1}


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it


def split(dy, x, s):
    m = dy.shape[0] // s
    part = torch.bmm(dy.reshape(s, m, -1).transpose(1, 2), x.reshape(s, m, -1), out_dtype=torch.float32)
    return part.sum(0)


best_total = cur_total = 0.0
for name, (m, n, k) in shapes.items():
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    wt = w.t().contiguous()
    dy = torch.randn(m, n, device="cuda", dtype=torch.bfloat16)
    fl = 2 * m * n * k
    res = {
        "fwd_nt": t(lambda: x @ w.t()), "fwd_nn": t(lambda: x @ wt),
        "dgrad_nn": t(lambda: dy @ w), "dgrad_nt": t(lambda: dy @ wt.t()),
        "wg_direct": t(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)),
        "wg_swapped": t(lambda: torch.mm(x.t(), dy, out_dtype=torch.float32)),
        "wg_bf16": t(lambda: dy.t() @ x),
    }
    for s in (2, 4, 8):
        if m % s == 0 and m >= 2048:
            res[f"wg_split{s}"] = t(lambda: split(dy, x, s))
    line = " ".join(f"{kk}={fl / v / 1e9:5.0f}" for kk, v in res.items())
    print(f"{name:9s} m={m:6d} n={n:5d} k={k:5d} TF/s: {line}", flush=True)
    cur = res["fwd_nt"] + res["dgrad_nn"] + res.get("wg_split4", res["wg_direct"])
    best = min(res["fwd_nt"], res["fwd_nn"]) + min(res["dgrad_nn"], res["dgrad_nt"]) + \
        min(v for kk, v in res.items() if kk.startswith("wg_") and kk != "wg_bf16")
    cur_total += cur
    best_total += best
print(f"per layer: current {cur_total:.3f} ms, best-of {best_total:.3f} ms; x12 = {12 * cur_total:.2f} / "
      f"{12 * best_total:.2f} ms")
