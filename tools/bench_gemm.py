"""Time every C2 GEMM shape (fwd, dgrad, wgrad) with torch.matmul (hipBLASLt), bf16."""
import torch, math
M = 8 * 2048
d, di, r, N, dff, S = 1024, 2048, 64, 16, 2048, 8 * 128
shapes = {  # name: (m, n, k) for C[m,n] = A[m,k] @ B[k,n]
    "in_proj": (M, 2 * di, d), "x_proj": (M, r + 2 * N, di), "dt_proj": (M, di, r), "out_proj": (M, d, di),
    "q_proj": (M, d, d), "kv_proj": (S, 2 * d, d), "o_proj": (M, d, d), "ff1": (M, dff, d), "ff2": (M, d, dff),
}
def t(fn, it=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / it
tot_ms = tot_fl = 0
for name, (m, n, k) in shapes.items():
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(m, n, device="cuda", dtype=torch.bfloat16)
    fl = 2 * m * n * k
    f = t(lambda: x @ w.t()); g = t(lambda: dy @ w); h = t(lambda: dy.t() @ x)
    tot_ms += f + g + h; tot_fl += 3 * fl
    print(f"{name:9s} m={m:6d} n={n:5d} k={k:5d}  fwd {f*1e3:7.1f}us {fl/f/1e9:6.0f}TF  dgrad {g*1e3:7.1f}us {fl/g/1e9:6.0f}TF  wgrad {h*1e3:7.1f}us {fl/h/1e9:6.0f}TF", flush=True)
print(f"per layer: {tot_ms:.3f} ms, {tot_fl/tot_ms/1e9:.0f} TF avg; x12 layers = {12*tot_ms:.2f} ms")
