"""Benchmark: MambaTTSDecoder teacher-forced training step on MI355X.

python bench.py --gpus N --steps K --warmup W
  N > 1: one rank per GPU over RCCL.  Under torch.distributed.run (WORLD_SIZE
  set) the ranks run directly; a plain `python bench.py --gpus N` starts
  `python -m torch.distributed.run --nproc-per-node N ... bench.py` as a
  child process before touching the GPU and relays its exit code (rank 0
  prints the JSON line).

Headline (BASELINE.json metric, configs[1] = C2): audio tokens/s of one
fwd+bwd+clip+Adam step of the 12-layer d_model=1024 decoder at B=8 per GPU,
T_audio=2048, T_text=128 (10 % padded), bf16 compute, random-init weights,
synthetic tokens.  Batch-DP across ranks (weak scaling) with an RCCL
all-reduce of the gradients.

`value` is the whole job's throughput (all ranks' tokens / max-over-ranks
time, weak scaling: B=8 per GPU); `value_per_gpu` = value / N.

Every N: `scan_scaling` -- the north-star selective_scan forward (B=32,
L=8192, d_inner=2048, fp32 I/O) as a second scaling leg, no collective on the
data path: "weak" (every rank scans its own B=32 batch) and "strong" (the
B=32 batch sharded 32/N rows per rank); bytes of all ranks / max-over-ranks
time.

Also reported on rank 0 at N = 1 (same JSON line):
  roofline      selective_scan fwd at the north-star shape (B=32, L=8192,
                d_inner=2048, N=16) with fp32 I/O -- the reference's own
                precision (train.py runs mamba-ssm in fp32) -- HIP-event
                timed on the launch stream, HBM-bound
  roofline_bf16 the same with bf16 I/O (VALU-bound: DESIGN.md section 3)
  step_mfma     the step's algorithmic FLOPs / step time vs dense bf16 peak
  decode        decode_step p50/p90 latency (C4, B=32, 12L)
  c5_step       BASELINE configs[4]: the whole train.py step (text encoder,
                duration loss, style pipeline, voice-prompt reference, 8L
                d_model=512 decoder at T_audio = 5x1024, 3-term loss, clip +
                Adam) on synthetic batches, B=8 per rank, every N
  text_encoder  TextEncoder + DurationPredictor fwd+bwd
  style         style pipeline: HIP length regulator
                roofline, StyleConditioningPipeline eval / train times
  cpu_baseline  the pure-PyTorch oracle (oracle/mamba_ref.py) fwd+bwd of the
                same 12L model on a bounded sample, host cores
  cpu_baseline_scan  the oracle's selective_scan_ref on a bounded slice of
                the north-star scan (one batch row: B=1, L=8192), host cores
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "mamba-tts-project_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK = 8.0e12      # B/s, MI355X spec (MI355X_MICROARCH.md)
BF16_PEAK = 2.5e15     # dense bf16 MFMA FLOP/s (spec)

C2 = dict(n_layers=12, d_model=1024, n_heads=8, d_ff=2048, d_style=256, vocab=10, B=8, T=2048, T_text=128)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def flops_per_step(c):
    d, di, r, N, dff = c["d_model"], 2 * c["d_model"], math.ceil(c["d_model"] / 16), 16, c["d_ff"]
    M = c["B"] * c["T"]
    fwd = 2 * M * (d * 2 * di + di * (r + 2 * N) + r * di + di * d + 2 * d * d + 2 * d * dff)
    fwd += 2 * (c["B"] * c["T_text"]) * d * 2 * d + 4 * c["B"] * c["T"] * c["T_text"] * d
    return 3 * fwd * c["n_layers"]


def make_batch(c, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    B, T, Tt = c["B"], c["T"], c["T_text"]
    tokens = torch.randint(0, c["vocab"], (B, T), device=dev, generator=g)
    text = torch.randn(B, Tt, c["d_model"], device=dev, generator=g)
    z = torch.randn(B, c["d_style"], device=dev, generator=g)
    mask = torch.ones(B, Tt, dtype=torch.bool, device=dev)
    mask[:, int(Tt * 0.9):] = False   # decoder semantics: True = attend (kpm = ~mask)
    return tokens, text, z, mask


def train_bench(args, rank, world, dev):
    import mamba_decoder
    from mtts.optim import FusedClipAdam
    from mtts.loss import cross_entropy
    from mtts import wgrad
    c = dict(C2)
    torch.manual_seed(0)
    model = mamba_decoder.MambaTTSDecoder(c["vocab"], d_model=c["d_model"], n_layers=c["n_layers"],
                                          n_heads=c["n_heads"], d_ff=c["d_ff"], d_style=c["d_style"]).to(dev)
    model.compute_dtype = torch.bfloat16
    params = list(model.parameters())
    dp = None
    if world > 1:
        from mtts.dp import GradAllReduce
        dp = GradAllReduce(params, bucket_mb=128)   # bucketed RCCL all-reduce overlapped with backward
    # torch.optim.Adam(lr=1e-4) + clip_grad_norm_(params, 1.0) (train.py:152-158, 232-235), fused (mtts_clip_adam)
    opt = FusedClipAdam(params, lr=1e-4, max_grad_norm=1.0)
    tokens, text, z, mask = make_batch(c, dev, seed=1234 + rank)

    def step():
        logits = model(tokens, text, z, text_mask=mask)
        loss = cross_entropy(logits.view(-1, c["vocab"]), tokens.view(-1), ignore_index=0)   # csrc/loss.hip
        if dp is not None:
            dp.zero_grad()         # grads are views into the flat all-reduce buffer
        else:
            opt.zero_grad(set_to_none=True)
        with wgrad.deferred():     # projection weight gradients grouped per layer (mtts/wgrad.py)
            loss.backward()
        if dp is not None:
            dp.finish()
        opt.step()
        return loss

    first_loss = None
    run = step
    if args.graph:
        # the whole step (forward, backward, fused clip+Adam) captured once in
        # a hipGraph and replayed: every kernel of the step, no host launch
        # work (the optimizer's step count lives on the device).  Warm-up
        # steps run eagerly on a side stream, as torch's capture recipe asks.
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(args.warmup, 1)):
                l0 = step()
                first_loss = float(l0.item()) if first_loss is None else first_loss
            del l0
        torch.cuda.current_stream().wait_stream(side)
        opt.zero_grad(set_to_none=True)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static_loss = step()

        def run():
            graph.replay()
            return static_loss
    else:
        for _ in range(args.warmup):
            l0 = step()
            first_loss = float(l0.item()) if first_loss is None else first_loss
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    assert torch.isfinite(loss).item(), "non-finite loss"
    dpinfo = None
    if dp is not None:
        dpinfo = dp_breakdown(lambda: cross_entropy(model(tokens, text, z, text_mask=mask).view(-1, c["vocab"]),
                                                    tokens.view(-1), ignore_index=0), dp, dev)
        log(f"[bench] data parallel: {dpinfo}")
    ms = dt / args.steps * 1e3
    tokens_per_s = world * c["B"] * c["T"] * args.steps / dt
    ups = sum(p["uploads"] for p in opt._plans.values())
    log(f"[bench] optimizer descriptor uploads over {args.warmup + args.steps} steps: {ups}")
    del model, opt
    return c, ms, tokens_per_s, (first_loss, float(loss.item())), dpinfo


def scan_roofline(dtype, B=32, L=8192, D=2048, iters=20, rounds=5, barrier=False):
    """selective_scan fwd at the north-star shape; returns (ms, bytes, GB/s):
    the median over `rounds` of the per-launch HIP-event time of `iters`
    back-to-back launches on the launch stream (torch's current stream, which
    ops.scan_fwd launches on).  barrier: bracket each round by a process-group
    barrier (scaling leg)."""
    from mtts import ops
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    N = 16
    u = torch.randn(B, L, D, device=dev, generator=g).to(dtype)
    z = torch.randn(B, L, D, device=dev, generator=g).to(dtype)
    delta = (torch.randn(B, L, D, device=dev, generator=g) * 0.1).to(dtype)
    Bm = torch.randn(B, L, N, device=dev, generator=g).to(dtype)
    Cm = torch.randn(B, L, N, device=dev, generator=g).to(dtype)
    A = -torch.arange(1, N + 1, device=dev, dtype=torch.float32).repeat(D, 1)
    Dp = torch.ones(D, device=dev)
    dt0 = torch.exp(torch.rand(D, device=dev, generator=g) * (math.log(0.1) - math.log(1e-3)) + math.log(1e-3))
    bias = dt0 + torch.log(-torch.expm1(-dt0))
    out = torch.empty_like(u)
    run = lambda: ops.scan_fwd(u, delta, A, Bm, Cm, Dp, z, bias, True, out=out)  # noqa: E731
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    # median over 5 timed rounds of `iters` back-to-back launches (per-launch average of each round)
    times = []
    for _ in range(rounds):
        if barrier:
            torch.cuda.synchronize()
            dist.barrier()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(iters):
            run()
        ev1.record()
        ev1.synchronize()
        times.append(ev0.elapsed_time(ev1) / iters)
    ms = sorted(times)[len(times) // 2]
    es = torch.finfo(dtype).bits // 8
    nbytes = 4 * B * D * L * es + 2 * B * N * L * es + (D * N + 2 * D) * 4
    del u, z, delta, Bm, Cm, out
    torch.cuda.empty_cache()
    return ms, nbytes, nbytes / (ms * 1e-3)


def pmc_source():
    """The newest committed PMC summary of the roofline kernel
    (profiles/rNN_scan_pmc_summary.json, made by the round's evidence script +
    tools/pmc_summary.py)."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_scan_pmc_summary.json")))
    return paths[-1] if paths else None


def pmc_traffic(dtype_key):
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3
    PMC passes (pmc_source()): 2 x FETCH_SIZE (gfx950 counts half of wide
    coalesced streaming reads, MI355X_MICROARCH.md HBM section) + WRITE_SIZE,
    both KB x 1024."""
    path = pmc_source()
    try:
        with open(path) as f:
            return json.load(f)[dtype_key]["traffic_bytes"]
    except (OSError, KeyError, ValueError, TypeError):
        return None


def decode_bench(steps, B=32):
    import mamba_decoder
    c = dict(C2)
    dev = "cuda"
    torch.manual_seed(0)
    m = mamba_decoder.MambaTTSDecoder(c["vocab"], d_model=c["d_model"], n_layers=c["n_layers"],
                                      n_heads=c["n_heads"], d_ff=c["d_ff"], d_style=c["d_style"]).to(dev).eval()
    m.compute_dtype = torch.bfloat16
    c["B"] = B
    _, text, z, mask = make_batch(c, dev, 7)
    tok = torch.zeros(B, 1, dtype=torch.long, device=dev)
    states = [None] * c["n_layers"]
    lat = []
    with torch.no_grad():
        for t in range(steps):
            t0 = time.perf_counter()
            lg, states = m.decode_step(tok, text, z, states, t, text_mask=mask)
            tok = lg.argmax(-1)
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t0) * 1e3)
    lat = sorted(lat[min(100, steps // 4):])
    return {"B": B, "steps": steps, "p50_ms": lat[len(lat) // 2], "p90_ms": lat[int(len(lat) * 0.9)],
            "mode": m.decode_mode, "layers": c["n_layers"], "d_model": c["d_model"], "T_text": c["T_text"]}


def style_bench(B=8, T_text=128, d_model=1024, d_style=256, iters=20):
    """the style pipeline (style_cross_attention.py) at a
    C5-like shape, bf16: the HIP length regulator alone (HBM roofline: it
    moves out + in rows once) and the whole StyleConditioningPipeline, eval
    forward (single-key attention shortcut) and train fwd+bwd."""
    import style_cross_attention as sca
    from mtts import ops
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(3)
    text = torch.randn(B, T_text, d_model, device=dev, generator=g).to(torch.bfloat16)
    style = torch.randn(B, d_style, device=dev, generator=g).to(torch.bfloat16)
    dur = torch.randint(2, 15, (B, T_text), device=dev, generator=g).float()   # ~8 frames / phoneme
    max_len = int(ops.length_regulate_lengths(dur).max().item())

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / iters

    # the regulator kernel alone: 10 launches captured in a hipGraph, so the
    # per-launch time is GPU time, not Python/ctypes launch overhead
    with torch.no_grad():
        ops.LengthRegulateFn.apply(text, dur, max_len)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(10):
                ops.LengthRegulateFn.apply(text, dur, max_len)
    reg_ms = timed(graph.replay) / 10
    reg_bytes = B * max_len * d_model * 2 + B * T_text * d_model * 2
    # as train_harness runs it: fp32 master parameters, bf16 compute
    # (compute_dtype), gradients set to None before each step (no accumulation
    # kernels), and a fixed upstream gradient for the frames (the loss that
    # would consume them is not part of the pipeline)
    pipe = sca.StyleConditioningPipeline(d_style=d_style, d_model=d_model, num_heads=8, dropout=0.1).to(dev)
    pipe.compute_dtype = torch.bfloat16
    pipe.eval()
    with torch.no_grad():
        eval_ms = timed(lambda: pipe(text, style, dur, max_frame_len=max_len))
    pipe.train()
    textg = text.detach().requires_grad_(True)
    gframes = torch.randn(B, max_len, d_model, device=dev, generator=g).to(torch.bfloat16)
    params = list(pipe.parameters())

    from mtts import dropout as DO

    def train_step():
        DO.advance()             # fresh dropout masks on every (replayed) step
        for prm in params:
            prm.grad = None
        textg.grad = None
        frames, _, _, _ = pipe(textg, style, dur, max_frame_len=max_len)
        frames.backward(gframes)
    train_ms = timed(train_step)
    # the same step captured once as a hipGraph (~110 launches: the eager
    # step is partly bound by host launch work)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        train_step()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        train_step()
    graph_ms = timed(graph.replay)
    return {"B": B, "T_text": T_text, "T_frame": max_len, "d_model": d_model, "dtype": "bf16",
            "regulator": {"ms": reg_ms, "bound": "hbm", "achieved": reg_bytes / reg_ms / 1e6, "peak": HBM_PEAK / 1e9,
                          "unit": "GB/s", "frac": reg_bytes / (reg_ms * 1e-3) / HBM_PEAK},
            "pipeline_eval_ms": eval_ms, "pipeline_train_fwd_bwd_ms": train_ms,
            "pipeline_train_fwd_bwd_graph_ms": graph_ms}


def c5_step_bench(rank, world, dev, B=8, T_text=128, T_codec=1024, T_ref=1024, steps=3, warmup=2):
    """BASELINE configs[4] (C5): one train.py step (train.py:168-241) on
    synthetic batches through train_harness.TrainStep at train.py's widths
    (build_models: d_model 512, d_style 256, 8-layer decoder, 5 FACodec
    streams of 1024 frames flattened to T_audio = 5120, the voice prompt as
    5120 reference keys + 128 text keys, text encoder 4 FFT blocks, duration
    predictor, style pipeline (dead output, as in train.py), 3-term loss,
    clip (decoder) + Adam), decoder in bf16, dropout 0.1 as train.py, B per
    rank; with N ranks the gradients of every trainable parameter are
    all-reduced over RCCL before the optimizer (batch DP, weak scaling).
    Timed like the headline: barrier + synchronize on both sides, max over
    ranks; tokens = audio tokens (B * 5120) of all ranks."""
    import train_harness as th
    torch.manual_seed(0)
    models = th.build_models(dev, compute_dtype=torch.bfloat16)
    dp = None
    if world > 1:
        from mtts.dp import GradAllReduce
        trainable = [p for m in (models.text_encoder, models.dur_predictor, models.decoder)
                     for p in m.parameters() if p.requires_grad]
        dp = GradAllReduce(trainable, bucket_mb=128)
    step = th.TrainStep(models, lr=1e-4, grad_allreduce=dp)
    batch = th.synthetic_batch(B, dev, T_text=T_text, T_codec=T_codec, T_ref=T_ref, seed=77 + rank)
    for _ in range(warmup):
        first = step(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = _max_over_ranks(time.perf_counter() - t0, world, dev)
    ms = dt / steps * 1e3
    T_audio = T_codec * th.CODEC_STREAMS
    res = {"B_per_rank": B, "T_audio": T_audio, "T_kv": T_ref * th.CODEC_STREAMS + T_text, "T_text": T_text,
           "n_gpus": world, "ms_per_step": ms, "tokens_per_s": world * B * T_audio / dt * steps,
           "dtype": "decoder and (dead) style branch bf16, text encoder / duration predictor fp32",
           "losses_first_last": [float(first["loss_total"]), float(out["loss_total"])]}
    del models, step, dp
    torch.cuda.empty_cache()
    return res


def text_bench(B=8, T_text=128, d_model=512, iters=10):
    """TextEncoder (4 FFT blocks, 2 heads of 64, conv FFN
    k=9 to 1024) + DurationPredictor at train.py's width (d_model 512), fp32
    as the reference, fwd + bwd of encoder output and duration loss."""
    import text_encoder as te
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

    from mtts import dropout as DO

    def step():
        DO.advance()             # fresh dropout masks on every (replayed) step
        for p in params:
            p.grad = None
        h = enc(ids, mask=mask)
        loss = dur.compute_loss(dur(h, mask=mask), target, mask=mask) + h.square().mean()
        loss.backward()

    def clock(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / iters * 1e3

    side = torch.cuda.Stream()      # eager warm-up on a side stream (torch's capture recipe)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(side)
    eager_ms = clock(step)
    # the same fwd + bwd (dropout included: the HIP dropout's device seed
    # base advances per replay, mtts.dropout.advance) captured once as a
    # hipGraph: ~400 launches of 2-15 us each, so an eager step is bound by
    # host launch work on a slow host core
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    graph_ms = clock(graph.replay)
    return {"B": B, "T_text": T_text, "d_model": d_model, "dtype": "fp32",
            "fwd_bwd_ms": graph_ms, "mode": "hipGraph replay", "fwd_bwd_eager_ms": eager_ms}


def cpu_baseline_scan(L=8192, D=2048):
    """oracle selective_scan_ref (pure PyTorch, fp32, CPU) on a bounded slice
    of the north-star scan (one of its 32 batch rows: B=1, L=8192,
    d_inner=2048, N=16), softplus + z
    gate; reported in the roofline's unit (algorithmic bytes / s, fp32 I/O)."""
    from oracle import mamba_ref as R
    torch.set_num_threads(min(os.cpu_count() or 1, 64))
    g = torch.Generator().manual_seed(0)
    N = 16
    u, z = torch.randn(1, D, L, generator=g), torch.randn(1, D, L, generator=g)
    delta = torch.randn(1, D, L, generator=g) * 0.1
    Bm, Cm = torch.randn(1, N, L, generator=g), torch.randn(1, N, L, generator=g)
    A = -torch.arange(1, N + 1, dtype=torch.float32).repeat(D, 1)
    bias = torch.full((D,), -4.0)
    t0 = time.perf_counter()
    R.selective_scan_ref(u, delta, A, Bm, Cm, torch.ones(D), z, bias, True)
    dt = time.perf_counter() - t0
    nbytes = 4 * D * L * 4 + 2 * N * L * 4 + (D * N + 2 * D) * 4
    return {"value": nbytes / dt / 1e9, "unit": "GB/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle/mamba_ref.py selective_scan_ref, B=1 L={L} d_inner={D} N=16 fp32, {dt:.1f}s "
                      f"({D * L / dt / 1e6:.2f} M (b,d,l)/s)"}


def cpu_baseline(budget_s=20.0):
    """oracle (pure PyTorch, CPU) fwd+bwd of the same 12L d=1024 decoder on a
    bounded sample (B=1, T=64, T_text=128)."""
    from oracle import mamba_ref as R
    import mamba_decoder
    torch.set_num_threads(min(os.cpu_count() or 1, 64))
    c = dict(C2)
    torch.manual_seed(0)
    m = mamba_decoder.MambaTTSDecoder(c["vocab"], d_model=c["d_model"], n_layers=c["n_layers"],
                                      n_heads=c["n_heads"], d_ff=c["d_ff"], d_style=c["d_style"])
    p = {k: v.detach().float().requires_grad_(True) for k, v in m.state_dict().items()}
    B, T = 1, 64
    g = torch.Generator().manual_seed(0)
    tok = torch.randint(0, 10, (B, T), generator=g)
    text = torch.randn(B, c["T_text"], c["d_model"], generator=g)
    z = torch.randn(B, c["d_style"], generator=g)
    mask = torch.ones(B, c["T_text"], dtype=torch.bool)
    mask[:, int(c["T_text"] * 0.9):] = False
    n, t0 = 0, time.perf_counter()
    while True:
        lg = R.decoder_forward_ref(p, c["n_layers"], c["n_heads"], tok, text, z, text_mask=mask)
        torch.nn.functional.cross_entropy(lg.view(-1, 10), tok.view(-1), ignore_index=0).backward()
        n += 1
        if time.perf_counter() - t0 > budget_s or n >= 50:
            break
    dt = time.perf_counter() - t0
    return {"value": n * B * T / dt, "unit": "tokens/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle/mamba_ref.py decoder fwd+bwd, 12L d=1024, B=1 T_audio=64 T_text=128, fp32, "
                      f"{n} iters in {dt:.1f}s"}


def launch_ranks(n):
    """`python bench.py --gpus N` without a launcher: run torch.distributed.run
    with N ranks (one per GPU) as a CHILD process -- started before anything
    here touches the GPU -- and return its exit code.  Rank 0's JSON line
    reaches stdout directly (inherited descriptors)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    log(f"[bench] launching {n} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


def _max_over_ranks(v, world, dev):
    if world == 1:
        return v
    t = torch.tensor([v], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def dp_breakdown(forward_loss, dp, dev, steps=3):
    """N > 1: why a scaling record looks the way it does.  Runs
    `steps` extra data-parallel steps after the timed region and reports, per
    rank, the backward time (loss.backward() with the bucketed all-reduces
    overlapping it) and the all-reduce time left EXPOSED after it (backward
    end -> GradAllReduce.finish() return: the stream waits for the buckets
    still in flight), medians over the steps, max over ranks; plus the bucket
    layout.  HIP events on the compute stream on GPU, wall clock on CPU."""
    import statistics
    from mtts import wgrad
    cuda = torch.device(dev).type == "cuda"
    world = dist.get_world_size() if dist.is_initialized() else 1
    bwd, exposed = [], []
    for _ in range(steps):
        loss = forward_loss()
        dp.zero_grad()
        if cuda:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record()
        t0 = time.perf_counter()
        with wgrad.deferred():
            loss.backward()
        if cuda:
            ev[1].record()
        t1 = time.perf_counter()
        dp.finish()
        if cuda:
            ev[2].record()
            torch.cuda.synchronize()
            bwd.append(ev[0].elapsed_time(ev[1]))
            exposed.append(ev[1].elapsed_time(ev[2]))
        else:
            t2 = time.perf_counter()
            bwd.append((t1 - t0) * 1e3)
            exposed.append((t2 - t1) * 1e3)
    rec = {"backward_ms": _max_over_ranks(statistics.median(bwd), world, dev),
           "allreduce_exposed_ms": _max_over_ranks(statistics.median(exposed), world, dev),
           "steps": steps,
           "timing": ("median over steps of per-rank " + ("HIP-event" if cuda else "wall-clock") +
                      " times on the compute stream, max over ranks; exposed = backward end -> "
                      "GradAllReduce.finish() return")}
    rec.update(dp.describe())
    return rec


def launch_check(args, world):
    """The N-rank plumbing without GPU work (CPU, gloo): process group,
    barrier-bracketed 'timed region', max-over-ranks time, rank-0 JSON."""
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group(os.environ.get("MTTS_DIST_BACKEND", "gloo"))
        dist.barrier()
    t0 = time.perf_counter()
    x = torch.ones(1024) * (rank + 1)
    if world > 1:
        dist.all_reduce(x)
        dist.barrier()
    dt = _max_over_ranks(time.perf_counter() - t0, world, "cpu")
    rec = {"metric": "launch-check", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "allreduce_ok": bool(x[0].item() == world * (world + 1) / 2), "seconds": dt}
    if world > 1:
        # the N > 1 line's data-parallel breakdown on a small CPU model (gloo)
        from mtts.dp import GradAllReduce
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.GELU(), torch.nn.Linear(512, 256))
        dp = GradAllReduce(list(model.parameters()), bucket_mb=0.25, first_bucket_mb=0.125)
        xin = torch.randn(64, 256)
        rec["dp"] = dp_breakdown(lambda: model(xin).square().mean(), dp, "cpu", steps=args.steps)
        dp.remove()
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


def scan_scaling(rank, world, dev, iters=10):
    """Second scaling leg: the north-star selective_scan forward (fp32 I/O)
    with no collective on the data path.  weak: every rank scans its own
    B=32 batch; strong: the B=32 batch split 32/N rows per rank.  Per leg:
    barrier, `iters` launches, synchronize, barrier; time = max over ranks;
    value = algorithmic bytes of all ranks / time."""
    out = {}
    for leg in ("weak", "strong"):
        B = 32 if leg == "weak" else max(1, 32 // world)
        if world > 1:
            dist.barrier()
        ms, nbytes, _ = scan_roofline(torch.float32, B=B, iters=iters, rounds=1, barrier=world > 1)
        ms = _max_over_ranks(ms, world, dev)
        total = nbytes * world
        out[leg] = {"batch_per_rank": B, "ms_per_launch": ms, "GB_per_s": total / (ms * 1e-3) / 1e9,
                    "frac_of_n_x_hbm_peak": total / (ms * 1e-3) / (world * HBM_PEAK)}
    out["unit"] = "GB/s (algorithmic bytes of all ranks / max-over-ranks time)"
    log(f"[bench] scan scaling N={world}: {out}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--decode-steps", type=int, default=4096)   # C4: 4096-step AR loop
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--skip-extras", action="store_true")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: replay the training step as one captured hipGraph (equal speed here: the step is GPU-bound)")
    ap.add_argument("--launch-check", action="store_true",
                    help="distributed plumbing only (process group, barrier, max-over-ranks timing, JSON line), "
                         "no GPU work: CPU rehearsal of the N-rank launch with MTTS_DIST_BACKEND=gloo")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; reporting n_gpus={world}")
    if args.launch_check:
        return launch_check(args, world)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # MTTS_DIST_BACKEND=gloo + more ranks than GPUs: a rehearsal of the
        # data-parallel path on one card (ranks share it); the product path is
        # "nccl" (RCCL over xGMI), one rank per GPU
        local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("MTTS_DIST_BACKEND", "nccl"))
    dev = torch.device("cuda", local)
    from mtts import _lib
    _lib.lib()

    # the roofline kernel is timed first, on the chip as the driver hands it over
    # (after the C2 training loop the same launches measure ~5-7 % slower: clocks)
    roof = None
    if rank == 0 and world == 1 and not args.skip_extras:
        roof = (scan_roofline(torch.float32), scan_roofline(torch.bfloat16))
    c, ms, tps, loss, dpinfo = train_bench(args, rank, world, dev)
    scaling_leg = scan_scaling(rank, world, dev)
    log(f"[bench] step {ms:.2f} ms  {tps:.0f} tok/s  loss first warmup step {loss[0]} -> last timed step {loss[1]:.3e} "
        f"(one fixed batch; the decoder's unshifted targets, SURVEY quirk 4, make it learn the identity fast)")
    rec = {
        "metric": "audio tokens/sec (teacher-forced fwd+bwd) per GPU; decode_step p50 latency",
        "value_meaning": "whole job: tokens of all ranks / max-over-ranks time (value_per_gpu = value / n_gpus)",
        "value": tps, "value_per_gpu": tps / world, "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (random tokens/text/z_style, random-init weights)",
        "config": {"workload": "C2: MambaTTSDecoder 12L d_model=1024 fwd+bwd+clip+Adam, B=8/GPU T_audio=2048 "
                               "T_text=128", "model": "MambaTTSDecoder-12L-d1024", "global_batch": c["B"] * world,
                   "seq_len": c["T"], "parallelism": f"dp{world}"},
    }
    fl = flops_per_step(c)
    rec["step_mfma"] = {"bound": "mfma", "achieved": fl / (ms * 1e-3) / 1e12, "peak": BF16_PEAK / 1e12,
                        "unit": "TFLOP/s", "frac": fl / (ms * 1e-3) / BF16_PEAK, "flops_per_step": fl}
    rec["scan_scaling"] = scaling_leg
    if dpinfo is not None:
        rec["dp"] = dpinfo
    if roof is None:
        # N > 1 (or --skip-extras): the roofline kernel's per-GPU figure from the
        # weak leg (each rank ran the full north-star batch; slowest rank)
        wk = scaling_leg["weak"]
        nb = wk["GB_per_s"] * 1e9 * wk["ms_per_launch"] * 1e-3 / world
        roof = ((wk["ms_per_launch"], nb, nb / (wk["ms_per_launch"] * 1e-3)), None)
    if rank == 0:
        (fms, fb, fbw) = roof[0]
        log(f"[bench] scan fp32 north-star {fms:.3f} ms {fbw / 1e9:.0f} GB/s")
        rec["roofline"] = {"kernel": "selective_scan_fwd (north-star B=32 L=8192 d_inner=2048 N=16, fp32 I/O = the "
                                     "reference's precision, f32 math)",
                           "bound": "hbm", "achieved": fbw / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                           "frac": fbw / HBM_PEAK, "traffic": pmc_traffic("fp32"), "ms": fms, "algorithmic_bytes": fb,
                           "traffic_source": f"{os.path.relpath(pmc_source() or 'none', ROOT)} "
                                             "(2*FETCH_SIZE+WRITE_SIZE)"}
        if roof[1] is not None:
            (sms, sb, sbw) = roof[1]
            log(f"[bench] scan bf16 north-star {sms:.3f} ms {sbw / 1e9:.0f} GB/s")
            rec["roofline_bf16"] = {"bound": "hbm (VALU-limited, DESIGN.md section 3)", "achieved": sbw / 1e9,
                                    "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": sbw / HBM_PEAK, "ms": sms,
                                    "algorithmic_bytes": sb, "traffic": pmc_traffic("bf16")}
    if not args.skip_extras:
        rec["c5_step"] = c5_step_bench(rank, world, dev)
        log(f"[bench] c5 step {rec['c5_step']}")
    if rank == 0 and world == 1 and not args.skip_extras:
        rec["text_encoder"] = text_bench()
        log(f"[bench] text encoder {rec['text_encoder']}")
        rec["style"] = style_bench()
        log(f"[bench] style {rec['style']}")
        if args.decode_steps > 0:
            rec["decode"] = decode_bench(args.decode_steps)
            log(f"[bench] decode {rec['decode']}")
        if args.cpu_budget > 0:
            rec["cpu_baseline"] = cpu_baseline(args.cpu_budget)
            log(f"[bench] cpu {rec['cpu_baseline']}")
            rec["cpu_baseline_scan"] = cpu_baseline_scan()
            log(f"[bench] cpu scan {rec['cpu_baseline_scan']}")
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
