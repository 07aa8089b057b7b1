"""Multi-process data-parallel gradient all-reduce (mtts/dp.py) on CPU with
the gloo backend, world_size 2, on the DECODER's parameter set: a 2-layer
MambaTTSDecoder's state_dict as trainable tensors, its forward evaluated by
the float64 oracle restatement (the HIP forward needs a GPU: the same test on
the real module + FusedClipAdam is tests/test_gpu_dp.py), CE(ignore 0) loss,
clip_grad_norm_(1.0) + Adam (train.py:228-235).

Checks: after 2 steps the averaged gradients and the updated parameters of
every rank equal a single process stepping on the mean of the per-shard
losses; small buckets (many overlapped all-reduces) and one big bucket;
zero_grad through GradAllReduce, and through the optimizer's
zero_grad(set_to_none=True) (the hooks re-bind fresh gradients into the
flat buffer)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2
SHARD = 2        # sequences per rank
T, TT, D = 16, 6, 32


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    """The drop-in module only for its parameter set (keys / shapes / init)."""
    import mamba_decoder
    torch.manual_seed(0)
    m = mamba_decoder.MambaTTSDecoder(10, d_model=D, n_layers=2, n_heads=4, d_ff=64, d_style=8, max_len=64)
    return {k: torch.nn.Parameter(v.detach().double().clone()) for k, v in m.state_dict().items()}


def _batch():
    g = torch.Generator().manual_seed(100)
    tok = torch.randint(0, 10, (WORLD * SHARD, T), generator=g)
    text = torch.randn(WORLD * SHARD, TT, D, generator=g, dtype=torch.float64)
    z = torch.randn(WORLD * SHARD, 8, generator=g, dtype=torch.float64)
    mask = torch.ones(WORLD * SHARD, TT, dtype=torch.bool)
    mask[:, 4:] = False
    return tok, text, z, mask


def _loss(p, tok, text, z, mask):
    from oracle import mamba_ref as R
    logits = R.decoder_forward_ref(p, 2, 4, tok, text, z, text_mask=mask)
    return torch.nn.functional.cross_entropy(logits.reshape(-1, 10), tok.reshape(-1), ignore_index=0)


def _worker(rank, port, bucket_mb, zero_mode, q, comm="fp32"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from mtts.dp import GradAllReduce
    p = _model()
    if comm == "bf16":   # fp32 masters (GradAllReduce's product dtype), bf16 on the wire
        p = {k: torch.nn.Parameter(v.detach().float()) for k, v in p.items()}
    params = list(p.values())
    tok, text, z, mask = _batch()
    if comm == "bf16":
        text, z = text.float(), z.float()
    sl = slice(rank * SHARD, (rank + 1) * SHARD)
    dp = GradAllReduce(params, bucket_mb=bucket_mb, comm_dtype=torch.bfloat16 if comm == "bf16" else None,
                       first_bucket_mb=bucket_mb / 4)
    opt = torch.optim.Adam(params, lr=1e-3)
    for _ in range(2):  # twice: bucket state and gradient views must reset between steps
        if zero_mode == "dp":
            dp.zero_grad()
        else:
            opt.zero_grad(set_to_none=True)
        _loss(p, tok[sl], text[sl], z[sl], mask[sl]).backward()
        dp.finish()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
    # numpy copies travel by value (no shared memory that dies with this process)
    q.put((rank, {k: (v.grad.detach().numpy().copy(), v.detach().numpy().copy()) for k, v in p.items()},
           len(dp.buckets)))
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb,zero_mode", [(1e-3, "dp"), (128.0, "dp"), (1e-2, "set_to_none")])
def test_decoder_grad_allreduce_gloo_world2(bucket_mb, zero_mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, bucket_mb, zero_mode, q)) for r in range(WORLD)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=300) for _ in range(WORLD)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    # single process: mean over ranks of the per-shard losses (each rank's CE
    # averages over its own non-ignored tokens, so this is what DP computes)
    p = _model()
    params = list(p.values())
    tok, text, z, mask = _batch()
    opt = torch.optim.Adam(params, lr=1e-3)
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        sum(_loss(p, tok[r * SHARD:(r + 1) * SHARD], text[r * SHARD:(r + 1) * SHARD], z[r * SHARD:(r + 1) * SHARD],
                  mask[r * SHARD:(r + 1) * SHARD]) for r in range(WORLD)).div(WORLD).backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
    for rank, got, nb in res:
        if bucket_mb < 1:
            assert nb > 1, "small buckets must split the flat buffer"
        for k, v in p.items():
            g, w = got[k]
            ref_g = v.grad if v.grad is not None else torch.zeros_like(v)
            torch.testing.assert_close(torch.from_numpy(g), ref_g, rtol=1e-9, atol=1e-12, msg=f"grad {k}")
            torch.testing.assert_close(torch.from_numpy(w), v.detach(), rtol=1e-9, atol=1e-12, msg=f"param {k}")


def test_decoder_grad_allreduce_bf16_wire_gloo_world2():
    """comm_dtype=bf16: each rank's fp32 gradients are rounded once to bf16,
    summed in bf16 and widened back.  Bounds (stated): per tensor, the
    averaged gradients within 2e-2 of max|ref| (two bf16 roundings of 2^-9
    each plus the bf16 sum); the parameter UPDATE of two Adam steps within 10 %
    of the reference update in L2 norm per tensor (Adam normalises every
    element by its own history, so an element whose gradient is near zero can
    flip sign under any rounding: an element-wise bound would test noise)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, 1e-2, "dp", q, "bf16")) for r in range(WORLD)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=300) for _ in range(WORLD)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p0 = {k: v.detach().clone() for k, v in _model().items()}
    p = _model()
    params = list(p.values())
    tok, text, z, mask = _batch()
    opt = torch.optim.Adam(params, lr=1e-3)
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        sum(_loss(p, tok[r * SHARD:(r + 1) * SHARD], text[r * SHARD:(r + 1) * SHARD], z[r * SHARD:(r + 1) * SHARD],
                  mask[r * SHARD:(r + 1) * SHARD]) for r in range(WORLD)).div(WORLD).backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
    for rank, got, nb in res:
        assert nb > 2
        for k, v in p.items():
            g, w = got[k]
            ref_g = v.grad if v.grad is not None else torch.zeros_like(v)
            err = (torch.from_numpy(g).double() - ref_g).abs().max().item()
            assert err <= 2e-2 * max(ref_g.abs().max().item(), 1e-12), f"grad {k}: {err}"
            du_ref = v.detach() - p0[k]
            du = torch.from_numpy(w).double() - p0[k]
            assert (du - du_ref).norm() <= 0.1 * du_ref.norm() + 1e-9, f"update {k}"
