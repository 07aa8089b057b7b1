"""Multi-process data-parallel gradient all-reduce (mtts/dp.py) on CPU with
the gloo backend, world_size 2: averaged gradients equal the single-process
gradient of the concatenated batch, buckets overlap the backward, unused
parameters still reduce."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Toy(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(16, 32)
        self.b = torch.nn.Linear(32, 8)
        self.unused = torch.nn.Linear(4, 4)

    def forward(self, x):
        return self.b(torch.tanh(self.a(x)))


def _worker(rank, world, port, bucket_mb, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mtts.dp import GradAllReduce
    torch.manual_seed(0)
    m = Toy()
    g = torch.Generator().manual_seed(100)
    x = torch.randn(world * 6, 16, generator=g)
    dp = GradAllReduce(m.parameters(), bucket_mb=bucket_mb)
    for _ in range(2):  # twice: state must reset between steps
        dp.zero_grad()
        m(x[rank * 6:(rank + 1) * 6]).square().mean().backward()
        dp.finish()
    # numpy copies travel by value: a torch tensor would go through shared memory
    # that can vanish when this process exits before the parent reads it
    q.put((rank, {n: p.grad.detach().numpy().copy() for n, p in m.named_parameters()}, len(dp.buckets)))
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb", [1e-3, 128.0])
def test_grad_allreduce_gloo_world2(bucket_mb):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_mb, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    m = Toy()
    g = torch.Generator().manual_seed(100)
    x = torch.randn(world * 6, 16, generator=g)
    # mean over ranks of per-shard mean losses == gradient of the average
    sum(m(x[r * 6:(r + 1) * 6]).square().mean() for r in range(world)).div(world).backward()
    for rank, grads, nb in res:
        if bucket_mb < 1:
            assert nb > 1
        for n, p in m.named_parameters():
            ref = p.grad if p.grad is not None else torch.zeros_like(p)
            torch.testing.assert_close(torch.from_numpy(grads[n]), ref, rtol=1e-5, atol=1e-6)
