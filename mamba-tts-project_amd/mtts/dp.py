"""Batch data parallelism for the decoder training step.

One process per GPU; every rank runs the full model on its own batch shard;
the only exchange is the gradient all-reduce (torch.distributed, backend
"nccl" = RCCL over xGMI on MI355X, "gloo" on CPU for tests).

Design: all trainable gradients live in ONE flat fp32 buffer (param.grad are
views into it, laid out in reverse registration order ~ backward order), cut
into buckets of `bucket_mb`.  A post-accumulate-grad hook counts finished
parameters per bucket; a full bucket is all-reduced asynchronously while the
backward continues (overlap), and `finish()` waits for the stragglers and
applies the 1/world averaging.  Large buckets (default 128 MB) suit xGMI's
point-to-point links: few, large ring collectives.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class GradAllReduce:
    def __init__(self, params, bucket_mb: float = 128.0, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.params = [p for p in params if p.requires_grad]
        order = list(reversed(self.params))
        dev = order[0].device
        total = sum(p.numel() for p in order)
        self.flat = torch.zeros(total, device=dev, dtype=torch.float32)
        cap = max(1, int(bucket_mb * 1024 * 1024 // 4))
        self.buckets = []        # (start, end, n_params)
        self.bucket_of = {}
        off, start, count = 0, 0, 0
        for p in order:
            if p.dtype != torch.float32:
                raise TypeError("GradAllReduce expects fp32 master parameters")
            n = p.numel()
            p.grad = self.flat[off:off + n].view_as(p)
            self.bucket_of[p] = len(self.buckets)
            off += n
            count += 1
            if off - start >= cap:
                self.buckets.append([start, off, count])
                start, count = off, 0
        if count:
            self.buckets.append([start, off, count])
        self.pending = [0] * len(self.buckets)
        self.handles = [None] * len(self.buckets)
        self.hooks = [p.register_post_accumulate_grad_hook(self._hook) for p in self.params]

    def zero_grad(self):
        self.flat.zero_()
        self.pending = [0] * len(self.buckets)
        self.handles = [None] * len(self.buckets)

    def _hook(self, p):
        b = self.bucket_of[p]
        self.pending[b] += 1
        if self.pending[b] == self.buckets[b][2]:
            s, e, _ = self.buckets[b]
            self.handles[b] = dist.all_reduce(self.flat[s:e], group=self.group, async_op=True)

    def finish(self):
        """Wait for every bucket (launching any whose hooks did not all fire,
        e.g. unused parameters) and average over ranks."""
        for b, (s, e, _) in enumerate(self.buckets):
            if self.handles[b] is None:
                self.handles[b] = dist.all_reduce(self.flat[s:e], group=self.group, async_op=True)
        for h in self.handles:
            h.wait()
        if self.world > 1:
            self.flat.mul_(1.0 / self.world)
        self.handles = [None] * len(self.buckets)
        self.pending = [0] * len(self.buckets)

    def remove(self):
        for h in self.hooks:
            h.remove()
