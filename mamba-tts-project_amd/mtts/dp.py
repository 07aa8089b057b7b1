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
point-to-point links: few, large ring collectives.  The FIRST bucket (the
parameters whose gradients the backward finishes first: the head and the
last layer) is capped at `first_bucket_mb` so the first all-reduce starts
early in the backward.  Gradients are not accumulated in place: each step
starts with p.grad = None, autograd allocates every gradient fresh and the
post-accumulate hook copies it into its view (one copy instead of a zero-fill
of the whole buffer plus an in-place add per parameter); with RCCL the
collective averages (ReduceOp.AVG).

`comm_dtype=torch.bfloat16` all-reduces a bf16 image of each bucket (half
the bytes on the links; the fp32 gradients are rounded once to bf16 before
the sum and the bf16 sum is widened back into the fp32 buffer before the
averaging), the gradient-compression option for xGMI-bound steps.  The
default is fp32 (exact sums up to the collective's order).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import wgrad

DEFER_LISTENER_LAUNCH = True


class GradAllReduce:
    def __init__(self, params, bucket_mb: float = 128.0, group=None, first_bucket_mb: float = 8.0,
                 comm_dtype: torch.dtype = None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.bucket_mb, self.first_bucket_mb = bucket_mb, first_bucket_mb
        self.params = [p for p in params if p.requires_grad]
        order = list(reversed(self.params))
        dev = order[0].device
        dtype = order[0].dtype
        # every parameter's view starts on a 256-byte boundary (the deferred
        # weight-gradient GEMMs, mtts.wgrad, store 16-byte pieces straight
        # into it); the padding stays zero and rides along in the all-reduce
        al = max(1, 256 // torch.empty(0, dtype=dtype).element_size())
        pad = lambda n: -(-n // al) * al  # noqa: E731
        total = sum(pad(p.numel()) for p in order)
        self.flat = torch.zeros(total, device=dev, dtype=dtype)
        cap_rest = max(1, int(bucket_mb * 1024 * 1024 // self.flat.element_size()))
        cap = max(1, int(min(first_bucket_mb, bucket_mb) * 1024 * 1024 // self.flat.element_size()))
        if comm_dtype is not None and comm_dtype not in (torch.bfloat16, dtype):
            raise TypeError("GradAllReduce: comm_dtype must be None, the parameter dtype or torch.bfloat16")
        self.comm_dtype = None if comm_dtype in (None, dtype) else comm_dtype
        self.buckets = []        # (start, end, n_params)
        self.bucket_of = {}
        off, start, count = 0, 0, 0
        self.views = {}
        for p in order:
            if p.dtype != dtype or dtype not in (torch.float32, torch.float64):
                raise TypeError("GradAllReduce expects fp32 (or, for tests, fp64) master parameters of one dtype")
            n = p.numel()
            # the bucket view takes p's own (dense) strides: a gradient of p's
            # layout folds into it with a straight copy and the fused optimizer
            # sees p, grad and moments in one storage order
            self.views[p] = self.flat[off:off + n].as_strided(p.shape, p.stride())
            p.grad = self.views[p]
            self.bucket_of[p] = len(self.buckets)
            off += pad(n)
            count += 1
            if off - start >= cap:
                self.buckets.append([start, off, count])
                start, count = off, 0
                cap = cap_rest
        if count:
            self.buckets.append([start, off, count])
        self.cbuf = None if self.comm_dtype is None else torch.empty(total, device=dev, dtype=self.comm_dtype)
        self.pending = [0] * len(self.buckets)
        self.handles = [None] * len(self.buckets)
        self.counted = set()     # ids of the parameters counted into their bucket this step
        self.ready = []          # buckets completed inside a deferred flush, launched at the next hook
        self.hooks = [p.register_post_accumulate_grad_hook(self._hook) for p in self.params]
        # deferred weight gradients (mtts.wgrad) are written straight into the
        # bucket views and announced through the engine's listener
        for p, v in self.views.items():
            p._mtts_grad_view = v
        wgrad.add_listener(self._deferred_ready)

    def _deferred_ready(self, p):
        if p in self.views:
            self._hook(p, from_listener=True)

    def zero_grad(self):
        """Start a step: drop the gradients (p.grad = None).  Autograd then
        hands each parameter a fresh gradient (no zero-fill of the flat buffer,
        no in-place accumulation into it) and the hook folds it into its view
        with one copy; parameters that receive no gradient are zeroed at
        finish().  optimizer.zero_grad(set_to_none=True) is equivalent."""
        for p in self.views:
            p.grad = None
        self.pending = [0] * len(self.buckets)
        self.handles = [None] * len(self.buckets)
        self.counted = set()

    def _hook(self, p, from_listener=False):
        if p.grad is None:
            # autograd runs post-accumulate hooks even when a backward returned
            # no gradient for p -- the deferred weight gradients (mtts.wgrad)
            # do exactly that and announce p through the engine's listener
            return
        if not from_listener and wgrad.owns(p):
            # a deferred gradient still incomplete (some row slices queued or
            # not yet submitted): the engine's listener announces it when done
            return
        if id(p) in self.counted:
            # counted once per step: a deferred gradient flushed inside p's own
            # backward (mtts.wgrad's mid-backward flush) is announced by the
            # engine's listener AND then seen here by autograd's hook
            return
        self.counted.add(id(p))
        v = self.views[p]
        if p.grad is not v and p.grad.data_ptr() != v.data_ptr():
            # autograd allocated a fresh gradient (the optimizer's zero_grad
            # set_to_none=True dropped the view): fold it into the bucket view
            # (the stale bucket content is overwritten, as after a zeroing) so
            # the all-reduce sees it, and re-bind
            v.copy_(p.grad)
            p.grad = v
        b = self.bucket_of[p]
        self.pending[b] += 1
        if self.pending[b] == self.buckets[b][2]:
            if from_listener and DEFER_LISTENER_LAUNCH:
                self.ready.append(b)
            else:
                self._launch_ready()
                self._launch(b)
        elif not from_listener:
            self._launch_ready()

    def _launch_ready(self):
        while self.ready:
            self._launch(self.ready.pop(0))

    def _avg_op(self):
        """RCCL averages in the collective (ReduceOp.AVG: no separate 1/world
        pass over the buffer); gloo sums and finish() scales."""
        if not hasattr(self, "_avg"):
            self._avg = dist.get_backend(self.group) == "nccl"
        return self._avg

    def _launch(self, b):
        s, e, _ = self.buckets[b]
        buf = self.flat[s:e]
        if self.cbuf is not None:
            self.cbuf[s:e].copy_(buf)          # one rounding to the wire dtype
            buf = self.cbuf[s:e]
        if self._avg_op():
            try:
                self.handles[b] = dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
                return
            except (RuntimeError, ValueError):   # a backend build without AVG: sum + scale in finish()
                if any(h is not None for h in self.handles):
                    raise
                self._avg = False
        self.handles[b] = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def finish(self):
        """Wait for every bucket (launching any whose hooks did not all fire,
        e.g. unused parameters) and average over ranks."""
        self._launch_ready()
        for p, v in self.views.items():   # no gradient this step: contributes zeros
            if p.grad is None:
                v.zero_()
                p.grad = v
        for b in range(len(self.buckets)):
            if self.handles[b] is None:
                self._launch(b)
        for b, h in enumerate(self.handles):
            h.wait()
            if self.cbuf is not None:
                s, e, _ = self.buckets[b]
                self.flat[s:e].copy_(self.cbuf[s:e])
        for p, v in self.views.items():
            if p.grad is not None and p.grad is not v and p.grad.data_ptr() != v.data_ptr():
                raise RuntimeError("GradAllReduce: a gradient left the flat buffer after its hook; "
                                   "zero gradients with GradAllReduce.zero_grad()")
        if self.world > 1 and not self._avg_op():
            self.flat.mul_(1.0 / self.world)
        self.handles = [None] * len(self.buckets)
        self.pending = [0] * len(self.buckets)
        self.counted = set()

    def describe(self) -> dict:
        """Bucket layout, for the bench line (bench.py dp_breakdown)."""
        es = self.flat.element_size()
        return {"buckets": len(self.buckets), "bucket_mb": self.bucket_mb, "first_bucket_mb": self.first_bucket_mb,
                "grad_MB": self.flat.numel() * es / 2 ** 20,
                "bucket_MB": [round((e - s) * es / 2 ** 20, 3) for s, e, _ in self.buckets],
                "comm_dtype": str(self.comm_dtype or self.flat.dtype).replace("torch.", ""),
                "reduce_op": "avg" if self._avg_op() else "sum+scale"}

    def remove(self):
        for h in self.hooks:
            h.remove()
        wgrad.remove_listener(self._deferred_ready)
        for p in self.views:
            if getattr(p, "_mtts_grad_view", None) is not None:
                del p._mtts_grad_view
