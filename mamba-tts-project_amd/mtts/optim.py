"""Optimizer step of the training loop (reference train.py:232-235:
clip_grad_norm_(decoder.parameters(), 1.0); optim.step() with
torch.optim.Adam(lr)).

FusedClipAdam is torch.optim.Adam (same hyper-parameters, same state names
`step` / `exp_avg` / `exp_avg_sq`, so state_dicts interchange) whose step()
also applies clip_grad_norm_(params, max_grad_norm) -- in three HIP launches
for the whole parameter list (mtts_clip_adam: partial sums of g^2, the norm
and clip coefficient on device, then Adam on g * coef).  Gradients are left
unclipped; `last_grad_norm` holds the total norm (device scalar).  The step
count is kept on the device too, so a training step that ends in step()
can be captured in a hipGraph (bench.py --graph).

clip_into_optimizer is the torch-optimizer variant (norm by foreach, the
clip folded into a fused torch Adam via grad_scale).
"""
from __future__ import annotations

import torch

from . import _lib as L


def dense(t: torch.Tensor) -> bool:
    """t covers its storage span without gaps or overlap (a permutation of a
    contiguous tensor)."""
    if t.is_contiguous():
        return True
    order = sorted(range(t.dim()), key=lambda d: -t.stride(d))
    return t.permute(order).is_contiguous()


def same_layout(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Equal shapes and strides (a size-1 dimension's stride does not matter)."""
    return a.shape == b.shape and all(n == 1 or sa == sb for n, sa, sb in zip(a.shape, a.stride(), b.stride()))


class FusedClipAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_grad_norm=None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        if max_grad_norm is not None and len(self.param_groups) > 1:
            raise ValueError("FusedClipAdam: clipping spans one parameter group")
        self.max_grad_norm = max_grad_norm
        self.last_grad_norm = None
        self._plans = {}

    def _plan(self, ps, dev):
        """Device descriptor array of (p, g, exp_avg, exp_avg_sq).  Parameters
        and moments are fixed; gradients may move between steps (zero_grad
        set_to_none), so a changed list is re-uploaded from a pinned buffer
        with an asynchronous copy (no host stall)."""
        # the descriptors hold raw pointers of p AND of its moments: key on
        # both, so replaced state tensors (load_state_dict) get a new plan
        pkey = tuple((p.data_ptr(), self.state[p]["exp_avg"].data_ptr(), self.state[p]["exp_avg_sq"].data_ptr())
                     for p in ps)
        gkey = tuple(p.grad.data_ptr() for p in ps)
        plan = self._plans.get(pkey)
        lib = L.lib()
        if plan is None:
            ts = (L.AdamTensor * len(ps))()
            c0 = 0
            for i, p in enumerate(ps):
                st = self.state[p]
                ts[i].p = p.data_ptr()
                ts[i].m, ts[i].v = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
                ts[i].n, ts[i].chunk0 = p.numel(), c0
                c0 += lib.mtts_adam_chunks(p.numel())
            nbytes = len(bytes(ts))
            plan = {"ts": ts, "nch": c0, "gkey": None, "uploads": 0,
                    "host": torch.empty(nbytes, dtype=torch.uint8, pin_memory=True),
                    "cap_host": torch.empty(nbytes, dtype=torch.uint8, pin_memory=True),
                    "dev": torch.empty(nbytes, dtype=torch.uint8, device=dev),
                    "ws": torch.empty(lib.mtts_adam_workspace(c0), device=dev, dtype=torch.uint8),
                    "norm": torch.zeros(4, device=dev, dtype=torch.float32), "ev": torch.cuda.Event()}
            if len(self._plans) > 8:
                self._plans.clear()
            self._plans[pkey] = plan
        if torch.cuda.is_current_stream_capturing():
            # hipGraph capture: the gradients live in the graph's pool at fixed
            # addresses; the descriptors go into a pinned buffer reserved for
            # the capture (allocated before it; nothing rewrites it later), and
            # its upload is a captured copy
            if plan.get("captured"):
                raise RuntimeError("FusedClipAdam: one captured graph per parameter list")
            ts = plan["ts"]
            for i, p in enumerate(ps):
                ts[i].g = p.grad.data_ptr()
            plan["cap_host"].numpy()[:] = memoryview(bytes(ts))
            dev_buf = torch.empty(plan["cap_host"].numel(), dtype=torch.uint8, device=dev)
            dev_buf.copy_(plan["cap_host"], non_blocking=True)
            plan["captured"] = dev_buf
            return dev_buf, plan["nch"], plan["ws"], plan["norm"]
        if plan["gkey"] != gkey:
            ts = plan["ts"]
            for i, p in enumerate(ps):
                ts[i].g = p.grad.data_ptr()
            plan["ev"].synchronize()          # the previous upload has left the pinned buffer
            plan["host"].numpy()[:] = memoryview(bytes(ts))
            plan["dev"].copy_(plan["host"], non_blocking=True)
            plan["ev"].record()
            plan["gkey"] = gkey
            plan["uploads"] += 1
        return plan["dev"], plan["nch"], plan["ws"], plan["norm"]

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        capturing = torch.cuda.is_current_stream_capturing()
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            for p in ps:
                if p.dtype != torch.float32 or not p.is_cuda or p.grad.dtype != torch.float32:
                    raise TypeError("FusedClipAdam takes fp32 CUDA (HIP) parameters and gradients")
                # the kernel walks storage order: p, grad and moments need one
                # dense layout (contiguous, or e.g. a conv weight kept [O][K][C])
                if p.grad.is_sparse or not dense(p) or not same_layout(p.grad, p):
                    raise ValueError("FusedClipAdam needs dense parameters and gradients of the same strides")
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            steps = {float(self.state[p]["step"]) for p in ps}
            if len(steps) != 1:
                raise ValueError("FusedClipAdam: parameters of a group must share the step count")
            # the step count lives on the device (the kernels derive the bias
            # corrections from it), so a captured hipGraph of the whole training
            # step replays correctly; state["step"] mirrors it on the host in
            # eager mode (sync_steps() after graph replays)
            dstep = group.get("_dstep")
            if dstep is None:
                dstep = torch.full((1,), int(steps.pop()), device=ps[0].device, dtype=torch.int32)
                group["_dstep"] = dstep
            if not capturing:
                for p in ps:
                    self.state[p]["step"] += 1
            raw, nch, ws, norm = self._plan(ps, ps[0].device)
            b1, b2 = group["betas"]
            mx = float(self.max_grad_norm) if self.max_grad_norm is not None else 0.0
            L.call_raw("mtts_clip_adam", raw.data_ptr(), len(ps), nch, dstep.data_ptr(), float(group["lr"]), float(b1),
                       float(b2), float(group["eps"]), float(group["weight_decay"]), mx, ws.data_ptr(), norm.data_ptr())
            self.last_grad_norm = norm[0]
        return loss

    def sync_steps(self):
        """Copy the device step counters into state["step"] (after replays)."""
        for group in self.param_groups:
            dstep = group.get("_dstep")
            if dstep is None:
                continue
            n = float(dstep.item())
            for p in group["params"]:
                if p in self.state and self.state[p]:
                    self.state[p]["step"].fill_(n)

    def state_dict(self):
        sd = super().state_dict()
        for g in sd["param_groups"]:
            g.pop("_dstep", None)
        return sd

    def load_state_dict(self, state_dict):
        """torch.optim.Adam.load_state_dict, then drop every cached descriptor
        plan (they point at the replaced moment tensors) and the device step
        counters (re-seeded from the loaded state["step"] on the next step)."""
        super().load_state_dict(state_dict)
        self._plans = {}
        for g in self.param_groups:
            g.pop("_dstep", None)
        for st in self.state.values():
            # torch's loader may move "step" to the parameter's device; keep it a host scalar as __init__ does
            if "step" in st and torch.is_tensor(st["step"]) and st["step"].device.type != "cpu":
                st["step"] = st["step"].detach().cpu()


@torch.no_grad()
def clip_into_optimizer(optimizer, params, max_norm: float, eps: float = 1e-6):
    """Return the total gradient norm; arm `optimizer` (fused Adam/AdamW) to
    apply clip_grad_norm_'s scaling in its next step()."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return torch.zeros(())
    norms = torch._foreach_norm(grads, 2.0)
    total = torch.linalg.vector_norm(torch.stack([n.float() for n in norms]), 2.0)
    coef = torch.clamp(max_norm / (total + eps), max=1.0)
    scale = getattr(optimizer, "grad_scale", None)
    if scale is None or scale.device != total.device:
        optimizer.grad_scale = torch.empty((), device=total.device, dtype=torch.float32)
    optimizer.grad_scale.copy_(1.0 / coef)
    return total
