"""World-2 gloo data parallelism + deferred weight gradients on one GPU:
how often does a pass's averaged gradient differ from the first pass of the
same mode?  MODE = imm | dfr | mid (mid: GROUP_TILES 1, every submit flushed
inside its parameter's backward); SYNC = before | after | both (device
synchronize around every deferred flush); LATE = 1: every bucket all-reduced
in finish().  Prints one line per rank."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd"), os.path.join(ROOT, "tests")]
import torch
import torch.multiprocessing as mp


def worker(rank, port, world):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd"), os.path.join(ROOT, "tests")]
    import faulthandler
    faulthandler.dump_traceback_later(150, exit=True)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    nodp = os.environ.get("NODP") == "1"
    if not nodp:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    import test_gpu_wgrad as T
    from mtts import wgrad
    from mtts.dp import GradAllReduce
    mode = os.environ.get("MODE", "mid")
    sync = os.environ.get("SYNC", "")
    wgrad.MIN_GROUP_TILES = 0
    wgrad.GROUP_TILES = 1 if mode == "mid" else 192
    m = T._model()
    dp = None if nodp else GradAllReduce(list(m.parameters()), bucket_mb=1.0)
    # trace: every module output (forward) and its gradient (backward), in order
    trace = []

    def fwd_hook(mod, inp, out, name=None):
        outs = out if isinstance(out, (tuple, list)) else (out,)
        for i, o in enumerate(outs):
            if torch.is_tensor(o) and o.is_floating_point():
                trace.append((f"fwd {name}[{i}]", o.detach().clone()))
                if o.requires_grad:
                    o.register_hook(lambda g, nm=f"grad {name}[{i}]": trace.append((nm, g.detach().clone())))
    for nm, mod in m.named_modules():
        if nm:
            mod.register_forward_hook(lambda mod, i, o, nm=nm: fwd_hook(mod, i, o, nm))
    if sync and dp is not None:
        real_flush = wgrad._flush

        def _flush(jobs, side=None):
            if sync in ("before", "both"):
                torch.cuda.synchronize()
            real_flush(jobs, side)
            if sync in ("after", "both"):
                torch.cuda.synchronize()
        wgrad._flush = _flush
    if os.environ.get("SYNC_LAUNCH") == "1" and dp is not None:   # device idle before every collective
        _launch0 = dp._launch

        def _launch_sync(b):
            torch.cuda.synchronize()
            _launch0(b)
        dp._launch = _launch_sync
    if os.environ.get("HOST_STAGE") == "1" and dp is not None:   # gloo on a synchronous host copy of the bucket
        import torch.distributed as dist

        class _H:
            def __init__(self, dev_buf):
                self.dev, self.host = dev_buf, dev_buf.to("cpu")
                self.work = dist.all_reduce(self.host, async_op=True)

            def wait(self):
                self.work.wait()
                self.dev.copy_(self.host)

        def _launch_host(b):
            dp._order = getattr(dp, "_order", []) + [b]
            s0, e0, _ = dp.buckets[b]
            dp.handles[b] = _H(dp.flat[s0:e0])
        dp._avg = False
        dp._launch = _launch_host
    if os.environ.get("LATE") == "1" and dp is not None:
        launch_now = dp._launch
        dp._launch = lambda b: None
        real_finish = dp.finish

        def finish():
            for b in range(len(dp.buckets)):
                if dp.handles[b] is None:
                    launch_now(b)
            real_finish()
        dp.finish = finish
    tok, text, z, mask = T._batch(2 * T.B)
    sl = slice(rank * T.B, (rank + 1) * T.B)
    n = int(os.environ.get("N", "8"))
    first, nbad, worst = None, 0, ""
    first_trace = None
    for i in range(n + 1):
        trace.clear()
        if dp is not None:
            dp.zero_grad()
        else:
            m.zero_grad(set_to_none=True)
        snaps, calls = {}, {}
        if dp is not None and os.environ.get("SNAP") == "1":
            names = {id(p): nm for nm, p in m.named_parameters()}
            hk = dp._hook

            def _snap_hook(p, *a, **k):
                nm = names[id(p)]
                calls[nm] = calls.get(nm, 0) + 1
                hk(p, *a, **k)
                if p.grad is not None:
                    snaps[nm] = p.grad.detach().clone()
            dp._hook = _snap_hook
            if not hasattr(dp, "_snap_hooks"):
                for h in dp.hooks:
                    h.remove()
                dp.hooks = [p.register_post_accumulate_grad_hook(lambda p: dp._hook(p)) for p in dp.params]
                dp._snap_hooks = True
        with wgrad.deferred(mode != "imm"):
            T._loss(m, tok[sl], text[sl], z[sl], mask[sl]).backward()
        if snaps:
            torch.cuda.synchronize()
            dp._hook = hk
            multi = {k: v for k, v in calls.items() if v != 1}
            changed = [nm for nm, p in m.named_parameters() if nm in snaps and not torch.equal(snaps[nm], dp.views[p])]
            missing = [nm for nm, _ in m.named_parameters() if nm not in snaps]
            if i == 0 or not hasattr(dp, "_snap0"):
                dp._snap0 = snaps
            else:
                loc = [k for k in snaps if not torch.equal(snaps[k], dp._snap0[k])]
                if loc:
                    print(f"[rank {rank}] pass {i}: LOCAL grads differ from pass 0: {loc[:6]}", flush=True)
            if multi or changed or missing:
                print(f"[rank {rank}] pass {i}: hooks != 1: {multi}; grad changed after its hook: {changed}; "
                      f"no hook: {missing}", flush=True)
        if dp is not None:
            dp.finish()
            if hasattr(dp, "_order"):
                dp._order = []
        torch.cuda.synchronize()
        g = {nm: p.grad.detach().clone() for nm, p in m.named_parameters()}
        if first is None:
            first = g
            first_trace = list(trace)
            continue
        for (na, a), (nb, b) in zip(first_trace, trace):
            if na != nb or not torch.equal(a, b):
                print(f"[rank {rank}] pass {i}: first differing traced tensor: {na} "
                      f"(max abs diff {(a.float() - b.float()).abs().max().item():.2e})", flush=True)
                break
        errs = sorted((((g[k] - first[k]).abs().max() / first[k].abs().max().clamp_min(1e-12)).item(), k) for k in g)
        if errs[-1][0] > 0:
            nbad += 1
            worst = f"{errs[-1][1]} {errs[-1][0]:.1e}"
    print(f"[rank {rank}] MODE={mode} SYNC={sync or '-'} LATE={os.environ.get('LATE', '0')}: "
          f"{nbad} of {n} passes differ from the first ({worst})", flush=True)
    if not nodp:
        dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(worker, args=(port, 2), nprocs=2)
