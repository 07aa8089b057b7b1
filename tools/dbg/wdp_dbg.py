import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd"), os.path.join(ROOT, "tests")]
import torch
import torch.multiprocessing as mp


def worker(rank, port, world):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mamba-tts-project_amd"), os.path.join(ROOT, "tests")]
    import faulthandler
    faulthandler.dump_traceback_later(100, exit=True)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import test_gpu_wgrad as T
    from mtts import wgrad
    from mtts.dp import GradAllReduce
    wgrad.MIN_GROUP_TILES = int(os.environ.get("MIN_GROUP_TILES", "128"))
    m = T._model()
    use_dp = os.environ.get("NODP") != "1"
    dp = GradAllReduce(list(m.parameters()), bucket_mb=1.0) if use_dp else None
    if os.environ.get("SYNC_FLUSH") == "1":   # every deferred flush completes on the device before anything else
        real_flush = wgrad._flush
        def _flush(jobs, side=None):
            torch.cuda.synchronize()
            real_flush(jobs, side)
            torch.cuda.synchronize()
        wgrad._flush = _flush
    if dp is not None:
        dp._order = []
        _real_launch = dp._launch
        def _logged_launch(b):
            if wgrad.GROUP_TILES == 1:
                dp._order.append(b)
            _real_launch(b)
        dp._launch = _logged_launch
    if dp is not None and os.environ.get("LATE_LAUNCH") == "1":   # every bucket all-reduced in finish()
        dp._launch_now = dp._launch
        dp._launch = lambda b: None
        real_finish = dp.finish
        def finish():
            for b in range(len(dp.buckets)):
                dp._launch_now(b)
            dp._launch = dp._launch_now
            real_finish()
            dp._launch = lambda b: None
        dp.finish = finish
    tok, text, z, mask = T._batch(2 * T.B)
    sl = slice(rank * T.B, (rank + 1) * T.B)
    runs = {}
    import mtts.dp as DPM
    DPM.DEFER_LISTENER_LAUNCH = os.environ.get("DEFER", "1") == "1"
    nmid = int(os.environ.get("NMID", "1"))
    tags = [("imm1", False), ("imm2", False), ("dfr1", True), ("dfr2", True)] + [(f"mid{i + 1}", True) for i in range(nmid)]
    for tag, defer in tags:
        wgrad.GROUP_TILES = 1 if tag.startswith("mid") else 192
        if dp: dp.zero_grad()
        else: m.zero_grad(set_to_none=True)
        with wgrad.deferred(defer):
            T._loss(m, tok[sl], text[sl], z[sl], mask[sl]).backward()
        if dp: dp.finish()
        torch.cuda.synchronize()
        runs[tag] = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    for a, b in (("imm1", "imm2"), ("dfr1", "dfr2"), ("imm1", "dfr1"), ("dfr1", "mid1"), ("imm1", "mid1")):
        worst = sorted(((((runs[a][n] - runs[b][n]).abs().max() / runs[b][n].abs().max().clamp_min(1e-12)).item(), n)
                        for n in runs[a]), reverse=True)[:4]
        print(f"[rank {rank} dp={use_dp}] {a} vs {b}: " + ", ".join(f"{n} {e:.2e}" for e, n in worst), flush=True)
    if dp is not None and rank == 0:
        nbad = 0
        for i in range(nmid):
            errs = [((runs[f"mid{i + 1}"][n] - runs["dfr1"][n]).abs().max() / runs["dfr1"][n].abs().max().clamp_min(1e-12)).item()
                    for n in runs["dfr1"]]
            nbad += max(errs) > 1e-6
        print(f"DEFER={DPM.DEFER_LISTENER_LAUNCH}: {nbad} of {nmid} mid-flush passes differ from dfr1", flush=True)
        bad = [(n, dp.bucket_of[p], ((runs["mid1"][n] - runs["dfr1"][n]).abs().max() /
                                     runs["dfr1"][n].abs().max().clamp_min(1e-12)).item())
               for n, p in m.named_parameters()]
        print("mid1 vs dfr1 per param (bucket, rel err):", [(n, b, f"{e:.1e}") for n, b, e in bad if e > 1e-6])
        print("launch order:", getattr(dp, "_order", None))
    dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    world = int(os.environ.get("WORLD", "2"))
    mp.spawn(worker, args=(port, world), nprocs=world)
