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
    m = T._model()
    use_dp = os.environ.get("NODP") != "1"
    dp = GradAllReduce(list(m.parameters()), bucket_mb=1.0) if use_dp else None
    tok, text, z, mask = T._batch(2 * T.B)
    sl = slice(rank * T.B, (rank + 1) * T.B)
    runs = {}
    for tag, defer in (("imm1", False), ("imm2", False), ("dfr1", True), ("dfr2", True)):
        if dp: dp.zero_grad()
        else: m.zero_grad(set_to_none=True)
        with wgrad.deferred(defer):
            T._loss(m, tok[sl], text[sl], z[sl], mask[sl]).backward()
        if dp: dp.finish()
        torch.cuda.synchronize()
        runs[tag] = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    for a, b in (("imm1", "imm2"), ("dfr1", "dfr2"), ("imm1", "dfr1")):
        worst = sorted(((((runs[a][n] - runs[b][n]).abs().max() / runs[b][n].abs().max().clamp_min(1e-12)).item(), n)
                        for n in runs[a]), reverse=True)[:4]
        print(f"[rank {rank} dp={use_dp}] {a} vs {b}: " + ", ".join(f"{n} {e:.2e}" for e, n in worst), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    world = int(os.environ.get("WORLD", "2"))
    mp.spawn(worker, args=(port, world), nprocs=world)
