"""World-2 gloo DP + deferred weight gradients with every submit flushed at
once (GROUP_TILES 1): log every bucket launch and every gradient write
(deferred flush / autograd hook) and report writes into already-launched
buckets (the race behind a mid-backward-flush DP mismatch)."""
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
    from mtts import dp as DPM
    wgrad.MIN_GROUP_TILES = 0
    wgrad.GROUP_TILES = 1
    m = T._model()
    names = {id(p): n for n, p in m.named_parameters()}
    dp = DPM.GradAllReduce(list(m.parameters()), bucket_mb=1.0)
    launched = set()
    log = []
    real_launch = dp._launch

    def launch(b):
        launched.add(b)
        log.append(("launch", b))
        real_launch(b)
    dp._launch = launch
    real_flush = wgrad._flush

    def flush(jobs, side=None):
        for j in jobs:
            b = dp.bucket_of.get(j.param)
            log.append(("flush", names[id(j.param)], b))
            if j.param.grad is not None:
                print(f"[rank {rank}] flush accumulates into existing grad of {names[id(j.param)]}", flush=True)
            if b in launched:
                print(f"[rank {rank}] RACE: flush writes {names[id(j.param)]} into launched bucket {b}", flush=True)
        real_flush(jobs, side)
    wgrad._flush = flush
    real_hook = dp._hook

    def hook(p):
        b = dp.bucket_of[p]
        if p.grad is not None and b in launched and id(p) not in dp.counted:
            print(f"[rank {rank}] RACE: hook of {names[id(p)]} after its bucket {b} launched", flush=True)
        real_hook(p)
    dp._hook = hook
    for h in dp.hooks:
        h.remove()
    dp.hooks = [p.register_post_accumulate_grad_hook(hook) for p in dp.params]
    wgrad.remove_listener(dp._deferred_ready)
    wgrad.add_listener(lambda p: hook(p) if p in dp.views else None)
    tok, text, z, mask = T._batch(2 * T.B)
    sl = slice(rank * T.B, (rank + 1) * T.B)
    dp.zero_grad()
    with wgrad.deferred(True):
        T._loss(m, tok[sl], text[sl], z[sl], mask[sl]).backward()
    dp.finish()
    torch.cuda.synchronize()
    if rank == 0:
        print("buckets:", [(i, b[2]) for i, b in enumerate(dp.buckets)])
        for b in range(len(dp.buckets)):
            print(b, sorted(names[id(p)] for p, bb in dp.bucket_of.items() if bb == b))
        print(log)
    dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(worker, args=(port, 2), nprocs=2)
