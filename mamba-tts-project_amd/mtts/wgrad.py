"""Deferred, grouped weight gradients for the decoder training step.

The reference computes every projection's weight gradient inside its own
backward (nn.Linear / MHA / Mamba in_proj / out_proj, mamba_decoder.py:29-43
applied at :61-88): dW = dy^T x over the B*T token axis.  Those are TN GEMMs
with a small output (1-4 M elements) and a long reduction (16 k tokens at
C2), so run one by one they need split-K (fp32 partial slabs written, read
back and summed by a second launch) to fill the chip.

Here the layer's backward functions only QUEUE (dy, x, parameter, rows) and
return no weight gradient; once the queue holds about one round of 256x256
output tiles (one decoder layer: in_proj, out_proj, q, kv, out, FFN up and
down -- 224 tiles at C2) the jobs run as ONE grouped launch
(`mtts_gemm_grouped`): every tile reduces its problem's whole K in one
workgroup, straight into the fp32 master gradient (no slabs, no reduce pass,
no per-GEMM launch).  The rest of the queue is flushed by a callback at the
end of the backward pass, before `loss.backward()` returns.

The grouped launches can run on a side stream (SIDE_STREAM, off: no gain),
so the next layer's data-gradient kernels fill the CUs the ~224 long tiles
leave idle; the end-of-backward callback makes the caller's stream wait for
it.

Gradient semantics are autograd's: a parameter whose .grad is None gets a
fresh gradient (or its data-parallel bucket view, mtts.dp), one whose .grad
exists is accumulated into (beta = 1).  Listeners (mtts.dp.GradAllReduce)
are told ONCE per backward when a parameter's gradient is complete, so
bucketed all-reduces still overlap the rest of the backward: at the flush
that completes the union of its row slices (a parameter reached by several
row-sliced projections, e.g. CrossAttention's separate q / k / v
in-projections, is complete only when every slice has run), or at the end of
the backward for one whose slices never cover it (the single-key path's
value rows) or overlap (a weight used twice).  A parameter submitted again
after it was announced would reach its all-reduce with a stale gradient:
that raises.

Opt-in per backward pass:  `with mtts.wgrad.deferred(): loss.backward()`
(bench.py and train_harness.py do).  Outside it, or when a shape does not
take the TN route, the immediate path (linear.wgrad) runs as before.  Not for
torch.autograd.grad() on parameters: queued weights receive no gradient
there (the call then fails with "appears to not have been used").
"""
from __future__ import annotations

import contextlib
import ctypes as C

import torch

from . import _lib as L
from . import gemm as G

GROUP_TILES = 192       # flush once the queue holds this many 256x256 output tiles
MAX_PROBLEMS = 24       # mtts_gemm_grouped's problem limit
# a flush with fewer tiles than this leaves most CUs idle for its whole-K
# tiles (C5's d_model 512 layers: ~68 tiles of 640 K-tiles each): its jobs
# run one by one on the split-K TN path instead (tools/c5_once.py trace:
# grouped 5.4 vs split-K 4.0 ms of weight gradients per step at 100 tiles)
MIN_GROUP_TILES = 128
# run the grouped launches on a side stream (the layer's long tiles leave some
# CUs idle for the next layer's data-gradient kernels); the end-of-backward
# callback joins the streams
# Off: no gain (31.8-32.0 ms either way, profiles/r05_c2_ab_side_stream.txt).
# It lets the grouped GEMM's MFMA waves share SIMDs with the next layer's scan
# backward: the overlap that exposed the round-6 packed-f32 hazard there
# (fixed, scan.hip kPackedHazard; profiles/r06_race_bg.txt).  The GPU test
# suite does not run this path.
SIDE_STREAM = False

_depth = 0


class _Job:
    __slots__ = ("dy", "x", "param", "rows")

    def __init__(self, dy, x, param, rows):
        self.dy, self.x, self.param, self.rows = dy, x, param, rows

    def tiles(self):
        m, n = self.dy.shape[1], self.x.shape[1]
        return -(-m // G.TILE) * -(-n // G.TILE)


class _Engine:
    def __init__(self):
        self.jobs = []
        self.tiles = 0
        self.callback_queued = False
        self.done = set()        # ids of params announced complete this backward
        self.covered = {}        # id(param) -> (param, [(r0, r1), ...] rows flushed this backward, overlapped)
        self.listeners = []
        self.side = {}           # device index -> side stream
        self.used_side = None    # (main, side) streams of this backward

    def reset_pass(self):
        self.callback_queued = False
        self.done = set()
        self.covered = {}
        self.used_side = None


_E = _Engine()


def active() -> bool:
    return _depth > 0


@contextlib.contextmanager
def deferred(enable: bool = True):
    """Run the weight gradients of the backward passes inside the block
    through the grouped engine."""
    global _depth
    if not enable:
        yield
        return
    _depth += 1
    try:
        yield
    finally:
        _depth -= 1
        if _depth == 0 and (_E.jobs or _E.used_side is not None):   # a backward that raised midway
            _end_of_backward()


def owns(p) -> bool:
    """True while this backward's engine holds jobs for `p` that it has not
    announced: queued, or flushed for only some of its row slices (e.g. the
    q rows of a cross-attention in_proj_weight before the layers' batched K/V
    rows).  A listener must then wait for the announcement, even if autograd's
    post-accumulate hook already sees a partial p.grad."""
    if id(p) in _E.done:
        return False
    return id(p) in _E.covered or any(j.param is p for j in _E.jobs)


def add_listener(fn):
    """fn(param) is called once per backward when param.grad is complete."""
    _E.listeners.append(fn)


def remove_listener(fn):
    if fn in _E.listeners:
        _E.listeners.remove(fn)


def _eligible(dy, x, param, narrow=False):
    return (active() and param is not None and param.requires_grad and param.dtype == torch.float32
            and param.dim() == 2 and (narrow or (dy.shape[1] >= 256 and x.shape[1] >= 256)) and G.tn_ok(dy, x))


def _end_of_backward():
    flush()
    if _E.used_side is not None:   # gradients complete before anything after the backward
        main, side = _E.used_side
        main.wait_stream(side)
    # parameters whose flushed slices never covered them or overlapped
    for key, (p, _, _) in list(_E.covered.items()):
        if key not in _E.done:
            _announce(p)
    _E.reset_pass()


def _announce(p):
    _E.done.add(id(p))
    for fn in _E.listeners:
        fn(p)


def _cover(p, rows):
    """Record rows (r0, r1) of p as flushed; True once their union is all of p
    and no two slices overlapped."""
    r0, r1 = rows if rows is not None else (0, p.shape[0])
    _, ivs, overlap = _E.covered.get(id(p), (p, [], False))
    overlap = overlap or any(a < r1 and r0 < b for a, b in ivs)
    ivs = ivs + [(r0, r1)]
    _E.covered[id(p)] = (p, ivs, overlap)
    if overlap:
        return False
    return sum(b - a for a, b in ivs) >= p.shape[0]


def _side_stream(dev):
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    st = _E.side.get(i)
    if st is None:
        st = _E.side[i] = torch.cuda.Stream(device=i)
    return st


def submit(jobs, narrow=False) -> bool:
    """Queue [(dy (K, m) bf16, x (K, n) bf16, param, rows (r0, r1) | None), ...]
    -- the weight gradient(s) of ONE parameter, dW[rows] = dy^T x -- when the
    engine is active and every job takes the TN route; returns False (nothing
    queued) otherwise, and the caller computes them immediately.  `narrow`:
    also when a side is below 256 (Mamba's x_proj / dt_proj: a few mostly
    empty tiles that ride in CUs the layer's long tiles leave idle)."""
    if not jobs or not all(_eligible(dy, x, p, narrow) for dy, x, p, _ in jobs):
        return False
    param = jobs[0][2]
    for dy, x, p, rows in jobs:
        r0, r1 = rows if rows is not None else (0, p.shape[0])
        if p is not param or p.shape[1] != x.shape[1] or r1 - r0 != dy.shape[1]:
            return False
    if id(param) in _E.done and _E.listeners:
        raise RuntimeError("wgrad: a parameter's weight gradient was submitted after its gradient was announced "
                           "complete to a listener (a weight used again later in the backward under GradAllReduce); "
                           "run this backward outside mtts.wgrad.deferred()")
    if any(j.param is param for j in _E.jobs):   # e.g. a weight shared by two modules: keep the order
        flush()
    if not _E.callback_queued:
        torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
        _E.callback_queued = True
    for dy, x, p, rows in jobs:
        j = _Job(dy, x, p, rows)
        _E.jobs.append(j)
        _E.tiles += j.tiles()
    if _E.tiles >= GROUP_TILES or len(_E.jobs) >= MAX_PROBLEMS - 2:
        flush()
    return True


def flush():
    """Run every queued weight gradient (grouped launches) and publish the
    completed parameters' gradients."""
    jobs, _E.jobs, _E.tiles = _E.jobs, [], 0
    if not jobs:
        return
    if not (SIDE_STREAM and _E.callback_queued):
        _flush(jobs)
        return
    main = torch.cuda.current_stream()
    side = _side_stream(jobs[0].dy.device)
    side.wait_stream(main)          # the layer's dy / x are complete
    _E.used_side = (main, side)
    for j in jobs:                  # the caching allocator must not reuse them before the side stream is done
        j.dy.record_stream(side)
        j.x.record_stream(side)
    with torch.cuda.stream(side):
        _flush(jobs, side)


def _flush(jobs, side=None):
    # destinations: accumulate into an existing .grad; else the data-parallel
    # bucket view (mtts.dp) or a fresh tensor (zeroed when this flush does not
    # cover all of its rows)
    dest = {}
    for j in jobs:
        p = j.param
        if id(p) in dest:
            continue
        if p.grad is not None:
            dest[id(p)] = (p.grad, 1.0, False)
            continue
        cover = sum((j2.rows[1] - j2.rows[0]) if j2.rows else p.shape[0] for j2 in jobs if j2.param is p)
        view = getattr(p, "_mtts_grad_view", None)
        full = cover >= p.shape[0]
        if view is not None:
            if not full:
                view.zero_()
            g = view
        else:
            g = torch.empty(p.shape, device=p.device, dtype=torch.float32) if full else \
                torch.zeros(p.shape, device=p.device, dtype=torch.float32)
        if side is not None:
            g.record_stream(side)
        dest[id(p)] = (g, 0.0 if full else 1.0, True)
    probs, fixups = [], []
    for j in jobs:
        g, beta, _ = dest[id(j.param)]
        out = g if j.rows is None else g[j.rows[0]:j.rows[1]]
        if not _addressable(out):   # e.g. a view at an odd offset of a caller's flat buffer
            tmp = torch.empty(out.shape, device=out.device, dtype=torch.float32)
            if side is not None:
                tmp.record_stream(side)
            fixups.append((out, tmp, beta))
            out, beta = tmp, 0.0
        probs.append((j.dy, j.x, out, beta))
    probs.sort(key=lambda t: -t[0].shape[0])   # longest reduction first (tail balance)
    if sum(-(-dy.shape[1] // G.TILE) * -(-x.shape[1] // G.TILE) for dy, x, _, _ in probs) < MIN_GROUP_TILES:
        for dy, x, out, beta in probs:
            G.mm_tn(dy, x, out=out, beta=beta)
    else:
        for s in range(0, len(probs), MAX_PROBLEMS):
            _launch(probs[s:s + MAX_PROBLEMS])
    for out, tmp, beta in fixups:
        if beta:
            out.add_(tmp)
        else:
            out.copy_(tmp)
    for j in jobs:
        g, _, fresh = dest[id(j.param)]
        if fresh and j.param.grad is None:
            j.param.grad = g
    complete = {}
    for j in jobs:
        if _cover(j.param, j.rows) and id(j.param) not in _E.done:
            complete[id(j.param)] = j.param
    for p in complete.values():
        _announce(p)


def _addressable(out):
    return out.stride(1) == 1 and out.stride(0) % 4 == 0 and out.data_ptr() % 16 == 0


def _launch(probs):
    arr = (L.GemmArgs * len(probs))()
    for a, (dy, x, out, beta) in zip(arr, probs):
        k, m = dy.shape
        n = x.shape[1]
        if not _addressable(out) or tuple(out.shape) != (m, n):
            raise RuntimeError("wgrad: gradient destination not 16-byte addressable")
        a.m, a.n, a.k, a.layout, a.splits, a.out_dtype = m, n, k, G.TN, 1, 0
        a.lda, a.ldb, a.ldc = dy.stride(0), x.stride(0), out.stride(0)
        a.a, a.b, a.c = dy.data_ptr(), x.data_ptr(), out.data_ptr()
        a.beta = beta
    lib = L.lib()
    rc = lib.mtts_gemm_grouped(arr, len(probs), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError(f"mtts_gemm_grouped failed ({rc}): {lib.mtts_last_error().decode()}")
