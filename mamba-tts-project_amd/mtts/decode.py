"""Incremental decoding engine for MambaTTSDecoder.decode_step (C4).

Reference: mamba_decoder.py:188-256.  Each AR step embeds one token (no
quant_embed, pos = step_index), runs every layer with its Mamba state and
cross-attends to [ref ‖ text].  The reference recomputes, every step, the
K/V projections of the (constant) conditioning sequence and the FiLM
gamma/beta of the (constant) style vector; the engine computes them once per
conditioning context and keeps them in HBM with the per-layer SSM/conv state.

Engine path (inference only: torch.no_grad, HIP tensors):
  * context cache keyed on the object identity (strong references are
    held, so addresses cannot be recycled) and autograd version of
    text_hidden, text_mask, ref_hidden, ref_mask, z_style, plus the compute
    dtype and batch shape;
  * per step: token+pos embedding, then per layer LN -> Mamba.step (HIP
    conv-window + state-update kernels, states updated in place) -> fused
    residual+LN -> q-projection + attention over cached K/V -> fused
    residual+LN+FiLM -> FFN; the FFN residual is fused into the next LN;
  * the <= 32-row projections (in/x/dt/out_proj, q/out_proj, FFN, head) on
    the HIP skinny GEMM of csrc/rows.hip (bias + GELU fused) for bf16;
  * dt_proj fused into the selective state update (B / C read in place);
  * optional hipGraph capture of the whole step (static token / position /
    state buffers): replay costs one launch instead of ~25 per layer.
Numerics are those of the eager module path (tests/test_gpu_modules.py).
Call `reset()` after modifying weights in place between decode steps.
"""
from __future__ import annotations


import torch
import torch.nn.functional as F

from . import _lib as L
from . import ops
from .embed import _err_flag
from .attn_kernels import attention, attention_decode_packed, attention_decode_qproj_packed
from .linear import cast_weight


def _same_ctx(refs, versions, tensors):
    """True when `tensors` are the very objects cached in `refs` (identity,
    not address: the engine holds strong references, so a freed tensor's
    address can never be reused for a new one while the cache is alive)
    and none was modified in place since (autograd version counter)."""
    if refs is None or len(refs) != len(tensors):
        return False
    for r, v, t in zip(refs, versions, tensors):
        if r is not t:
            return False
        if t is not None and t._version != v:
            return False
    return True


def _proj_blas(x, w, b=None, act=None):
    y = x @ w.t() if b is None else torch.addmm(b, x, w.t())
    return F.gelu(y) if act == "gelu" else y


def _proj_rows(x, w, b=None, act=None):
    """HIP skinny GEMM (csrc/rows.hip) for the <= 32-row decode projections."""
    if ops.gemm_rows_ok(x, w):
        return ops.gemm_rows(x, w, b, act)
    return _proj_blas(x, w, b, act)


class DecodeEngine:
    # routing switches for in-process A/B timing (tools/decode_ab.py); the
    # defaults are the measured-fastest path (DESIGN.md §4 decode)
    OPTIONS = {"rows": True,       # HIP row-GEMMs (csrc/rows.hip / gemv.hip) instead of hipBLASLt
               "fused": True,      # fused-epilogue step (LN prologues, residual / conv epilogues)
               "fuse_conv": True,  # conv update in in_proj's epilogue
               "packed": True,     # weights re-laid in MFMA fragment order (gemv16)
               "xpacked": True,    # activation images packed too
               # cross-attention LN + q projection inside the decode attention kernel
               # (mtts_attention_decode_qproj): measured 1.13 vs 0.76 ms p50 per
               # step (profiles/r05_decode_ab_fuse_q.txt) -- every (batch, head)
               # workgroup re-reads its head's Wq rows (256 KiB) from L2, 64 MiB
               # per layer against 2 MiB for one projection over the 32 rows
               "fuse_q": False}

    def __init__(self, model, use_graph=True, use_rows=True):
        self.m = model
        self.use_graph = use_graph
        self.use_rows = use_rows and self.OPTIONS["rows"]
        self.reset()

    def reset(self):
        # a flag left by the previous session must not surface in the next one,
        # and must not be lost either (nn.Embedding raises on every such step,
        # mamba_decoder.py:217): wait for its copy, clear host and device
        # flags, reset the engine, then raise it
        flagged = False
        if getattr(self, "_err_ev", None) is not None:
            self._err_ev.synchronize()
            flagged = int(self._err_host[0]) != 0
            self._err_host.zero_()
            _err_flag(self._err_dev).zero_()
        self._err_host = None
        self._err_ev = None
        self._err_dev = None
        self.xpk = False
        self.fuse_q = False
        self.ctx_key = None
        self.ctx_refs = None
        self.ctx_versions = None
        self.ctx = None
        self.graph = None
        self.states = None
        if flagged:
            raise IndexError("decode_step: last_token id out of range of token_embed (index out of range in self)")

    # -- conditioning context -------------------------------------------------
    def _build_ctx(self, text_hidden, z_style, text_mask, ref_hidden, ref_mask, cd):
        m = self.m
        B = text_hidden.shape[0]
        th = text_hidden.to(cd)
        th, tm = m._concat_ref(th, text_mask, ref_hidden, ref_mask, B, th.device)
        kpm = None if tm is None else ~tm                                   # mamba_decoder.py:68-70
        d = m.token_embed.weight.shape[1]
        layers = []
        for l in m.layers:
            ca = l.cross_attn
            W = cast_weight(ca.in_proj_weight, cd)
            b = cast_weight(ca.in_proj_bias, cd)
            kv = torch.addmm(b[d:], th.reshape(-1, d), W[d:].t()).view(B, -1, 2 * d)
            gb = torch.tanh(F.linear(z_style.to(l.style_mlp[0].weight.dtype), l.style_mlp[0].weight,
                                     l.style_mlp[0].bias)).to(cd)
            gamma, beta = gb[:, :d].contiguous(), gb[:, d:].contiguous()
            mm = l.mamba
            di = mm.d_inner
            layers.append(dict(
                k=kv[..., :d], v=kv[..., d:], gamma=gamma, beta=beta,
                Wq=W[:d], bq=b[:d], Wo=cast_weight(ca.out_proj.weight, cd), bo=cast_weight(ca.out_proj.bias, cd),
                W1=cast_weight(l.ff[0].weight, cd), b1=cast_weight(l.ff[0].bias, cd),
                W2=cast_weight(l.ff[2].weight, cd), b2=cast_weight(l.ff[2].bias, cd),
                Win=cast_weight(mm.in_proj.weight, cd), Wx=cast_weight(mm.x_proj.weight, cd),
                Wdt=cast_weight(mm.dt_proj.weight, cd), Wout=cast_weight(mm.out_proj.weight, cd),
                conv_w=mm.conv1d.weight.detach().reshape(di, -1).float().contiguous(),
                conv_b=mm.conv1d.bias.detach().float().contiguous(),
                A=(-torch.exp(mm.A_log.detach().float())).contiguous(), D=mm.D.detach().float().contiguous(),
                dt_bias=mm.dt_proj.bias.detach().float().contiguous(),
            ))
        dev = text_hidden.device
        return dict(B=B, kpm=kpm, layers=layers, cd=cd,
                    tok_w=m.token_embed.weight.detach().float().contiguous(),
                    pos_w=m.pos_embed.weight.detach().float().contiguous(),
                    q0_w=torch.zeros(1, d, device=dev), q0_id=torch.zeros(1, device=dev, dtype=torch.int32),
                    Wh=cast_weight(m.head.weight, cd), bh=cast_weight(m.head.bias, cd))

    def _fused_ok(self, cd, B):
        """The fused-epilogue step (_step_rows) applies: bf16, <= 32 rows and
        the shapes csrc/rows.hip takes (checked once per context)."""
        m = self.m
        if (not self.use_rows or cd != torch.bfloat16 or B > ops.GEMM_ROWS_MAX
                or not self.OPTIONS["fused"]):
            return False
        d = m.token_embed.weight.shape[1]
        if not ops.gemm_rows_ln_ok(d):
            return False
        for l in m.layers:
            mm = l.mamba
            if (mm.d_conv != 4 or d % 64 or mm.d_inner % 64 or d % 8 or d > 2048 or l.ff[0].weight.shape[0] % 64
                    or any(n.weight.dtype != torch.float32 for n in (l.norm_mamba, l.norm_cross, l.norm_ff))):
                return False
        return m.norm_out.weight.dtype == torch.float32

    def _embed(self, tok):
        """token_embed(last_token) + pos_embed(step_index) in the compute dtype
        (mamba_decoder.py:188-256; no quant_embed in decode_step) as ONE
        mtts_embed_sum launch (a zero quantizer row, the step's position id
        from the int32 buffer pos32) instead of two gathers, an add and a
        cast."""
        m, c = self.m, self.ctx
        B = c["B"]
        d = m.token_embed.weight.shape[1]
        out = torch.empty(B, d, device=tok.device, dtype=c["cd"])
        tw, pw = c["tok_w"], c["pos_w"]
        L.call_raw("mtts_embed_sum", tok.data_ptr(), tok.stride(0), c["q0_id"].data_ptr(), self.pos32.data_ptr(),
                   tw.data_ptr(), c["q0_w"].data_ptr(), pw.data_ptr(), B, 1, d, tw.shape[0], out.data_ptr(),
                   L.dtype_code(out), out.stride(0), _err_flag(tok.device).data_ptr())
        return out

    _PACKED = ("Win", "Wx", "Wout", "Wq", "Wo", "W1", "W2")

    def _pack_ctx(self):
        """Packed (MFMA-fragment order) images of the step's projection
        weights for csrc/gemv.hip, made once per context; shapes the packed
        kernel does not take keep the row-major weight."""
        c = self.ctx
        for p in c["layers"]:
            for k in self._PACKED:
                if ops.gemv_split_ok(p[k].shape[1], ln=k in ("Win", "Wq", "W1")):
                    p[k + "_p"] = ops.pack_rows_weight(p[k])
        if ops.gemv_split_ok(c["Wh"].shape[1], ln=True):
            c["Wh_p"] = ops.pack_rows_weight(c["Wh"])

    # -- one step, fused epilogues (bf16, <= 32 sequences) ---------------------
    def _step_rows(self, tok, pos, states):
        """Per layer, 9 launches and no LayerNorm kernel (csrc/rows.hip):
        in_proj (LN prologue, conv-update + SiLU epilogue) -> x_proj ->
        state update (+dt_proj) -> out_proj (+residual) -> q (LN prologue)
        -> attention -> out_proj (+residual) -> FFN up (LN + FiLM prologue,
        GELU) -> FFN down (+residual); the head LayerNorms in its prologue.
        x is the bf16 residual stream, exactly as the LayerNorm kernels'
        x_sum of the generic step."""
        m, c = self.m, self.ctx
        cd = c["cd"]
        x = self._embed(tok)

        def ln(norm, gamma=None, beta=None):
            return (norm.weight, norm.bias, norm.eps, gamma, beta)

        def w(p, k):   # packed image when there is one (csrc/gemv.hip)
            return p.get(k + "_p", p[k])

        if self.xpk:
            return self._step_xpk(x, states, ln)

        fuse_conv = self.OPTIONS["fuse_conv"]
        for i, (l, p) in enumerate(zip(m.layers, c["layers"])):
            conv_state, ssm_state = states[i]
            mm = l.mamba
            di, N, r = mm.d_inner, mm.d_state, mm.dt_rank
            if fuse_conv:
                xz, u = ops.gemm_rows(x, w(p, "Win"), conv=(conv_state, p["conv_w"], p["conv_b"]),
                                      ln=ln(l.norm_mamba))
            else:
                xz = ops.gemm_rows(x, w(p, "Win"), ln=ln(l.norm_mamba))
                u = ops.conv_update(xz[:, :di], conv_state, p["conv_w"], p["conv_b"], True)
            x_dbl = ops.gemm_rows(u, w(p, "Wx"))
            y = ops.state_update(ssm_state, u, x_dbl[:, :r], p["A"], x_dbl[:, r:r + N], x_dbl[:, r + N:], p["D"],
                                 xz[:, di:], p["dt_bias"], True, dt_w=p["Wdt"])
            x = ops.gemm_rows(y, w(p, "Wout"), res=x)
            q = ops.gemm_rows(x, w(p, "Wq"), p["bq"], ln=ln(l.norm_cross))
            o = attention(q[:, None], p["k"], p["v"], l.cross_attn.num_heads, c["kpm"])[:, 0]
            x = ops.gemm_rows(o, w(p, "Wo"), p["bo"], res=x)
            f = ops.gemm_rows(x, w(p, "W1"), p["b1"], "gelu", ln=ln(l.norm_ff, p["gamma"], p["beta"]))
            x = ops.gemm_rows(f, w(p, "W2"), p["b2"], res=x)
        return ops.gemm_rows(x, w(c, "Wh"), c["bh"], ln=ln(m.norm_out))[:, None]

    def _xpk_ok(self):
        """Every projection packed and every operand shape the packed
        activation images take (K, N % 32; short key side): the step of
        _step_xpk applies."""
        if not self.OPTIONS["xpacked"]:
            return False
        c = self.ctx
        names = self._PACKED
        if not all(k + "_p" in p for p in c["layers"] for k in names) or "Wh_p" not in c:
            return False
        for l, p in zip(self.m.layers, c["layers"]):
            ca = l.cross_attn
            hd = ca.embed_dim // ca.num_heads
            if (any(p[k].shape[0] % 32 or p[k].shape[1] % 32 for k in names)
                    or p["k"].shape[1] > 8 * (256 // (hd // 8)) or l.mamba.d_inner % 32):
                return False
        for l, p in zip(self.m.layers, c["layers"]):   # head-major K / V: one contiguous block per (b, h)
            H = l.cross_attn.num_heads
            Bk, S, d = p["k"].shape
            p["khm"] = p["k"].reshape(Bk, S, H, d // H).permute(0, 2, 1, 3).contiguous()
            p["vhm"] = p["v"].reshape(Bk, S, H, d // H).permute(0, 2, 1, 3).contiguous()
        for p in c["layers"]:   # FiLM rows as packed images (per-context constants)
            if "gamma_p" not in p:
                p["gamma_p"] = ops.PackedAct.pack(p["gamma"])
                p["beta_p"] = ops.PackedAct.pack(p["beta"])
        return True

    def _fuse_q_ok(self, B):
        """Shapes mtts_attention_decode_qproj takes (head_dim 64 / 128,
        d_model <= 2048, <= 32 sequences, the single-pass key range)."""
        for l, p in zip(self.m.layers, self.ctx["layers"]):
            ca = l.cross_attn
            hd = ca.embed_dim // ca.num_heads
            if (hd not in (64, 128) or ca.embed_dim > 2048 or ca.embed_dim % 8 or B > 32
                    or p["khm"].shape[2] > 8 * (256 // (hd // 8)) or p["Wq"].stride(0) != ca.embed_dim):
                return False
        return True

    def _step_xpk(self, x, states, ln):
        """_step_rows with packed activations (csrc/gemv.hip, common.h
        xpk_index): every producer writes the packed image of what the next
        projection reads (residual epilogues the residual stream besides its
        row-major copy, the conv-update u for x_proj, the state-update y for
        out_proj, attention o, FFN-up f) and the FiLM rows are packed once
        per context, so every projection loads its operands as coalesced KiB
        like its weights; the LayerNorm(+FiLM) prologues run on the packed
        rows.  9 launches per layer, as _step_rows."""
        m, c = self.m, self.ctx
        xp = None   # packed image of the residual stream (none before layer 0)
        for i, (l, p) in enumerate(zip(m.layers, c["layers"])):
            conv_state, ssm_state = states[i]
            mm = l.mamba
            di, N, r = mm.d_inner, mm.d_state, mm.dt_rank
            xz, u, up = ops.gemm_rows(x if xp is None else xp, p["Win_p"],
                                      conv=(conv_state, p["conv_w"], p["conv_b"]), ln=ln(l.norm_mamba),
                                      u_packed=True)
            # (x_proj fused into the state update measured slower, 1.10 vs 0.77 ms
            # per step: every workgroup pulls 512 KiB through dependent L2 trips)
            x_dbl = ops.gemm_rows(up, p["Wx_p"])
            y = ops.state_update(ssm_state, u, x_dbl[:, :r], p["A"], x_dbl[:, r:r + N], x_dbl[:, r + N:], p["D"],
                                 xz[:, di:], p["dt_bias"], True, dt_w=p["Wdt"], packed_out=True)
            x, xp = ops.gemm_rows(y, p["Wout_p"], res=x, packed_out="also")
            if self.fuse_q:   # one launch: LN + q projection in the attention kernel's prologue
                nc = l.norm_cross
                o = attention_decode_qproj_packed(x, p["Wq"], p["bq"], nc.weight, nc.bias, nc.eps, p["khm"],
                                                  p["vhm"], l.cross_attn.num_heads, c["kpm"])
            else:
                q = ops.gemm_rows(xp, p["Wq_p"], p["bq"], ln=ln(l.norm_cross))
                o = attention_decode_packed(q, p["khm"], p["vhm"], l.cross_attn.num_heads, c["kpm"])
            x, xp = ops.gemm_rows(o, p["Wo_p"], p["bo"], res=x, packed_out="also")
            f = ops.gemm_rows(xp, p["W1_p"], p["b1"], "gelu", ln=ln(l.norm_ff, p["gamma_p"], p["beta_p"]),
                              packed_out="only")
            x, xp = ops.gemm_rows(f, p["W2_p"], p["b2"], res=x, packed_out="also")
        return ops.gemm_rows(xp, c["Wh_p"], c["bh"], ln=ln(m.norm_out))[:, None]

    # -- one step, eager -----------------------------------------------------
    def _step(self, tok, pos, states):
        m, c = self.m, self.ctx
        cd = c["cd"]
        x = (F.embedding(tok, m.token_embed.weight) + F.embedding(pos, m.pos_embed.weight)[None]).to(cd)
        x = x.view(c["B"], -1)                                               # (B, d)
        mm_ = _proj_rows if (self.use_rows and cd == torch.bfloat16) else _proj_blas
        pending = None
        for i, (l, p) in enumerate(zip(m.layers, c["layers"])):
            conv_state, ssm_state = states[i]
            h, xs = ops.layer_norm(x if pending is None else pending, l.norm_mamba.weight, l.norm_mamba.bias,
                                   l.norm_mamba.eps, res=None if pending is None else x)
            if pending is not None:
                x = xs
            mm = l.mamba
            di, N, r = mm.d_inner, mm.d_state, mm.dt_rank
            xz = mm_(h, p["Win"])
            u = ops.conv_update(xz[:, :di], conv_state, p["conv_w"], p["conv_b"], True)
            x_dbl = mm_(u, p["Wx"])
            # dt_proj fused into the state update; B / C read in place from x_dbl
            y = ops.state_update(ssm_state, u, x_dbl[:, :r], p["A"], x_dbl[:, r:r + N], x_dbl[:, r + N:], p["D"],
                                 xz[:, di:], p["dt_bias"], True, dt_w=p["Wdt"])
            h_m = mm_(y, p["Wout"])
            h, x = ops.layer_norm(h_m, l.norm_cross.weight, l.norm_cross.bias, l.norm_cross.eps, res=x)
            q = mm_(h, p["Wq"], p["bq"])
            o = attention(q[:, None], p["k"], p["v"], l.cross_attn.num_heads, c["kpm"])[:, 0]
            a = mm_(o, p["Wo"], p["bo"])
            h, x = ops.layer_norm(a, l.norm_ff.weight, l.norm_ff.bias, l.norm_ff.eps, res=x,
                                  gamma=p["gamma"], beta=p["beta"], rows_per_group=1)
            pending = mm_(mm_(h, p["W1"], p["b1"], "gelu"), p["W2"], p["b2"])
        h, _ = ops.layer_norm(pending, m.norm_out.weight, m.norm_out.bias, m.norm_out.eps, res=x)
        return mm_(h, c["Wh"], c["bh"])[:, None]

    # -- out-of-range token ids --------------------------------------------------
    def _check_token_flag(self, dev, blocking=False):
        """The fused step embeds through mtts_embed_sum, which zero-fills and
        flags a row whose token id is outside token_embed (nn.Embedding raises
        there, mamba_decoder.py:217).  The flag of an earlier step is read from
        a pinned copy; without `blocking` only once its event has completed (no
        host sync), so the IndexError is best-effort and deferred: it comes at
        a later decode_step once the GPU has caught up, or at check_errors(),
        which waits for the copy and is the guarantee."""
        if self._err_ev is None:
            return
        if blocking:
            self._err_ev.synchronize()
        elif not self._err_ev.query():
            return
        if int(self._err_host[0]) != 0:
            self._err_host.zero_()
            _err_flag(dev).zero_()
            raise IndexError("decode_step: last_token id out of range of token_embed (index out of range in self)")

    def check_errors(self):
        """Blocking: raise IndexError if any step since the last check embedded
        an out-of-range token id (call before reset() / at the end of a
        generation to observe every error)."""
        if self._err_dev is not None:
            self._check_token_flag(self._err_dev, blocking=True)

    def _post_token_flag(self, dev):
        if self._err_host is None:
            self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._err_ev = torch.cuda.Event()
            self._err_dev = dev
        self._err_host.copy_(_err_flag(dev), non_blocking=True)
        self._err_ev.record()

    # -- public ----------------------------------------------------------------
    @torch.no_grad()
    def step(self, last_token, text_hidden, z_style, mamba_states, step_index, text_mask=None, ref_hidden=None,
             ref_mask=None):
        m = self.m
        self._check_token_flag(last_token.device)
        cd = m._cd()
        conds = (text_hidden, z_style, text_mask, ref_hidden, ref_mask)
        key = (cd, tuple(last_token.shape))
        if key != self.ctx_key or not _same_ctx(self.ctx_refs, self.ctx_versions, conds):
            self.ctx = self._build_ctx(text_hidden, z_style, text_mask, ref_hidden, ref_mask, cd)
            self.ctx_key = key
            self.ctx_refs = conds                  # strong references (see _same_ctx)
            self.ctx_versions = tuple(None if t is None else t._version for t in conds)
            self.fused = self._fused_ok(cd, last_token.shape[0])
            if self.fused and self.OPTIONS["packed"]:
                self._pack_ctx()
            self.xpk = self.fused and self._xpk_ok()
            self.fuse_q = self.xpk and self.OPTIONS["fuse_q"] and self._fuse_q_ok(last_token.shape[0])
            self.graph = None
            self.states = None
        B = last_token.shape[0]
        dev = last_token.device
        if self.states is None:
            self.states = []
            for l in m.layers:
                mm = l.mamba
                self.states.append((torch.zeros(B, mm.d_inner, mm.d_conv, device=dev),
                                    torch.zeros(B, mm.d_inner, mm.d_state, device=dev)))
            self.tok_buf = torch.zeros(B, 1, dtype=torch.long, device=dev)
            self.pos_buf = torch.zeros(1, dtype=torch.long, device=dev)
            self.pos32 = torch.zeros(1, dtype=torch.int32, device=dev)
        # adopt the caller's states (None = start of sequence)
        for i, st in enumerate(self.states):
            given = None if mamba_states is None else mamba_states[i]
            if given is None:
                st[0].zero_()
                st[1].zero_()
            elif given[0] is not st[0] or given[1] is not st[1]:
                st[0].copy_(given[0])
                st[1].copy_(given[1])
        self.tok_buf.copy_(last_token)
        if not 0 <= int(step_index) < m.pos_embed.num_embeddings:   # pos_embed(step_index) raises (:226)
            raise IndexError("index out of range in self")
        if self.fused:   # the fused step embeds through mtts_embed_sum (int32 position id)
            self.pos32.fill_(int(step_index))
        else:
            self.pos_buf.fill_(int(step_index))
        step = self._step_rows if self.fused else self._step
        if not self.use_graph:
            logits = step(self.tok_buf, self.pos_buf, self.states)
            if self.fused:
                self._post_token_flag(dev)
            return logits, list(self.states)
        if self.graph is None:
            saved = [(a.clone(), b.clone()) for a, b in self.states]
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):  # warm up (allocator, library handles)
                    step(self.tok_buf, self.pos_buf, self.states)
            torch.cuda.current_stream().wait_stream(s)
            for (a, b), (sa, sb) in zip(self.states, saved):
                a.copy_(sa)
                b.copy_(sb)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.out_buf = step(self.tok_buf, self.pos_buf, self.states)
            for (a, b), (sa, sb) in zip(self.states, saved):  # capture ran the step once
                a.copy_(sa)
                b.copy_(sb)
            self.graph = g
        self.graph.replay()
        if self.fused:
            self._post_token_flag(dev)
        return self.out_buf.clone(), list(self.states)
