"""Fused VAE train step + data-parallel gradient sync.

One step = the body of the reference's batch loop (src/Convolutional_VAE.py:224-240,
src/Conditional_VAE.py:321-331): forward -> loss -> backward -> optimizer.step, issued as a fixed
sequence of libhlmc calls on the current stream with no host synchronisation (the reference's
per-batch ``loss.item()`` is replaced by device-side loss sums that the caller may read lazily).

Data parallel: one process per GPU; the flat fp32 gradient buffer is all-reduced with SUM over
``torch.distributed`` (backend "nccl" = RCCL over xGMI on MI355X), i.e. gradients of the loss summed
over the global batch — the reference's sum-reduced losses make SUM the matching reduction.
BatchNorm batch statistics stay per rank (DDP semantics).  The buffer is reduced in the engine's gradient
buckets (hlmc_net_grad_buckets: contiguous parameter ranges in the order backward finishes them); on a
GPU each bucket's all-reduce is issued on a communication stream that waits on the bucket's event, so
RCCL overlaps the rest of the backward pass, and Adam waits for all of them.

BatchNorm running statistics follow DDP's ``broadcast_buffers=True``: DDP broadcasts rank 0's buffers at the
start of every forward, so step k's forward on rank r updates rank 0's step-(k-1) statistics with rank r's
batch, and any later forward (train or eval) sees rank 0's.  Here the running means / variances live in one
flat fp32 tensor per model and rank 0's copy is broadcast right after each forward, on the communication
stream under the backward pass: every forward after step k starts from rank 0's post-step-k statistics, the
same values DDP's pre-forward broadcast hands it, and all ranks hold identical buffers between steps (so
eval-mode ``encode`` — the latents K-Means clusters — agrees across ranks).
"""
from __future__ import annotations

import os

import torch

from . import _lib as L
from .models import ConditionalVAE, HybridVAE, VAE


class Trainer:
    def __init__(self, model, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, beta=None, text_weight=None,
                 process_group=None, distributed=False, grad_dtype=torch.float32, broadcast_buffers=True):
        self.model = model
        self.distributed = distributed or process_group is not None
        self.process_group = process_group
        self.broadcast_buffers = bool(broadcast_buffers) and self.distributed
        # BatchNorm running stats as views of one flat tensor: one broadcast per step (before the native net
        # binds their addresses)
        self.bn_flat = model._flatten_bn_buffers() if self.broadcast_buffers else None
        self.kind = "simple" if isinstance(model, VAE) else ("cvae" if isinstance(model, ConditionalVAE) else "hybrid")
        self.net = model._native_net()
        dev = next(model.parameters()).device
        self.device = dev
        self.params = list(model.parameters())
        self.gflat = model._gflat
        self.grads = model._grad_views
        n = self.gflat.numel()
        self.m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        mv, vv, off = [], [], 0
        for p in self.params:
            mv.append(self.m[off:off + p.numel()])
            vv.append(self.v[off:off + p.numel()])
            off += p.numel()
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.step_count = 0
        if beta is None:
            beta = {"hybrid": 1.0, "cvae": 4.0, "simple": 0.8}[self.kind]
        if text_weight is None:
            text_weight = {"hybrid": 350.0, "cvae": 200.0, "simple": 0.0}[self.kind]
        self.beta, self.text_weight = float(beta), float(text_weight)
        self.grad_dtype = grad_dtype
        self.buckets = self._bucket_ranges()
        self._comm = None
        self._fwd_done = None
        self._rng_key = 0
        if self.distributed:
            # per-rank reparameterisation noise: every rank builds its model after the same torch.manual_seed, so
            # the engine's Philox streams start equal; rank r > 0 re-keys its seed (rank 0 keeps the single-process
            # stream), so the ranks' clips get independent eps as separate torch.randn_like draws would
            import torch.distributed as dist
            rank = dist.get_rank(process_group) if process_group is not None else dist.get_rank()
            self._rng_key = rank_rng_key(rank)
            if rank:
                seed, off = model.get_rng_state()
                model.set_rng_state((keyed_seed(seed, self._rng_key), off))
        if self.distributed and dev.type == "cuda":
            self._fwd_done = torch.cuda.Event()
            L.check(L.lib().hlmc_net_set_bucket_sync(self.net.h, 1), "hlmc_net_set_bucket_sync")
            self._comm = torch.cuda.Stream(device=dev)
        else:  # single process, HLMC_OVERLAP_ADAM=1: Adam starts under the tail of the backward pass (measured
            # 0.5% slower than joining first on MI355X, so off by default)
            on = int(os.environ.get("HLMC_OVERLAP_ADAM", "0") == "1")
            L.check(L.lib().hlmc_net_set_overlap_adam(self.net.h, on), "hlmc_net_set_overlap_adam")
        self._mv = (L.vp_array([t.data_ptr() for t in mv]), L.vp_array([t.data_ptr() for t in vv]))
        # graph replay (GraphedStep): Adam reads its step-dependent coefficients from _coef_dev, refreshed from a
        # pinned host ring before every launch
        self._graph = False
        self._coef_dev = torch.zeros(6, dtype=torch.float32, device=dev)
        self._coef_ring = torch.zeros(1024, 6, dtype=torch.float32).pin_memory() if dev.type == "cuda" else None
        # weights change only through hlmc_net_adam_step (which refreshes the packed GEMM layouts)
        L.check(L.lib().hlmc_net_set_trust_packs(self.net.h, 1))
        self._cache = {}

    def _buffers(self, B):
        if B not in self._cache:
            dev = self.device
            m = self.model
            out = m._alloc_outputs(B, dev)
            d = {k: torch.empty_like(v) for k, v in out.items()}
            ws = self.net.new_workspace(B, dev)
            na = out["recon"].numel()
            nt = out["recon_text"].numel() if "recon_text" in out else 0
            nl = out["mu"].numel()
            lws = torch.empty(max(16, int(L.lib().hlmc_loss_workspace(na, nt, nl))), dtype=torch.uint8, device=dev)
            sums = torch.zeros(3, dtype=torch.float64, device=dev)
            if self.kind == "simple":
                coef = torch.tensor([2.0 / na, 0.0, self.beta / nl], device=dev)
            else:
                coef = torch.tensor([2.0, 2.0 * self.text_weight, self.beta], device=dev)
            self._cache[B] = dict(out=out, d=d, ws=ws, lws=lws, sums=sums, coef=coef, n=(na, nt, nl))
        return self._cache[B]

    def state_dict(self):
        """Optimizer + noise state for checkpoint / resume (the model's own state_dict holds the parameters and
        BatchNorm buffers): Adam step count and moments, and the engine's Philox (seed, offset).  The seed is stored
        un-keyed (the single-process / rank-0 stream), so the usual DP checkpoint -- written by rank 0, loaded on every
        rank -- restores each rank's own noise stream: load_state_dict re-applies the loading rank's key."""
        seed, off = self.model.get_rng_state()
        return {"step": self.step_count, "exp_avg": self.m.detach().clone(), "exp_avg_sq": self.v.detach().clone(),
                "rng": (keyed_seed(seed, -self._rng_key), off)}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.m.copy_(sd["exp_avg"])
        self.v.copy_(sd["exp_avg_sq"])
        seed, off = sd["rng"]
        self.model.set_rng_state((keyed_seed(int(seed), self._rng_key), int(off)))

    def step(self, in0, in1=None, in2=None, eps=None, dropout=None, before_adam=None):
        """One optimisation step on a batch; returns device float64 sums (sum sq audio err, sum sq text err,
        sum(1+lv-mu^2-e^lv)) from which the reference's loss tuple follows.  before_adam (optional callable)
        is invoked once the backward pass is enqueued, before the optimizer update (the inputs are no longer
        read from there on: a caller may start refilling them on another stream)."""
        lib = L.lib()
        s = L.stream()
        B = in0.shape[0]
        if self.broadcast_buffers:
            self._check_bn_flat()
        c = self._buffers(B)
        out, d = c["out"], c["d"]
        # eps None: the engine draws the reparameterisation noise on the device (Philox, hlmc_net_set_rng) — except
        # under graph capture, where the host-side stream offset would freeze into the graph: torch's graph-safe randn
        if eps is None and self._graph:
            eps = torch.randn(B, self.model.latent_dim, device=self.device)
        if self.kind == "simple" and dropout is None:
            dropout = self.model.make_dropout_mask(B, self.device)
        L.check(lib.hlmc_net_forward(self.net.h, s, B, 1, L.ptr(in0), L.ptr(in1), L.ptr(in2), L.ptr(eps),
                                     L.ptr(dropout), L.ptr(out["recon"]), L.ptr(out.get("recon_text")),
                                     L.ptr(out["mu"]), L.ptr(out["logvar"]), L.ptr(out.get("z")), c["ws"].data_ptr()),
                "hlmc_net_forward")
        bcast = None
        if self.broadcast_buffers:
            bcast = self._broadcast_buffers_after_forward()
        na, nt, nl = c["n"]
        rt, t = out.get("recon_text"), (in1 if nt else None)
        # the loss sums and their gradient in one pass (hlmc_loss_sums + hlmc_loss_backward fused)
        L.check(lib.hlmc_loss_sums_backward(s, L.ptr(out["recon"]), L.ptr(in0), na, L.ptr(d["recon"]), L.ptr(rt),
                                            L.ptr(t), nt, L.ptr(d.get("recon_text")), L.ptr(out["mu"]),
                                            L.ptr(out["logvar"]), nl, c["coef"].data_ptr(), L.ptr(d["mu"]),
                                            L.ptr(d["logvar"]), c["sums"].data_ptr(), c["lws"].data_ptr()),
                "hlmc_loss_sums_backward")
        L.check(lib.hlmc_net_backward(self.net.h, s, B, L.ptr(d["recon"]), L.ptr(d.get("recon_text")), L.ptr(d["mu"]),
                                      L.ptr(d["logvar"]), c["ws"].data_ptr()), "hlmc_net_backward")
        if self.distributed:
            if self._comm is not None:
                self._allreduce_overlapped(bcast)
            else:
                self.allreduce_grads()
        if before_adam is not None:
            # the inputs must be out of every reader's hands: with the tail weight gradients left on the side stream
            # (overlap_adam) the encoder's first weight gradient still reads in0 -> join it first
            L.check(lib.hlmc_net_settle(self.net.h, s), "hlmc_net_settle")
            before_adam()
        if self._graph:  # coefficients staged by prepare_step_coefficients()
            L.check(lib.hlmc_net_adam_step_dev(self.net.h, s, *self._mv, self._coef_dev.data_ptr()),
                    "hlmc_net_adam_step_dev")
            return c["sums"]
        self.step_count += 1
        b1, b2 = self.betas
        L.check(lib.hlmc_net_adam_step(self.net.h, s, *self._mv, float(self.lr), float(b1), float(b2), float(self.eps),
                                       float(self.wd), self.step_count), "hlmc_net_adam_step")
        return c["sums"]

    def prepare_step_coefficients(self):
        """Advance the step counter and stage that step's Adam coefficients (host -> pinned ring -> device,
        stream-ordered) for the next graph-mode step."""
        self.step_count += 1
        slot = self._coef_ring[self.step_count % self._coef_ring.shape[0]]
        b1, b2 = self.betas
        L.check(L.lib().hlmc_adam_coef(float(self.lr), float(b1), float(b2), float(self.eps), float(self.wd),
                                       self.step_count, slot.data_ptr()), "hlmc_adam_coef")
        self._coef_dev.copy_(slot, non_blocking=True)

    def release(self):
        """Hand the model back to the nn.Module path (forward re-packs weights every call again)."""
        L.check(L.lib().hlmc_net_set_trust_packs(self.net.h, 0))
        L.check(L.lib().hlmc_net_set_overlap_adam(self.net.h, 0))

    def _bucket_ranges(self):
        """[(lo, hi)] element ranges of the flat gradient buffer, one per engine bucket, in backward order."""
        offs = [0]
        for p in self.params:
            offs.append(offs[-1] + p.numel())
        cap = 64
        starts = (L.c_int * cap)()
        nb = L.lib().hlmc_net_grad_buckets(self.net.h, starts, cap)
        if nb < 0:
            L.check(nb, "hlmc_net_grad_buckets")
        return bucket_ranges(list(starts)[:nb], offs)

    def _check_bn_flat(self):
        """The buffer broadcast sends the flat tensor the BatchNorm running statistics were re-pointed at when this
        Trainer was built; a later module._apply (device move, .half()) or load_state_dict(assign=True) replaces
        them with new tensors, and a silent broadcast of the stale flat copy would let the ranks drift apart."""
        bns = [m for m in self.model.modules() if isinstance(m, torch.nn.modules.batchnorm._BatchNorm)]
        if bns and bns[0].running_mean.data_ptr() != self.bn_flat.data_ptr():
            raise L.HLMCError("BatchNorm running statistics were replaced after the Trainer was built "
                              "(module._apply / load_state_dict(assign=True)); build a new Trainer")

    def _broadcast_buffers_after_forward(self):
        """Rank 0's BatchNorm running statistics to every rank (DDP broadcast_buffers), issued right after the
        forward that updated them: on the comm stream (under the backward pass) on a GPU, else synchronously."""
        import torch.distributed as dist
        src = dist.get_global_rank(self.process_group, 0) if self.process_group is not None else 0
        if self._comm is None:
            dist.broadcast(self.bn_flat, src=src, group=self.process_group)
            return None
        self._fwd_done.record()
        self._comm.wait_event(self._fwd_done)
        with torch.cuda.stream(self._comm):
            return dist.broadcast(self.bn_flat, src=src, group=self.process_group, async_op=True)

    def sync_buffers(self):
        """Broadcast rank 0's BatchNorm running statistics now (what DDP does before an eval-mode forward)."""
        if self.broadcast_buffers:
            import torch.distributed as dist
            src = dist.get_global_rank(self.process_group, 0) if self.process_group is not None else 0
            dist.broadcast(self.bn_flat, src=src, group=self.process_group)

    def _allreduce_overlapped(self, bcast=None):
        """Per-bucket SUM all-reduces on the comm stream, each gated on its bucket's backward event; the
        current stream (Adam, then the next step's forward and backward) waits for all of them — and for the
        comm stream itself, which also runs the bf16 wire copies and the buffer broadcast."""
        lib = L.lib()
        works = [] if bcast is None else [bcast]
        with torch.cuda.stream(self._comm):
            for k, (lo, hi) in enumerate(self.buckets):
                L.check(lib.hlmc_net_bucket_wait(self.net.h, k, self._comm.cuda_stream), "hlmc_net_bucket_wait")
                works.append(_allreduce_sum(self.gflat[lo:hi], self.grad_dtype, self.process_group, async_op=True))
            # every bucket's collective is in flight before the first wait; the wait makes the comm stream (not
            # the host, under RCCL) wait for it, and a bf16 wire's copy-back follows on the comm stream
            for w in works:
                w.wait()
        torch.cuda.current_stream().wait_stream(self._comm)

    def allreduce_grads(self):
        """SUM all-reduce of the flat gradient buffer, bucket by bucket (RCCL under 'nccl', gloo on CPU)."""
        for lo, hi in getattr(self, "buckets", None) or [(0, self.gflat.numel())]:
            _allreduce_sum(self.gflat[lo:hi], self.grad_dtype, self.process_group)

    def loss_tuple(self, sums, batch=None):
        """Host floats (total, l_audio, l_text, kld) from device sums (synchronises; raises HLMCError when a kernel
        of the step reported a fault through the library's device status word)."""
        s = sums.cpu().tolist()
        L.check_device("Trainer.step")
        if self.kind == "simple":
            na, _, nl = self._cache[batch or next(iter(self._cache))]["n"]
            la, kl = s[0] / na, -0.5 * s[2] / nl
            return la + self.beta * kl, la, 0.0, kl
        kld = -0.5 * s[2]
        return s[0] + self.text_weight * s[1] + self.beta * kld, s[0], s[1], kld


_RNG_KEY_STEP = 0x9E3779B97F4A7C15  # 2^64 / golden ratio: distinct, well-spread Philox keys per rank


def rank_rng_key(rank):
    """The additive Philox seed key of a data-parallel rank (0 for rank 0: the single-process stream)."""
    return (int(rank) * _RNG_KEY_STEP) & 0xFFFFFFFFFFFFFFFF


def keyed_seed(seed, key):
    """seed + key modulo 2^64 (key may be negative: un-keying)."""
    return (int(seed) + int(key)) & 0xFFFFFFFFFFFFFFFF


def bucket_ranges(starts, offsets):
    """Flat-buffer element ranges of engine gradient buckets.  starts: first parameter index of each bucket in
    backward order (strictly decreasing, last 0); offsets: element offset of every parameter (+ the total)."""
    if not starts or starts[-1] != 0 or any(a <= b for a, b in zip(starts, starts[1:])):
        raise ValueError(f"bucket starts must decrease strictly to 0: {starts}")
    hi_idx = len(offsets) - 1
    out = []
    for st in starts:
        out.append((offsets[st], offsets[hi_idx]))
        hi_idx = st
    return out


def _allreduce_sum(buf, grad_dtype, group, async_op=False):
    """SUM all-reduce of a contiguous fp32 gradient slice, optionally on a bf16 wire copy (half the bytes over
    xGMI): converted on the current stream, reduced in place, and copied back into `buf` by the handle's wait()
    on the stream wait() is called from (the caller makes its consumers wait for that stream)."""
    import torch.distributed as dist
    if grad_dtype == torch.float32:
        return dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
    g = buf.to(grad_dtype)
    w = _WireWork(dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group, async_op=True), g, buf)
    if not async_op:
        w.wait()
    return w


class _WireWork:
    """Handle of a reduced-precision wire all-reduce: wait() orders the current stream after the collective
    (RCCL: a stream wait, the host does not block) and copies the reduced wire values back into the fp32
    buffer on that stream."""

    def __init__(self, work, wire, buf):
        self.work, self.wire, self.buf = work, wire, buf

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.buf.copy_(self.wire)
            self.work = None
        return True


class GraphedStep:
    """A whole train step captured once into a HIP graph and replayed (hipGraphLaunch): `body()` issues the
    step's device work on static tensors — e.g. the mel stage followed by ``trainer.step(...)`` — and returns
    its outputs.  The engine's weight-gradient stream joins the capture through its fork/join events; torch's
    RNG (the reparameterisation noise) is graph-safe; Adam's step-dependent coefficients are staged before
    every replay.  `warmup` eager steps (real optimisation steps) run first so every buffer, packed weight
    and job list exists before capture.  Single-process only: the data-parallel path keeps the eager
    bucketed all-reduce."""

    def __init__(self, trainer, body, warmup=2, before_capture=None):
        if trainer.distributed:
            raise L.HLMCError("GraphedStep is single-process; data parallel training uses Trainer.step")
        self.trainer = trainer
        trainer._graph = True
        try:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(max(1, warmup)):
                    trainer.prepare_step_coefficients()
                    body()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            if before_capture is not None:
                before_capture()
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.out = body()
        except Exception:
            trainer._graph = False
            raise

    def __call__(self):
        self.trainer.prepare_step_coefficients()
        self.graph.replay()
        return self.out

    def release(self):
        """Back to eager Trainer.step."""
        self.trainer._graph = False
        self.graph.reset()
