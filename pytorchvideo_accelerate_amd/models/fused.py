"""Fused MI355X training/eval executor for SlowFast and Slow ResNet3D.

This replaces PyTorch autograd for the backbone with an explicit, static forward/backward plan over the
gfx950 kernels (``ops/conv.py`` + ``csrc/kernels``).  Design:

* Activations are NDHWC bf16 :class:`Act` views.  Each conv stores only its **raw** output ``y``; the
  training-mode BatchNorm (+ReLU) of ``y`` is applied by the *consumer* conv while it stages its input
  tile (per-channel affine in the MFMA prologue), so normalised activations inside a bottleneck are
  never written to HBM.  The conv epilogue emits the BN partial sums; ``bn_finalize`` produces
  mean/rstd, the running-stat update and the consumer affine.
* Residual-unit outputs (consumed by two convs and the identity path) are materialised once by the
  ``res_out`` kernel.  The slow pathway's output of a fused stage is written straight into the channel
  slice of the concatenation buffer, and the lateral fusion's BN-ReLU writes the other slice: the
  concat costs nothing.
* Backward reuses the same kernels: BN backward = deterministic reduce → finalize (dγ, dβ into the flat
  fp32 gradient buffer) → apply (dy); wgrad recomputes the consumer's input BN-ReLU on the fly; dgrad
  accumulates into shared input gradients (identity shortcut, fast-pathway fan-out).
* Parameters live in ONE flat fp32 buffer (module parameters become views, so ``state_dict`` keys and
  optimizers are untouched); gradients likewise — that is what the bucketed RCCL all-reduce
  (``parallel/ddp.py``) and the single-launch fused SGD (``ops/optim.py``) operate on.  bf16 packed
  weights (forward ``[Cout][taps][Cin]`` and dgrad ``[Cin][taps][Cout]`` layouts) are refreshed by one
  multi-tensor kernel after each optimizer step.
* The classification head (dropout → linear → position mean → softmax-CE, forward and backward) runs on
  the fp32-MFMA head kernels (``csrc/kernels/head.hip``), writing dW/db straight into the flat gradient.

Semantics follow the pytorchvideo modules in ``models/reference.py`` (reference ``run.py:105-118``);
``tests/test_fused_gpu.py`` pins loss / gradient / running-stat parity against that oracle.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..utils.arms import arm, on
from ..ops._ext import require
from ..ops.conv import Act, ConvSpec, dgrad_phases, fwd_geometry
from . import reference as R
from ..utils.profiling import trace_range


class _Xf:
    """Consumer-side input transform: y -> act(y*scale + shift)."""
    __slots__ = ("scale", "shift", "relu")

    def __init__(self, scale, shift, relu=True):
        self.scale, self.shift, self.relu = scale, shift, relu


class FlatParams:
    """All parameters of a module in one flat fp32 buffer (plus a same-shaped gradient buffer).

    Order = reverse of forward execution so that gradient buckets complete front-to-back during the
    backward pass (first bucket = head, last = stems).
    """

    def __init__(self, params: Sequence[Tuple[str, nn.Parameter]], device):
        self.names = [n for n, _ in params]
        self.params = [p for _, p in params]
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + 3) // 4 * 4  # 16-B alignment of every tensor
        self.numel = off
        self.data = torch.zeros(off, device=device, dtype=torch.float32)
        self.grad = torch.zeros(off, device=device, dtype=torch.float32)
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            self.data[o:o + n].copy_(p.data.reshape(-1).to(device))
            p.data = self.data[o:o + n].view(p.shape)
            p.grad = self.grad[o:o + n].view(p.shape)
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.zeroed = True  # gradient buffer logically zero: next backward overwrites it

    def view(self, p: nn.Parameter) -> torch.Tensor:
        i = self.index[id(p)]
        return self.data[self.offsets[i]:self.offsets[i] + p.numel()].view(p.shape)

    def gview(self, p: nn.Parameter) -> torch.Tensor:
        i = self.index[id(p)]
        return self.grad[self.offsets[i]:self.offsets[i] + p.numel()].view(p.shape)

    def span(self, p: nn.Parameter) -> Tuple[int, int]:
        i = self.index[id(p)]
        return self.offsets[i], self.offsets[i] + p.numel()

    def rebind(self):
        """Re-point module parameters at the flat storage (after e.g. ``load_state_dict`` replaced data)."""
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            if p.data.data_ptr() != self.data[o:o + n].data_ptr():
                self.data[o:o + n].copy_(p.data.reshape(-1))
                p.data = self.data[o:o + n].view(p.shape)
            gv = self.grad[o:o + n].view(p.shape)
            if p.grad is None or p.grad.data_ptr() != gv.data_ptr():
                if p.grad is not None:  # autograd replaced the view: keep its values
                    gv.copy_(p.grad)
                p.grad = gv


class _ConvBN:
    """One conv (bias-free) + its BatchNorm3d."""

    def __init__(self, eng: "FusedNet", conv: nn.Conv3d, bn: nn.BatchNorm3d, name: str, cin_pad: int = 0):
        self.eng, self.conv, self.bn, self.name = eng, conv, bn, name
        self.spec = ConvSpec(conv.in_channels, conv.out_channels, tuple(conv.kernel_size), tuple(conv.stride),
                             tuple(conv.padding), cin_pad)
        C, dev = conv.out_channels, eng.device
        self.mean = torch.zeros(C, device=dev)
        self.rstd = torch.ones(C, device=dev)
        self.scale = torch.ones(C, device=dev)
        self.shift = torch.zeros(C, device=dev)
        self.coef = torch.zeros(4 * C, device=dev)   # BN-backward coefficients (+ mean(dz) for BN folding)
        self._geo = {}
        self.wf = None  # bf16 forward pack view [Cout, taps*Cin_pad]
        self.wd = None  # bf16 dgrad pack view [Cin, taps*Cout]

    @property
    def C(self):
        return self.spec.cout

    @property
    def fin(self):
        """Two-level BN finalize workspace of the current stream lane (``FusedNet.fin_ws``)."""
        return self.eng.fin_ws()

    def xf(self, relu=True) -> _Xf:
        return _Xf(self.scale, self.shift, relu)

    # ---- forward ----
    def fwd(self, x: Act, xf: Optional[_Xf], train: bool, tag: str) -> Act:
        C = self.eng.C
        s = self.spec
        self.eng.mark(self.name + ".fwd")
        To, Ho, Wo = s.out_dims(x.T, x.H, x.W)
        M = x.N * To * Ho * Wo
        y = self.eng.ws((self.name, "y", tag), (M, s.cout), self.eng.cdt)
        stats = None
        if train:  # sized for the smallest row tile (128); the launch writes ceil(M / BM) of them
            stats = self.eng.ws((self.name, "stats"), ((M + 127) // 128, 2, s.cout), torch.float32)
        aff = 0 if xf is None else (2 if xf.relu else 1)
        key = ("fg", x.N, x.T, x.H, x.W, x.ld)
        g = self._geo.get(key)
        if g is None:
            g = self._geo[key] = fwd_geometry(s, x.N, x.T, x.H, x.W, x.ld, s.cout)
        sc_, sh_ = (None, None) if xf is None else (xf.scale, xf.shift)
        tuner = self.eng.tuner

        def run(cfg, scratch):
            C.conv_igemm(x.t, self.wf, tuner.scratch_like(y) if scratch else y,
                         None if stats is None else (tuner.scratch_like(stats) if scratch else stats),
                         sc_, sh_, aff, 0, g, s.chunk, cfg)
        cfg = tuner.launch(("f", s.chunk, aff, train) + tuple(g), g, s.chunk, run, aff=aff)
        bn = self.bn
        if train:
            tiles = (M + tuner.bm(cfg, s.cout) - 1) // tuner.bm(cfg, s.cout)
            C.bn_finalize(stats, tiles, s.cout, M, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                          bn.num_batches_tracked, bn.momentum if bn.momentum is not None else 0.1, bn.eps,
                          self.mean, self.rstd, self.scale, self.shift, self.fin)
        else:
            C.bn_eval_affine(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, self.scale, self.shift)
        return Act(y, x.N, To, Ho, Wo)

    # ---- backward pieces ----
    def wgrad(self, dy: Act, x: Act, xf: Optional[_Xf], spec: Optional[ConvSpec] = None,
              dest: Optional[torch.Tensor] = None, beta: Optional[float] = None, gram: bool = False,
              colsum: Optional[torch.Tensor] = None):
        """Weight gradient dy^T im2col(x) (x through ``xf`` when given) into ``dest`` (default: this conv's
        slot of the flat gradient, accumulated with the executor's ``grad_beta``).  ``gram``: Gram mode of the
        BN folding — dy is x itself, both through ``xf`` (``spec`` = the c->c 1x1 shape), per-split column
        sums into ``colsum`` [splits][c]; returns the number of splits."""
        eng, C = self.eng, self.eng.C
        s = spec or self.spec
        eng.mark(self.name + (".gram" if gram else ".wgrad"))
        K = s.taps * s.cin_pad
        from ..ops.conv import RT, box_wgrad_plan, box_wgrad_slabs, wgrad_splits
        aff = 0 if xf is None else (2 if xf.relu else 1)
        sc_, sh_ = (None, None) if xf is None else (xf.scale, xf.shift)
        slab = 1 if (eng.deterministic or eng.reproducible or (eng.fold_slabs and dest is not None)) else 0
        dya = 1 if gram else 0

        def geometry(cfg):
            """(splits, rows per split, kernel variant word) of launch configuration ``cfg``."""
            key = (self.name, "wsplit", dy.M, cfg, gram)
            sp = eng._splits.get(key)
            if sp is None:
                if cfg < 0:
                    sp = wgrad_splits(dy.M, s.cout, K, target_blocks=256 if slab else 1024) + (-1,)
                elif cfg & 1024:  # box-staged (1,3,3) kernel (wgrad_box.hip): own slabs, fixed-order reduction
                    sp = box_wgrad_plan(s, dy.M, (dy.T, dy.H, dy.W), dy.ld, x.ld)
                elif cfg & 2048:  # row-table kernel (wgrad_rt_impl.h): tile / split-K / stage bits as below
                    v = (cfg & 3) | (8 if cfg & 64 else 0)
                    tb = (512, 1024, 2048, 4096)[(cfg >> 2) & 3]
                    sp = wgrad_splits(dy.M, s.cout, K, target_blocks=tb, variant=v) + (
                        v | (4 if cfg & 32 else 0) | RT,)
                elif cfg & 256:   # halo-staged kernel (wgrad_halo.hip): bit 9 = box option
                    from ..ops.conv import halo_wgrad_plan
                    sp = halo_wgrad_plan(s, dy.M, (dy.T, dy.H, dy.W), (cfg >> 9) & 1)
                elif cfg & 128:   # narrow per-wave kernel: bits 2-3 = wave count target, 64 rows per chunk
                    nw = (1024, 2048, 4096, 8192)[(cfg >> 2) & 3]
                    pps = ((dy.M + nw - 1) // nw + 63) // 64 * 64
                    sp = ((dy.M + pps - 1) // pps, pps, 16)
                else:   # bits 0-1 (+ bit 6: tiles 4-7) tile variant, 2-3 split-K target, 5: 64-position stages
                    v = (cfg & 3) | (8 if cfg & 64 else 0)
                    tb = (512, 1024, 2048, 4096)[(cfg >> 2) & 3]
                    sp = wgrad_splits(dy.M, s.cout, K, target_blocks=tb, variant=v) + (v | (4 if cfg & 32 else 0),)
                eng._splits[key] = sp
            return sp

        def launch(cfg, part, cs=None):
            splits, pps, v = geometry(cfg)
            g = [dy.M, s.cout, K, s.cin_pad, dy.ld, x.ld, x.T, x.H, x.W, dy.T, dy.H, dy.W,
                 *s.k, *s.stride, *s.pad, splits, pps]
            C.conv_wgrad(dy.t, x.t, part, sc_, sh_, aff, g, s.chunk, 1 if cfg >= 0 and cfg & 1024 else slab, v, dya,
                         None if cs is None else cs[:splits * s.cout])
            return splits

        def box_run(cfg, grad, beta_):
            """box-staged kernel into its per-range slabs, then the two-pass fixed-order reduction into ``grad``"""
            nslab = box_wgrad_slabs(s, geometry(cfg)[0])
            part = eng.scratch("wgrad_box_slab", nslab * s.cout * K)
            launch(cfg, part)
            tmp = eng.scratch("wgrad_box_tmp", C.box_reduce_groups(nslab) * s.cout * K)
            C.wgrad_box_reduce(part, tmp, grad, nslab, s.cout, s.taps, s.cin_pad, s.cin, 1.0, beta_)
            return nslab

        tkey = ("w", dy.M, dy.ld, x.ld, x.T, x.H, x.W, s.cout, K, s.chunk, aff, gram, slab) + tuple(s.k) + tuple(
            s.stride)
        cfg = eng.wtune.get(tkey)
        if cfg is None:
            cfg = -1
            if eng.tuner.enabled and not eng.deterministic:
                # first use: time tile variant x split-K target on a scratch accumulator (atomic adds; the
                # scratch content is irrelevant), keep the fastest.  Slab launches (BN-folding Gram / G products
                # under fold_slabs) are timed with their fixed-order reduction, whose cost grows with the split count
                scratch = eng.scratch("wgrad_tune", s.cout * K)
                cs_scr = eng.scratch("wgrad_tune_cs", 4096 * s.cout) if gram else None
                cands = []
                for v in range(8):
                    vw = (v & 3) | (8 if v >= 4 else 0)
                    bmw, bnw = C.wgrad_tile(s.cout, K, vw)
                    # a tile up to twice Cout tall is a candidate (awkward Cout such as 80: one 128-row tile per split
                    # re-reads dy once, where 64-row tiles re-read it per tile)
                    if bmw > max(16, 2 * s.cout) or bmw * 8 < s.cout or (v >= 4 and bnw > 2 * K):
                        continue
                    for tbi, bp in ((t, b) for t in range(4) for b in (0, 32)):
                        c = 16 | (v & 3) | (64 if v >= 4 else 0) | (tbi << 2) | bp
                        if gram and geometry(c)[0] > 4096:
                            continue
                        cands.append(c)
                dense = s.taps == 1 and tuple(s.stride) == (1, 1, 1)
                if not gram and not dense and C.wgrad_rt_legal(s.cout, s.cin_pad, dy.ld, x.ld, s.chunk):
                    # row-table kernel for gathered shapes: tiles 2-7, both stage depths, 512-2048 blocks
                    for v in range(2, 8):
                        vw = (v & 3) | (8 if v >= 4 else 0)
                        bmw, bnw = C.wgrad_tile(s.cout, K, vw)
                        if bmw > max(64, 2 * s.cout) or (v >= 4 and bnw > 2 * K):
                            continue
                        for tbi, bp in ((t, b) for t in range(3) for b in (0, 32)):
                            cands.append(16 | 2048 | (v & 3) | (64 if v >= 4 else 0) | (tbi << 2) | bp)
                if C.wgrad_narrow_legal(s.cout, s.cin_pad, K) and s.chunk == 8 and not slab:
                    cands += [c for c in (16 | 128 | (tbi << 2) for tbi in range(4))
                              if not (gram and geometry(c)[0] > 4096)]   # colsum slab holds 4096 splits
                if not gram and box_wgrad_plan(s, dy.M, (dy.T, dy.H, dy.W), dy.ld, x.ld) is not None:
                    cands.append(16 | 1024)
                if not gram and not slab:   # halo-staged kernel, two box sizes
                    from ..ops.conv import halo_wgrad_plan
                    for o in (0, 1):
                        plan = halo_wgrad_plan(s, dy.M, (dy.T, dy.H, dy.W), o)
                        if plan is None:
                            continue
                        gh = [dy.M, s.cout, K, s.cin_pad, dy.ld, x.ld, x.T, x.H, x.W, dy.T, dy.H, dy.W,
                              *s.k, *s.stride, *s.pad, plan[0], plan[1]]
                        if C.wgrad_halo_legal(gh, plan[2], aff):
                            cands.append(16 | 256 | (o << 9))
                gscr = eng.scratch("wgrad_tune_grad", s.cout * K)
                # configurations borrowed from another batch size's table (ConvTuner.borrow), when still legal here
                bc = eng.tuner.borrow_lookup("wgrad", tkey, 1)
                if bc is not None and bc in cands:
                    cfg = bc
                else:
                    eng.tuner.tuned += 1

                    def trial(c):
                        if c & 1024:
                            box_run(c, gscr, 0.0)
                        elif slab:
                            part = eng.scratch("wgrad_tune_slab", geometry(c)[0] * s.cout * K)
                            sp = launch(c, part, cs_scr)
                            C.wgrad_reduce(part, gscr, sp, s.cout, s.taps, s.cin_pad, s.cin, 1.0, 0.0, 1)
                        else:
                            launch(c, scratch, cs_scr)
                    # two-phase timing, agreed across data-parallel ranks (ops/tune.ConvTuner.time_candidates)
                    times = eng.tuner.time_candidates(cands, trial) if cands else []
                    cfg = cands[min(range(len(cands)), key=times.__getitem__)] if cands else -1
                    if eng.tuner.log:
                        import sys
                        print("wtune %s%s P=%d Cout=%d K=%d: " % (self.name, ".gram" if gram else "", dy.M, s.cout, K)
                              + " ".join("%d=%.1fus" % (c, 1e3 * t) for c, t in zip(cands, times))
                              + " -> %d" % cfg, file=sys.stderr, flush=True)
            eng.wtune[tkey] = cfg
        # off the critical path: a weight gradient that lands in the flat buffer runs on the lane's wgrad
        # stream, concurrently with the dgrad chain (its inputs are per-unit buffers nothing rewrites before
        # the end-of-backward join)
        wst = eng._wgrad_stream() if (dest is None and not gram and (not slab or eng.reproducible)
                                      and eng._ms_active()) else None
        if wst is not None:
            src = torch.cuda.current_stream(eng.device)
            ev = torch.cuda.Event()
            ev.record(src)
            wst.wait_event(ev)
            lane0 = eng.lane
            eng.lane = 2 + lane0
            try:
                with torch.cuda.stream(wst):
                    if cfg >= 0 and cfg & 1024:
                        splits = box_run(cfg, eng.flat.gview(self.conv.weight), eng.grad_beta)
                    else:
                        part = (eng.scratch("wgrad_slab", geometry(cfg)[0] * s.cout * K) if slab else
                                eng.scratch("wgrad_acc", s.cout * K, zero=True))
                        splits = launch(cfg, part, colsum)
                        C.wgrad_reduce(part, eng.flat.gview(self.conv.weight), splits, s.cout, s.taps, s.cin_pad,
                                       s.cin, 1.0, eng.grad_beta, slab)
            finally:
                eng.lane = lane0
            return splits
        if cfg >= 0 and cfg & 1024:
            return box_run(cfg, eng.flat.gview(self.conv.weight) if dest is None else dest,
                           eng.grad_beta if beta is None else beta)
        if slab:  # per-split slabs summed in a fixed order: bitwise reproducible weight gradients
            part = eng.scratch("wgrad_slab", geometry(cfg)[0] * s.cout * K)
        else:     # fp32 atomics into one zeroed accumulator (kept zero by wgrad_reduce)
            part = eng.scratch("wgrad_acc", s.cout * K, zero=True)
        if gram:
            assert colsum is not None and colsum.numel() >= geometry(cfg)[0] * s.cout, "colsum slab too small"
        splits = launch(cfg, part, colsum)
        C.wgrad_reduce(part, eng.flat.gview(self.conv.weight) if dest is None else dest, splits, s.cout, s.taps,
                       s.cin_pad, s.cin, 1.0, eng.grad_beta if beta is None else beta, slab)
        return splits

    # ---- BatchNorm folding of a 1x1 conv_c (csrc/kernels/bn_fold.hip) ----
    def fold_forward(self, yb: Act, bxf: _Xf, train: bool):
        """BN statistics of this conv's output computed from the Gram matrix of its input act_b(yb) — the raw
        output is never materialised.  Keeps T = Wc Ga and the column sums for the backward."""
        eng, C, s = self.eng, self.eng.C, self.spec
        bn = self.bn
        if not train:
            C.bn_eval_affine(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, self.scale, self.shift)
            return
        c, Co = s.cin, s.cout
        if not hasattr(self, "gspec"):
            self.gspec = ConvSpec(c, c, (1, 1, 1), (1, 1, 1), (0, 0, 0))
        Ga = eng.scratch("fold_gram", c * c)
        slab = eng.scratch("fold_colsum", 4096 * c)
        splits = self.wgrad(yb, yb, bxf, spec=self.gspec, dest=Ga, beta=0.0, gram=True, colsum=slab)
        self.T = eng.ws((self.name, "foldT"), (Co, c), torch.float32)
        self.s = eng.ws((self.name, "folds"), (c,), torch.float32)
        exact = c < eng.fold_exact_below
        eng.mark(self.name + ".foldstats")
        # T = Wc Ga and the column sums (backward); with ``exact`` the statistics come from the pass below
        C.bnfold_fwd_stats(self.wf, Ga, slab, splits, Co, c, yb.M, self.T, self.s, bn.weight, bn.bias,
                           None if exact else bn.running_mean, None if exact else bn.running_var,
                           None if exact else bn.num_batches_tracked,
                           bn.momentum if bn.momentum is not None else 0.1, bn.eps, self.mean, self.rstd,
                           self.scale, self.shift)
        if exact:
            # narrow (fast-pathway) folds: E[y^2] - E[y]^2 from fp32-atomic Gram sums loses the variance of
            # near-constant channels, so their statistics come from a statistics-only conv pass instead (the
            # per-tile two-moment slabs of the unfolded path; the output is computed but never stored)
            eng.mark(self.name + ".foldexact")
            key = ("fg", yb.N, yb.T, yb.H, yb.W, yb.ld)
            g = self._geo.get(key)
            if g is None:
                g = self._geo[key] = fwd_geometry(s, yb.N, yb.T, yb.H, yb.W, yb.ld, Co)
            stats = eng.ws((self.name, "stats"), ((yb.M + 127) // 128, 2, Co), torch.float32)
            dummy = eng.ws(("nostore_y",), (1, 8), eng.cdt)
            tuner = eng.tuner
            aff = 2 if bxf.relu else 1

            def run(cfg, scratch):
                C.conv_igemm(yb.t, self.wf, dummy, tuner.scratch_like(stats) if scratch else stats, bxf.scale,
                             bxf.shift, aff, 0, g, s.chunk, cfg, None, 1)
            cfg = tuner.launch(("fst", aff) + tuple(g), g, s.chunk, run, aff=aff, direct=False)
            tiles = (yb.M + tuner.bm(cfg, Co) - 1) // tuner.bm(cfg, Co)
            C.bn_finalize(stats, tiles, Co, yb.M, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                          bn.num_batches_tracked, bn.momentum if bn.momentum is not None else 0.1, bn.eps,
                          self.mean, self.rstd, self.scale, self.shift, self.fin)

    def narrow_fold_stats(self, yb: Act, bxf: _Xf, train: bool):
        """BN statistics of a narrow folded conv_c (``_ResBlock.narrow_fold``) from a statistics-only conv pass over
        act_b(yb) (the output is computed, never stored); no Gram matrix — its backward recomputes yc
        (csrc/kernels/narrow_bwd.hip forms 1 and 2) instead of the algebraic fold backward."""
        eng, C, s = self.eng, self.eng.C, self.spec
        bn = self.bn
        if not train:
            C.bn_eval_affine(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, self.scale, self.shift)
            return
        Co = s.cout
        eng.mark(self.name + ".foldexact")
        key = ("fg", yb.N, yb.T, yb.H, yb.W, yb.ld)
        g = self._geo.get(key)
        if g is None:
            g = self._geo[key] = fwd_geometry(s, yb.N, yb.T, yb.H, yb.W, yb.ld, Co)
        stats = eng.ws((self.name, "stats"), ((yb.M + 127) // 128, 2, Co), torch.float32)
        dummy = eng.ws(("nostore_y",), (1, 8), eng.cdt)
        tuner = eng.tuner
        aff = 2 if bxf.relu else 1

        def run(cfg, scratch):
            C.conv_igemm(yb.t, self.wf, dummy, tuner.scratch_like(stats) if scratch else stats, bxf.scale,
                         bxf.shift, aff, 0, g, s.chunk, cfg, None, 1)
        cfg = tuner.launch(("fst", aff) + tuple(g), g, s.chunk, run, aff=aff, direct=False)
        tiles = (yb.M + tuner.bm(cfg, Co) - 1) // tuner.bm(cfg, Co)
        C.bn_finalize(stats, tiles, Co, yb.M, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                      bn.num_batches_tracked, bn.momentum if bn.momentum is not None else 0.1, bn.eps,
                      self.mean, self.rstd, self.scale, self.shift, self.fin)

    def fold_output(self, yb: Act, bxf: _Xf, out: torch.Tensor, res: Act, rxf: Optional[_Xf],
                    mask: torch.Tensor, tag: str) -> Act:
        """out = relu(BN(conv(act_b(yb))) + r), r = res (identity) or BN_1(res) (``rxf``); ReLU bits -> mask."""
        eng, C, s = self.eng, self.eng.C, self.spec
        eng.mark(self.name + ".fwdres")
        key = ("fg", yb.N, yb.T, yb.H, yb.W, yb.ld)
        g = self._geo.get(key)
        if g is None:
            g = self._geo[key] = fwd_geometry(s, yb.N, yb.T, yb.H, yb.W, yb.ld, out.stride(0))
        g = list(g)
        g[5] = out.stride(0)
        tuner = eng.tuner

        def run(cfg, scratch):
            C.conv_igemm_fres(yb.t, self.wf, tuner.scratch_like(out) if scratch else out, bxf.scale, bxf.shift,
                              2 if bxf.relu else 1, g, s.chunk, cfg, self.scale, self.shift, res.t, res.ld,
                              None if rxf is None else rxf.scale, None if rxf is None else rxf.shift,
                              tuner.scratch_like(mask) if scratch else mask)
        tuner.launch(("fres", rxf is not None) + tuple(g), g, s.chunk, run, aff=2, epi=False, direct=False)
        return Act(out, yb.N, yb.T, yb.H, yb.W)

    def fold_backward(self, dz: Act, part, tiles: int, yb: Act, b: "_ConvBN", dab: torch.Tensor):
        """BN_c + conv_c backward from dz without yc: G = dz^T act_b(yb) (wgrad kernel), coefficients, dWc,
        dgamma/dbeta (bnfold_bwd), then d act_b = act_b(yb) W2 + bias (1x1 conv) followed by the dgrad of dz with
        W1 = diag(A) Wc accumulated on top, whose epilogue applies b's ReLU mask and reduces b's BN-backward
        sums.  Returns (partials, tiles) for ``b.bn_backward(pre=...)``."""
        eng, C, s = self.eng, self.eng.C, self.spec
        c, Co = s.cin, s.cout
        bxf = b.xf()
        G = eng.scratch("fold_G", Co * c)
        self.wgrad(dz, yb, bxf, dest=G, beta=0.0)
        if getattr(self, "W1t", None) is None:
            self.W1t = torch.empty(c, Co, device=eng.device, dtype=eng.cdt)
            self.W2 = torch.empty(c, c, device=eng.device, dtype=eng.cdt)
            self.fbias = torch.empty(2 * c, device=eng.device, dtype=torch.float32)   # [biasA | biasB]
        fg = eng.flat
        eng.mark(self.name + ".foldbwd")
        C.bnfold_bwd(part, tiles, self.wf, self.wd, G, self.T, self.s, Co, c, dz.M, self.bn.weight, self.mean,
                     self.rstd, fg.gview(self.bn.weight), fg.gview(self.bn.bias), fg.gview(self.conv.weight),
                     eng.grad_beta, self.coef, self.W1t, self.W2, self.fbias)
        # (act_b(yb) - abar) W2 + c0 : a c->c 1x1 conv with the consumer-side BN_b fold and a bias epilogue
        if not hasattr(self, "gspec"):
            self.gspec = ConvSpec(c, c, (1, 1, 1), (1, 1, 1), (0, 0, 0))
        eng.mark(self.name + ".foldw2")
        g2 = fwd_geometry(self.gspec, yb.N, yb.T, yb.H, yb.W, yb.ld, c)
        tuner = eng.tuner

        def run(cfg, scratch):
            C.conv_igemm(yb.t, self.W2, tuner.scratch_like(dab) if scratch else dab, None, bxf.scale, bxf.shift,
                         2 if bxf.relu else 1, 0, g2, 8, cfg, self.fbias[c:])
        tuner.launch(("fw2",) + tuple(g2), g2, 8, run, aff=2, direct=False)
        return self.dgrad(dz, (yb.T, yb.H, yb.W), dab, True, bn=(b, yb), wd=self.W1t, bias=self.fbias[:c])

    # ---- backward BatchNorm folding of a stride-1 1x1 branch1 (same algebra as conv_c's, with a = x, no affine) ----
    def fold_branch1_forward(self, x: Act):
        """Gram matrix of the branch input x (wgrad kernel, Gram mode) -> T1 = W1 Gx and s1 = colsum(x), kept for the
        backward.  The branch's own BN statistics still come from its conv epilogue (y1 is materialised for the unit
        output); the fold's statistics outputs go to scratch (no running-stat update)."""
        eng, C, s = self.eng, self.eng.C, self.spec
        c, Co = s.cin, s.cout
        if not hasattr(self, "gspec"):
            self.gspec = ConvSpec(c, c, (1, 1, 1), (1, 1, 1), (0, 0, 0))
        Gx = eng.scratch("fold1_gram", c * c)
        slab = eng.scratch("fold_colsum", 4096 * c)
        if not hasattr(self, "ident"):   # the Gram mode of the wgrad kernel applies an input affine: identity here
            self.ident = _Xf(torch.ones(c, device=eng.device), torch.zeros(c, device=eng.device), relu=False)
        splits = self.wgrad(x, x, self.ident, spec=self.gspec, dest=Gx, beta=0.0, gram=True, colsum=slab)
        self.T = eng.ws((self.name, "foldT"), (Co, c), torch.float32)
        self.s = eng.ws((self.name, "folds"), (c,), torch.float32)
        dummy = eng.ws((self.name, "fold1_stats"), (4, Co), torch.float32)
        bn = self.bn
        eng.mark(self.name + ".foldstats")
        C.bnfold_fwd_stats(self.wf, Gx, slab, splits, Co, c, x.M, self.T, self.s, bn.weight, bn.bias, None, None,
                           None, 0.0, bn.eps, dummy[0], dummy[1], dummy[2], dummy[3])

    def fold_branch1_backward(self, dz: Act, part, tiles: int, x: Act, dx: torch.Tensor, dx_accum: bool):
        """Branch-1 backward from dz without dy1 or y1: G1 = dz^T x (wgrad kernel), then bnfold_bwd (BN_1 dgamma / dbeta,
        dW1, W1t = diag(A1) W1, W2 = W1^T diag(B1) W1, the split mean-correction biases); dx = x W2 + biasB (1x1
        c->c conv, written or accumulated per ``dx_accum``), then dx += dz W1t + biasA (dgrad)."""
        eng, C, s = self.eng, self.eng.C, self.spec
        c, Co = s.cin, s.cout
        G = eng.scratch("fold_G", Co * c)
        self.wgrad(dz, x, None, dest=G, beta=0.0)
        if getattr(self, "W1t", None) is None:
            self.W1t = torch.empty(c, Co, device=eng.device, dtype=eng.cdt)
            self.W2 = torch.empty(c, c, device=eng.device, dtype=eng.cdt)
            self.fbias = torch.empty(2 * c, device=eng.device, dtype=torch.float32)   # [biasA | biasB]
        fg = eng.flat
        eng.mark(self.name + ".foldbwd")
        C.bnfold_bwd(part, tiles, self.wf, self.wd, G, self.T, self.s, Co, c, dz.M, self.bn.weight, self.mean,
                     self.rstd, fg.gview(self.bn.weight), fg.gview(self.bn.bias), fg.gview(self.conv.weight),
                     eng.grad_beta, self.coef, self.W1t, self.W2, self.fbias)
        eng.mark(self.name + ".foldw2")
        g2 = fwd_geometry(self.gspec, x.N, x.T, x.H, x.W, x.ld, dx.stride(0))
        tuner = eng.tuner

        def run(cfg, scratch):
            C.conv_igemm(x.t, self.W2, tuner.scratch_like(dx) if scratch else dx, None, None, None, 0,
                         1 if dx_accum else 0, g2, 8, cfg, self.fbias[c:])
        tuner.launch(("fw2x", dx_accum) + tuple(g2), g2, 8, run, direct=False, halo=False)
        self.dgrad(dz, (x.T, x.H, x.W), dx, True, wd=self.W1t, bias=self.fbias[:c])

    def dgrad(self, dy: Act, in_dims, out: torch.Tensor, accum: bool, res: Optional[Act] = None,
              epi: Optional["_ResBlock"] = None, bn: Optional[Tuple["_ConvBN", Act]] = None,
              wd: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None):
        """grad wrt the conv input into ``out`` (``accum``: added).  With ``res`` / ``epi`` the single-phase
        launch also adds the residual gradient ``res``, applies the ReLU mask of residual unit ``epi``'s
        output and emits the partial sums of ``epi``'s conv_c (+branch1) BN backward; returns
        (partials, tiles) for ``epi.bwd(pre=...)``.  With ``bn = (unit, y)`` (this conv's input is
        relu(BN_unit(y))) it applies that ReLU mask and emits ``unit``'s BN-backward partial sums instead;
        returns (partials, tiles) for ``unit.bn_backward(pre=...)``, or None when not fusable."""
        s, C = self.spec, self.eng.C
        self.eng.mark(self.name + ".dgrad")
        wd = self.wd if wd is None else wd   # (BN folding passes diag(A)-scaled weights)
        Ti, Hi, Wi = in_dims
        key = ("dg", dy.N, tuple(in_dims), dy.ld, out.stride(0))
        geo = self._geo.get(key)
        if geo is None:
            geo = self._geo[key] = dgrad_phases(s, dy.N, tuple(in_dims), (dy.T, dy.H, dy.W), dy.ld, out.stride(0))
        tuner = self.eng.tuner
        if bn is not None and res is None and epi is None and len(geo) == 1:
            u, y = bn
            g = geo[0]
            part = self.eng.scratch("bnepi", ((g[0] + 127) // 128) * 3 * g[1])
            # accum: the scratch launches of the autotuner add onto garbage — harmless, outputs are discarded

            def run(cfg, scratch):
                C.conv_igemm_epi(dy.t, wd, tuner.scratch_like(out) if scratch else out, 1 if accum else 0, g, 8, None,
                                 0, None, y.t, u.mean, u.rstd, None, None, None,
                                 tuner.scratch_like(part) if scratch else part, u.scale, u.shift, cfg, bias)
            cfg = tuner.launch(("eb", accum, bias is not None) + tuple(g), g, 8, run, epi=True,
                               direct=bias is None)
            bm = tuner.bm(cfg, g[1])
            return part, (g[0] + bm - 1) // bm
        if res is not None or epi is not None:
            assert len(geo) == 1, "fused dgrad epilogue needs a single-phase (stride-1) dgrad"
            g = geo[0]
            part, c, one = None, None, None
            if epi is not None:
                part = self.eng.scratch("bnepi", ((g[0] + 127) // 128) * 3 * g[1])
                # folded branch1: its sums come from G1; narrow-fold unit: from its own reduce pass
                c, one = epi.c, (None if (epi.fold1 or epi.narrow_fold) else epi.one)

            yc = None if (epi is None or epi.yc is None) else epi.yc   # folded conv_c: no raw output

            def run(cfg, scratch):
                C.conv_igemm_epi(dy.t, wd, tuner.scratch_like(out) if scratch else out, 1 if accum else 0, g, 8,
                                 None if res is None else res.t, 0 if res is None else res.ld,
                                 None if epi is None else epi.mask, None if yc is None else yc.t,
                                 None if yc is None else c.mean, None if yc is None else c.rstd,
                                 None if epi is None or one is None else epi.y1.t,
                                 None if epi is None or one is None else one.mean,
                                 None if epi is None or one is None else one.rstd,
                                 None if part is None else (tuner.scratch_like(part) if scratch else part),
                                 None, None, cfg)
            cfg = tuner.launch(("er", accum, res is not None, epi is not None,
                                epi is not None and one is not None) + tuple(g), g, 8, run, epi=True)
            if epi is None:
                return None
            bm = tuner.bm(cfg, g[1])
            return part, (g[0] + bm - 1) // bm
        for g in geo:
            if accum and g[28] == 0:
                continue

            def run(cfg, scratch, g=g):
                C.conv_igemm(dy.t, wd, tuner.scratch_like(out) if scratch else out, None, None, None, 0,
                             1 if accum else 0, g, 8, cfg, bias)
            # (the direct kernel has no bias epilogue)
            tuner.launch(("d", accum, bias is not None) + tuple(g), g, 8, run, halo=not accum and bias is None,
                         direct=bias is None)
        return None

    def bn_backward(self, g: Act, y: Act, mask_mode: int, mo: Optional[Act], mxf: Optional[_Xf],
                    dz_out: Optional[Act] = None, dz_accum: bool = False, other: Optional["_ConvBN"] = None,
                    other_y: Optional[Act] = None, pre=None) -> Tuple[Act, Optional[Act]]:
        """dz = g*mask ; returns (dy_self, dy_other) for one or two BNs sharing dz.

        mask_mode 0: none, 1: ``mo`` (Act) > 0, 2: affine(y) > 0, 3: ``mo`` = uint8 ReLU bits [M, C/8].
        ``pre`` = (partials, tiles) already produced by a consumer dgrad epilogue: skips the reduce."""
        eng, C = self.eng, self.eng.C
        M, Cc = y.M, self.C
        if isinstance(mo, Act):
            mo_t, mo_ld = mo.t, mo.ld
        else:
            mo_t, mo_ld = mo, (0 if mo is None else mo.shape[1])
        if pre is not None:
            part, blocks = pre
        else:
            blocks, rpb = eng._bn_blocks(M, Cc)
            eng.mark(self.name + ".bnred")
            part = eng.scratch("bnpart", blocks * 3 * Cc)
            C.bn_bwd_reduce(g.t, g.ld, mask_mode, mo_t, mo_ld,
                            None if mxf is None else mxf.scale, None if mxf is None else mxf.shift,
                            y.t, self.mean, self.rstd,
                            None if other is None else other_y.t, None if other is None else other.mean,
                            None if other is None else other.rstd, M, Cc, blocks, rpb, part)
        fg = eng.flat
        C.bn_bwd_finalize(part, blocks, Cc, M, 0, self.bn.weight, self.mean, self.rstd,
                          fg.gview(self.bn.weight), fg.gview(self.bn.bias), eng.grad_beta, self.coef, self.fin)
        if other is not None:
            C.bn_bwd_finalize(part, blocks, Cc, M, 1, other.bn.weight, other.mean, other.rstd,
                              fg.gview(other.bn.weight), fg.gview(other.bn.bias), eng.grad_beta, other.coef,
                              other.fin)
        dy = eng.ws((self.name, "dy"), (M, Cc), eng.cdt)
        dy1 = eng.ws((other.name, "dy"), (M, Cc), eng.cdt) if other is not None else None
        eng.mark(self.name + ".bnapply")
        C.bn_bwd_apply(g.t, g.ld, mask_mode, mo_t, mo_ld,
                       None if mxf is None else mxf.scale, None if mxf is None else mxf.shift,
                       y.t, self.coef, dy, None if other is None else other_y.t,
                       None if other is None else other.coef, dy1,
                       None if dz_out is None else dz_out.t, 0 if dz_out is None else dz_out.ld,
                       1 if dz_accum else 0, M, Cc)
        a = Act(dy, y.N, y.T, y.H, y.W)
        b = Act(dy1, y.N, y.T, y.H, y.W) if other is not None else None
        return a, b


def to_s2d(x_ncthw: torch.Tensor, dtype: torch.dtype = torch.bfloat16) -> Act:
    """NCTHW float clip -> space-to-depth stem input: 2x2 pixel blocks x RGB0 = 16 channels of ``dtype``."""
    N, C, T, H, W = x_ncthw.shape
    x = F.pad(x_ncthw, (0, 0, 0, 0, 0, 0, 0, 4 - C))                  # RGB0
    x = x.reshape(N, 4, T, H // 2, 2, W // 2, 2).permute(0, 2, 3, 5, 4, 6, 1)  # N,T,Hs,Ws,sy,sx,c
    x = x.reshape(N * T * (H // 2) * (W // 2), 16).contiguous().to(dtype)
    return Act(x, N, T, H // 2, W // 2)


class _Stem:
    """conv(kt,7,7)/s(1,2,2) + BN + ReLU + MaxPool(1,3,3)/s2.

    With ``eng.stem_s2d`` the conv runs as the direct space-to-depth kernel (csrc/kernels/stem_s2d.hip)
    on an s2d input Act (C = 16, H/2 x W/2); otherwise as a generic implicit GEMM on RGB0 input."""

    def __init__(self, eng, stem: R.ResNetBasicStem, name: str):
        self.u = _ConvBN(eng, stem.conv, stem.norm, name + ".conv", cin_pad=4)
        self.eng, self.name = eng, name
        self.units = [self.u]
        k = tuple(stem.conv.kernel_size)
        self.kt = k[0]
        self.s2d = (eng.stem_s2d and k[1:] == (7, 7) and tuple(stem.conv.stride) == (1, 2, 2)
                    and tuple(stem.conv.padding) == (self.kt // 2, 3, 3) and stem.conv.in_channels == 3
                    and eng.C.stem_supported(self.u.C, self.kt))
        if self.s2d:
            cpad = (self.u.C + 15) // 16 * 16
            self.wpack = torch.zeros(cpad * self.kt * 256, device=eng.device, dtype=eng.cdt)

    def out_channels(self):
        return self.u.C

    def out_dims(self, T, H, W):
        if self.s2d:  # input dims are the s2d grid = conv output grid
            return T, (H - 1) // 2 + 1, (W - 1) // 2 + 1
        To, Ho, Wo = self.u.spec.out_dims(T, H, W)
        return To, (Ho - 1) // 2 + 1, (Wo - 1) // 2 + 1

    def pack(self):
        if self.s2d:
            self.eng.C.stem_pack(self.eng.flat.view(self.u.conv.weight), self.wpack, self.u.C, self.kt)

    def _conv_s2d(self, x: Act, train: bool, tag: str) -> Act:
        eng, C, u = self.eng, self.eng.C, self.u
        assert x.C == 16 and x.t.is_contiguous(), "s2d stem expects a dense [M, 16] space-to-depth input"
        M = x.M
        y = eng.ws((u.name, "y", tag), (M, u.C), eng.cdt)
        tiles = C.stem_tiles(x.H, x.W, x.N)
        stats = eng.ws((u.name, "stats"), (tiles, 2, u.C), torch.float32)
        eng.mark(u.name + ".fwd")
        C.stem_fwd(x.t, self.wpack, y, stats, [x.N, x.T, x.H, x.W], u.C, self.kt)
        bn = u.bn
        if train:
            C.bn_finalize(stats, tiles, u.C, M, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                          bn.num_batches_tracked, bn.momentum if bn.momentum is not None else 0.1, bn.eps,
                          u.mean, u.rstd, u.scale, u.shift, u.fin)
        else:
            C.bn_eval_affine(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, u.scale, u.shift)
        return Act(y, x.N, x.T, x.H, x.W)

    def fwd(self, x: Act, out: torch.Tensor, train: bool, tag: str) -> Act:
        C = self.eng.C
        y = self._conv_s2d(x, train, tag) if self.s2d else self.u.fwd(x, None, train, tag)
        Ho, Wo = (y.H - 1) // 2 + 1, (y.W - 1) // 2 + 1
        P = y.N * y.T * Ho * Wo
        arg = self.eng.ws((self.name, "arg"), (P, self.u.C), torch.uint8)
        # training: also the raw y at every window argmax — the BN-backward sums are then taken on the pooled grid
        ymax = self.eng.ws((self.name, "ymax"), (P, self.u.C), self.eng.cdt) if train else None
        self.eng.mark(self.name + ".pool")
        C.stem_pool_fwd(y.t, self.u.scale, self.u.shift, out, out.stride(0), arg, y.N * y.T, y.H, y.W, Ho, Wo,
                        self.u.C, ymax)
        self.x, self.y, self.arg, self.ymax = x, y, arg, ymax
        return Act(out, y.N, y.T, Ho, Wo)

    def bwd(self, dout: Act):
        """Max-pool + ReLU + BN backward without materialising the full-resolution dz: the BN sums come from the
        pooled grid (dout and the raw y at each argmax), then one kernel gathers dz through the argmax bytes and
        writes dy = A dz mask + B y + C (csrc/kernels/bn_eltwise.hip stem_pool_bn_apply)."""
        eng, C, u = self.eng, self.eng.C, self.u
        y = self.y
        assert self.ymax is not None, "stem backward needs a training-mode forward"
        P = dout.M
        blocks, rpb = eng._bn_blocks(P, u.C)
        eng.mark(u.name + ".bnred")
        part = eng.scratch("bnpart", blocks * 3 * u.C)
        C.bn_bwd_reduce(dout.t, dout.ld, 2, None, 0, u.scale, u.shift, self.ymax, u.mean, u.rstd, None, None, None,
                        P, u.C, blocks, rpb, part)
        fg = eng.flat
        C.bn_bwd_finalize(part, blocks, u.C, y.M, 0, u.bn.weight, u.mean, u.rstd, fg.gview(u.bn.weight),
                          fg.gview(u.bn.bias), eng.grad_beta, u.coef, u.fin)
        dyt = eng.ws((u.name, "dy"), (y.M, u.C), eng.cdt)
        eng.mark(self.name + ".poolbwd")
        C.stem_pool_bn_apply(dout.t, dout.ld, self.arg, y.t, u.scale, u.shift, u.coef, dyt, y.N * y.T, y.H, y.W,
                             dout.H, dout.W, u.C)
        dy = Act(dyt, y.N, y.T, y.H, y.W)
        if self.s2d:
            x = self.x
            acc = eng.scratch("stem_acc_" + self.name, self.u.C * self.kt * 256, zero=True)
            eng.mark(self.u.name + ".wgrad")
            slab = None
            if eng.reproducible:   # per-workgroup partials summed in a fixed order instead of fp32 atomics
                slab = eng.scratch("stem_slab_" + self.name,
                                   C.stem_tiles(x.H, x.W, x.N) * self.u.C * self.kt * 256)
            C.stem_wgrad(x.t, dy.t, acc, [x.N, x.T, x.H, x.W], self.u.C, self.kt, slab)
            C.stem_wgrad_convert(acc, eng.flat.gview(self.u.conv.weight), self.u.C, self.kt, eng.grad_beta)
        else:
            self.u.wgrad(dy, self.x, None)


class _ResBlock:
    def __init__(self, eng, blk: R.ResBlock, name: str):
        b2 = blk.branch2
        self.eng, self.name = eng, name
        self.a = _ConvBN(eng, b2.conv_a, b2.norm_a, name + ".a")
        self.b = _ConvBN(eng, b2.conv_b, b2.norm_b, name + ".b")
        self.c = _ConvBN(eng, b2.conv_c, b2.norm_c, name + ".c")
        self.one = _ConvBN(eng, blk.branch1_conv, blk.branch1_norm, name + ".1") if blk.branch1_conv is not None else None
        self.units = [u for u in (self.a, self.b, self.c, self.one) if u is not None]
        sc = self.c.spec
        # BN folding of the 1x1 conv_c: its raw output (the widest tensor of the unit) is never written
        self.fold = (eng.bn_fold and tuple(sc.k) == (1, 1, 1) and tuple(sc.stride) == (1, 1, 1) and sc.cin % 8 == 0
                     and sc.cout % 8 == 0 and sc.cin >= eng.fold_min_c)
        # BN folding of a stride-1 1x1 branch1 in the BACKWARD (slow res2 unit 0): its BN backward and weight/input
        # gradients come from G1 = dz^T x and the Gram matrix of x (_ConvBN.fold_branch1_*), so neither the
        # branch-1 BN-backward apply pass (dy1) nor the dual y1 read in the next unit's dgrad epilogue happens
        # narrow unfolded 1x1 conv_c (fast res2: 8 -> 32): fused BN-apply + wgrad + dgrad backward (_bwd_narrow)
        self.narrow_c = (not self.fold and eng.narrow_bwd and tuple(sc.k) == (1, 1, 1) and tuple(sc.stride) == (1, 1, 1)
                         and sc.cin == 8 and sc.cin_pad == 8 and bool(eng.C.narrow_c_bwd_legal(sc.cout, sc.cin)))
        # ... and BN-folded in the forward: the unit output is written by fold_output (no raw yc, no res_out pass);
        # the backward recomputes yc from act_b (a reduce pass + the fused pass)
        self.narrow_fold = self.narrow_c and eng.narrow_fold
        s1 = self.one.spec if self.one is not None else None
        self.fold1 = (self.fold and s1 is not None and eng.bn_fold1 and tuple(s1.k) == (1, 1, 1)
                      and tuple(s1.stride) == (1, 1, 1) and s1.cin % 8 == 0 and s1.cin == s1.cin_pad
                      and s1.cin <= 2048)

    def out_channels(self):
        return self.c.C

    def out_dims(self, T, H, W):
        return self.b.spec.out_dims(T, H, W)

    def fwd(self, x: Act, out: torch.Tensor, train: bool, tag: str) -> Act:
        C = self.eng.C
        ya = self.a.fwd(x, None, train, tag)
        yb = self.b.fwd(ya, self.a.xf(), train, tag)
        if self.fold:
            # conv_c statistics from the Gram matrix of act_b(yb), then ONE launch writes the unit output
            # relu(BN_c(conv_c) + shortcut) and its ReLU bits (no yc, no res_out pass)
            y1 = self.one.fwd(x, None, train, tag) if self.one is not None else None
            if self.fold1 and train:
                self.one.fold_branch1_forward(x)
            self.c.fold_forward(yb, self.b.xf(), train)
            mask = self.eng.ws((self.name, "mask", tag), (yb.M, self.c.C // 8), torch.uint8)
            res, rxf = (x, None) if y1 is None else (y1, self.one.xf(relu=False))
            o = self.c.fold_output(yb, self.b.xf(), out, res, rxf, mask, tag)
            self.mask = mask if train else None
            self.x, self.ya, self.yb, self.yc, self.y1, self.out = x, ya, yb, None, y1, o
            return o
        if self.narrow_fold:
            y1 = self.one.fwd(x, None, train, tag) if self.one is not None else None
            self.c.narrow_fold_stats(yb, self.b.xf(), train)
            mask = self.eng.ws((self.name, "mask", tag), (yb.M, self.c.C // 8), torch.uint8)
            res, rxf = (x, None) if y1 is None else (y1, self.one.xf(relu=False))
            o = self.c.fold_output(yb, self.b.xf(), out, res, rxf, mask, tag)
            self.mask = mask if train else None
            self.x, self.ya, self.yb, self.yc, self.y1, self.out = x, ya, yb, None, y1, o
            return o
        yc = self.c.fwd(yb, self.b.xf(), train, tag)
        y1 = self.one.fwd(x, None, train, tag) if self.one is not None else None
        M = yc.M
        self.eng.mark(self.name + ".res_out")
        mask = self.eng.ws((self.name, "mask"), (M, self.c.C // 8), torch.uint8) if train else None
        C.res_out(yc.t, self.c.scale, self.c.shift,
                  None if y1 is None else y1.t, None if y1 is None else self.one.scale,
                  None if y1 is None else self.one.shift, None if y1 is not None else x.t, x.ld,
                  out, out.stride(0), M, self.c.C, mask)
        self.mask = mask
        o = Act(out, yc.N, yc.T, yc.H, yc.W)
        self.x, self.ya, self.yb, self.yc, self.y1, self.out = x, ya, yb, yc, y1, o
        return o

    def bwd(self, dout: Act, dx: torch.Tensor, dx_accum: bool, pre=None, prev: Optional["_ResBlock"] = None):
        """dout: grad wrt block output; dx: [M_in, C_in] buffer receiving grad wrt block input.

        ``pre``: ``dout`` is already the ReLU-masked gradient and its conv_c/branch1 BN partial sums were
        emitted by the following unit's conv_a dgrad epilogue.  ``prev``: the preceding unit of the same
        stage — this unit's final dgrad then produces ``prev``'s masked gradient and partial sums (returned,
        to be passed as ``prev.bwd(pre=...)``)."""
        eng = self.eng
        x, ya, yb, yc, y1 = self.x, self.ya, self.yb, self.yc, self.y1
        dxa = Act(dx, x.N, x.T, x.H, x.W)
        res = None
        if self.fold:
            return self._bwd_fold(dout, dx, dx_accum, pre, prev)
        if self.narrow_c:
            return self._bwd_narrow(dout, dx, dx_accum, pre, prev)
        if pre is not None:
            dyc, dy1 = self.c.bn_backward(dout, yc, 0, None, None, other=self.one, other_y=y1, pre=pre)
            if self.one is None:
                res = dout          # identity shortcut: the masked gradient is added by conv_a's dgrad
        elif self.one is None:
            # identity shortcut: dz goes straight to dx
            dyc, _ = self.c.bn_backward(dout, yc, 3, self.mask, None, dz_out=dxa, dz_accum=dx_accum)
        else:
            dyc, dy1 = self.c.bn_backward(dout, yc, 3, self.mask, None, other=self.one, other_y=y1)
        self.c.wgrad(dyc, yb, self.b.xf())
        dab = eng.ws((self.name, "dab"), (yb.M, self.b.C), eng.cdt)
        # the dgrad epilogues apply the b / a ReLU masks and reduce their BN-backward sums (no separate pass)
        pb = self.c.dgrad(dyc, (yb.T, yb.H, yb.W), dab, False, bn=(self.b, yb))
        dyb, _ = self.b.bn_backward(Act(dab, yb.N, yb.T, yb.H, yb.W), yb, 0 if pb else 2, None,
                                    None if pb else self.b.xf(), pre=pb)
        self.b.wgrad(dyb, ya, self.a.xf())
        daa = eng.ws((self.name, "daa"), (ya.M, self.a.C), eng.cdt)
        pa = self.b.dgrad(dyb, (ya.T, ya.H, ya.W), daa, False, bn=(self.a, ya))
        dya, _ = self.a.bn_backward(Act(daa, ya.N, ya.T, ya.H, ya.W), ya, 0 if pa else 2, None,
                                    None if pa else self.a.xf(), pre=pa)
        self.a.wgrad(dya, x, None)
        if self.one is not None:
            self.one.wgrad(dy1, x, None)
            if self._strided_one(prev):
                return self._dgrad_strided_one(dya, dy1, dx, dx_accum)
            self.one.dgrad(dy1, (x.T, x.H, x.W), dx, dx_accum)
            acc = True
        else:
            acc = dx_accum if pre is not None else True
        if prev is not None and not self._epi_ok(prev):
            prev = None
        if res is None and prev is None:
            self.a.dgrad(dya, (x.T, x.H, x.W), dx, acc)
            return None
        return self.a.dgrad(dya, (x.T, x.H, x.W), dx, acc, res=res, epi=prev)

    def _bwd_narrow(self, dout: Act, dx: torch.Tensor, dx_accum: bool, pre, prev: Optional["_ResBlock"]):
        """Backward of a unit with a narrow, unfolded 1x1 conv_c (fast res2: 8 -> 32): the BN_c backward apply, the
        conv_c weight gradient and its input gradient (with BN_b's ReLU mask and BN-backward partial sums) in ONE
        streaming pass (csrc/kernels/narrow_bwd.hip), so dyc never reaches HBM; branch1's dy1 keeps its own apply."""
        eng, C = self.eng, self.eng.C
        x, ya, yb, yc, y1, one, c = self.x, self.ya, self.yb, self.yc, self.y1, self.one, self.c
        dxa = Act(dx, x.N, x.T, x.H, x.W)
        M, Cc = yb.M, c.C
        fg = eng.flat
        res = None
        rps = int(C.narrow_c_bwd_rps(M, Cc, eng.narrow_splits))
        splits = (M + rps - 1) // rps
        b = self.b
        if self.narrow_fold:
            # no yc: the BN_c (and BN_1) backward sums come from a reduce pass that recomputes yc from act_b
            if pre is not None:
                mode, mask, dz_out = 0, None, None
                if one is None:
                    res = dout
            else:
                mode, mask = 3, self.mask
                dz_out = dxa if one is None else None
            part = eng.scratch("narrow_cpart", splits * 3 * Cc)
            blocks = splits
            eng.mark(c.name + ".foldred")
            C.narrow_c_bwd(dout.t, dout.ld, mode, mask, None, c.coef, None, 0, 0, yb.t, b.scale, b.shift, b.mean,
                           b.rstd, c.wf, None, 8, 0, None, None, M, Cc, yb.C, rps, form=2,
                           y1=None if one is None else y1.t, mc=c.mean, rc=c.rstd,
                           m1=None if one is None else one.mean, r1=None if one is None else one.rstd, cpart=part)
        elif pre is not None:   # dout is the masked dz, its partial sums came from the next unit's dgrad epilogue
            part, blocks = pre
            mode, mask, dz_out = 0, None, None
            if one is None:
                res = dout
        else:
            mode, mask = 3, self.mask
            blocks, rpb = eng._bn_blocks(M, Cc)
            eng.mark(c.name + ".bnred")
            part = eng.scratch("bnpart", blocks * 3 * Cc)
            C.bn_bwd_reduce(dout.t, dout.ld, 3, self.mask, Cc // 8, None, None, yc.t, c.mean, c.rstd,
                            None if one is None else y1.t, None if one is None else one.mean,
                            None if one is None else one.rstd, M, Cc, blocks, rpb, part)
            dz_out = dxa if one is None else None
        C.bn_bwd_finalize(part, blocks, Cc, M, 0, c.bn.weight, c.mean, c.rstd, fg.gview(c.bn.weight),
                          fg.gview(c.bn.bias), eng.grad_beta, c.coef, c.fin)
        dy1 = None
        s1 = one.spec if one is not None else None
        # branch1 (8 -> 32, stride 1, input = the unit input activation): the same fused pass, without the input
        # affine / mask, accumulating into dx (after conv_a's weight gradient, before its dgrad)
        one_fused = (one is not None and tuple(s1.k) == (1, 1, 1) and tuple(s1.stride) == (1, 1, 1) and s1.cin == 8
                     and s1.cin_pad == 8 and x.ld == 8 and bool(C.narrow_c_bwd_legal(s1.cout, s1.cin)))
        if one is not None:
            C.bn_bwd_finalize(part, blocks, Cc, M, 1, one.bn.weight, one.mean, one.rstd, fg.gview(one.bn.weight),
                              fg.gview(one.bn.bias), eng.grad_beta, one.coef, one.fin)
            if not one_fused:
                dy1 = eng.ws((one.name, "dy"), (M, Cc), eng.cdt)
                eng.mark(one.name + ".bnapply")
                C.bn_bwd_apply(dout.t, dout.ld, mode, mask, Cc // 8 if mask is not None else 0, None, None, None,
                               None, None, y1.t, one.coef, dy1, None, 0, 0, M, Cc)
        dab = eng.ws((self.name, "dab"), (yb.M, self.b.C), eng.cdt)
        slab = eng.scratch("narrow_slab", splits * Cc * yb.C)
        partb = eng.scratch("narrow_part", splits * 3 * yb.C)
        eng.mark(c.name + ".fusedbwd")
        C.narrow_c_bwd(dout.t, dout.ld, mode, mask, None if yc is None else yc.t, c.coef,
                       None if dz_out is None else dz_out.t, 0 if dz_out is None else dz_out.ld,
                       1 if (dz_out is not None and dx_accum) else 0, yb.t, b.scale, b.shift, b.mean, b.rstd, c.wf, dab,
                       yb.C, 0, slab, partb, M, Cc, yb.C, rps, form=1 if self.narrow_fold else 0)
        C.wgrad_reduce(slab, fg.gview(c.conv.weight), splits, Cc, 1, c.spec.cin_pad, c.spec.cin, 1.0,
                       eng.grad_beta, 1)
        dyb, _ = b.bn_backward(Act(dab, yb.N, yb.T, yb.H, yb.W), yb, 0, None, None, pre=(partb, splits))
        b.wgrad(dyb, ya, self.a.xf())
        daa = eng.ws((self.name, "daa"), (ya.M, self.a.C), eng.cdt)
        pa = b.dgrad(dyb, (ya.T, ya.H, ya.W), daa, False, bn=(self.a, ya))
        dya, _ = self.a.bn_backward(Act(daa, ya.N, ya.T, ya.H, ya.W), ya, 0 if pa else 2, None,
                                    None if pa else self.a.xf(), pre=pa)
        self.a.wgrad(dya, x, None)
        if one is not None and one_fused:
            eng.mark(one.name + ".fusedbwd")
            slab1 = eng.scratch("narrow_slab", splits * Cc * x.C)
            C.narrow_c_bwd(dout.t, dout.ld, mode, mask, y1.t, one.coef, None, 0, 0, x.t, None, None, None, None,
                           one.wf, dx, dx.stride(0), 1 if dx_accum else 0, slab1, None, M, Cc, x.C, rps, form=0)
            C.wgrad_reduce(slab1, fg.gview(one.conv.weight), splits, Cc, 1, s1.cin_pad, s1.cin, 1.0,
                           eng.grad_beta, 1)
            acc = True
        elif one is not None:
            d1 = Act(dy1, x.N, yb.T, yb.H, yb.W)
            one.wgrad(d1, x, None)
            if self._strided_one(prev):
                return self._dgrad_strided_one(dya, d1, dx, dx_accum)
            one.dgrad(d1, (x.T, x.H, x.W), dx, dx_accum)
            acc = True
        else:
            acc = dx_accum if pre is not None else True
        if prev is not None and not self._epi_ok(prev):
            prev = None
        if res is None and prev is None:
            self.a.dgrad(dya, (x.T, x.H, x.W), dx, acc)
            return None
        return self.a.dgrad(dya, (x.T, x.H, x.W), dx, acc, res=res, epi=prev)

    def _bwd_fold(self, dout: Act, dx: torch.Tensor, dx_accum: bool, pre, prev: Optional["_ResBlock"]):
        """Backward of a unit whose conv_c BN is folded (see ``_ConvBN.fold_backward``)."""
        eng, C = self.eng, self.eng.C
        x, ya, yb, y1, one = self.x, self.ya, self.yb, self.y1, self.one
        dxa = Act(dx, x.N, x.T, x.H, x.W)
        M, Cc = yb.M, self.c.C
        fg = eng.flat
        res = None
        fold1 = self.fold1
        dy1 = eng.ws((one.name, "dy"), (M, Cc), eng.cdt) if (one is not None and not fold1) else None
        if pre is not None:
            # dout is already the masked dz; its partial sums came from the next unit's dgrad epilogue
            part, tiles = pre
            dz = dout
            if one is None:
                res = dout          # identity shortcut: added by conv_a's dgrad below
        else:
            # dz = dout * ReLU bits, with sum(dz) (+ the branch1 BN's sum(dz xhat1)) reduced in one pass
            blocks, rpb = eng._bn_blocks(M, Cc)
            eng.mark(self.c.name + ".bnred")
            part = eng.scratch("bnpart", blocks * 3 * Cc)
            # identity shortcut: the same pass writes dz = dout * bits into dx (conv_a's dgrad accumulates on it)
            dual = one is not None and not fold1
            dzb = None
            if one is not None and fold1:   # the folded branch1 needs dz itself: the same pass writes it
                dzb = Act(eng.ws((self.name, "dz"), (M, Cc), eng.cdt), x.N, yb.T, yb.H, yb.W)
            C.bn_bwd_reduce(dout.t, dout.ld, 3, self.mask, Cc // 8, None, None, None, None, None,
                            y1.t if dual else None, one.mean if dual else None,
                            one.rstd if dual else None, M, Cc, blocks, rpb, part,
                            dxa.t if one is None else (dzb.t if dzb is not None else None),
                            dxa.ld if one is None else (dzb.ld if dzb is not None else 0))
            tiles = blocks
            if one is None:
                assert not dx_accum, "identity unit with an accumulating input gradient"
                dz = dxa
            elif dzb is not None:
                dz = dzb
            else:
                dz = Act(eng.ws((self.name, "dz"), (M, Cc), eng.cdt), x.N, yb.T, yb.H, yb.W)
        if one is not None and fold1:
            # branch1 first: it consumes the dz partials (`part`) before the conv_c dgrad epilogue reuses that scratch
            one.fold_branch1_backward(dz, part, tiles, x, dx, dx_accum)
        elif one is not None:
            # branch1 BN backward from the same sums: dy1 = A1 dz + B1 y1 + C1 (and dz itself when not yet stored)
            C.bn_bwd_finalize(part, tiles, Cc, M, 1, one.bn.weight, one.mean, one.rstd, fg.gview(one.bn.weight),
                              fg.gview(one.bn.bias), eng.grad_beta, one.coef, one.fin)
            eng.mark(one.name + ".bnapply")
            if pre is not None:
                C.bn_bwd_apply(dz.t, dz.ld, 0, None, 0, None, None, None, None, None, y1.t, one.coef, dy1, None, 0,
                               0, M, Cc)
            else:
                C.bn_bwd_apply(dout.t, dout.ld, 3, self.mask, Cc // 8, None, None, None, None, None, y1.t, one.coef,
                               dy1, dz.t, dz.ld, 0, M, Cc)
        dab = eng.ws((self.name, "dab"), (yb.M, self.b.C), eng.cdt)
        pb = self.c.fold_backward(dz, part, tiles, yb, self.b, dab)
        dyb, _ = self.b.bn_backward(Act(dab, yb.N, yb.T, yb.H, yb.W), yb, 0, None, None, pre=pb)
        self.b.wgrad(dyb, ya, self.a.xf())
        daa = eng.ws((self.name, "daa"), (ya.M, self.a.C), eng.cdt)
        pa = self.b.dgrad(dyb, (ya.T, ya.H, ya.W), daa, False, bn=(self.a, ya))
        dya, _ = self.a.bn_backward(Act(daa, ya.N, ya.T, ya.H, ya.W), ya, 0 if pa else 2, None,
                                    None if pa else self.a.xf(), pre=pa)
        self.a.wgrad(dya, x, None)
        if one is not None and fold1:
            acc = True   # dx already holds the folded branch1's input gradient
        elif one is not None:
            d1 = Act(dy1, x.N, yb.T, yb.H, yb.W)
            one.wgrad(d1, x, None)
            if self._strided_one(prev):
                return self._dgrad_strided_one(dya, d1, dx, dx_accum)
            one.dgrad(d1, (x.T, x.H, x.W), dx, dx_accum)
            acc = True
        else:
            acc = dx_accum if pre is not None else True
        if prev is not None and not self._epi_ok(prev):
            prev = None
        if res is None and prev is None:
            self.a.dgrad(dya, (x.T, x.H, x.W), dx, acc)
            return None
        return self.a.dgrad(dya, (x.T, x.H, x.W), dx, acc, res=res, epi=prev)

    def _strided_one(self, prev) -> bool:
        """Spatially strided branch1 and no fused epilogue on conv_a's dgrad (first unit of a stage)."""
        return (self.one is not None and tuple(self.one.spec.stride) != (1, 1, 1)
                and tuple(self.a.spec.stride) == (1, 1, 1) and (prev is None or not self._epi_ok(prev)))

    def _dgrad_strided_one(self, dya: Act, dy1: Act, dx: torch.Tensor, dx_accum: bool):
        """conv_a's dgrad covers every input position, the strided 1x1 branch1 only the stride-phase positions:
        writing conv_a's first and accumulating branch1's second touches dx once in full plus once at those
        positions (the other order writes zeros at 3/4 of dx and then reads + rewrites all of it)."""
        x = self.x
        self.a.dgrad(dya, (x.T, x.H, x.W), dx, dx_accum)
        self.one.dgrad(dy1, (x.T, x.H, x.W), dx, True)
        return None

    def _epi_ok(self, prev: "_ResBlock") -> bool:
        s = self.a.spec
        return (tuple(s.stride) == (1, 1, 1) and prev.out.t.is_contiguous() and prev.c.C % 8 == 0
                and prev.mask is not None)


class _Stage:
    def __init__(self, eng, stage: R.ResStage, name: str):
        self.blocks = [_ResBlock(eng, b, f"{name}.{i}") for i, b in enumerate(stage.res_blocks)]
        self.eng, self.name = eng, name
        self.units = [u for b in self.blocks for u in b.units]

    def out_channels(self):
        return self.blocks[-1].out_channels()

    def out_dims(self, T, H, W):
        for b in self.blocks:
            T, H, W = b.out_dims(T, H, W)
        return T, H, W

    def fwd(self, x: Act, out: torch.Tensor, train: bool, tag: str) -> Act:
        eng = self.eng
        for i, b in enumerate(self.blocks):
            if i == len(self.blocks) - 1:
                o = out
            else:
                T, H, W = b.out_dims(x.T, x.H, x.W)
                o = eng.ws((b.name, "out", tag), (x.N * T * H * W, b.out_channels()), eng.cdt)
            x = b.fwd(x, o, train, tag)
        return x

    def bwd(self, dout: Act, dx: torch.Tensor, dx_accum: bool):
        eng = self.eng
        pre = None
        for i in range(len(self.blocks) - 1, -1, -1):
            b = self.blocks[i]
            if i == 0:
                tgt, acc = dx, dx_accum
            else:
                xin = b.x
                tgt, acc = eng.ws((b.name, "dx"), (xin.M, xin.C), eng.cdt), False
            pre = b.bwd(dout, tgt, acc, pre=pre, prev=self.blocks[i - 1] if i > 0 else None)
            b.eng_progress(b.flat_hi)
            if i > 0:
                xin = b.x
                dout = Act(tgt, xin.N, xin.T, xin.H, xin.W)


class _Fuse:
    def __init__(self, eng, f: R.FuseFastToSlow, name: str):
        self.u = _ConvBN(eng, f.conv_fast_to_slow, f.norm, name)
        self.eng, self.name = eng, name
        self.units = [self.u]
        self.lateral_used = False   # the last backward ran the fused lateral kernel

    def fwd(self, xf: Act, cat_slice: torch.Tensor, train: bool, tag: str):
        y = self.u.fwd(xf, None, train, tag)
        self.eng.mark(self.name + ".bn_act")
        self.eng.C.bn_act(y.t, y.ld, cat_slice, cat_slice.stride(0), self.u.scale, self.u.shift, 1, y.M, self.u.C)
        self.xf_in, self.y = xf, y

    def _lateral_ok(self, x: Act, dcat_slice: Act, dfast: torch.Tensor) -> bool:
        s, y = self.u.spec, self.y
        return (self.eng.lateral_bwd and tuple(s.k[1:]) == (1, 1) and tuple(s.stride[1:]) == (1, 1)
                and tuple(s.pad[1:]) == (0, 0) and s.cin_pad == s.cin and (y.H, y.W) == (x.H, x.W)
                and dcat_slice.ld % 8 == 0 and dfast.stride(0) % 8 == 0
                and bool(self.eng.C.lateral_bwd_legal(s.cout, s.cin, s.stride[0], y.T, x.T, s.k[0], s.pad[0])))

    def bwd(self, dcat_slice: Act, dfast: torch.Tensor):
        """dcat_slice: grad wrt the fusion output slice; accumulates into dfast (grad wrt fast input).

        Fused path (csrc/kernels/lateral_bwd.hip): after the BN-backward reduce, one kernel applies the BN backward
        and accumulates the strided temporal input gradient (dy formed in registers, every dx frame read and written
        once); it also stores dy for the weight gradient.  Otherwise: apply, weight gradient, stride-phase dgrad."""
        y, u, eng = self.y, self.u, self.eng
        x = self.xf_in
        self.lateral_used = self._lateral_ok(x, dcat_slice, dfast)
        if self.lateral_used:
            C = eng.C
            M, Cc = y.M, u.C
            blocks, rpb = eng._bn_blocks(M, Cc)
            eng.mark(u.name + ".bnred")
            part = eng.scratch("bnpart", blocks * 3 * Cc)
            C.bn_bwd_reduce(dcat_slice.t, dcat_slice.ld, 2, None, 0, u.scale, u.shift, y.t, u.mean, u.rstd,
                            None, None, None, M, Cc, blocks, rpb, part)
            fg = eng.flat
            C.bn_bwd_finalize(part, blocks, Cc, M, 0, u.bn.weight, u.mean, u.rstd, fg.gview(u.bn.weight),
                              fg.gview(u.bn.bias), eng.grad_beta, u.coef, u.fin)
            dy = eng.ws((u.name, "dy"), (M, Cc), eng.cdt)
            eng.mark(self.name + ".latbwd")
            C.lateral_bwd(dcat_slice.t, dcat_slice.ld, y.t, u.scale, u.shift, u.coef, u.wd, dy, dfast,
                          dfast.stride(0), x.N, y.T, x.T, y.H * y.W, Cc, u.spec.cin, u.spec.stride[0])
            u.wgrad(Act(dy, y.N, y.T, y.H, y.W), x, None)
            return
        dy, _ = u.bn_backward(dcat_slice, y, 2, None, u.xf())
        u.wgrad(dy, x, None)
        u.dgrad(dy, (x.T, x.H, x.W), dfast, True)


class FusedNet:
    """Executor bound to a reference ``Net`` (SlowFast or Slow ResNet3D) whose parameters it shares."""

    def __init__(self, model: R.Net, device: torch.device, stem_s2d: bool = True, deterministic: bool = False,
                 load_tuning: bool = True, compute_dtype: torch.dtype = torch.bfloat16, reproducible: bool = False):
        """``deterministic``: bitwise-reproducible gradients (slab wgrad reduction, generic stems; BN
        statistics are always reduced in a fixed order) on one stream with heuristic kernel choices.  Costs a little
        speed.  ``reproducible``: the production schedule (both pathway streams, the weight-gradient streams, s2d
        stems, autotuned kernels) with every fp32 atomic replaced by a fixed-order (slab) reduction — once the kernel
        choices are fixed (tuned on the first step, or loaded from the persistent table) every step is bitwise
        reproducible, so a race in the stream schedule shows up as a bitwise difference (tests/test_race_gpu.py).  ``load_tuning``: restore the
        persistent autotuner table now (data parallelism restores rank 0's copy instead: ``FusedBackend``).
        ``compute_dtype``: the 16-bit MFMA operand / activation type, bf16 or fp16 (``--mixed_precision fp16``: the
        fp16 build of every kernel, csrc/kernels/common.h; fp32 accumulation, statistics and master weights)."""
        assert compute_dtype in (torch.bfloat16, torch.float16), compute_dtype
        self.cdt = compute_dtype
        self.C = require()
        self.deterministic = deterministic
        self.reproducible = reproducible
        # fixed-order (slab) reduction for the weight-gradient launches whose results feed back into the step —
        # the BN-fold Gram matrices (forward statistics) and G = dz^T act (backward coefficients) — while the
        # leaf weight gradients keep their fp32 atomics: the loss and the dgrad chain are then reproducible
        # run to run *for the same tuned launch configurations* (the slab count of a Gram / G launch is an
        # autotuner choice, and with it the summation order: two processes agree bitwise only when they share the
        # persisted tune table, ops/tune.py TuneStore, or run deterministic=True, which fixes the split heuristic)
        # and only the weight gradients carry atomic-order noise (~1e-6).  Without it that noise
        # flips ReLU masks and the random-init network's chaotic backward decorrelates two runs' gradients
        # (cosine ~0.65 at B=4-32: scripts/diag_ms_race.py @ a59cdac).  On by default (only the few Gram / G launches pay the
        # slab reduction); arm fold_slabs=0 (PVA_ARMS) turns it off; implied by ``deterministic``.
        self.fold_slabs = deterministic or reproducible or on("fold_slabs")
        # fused lateral-connection backward (apply + strided dgrad in one pass); arm lateral_bwd=0: the unfused path
        self.lateral_bwd = on("lateral_bwd")
        # two-stream backward: the lateral fusion's backward on the fast-pathway stream (arm side_fuse=0: on the main
        # stream, both streams joined around it and at every stage end)
        self.side_fuse = on("side_fuse")
        self.stem_s2d = stem_s2d and not deterministic
        self.model = model
        self.device = torch.device(device)
        model.to(self.device)
        self.prof: Optional[List] = None   # [(label, event)] when per-op profiling is enabled
        from ..ops.tune import ConvTuner
        self.tuner = ConvTuner(require(), enabled=not deterministic and torch.device(device).type == "cuda")
        self.wtune: Dict = {}
        # eval-only geometries are tuned rank-locally (forward_eval): their choices live in a table of their own so a
        # training launch never finds an un-agreed choice
        self._eval_tune: Dict = {}
        from ..ops.tune import TuneStore
        self.tune_store = None
        if self.tuner.enabled:
            self.tune_store = TuneStore({"conv": self.tuner.cache, "eval": self._eval_tune, "wgrad": self.wtune},
                                        TuneStore.build_ident(self.device, str(compute_dtype)))
            if load_tuning:
                self.tune_store.load()
        self._ws: Dict = {}
        self._splits: Dict = {}
        self._bnb: Dict = {}
        self._scratch: Dict[Tuple, torch.Tensor] = {}
        self._fin: Dict[int, torch.Tensor] = {}
        self._cmax = 8
        self.grad_beta = 0.0
        self.lane = 0          # 0: main stream, 1: fast-pathway stream (per-lane scratch)
        self._side = None
        self._seed_dev = None   # device-resident dropout key (int64 [1]), see _head_forward
        self._ms_warm = False  # set after the first training step (autotuning runs on one stream)
        self._ms_bwd = False
        self._wst = [None, None]          # weight-gradient streams of the two lanes
        self._wst_used = [False, False]
        self.debug_skip_joins = set()      # race-detection tests only (see _join)
        self._ms_ok = (not deterministic and torch.device(device).type == "cuda"
                       and on("streams"))
        # BN folding of the 1x1 conv_c (never materialise its output); units whose conv_c input has at least
        # fold_min_c channels.  Narrow (fast-pathway) folds take exact statistics from a statistics-only conv pass
        # (Gram-derived variances E[y^2] - E[y]^2 over fp32-atomic sums were not reproducible there:
        # scripts/diag_ms_fold.py @ a59cdac).  Measured (profiles/r4_fold): min C 32 / 16 / 8 -> 1182.4 / 1192.5 / 1190.6
        # clips/s once the fold's slab reductions were parallel, so the fast res3+ units fold too (default 16).
        self.bn_fold = on("bn_fold")
        self.fold_min_c = int(arm("bn_fold_min_c"))
        self.bn_fold1 = self.bn_fold and on("bn_fold1")
        # folds with fewer input channels than this take exact statistics from a statistics-only conv pass
        self.fold_exact_below = int(arm("bn_fold_exact_below"))
        # fused narrow conv_c backward (csrc/kernels/narrow_bwd.hip); workgroups (= slab count) per launch
        self.narrow_bwd = on("narrow_bwd")
        self.narrow_splits = int(arm("narrow_splits"))
        self.narrow_fold = self.narrow_bwd and on("narrow_fold")
        blocks = list(model.blocks)
        self.slowfast = isinstance(blocks[0], R.MultiPathWayWithFuse)
        self.stages: List[Tuple[List, Optional[_Fuse]]] = []
        if self.slowfast:
            for i, b in enumerate(blocks):
                if not isinstance(b, R.MultiPathWayWithFuse):
                    break
                paths = []
                for p, m in enumerate(b.multipathway_blocks):
                    nm = f"b{i}.p{p}"
                    paths.append(_Stem(self, m, nm) if isinstance(m, R.ResNetBasicStem) else _Stage(self, m, nm))
                fuse = _Fuse(self, b.multipathway_fusion, f"b{i}.fuse") if b.multipathway_fusion is not None else None
                self.stages.append((paths, fuse))
            pool = blocks[-2]
            assert isinstance(pool, R.PoolConcatPathway)
            self.head_pools = [tuple(p.kernel_size) for p in pool.pool]
            self.head = blocks[-1]
        else:
            for i, b in enumerate(blocks[:-1]):
                nm = f"b{i}.p0"
                self.stages.append(([_Stem(self, b, nm) if isinstance(b, R.ResNetBasicStem) else _Stage(self, b, nm)],
                                    None))
            self.head = blocks[-1]
            self.head_pools = [tuple(self.head.pool.kernel_size)] if self.head.pool is not None else [None]
        self.npath = len(self.stages[0][0])
        self.units: List[_ConvBN] = []
        for paths, fuse in self.stages:
            for p in paths:
                self.units += p.units
            if fuse is not None:
                self.units += fuse.units
        self._cmax = max(u.C for u in self.units)
        # flat parameters in reverse execution order (head first)
        order = list(self.head.named_parameters(prefix="head"))
        for u in reversed(self.units):
            order += [(u.name + ".bn.w", u.bn.weight), (u.name + ".bn.b", u.bn.bias), (u.name + ".w", u.conv.weight)]
        seen = set()
        named = []
        for n, p in order:
            if id(p) not in seen:
                seen.add(id(p))
                named.append((n, p))
        assert len(named) == len(list(model.parameters())), "executor does not cover every parameter"
        self.flat = FlatParams(named, self.device)
        self._build_packs()
        self.pack()
        # backward progress reporting for overlapped gradient all-reduce (parallel/ddp.GradSync); grad_multi_stream:
        # the sync waits on producer_streams() itself (its own comm stream), so reports need no stream joins
        self.grad_hook = None
        self.grad_multi_stream = False
        self._head_hi = max(self.flat.span(p)[1] for p in self.head.parameters())
        for paths, fuse in self.stages:
            mods = list(paths) + ([fuse] if fuse is not None else [])
            for m in mods:
                subs = m.blocks if isinstance(m, _Stage) else [m]
                for sub in subs:
                    sub.flat_hi = max(self.flat.span(w)[1] for u in sub.units
                                      for w in (u.conv.weight, u.bn.weight, u.bn.bias))
                    sub.eng_progress = self._progress

    def mark(self, label: str):
        """Per-op profiling: the interval up to the next mark is charged to ``label``."""
        if self.prof is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.prof.append((label, ev))

    def profile_report(self) -> List[Tuple[str, float]]:
        """(label, ms) for the marks recorded since ``prof`` was set to ``[]`` (synchronizes)."""
        torch.cuda.synchronize()
        p = self.prof or []
        return [(a, e0.elapsed_time(e1)) for (a, e0), (_, e1) in zip(p, p[1:])]

    def producer_streams(self) -> List:
        """Every stream that writes the flat gradient (the current one, the fast-pathway stream, the weight-gradient
        streams): ``parallel/ddp.GradSync`` records an event on each before it launches a bucket."""
        out = [torch.cuda.current_stream(self.device)]
        if self._side is not None:
            out.append(self._side)
        out += [st for st in self._wst if st is not None]
        return out

    def _progress(self, hi: int, force: bool = False):
        """grad[:hi] is final once the work issued so far completes.  With a multi-stream gradient sync (its comm
        stream waits on every producer stream) every block reports as soon as it is issued.  Otherwise, during
        two-stream backward, the per-block reports are dropped (the stage's pathways finish in any order) and
        progress is reported once per stage after the streams are joined (``force``)."""
        if self.grad_hook is not None and self.grad_multi_stream:
            self.grad_hook(hi)
            return
        if self.grad_hook is not None and (force or not self._ms_bwd):
            if force:
                self._join_wgrads()   # the bucket's weight gradients may still be in flight on the wgrad streams
            self.grad_hook(hi)

    # ------------------------------------------------------------------ buffers
    def ws(self, key, shape, dtype) -> torch.Tensor:
        t = self._ws.get(key)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = torch.empty(shape, device=self.device, dtype=dtype)
            self._ws[key] = t
        return t

    def fin_ws(self) -> Optional[torch.Tensor]:
        """Two-level BN finalize workspace (partial doubles + counters the kernels keep zero), ONE per stream lane
        sized for the widest BatchNorm: the finalizes of a lane are stream-ordered, so every BN of the lane shares it
        (one per unit held ~120 MB)."""
        if self.device.type != "cuda":
            return None
        t = self._fin.get(self.lane)
        if t is None:
            t = self._fin[self.lane] = torch.zeros(self.C.fin_doubles(self._cmax), device=self.device,
                                                   dtype=torch.float64)
        return t

    def scratch(self, key: str, numel: int, zero: bool = False) -> torch.Tensor:
        """Grow-only fp32 scratch shared by sequential (stream-ordered) users of one lane (the main stream
        and the fast-pathway stream each have their own).  ``zero``: allocated zeroed (the wgrad
        accumulator is kept zero by its consumer, wgrad_reduce)."""
        k = (key, self.lane)
        t = self._scratch.get(k)
        if t is None or t.numel() < numel:
            alloc = torch.zeros if zero else torch.empty
            t = alloc(max(numel, 1 << 20), device=self.device, dtype=torch.float32)
            self._scratch[k] = t
        return t[:numel]

    # ------------------------------------------------------------------ two-stream execution
    def _ms_active(self) -> bool:
        """The fast pathway runs on its own HIP stream, concurrently with the slow pathway (both are
        independent between lateral fusions; the narrow fast-path kernels are latency-bound and fill the CUs
        the slow path's MFMA kernels leave idle).  Off for the first (autotuning) step, in deterministic
        mode, for single-pathway nets, under the per-op profiler and with the arm ``streams=0``."""
        return (self._ms_ok and self._ms_warm and self.npath == 2 and self.prof is None)

    def _side_stream(self):
        if self._side is None:
            # arm side_priority: HIP stream priority of the fast-pathway stream (lower = higher priority)
            self._side = torch.cuda.Stream(device=self.device,
                                           priority=int(arm("side_priority")))
        return self._side

    def _wgrad_stream(self):
        """The weight-gradient stream of the current lane (0: main, 1: fast pathway)."""
        i = self.lane
        if self._wst[i] is None:
            self._wst[i] = torch.cuda.Stream(device=self.device)
        self._wst_used[i] = True
        return self._wst[i]

    def _join_wgrads(self):
        main = torch.cuda.current_stream(self.device)
        for i, st in enumerate(self._wst):
            if st is not None and self._wst_used[i]:
                self._join(main, st)
                self._wst_used[i] = False

    def _join(self, waiter, signaller, tag: Optional[str] = None):
        """``waiter`` waits for everything issued so far on ``signaller`` (one event).  ``tag`` names joins that a
        race-detection test may drop on purpose (``debug_skip_joins``, tests/test_race_gpu.py)."""
        if tag is not None and tag in self.debug_skip_joins:
            return
        ev = torch.cuda.Event()
        ev.record(signaller)
        waiter.wait_event(ev)

    def _bn_blocks(self, M, C):
        k = (M, C)
        v = self._bnb.get(k)
        if v is None:
            v = self._bnb[k] = tuple(self.C.bn_bwd_blocks(M, C))
        return v

    def _build_packs(self):
        fwd_n, dgr_n = 0, 0
        offs = []
        for u in self.units:
            s = u.spec
            nf = s.cout * s.taps * s.cin_pad
            nd = s.cin * s.taps * s.cout if s.cin % 8 == 0 else 0
            offs.append((fwd_n, dgr_n if nd else -1))
            fwd_n += (nf + 7) // 8 * 8
            dgr_n += (nd + 7) // 8 * 8
        self.pack_fwd = torch.zeros(fwd_n, device=self.device, dtype=self.cdt)
        self.pack_dgr = torch.zeros(max(dgr_n, 8), device=self.device, dtype=self.cdt)
        import numpy as np
        dsz = self.C.pack_desc_size()
        assert dsz == 40
        rec = np.zeros(len(self.units), dtype=np.dtype([("src", "<i8"), ("fwd", "<i8"), ("dgr", "<i8"),
                                                        ("cout", "<i4"), ("cin", "<i4"), ("cin_pad", "<i4"),
                                                        ("taps", "<i4")]))
        for i, (u, (fo, do)) in enumerate(zip(self.units, offs)):
            s = u.spec
            a, _ = self.flat.span(u.conv.weight)
            rec[i] = (a, fo, do, s.cout, s.cin, s.cin_pad, s.taps)
            u.wf = self.pack_fwd[fo:fo + s.cout * s.taps * s.cin_pad].view(s.cout, s.taps * s.cin_pad)
            if do >= 0:
                u.wd = self.pack_dgr[do:do + s.cin * s.taps * s.cout].view(s.cin, s.taps * s.cout)
        self.pack_desc = torch.from_numpy(rec.view(np.uint8).copy()).to(self.device)

    def pack(self):
        """Refresh bf16 packed weights from the fp32 master buffer (one multi-tensor launch + s2d stems)."""
        self.C.pack_weights(self.flat.data, self.pack_fwd, self.pack_dgr, self.pack_desc, len(self.units))
        for paths, _ in self.stages:
            for m in paths:
                if isinstance(m, _Stem):
                    m.pack()

    @property
    def input_s2d(self) -> bool:
        """Whether the stems consume space-to-depth inputs (set GpuClipBatch(s2d=...) accordingly)."""
        return any(isinstance(m, _Stem) and m.s2d for paths, _ in self.stages for m in paths)

    # ------------------------------------------------------------------ forward
    def _forward_backbone(self, xs: List[Act], train: bool) -> List[Act]:
        tag = "t" if train else "e"
        cur = list(xs)
        self._cats = []
        ms = self._ms_active()
        main = torch.cuda.current_stream(self.device) if ms else None
        side = self._side_stream() if ms else None
        if ms:
            self._join(side, main)   # inputs were produced on the main stream
        for si, (paths, fuse) in enumerate(self.stages):
            with trace_range(f"fwd/b{si}"):
                outs = [None] * len(paths)
                cat = None
                # fast pathway first (issued to its own stream when two-stream execution is on)
                for p in range(len(paths) - 1, -1, -1):
                    mod = paths[p]
                    x = cur[p]
                    T, H, W = mod.out_dims(x.T, x.H, x.W)
                    M = x.N * T * H * W
                    co = mod.out_channels()
                    if p == 0 and fuse is not None:
                        cat = self.ws(("cat", si, tag), (M, co + fuse.u.C), self.cdt)
                        out = cat[:, :co]
                    else:
                        out = self.ws(("pout", si, p, tag), (M, co), self.cdt)
                    if ms and p == 1:
                        self.lane = 1
                        with torch.cuda.stream(side):
                            outs[p] = mod.fwd(x, out, train, tag)
                        self.lane = 0
                    else:
                        outs[p] = mod.fwd(x, out, train, tag)
                if fuse is not None:
                    if ms:
                        self._join(main, side)   # the fusion reads the fast pathway's output
                    co = outs[0].C
                    fuse.fwd(outs[1], cat[:, co:], train, tag)
                    outs[0] = Act(cat, outs[0].N, outs[0].T, outs[0].H, outs[0].W)
                self._cats.append(cat)
                cur = outs
        if ms:
            self._join(main, side)
        return cur

    def _pool_features(self, outs: List[Act], tag: str) -> Tuple[torch.Tensor, List]:
        shapes = []
        for o, k in zip(outs, self.head_pools):
            k = (o.T, o.H, o.W) if k is None else k
            shapes.append(tuple(max(d - kk + 1, 0) for d, kk in zip((o.T, o.H, o.W), k)))
        if not (all(s == shapes[0] for s in shapes) and all(v > 0 for v in shapes[0])):
            # documented fallback (64-frame SlowFast): global average per pathway
            ks = [(o.T, o.H, o.W) for o in outs]
            P = 1
        else:
            ks = [((o.T, o.H, o.W) if k is None else k) for o, k in zip(outs, self.head_pools)]
            P = shapes[0][0] * shapes[0][1] * shapes[0][2]
        Ctot = sum(o.C for o in outs)
        N = outs[0].N
        feat = self.ws(("feat", tag), (N, P, Ctot), torch.float32)
        self.mark("head.pool")
        coff = 0
        for o, k in zip(outs, ks):
            assert o.t.is_contiguous()
            self.C.avgpool_fwd(o.t, [o.N, o.T, o.H, o.W, o.C], list(k), feat, Ctot, coff)
            coff += o.C
        return feat, ks

    # ------------------------------------------------------------------ head (csrc/kernels/head.hip)
    def _head_forward(self, feat: torch.Tensor, train: bool, tag: str):
        """Dropout -> Linear per position -> position mean (K17-K19) on the HIP head kernels.
        Returns (logits [N, K] fp32, xm [N, C] = dropped position-mean features, p_drop, seed)."""
        h = self.head
        W, b = h.proj.weight, h.proj.bias
        p = float(h.dropout.p) if (train and h.dropout is not None) else 0.0
        # per-step Philox key kept on the device: first drawn from torch's CPU generator (reproducible under
        # set_seed), then advanced by one splitmix64 step per training forward ON the device, so a step captured
        # into a HIP graph (engine/graph.py) draws a fresh mask on every replay exactly as the eager step does
        seed = 0
        if p > 0:
            if self._seed_dev is None:
                self._seed_dev = torch.tensor([int(torch.randint(0, 2 ** 62, (1,)).item())], device=self.device,
                                              dtype=torch.long)
            self.C.head_seed_advance(self._seed_dev)
        N = feat.shape[0]
        xm = self.ws(("head_xm", tag), (N, feat.shape[2]), torch.float32)
        logits = torch.empty(N, W.shape[0], device=self.device, dtype=torch.float32)
        self.mark("head.fwd")
        self.C.head_forward(feat, self.flat.view(W), None if b is None else self.flat.view(b), p, seed, xm, logits,
                            self._seed_dev if p > 0 else None)
        return logits, xm, p, seed

    @torch.no_grad()
    def forward_eval(self, xs: List[Act]) -> torch.Tensor:
        """Eval forward.  Kernel choices for eval geometries are tuned rank-locally: under data parallelism each
        rank's validation shard has its own batch count and last-batch size (uniform clips per video differ), so
        a cross-rank agreement collective here would only run on the ranks that see a new shape and hang the
        others.  No cross-rank math depends on eval kernel choices (every configuration computes the same sums)."""
        agree, self.tuner.agree = self.tuner.agree, None
        train_cache, self.tuner.cache = self.tuner.cache, self._eval_tune
        try:
            outs = self._forward_backbone(xs, train=False)
            feat, _ = self._pool_features(outs, "e")
            logits, _, _, _ = self._head_forward(feat, False, "e")
        finally:
            self.tuner.agree = agree
            self.tuner.cache = train_cache
        if self.tune_store is not None:
            self.tune_store.save()
        return logits

    @torch.no_grad()
    def eval_counts(self, logits: torch.Tensor, labels: torch.Tensor,
                    counts: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Top-1 (correct, total) int64 counters of ``logits`` vs ``labels`` (argmax, first maximum on ties;
        reference run.py:297), accumulated into ``counts`` when given (HIP head_ce kernel, no host sync)."""
        N, K = logits.shape
        if counts is None:
            counts = torch.zeros(2, device=self.device, dtype=torch.long)
            acc = 0
        else:
            acc = 1
        rl = self.ws(("head_rl",), (max(N, 1),), torch.float32)
        rc = self.ws(("head_rc",), (max(N, 1),), torch.int32)
        self.C.head_ce(logits.contiguous(), labels.to(self.device, torch.long).contiguous(), 0.0, None, None, counts,
                       acc, rl, rc)
        return counts

    def forward_backward(self, xs: List[Act], labels: torch.Tensor, loss_scale: float = 1.0,
                         accumulate: Optional[bool] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """One training micro-step.  Gradients of ``loss * loss_scale`` are written (``accumulate=False``)
        or added (``accumulate=True``) into the flat fp32 gradient buffer; by default they accumulate
        unless the optimizer's ``zero_grad`` marked the buffer zero.  Returns (loss, logits)."""
        if accumulate is None:
            accumulate = not self.flat.zeroed
        self.flat.zeroed = False
        self.grad_beta = 1.0 if accumulate else 0.0
        with torch.no_grad():
            outs = self._forward_backbone(xs, train=True)
            feat, ks = self._pool_features(outs, "t")
            logits, xm, p, seed = self._head_forward(feat, True, "t")
            N, K = logits.shape
            Ct = feat.shape[2]
            labels = labels.to(self.device, torch.long).contiguous()
            loss = torch.empty(1, device=self.device, dtype=torch.float32)
            dlogits = self.ws(("head_dl",), (N, K), torch.float32)
            rl = self.ws(("head_rl",), (max(N, 1),), torch.float32)
            rc = self.ws(("head_rc",), (max(N, 1),), torch.int32)
            self.mark("head.ce")
            # softmax cross-entropy (mean over the batch, reference run.py:254) and its gradient
            self.C.head_ce(logits, labels, float(loss_scale) / max(N, 1), dlogits, loss, None, 0, rl, rc)
            h = self.head
            W, b = h.proj.weight, h.proj.bias
            train_backbone = any(q.requires_grad for q in self.units[0].conv.parameters())  # else frozen backbone
            gfeat = self.ws(("gfeat",), tuple(feat.shape), torch.float32) if train_backbone else None
            scratch = self.scratch("head_bwd", K * N + Ct * N + Ct * K)
            self.mark("head.bwd")
            self.C.head_backward(dlogits, xm, self.flat.view(W), feat.shape[1], p, seed, self.flat.gview(W),
                                 None if b is None else self.flat.gview(b), self.grad_beta, gfeat, scratch,
                                 self._seed_dev if p > 0 else None)
            self._progress(self._head_hi)
            if train_backbone:
                self._backward_backbone(outs, gfeat, ks)
        self._ms_warm = True
        if self.tune_store is not None:
            self.tune_store.save()
        return loss[0], logits

    def _backward_backbone(self, outs: List[Act], gfeat: torch.Tensor, ks):
        C = self.C
        Ctot = gfeat.shape[-1]
        # head pools -> grads of the last stage outputs
        douts = []
        coff = 0
        self.mark("head.poolbwd")
        for p, (o, k) in enumerate(zip(outs, ks)):
            d = self.ws(("dlast", p), (o.M, o.C), self.cdt)
            C.avgpool_bwd(gfeat, Ctot, coff, [o.N, o.T, o.H, o.W, o.C], list(k), d)
            douts.append(Act(d, o.N, o.T, o.H, o.W))
            coff += o.C
        ms = self._ms_active()
        main = torch.cuda.current_stream(self.device) if ms else None
        side = self._side_stream() if ms else None
        self._ms_bwd = ms   # per-block progress reports are deferred to stage ends (grads come from two streams)
        # Per stage: the lateral fusion's backward (its input is the slow stage above's dcat, its output the fast
        # pathway's dfast) runs on the fast-pathway stream — the slow pathway depends on neither, so the main stream goes
        # straight on with the slow stage instead of waiting for it (it ran alone: ~1 ms/step in the steady-state
        # trace, profiles/r5_final).  Without a gradient hook (or with the multi-stream GradSync, whose comm stream
        # waits on every producer) the streams are not joined per stage at all: the main stream runs ahead and each
        # stage's fusion waits only for the dcat it reads.
        side_fuse = ms and self.side_fuse
        free = side_fuse and (self.grad_hook is None or self.grad_multi_stream)
        for si in range(len(self.stages) - 1, -1, -1):
            with trace_range(f"bwd/b{si}"):
                paths, fuse = self.stages[si]
                if ms and not free:
                    self._join(main, side)   # the fast pathway's dx of the stage above is final
                # grads for this stage's pathway outputs: douts (slow may be the full concat grad)
                if fuse is not None:
                    dcat = douts[0]
                    co = paths[0].out_channels()
                    if side_fuse:
                        self._join(side, main)   # dcat: written by the slow stage above (main stream)
                        self.lane = 1
                        with torch.cuda.stream(side):
                            fuse.bwd(dcat.narrow(co, fuse.u.C), douts[1].t)
                        self.lane = 0
                        if not free:
                            self._join(main, side)   # the per-stage report below follows the current stream
                    else:
                        fuse.bwd(dcat.narrow(co, fuse.u.C), douts[1].t)
                        if ms:
                            self._join(side, main)   # the fast pathway's dx now includes the lateral term
                    self._progress(fuse.flat_hi, force=True)
                    douts[0] = dcat.narrow(0, co)
                elif ms:
                    # the head's pooled-gradient scatter (main stream) feeds the fast stage
                    self._join(side, main, tag="head_scatter")
                new = [None] * len(paths)
                # pathways in reverse order: matches the flat (reverse-execution) gradient layout
                for p in range(len(paths) - 1, -1, -1):
                    mod = paths[p]
                    on_side = ms and p == 1
                    if on_side:
                        self.lane = 1
                        ctx = torch.cuda.stream(side)
                        ctx.__enter__()
                    try:
                        if isinstance(mod, _Stem):
                            mod.bwd(douts[p])
                            if not ms:
                                self._progress(mod.flat_hi)
                        else:
                            xin = mod.blocks[0].x
                            dx = self.ws(("dstage_in", si, p), (xin.M, xin.C), self.cdt)
                            mod.bwd(douts[p], dx, False)
                            new[p] = Act(dx, xin.N, xin.T, xin.H, xin.W)
                    finally:
                        if on_side:
                            ctx.__exit__(None, None, None)
                            self.lane = 0
                if ms:
                    if not free:
                        self._join(main, side)
                    self._progress(max(m.flat_hi if isinstance(m, _Stem) else m.blocks[0].flat_hi for m in paths),
                                   force=True)
                douts = new
        if ms:
            self._join(main, side)
            self._join_wgrads()
        self._ms_bwd = False

    # ------------------------------------------------------------------ misc
    def prepare_inputs(self, xs_ncthw: Sequence[torch.Tensor]) -> List[Act]:
        """NCTHW float clips (already normalised) -> stem input Acts (s2d or NDHWC RGB0)."""
        if self.input_s2d:
            return [to_s2d(x.to(self.device), self.cdt) for x in xs_ncthw]
        return [Act.from_ncthw(x.to(self.device), c_pad=4, dtype=self.cdt) for x in xs_ncthw]
