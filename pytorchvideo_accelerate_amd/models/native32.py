"""Native fp32 executor: the reference's default precision (``--mixed_precision no``, reference run.py:330) on the
gfx950 fp32 kernels (``csrc/fp32``: split-bf16 MFMA convolutions (three pieces per operand), fp32 BatchNorm / pooling, the fp32 head kernels).

``NativeF32Net`` runs the pytorchvideo-keyed module tree of ``models/reference.py`` — SlowFast-R50/R101 and
Slow-R50 (reference run.py:105-118, the default ``is_slowfast=False`` model at run.py:338-351) — with its own tape
instead of autograd: the forward records, per op, what its backward needs; the backward walks the tape in reverse,
writes parameter gradients straight into the flat fp32 gradient buffer (``FlatParams``: written on the first
micro-step, accumulated on later ones) and reports each finished parameter to ``grad_hook`` (the bucketed gradient
all-reduce, ``parallel/ddp.GradSync``), so communication overlaps the rest of the backward as on the bf16 path.

Numerics (what PyTorch fp32 computes): convolutions accumulate in fp32 with 24-bit operands (three bf16 pieces
per fp32 value, six MFMA products per fragment pair; arm ``f32_pieces=2``: 16-bit operands, three products); BatchNorm statistics are fp32 partials summed in double;
running statistics use the unbiased variance with momentum 0.1; the max pool picks the first maximum of each
window; head dropout draws a Philox stream (same distribution as torch's, not its bits).

Layout: NDHWC fp32 activations (``[N, T, H, W, C]``); the stems' RGB input is padded to 4 channels.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch
import torch.nn as nn

from ..ops._ext import require
from ..ops.f32 import ConvGeom, conv_dgrad, conv_fwd, conv_wgrad, pack_weight, pieces
from . import reference as R
from .fused import FlatParams


def ordered_params(model: nn.Module):
    """Flat-buffer order = reverse of forward execution (head first), as the backends use for bucketing."""
    return [(n, p) for n, p in reversed(list(model.named_parameters()))]


class Lazy:
    """An activation its consumers recompute: relu(y * scale + shift) with scale / shift = rows 2 / 3 of the
    BatchNorm table ``stat`` [4][C].  The next conv's operand loaders (forward and weight gradient) apply the affine and
    the ReLU while staging, and the BatchNorm backward derives the ReLU mask from y — the normalised tensor is never
    written (saves its write, and a read in every consumer and in the backward)."""

    __slots__ = ("y", "stat", "shape")

    def __init__(self, y: torch.Tensor, stat: torch.Tensor):
        self.y, self.stat, self.shape = y, stat, y.shape


class _ConvBN:
    """conv (bias-free) -> BatchNorm3d (training batch statistics or running statistics) -> optional ReLU."""

    def __init__(self, net: "NativeF32Net", conv: nn.Conv3d, bn: nn.BatchNorm3d, relu: bool, cip: int = 0):
        self.net, self.conv, self.bn, self.relu = net, conv, bn, relu
        self.g = ConvGeom(conv.in_channels, conv.out_channels, tuple(conv.kernel_size), tuple(conv.stride),
                          tuple(conv.padding), cip)
        self.taps = self.g.taps_fwd(net.device)
        self.phases = self.g.phases(net.device) if conv.in_channels % 4 == 0 else None

    def forward(self, x, train: bool, add: Optional[torch.Tensor] = None, lazy: bool = False):
        """Returns (out, saved) — saved is what backward needs (None in eval).  ``x`` may be a :class:`Lazy`
        activation; ``lazy``: return this layer's output as one too (BN + ReLU applied by its consumers)."""
        F, g, dev = self.net.F, self.g, self.net.device
        N, T, H, W, _ = x.shape
        To, Ho, Wo = g.out_thw((T, H, W))
        C = g.cout
        wf = pack_weight(F, g, self.conv.weight, 0)
        y = torch.empty(N, To, Ho, Wo, C, device=dev)
        M = N * To * Ho * Wo
        tiles = -(-M // F.igemm32_bm(C))
        # training: BatchNorm statistics from the conv epilogue (per-tile sums, no re-read of y), reduced in two levels
        tstat = torch.empty(tiles, 2, C, device=dev) if train else None
        conv_fwd(F, g, x, wf, y, self.taps, stats=tstat)
        stat = torch.empty(4, C, device=dev)
        bn = self.bn
        if train:
            part = torch.empty(F.chan_reduce32_blocks(tiles, 2 * C), 2, C, device=dev)
            F.chan_reduce32(tstat, 2 * C, None, 2 * C, None, 2 * C, None, 3, 0, tiles, 2 * C, part)
            F.bn32_finalize(part, C, M, 0, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                            bn.num_batches_tracked, bn.momentum, bn.eps, stat, None, None, None, None, 0.0)
        else:
            F.bn32_finalize(None, C, M, 2, bn.weight, bn.bias, bn.running_mean, bn.running_var, None,
                            bn.momentum, bn.eps, stat, None, None, None, None, 0.0)
        if lazy:
            assert self.relu and add is None
            out = Lazy(y, stat)
            return out, ((x, y, None, stat) if train else None)
        out = torch.empty_like(y)
        F.bn32_apply(y, C, stat, add, C, int(self.relu), out, C, M, C)
        return out, ((x, y, out, stat) if train else None)

    def backward(self, saved, dout: torch.Tensor, need_dx: bool, dx_acc: Optional[torch.Tensor] = None,
                 want_g: bool = False):
        """Gradients of one conv+BN(+ReLU): parameter gradients into the flat buffer; returns (dx, g) where g is
        the gradient at the BN(+add) output (for a residual add's other operand) when ``want_g``.  ``dx_acc``:
        accumulate the input gradient into this buffer instead of a fresh one."""
        F, g, net = self.net.F, self.g, self.net
        x, y, out, stat = saved
        N, To, Ho, Wo, C = y.shape
        M = N * To * Ho * Wo
        dev = net.device
        bn = self.bn
        part = torch.empty(F.chan_reduce32_blocks(M, C), 2, C, device=dev)
        # (a lazy output has no stored tensor: the ReLU mask is recomputed from y and the statistics)
        F.chan_reduce32(y, C, dout, C, out if self.relu else None, C, stat[0], 1, int(self.relu), M, C, part)
        coef = torch.empty(3, C, device=dev)
        gb = net.grad_beta
        train_bn = bn.weight.requires_grad
        F.bn32_finalize(part, C, M, 1, bn.weight, bn.bias, None, None, None, 0.0, bn.eps, None, stat,
                        net.flat.gview(bn.weight) if train_bn else None,
                        net.flat.gview(bn.bias) if train_bn else None, coef, gb)
        dy = torch.empty_like(y)
        gout = torch.empty_like(y) if want_g else None
        F.bn32_bwd_apply(dout, C, out if self.relu else None, C, int(self.relu), y, C, stat, coef, dy, C, gout, C, M, C)
        if train_bn:
            net.done(bn.weight, bn.bias)
        if self.conv.weight.requires_grad:
            dwf = torch.empty(C, g.ntap * g.cip, device=dev)
            F.zero32(dwf)
            conv_wgrad(F, g, dy, x, dwf, self.taps)   # (x may be Lazy: the loader applies its BN + ReLU)
            F.wpack32(2, dwf, net.flat.gview(self.conv.weight), C, g.cin, g.ntap, g.cip, gb)
            net.done(self.conv.weight)
        dx = None
        if need_dx:
            assert self.phases is not None, "input gradient of a padded-channel conv"
            wt = pack_weight(F, g, self.conv.weight, 1)
            if dx_acc is not None:
                dx = dx_acc
                geo_acc = True
            else:
                dx = torch.empty(x.shape[0], x.shape[1], x.shape[2], x.shape[3], g.cin, device=dev)
                geo_acc = False
            self._dgrad(dy, wt, dx, geo_acc)
        return dx, gout

    def _dgrad(self, dy, wt, dx, acc: bool):
        F, g = self.net.F, self.g
        if not acc:
            conv_dgrad(F, g, dy, wt, dx, self.phases)
            return
        # accumulate: every dX position belongs to exactly one stride phase, so each phase GEMM adds in place
        N, T, H, W, C = dx.shape
        To, Ho, Wo = dy.shape[1:4]
        for (rt, rh, rw), taps, nt in self.phases:
            Qt, Qh, Qw = -(-(T - rt) // g.s[0]), -(-(H - rh) // g.s[1]), -(-(W - rw) // g.s[2])
            if min(Qt, Qh, Qw) <= 0 or nt == 0:
                continue
            geo = [g.cout, g.ntap * g.cout, g.cin, N * Qt * Qh * Qw, g.cin, nt * g.cout, g.cout, 1, Qt, Qh, Qw,
                   To, Ho, Wo, 1, 1, 1, T, H, W, *g.s, rt, rh, rw]
            F.conv32(dy, wt, dx, taps, geo, np=pieces())


class _ResUnit:
    """pytorchvideo ResBlock: relu(branch1(x) + branch2(x)), branch2 = conv_a/b/c bottleneck."""

    def __init__(self, net, blk: R.ResBlock):
        b2 = blk.branch2
        self.a = _ConvBN(net, b2.conv_a, b2.norm_a, True)
        self.b = _ConvBN(net, b2.conv_b, b2.norm_b, True)
        self.c = _ConvBN(net, b2.conv_c, b2.norm_c, True)   # relu after the residual add
        self.sc = _ConvBN(net, blk.branch1_conv, blk.branch1_norm, False) if blk.branch1_conv is not None else None

    def forward(self, x, train):
        if self.sc is not None:
            s, ss = self.sc.forward(x, train)
        else:
            s, ss = x, None
        a, sa = self.a.forward(x, train, lazy=True)    # conv_a / conv_b outputs: BN + ReLU applied by the consumer
        b, sb = self.b.forward(a, train, lazy=True)
        out, sc = self.c.forward(b, train, add=s)
        return out, ((sa, sb, sc, ss) if train else None)

    def backward(self, saved, dout, need_dx, dx_acc=None):
        sa, sb, sc, ss = saved
        db, g = self.c.backward(sc, dout, True, want_g=True)
        da, _ = self.b.backward(sb, db, True)
        del db
        if self.sc is None:
            # identity shortcut: dx = g + conv_a's input gradient (accumulated into g's buffer, or the caller's)
            if dx_acc is not None:
                net = self.a.net
                C = g.shape[-1]
                net.F.copy32(g, C, dx_acc, C, g.numel() // C, C, 1)
                g = dx_acc
            dx, _ = self.a.backward(sa, da, need_dx, dx_acc=g)
            return dx
        # projection shortcut: dx = dgrad(a) + dgrad(branch1); branch1 after conv_a (parameter order)
        dx, _ = self.a.backward(sa, da, need_dx, dx_acc=dx_acc)
        dx, _ = self.sc.backward(ss, g, need_dx, dx_acc=dx)
        return dx


class _Stem:
    def __init__(self, net, stem: R.ResNetBasicStem):
        self.net = net
        self.cb = _ConvBN(net, stem.conv, stem.norm, True, cip=4)
        p = stem.pool
        self.pk, self.ps, self.pp = (tuple(p.kernel_size), tuple(p.stride), tuple(p.padding))

    def forward(self, x, train):
        F, dev = self.net.F, self.net.device
        y, s = self.cb.forward(x, train)
        N, T, H, W, C = y.shape
        To, Ho, Wo = ((i + 2 * p - k) // st + 1 for i, k, st, p in zip((T, H, W), self.pk, self.ps, self.pp))
        out = torch.empty(N, To, Ho, Wo, C, device=dev)
        arg = torch.empty(N, To, Ho, Wo, C, device=dev, dtype=torch.uint8)
        F.maxpool32(0, y, out, arg, [N, T, H, W, To, Ho, Wo, C], list(self.pk), list(self.ps), list(self.pp))
        return out, ((s, arg, tuple(y.shape)) if train else None)

    def backward(self, saved, dout):
        F, dev = self.net.F, self.net.device
        s, arg, (N, T, H, W, C) = saved
        To, Ho, Wo = dout.shape[1:4]
        dy = torch.empty(N, T, H, W, C, device=dev)
        F.maxpool32(1, dout.contiguous(), dy, arg, [N, T, H, W, To, Ho, Wo, C], list(self.pk), list(self.ps),
                    list(self.pp))
        self.cb.backward(s, dy, False)


class _Fuse:
    """FuseFastToSlow: conv(kt,1,1)/(alpha,1,1) + BN + ReLU on the fast pathway, concatenated to the slow one."""

    def __init__(self, net, f: R.FuseFastToSlow):
        self.net = net
        self.cb = _ConvBN(net, f.conv_fast_to_slow, f.norm, True)

    def forward(self, xs, xf, train):
        F, dev = self.net.F, self.net.device
        lat, s = self.cb.forward(xf, train)
        Cs, Cl = xs.shape[-1], lat.shape[-1]
        assert xs.shape[:4] == lat.shape[:4], "lateral output grid must match the slow pathway"
        cat = torch.empty(*xs.shape[:4], Cs + Cl, device=dev)
        M = xs.numel() // Cs
        F.copy32(xs, Cs, cat, Cs + Cl, M, Cs, 0)
        F.copy32(lat, Cl, cat[..., Cs:], Cs + Cl, M, Cl, 0)
        return cat, ((s, Cs, Cl) if train else None)

    def backward(self, saved, dcat, dfast: torch.Tensor):
        """Returns the slow pathway's gradient; the lateral conv's input gradient is added into ``dfast``."""
        F, dev = self.net.F, self.net.device
        s, Cs, Cl = saved
        M = dcat.numel() // (Cs + Cl)
        gs = torch.empty(*dcat.shape[:4], Cs, device=dev)
        gl = torch.empty(*dcat.shape[:4], Cl, device=dev)
        F.copy32(dcat, Cs + Cl, gs, Cs, M, Cs, 0)
        F.copy32(dcat[..., Cs:], Cs + Cl, gl, Cl, M, Cl, 0)
        self.cb.backward(s, gl, True, dx_acc=dfast)
        return gs


class NativeF32Net:
    """fp32 training/eval executor over the reference module tree (SlowFast-R50/R101, Slow-R50)."""

    def __init__(self, model: nn.Module, device, flat: Optional[FlatParams] = None):
        self.C = require()
        self.F = self.C.f32
        self.device = torch.device(device)
        self.model = model.to(self.device)
        self.flat = flat if flat is not None else FlatParams(ordered_params(self.model), self.device)
        self.grad_hook = None
        self.grad_beta = 0.0
        blocks = list(model.blocks)
        self.slowfast = isinstance(blocks[0], R.MultiPathWayWithFuse)
        self.head = blocks[-1]
        if self.slowfast:
            mp0 = blocks[0]
            self.stems = [_Stem(self, s) for s in mp0.multipathway_blocks]
            self.fuses = [_Fuse(self, mp0.multipathway_fusion)]
            self.stages = []
            for b in blocks[1:-2]:
                self.stages.append([[_ResUnit(self, u) for u in st.res_blocks] for st in b.multipathway_blocks])
                self.fuses.append(_Fuse(self, b.multipathway_fusion) if b.multipathway_fusion is not None else None)
            self.head_pools = [tuple(p.kernel_size) for p in blocks[-2].pool]
        else:
            self.stems = [_Stem(self, blocks[0])]
            self.fuses = []
            self.stages = [[[_ResUnit(self, u) for u in st.res_blocks]] for st in blocks[1:-1]]
            self.head_pools = [tuple(self.head.pool.kernel_size) if self.head.pool is not None else None]
        self._pidx = {id(p): i for i, p in enumerate(self.flat.params)}
        self._reset_progress()

    # ------------------------------------------------------------------ gradient progress (bucketed all-reduce)
    def _reset_progress(self):
        self._ready = [not p.requires_grad for p in self.flat.params]
        self._front = 0

    def done(self, *params):
        for p in params:
            self._ready[self._pidx[id(p)]] = True
        f = self._front
        while f < len(self._ready) and self._ready[f]:
            f += 1
        if f != self._front:
            self._front = f
            if self.grad_hook is not None:
                self.grad_hook(self.flat.span(self.flat.params[f - 1])[1])

    # ------------------------------------------------------------------ input
    def _inputs(self, video) -> List[torch.Tensor]:
        xs = list(video) if isinstance(video, (list, tuple)) else [video]
        out = []
        for v in xs:
            v = v.to(self.device, torch.float32, non_blocking=True).contiguous()
            N, Cin, T, H, W = v.shape
            y = torch.empty(N, T, H, W, 4, device=self.device)
            self.F.to_ndhwc32(v, y, N, Cin, T * H * W, 4)
            out.append(y)
        return out

    # ------------------------------------------------------------------ forward
    def _backbone(self, xs: List[torch.Tensor], train: bool, tape: Optional[list]):
        rec = tape.append if tape is not None else (lambda e: None)
        cur = []
        for st, x in zip(self.stems, xs):
            y, s = st.forward(x, train)
            cur.append(y)
            rec(("stem", st, s))
        if self.slowfast:
            cat, s = self.fuses[0].forward(cur[0], cur[1], train)
            rec(("fuse", self.fuses[0], s))
            cur = [cat, cur[1]]
        for i, stage in enumerate(self.stages):
            for pw, units in enumerate(stage):
                x = cur[pw]
                for u in units:
                    x, s = u.forward(x, train)
                    rec(("unit", (pw, u), s))
                cur[pw] = x
            if self.slowfast and self.fuses[i + 1] is not None:
                cat, s = self.fuses[i + 1].forward(cur[0], cur[1], train)
                rec(("fuse", self.fuses[i + 1], s))
                cur = [cat, cur[1]]
        return cur

    def _pool(self, outs: List[torch.Tensor]):
        """PoolConcatPathway / head AvgPool3d (stride 1) into feat [N, P, sum C]; global mean per pathway when the
        pooled grids disagree (models/reference.PoolConcatPathway)."""
        shapes, ks = [], []
        for o, k in zip(outs, self.head_pools):
            thw = tuple(o.shape[1:4])
            k = thw if k is None else k
            ks.append(k)
            shapes.append(tuple(max(d - kk + 1, 0) for d, kk in zip(thw, k)))
        if not (all(s == shapes[0] for s in shapes) and all(v > 0 for v in shapes[0])):
            ks = [tuple(o.shape[1:4]) for o in outs]
            shapes = [(1, 1, 1)] * len(outs)
        P = shapes[0][0] * shapes[0][1] * shapes[0][2]
        Ct = sum(o.shape[-1] for o in outs)
        N = outs[0].shape[0]
        feat = torch.empty(N, P, Ct, device=self.device)
        coff = 0
        for o, k in zip(outs, ks):
            N, T, H, W, C = o.shape
            self.F.avgpool32(0, o, feat, [N, T, H, W, C], list(k), Ct, coff)
            coff += C
        return feat, ks

    def _head_forward(self, feat, train: bool):
        h = self.head
        W, b = h.proj.weight, h.proj.bias
        p = float(h.dropout.p) if (train and h.dropout is not None) else 0.0
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0
        N = feat.shape[0]
        xm = torch.empty(N, feat.shape[2], device=self.device)
        logits = torch.empty(N, W.shape[0], device=self.device)
        self.C.head_forward(feat, W, b, p, seed, xm, logits, None)
        return logits, xm, p, seed

    @torch.no_grad()
    def forward_eval(self, video) -> torch.Tensor:
        outs = self._backbone(self._inputs(video), False, None)
        feat, _ = self._pool(outs)
        logits, _, _, _ = self._head_forward(feat, False)
        return logits

    @torch.no_grad()
    def eval_counts(self, logits: torch.Tensor, labels: torch.Tensor, counts: Optional[torch.Tensor] = None):
        """Top-1 (correct, total) int64 counters on the HIP argmax/count kernel (reference run.py:297)."""
        N = logits.shape[0]
        acc = 1
        if counts is None:
            counts = torch.zeros(2, device=self.device, dtype=torch.long)
            acc = 0
        rl = torch.empty(max(N, 1), device=self.device)
        rc = torch.empty(max(N, 1), device=self.device, dtype=torch.int32)
        self.C.head_ce(logits.contiguous(), labels.to(self.device, torch.long).contiguous(), 0.0, None, None, counts,
                       acc, rl, rc)
        return counts

    # ------------------------------------------------------------------ training step
    @torch.no_grad()
    def forward_backward(self, video, labels: torch.Tensor, loss_scale: float = 1.0,
                         accumulate: Optional[bool] = None):
        """One training micro-step: gradients of ``loss * loss_scale`` written (first micro-step after zero_grad) or
        added into the flat fp32 gradient buffer.  Returns (loss [1], logits [N, K])."""
        if accumulate is None:
            accumulate = not self.flat.zeroed
        self.flat.zeroed = False
        self.grad_beta = 1.0 if accumulate else 0.0
        self._reset_progress()
        tape: list = []
        outs = self._backbone(self._inputs(video), True, tape)
        feat, ks = self._pool(outs)
        logits, xm, p, seed = self._head_forward(feat, True)
        N, K = logits.shape
        labels = labels.to(self.device, torch.long).contiguous()
        loss = torch.empty(1, device=self.device)
        dlogits = torch.empty(N, K, device=self.device)
        rl = torch.empty(max(N, 1), device=self.device)
        rc = torch.empty(max(N, 1), device=self.device, dtype=torch.int32)
        self.C.head_ce(logits, labels, float(loss_scale) / max(N, 1), dlogits, loss, None, 0, rl, rc)
        h = self.head
        W, b = h.proj.weight, h.proj.bias
        train_backbone = any(q.requires_grad for u in self.stems for q in u.cb.conv.parameters())
        Ct = feat.shape[2]
        dfeat = torch.empty_like(feat) if train_backbone else None
        scratch = torch.empty(K * N + Ct * N + Ct * K, device=self.device)
        self.C.head_backward(dlogits, xm, W, feat.shape[1], p, seed, self.flat.gview(W),
                             None if b is None else self.flat.gview(b), self.grad_beta, dfeat, scratch, None)
        self.done(*[q for q in (W, b) if q is not None])
        if train_backbone:
            self._backward_backbone(tape, outs, dfeat, ks)
        return loss, logits

    def _backward_backbone(self, tape, outs, dfeat, ks):
        """Reverse walk of the tape.  The tape order (per stage block: slow units, fast units, fusion) reversed is
        the flat parameter order (fusion, fast units, slow units), so gradients complete front to back."""
        F = self.F
        Ct = dfeat.shape[2]
        grads: List[Optional[torch.Tensor]] = []
        coff = 0
        for o, k in zip(outs, ks):
            N, T, H, W, C = o.shape
            d = torch.empty_like(o)
            F.avgpool32(1, dfeat, d, [N, T, H, W, C], list(k), Ct, coff)
            grads.append(d)
            coff += C
        del outs
        while tape:
            kind, op, s = tape.pop()
            if kind == "fuse":
                # the fast pathway tensor feeds both the lateral conv and the next fast stage, whose input gradient
                # (grads[1]) is already complete: the lateral input gradient is accumulated into it
                grads[0] = op.backward(s, grads[0], grads[1])
            elif kind == "unit":
                pw, u = op
                grads[pw] = u.backward(s, grads[pw], True)
            else:   # stem
                pw = self.stems.index(op)
                op.backward(s, grads[pw])
                grads[pw] = None
