"""3-D convolution ops on the gfx950 implicit-GEMM kernels (NDHWC bf16).

An activation is an :class:`Act`: a 2-D ``[positions, channels]`` bf16 tensor (possibly a channel
slice of a wider buffer — its row stride is the NDHWC channel pitch) plus the (N, T, H, W) extents.

* :func:`conv_fwd`   — forward; optional per-input-channel affine(+ReLU) on load (the producer's BN),
  optional BN partial statistics of the output.
* :func:`conv_dgrad` — data gradient (optionally accumulated into an existing gradient buffer).
* :func:`conv_wgrad` — weight gradient, split-K over positions, reduced straight into the fp32
  master-gradient tensor in PyTorch's ``[Cout, Cin, kt, kh, kw]`` layout.

Reference semantics: ``torch.nn.functional.conv3d`` with ``bias=False`` (pytorchvideo convs,
SURVEY.md §2.3); numerics are pinned against it in ``tests/test_kernels_gpu.py``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from ._ext import require

Triple = Tuple[int, int, int]


@dataclass
class Act:
    t: torch.Tensor      # [M, C] view, row stride = channel pitch
    N: int
    T: int
    H: int
    W: int

    @property
    def C(self) -> int:
        return self.t.shape[1]

    @property
    def ld(self) -> int:
        return self.t.stride(0)

    @property
    def M(self) -> int:
        return self.N * self.T * self.H * self.W

    def narrow(self, c0: int, c: int) -> "Act":
        return Act(self.t.narrow(1, c0, c), self.N, self.T, self.H, self.W)

    def to_ncthw(self) -> torch.Tensor:
        return self.t.reshape(self.N, self.T, self.H, self.W, self.C).permute(0, 4, 1, 2, 3)

    @staticmethod
    def from_ncthw(x: torch.Tensor, c_pad: Optional[int] = None, dtype: torch.dtype = torch.bfloat16) -> "Act":
        N, C, T, H, W = x.shape
        y = x.permute(0, 2, 3, 4, 1)
        if c_pad is not None and c_pad > C:
            y = torch.nn.functional.pad(y, (0, c_pad - C))
        y = y.contiguous().to(dtype)
        return Act(y.reshape(N * T * H * W, y.shape[-1]), N, T, H, W)


@dataclass
class ConvSpec:
    cin: int
    cout: int
    k: Triple
    stride: Triple = (1, 1, 1)
    pad: Triple = (0, 0, 0)
    cin_pad: int = 0          # packed input channels (stems: 3 -> 4)

    def __post_init__(self):
        if not self.cin_pad:
            self.cin_pad = self.cin

    @property
    def taps(self) -> int:
        return self.k[0] * self.k[1] * self.k[2]

    @property
    def chunk(self) -> int:
        return 8 if self.cin_pad % 8 == 0 else 4

    def out_dims(self, T: int, H: int, W: int) -> Triple:
        o = []
        for i, n in enumerate((T, H, W)):
            o.append((n + 2 * self.pad[i] - self.k[i]) // self.stride[i] + 1)
        return tuple(o)

    def flops(self, N: int, T: int, H: int, W: int) -> int:
        To, Ho, Wo = self.out_dims(T, H, W)
        return 2 * N * To * Ho * Wo * self.cout * self.cin * self.taps


def pack_weight(w: torch.Tensor, spec: ConvSpec, dtype: torch.dtype = torch.bfloat16) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 [Cout, Cin, kt, kh, kw] -> (16-bit forward pack [Cout, taps, Cin_pad], dgrad pack [Cin, taps, Cout]).

    Host-side (torch) version used by tests and one-off packs; the training loop uses the multi-tensor
    ``pack_weights`` kernel (ops/optim.py).
    """
    co, ci = w.shape[:2]
    wf = w.reshape(co, ci, -1).permute(0, 2, 1)  # [Cout, taps, Cin]
    if spec.cin_pad > ci:
        wf = torch.nn.functional.pad(wf, (0, spec.cin_pad - ci))
    wd = w.reshape(co, ci, -1).permute(1, 2, 0)  # [Cin, taps, Cout]
    return wf.contiguous().to(dtype), wd.contiguous().to(dtype)


def fwd_geometry(spec: ConvSpec, N: int, T: int, H: int, W: int, ldx: int, ldy: int) -> list:
    """Forward geometry vector (see ConvParams in csrc/kernels/conv_params.h)."""
    To, Ho, Wo = spec.out_dims(T, H, W)
    (kt, kh, kw), (st, sh, sw), (pt, ph, pw) = spec.k, spec.stride, spec.pad
    M = N * To * Ho * Wo
    return [M, spec.cout, spec.taps * spec.cin_pad, spec.cin_pad, ldx, ldy, T, H, W, To, Ho, Wo, To, Ho, Wo,
            1, 1, 1, 0, 0, 0, st, sh, sw, -pt, -ph, -pw, 1, kt, kh, kw, kh, kw, 0, 0, 0, 1, 1, 1]


def dgrad_phases(spec: ConvSpec, N: int, in_dims: Triple, out_dims: Triple, ldx: int, ldy: int) -> list:
    """Per-stride-phase dgrad geometry vectors.

    Input positions i = q*s + r (phase r) receive contributions only from taps d = d0 + j*s with
    d0 = (r + pad) mod s, gathered at g = q + (r + pad - d0)/s - j: a dense stride-1 gather per phase.
    A phase with no contributing tap (e.g. odd positions of a 1x1 stride-2 conv) has n = 0: the launch
    just writes zeros.
    """
    geo = []
    Ti, Hi, Wi = in_dims
    To, Ho, Wo = out_dims
    k, s, p = spec.k, spec.stride, spec.pad
    for rt in range(s[0]):
        for rh in range(s[1]):
            for rw in range(s[2]):
                R, ao, d0, n = [], [], [], []
                for dim, r in enumerate((rt, rh, rw)):
                    I = in_dims[dim]
                    dd = (r + p[dim]) % s[dim]
                    nn = (k[dim] - dd + s[dim] - 1) // s[dim] if dd < k[dim] else 0
                    R.append((I - r + s[dim] - 1) // s[dim])
                    ao.append((r + p[dim] - dd) // s[dim])
                    d0.append(dd)
                    n.append(nn)
                if min(R) <= 0:
                    continue
                if min(n) == 0:
                    n = [0, 0, 0]
                M = N * R[0] * R[1] * R[2]
                geo.append([M, spec.cin, spec.taps * spec.cout, spec.cout, ldx, ldy, To, Ho, Wo, R[0], R[1], R[2],
                            Ti, Hi, Wi, s[0], s[1], s[2], rt, rh, rw, 1, 1, 1, ao[0], ao[1], ao[2], -1,
                            n[0], n[1], n[2], k[1], k[2], d0[0], d0[1], d0[2], s[0], s[1], s[2]])
    return geo


def conv_m_tiles(M: int, N: int, spec: Optional["ConvSpec"] = None) -> int:
    """Row tiles of the forward BN partial sums (``spec`` selects the kernel family the launch will use)."""
    if spec is None:
        return require().conv_m_tiles(M, N)
    return require().conv_m_tiles(M, N, spec.taps * spec.cin_pad, spec.cin_pad)


def conv_fwd(x: Act, wpack: torch.Tensor, spec: ConvSpec, out: Optional[torch.Tensor] = None,
             stats: Optional[torch.Tensor] = None, in_scale: Optional[torch.Tensor] = None,
             in_shift: Optional[torch.Tensor] = None, in_relu: bool = True, cfg: int = -1) -> Act:
    """``cfg``: launch configuration word (ops/tune.py; -1 = the kernel's heuristic)."""
    C = require()
    assert x.C == spec.cin_pad, (x.C, spec.cin_pad)
    To, Ho, Wo = spec.out_dims(x.T, x.H, x.W)
    M = x.N * To * Ho * Wo
    if out is None:
        out = torch.empty(M, spec.cout, device=x.t.device, dtype=x.t.dtype)
    affine = 0 if in_scale is None else (2 if in_relu else 1)
    g = fwd_geometry(spec, x.N, x.T, x.H, x.W, x.ld, out.stride(0))
    C.conv_igemm(x.t, wpack, out, stats, in_scale, in_shift, affine, 0, g, spec.chunk, cfg)
    return Act(out, x.N, To, Ho, Wo)


def conv_dgrad(dy: Act, wt_pack: torch.Tensor, spec: ConvSpec, in_dims: Triple, out: Optional[torch.Tensor] = None,
               accum: bool = False, cfg: int = -1) -> Act:
    """dX[N,Ti,Hi,Wi,Cin] = conv_transpose(dY, W); ``accum`` adds into ``out``."""
    C = require()
    Ti, Hi, Wi = in_dims
    assert dy.C == spec.cout and spec.cin % 8 == 0 and spec.cout % 8 == 0
    M = dy.N * Ti * Hi * Wi
    if out is None:
        out = torch.empty(M, spec.cin, device=dy.t.device, dtype=dy.t.dtype)
    for g in dgrad_phases(spec, dy.N, in_dims, (dy.T, dy.H, dy.W), dy.ld, out.stride(0)):
        if accum and g[28] == 0:
            continue
        C.conv_igemm(dy.t, wt_pack, out, None, None, None, 0, 1 if accum else 0, g, 8, cfg)
    return Act(out, dy.N, Ti, Hi, Wi)


def wgrad_splits(P: int, Cout: int, K: int, target_blocks: int = 1024, min_rows: int = 1024,
                 variant: int = -1) -> Tuple[int, int]:
    C = require()
    bmw, bnw = C.wgrad_tile(Cout, K, variant)
    tiles = ((Cout + bmw - 1) // bmw) * ((K + bnw - 1) // bnw)
    splits = max(1, min(target_blocks // max(tiles, 1), (P + min_rows - 1) // min_rows))
    pps = (P + splits - 1) // splits
    pps = (pps + 63) // 64 * 64      # whole 32- or 64-position stages
    splits = (P + pps - 1) // pps
    return splits, pps


HALO = 32   # wgrad launch-word bit of the halo-staged kernel (csrc/kernels/wgrad_halo.hip)


def halo_wgrad_plan(spec: "ConvSpec", P: int, dims: Tuple[int, int, int], option: int = 0,
                    target_blocks: int = 512) -> Optional[Tuple[int, int, int]]:
    """(workgroups along the boxes, boxes per workgroup, launch word) of the halo-staged weight gradient for a
    stride-1 'same'-padded conv whose output grid is ``dims`` = (T, H, W), or None when the shape does not
    suit it.  ``option`` picks the box size: 0 ~32 KB, 1 ~64 KB staged (BT frames x BH rows of the full width)."""
    T, H, W = dims
    kt, kh, kw = spec.k
    if tuple(spec.stride) != (1, 1, 1) or tuple(spec.pad) != ((kt - 1) // 2, (kh - 1) // 2, (kw - 1) // 2):
        return None
    if spec.taps == 1 or spec.cout > 128 or spec.cin_pad % 8 or spec.chunk != 8 or W >= 1024 or H >= 1024:
        return None
    # box size by bytes staged per box (dY + halo): ~32 KB (option 0) / ~64 KB (option 1); rows first (up to
    # the full height), then frames (a kt=1 box of several frames is several 2-D halos)
    target = (32 << 10) << option
    coutp = (spec.cout + 15) // 16 * 16
    per_pos = 2 * (coutp + spec.cin_pad)
    BT = 1 if kt == 1 else 2
    BH = max(1, min(H, 15, target // max(1, per_pos * BT * W)))
    if BH >= H:
        BT = max(BT, min(T, 7, target // max(1, per_pos * H * W)))

    def fits(bt, bh):   # the kernel's staging limits (wgrad_halo.hip: HX_RA / HX_RB registers, LDS budget)
        pbp = (bt * bh * W + 31) // 32 * 32
        hp = (bt + kt - 1) * (bh + kh - 1) * (W + kw - 1)
        lds = pbp * coutp * 2 + hp * spec.cin_pad * 2 + (2 * pbp + hp) * 4 + spec.cin_pad * 8
        return pbp * coutp // 8 <= 4 * 512 and hp * spec.cin_pad // 8 <= 6 * 512 and lds <= 150 * 1024
    while not fits(BT, BH) and (BT > (1 if kt == 1 else 2) or BH > 1):
        if BT > (1 if kt == 1 else 2):
            BT -= 1
        else:
            BH -= 1
    if not fits(BT, BH):
        return None
    NT = (spec.cout + 15) // 16
    if NT not in (1, 2, 4, 8):
        return None
    K = spec.taps * spec.cin_pad
    KT = (K + 15) // 16
    WK = 8 if KT >= 16 else (2 if KT >= 4 else 1)
    wpl = {8: 0, 2: 2, 1: 3}[WK]
    ktw_max = min(8, 24 // NT)   # accumulators <= 96 VGPRs (the box staging needs the rest)
    groups = -(-KT // (WK * ktw_max))
    ktb = -(-KT // groups)
    if ktb > 255:
        return None
    nboxes = (P // (T * H * W)) * -(-T // BT) * -(-H // BH)
    splits = max(1, min(nboxes, -(-target_blocks // groups)))
    bps = -(-nboxes // splits)
    splits = -(-nboxes // bps)
    return splits, bps, HALO | (BH << 8) | (BT << 12) | (wpl << 15) | (ktb << 17)


RT = 1 << 25    # wgrad launch-word bit of the row-table kernel for gathered shapes (csrc/kernels/wgrad_rt_impl.h)
BOX = 1 << 26   # wgrad launch-word bit of the box-staged (1,3,3) kernel (csrc/kernels/wgrad_box.hip)


def box_wgrad_plan(spec: "ConvSpec", P: int, dims: Tuple[int, int, int], ldd: int, ldx: int,
                   target_blocks: int = 512) -> Optional[Tuple[int, int, int]]:
    """(box ranges, boxes per range, launch word) of the box-staged weight gradient of a stride-1 'same' (1,3,3)
    conv with 64-multiple channel counts (or Cin = Cout in {8, 16, 32}) whose output grid is ``dims``, or None.
    The grid is (Cout/64)*(Cin/64) channel groups x box ranges, ~``target_blocks`` workgroups (two per CU); each
    range writes its own slab (narrow: four, one per wave — see ``box_wgrad_slabs``)."""
    T, H, W = dims
    g = [P, spec.cout, spec.taps * spec.cin_pad, spec.cin_pad, ldd, ldx, T, H, W, T, H, W, *spec.k, *spec.stride,
         *spec.pad]
    R = int(require().wgrad_box_legal(g))
    if R <= 0 or spec.cin_pad != spec.cin:
        return None
    # wide: (Cout/64)*(Cin/64) channel groups per box range; narrow (C <= 32): one workgroup per range
    groups = (spec.cout // 64) * (spec.cin // 64) if spec.cin >= 64 else 1
    nboxes = P // (R * W)
    splits = max(1, min(nboxes, -(-target_blocks // groups)))
    bps = -(-nboxes // splits)
    return -(-nboxes // bps), bps, BOX


def box_wgrad_slabs(spec: "ConvSpec", splits: int) -> int:
    """Slabs the box-staged kernel writes for ``splits`` box ranges (narrow variant: one per wave)."""
    return splits * (4 if spec.cin < 64 else 1)


def conv_wgrad(dy: Act, x: Act, spec: ConvSpec, grad: torch.Tensor, workspace: Optional[torch.Tensor] = None,
               in_scale: Optional[torch.Tensor] = None, in_shift: Optional[torch.Tensor] = None,
               in_relu: bool = True, scale: float = 1.0, beta: float = 0.0,
               splits_pps: Optional[Tuple[int, int]] = None, variant: int = -1, slab: bool = False) -> torch.Tensor:
    """grad (fp32, [Cout, Cin, kt, kh, kw]) = beta*grad + scale * dW.

    ``slab``: every split writes its own fp32 slab (no atomics) and the slabs are summed in a fixed order
    (bitwise reproducible; the fused executor's deterministic mode and BN-fold products).

    ``variant``: -1 = heuristic tile; else bits 0-1 (+ bit 3 -> tiles 4-7) = tile (16x128, 32x128, 64x64, 128x64,
    128x128, 256x128, 128x256, 256x256), bit 2 = 64-position LDS stages (two MFMA k-steps per barrier);
    ``HALO | option`` (option 0/1 in bits 0-1) = the halo-staged kernel with box option ``option``; ``BOX`` = the
    box-staged (1,3,3) kernel (64-multiple channels)."""
    C = require()
    P = dy.M
    K = spec.taps * spec.cin_pad
    if splits_pps is None and variant >= 0 and variant & 16:   # narrow per-wave kernel (Cout <= 32, K <= 128)
        nw = 2048
        pps = ((P + nw - 1) // nw + 63) // 64 * 64
        splits_pps = ((P + pps - 1) // pps, pps)
        variant = 16
    if variant == BOX:   # box-staged kernel: per-range slabs + fixed-order two-pass reduction
        C = require()
        plan = box_wgrad_plan(spec, P, (dy.T, dy.H, dy.W), dy.ld, x.ld)
        assert plan is not None, "box wgrad does not apply to this conv"
        splits, bps, word = plan
        K = spec.taps * spec.cin_pad
        nslab = box_wgrad_slabs(spec, splits)
        slab = torch.empty(nslab * spec.cout * K, device=dy.t.device, dtype=torch.float32)
        tmp = torch.empty(C.box_reduce_groups(nslab) * spec.cout * K, device=dy.t.device, dtype=torch.float32)
        affine = 0 if in_scale is None else (2 if in_relu else 1)
        g = [P, spec.cout, K, spec.cin_pad, dy.ld, x.ld, x.T, x.H, x.W, dy.T, dy.H, dy.W,
             *spec.k, *spec.stride, *spec.pad, splits, bps]
        C.conv_wgrad(dy.t, x.t, slab, in_scale, in_shift, affine, g, spec.chunk, 1, word)
        C.wgrad_box_reduce(slab, tmp, grad, nslab, spec.cout, spec.taps, spec.cin_pad, spec.cin, scale, beta)
        return grad
    if splits_pps is None and variant >= 0 and variant & HALO and variant < 256:   # halo kernel, box option
        plan = halo_wgrad_plan(spec, P, (dy.T, dy.H, dy.W), variant & 3)
        assert plan is not None, "halo wgrad does not apply to this conv"
        splits_pps, variant = plan[:2], plan[2]
    splits, pps = splits_pps or wgrad_splits(P, spec.cout, K, variant=(variant & 11) if variant >= 0 else -1)
    need = spec.cout * K * (splits if slab else 1)
    if workspace is None or workspace.numel() < need:
        workspace = torch.zeros(need, device=dy.t.device, dtype=torch.float32)  # kept zero by wgrad_reduce
    affine = 0 if in_scale is None else (2 if in_relu else 1)
    g = [P, spec.cout, K, spec.cin_pad, dy.ld, x.ld, x.T, x.H, x.W, dy.T, dy.H, dy.W,
         *spec.k, *spec.stride, *spec.pad, splits, pps]
    C.conv_wgrad(dy.t, x.t, workspace, in_scale, in_shift, affine, g, spec.chunk, int(slab), variant)
    C.wgrad_reduce(workspace, grad, splits, spec.cout, spec.taps, spec.cin_pad, spec.cin, scale, beta, int(slab))
    return grad


# --------------------------------------------------------------------------------------------
# torch references (used by tests and by the CPU path)
# --------------------------------------------------------------------------------------------
def ref_conv(x_ncthw: torch.Tensor, w: torch.Tensor, spec: ConvSpec) -> torch.Tensor:
    return torch.nn.functional.conv3d(x_ncthw, w, None, spec.stride, spec.pad)
