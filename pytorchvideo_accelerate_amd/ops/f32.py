"""Host side of the fp32 kernels (``csrc/fp32``, ``_C.f32``): convolution geometry, tap tables and launch helpers.

Activations are NDHWC fp32 tensors ``[N, T, H, W, C]`` (rows of C channels, C a multiple of 4).  A convolution
(PyTorch ``Conv3d`` semantics, weight ``[Cout, Cin, kt, kh, kw]``) runs as

* forward: one implicit GEMM over output positions, K = taps x Cin (``igemm32``);
* input gradient: one implicit GEMM per stride phase (dX positions ``q*s + r``): only the taps whose
  ``(r + p - a) % s == 0`` contribute, each reading dY at ``q + (r + p - a) / s`` — dense gathers, no structural
  zeros (a phase with no tap writes zeros);
* weight gradient: positions on the reduction axis (``wgrad32``), then an unpack into PyTorch's weight layout.

All three run on split-bf16 MFMA (``csrc/fp32/conv32.hip``): each fp32 operand as ``pieces`` bf16 values — 3 (the
default, arm ``f32_pieces``): 24-bit operands and six products per fragment pair, fp32 accuracy at a sixth of the
bf16 matrix rate; 2: ~16-bit operands, three products.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import torch

Triple = Tuple[int, int, int]


def ceil_div(a: int, b: int) -> int:
    return -(-a // b)


@dataclass
class ConvGeom:
    cin: int
    cout: int
    k: Triple
    s: Triple
    p: Triple
    cip: int = 0          # input channels as stored (>= cin, multiple of 4; the stem's RGB is padded to 4)
    _taps: Dict = field(default_factory=dict, repr=False)

    def __post_init__(self):
        if not self.cip:
            self.cip = self.cin
        assert self.cip % 4 == 0 and self.cip >= self.cin, "fp32 convs need channel counts that are multiples of 4"
        assert self.cout % 4 == 0

    @property
    def ntap(self) -> int:
        return self.k[0] * self.k[1] * self.k[2]

    def out_thw(self, thw: Triple) -> Triple:
        return tuple((i + 2 * p - k) // s + 1 for i, k, s, p in zip(thw, self.k, self.s, self.p))

    def _tab(self, key, rows: List[Tuple[int, int, int, int]], device) -> torch.Tensor:
        t = self._taps.get((key, str(device)))
        if t is None:
            flat = [v for r in rows for v in r] or [0, 0, 0, 0]
            t = torch.tensor(flat, dtype=torch.int32).to(device)
            self._taps[(key, str(device))] = t
        return t

    def taps_fwd(self, device) -> torch.Tensor:
        kt, kh, kw = self.k
        pt, ph, pw = self.p
        rows = [(a - pt, b - ph, e - pw, (a * kh + b) * kw + e) for a in range(kt) for b in range(kh) for e in range(kw)]
        return self._tab("fwd", rows, device)

    def phases(self, device):
        """[(phase r, tap table, number of taps)] of the input gradient."""
        out = []
        kt, kh, kw = self.k
        st, sh, sw = self.s
        pt, ph, pw = self.p
        for rt in range(st):
            for rh in range(sh):
                for rw in range(sw):
                    rows = []
                    for a in range(kt):
                        if (rt + pt - a) % st:
                            continue
                        for b in range(kh):
                            if (rh + ph - b) % sh:
                                continue
                            for e in range(kw):
                                if (rw + pw - e) % sw:
                                    continue
                                rows.append(((rt + pt - a) // st, (rh + ph - b) // sh, (rw + pw - e) // sw,
                                             (a * kh + b) * kw + e))
                    out.append(((rt, rh, rw), self._tab(("ph", rt, rh, rw), rows, device), len(rows)))
        return out


def pieces() -> int:
    from ..utils.arms import arm
    return int(arm("f32_pieces"))


def pack_weight(F, g: ConvGeom, w: torch.Tensor, mode: int) -> torch.Tensor:
    """The implicit GEMM's B rows of a torch weight ``[Cout, Cin, kt, kh, kw]`` (fp32), pre-split into the three bf16
    pieces the kernels multiply (``[3][rows][K]``): mode 0 forward rows ``[Cout][taps][cip]``, mode 1 input-gradient
    rows ``[Cin][taps][Cout]``.  Split once per step here instead of once per output tile in every launch."""
    rows, K = (g.cout, g.ntap * g.cip) if mode == 0 else (g.cin, g.ntap * g.cout)
    out = torch.empty(3, rows, K, device=w.device, dtype=torch.bfloat16)
    F.wpack32(mode, w, out, g.cout, g.cin, g.ntap, g.cip, 0.0)
    return out


def _unlazy(x):
    """(tensor, isc, ish, irelu) of a conv operand that may be a models.native32.Lazy activation."""
    if hasattr(x, "stat") and hasattr(x, "y"):
        return x.y, x.stat[2], x.stat[3], 1
    return x, None, None, 0


def conv_fwd(F, g: ConvGeom, x, wf: torch.Tensor, y: torch.Tensor, taps: torch.Tensor,
             stats: torch.Tensor = None):
    """y [N, To, Ho, Wo, Cout] = conv(x [N, T, H, W, cip]) with forward-packed weights wf (pack_weight mode 0);
    ``stats``: per-tile channel sums of y and y^2 ([ceil(M / igemm32_bm(Cout))][2][Cout]) from the epilogue."""
    x, isc, ish, irelu = _unlazy(x)
    N, T, H, W, C = x.shape
    assert C == g.cip
    To, Ho, Wo = g.out_thw((T, H, W))
    assert tuple(y.shape) == (N, To, Ho, Wo, g.cout)
    K = g.ntap * g.cip
    geo = [g.cip, K, g.cout, N * To * Ho * Wo, g.cout, K, g.cip, 0, To, Ho, Wo, T, H, W, *g.s, To, Ho, Wo,
           1, 1, 1, 0, 0, 0]
    F.conv32(x, wf, y, taps, geo, isc=isc, ish=ish, irelu=irelu, np=pieces(), stats=stats)


def conv_dgrad(F, g: ConvGeom, dy: torch.Tensor, wt: torch.Tensor, dx: torch.Tensor, phases):
    """dx [N, T, H, W, cin] = input gradient of dy [N, To, Ho, Wo, Cout] (wt = pack_weight mode 1)."""
    N, T, H, W, C = dx.shape
    assert C == g.cin and C % 4 == 0
    To, Ho, Wo = dy.shape[1:4]
    for (rt, rh, rw), taps, nt in phases:
        Qt, Qh, Qw = ceil_div(T - rt, g.s[0]), ceil_div(H - rh, g.s[1]), ceil_div(W - rw, g.s[2])
        if min(Qt, Qh, Qw) <= 0:
            continue
        geo = [g.cout, g.ntap * g.cout, g.cin, N * Qt * Qh * Qw, g.cin, nt * g.cout, g.cout, 0, Qt, Qh, Qw,
               To, Ho, Wo, 1, 1, 1, T, H, W, *g.s, rt, rh, rw]
        F.conv32(dy, wt, dx, taps, geo, np=pieces())


def conv_wgrad(F, g: ConvGeom, dy: torch.Tensor, x: torch.Tensor, dwf: torch.Tensor, taps: torch.Tensor):
    """dwf [Cout][taps*cip] += weight gradient (caller zeroes it).  ``x`` may be a Lazy activation."""
    x, isc, ish, irelu = _unlazy(x)
    N, T, H, W, C = x.shape
    To, Ho, Wo = dy.shape[1:4]
    K = g.ntap * g.cip
    geo = [g.cout, g.cip, K, g.cout, K, g.cip, N * To * Ho * Wo, To, Ho, Wo, T, H, W, *g.s]
    F.wgrad32(dy, x, dwf, taps, geo, isc=isc, ish=ish, irelu=irelu, np=pieces())
