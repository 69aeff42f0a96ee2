"""Pure-PyTorch reference ("oracle") networks: SlowFast-R50/R101 and Slow-R50.

These modules mirror the module tree of pytorchvideo's model builders so that the
``state_dict`` key names are identical to what ``torch.hub.load(
"facebookresearch/pytorchvideo", "slowfast_r50")`` produces and what the
reference script checkpoints (reference ``run.py:105-118``).
Key layout examples::

    blocks.0.multipathway_blocks.0.conv.weight
    blocks.1.multipathway_blocks.0.res_blocks.0.branch2.conv_a.weight
    blocks.0.multipathway_fusion.conv_fast_to_slow.weight
    blocks.6.proj.weight

They are built only from ``torch.nn`` ops, run on CPU, and are the numerical
oracle for the fused HIP engine (``models/fused.py``), which shares their
parameters and buffers.  Layout is NCTHW (PyTorch's native Conv3d layout).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

Triple = Tuple[int, int, int]

BN_EPS = 1e-5
BN_MOMENTUM = 0.1


def _conv(cin: int, cout: int, k: Triple, s: Triple = (1, 1, 1), p: Optional[Triple] = None) -> nn.Conv3d:
    if p is None:
        p = tuple(x // 2 for x in k)
    return nn.Conv3d(cin, cout, kernel_size=k, stride=s, padding=p, bias=False)


def _bn(c: int) -> nn.BatchNorm3d:
    return nn.BatchNorm3d(c, eps=BN_EPS, momentum=BN_MOMENTUM)


class ResNetBasicStem(nn.Module):
    """conv → BN → ReLU → MaxPool3d (pytorchvideo ``ResNetBasicStem``)."""

    def __init__(self, cin: int, cout: int, k: Triple, s: Triple, p: Triple,
                 pool_k: Triple = (1, 3, 3), pool_s: Triple = (1, 2, 2), pool_p: Triple = (0, 1, 1)):
        super().__init__()
        self.conv = _conv(cin, cout, k, s, p)
        self.norm = _bn(cout)
        self.activation = nn.ReLU(inplace=True)
        self.pool = nn.MaxPool3d(pool_k, pool_s, pool_p)

    def forward(self, x):
        return self.pool(self.activation(self.norm(self.conv(x))))


class BottleneckBlock(nn.Module):
    """conv_a (kt,1,1) → conv_b (1,3,3)/stride → conv_c (1,1,1); BN after each."""

    def __init__(self, cin: int, inner: int, cout: int, kt: int, spatial_stride: int):
        super().__init__()
        self.conv_a = _conv(cin, inner, (kt, 1, 1))
        self.norm_a = _bn(inner)
        self.act_a = nn.ReLU(inplace=True)
        self.conv_b = _conv(inner, inner, (1, 3, 3), (1, spatial_stride, spatial_stride), (0, 1, 1))
        self.norm_b = _bn(inner)
        self.act_b = nn.ReLU(inplace=True)
        self.conv_c = _conv(inner, cout, (1, 1, 1))
        self.norm_c = _bn(cout)

    def forward(self, x):
        x = self.act_a(self.norm_a(self.conv_a(x)))
        x = self.act_b(self.norm_b(self.conv_b(x)))
        return self.norm_c(self.conv_c(x))


class ResBlock(nn.Module):
    """Residual unit: ``relu(branch1(x) + branch2(x))``; branch1 only when shapes change."""

    def __init__(self, cin: int, inner: int, cout: int, kt: int, spatial_stride: int):
        super().__init__()
        if cin != cout or spatial_stride != 1:
            self.branch1_conv = _conv(cin, cout, (1, 1, 1), (1, spatial_stride, spatial_stride), (0, 0, 0))
            self.branch1_norm = _bn(cout)
        else:
            self.branch1_conv = None
            self.branch1_norm = None
        self.branch2 = BottleneckBlock(cin, inner, cout, kt, spatial_stride)
        self.activation = nn.ReLU(inplace=True)

    def forward(self, x):
        sc = x if self.branch1_conv is None else self.branch1_norm(self.branch1_conv(x))
        return self.activation(sc + self.branch2(x))


class ResStage(nn.Module):
    def __init__(self, depth: int, cin: int, inner: int, cout: int, kt: int, spatial_stride: int):
        super().__init__()
        blocks = []
        for i in range(depth):
            blocks.append(ResBlock(cin if i == 0 else cout, inner, cout, kt, spatial_stride if i == 0 else 1))
        self.res_blocks = nn.ModuleList(blocks)

    def forward(self, x):
        for b in self.res_blocks:
            x = b(x)
        return x


class FuseFastToSlow(nn.Module):
    """Lateral connection: conv(7,1,1)/stride(α,1,1) on fast → BN → ReLU → concat to slow."""

    def __init__(self, fast_c: int, fusion_ratio: int = 2, kt: int = 7, alpha: int = 4):
        super().__init__()
        self.conv_fast_to_slow = nn.Conv3d(fast_c, fast_c * fusion_ratio, (kt, 1, 1), (alpha, 1, 1),
                                           (kt // 2, 0, 0), bias=False)
        self.norm = _bn(fast_c * fusion_ratio)
        self.activation = nn.ReLU(inplace=True)

    def forward(self, xs: List[torch.Tensor]):
        x_s, x_f = xs
        f = self.activation(self.norm(self.conv_fast_to_slow(x_f)))
        return [torch.cat([x_s, f], 1), x_f]


class MultiPathWayWithFuse(nn.Module):
    def __init__(self, multipathway_blocks: Sequence[nn.Module], multipathway_fusion: Optional[nn.Module]):
        super().__init__()
        self.multipathway_blocks = nn.ModuleList(multipathway_blocks)
        self.multipathway_fusion = multipathway_fusion

    def forward(self, xs):
        ys = [blk(x) for blk, x in zip(self.multipathway_blocks, xs)]
        if self.multipathway_fusion is not None:
            ys = self.multipathway_fusion(ys)
        return ys


class PoolConcatPathway(nn.Module):
    """Per-pathway AvgPool3d (stride 1) then channel concat.

    Exact overlapping-window semantics when the pooled shapes agree (e.g. 256²
    crops give a (1,2,2) grid).  When they do not agree (the
    64-frame SlowFast config, which crashes the stock pytorchvideo head) we fall
    back to a global average per pathway — a documented deviation.
    """

    def __init__(self, kernels: Sequence[Triple]):
        super().__init__()
        self.pool = nn.ModuleList([nn.AvgPool3d(k, stride=1) for k in kernels])

    @staticmethod
    def pooled_shape(in_thw: Triple, k: Triple) -> Triple:
        return tuple(max(i - kk + 1, 0) for i, kk in zip(in_thw, k))

    def forward(self, xs):
        shapes = [self.pooled_shape(tuple(x.shape[2:]), p.kernel_size) for x, p in zip(xs, self.pool)]
        if all(s == shapes[0] for s in shapes) and all(v > 0 for v in shapes[0]):
            return torch.cat([p(x) for p, x in zip(self.pool, xs)], 1)
        return torch.cat([x.mean(dim=(2, 3, 4), keepdim=True) for x in xs], 1)


class ResNetBasicHead(nn.Module):
    """pool? → Dropout → Linear (channels-last) → AdaptiveAvgPool3d(1) → flatten."""

    def __init__(self, in_features: int, out_features: int, pool: Optional[nn.Module], dropout_rate: float = 0.5):
        super().__init__()
        self.pool = pool
        self.dropout = nn.Dropout(dropout_rate) if dropout_rate > 0 else None
        self.proj = nn.Linear(in_features, out_features)
        self.output_pool = nn.AdaptiveAvgPool3d(1)
        nn.init.normal_(self.proj.weight, mean=0.0, std=0.01)
        nn.init.zeros_(self.proj.bias)

    def forward(self, x):
        if self.pool is not None:
            x = self.pool(x)
        if self.dropout is not None:
            x = self.dropout(x)
        x = x.permute(0, 2, 3, 4, 1)
        x = self.proj(x)
        x = x.permute(0, 4, 1, 2, 3)
        x = self.output_pool(x)
        return x.reshape(x.shape[0], -1)


class Net(nn.Module):
    def __init__(self, blocks: Sequence[nn.Module]):
        super().__init__()
        self.blocks = nn.ModuleList(blocks)

    def forward(self, x):
        for b in self.blocks:
            x = b(x)
        return x


def create_res_basic_head(in_features: int, out_features: int, pool: Optional[str] = "default",
                          pool_kernel_size: Triple = (1, 7, 7), dropout_rate: float = 0.5) -> ResNetBasicHead:
    """Same contract as pytorchvideo ``create_res_basic_head`` (reference run.py:109,117).

    ``pool=None`` → no pooling before the projection (SlowFast head); the default
    is ``AvgPool3d(pool_kernel_size, stride 1)`` (Slow-R50 head).
    """
    p = None if pool is None else nn.AvgPool3d(pool_kernel_size, stride=1)
    return ResNetBasicHead(in_features, out_features, p, dropout_rate)


def init_net_weights(model: nn.Module, init_std: float = 0.01) -> nn.Module:
    """pytorchvideo ``init_net_weights(style="resnet")``: kaiming-normal fan_out convs,
    BN γ=1 β=0, Linear N(0, std)."""
    for m in model.modules():
        if isinstance(m, nn.Conv3d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.BatchNorm3d):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, mean=0.0, std=init_std)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
    return model


# --------------------------------------------------------------------------------------
# Builders
# --------------------------------------------------------------------------------------
_DEPTHS = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3)}


def create_slowfast(model_depth: int = 50, num_classes: int = 400, alpha: int = 4, beta_inv: int = 8,
                    fusion_ratio: int = 2, fusion_kt: int = 7,
                    head_pool_kernel_sizes: Sequence[Triple] = ((8, 7, 7), (32, 7, 7)),
                    dropout_rate: float = 0.5, head_pool: bool = True) -> Net:
    """SlowFast (Feichtenhofer et al. 2019) as built by pytorchvideo ``create_slowfast``.

    Slow pathway: stem 64 ch (1,7,7); stages 256/512/1024/2048 with inner 64..512.
    Fast pathway: stem 64/β ch (5,7,7); stages /β.  Lateral fusion after stem and
    res2..res4: conv (fusion_kt,1,1) stride (α,1,1), ×fusion_ratio channels.
    """
    depths = _DEPTHS[model_depth]
    s_stem, f_stem = 64, 64 // beta_inv
    s_out = [256, 512, 1024, 2048]
    s_inner = [64, 128, 256, 512]
    f_out = [c // beta_inv for c in s_out]
    f_inner = [c // beta_inv for c in s_inner]
    s_kt = [1, 1, 3, 3]
    f_kt = [3, 3, 3, 3]
    strides = [1, 2, 2, 2]

    def fuse(fc):
        return FuseFastToSlow(fc, fusion_ratio, fusion_kt, alpha)

    blocks: List[nn.Module] = []
    blocks.append(MultiPathWayWithFuse(
        [ResNetBasicStem(3, s_stem, (1, 7, 7), (1, 2, 2), (0, 3, 3)),
         ResNetBasicStem(3, f_stem, (5, 7, 7), (1, 2, 2), (2, 3, 3))],
        fuse(f_stem)))
    s_in = s_stem + f_stem * fusion_ratio
    f_in = f_stem
    for i in range(4):
        fusion = fuse(f_out[i]) if i < 3 else None
        blocks.append(MultiPathWayWithFuse(
            [ResStage(depths[i], s_in, s_inner[i], s_out[i], s_kt[i], strides[i]),
             ResStage(depths[i], f_in, f_inner[i], f_out[i], f_kt[i], strides[i])],
            fusion))
        s_in = s_out[i] + (f_out[i] * fusion_ratio if i < 3 else 0)
        f_in = f_out[i]
    blocks.append(PoolConcatPathway(head_pool_kernel_sizes))
    init_net_weights(nn.Sequential(*blocks))
    blocks.append(create_res_basic_head(s_out[-1] + f_out[-1], num_classes, pool=None, dropout_rate=dropout_rate))
    return Net(blocks)


def create_resnet(model_depth: int = 50, num_classes: int = 400, head_pool_kernel_size: Triple = (8, 7, 7),
                  dropout_rate: float = 0.5) -> Net:
    """Slow-only ResNet3D (pytorchvideo ``create_resnet`` as used by hub ``slow_r50``)."""
    depths = _DEPTHS[model_depth]
    out = [256, 512, 1024, 2048]
    inner = [64, 128, 256, 512]
    kt = [1, 1, 3, 3]
    strides = [1, 2, 2, 2]
    blocks: List[nn.Module] = [ResNetBasicStem(3, 64, (1, 7, 7), (1, 2, 2), (0, 3, 3))]
    cin = 64
    for i in range(4):
        blocks.append(ResStage(depths[i], cin, inner[i], out[i], kt[i], strides[i]))
        cin = out[i]
    init_net_weights(nn.Sequential(*blocks))
    blocks.append(create_res_basic_head(2048, num_classes, pool="default", pool_kernel_size=head_pool_kernel_size,
                                        dropout_rate=dropout_rate))
    return Net(blocks)


def slowfast_r50(num_classes: int = 400, **kw) -> Net:
    return create_slowfast(50, num_classes, **kw)


def slowfast_r101(num_classes: int = 400, fusion_kt: int = 5, **kw) -> Net:
    # The hub slowfast_r101 reportedly uses a (5,1,1) fusion kernel (SURVEY.md §2.3,
    # unverified offline); exposed as a parameter.
    return create_slowfast(101, num_classes, fusion_kt=fusion_kt, **kw)


def slow_r50(num_classes: int = 400, **kw) -> Net:
    return create_resnet(50, num_classes, **kw)


def count_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
