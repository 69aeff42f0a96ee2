"""Join a layer_profile.py dump with conv shapes: achieved TFLOP/s and an HBM lower bound per op.

    python scripts/layer_roofline.py gpurun_out/layers.txt [--batch 32]"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchvideo_accelerate_amd.models import reference as R  # noqa: E402


def conv_shapes(batch, T=32, S=224, alpha=4, depth=50):
    net = R.create_slowfast(depth, 400, head_pool_kernel_sizes=((T // alpha, S // 32, S // 32), (T, S // 32, S // 32)))
    shapes = {}
    hooks = []

    def reg(name, conv):
        def h(m, inp, out):
            x = inp[0]
            shapes[name] = dict(cin=m.in_channels, cout=m.out_channels, k=tuple(m.kernel_size),
                                Mi=batch * x.shape[2] * x.shape[3] * x.shape[4],
                                Mo=batch * out.shape[2] * out.shape[3] * out.shape[4])
        hooks.append(conv.register_forward_hook(h))

    for i, b in enumerate(net.blocks):
        if not isinstance(b, R.MultiPathWayWithFuse):
            continue
        for p, m in enumerate(b.multipathway_blocks):
            if isinstance(m, R.ResNetBasicStem):
                reg(f"b{i}.p{p}.conv", m.conv)
            else:
                for j, rb in enumerate(m.res_blocks):
                    reg(f"b{i}.p{p}.{j}.a", rb.branch2.conv_a)
                    reg(f"b{i}.p{p}.{j}.b", rb.branch2.conv_b)
                    reg(f"b{i}.p{p}.{j}.c", rb.branch2.conv_c)
                    if rb.branch1_conv is not None:
                        reg(f"b{i}.p{p}.{j}.1", rb.branch1_conv)
        if b.multipathway_fusion is not None:
            reg(f"b{i}.fuse", b.multipathway_fusion.conv_fast_to_slow)
    x = torch.randn(1, 3, T, S, S)
    idx = torch.linspace(0, T - 1, T // alpha).long()
    with torch.no_grad():
        net.eval()
        net([x[:, :, idx], x])
    return shapes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--crop", type=int, default=224)
    ap.add_argument("--depth", type=int, default=50)
    a = ap.parse_args()
    sh = conv_shapes(a.batch, a.frames, a.crop, 4, a.depth)
    rows = [l.split() for l in open(a.dump) if l.strip().endswith(" us")]
    print(f"{'op':26s} {'us':>8s} {'TF/s':>7s} {'GB min':>7s} {'TB/s':>6s}")
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0.0])
    for lab, us, _ in rows:
        if "." not in lab:
            continue
        unit, kind = lab.rsplit(".", 1)
        s = sh.get(unit)
        if s is None or kind not in ("fwd", "dgrad", "wgrad"):
            continue
        taps = s["k"][0] * s["k"][1] * s["k"][2]
        flops = 2.0 * s["Mo"] * s["cout"] * s["cin"] * taps
        x_b, y_b = s["Mi"] * s["cin"] * 2, s["Mo"] * s["cout"] * 2
        gb = {"fwd": x_b + y_b, "dgrad": x_b + y_b, "wgrad": x_b + y_b}[kind] / 1e9
        t = float(us) * 1e-6
        print(f"{lab:26s} {float(us):8.1f} {flops / t / 1e12:7.1f} {gb:7.3f} {gb / t / 1e3:6.2f}")
        path = unit.split(".")[1]
        agg[(path, kind)][0] += t
        agg[(path, kind)][1] += flops
        agg[(path, kind)][2] += gb
    print("\n# totals")
    for k, (t, f, g) in sorted(agg.items()):
        print(f"{k[0]:5s} {k[1]:6s} {t * 1e3:7.2f} ms  {f / t / 1e12:6.1f} TF/s  {g / t / 1e3:5.2f} TB/s(min)  "
              f"floor {max(f / 2.0e15, g / 5.0e3 / 1e-3 * 1e-3) * 1e3:6.2f} ms")


if __name__ == "__main__":
    main()
