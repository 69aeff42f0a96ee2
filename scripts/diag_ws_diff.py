"""Find the first FusedNet workspace tensor (in creation order) whose contents differ between two identical
training steps (chasing nondeterminism; PVA_PW_KINDS narrows the pointwise launches)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def main():
    from test_fused_gpu import _build, _inputs, DEV
    from pytorchvideo_accelerate_amd.models.fused import FusedNet
    model = _build(True)
    eng = FusedNet(model, DEV)
    acts = eng.prepare_inputs(_inputs(True, seed=3))
    labels = torch.tensor([2, 5], device=DEV)
    eng.forward_backward(acts, labels)
    eng._ms_ok = False
    snaps = []
    fwd_only = os.environ.get("FWD_ONLY", "1") == "1"
    for step in range(3):
        if fwd_only:
            with torch.no_grad():
                eng._forward_backbone(acts, train=True)
        else:
            eng.forward_backward(acts, labels, accumulate=False)
        torch.cuda.synchronize()
        snaps.append({k: v.clone() for k, v in eng._ws.items()})
    keys = list(eng._ws.keys())
    for a, b in ((0, 1), (1, 2)):
        nd = 0
        for k in keys:
            x, y = snaps[a][k], snaps[b][k]
            if x.dtype.is_floating_point:
                same = torch.equal(torch.nan_to_num(x.float(), 7.0), torch.nan_to_num(y.float(), 7.0))
            else:
                same = torch.equal(x, y)
            if not same:
                d = (x.float() - y.float()).abs()
                bad = (d > 1e-3 * (x.float().abs() + 1e-3)).nonzero()
                print("step %d vs %d: %s shape %s differs: max %.3e, %d elems > tol, first %s" % (
                    a, b, k, tuple(x.shape), d.max().item(), bad.shape[0], bad[:4].tolist()), flush=True)
                nd += 1
                if nd >= 12:
                    break
        print("step %d vs %d: %d differing buffers" % (a, b, nd), flush=True)


if __name__ == "__main__":
    main()
