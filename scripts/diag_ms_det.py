"""Determinism check of FusedNet.forward_backward: loss over repeated single- / two-stream steps on the same
inputs (used to chase a forward mismatch between the two schedules).  PVA_CONV_PW=0 excludes the pointwise
kernel from autotuning."""
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
    out = []
    for ms in (False, False, True, True, False):
        eng._ms_ok = ms
        loss, logits = eng.forward_backward(acts, labels, accumulate=False)
        torch.cuda.synchronize()
        out.append((ms, float(loss), float(logits.float().abs().sum())))
    for r in out:
        print("ms=%d loss %.6f |logits| %.6f" % r, flush=True)


if __name__ == "__main__":
    main()
