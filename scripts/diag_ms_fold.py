"""Loss spread of repeated single-stream vs two-stream steps (toy SlowFast-R50, S=64) with the conv_c BN fold
on every unit: separates fp32-atomic (Gram) ordering noise from a cross-stream race."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from test_fused_gpu import _build, _inputs  # noqa: E402
from pytorchvideo_accelerate_amd.models.fused import FusedNet  # noqa: E402

DEV = torch.device("cuda")
model = _build(True)
eng = FusedNet(model, DEV)
acts = eng.prepare_inputs(_inputs(True, seed=3))
labels = torch.tensor([2, 5], device=DEV)
eng.forward_backward(acts, labels)
for ms in (False, False, False, True, True, True):
    eng._ms_ok = ms
    loss, logits = eng.forward_backward(acts, labels, accumulate=False)
    torch.cuda.synchronize()
    print("two-stream" if ms else "one-stream", "%.7f" % float(loss), float(eng.flat.grad.norm()), flush=True)
