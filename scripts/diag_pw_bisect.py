"""Bisect a forward nondeterminism over the pointwise-kernel launches: for each PW-legal tuning index n,
build a fresh engine whose tuner may pick the pointwise kernel only there (forcing it), then compare two
forward passes' workspaces."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def main():
    from test_fused_gpu import _build, _inputs, DEV
    from pytorchvideo_accelerate_amd.models.fused import FusedNet
    from pytorchvideo_accelerate_amd.ops import tune as T
    model = _build(True)
    labels = torch.tensor([2, 5], device=DEV)
    n = 0
    while True:
        eng = FusedNet(model, DEV)
        eng.tuner.pw_only = n
        orig = eng.tuner._tune

        def forced(g, chunk, run, aff=0, epi=False, direct=True, tuner=eng.tuner):
            cands = tuner.candidates(g, chunk, aff, epi, direct)
            pw = [c for c in cands if c & T.PW]
            return pw[0] if pw else orig(g, chunk, run, aff, epi, direct)
        # candidates() counts PW-legal tunings; calling it twice per tuning would double count
        seen = [0]

        def forced2(g, chunk, run, aff=0, epi=False, direct=True, tuner=eng.tuner):
            before = tuner._pw_seen
            cands = tuner.candidates(g, chunk, aff, epi, direct)
            pw = [c for c in cands if c & T.PW]
            if pw:
                seen[0] = (tuple(g[:4]), tuner._pw_seen - 1)
                return pw[0]
            if tuner._pw_seen > before:
                tuner._pw_seen -= 1
            r = orig(g, chunk, run, aff, epi, direct)
            return r
        eng.tuner._tune = forced2
        acts = eng.prepare_inputs(_inputs(True, seed=3))
        eng.forward_backward(acts, labels)
        total = eng.tuner._pw_seen
        snaps = []
        for step in range(2):
            with torch.no_grad():
                eng._forward_backbone(acts, train=True)
            torch.cuda.synchronize()
            snaps.append({k: v.clone() for k, v in eng._ws.items()})
        diff = [k for k in snaps[0] if not torch.equal(snaps[0][k], snaps[1][k])]
        print("pw launch %d (%s) of %d: %d differing buffers %s" % (n, seen[0], total, len(diff), diff[:3]),
              flush=True)
        n += 1
        if n >= total:
            break


if __name__ == "__main__":
    main()
