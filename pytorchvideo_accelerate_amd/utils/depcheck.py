"""Cross-stream dependency checker for the multi-stream executors (SURVEY.md §5 "Race detection").

``FusedNet`` issues its kernels on up to five HIP streams (main / fast-pathway lanes, their weight-gradient streams,
the gradient all-reduce's comm stream) and orders them only with events.  A missing ``wait_event`` is a data race
that a single-GPU test rarely sees: the result changes only when the two streams actually overlap.  This checker
finds it deterministically, from the launch order alone:

* every kernel launch through the extension (a proxy in place of ``FusedNet.C``) is recorded with its stream, a
  per-stream launch counter, and the byte ranges of its tensor arguments, split into reads and writes (``WRITES``:
  the output arguments of each binding; a written argument counts as read-modify-write);
* every ``Event.record`` snapshots the recording stream's vector clock; ``Stream.wait_event`` merges it into the
  waiting stream's clock (``wait_stream`` and ``torch.cuda.synchronize`` are covered through them);
* a launch on stream S that touches a range last written by stream W != S at launch count c (read-after-write or
  write-after-write), or writes a range last read by R != S at count c (write-after-read), needs S's clock to have
  reached c for W (or R) — otherwise it is reported as a ``Hazard`` naming both launches.

Same-stream order is implicit.  Host-side allocation reuse across streams is not modelled (the executors keep their
buffers), and ATen ops are not seen (the executors run none between their kernels on the hot path).
"""
from __future__ import annotations

import contextlib
import re
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

# output (written) arguments of every binding the executors launch
WRITES: Dict[str, Tuple[str, ...]] = {
    "conv_igemm": ("y", "stats"),
    "conv_igemm_epi": ("y", "part"),
    "conv_igemm_fres": ("y", "mask"),
    "conv_wgrad": ("partial", "colsum"),
    "wgrad_reduce": ("partial", "grad"),
    "wgrad_box_reduce": ("tmp", "grad"),
    "bn_finalize": ("rm", "rv", "nbt", "smean", "srstd", "scale", "shift", "fin"),
    "bn_eval_affine": ("scale", "shift"),
    "bn_act": ("out",),
    "res_out": ("out", "mask"),
    "bn_bwd_reduce": ("part", "dzout"),
    "bn_bwd_finalize": ("dgamma", "dbeta", "coef", "fin"),
    "bn_bwd_apply": ("dy0", "dy1", "dzout"),
    "stem_pool_fwd": ("out", "arg", "ymax"),
    "stem_pool_bn_apply": ("dy",),
    "stem_pool_bwd": ("dact",),
    "avgpool_fwd": ("out",),
    "avgpool_bwd": ("dx",),
    "pack_weights": ("fwd", "dgr"),
    "stem_fwd": ("y", "stats"),
    "stem_wgrad": ("acc", "slab"),
    "stem_wgrad_convert": ("acc", "grad"),
    "stem_pack": ("out",),
    "bnfold_fwd_stats": ("T", "s_out", "rm", "rv", "nbt", "smean", "srstd", "scale", "shift"),
    "bnfold_bwd": ("dgamma", "dbeta", "dW", "coef", "W1t", "W2", "bias"),
    "head_forward": ("xm", "logits"),
    "head_seed_advance": ("seed_dev",),
    "head_ce": ("dlogits", "loss", "counts", "row_loss", "row_correct"),
    "head_backward": ("dW", "db", "dfeat", "scratch"),
    "head_dropout_mask": ("out",),
    "lateral_bwd": ("dy", "dx"),
    "narrow_c_bwd": ("dz", "dab", "slab", "part", "cpart"),
    "nonfinite_check": ("flag",),
    "sgd_momentum": ("p", "buf", "found_inf"),
    "video_preprocess": ("out", "slow_out"),
}

# argument names of the bindings declared without py::arg names (csrc/runtime/bindings.cpp signatures)
ARGNAMES: Dict[str, Tuple[str, ...]] = {
    "avgpool_bwd": ("dout", "ldo", "coff", "dims", "k", "dx"),
    "avgpool_fwd": ("x", "dims", "k", "out", "ldo", "coff"),
    "bn_act": ("y", "ldy", "out", "ldo", "scale", "shift", "relu", "M", "C"),
    "bn_bwd_apply": ("g", "ldg", "mask_mode", "mo", "ldm", "ms", "mh", "y0", "coef0", "dy0", "y1", "coef1", "dy1",
                     "dzout", "lddz", "dz_accum", "M", "C"),
    "bn_eval_affine": ("gamma", "beta", "rm", "rv", "eps", "scale", "shift"),
    "bnfold_bwd": ("part", "tiles", "Wf", "Wd", "G", "T", "s", "C", "c", "count", "gamma", "mean", "rstd", "dgamma",
                   "dbeta", "dW", "beta_acc", "coef", "W1t", "W2", "bias"),
    "bnfold_fwd_stats": ("Wf", "Ga", "sslab", "splits", "C", "c", "count", "T", "s_out", "gamma", "beta", "rm", "rv",
                         "nbt", "momentum", "eps", "smean", "srstd", "scale", "shift"),
    "conv_igemm_fres": ("x", "w", "y", "scale", "shift", "affine", "g", "chunk", "cfg", "osc", "osh", "res", "ldr",
                        "rsc", "rsh", "mask"),
    "head_ce": ("logits", "labels", "gscale", "dlogits", "loss", "counts", "acc_counts", "row_loss", "row_correct"),
    "head_dropout_mask": ("out", "p_drop", "seed"),
    "head_seed_advance": ("seed_dev",),
    "lateral_bwd": ("g", "ldg", "y", "sc", "sh", "coef", "wd", "dy", "dx", "ldx", "N", "To", "Tf", "HW", "CO", "Cf",
                    "alpha"),
    "nonfinite_check": ("g", "gscale", "flag"),
    "pack_weights": ("master", "fwd", "dgr", "descs", "ntensors"),
    "res_out": ("yc", "sc", "hc", "y1", "s1", "h1", "x", "ldx", "out", "ldo", "M", "C", "mask"),
    "stem_fwd": ("x", "wpack", "y", "stats", "dims", "Cout", "kt"),
    "stem_pack": ("w", "out", "Cout", "kt"),
    "stem_pool_bn_apply": ("dout", "ldd", "arg", "y", "ms", "mh", "coef", "dy", "NT", "H", "W", "Ho", "Wo", "C"),
    "stem_pool_bwd": ("dout", "ldd", "arg", "dact", "NT", "H", "W", "Ho", "Wo", "C"),
    "stem_wgrad_convert": ("acc", "grad", "Cout", "kt", "beta"),
    "wgrad_box_reduce": ("slab", "tmp", "grad", "splits", "Cout", "taps", "Cin", "Cin_real", "scale", "beta"),
}


@dataclass
class Hazard:
    kind: str            # "RAW" / "WAW" / "WAR"
    fn: str              # the launch that lacks the wait
    arg: str
    stream: int
    count: int
    other_fn: str        # the earlier launch on the other stream
    other_stream: int
    other_count: int

    def __str__(self):
        return (f"{self.kind}: {self.fn}({self.arg}) on stream {self.stream:#x} #{self.count} vs {self.other_fn} on "
                f"stream {self.other_stream:#x} #{self.other_count} without a wait")


def _arg_names(fn, name: str) -> Optional[Tuple[str, ...]]:
    if name in ARGNAMES:
        return ARGNAMES[name]
    doc = (getattr(fn, "__doc__", "") or "").split("\n")[0]
    if "(" not in doc:
        return None
    inner = doc[doc.index("(") + 1:doc.rindex(")")]
    names = tuple(re.findall(r"(?:^|,\s*)(\w+):", inner))
    return None if any(n.startswith("arg") and n[3:].isdigit() for n in names) else names


def _span(t: torch.Tensor) -> Tuple[int, int, int]:
    """(storage base, byte lo, byte hi) of the memory a tensor view can touch."""
    base = t.untyped_storage().data_ptr()
    lo = t.data_ptr()
    if t.numel() == 0:
        return base, lo, lo
    ext = 1 + sum((s - 1) * st for s, st in zip(t.shape, t.stride()) if s > 0)
    return base, lo, lo + ext * t.element_size()


class DepChecker:
    def __init__(self, raise_on_hazard: bool = False):
        self.raise_on_hazard = raise_on_hazard
        self.count: Dict[int, int] = {}                 # launches issued per stream
        self.clock: Dict[int, Dict[int, int]] = {}      # stream -> {other stream: launches it has waited for}
        self.events: Dict[int, Dict[int, int]] = {}     # id(event) -> clock snapshot at record time
        # storage base -> {(lo, hi, kind, stream): (count, fn)}
        self.acc: Dict[int, Dict[Tuple[int, int, str, int], Tuple[int, str]]] = {}
        self.hazards: List[Hazard] = []
        self.launches = 0
        self._names: Dict[str, Optional[Tuple[str, ...]]] = {}

    # ---------------------------------------------------------------- clocks
    @staticmethod
    def _sid(stream=None) -> int:
        s = stream if stream is not None else torch.cuda.current_stream()
        return int(s.cuda_stream)

    def on_record(self, event, stream=None):
        s = self._sid(stream)
        snap = dict(self.clock.get(s, {}))
        snap[s] = self.count.get(s, 0)
        self.events[id(event)] = snap

    def on_wait(self, stream, event):
        snap = self.events.get(id(event))
        if snap is None:
            return
        c = self.clock.setdefault(self._sid(stream), {})
        for k, v in snap.items():
            if c.get(k, 0) < v:
                c[k] = v

    def on_sync(self):
        everything = dict(self.count)
        for s in set(self.count) | set(self.clock):
            c = self.clock.setdefault(s, {})
            for k, v in everything.items():
                if c.get(k, 0) < v:
                    c[k] = v

    # ---------------------------------------------------------------- launches
    def on_launch(self, name: str, fn, args, kwargs):
        names = self._names.get(name, False)
        if names is False:
            names = self._names[name] = _arg_names(fn, name)
        writes = set(WRITES.get(name, ()))
        tensors = []
        for i, a in enumerate(args):
            if isinstance(a, torch.Tensor) and a.is_cuda:
                nm = names[i] if names is not None and i < len(names) else f"arg{i}"
                tensors.append((nm, a))
        for k, a in kwargs.items():
            if isinstance(a, torch.Tensor) and a.is_cuda:
                tensors.append((k, a))
        s = self._sid()
        cnt = self.count.get(s, 0) + 1
        self.count[s] = cnt
        self.launches += 1
        seen = self.clock.setdefault(s, {})
        for nm, t in tensors:
            w = nm in writes or (names is None and name not in WRITES)   # unknown binding: assume written
            base, lo, hi = _span(t)
            if hi <= lo:
                continue
            recs = self.acc.setdefault(base, {})
            for (rlo, rhi, kind, rs), (rc, rfn) in recs.items():
                if rs == s or rhi <= lo or rlo >= hi:
                    continue
                if kind == "w" or w:
                    if seen.get(rs, 0) < rc:
                        hz = Hazard(("WAW" if w else "RAW") if kind == "w" else "WAR", name, nm, s, cnt, rfn, rs, rc)
                        self.hazards.append(hz)
                        if self.raise_on_hazard:
                            raise RuntimeError(str(hz))
            key_r = (lo, hi, "r", s)
            recs[key_r] = (cnt, name)
            if w:
                recs[(lo, hi, "w", s)] = (cnt, name)

    # ---------------------------------------------------------------- installation
    @contextlib.contextmanager
    def watching(self):
        """Route torch's event record / wait / device synchronize through the clocks while active."""
        ev_record = torch.cuda.Event.record
        st_wait = torch.cuda.Stream.wait_event
        dev_sync = torch.cuda.synchronize
        ev_sync = torch.cuda.Event.synchronize
        chk = self

        def record(ev, stream=None):
            chk.on_record(ev, stream)
            return ev_record(ev, stream) if stream is not None else ev_record(ev)

        def wait_event(st, ev):
            chk.on_wait(st, ev)
            return st_wait(st, ev)

        def synchronize(device=None):
            chk.on_sync()
            return dev_sync(device)

        def ev_synchronize(ev):
            chk.on_sync()
            return ev_sync(ev)

        torch.cuda.Event.record = record
        torch.cuda.Stream.wait_event = wait_event
        torch.cuda.synchronize = synchronize
        torch.cuda.Event.synchronize = ev_synchronize
        try:
            yield self
        finally:
            torch.cuda.Event.record = ev_record
            torch.cuda.Stream.wait_event = st_wait
            torch.cuda.synchronize = dev_sync
            torch.cuda.Event.synchronize = ev_sync


class CheckedExtension:
    """Stand-in for the ``_C`` module: every kernel launch is reported to the checker, then runs."""

    def __init__(self, C, checker: DepChecker):
        self._C = C
        self._chk = checker

    def __getattr__(self, name):
        fn = getattr(self._C, name)
        if not callable(fn) or name not in WRITES and name not in ARGNAMES and not name.startswith(
                ("conv_", "bn_", "wgrad_", "stem_", "head_", "narrow_", "lateral_", "avgpool_", "res_", "pack_")):
            return fn
        if name.endswith(("_legal", "_tile", "_tiles", "_blocks", "_groups", "_rps", "_doubles", "_size",
                          "_supported")) or name in ("conv_cfg_bm", "conv_m_tiles", "conv_set_bk", "conv_set_ut",
                                                     "wgrad_tile", "bn_bwd_blocks"):
            return fn
        chk = self._chk

        def launch(*args, **kwargs):
            chk.on_launch(name, fn, args, kwargs)
            return fn(*args, **kwargs)
        return launch


def install(net, raise_on_hazard: bool = False) -> DepChecker:
    """Wrap ``net.C`` (FusedNet) and the process-wide extension handle (``ops._ext.require()``, used by the conv
    helpers) with a checker; use ``with chk.watching(): ...`` around the steps to check, ``uninstall`` after."""
    from ..ops import _ext
    chk = DepChecker(raise_on_hazard)
    real = _ext.require()
    proxy = CheckedExtension(real, chk)
    chk._restore = (net, net.C, real)
    net.C = proxy
    _ext._C = proxy
    return chk


def uninstall(chk: DepChecker):
    from ..ops import _ext
    net, c, real = chk._restore
    net.C = c
    _ext._C = real
