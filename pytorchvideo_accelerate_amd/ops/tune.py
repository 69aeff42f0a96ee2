"""First-use autotuning of implicit-GEMM conv launch configurations (cuDNN-benchmark-mode analogue).

The gfx950 conv kernel (csrc/kernels/conv_igemm.hip) has several launch configurations per conv: output
tile (128x128, 128x64, 256x32, 256x16), K depth per LDS stage (BK 32 / 64) and the uniform-tap loader
on or off; convs with <= 64 output channels can also run the direct-to-register kernel
(csrc/kernels/conv_direct.hip, 512 or 2048 rows per workgroup; arm ``conv_direct=0`` (``PVA_ARMS``, utils/arms.py) excludes it), and dense
1x1x1 convs the streaming pointwise kernel (csrc/kernels/conv_pw.hip; ``conv_pw=0`` excludes it).  Which one wins depends on the layer (measured: the uniform-tap loader is 20-25 % faster on
3x3 convs with the consumer-side BN fold and 15-30 % slower on padded temporal convs; BK=64 wins only for
deep K).  The first time a geometry is launched, :class:`ConvTuner` times every legal configuration on
scratch outputs (same shapes and strides, so inputs and real outputs are untouched — including
accumulating dgrads), caches the fastest and launches it for real.  Every configuration accumulates K in
the same order, so the result does not depend on the choice.

Disabled by the arm ``autotune=0`` and in deterministic mode (the built-in heuristic is used instead).

Tuned choices persist across processes (:class:`TuneStore`): a JSON table under ``~/.cache/pva/`` (or
``$PVA_TUNE_CACHE``; ``PVA_TUNE_CACHE=0`` disables it) whose file name hashes the extension's embedded build id, the planner sources, the
device name, the HIP version, the compute dtype and the kernel-selection knobs — a rebuilt ``.so`` or another GPU
gets a fresh table.  Under data parallelism rank 0 reads it and broadcasts it (one collective), and only rank 0
writes it back.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

EXPLICIT = 16          # cfg bit: explicit configuration (else the kernel's heuristic)
BK64 = 4
UT = 8
DIRECT = 32           # narrow direct-to-register kernel (csrc/kernels/conv_direct.hip)
DIRECT_2K = 64        #   with 2048 rows per workgroup (else 512)
DMA = 128             # uniform-tap loader staged by LDS-DMA (buffer_load ... lds); launches without input affine
DIRECT_HALF = 1024    #   (with DIRECT) half the row groups in flight per wave: fewer VGPRs, more waves per SIMD
BIG = 256             # 256x256 tile of 8 waves (N >= 256; the backward-BN epilogue in 64-row slices);
BIG_HALF = 1          #   with bit 0: the 256x128 tile of 4 waves (N >= 128; two independent workgroups per CU)
BIG_PF = 4096         #   with BK64 + DMA: L2 touch-prefetch of the A rows one k-tile ahead (tools/gemm_lab.hip:
                      #   +14-20 % on the res4/res5 GEMM shapes)
PW = 512              # streaming pointwise kernel (csrc/kernels/conv_pw.hip): dense 1x1x1 GEMMs, K <= 256,
PW_ROWS = (1024, 2048, 4096)   # N % 32 == 0, weights in LDS; bits 0-1 select the rows per workgroup,
PW_SOLO = 4                     # bit 2 one workgroup per CU
PW_W4 = 8                       # bit 3 4-wave workgroups (three per CU at <= 168 VGPRs)
HALO = 2048           # halo-staged (1,3,3) stride-1 kernel (csrc/kernels/conv_halo.hip): bit 0 = 64-channel
                      # n-tiles (else 128), bits 12+ = positions per tile; bit 1 = persistent 64-channel variant
HALO_P = 2            #   (weights resident in LDS; bit 2: 4 workgroups per CU-slot instead of 1;
HALO_P4 = 4           #   bit 3: the double-buffered 8x28-tile variant, halo writes behind the MFMAs)
HALO_D = 8
TILE_BN = (128, 64, 32, 16)   # variants 0..3
TILE_BM = (128, 128, 256, 256)


def describe(cfg: int) -> str:
    """Human-readable configuration word (``PVA_TUNE_LOG=1`` prints every candidate's time)."""
    if cfg < 0 or not cfg & EXPLICIT:
        return "heuristic"
    if cfg & HALO:
        if cfg & HALO_P:
            return "halo%d/%s%d" % (cfg >> 12, "d" if cfg & HALO_D else "p", 1024 if cfg & HALO_P4 else 256)
        return "halo%d/n%d" % (cfg >> 12, 64 if cfg & 1 else 128)
    if cfg & PW:
        return "pw%d%s%s" % (PW_ROWS[cfg & 3], "s" if cfg & PW_SOLO else "", "/w4" if cfg & PW_W4 else "")
    if cfg & DIRECT:
        return "direct%d%s" % (2048 if cfg & DIRECT_2K else 512, "/rt2" if cfg & DIRECT_HALF else "")
    if cfg & BIG:
        return "256x%d/bk%d%s%s%s" % (128 if cfg & BIG_HALF else 256, 64 if cfg & BK64 else 32,
                                      "/ut" if cfg & UT else "", "/dma" if cfg & DMA else "",
                                      "/pf" if cfg & BIG_PF else "")
    return "%dx%d/bk%d%s%s" % (TILE_BM[cfg & 3], TILE_BN[cfg & 3], 64 if cfg & BK64 else 32, "/ut" if cfg & UT else "",
                               "/dma" if cfg & DMA else "")


def cfg_word(variant: int, bk: int, ut: bool) -> int:
    return EXPLICIT | variant | (BK64 if bk == 64 else 0) | (UT if ut else 0)


class ConvTuner:
    def __init__(self, C, enabled: bool = True, reps: int = 3):
        self.C = C
        from ..utils.arms import arm, on
        # candidate families: PVA_ARMS (utils/arms.py) selects the arms of the finished A/Bs
        self.enabled = enabled and on("autotune")
        self.direct = on("conv_direct")
        self.dma = on("conv_dma")
        self.pw = on("conv_pw")
        self.halo = on("conv_halo")
        self.halo_d = on("conv_halo_d")
        self.big_half = on("conv_big_half")
        self.pf = on("conv_pf")
        self.pw_w4 = on("conv_pw_w4")
        # debugging aid: pw_kinds=f:fres:er restricts the pointwise kernel to launches whose key starts with one of
        # these kinds (models/fused.py: f fres fw2 eb er d)
        kinds = arm("pw_kinds")
        self.pw_kinds = None if kinds is None else set(k for k in kinds.split(":") if k)
        self._pw_now = True
        self.pw_only: Optional[int] = None   # debugging aid: allow the pointwise kernel on the n-th PW-legal tuning only
        self._pw_seen = 0
        self.log = os.environ.get("PVA_TUNE_LOG", "0") != "0"
        self.reps = int(arm("tune_reps"))   # timed launches per re-timed contender
        self.top = max(1, int(arm("tune_top")))   # contenders re-timed after the single-shot pass
        self.tuned = 0          # geometries timed by this process (conv + weight-gradient tunings)
        self.cache: Dict[Tuple, int] = {}
        self._scratch: Dict[Tuple, torch.Tensor] = {}
        # borrowed choices (tests/test_benchcfg_gpu.py): {"conv": table, "wgrad": table, "ratio": M_src / M_dst} —
        # a geometry missing here takes the source table's choice for the same geometry at ``ratio`` times the rows
        # (another batch size), when that choice is a legal candidate here; borrow_stats counts (hits, misses)
        self.borrow: Optional[Dict] = None
        self.borrow_stats = [0, 0]
        # multi-rank consensus: ``agree(times) -> times`` (e.g. ``DistState.agree_times``, the per-candidate
        # max over ranks) so that every data-parallel rank picks the same configuration
        self.agree: Optional[Callable[[List[float]], List[float]]] = None

    # ---------------------------------------------------------------- candidates
    def candidates(self, g: Sequence[int], chunk: int, aff: int = 0, epi: bool = False,
                   direct: bool = True, pw: bool = True, halo: bool = True) -> List[int]:
        N, Cg = g[1], g[3]
        K = g[28] * g[29] * g[30] * Cg
        out = []
        for v, bn in enumerate(TILE_BN):
            if bn > 16 and bn >= 2 * N:      # tile much wider than the output channels
                continue
            if bn * 8 < N:                   # tile far narrower than N: many redundant A re-reads
                continue
            for bk in (32, 64):
                if bk == 64 and (chunk != 8 or K < 64):
                    continue
                uts = [False]
                if chunk == 8 and self.C.conv_ut_legal(list(g), chunk, bk):
                    uts.append(True)
                for ut in uts:
                    out.append(cfg_word(v, bk, ut))
                    if ut and aff == 0 and self.dma:
                        out.append(cfg_word(v, bk, ut) | DMA)
        if N >= 128 and chunk == 8:   # 256x256 / 256x128 tiles (UT loader only: the generic one is VALU-bound)
            halves = (0, BIG_HALF) if self.big_half else (0,)
            for half in (h for h in halves if N >= (128 if h else 256)):
                for bk in (32, 64):
                    if self.C.conv_ut_legal(list(g), chunk, bk):
                        w = EXPLICIT | BIG | half | UT | (BK64 if bk == 64 else 0)
                        out.append(w)
                        if aff == 0 and self.dma:
                            out.append(w | DMA)
                            if bk == 64 and self.pf:
                                out.append(w | DMA | BIG_PF)
        if direct and self.direct and self.C.conv_direct_legal(list(g), chunk):
            out += [EXPLICIT | DIRECT | r | h for r in (0, DIRECT_2K) for h in (0, DIRECT_HALF)]
        if halo and self.halo and (aff == 0 or not epi):
            P = int(self.C.conv_halo_legal(list(g), chunk))
            if P > 0:
                out += [EXPLICIT | HALO | (P << 12) | v for v in ((0, 1) if N % 128 == 0 else (1,))]
                lg = int(self.C.conv_halo64p_legal(list(g), chunk))
                if lg:
                    out += [EXPLICIT | HALO | (P << 12) | 1 | HALO_P | g4 for g4 in (0, HALO_P4)]
                if lg == 2 and self.halo_d:
                    out += [EXPLICIT | HALO | (P << 12) | 1 | HALO_P | HALO_D | g4 for g4 in (0, HALO_P4)]
        if pw and self.pw and self._pw_now and self.C.conv_pw_legal(list(g), chunk):
            self._pw_seen += 1
            if self.pw_only is None or self.pw_only == self._pw_seen - 1:
                out += [EXPLICIT | PW | s | v for s in (0, PW_SOLO) for v in range(len(PW_ROWS))]
                if self.pw_w4:
                    out += [EXPLICIT | PW | PW_W4 | v for v in range(len(PW_ROWS))]
        return out

    def bm(self, cfg: int, N: int) -> int:
        return int(self.C.conv_cfg_bm(cfg, N))

    def scratch_like(self, t: torch.Tensor) -> torch.Tensor:
        key = (tuple(t.shape), tuple(t.stride()), t.dtype, t.device)
        s = self._scratch.get(key)
        if s is None:
            s = torch.empty_strided(t.shape, t.stride(), dtype=t.dtype, device=t.device)
            if s.dtype.is_floating_point:
                s.zero_()
            self._scratch[key] = s
        return s

    # ---------------------------------------------------------------- launch
    def launch(self, key: Tuple, g: Sequence[int], chunk: int, run: Callable[[int, bool], None],
               aff: int = 0, epi: bool = False, direct: bool = True, pw: bool = True, halo: bool = True) -> int:
        """``run(cfg, scratch)`` performs the launch (into scratch outputs when ``scratch``).  Returns the
        configuration used for the real launch (-1 = kernel heuristic).  ``direct=False`` / ``pw=False``: the
        launch needs an epilogue the direct / pointwise kernel lacks (fused residual output, bias, statistics
        without the output); ``halo=False``: an accumulating launch (the halo kernel only stores)."""
        cfg = self.cache.get(key)
        if cfg is None and self.borrow is not None:
            b = self.borrow_lookup("conv", key, len(key) - len(g))
            if b is not None and (b == -1 or b in self.candidates(g, chunk, aff, epi, direct, pw, halo)):
                cfg = self.cache[key] = b
        if cfg is None:
            self._pw_now = self.pw_kinds is None or (len(key) > 0 and key[0] in self.pw_kinds)
            cfg = self._tune(g, chunk, run, aff, epi, direct, pw, halo) if self.enabled else -1
            self._pw_now = True
            self.cache[key] = cfg
        run(cfg, False)
        return cfg

    def borrow_lookup(self, table: str, key: Tuple, m_index: int) -> Optional[int]:
        """The borrowed table's choice for ``key`` with its row count (``key[m_index]``) scaled by the ratio, or None;
        counts a hit or a miss."""
        if self.borrow is None:
            return None
        r = self.borrow["ratio"]
        m = key[m_index] * r
        src = None
        if abs(m - round(m)) < 1e-6:
            src = self.borrow[table].get(key[:m_index] + (int(round(m)),) + key[m_index + 1:])
        self.borrow_stats[0 if src is not None else 1] += 1
        return src

    def time_candidates(self, cands: Sequence[int], trial: Callable[[int], None]) -> List[float]:
        """Per-candidate time (ms per launch), two-phase: every candidate once (after a warm-up launch), then the
        ``top`` fastest again ``reps`` times — the cold-start cost of a geometry drops from (1 + reps) to ~2 launches
        per candidate while the choice among close contenders keeps its ``reps``-launch average.  Untimed-again
        candidates keep their single-launch time (never below a re-timed contender's by construction of the top-k).
        With ``agree`` set (data parallelism) both phases use the per-candidate max over ranks, so every rank
        re-times the same contenders and picks the same winner."""
        def timed(c, n):
            trial(c)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                trial(c)
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) / n
        times = [timed(c, 1) for c in cands]
        if self.agree is not None:
            times = self.agree(times)
        if self.reps > 1 and len(cands) > 1:
            order = sorted(range(len(cands)), key=times.__getitem__)[:self.top]
            again = [timed(cands[i], self.reps) for i in order]
            if self.agree is not None:
                again = self.agree(again)
            for i, t in zip(order, again):
                times[i] = t
            # a contender that re-timed slower than a single-shot outsider keeps its rank among the contenders only
            worst = max(again)
            for i in range(len(cands)):
                if i not in order:
                    times[i] = max(times[i], worst + 1e-6)
        return times

    def _tune(self, g: Sequence[int], chunk: int, run: Callable[[int, bool], None], aff: int = 0,
              epi: bool = False, direct: bool = True, pw: bool = True, halo: bool = True) -> int:
        cands = self.candidates(g, chunk, aff, epi, direct, pw, halo)
        if len(cands) <= 1:
            return cands[0] if cands else -1
        self.tuned += 1
        times = list(zip(cands, self.time_candidates(cands, lambda c: run(c, True))))
        best, best_t = min(times, key=lambda ct: ct[1])
        if self.log:
            print("tune M=%d N=%d K=%d taps=%s: " % (g[0], g[1], g[2], tuple(g[28:31]))
                  + " ".join("%s=%.1fus" % (describe(c), 1e3 * t) for c, t in times)
                  + " -> " + describe(best), file=sys.stderr, flush=True)
        return best


def _tuplify(v):
    return tuple(_tuplify(x) for x in v) if isinstance(v, list) else v


class TuneStore:
    """Persistent autotuner table (module docstring).  ``tables``: name -> dict (the live caches, updated in place
    by :meth:`load` / :meth:`restore`); :meth:`save` writes them when they grew since the last save."""

    def __init__(self, tables: Dict[str, Dict], ident: Dict[str, str], root: Optional[str] = None):
        self.tables = tables
        env = os.environ.get("PVA_TUNE_CACHE", "")
        self.enabled = env != "0"
        root = root or env or os.path.join(os.path.expanduser("~"), ".cache", "pva")
        ident = dict(ident)
        from ..utils.arms import selected   # the selected A/B arms (PVA_ARMS) change kernel selection
        ident["arms"] = ",".join(f"{k}={v}" for k, v in sorted(selected().items()))
        self.ident = ident
        h = hashlib.sha1(json.dumps(ident, sort_keys=True).encode()).hexdigest()[:16]
        self.path = os.path.join(root, f"tune-{h}.json")
        self.writer = True
        self._saved = -1

    @staticmethod
    def build_ident(device, dtype: str) -> Dict[str, str]:
        from .. import _build
        import torch as _t
        so = _build.embedded_id(_build.ext_path()) or ""
        # the Python side interprets cached cfg words (split heuristics, legality filters): a change there must
        # invalidate the table too, not only a rebuilt binary
        h = hashlib.sha1()
        pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        for rel in ("ops/tune.py", "ops/conv.py", "models/fused.py"):
            try:
                with open(os.path.join(pkg, rel), "rb") as f:
                    h.update(f.read())
            except OSError:
                pass
        name = _t.cuda.get_device_name(device) if _t.device(device).type == "cuda" else "cpu"
        return {"so": so, "py": h.hexdigest()[:16], "device": name, "hip": str(_t.version.hip), "dtype": dtype}

    def _count(self) -> int:
        return sum(len(t) for t in self.tables.values())

    def read(self) -> Optional[Dict]:
        """The stored table (JSON-ready dict) or None (absent / unreadable / other identity)."""
        if not self.enabled or not os.path.exists(self.path):
            return None
        try:
            with open(self.path) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            return None
        return doc if doc.get("ident") == self.ident else None

    def restore(self, doc: Optional[Dict]) -> int:
        """Merge a stored table into the live caches; returns the number of entries restored."""
        n = 0
        if doc:
            for name, rows in doc.get("tables", {}).items():
                t = self.tables.get(name)
                if t is None:
                    continue
                for k, v in rows:
                    t.setdefault(_tuplify(k), v)
                    n += 1
        self._saved = self._count()
        return n

    def load(self) -> int:
        return self.restore(self.read())

    def save(self, force: bool = False) -> bool:
        n = self._count()
        if not self.enabled or not self.writer or (n == self._saved and not force):
            return False
        doc = {"ident": self.ident, "tables": {k: [[list(kk) if isinstance(kk, tuple) else kk, v]
                                                   for kk, v in t.items()] for k, t in self.tables.items()}}
        try:
            os.makedirs(os.path.dirname(self.path), exist_ok=True)
            tmp = "%s.%d.tmp" % (self.path, os.getpid())
            with open(tmp, "w") as f:
                json.dump(doc, f)
            os.replace(tmp, self.path)
        except OSError:
            return False
        self._saved = n
        return True
