"""Steady-state per-kernel summary from a rocprofv3 ``--kernel-trace`` CSV.

The first steps of a run include first-use autotuning (ops/tune.py) and warm-up, which pollute
``--stats``.  This keeps only the kernels of the last ``--steps`` training steps, using the fused SGD
kernel (one launch per optimizer step) as the step delimiter, and prints per-kernel and per-family GPU
time per step plus the wall span of those steps.

    python scripts/steady_state_kernels.py gpurun_out/prof/x_kernel_trace.csv --steps 2 > profiles/.../kernels.txt
"""
import argparse
import collections
import csv
import re


def family(name: str) -> str:
    m = re.search(r"(\w+_kernel)", name)
    base = m.group(1) if m else name[:40]
    t = re.search(r"<([^>]*)>", name)
    return base, (base + ("<" + t.group(1) + ">" if t else ""))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--delim", default="sgd_momentum_kernel")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if a.delim in r["Kernel_Name"]]
    assert len(ends) > a.steps, f"need > {a.steps} optimizer steps in the trace, found {len(ends)}"
    lo, hi = ends[-a.steps - 1] + 1, ends[-1] + 1
    sel = rows[lo:hi]
    span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e6 / a.steps
    per = collections.defaultdict(lambda: [0.0, 0])
    fam = collections.defaultdict(float)
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        f, full = family(r["Kernel_Name"])
        per[full][0] += d
        per[full][1] += 1
        fam[f] += d
    busy = sum(v[0] for v in per.values()) / a.steps
    print(f"# steady state over the last {a.steps} optimizer steps: wall span {span:.2f} ms/step, "
          f"kernel busy {busy:.2f} ms/step ({100 * busy / span:.1f}% of span), {len(sel) // a.steps} launches/step")
    print("\n# per kernel family (ms/step)")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"{v / a.steps:9.3f}  {100 * v / a.steps / busy:5.1f}%  {k}")
    print(f"\n# top {a.top} kernel instantiations (ms/step, launches/step)")
    for k, (t, n) in sorted(per.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"{t / a.steps:9.3f}  {n // a.steps:4d}  {k[:120]}")
    timeline(sel, a.steps)


def timeline(sel, steps):
    """Union of the kernel intervals: GPU-idle time (no kernel running) and time at each concurrency level."""
    ev = []
    for r in sel:
        ev.append((int(r["Start_Timestamp"]), 1))
        ev.append((int(r["End_Timestamp"]), -1))
    ev.sort()
    level, last = 0, ev[0][0]
    at = collections.defaultdict(int)
    gaps = []
    for t, d in ev:
        if t > last:
            at[level] += t - last
            if level == 0:
                gaps.append(t - last)
        level += d
        last = t
    tot = sum(at.values())
    print(f"\n# timeline (ms/step): span {tot / 1e6 / steps:.2f}, idle (no kernel) {at[0] / 1e6 / steps:.2f} "
          f"in {len(gaps) // steps} gaps/step (gaps > 20 us: {sum(g for g in gaps if g > 20000) / 1e6 / steps:.2f} ms)")
    for lv in sorted(at):
        if lv:
            print(f"  {lv} kernel(s) running: {at[lv] / 1e6 / steps:8.2f} ms/step")
    alone(sel, steps)


def alone(sel, steps, top=25):
    """Per kernel instantiation: time it ran with no other kernel beside it (the step's single-stream stretches —
    where the other streams had nothing to overlap)."""
    ev = []
    for i, r in enumerate(sel):
        ev.append((int(r["Start_Timestamp"]), 1, i))
        ev.append((int(r["End_Timestamp"]), -1, i))
    ev.sort()
    running, last = set(), ev[0][0]
    solo = collections.defaultdict(float)
    for t, d, i in ev:
        if t > last and len(running) == 1:
            solo[family(sel[next(iter(running))]["Kernel_Name"])[1]] += t - last
        if d > 0:
            running.add(i)
        else:
            running.discard(i)
        last = t
    print(f"\n# running alone (ms/step; top {top})")
    for k, v in sorted(solo.items(), key=lambda kv: -kv[1])[:top]:
        print(f"{v / 1e6 / steps:9.3f}  {k[:120]}")


if __name__ == "__main__":
    main()
