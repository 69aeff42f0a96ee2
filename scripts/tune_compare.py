"""Compare two autotuner logs (``PVA_TUNE_LOG=1`` stderr of bench.py): per geometry, the time of the chosen
configuration in each log and, for every configuration family present in both, its time.

    python scripts/tune_compare.py OLD.txt NEW.txt [--family 256x256]
Geometries are matched by their ``M N K taps`` key in order of appearance (a key that occurs several times is
matched occurrence by occurrence)."""
import argparse
import collections
import re

LINE = re.compile(r"tune M=(\d+) N=(\d+) K=(\d+) taps=\(([^)]*)\): (.*) -> (\S+)")


def parse(path):
    out = collections.defaultdict(list)
    for l in open(path, errors="replace"):
        m = LINE.search(l)
        if not m:
            continue
        key = (int(m.group(1)), int(m.group(2)), int(m.group(3)), m.group(4).replace(" ", ""))
        times = {}
        for tok in m.group(5).split():
            name, _, t = tok.rpartition("=")
            if t.endswith("us"):
                times[name] = float(t[:-2])
        out[key].append((times, m.group(6)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("old")
    ap.add_argument("new")
    ap.add_argument("--family", default="", help="also list every configuration containing this substring")
    ap.add_argument("--families", action="store_true",
                    help="only the median new/old time ratio per configuration family (tile / loader / staging)")
    a = ap.parse_args()
    old, new = parse(a.old), parse(a.new)
    if a.families:
        import statistics
        fam = collections.defaultdict(list)
        for key, runs in new.items():
            for i, (tn, _) in enumerate(runs):
                if key not in old or i >= len(old[key]):
                    continue
                to = old[key][i][0]
                for c in tn:
                    if c in to:
                        fam[re.sub(r"\d+(?=[a-z/]|$)", "", c) if not re.match(r"\d+x\d+", c) else c].append(tn[c] / to[c])
        for f, v in sorted(fam.items()):
            print(f"{f:26s} n={len(v):4d}  median new/old {statistics.median(v):.3f}")
        return
    tot_o = tot_n = 0.0
    print(f"{'M':>9s} {'N':>5s} {'K':>5s} {'taps':>7s}  {'old best':>26s} {'us':>8s}  {'new best':>26s} {'us':>8s}  {'ratio':>6s}")
    for key, runs in new.items():
        for i, (tn, bn) in enumerate(runs):
            if key not in old or i >= len(old[key]):
                continue
            to, bo = old[key][i]
            uo, un = to.get(bo, float("nan")), tn.get(bn, float("nan"))
            tot_o += uo
            tot_n += un
            print(f"{key[0]:9d} {key[1]:5d} {key[2]:5d} {key[3]:>7s}  {bo:>26s} {uo:8.1f}  {bn:>26s} {un:8.1f}  {un / uo:6.3f}")
            if a.family:
                for c in sorted(set(to) | set(tn)):
                    if a.family in c:
                        print(f"{'':30s} {c:>26s} {to.get(c, float('nan')):8.1f} -> {tn.get(c, float('nan')):8.1f}")
    print(f"# sum of chosen configurations: old {tot_o / 1e3:.2f} ms, new {tot_n / 1e3:.2f} ms (tuning-time timings, "
          f"serialised, one launch each)")


if __name__ == "__main__":
    main()
