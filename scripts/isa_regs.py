"""Per-kernel register footprint of two device-assembly dumps of the same source (e.g. before / after a change):
VGPR / AGPR / SGPR / spill counts from the code-object metadata, matched by demangled name with the 16-bit-type
namespace (``pva_bf16::`` / ``pva_f16::``) stripped, so a dump from before the dual build still lines up.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=fast --cuda-device-only -S -DPVA_F16=0 \\
        csrc/kernels/conv_igemm.hip -o new.s
    python scripts/isa_regs.py old.s new.s

A VGPR count crossing 512/w (w = waves per SIMD) costs a wave of occupancy: this is how the round-4 K-concatenated
loader and the BK=32 fragment ring were found to cost 8-56 VGPRs in every uniform-tap configuration
(profiles/r4_regress/README.md)."""
import re
import subprocess
import sys

FIELDS = (("vgpr_count", "v"), ("agpr_count", "a"), ("sgpr_count", "s"), ("vgpr_spill_count", "spill"))


def kernels(path):
    d, name = {}, None
    for line in open(path, errors="replace"):
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
        for key, tag in FIELDS:
            m = re.match(r"\s+\.%s:\s+(\d+)" % key, line)
            if m and name:
                d.setdefault(name, {})[tag] = int(m.group(1))
    names = list(d)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    return {re.sub(r"pva_(bf|f)16::", "", dm): d[n] for n, dm in zip(names, dem)}


def main():
    old, new = kernels(sys.argv[1]), kernels(sys.argv[2])
    same = changed = 0
    for k in old:
        if k not in new:
            continue
        if old[k] != new[k]:
            changed += 1
            print(k[:160], old[k], "->", new[k])
        else:
            same += 1
    print(f"# same {same}, changed {changed}, only old {len(set(old) - set(new))}, only new {len(set(new) - set(old))}")


if __name__ == "__main__":
    main()
