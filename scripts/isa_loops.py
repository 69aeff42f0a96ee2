"""Instruction mix of every MFMA loop of the kernels in a hipcc --save-temps .s file.

    python scripts/isa_loops.py /tmp/conv_igemm-hip-amdgcn-amd-amdhsa-gfx950.s [name-substring ...]
Prints, per kernel, each backward-branch loop that contains MFMAs: length and VALU/SALU/DS/VMEM/MFMA counts
(the k-loop of a conv kernel is the one to read: VALU+SALU per MFMA is the issue overhead)."""
import re
import sys


def main():
    s = open(sys.argv[1]).read().split("\n")
    pats = sys.argv[2:]
    starts = [(i, l.split(":")[0]) for i, l in enumerate(s) if re.match(r"^_Z\w+:", l)]
    for i0, name in starts:
        if pats and not all(p in name for p in pats):
            continue
        end = i0 + 1
        while not s[end].startswith(".Lfunc_end"):
            end += 1
        body = s[i0:end]
        labels = {}
        for i, l in enumerate(body):
            m = re.match(r"^(\.LBB\d+_\d+):", l)
            if m:
                labels[m.group(1)] = i
        out = []
        for i, l in enumerate(body):
            m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", l)
            if not m:
                continue
            t = m.group(1) or m.group(2)
            if t in labels and labels[t] < i:
                cnt = {}
                for x in body[labels[t]:i + 1]:
                    x = x.strip()
                    if not x or x.startswith((";", ".")):
                        continue
                    op = x.split()[0]
                    k = ("mfma" if "mfma" in op else "valu" if op.startswith("v_") else "salu" if op.startswith("s_")
                         else "ds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_"))
                         else "other")
                    cnt[k] = cnt.get(k, 0) + 1
                if cnt.get("mfma"):
                    out.append(cnt)
        print(name.replace("_ZN12_GLOBAL__N_1", ""), out)


if __name__ == "__main__":
    main()
