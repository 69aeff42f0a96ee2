"""HBM streaming ceilings on this GPU (torch kernels): read-only (sum), write-only (fill), read+write (copy), and
read 2 + write 1 (add) over 2 GiB bf16 tensors — the reference points for the memory-bound fused kernels' TB/s.
python scripts/stream_ceiling.py"""
import torch


def t(f, reps=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    n = 1 << 30
    a = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    c = torch.empty_like(a)
    g = 2 * n / 1e9
    for name, f, gb in (("read (sum)", lambda: a.sum(dtype=torch.float32), g),
                        ("write (fill)", lambda: c.fill_(1.0), g),
                        ("read+write (copy)", lambda: c.copy_(a), 2 * g),
                        ("2 reads + write (add)", lambda: torch.add(a, b, out=c), 3 * g)):
        ms = t(f)
        print(f"{name:24s} {ms * 1e3:8.1f} us  {gb / ms:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
