"""hipBLASLt (torch.matmul, bf16) on the network's GEMM shapes: a library ceiling to price the framework's own
implicit-GEMM kernels against.  python scripts/blas_ceiling.py"""
import torch

SHAPES = [  # (label, M, N, K, transA) - transA: wgrad form C[N,K] = A^T B over the long M axis
    ("square 8192^3", 8192, 8192, 8192, False),
    ("b1.p0 a.dgrad 1x1 (M=4.0M N=256 K=64)", 4014080, 256, 64, False),
    ("b1.p0 c.fwd 1x1 (M=4.0M N=256 K=64)", 4014080, 256, 64, False),
    ("b1.p0 a.fwd 1x1 (M=4.0M N=64 K=256)", 4014080, 64, 256, False),
    ("b3.p0.0.a.fwd as GEMM (M=1.0M N=256 K=1920)", 1003520, 256, 1920, False),
    ("b3.p0.0.a.dgrad as GEMM (M=1.0M N=640 K=768)", 1003520, 640, 768, False),
    ("b3.p0.x.a.fwd as GEMM (M=251K N=256 K=3072)", 250880, 256, 3072, False),
    ("b3.p0.x.a.dgrad as GEMM (M=251K N=1024 K=768)", 250880, 1024, 768, False),
    ("b4.p0.x.c.fwd (M=62.7K N=2048 K=512)", 62720, 2048, 512, False),
    ("lab 250880x1024x1024", 250880, 1024, 1024, False),
    ("b3.p0.0.a.wgrad as GEMM (256 x 1920 over M=1.0M)", 1003520, 256, 1920, True),
    ("b3.p0.x.a.wgrad as GEMM (256 x 3072 over M=251K)", 250880, 256, 3072, True),
]


def main():
    dev = torch.device("cuda")
    for label, M, N, K, ta in SHAPES:
        if ta:
            a = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
            b = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            f = lambda: torch.matmul(a.t(), b)
        else:
            a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
            f = lambda: torch.matmul(a, b)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        fl = 2.0 * M * N * K
        by = 2.0 * (M * K + K * N + M * N) if not ta else 2.0 * (M * N + M * K + N * K)
        print(f"{label:52s} {ms * 1e3:9.1f} us {fl / ms / 1e9:8.1f} TF/s {by / ms / 1e9:6.2f} TB/s", flush=True)
        del a, b


if __name__ == "__main__":
    main()
