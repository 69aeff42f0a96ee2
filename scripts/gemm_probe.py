"""hipBLASLt (torch.matmul, bf16) throughput at the im2col GEMM shapes of the SlowFast convs — the library
reference the hand-written conv kernels are compared against (python scripts/gemm_probe.py)."""
import torch


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    dev = torch.device("cuda")
    shapes = [(4014080, 64, 576), (1003520, 128, 1152), (250880, 256, 2304), (62720, 512, 4608),
              (250880, 256, 3072), (62720, 512, 6144), (1003520, 640, 768), (8192, 8192, 8192),
              (4014080, 256, 64), (1003520, 512, 128)]
    for M, N, K in shapes:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: a @ b)
        print("M=%8d N=%5d K=%5d  %8.1f us  %6.0f TF/s" % (M, N, K, t * 1e6, 2 * M * N * K / t / 1e12), flush=True)
        del a, b


if __name__ == "__main__":
    main()
