"""Library-GEMM ceiling for the path's GEMM shapes (developer calibration tool).

Times torch.matmul (hipBLASLt) on the shapes the engine's own kernels run —
the kNN score GEMM and the K >= 1024 1x1 convs of mod4/mod5 — so the hand-written
kernels' TFLOP/s can be read against what a tuned library reaches on the box.
Nothing here is on the product path."""
import torch


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    dev = torch.device("cuda:0")
    shapes = [  # (label, M, N, K, out dtype)
        ("knn score 262144x1024x2048 f32out", 262144, 1024, 2048, torch.float32),
        ("knn score 262144x128x2048 f32out", 262144, 128, 2048, torch.float32),
        ("mod4 conv1 393216x256x1024", 393216, 256, 1024, torch.bfloat16),
        ("mod5 conv1 98304x512x2048", 98304, 512, 2048, torch.bfloat16),
        ("mod5 proj 98304x2048x1024", 98304, 2048, 1024, torch.bfloat16),
        ("square 8192x8192x8192", 8192, 8192, 8192, torch.bfloat16),
    ]
    for label, m, n, k, od in shapes:
        a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        b = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
        if od == torch.float32:
            out = torch.empty(m, n, device=dev, dtype=torch.float32)
            fn = lambda: torch.matmul(a, b.t(), out_dtype=torch.float32) if hasattr(torch.matmul, "__call__") else None
            try:
                fn()
            except TypeError:
                fn = lambda: torch.mm(a, b.t()).float()
        else:
            fn = lambda: torch.mm(a, b.t())
        s = t(fn)
        print("%-40s %8.1f us  %7.1f TFLOP/s" % (label, s * 1e6, 2.0 * m * n * k / s / 1e12), flush=True)


if __name__ == "__main__":
    main()
