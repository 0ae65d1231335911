"""Calibration (developer tool, not the product path): torch.matmul (hipBLASLt) fp16 TFLOP/s
on the GEMM shapes of the body's MFMA-bound layers at 128 images, to compare with the
engine's own kernels (tools/layer_bench.py)."""
import torch

shapes = {  # name: (M pixels, N c_out, K)
    "mod4.c1 1x1 1024->256": (393216, 256, 1024),
    "mod4.c2 3x3 as GEMM": (393216, 256, 2304),
    "mod5.c1 1x1 2048->512": (98304, 512, 2048),
    "mod5.c2 3x3 as GEMM": (98304, 512, 4608),
    "mod3.c2 3x3 as GEMM": (1572864, 128, 1152),
    "mod2.c2 3x3 as GEMM": (6291456, 64, 576),
    "knn Q=1024 fp16": (1024, 1000000, 2048),
    "square 8192": (8192, 8192, 8192),
}
for name, (m, n, k) in shapes.items():
    a = torch.randn(m, k, device="cuda", dtype=torch.float16)
    b = torch.randn(k, n, device="cuda", dtype=torch.float16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print("%-24s M %8d N %7d K %5d  %8.1f us  %7.1f TFLOP/s" % (name, m, n, k, ms * 1e3, 2.0 * m * n * k / ms / 1e9))
    del a, b, c
    torch.cuda.empty_cache()
