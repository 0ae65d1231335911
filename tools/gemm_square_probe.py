"""Calibrate the 8-phase 256x256 GEMM (k_gemm8, through a 1x1 conv: P pixels x C_out x K, fp16) on
square shapes against torch.matmul (hipBLASLt) on the same box, random operands, HIP events.
Developer tool: is the conv shapes' ~1.05 PF the kernel or the shapes?"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    from cirtorch import _ops as ops
    from cirtorch import _engine as E
    if os.environ.get("G8"):  # RR_TUNE_GEMM8 value (2: k_gemm8 wherever legal, persistent)
        E.check(E.lib().rr_set_tuning(8, int(os.environ["G8"])), "rr_set_tuning")
    dt = torch.float16
    g = torch.Generator(device="cuda").manual_seed(1)
    shapes = ((4096, 4096, 4096), (8192, 8192, 8192), (16384, 4096, 2048), (393216, 256, 1024), (131072, 1024, 2048))
    if os.environ.get("SHAPES"):
        shapes = [tuple(int(v) for v in s.split("x")) for s in os.environ["SHAPES"].split(",")]
    for (p, c, k) in shapes:
        hw = p
        x = (torch.rand(1, 1, hw, k, generator=g, device="cuda") * 2 - 1).to(dt)
        wt = (torch.rand(c, k, 1, 1, generator=g, device="cuda") * 2 - 1) / k ** 0.5
        wp = ops.pack_conv_weights(wt, k, dt, perm32=True)
        one, zero = torch.ones(c, device="cuda"), torch.zeros(c, device="cuda")
        f = lambda: ops.conv2d_fused(x, wp, 1, 1, 1, 0, c, one, zero, leaky=False, perm32=True)  # noqa: E731
        a = x.view(hw, k)
        b = wt.view(c, k).to(dt).t()
        m = lambda: torch.matmul(a, b)  # noqa: E731
        fl = 2.0 * p * c * k
        t1, t2 = timed(f), timed(m)
        print("P=%d C=%d K=%d: k_gemm8 %.1f TF/s, hipBLASLt %.1f TF/s" % (p, c, k, fl / t1 / 1e12, fl / t2 / 1e12),
              flush=True)
        del x, wp, a, b


if __name__ == "__main__":
    main()
