"""Time the strided mod3 3x3 (128 -> 128, stride 2, 128 x 192 x 256 input) on k_gemm8a, persistent
(default) vs one block per tile (RR_TUNE_GEMM8 | 128), fp16, HIP events.  Developer tool."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    from cirtorch import _engine as E
    from cirtorch import _ops as ops
    dt = torch.float16
    g = torch.Generator(device="cuda").manual_seed(3)
    n = int(os.environ.get("N", "128"))
    x = (torch.randn(n, 192, 256, 128, generator=g, device="cuda") * 0.5).to(dt)
    wp = ops.pack_conv_weights(torch.randn(128, 128, 3, 3, generator=g, device="cuda") * 0.04, 128, dt, perm32=True)
    sc, sh = torch.ones(128, device="cuda"), torch.zeros(128, device="cuda")
    outs = {}
    for name, v in (("persistent", 1), ("per-tile", 1 | 128), ("persistent", 1)):
        E.check(E.lib().rr_set_tuning(8, v), "rr_set_tuning")
        f = lambda: ops.conv2d_fused(x, wp, 3, 3, 2, 1, 128, sc, sh, leaky=True, perm32=True)  # noqa: E731
        for _ in range(3):
            y = f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            y = f()
        e1.record()
        torch.cuda.synchronize()
        outs.setdefault(name, y)
        print("gemm8a %-10s n=%d: %.1f us" % (name, n, e0.elapsed_time(e1) / 10 * 1e3), flush=True)
    E.lib().rr_set_tuning(8, 1)
    print("bit-identical:", torch.equal(outs["persistent"], outs["per-tile"]))


if __name__ == "__main__":
    main()
