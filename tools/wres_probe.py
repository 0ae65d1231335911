"""Time the non-residual k_wres1x1 layers of the R50 bench step at 128 images (fp16, HIP events):
the strided mod3 projection (256 -> 512, two image groups), the strided mod4 projection (512 ->
1024) and mod4's block-1 conv1 (512 -> 256), with the deep tile rings (RR_TUNE_WRES_RING = 1,
default) vs two tiles ahead (0), alternated, plus a bit-identity check.  Developer tool."""
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
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    from cirtorch import _engine as E
    from cirtorch import _ops as ops
    dt = torch.float16
    g = torch.Generator(device="cuda").manual_seed(9)
    n = int(os.environ.get("N", "128"))
    layers = (("mod3.proj s2 256->512", (n, 192, 256, 256), 512, 2), ("mod4.proj s2 512->1024", (n, 96, 128, 512), 1024, 2),
              ("mod4.b1.c1 512->256", (n, 96, 128, 512), 256, 1))
    for name, shp, cout, stride in layers:
        x = (torch.randn(*shp, generator=g, device="cuda") * 0.5).to(dt)
        wp = ops.pack_conv_weights(torch.randn(cout, shp[3], 1, 1, generator=g, device="cuda") * 0.05, shp[3], dt,
                                   perm32=True)
        sc, sh = torch.ones(cout, device="cuda"), torch.zeros(cout, device="cuda")
        f = lambda: ops.conv2d_fused(x, wp, 1, 1, stride, 0, cout, sc, sh, leaky=True, perm32=True)  # noqa: E731
        t, out = {0: [], 1: []}, {}
        try:
            for _ in range(3):
                for mode in (0, 1):
                    E.check(E.lib().rr_set_tuning(16, mode), "rr_set_tuning")
                    out[mode] = f()
                    t[mode].append(timed(f))
        finally:
            E.lib().rr_set_tuning(16, 1)
        print("%-24s two ahead %s | deep %s us, bit-identical %s" % (
            name, " ".join("%.1f" % v for v in t[0]), " ".join("%.1f" % v for v in t[1]),
            torch.equal(out[0], out[1])), flush=True)
        del x


if __name__ == "__main__":
    main()
