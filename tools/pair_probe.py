"""Time the 256-channel stage's block at the bench shape (128 x 192 x 256 pixels), fp16, HIP
events: the unfused 3x3 launch + rr_conv1x1_pair vs the fused rr_conv3x3_pair, for the three
forms the stage has (projection / residual + C1 64 / residual + C1 128).  Developer tool."""
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
    from cirtorch import _ops as ops
    dt = torch.float16
    g = torch.Generator(device="cuda").manual_seed(5)
    n = int(os.environ.get("N", "128"))
    h, w = 192, 256
    rn = lambda *s, sc=0.5: (torch.randn(*s, generator=g, device="cuda") * sc).to(dt)  # noqa: E731
    t1, xin, res = rn(n, h, w, 64), rn(n, h, w, 64), rn(n, h, w, 256)
    w33 = ops.pack_conv_weights(torch.randn(64, 64, 3, 3, generator=g, device="cuda") * 0.06, 64, dt, perm32=True)
    w3 = rn(256, 64, sc=0.1)
    wp = rn(256, 64, sc=0.1)
    one = lambda c: torch.ones(c, device="cuda")  # noqa: E731
    zero = lambda c: torch.zeros(c, device="cuda")  # noqa: E731
    for name, c1, proj in (("proj/64", 64, True), ("res/64", 64, False), ("res/128", 128, False)):
        w1 = rn(c1, 256, sc=0.05)
        pj = (xin, wp, one(256), zero(256)) if proj else None
        r = None if proj else res

        def unfused():
            t2 = ops.conv2d_fused(t1, w33, 3, 3, 1, 1, 64, one(64), zero(64), leaky=True, perm32=True)
            return ops.conv1x1_pair(t2, w3, one(256), zero(256), r, True, 0.01, w1, one(c1), zero(c1), c1, True, 0.01,
                                    proj=pj)

        def fused(dyn=True):
            return ops.conv3x3_pair(t1, w33, one(64), zero(64), True, 0.01, w3, one(256), zero(256), r, True, 0.01,
                                    w1, one(c1), zero(c1), c1, True, 0.01, proj=pj, dynamic=dyn)

        t2 = ops.conv2d_fused(t1, w33, 3, 3, 1, 1, 64, one(64), zero(64), leaky=True, perm32=True)

        def pair_only():
            return ops.conv1x1_pair(t2, w3, one(256), zero(256), r, True, 0.01, w1, one(c1), zero(c1), c1, True, 0.01,
                                    proj=pj)

        ya, za = unfused()
        yb, zb = fused()
        same = torch.equal(ya, yb) and torch.equal(za, zb)
        tu, tf, tp, ts = timed(unfused), timed(fused), timed(pair_only), timed(lambda: fused(False))
        print("block %-8s n=%d: unfused %.1f us (pair alone %.1f), fused %.1f us (%.3fx; %.3f of the pair alone; "
              "static walk %.1f), bit-identical %s" % (name, n, tu, tp, tf, tu / tf, tf / tp, ts, same), flush=True)


if __name__ == "__main__":
    main()
