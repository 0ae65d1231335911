"""Time the mod3 boundary (rr_conv1x1_pair, 128 -> 512 -> 128, fp16) at the bench shape
(N x 96 x 128 pixels, two 2^20-pixel chunk launches at N = 128), HIP events: the 32-pixel
ring kernel (RR_TUNE_PAIR_MID = 1) vs the 64-pixel kernel (0), alternated, with the
algorithmic HBM rate and a bit-identity check.  Developer tool."""
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
    g = torch.Generator(device="cuda").manual_seed(5)
    n = int(os.environ.get("N", "128"))
    h, w = 96, 128
    rn = lambda *s, sc=0.5: (torch.randn(*s, generator=g, device="cuda") * sc).to(dt)  # noqa: E731
    x, res = rn(n, h, w, 128), rn(n, h, w, 512)
    w3, w1 = rn(512, 128, sc=0.1), rn(128, 512, sc=0.05)
    one = lambda c: torch.ones(c, device="cuda")  # noqa: E731
    zero = lambda c: torch.zeros(c, device="cuda")  # noqa: E731

    def run():
        return ops.conv1x1_pair(x, w3, one(512), zero(512), res, True, 0.01, w1, one(128), zero(128), 128, True, 0.01)

    p = n * h * w
    gb = p * 2 * (128 + 512 + 512 + 128) / 1e9
    out, t = {}, {0: [], 1: []}
    try:
        for rnd in range(3):
            for mode in (0, 1):
                E.check(E.lib().rr_set_tuning(15, mode), "rr_set_tuning")
                out[mode] = run()
                t[mode].append(timed(run))
    finally:
        E.lib().rr_set_tuning(15, 1)
    same = torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    for mode in (0, 1):
        best = min(t[mode])
        print("pair_mid mode %d (%s): %s us, best %.1f us = %.2f TB/s algorithmic" % (
            mode, "ring 32 px" if mode else "64 px", " ".join("%.1f" % v for v in t[mode]), best, gb / best * 1e3))
    print("bit-identical:", same)


if __name__ == "__main__":
    main()
