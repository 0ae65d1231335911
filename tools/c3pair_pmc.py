"""Run the fused mod2 block (rr_conv3x3_pair) and, for comparison, the boundary kernel alone
(rr_conv1x1_pair) 10 times each at the bench shape, for rocprofv3 counter passes.
    python3 tools/c3pair_pmc.py [proj|res64|res128]   Developer tool."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    from cirtorch import _ops as ops
    form = sys.argv[1] if len(sys.argv) > 1 else "res128"
    dt = torch.float16
    g = torch.Generator(device="cuda").manual_seed(5)
    n, h, w = 128, 192, 256
    rn = lambda *s, sc=0.5: (torch.randn(*s, generator=g, device="cuda") * sc).to(dt)  # noqa: E731
    t1, xin, res = rn(n, h, w, 64), rn(n, h, w, 64), rn(n, h, w, 256)
    w33 = ops.pack_conv_weights(torch.randn(64, 64, 3, 3, generator=g, device="cuda") * 0.06, 64, dt, perm32=True)
    w3, wp = rn(256, 64, sc=0.1), rn(256, 64, sc=0.1)
    one = lambda c: torch.ones(c, device="cuda")  # noqa: E731
    zero = lambda c: torch.zeros(c, device="cuda")  # noqa: E731
    proj = form == "proj"
    c1 = 128 if form == "res128" else 64
    w1 = rn(c1, 256, sc=0.05)
    pj = (xin, wp, one(256), zero(256)) if proj else None
    r = None if proj else res
    t2 = ops.conv2d_fused(t1, w33, 3, 3, 1, 1, 64, one(64), zero(64), leaky=True, perm32=True)
    for _ in range(10):
        ops.conv3x3_pair(t1, w33, one(64), zero(64), True, 0.01, w3, one(256), zero(256), r, True, 0.01,
                         w1, one(c1), zero(c1), c1, True, 0.01, proj=pj)
    for _ in range(10):
        ops.conv1x1_pair(t2, w3, one(256), zero(256), r, True, 0.01, w1, one(c1), zero(c1), c1, True, 0.01, proj=pj)
    torch.cuda.synchronize()
    print("done", form)


if __name__ == "__main__":
    main()
