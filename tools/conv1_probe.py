"""mod2 block 1 at the bench shape (128 x 192 x 256): conv1 (1x1 64 -> 64) as its own launch +
the fused block, vs conv1 inside the fused block (rr_conv3x3_pair with w0).  Developer tool."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
import torch  # noqa: E402
from cirtorch import _ops as ops  # noqa: E402
dt = torch.float16
g = torch.Generator(device="cuda").manual_seed(5)
n, h, w = 128, 192, 256
rn = lambda *s, sc=0.5: (torch.randn(*s, generator=g, device="cuda") * sc).to(dt)
x = rn(n, h, w, 64)
w0 = ops.pack_conv_weights(torch.randn(64, 64, 1, 1, generator=g, device="cuda") * 0.15, 64, dt, perm32=True)
w33 = ops.pack_conv_weights(torch.randn(64, 64, 3, 3, generator=g, device="cuda") * 0.06, 64, dt, perm32=True)
w3, wp, w1 = rn(256, 64, sc=0.1), rn(256, 64, sc=0.1), rn(64, 256, sc=0.05)
one = lambda c: torch.ones(c, device="cuda"); zero = lambda c: torch.zeros(c, device="cuda")
pj = (x, wp, one(256), zero(256))
def unf():
    t1 = ops.conv2d_fused(x, w0, 1, 1, 1, 0, 64, one(64), zero(64), leaky=True, perm32=True)
    return ops.conv3x3_pair(t1, w33, one(64), zero(64), True, 0.01, w3, one(256), zero(256), None, True, 0.01, w1, one(64), zero(64), 64, True, 0.01, proj=pj)
def fus():
    return ops.conv3x3_pair(x, w33, one(64), zero(64), True, 0.01, w3, one(256), zero(256), None, True, 0.01, w1, one(64), zero(64), 64, True, 0.01, proj=pj, conv1=(w0, one(64), zero(64), True, 0.01))
def tm(f):
    for _ in range(3): f()
    torch.cuda.synchronize(); a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10): f()
    b.record(); torch.cuda.synchronize(); return a.elapsed_time(b)/10*1e3
for _ in range(2):
    print("conv1 launch + block %.1f us, conv1 in the block %.1f us" % (tm(unf), tm(fus)), flush=True)
