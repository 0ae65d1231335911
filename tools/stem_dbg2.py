import sys, torch, itertools
sys.path.insert(0, "image-retrieval-for-image-based-localization_amd")
from cirtorch import _ops as ops, _engine as E
cuda = torch.device("cuda")
dt = torch.float16
n, h, w = 1, 96, 128
g = torch.Generator().manual_seed(5)
x = torch.rand(n, 3, h, w, generator=g)
wt = torch.randn(64, 3, 7, 7, generator=g) * 0.1
scale = torch.rand(64, generator=g) + 0.5
shift = torch.randn(64, generator=g) * 0.1
mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
wpk = ops.pack_stem_weights(wt.to(cuda), dt)
E.check(E.lib().rr_set_tuning(11, 1), "t")
v2 = ops.stem_conv_pool(x.to(cuda), wpk, scale.to(cuda), shift.to(cuda), leaky=True, slope=0.01, mean=mean, std=std).float().cpu()
xe = ops.image_to_nhwc(x.to(cuda), 8, dt, mean, std)
wp = ops.pack_conv_weights(wt.to(cuda), 8, dt, perm32=True)
S = ops.conv2d_fused(xe, wp, 7, 7, 2, 3, 64, scale.to(cuda), shift.to(cuda), leaky=True, perm32=True).float().cpu()[0]
print("stem map", S.shape, "pooled", v2.shape)
Sp = torch.full((S.shape[0] + 2, S.shape[1] + 2, 64), float("-inf"))
Sp[1:-1, 1:-1] = S
for (pr, pc) in [(0, 0), (0, 1), (1, 0), (1, 1), (0, 2), (2, 0), (2, 2)]:
    ref = Sp[2 * pr:2 * pr + 3, 2 * pc:2 * pc + 3].amax(dim=(0, 1))
    got = v2[0, pr, pc]
    ok = float((ref - got).abs().max())
    # which single stem pixel / window rows match?
    cand = []
    for r0 in range(0, 8):
        for c0 in range(0, 8):
            for hh, ww in [(3, 3), (2, 3), (3, 2), (2, 2), (1, 3), (3, 1), (1, 1), (1, 2), (2, 1)]:
                m = Sp[r0:r0 + hh, c0:c0 + ww].amax(dim=(0, 1))
                if float((m - got).abs().max()) < 2e-3:
                    cand.append((r0 - 1, c0 - 1, hh, ww))
    print((pr, pc), "maxdiff vs ref %.4f" % ok, "matching windows (stem r0, c0, h, w):", cand[:6])
