import sys, torch
sys.path.insert(0, "image-retrieval-for-image-based-localization_amd")
from cirtorch import _ops as ops, _engine as E
cuda = torch.device("cuda")
for dt in (torch.bfloat16, torch.float16):
    for shape in [(1, 96, 128), (2, 64, 64), (1, 96, 470)]:
        n, h, w = shape
        g = torch.Generator().manual_seed(h + 7 * w)
        x = torch.rand(n, 3, h, w, generator=g)
        wt = torch.randn(64, 3, 7, 7, generator=g) * 0.1
        scale = torch.rand(64, generator=g) + 0.5
        scale[::3] *= -1.0
        scale[5] = 0.0
        shift = torch.randn(64, generator=g) * 0.1
        mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
        wpk = ops.pack_stem_weights(wt.to(cuda), dt)
        outs = {}
        for mode in (0, 1):
            E.check(E.lib().rr_set_tuning(11, mode), "t")
            outs[mode] = ops.stem_conv_pool(x.to(cuda), wpk, scale.to(cuda), shift.to(cuda), leaky=True, slope=0.01, mean=mean, std=std).float().cpu()
        a, b = outs[0], outs[1]
        bad = (a != b)
        print(dt, shape, tuple(a.shape), "mismatch", int(bad.sum()), "maxdiff", float((a - b).abs().max()))
        if bad.any():
            idx = bad.nonzero()[:10]
            for t in idx.tolist():
                print("   ", t, float(a[tuple(t)]), float(b[tuple(t)]), "scale", float(scale[t[3]]))
            print("   channels", sorted(set(bad.nonzero()[:, 3].tolist()))[:20], "rows", sorted(set(bad.nonzero()[:, 1].tolist()))[:40], "cols", sorted(set(bad.nonzero()[:, 2].tolist()))[:60], "frac", float(bad.float().mean()))
