"""Time every GEMM tile configuration (rr_set_tuning) on the distinct conv
shapes of the extractor; prints a table (us per launch).  Developer tool.

    python tools/tune_layers.py [--batch 32]
"""

import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

CFG = {1: "128x128", 2: "64x256", 3: "256x128w", 4: "256x256w", 5: "256x64", 6: "A-stat", 7: "256x128w3", 8: "128x256w3"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from cirtorch import _engine as E, _ops
    from cirtorch.backbones import resnet
    from cirtorch.models.init import random_init_

    body = resnet.resnet50(precision="bf16")
    random_init_(body, 0)
    body = body.cuda().eval()
    x = torch.rand(args.batch, 3, 768, 1024, device="cuda")
    plan = body._build_plan()
    calls = []
    t = _ops.image_to_nhwc(x, 8, torch.bfloat16, [0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
    calls.append(("stem", t, plan["stem"], None))
    t = body._conv(t, plan["stem"])
    t = _ops.maxpool2d(t, 3, 2, 1)
    for mi, blocks in enumerate(plan["mods"]):
        for bi, (steps, proj) in enumerate(blocks):
            res = body._conv(t, proj) if proj is not None else t
            if proj is not None and bi == 0:
                calls.append(("mod%d.proj" % (mi + 2), t, proj, None))
            y = t
            for si, st in enumerate(steps[:-1]):
                if bi < 2:
                    calls.append(("mod%d.b%d.c%d" % (mi + 2, bi + 1, si + 1), y, st, None))
                y = body._conv(y, st)
            if bi < 1:
                calls.append(("mod%d.b%d.c3" % (mi + 2, bi + 1), y, steps[-1], res))
            t = body._conv(y, steps[-1], residual=res)

    def timeit(inp, st, res):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        body._conv(inp, st, residual=res)
        for a, b in ev:
            a.record()
            body._conv(inp, st, residual=res)
            b.record()
        torch.cuda.synchronize()
        ts = sorted(a.elapsed_time(b) for a, b in ev)
        return ts[len(ts) // 2] * 1e3

    # (label, {tuning key: value}); key 0 = tile config, 4 = XCD tile order
    # (label, {tuning key: value}); key 0 = tile config, 5 = streaming 1x1 kernel
    variants = [("auto", {0: 0, 5: 1, 1: 2}), ("auto/noS", {0: 0, 5: 0, 1: 2})] + \
               [(CFG[c], {0: c, 5: 0, 1: 2}) for c in CFG] + \
               [(CFG[c] + "s3", {0: c, 5: 0, 1: 3}) for c in (1, 2, 3, 5)]
    head = "%-14s %-26s" % ("layer", "P x Cout x K") + "".join("%12s" % v[0] for v in variants)
    print(head)
    for name, inp, st, res in calls:
        n, h, w, c = inp.shape
        ho = (h + 2 * st.pad - st.kh) // st.stride + 1
        wo = (w + 2 * st.pad - st.kw) // st.stride + 1
        row = "%-14s %-26s" % (name, "%d x %d x %d" % (n * ho * wo, st.c_out, st.kh * st.kw * c))
        for _, kv in variants:
            for k_, v_ in kv.items():
                E.lib().rr_set_tuning(k_, v_)
            try:
                row += "%12.1f" % timeit(inp, st, res)
            except Exception:
                row += "%12s" % "err"
        print(row, flush=True)
    E.lib().rr_set_tuning(0, 0)
    E.lib().rr_set_tuning(1, 2)
    E.lib().rr_set_tuning(5, 1)


if __name__ == "__main__":
    main()
