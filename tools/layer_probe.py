"""Run ONE conv layer of the ResNet-50 extractor repeatedly (for rocprofv3
counter passes).  Developer tool.

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -d gpurun_out/pmc -- python3 tools/layer_probe.py --layer mod2.b1.c2

The probe's own launches are the last --reps dispatches of the run.
"""

import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def walk(body, x):
    """(name, input, step, residual) for the first two blocks of every stage."""
    from cirtorch import _ops
    plan = body._build_plan()
    calls = []
    t = _ops.image_to_nhwc(x, body.stem_cin(), body.engine_dtype, [0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
    calls.append(("stem", t, plan["stem"], None))
    t = body._conv(t, plan["stem"])
    t = _ops.maxpool2d(t, 3, 2, 1)
    for mi, blocks in enumerate(plan["mods"]):
        for bi, (steps, proj) in enumerate(blocks):
            res = body._conv(t, proj) if proj is not None else t
            if proj is not None:
                calls.append(("mod%d.proj" % (mi + 2), t, proj, None))
            y = t
            for si, st in enumerate(steps[:-1]):
                calls.append(("mod%d.b%d.c%d" % (mi + 2, bi + 1, si + 1), y, st, None))
                y = body._conv(y, st)
            calls.append(("mod%d.b%d.c%d" % (mi + 2, bi + 1, len(steps)), y, steps[-1], res))
            t = body._conv(y, steps[-1], residual=res)
    return calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="mod2.b1.c2")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tune", default="", help="key=value,... passed to rr_set_tuning")
    args = ap.parse_args()
    from cirtorch import _engine as E
    from cirtorch.backbones import resnet
    from cirtorch.models.init import random_init_

    body = resnet.resnet50(precision="bf16")
    random_init_(body, 0)
    body = body.cuda().eval()
    x = torch.rand(args.batch, 3, 768, 1024, device="cuda")
    calls = {n: (i, s, r) for n, i, s, r in walk(body, x)}
    inp, st, res = calls[args.layer]
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        E.check(E.lib().rr_set_tuning(int(k), int(v)), "rr_set_tuning")
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(args.reps):
        body._conv(inp, st, residual=res)
    b.record()
    torch.cuda.synchronize()
    print("%s: %.1f us/launch" % (args.layer, a.elapsed_time(b) * 1e3 / args.reps))


if __name__ == "__main__":
    main()
