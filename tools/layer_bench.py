"""Per-layer timing of the extractor on the GPU engine: every distinct conv of
the body at the bench shape, timed with HIP events (median of reps), with its
algorithmic TFLOP/s.  Developer tool (not part of the product path).

    python tools/layer_bench.py [--arch resnet50 --batch 8 --precision bf16]
"""

import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--height", type=int, default=768)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tune", default="", help="rr_set_tuning pairs key=value[,key=value]")
    args = ap.parse_args()
    from cirtorch import _ops
    from cirtorch.backbones import resnet
    from cirtorch.models.init import random_init_
    from cirtorch import _engine as E
    for kv in filter(None, args.tune.split(",")):
        k_, v_ = kv.split("=")
        E.check(E.lib().rr_set_tuning(int(k_), int(v_)), "rr_set_tuning")

    body = resnet.__dict__[args.arch](precision=args.precision)
    random_init_(body, 0)
    body = body.cuda().eval()
    x = torch.rand(args.batch, 3, args.height, args.width, device="cuda")
    plan = body._build_plan()
    dt = body.engine_dtype
    # walk the plan once, recording each conv's input tensor
    calls = []
    t = _ops.image_to_nhwc(x, body.stem_cin(), dt, [0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
    calls.append(("stem", t, plan["stem"], None))
    t = body._conv(t, plan["stem"])
    t = _ops.maxpool2d(t, 3, 2, 1)
    for mi, blocks in enumerate(plan["mods"]):
        for bi, (steps, proj) in enumerate(blocks):
            if proj is not None:
                calls.append(("mod%d.b%d.proj" % (mi + 2, bi + 1), t, proj, None))
                res = body._conv(t, proj)
            else:
                res = t
            y = t
            for si, st in enumerate(steps[:-1]):
                calls.append(("mod%d.b%d.c%d" % (mi + 2, bi + 1, si + 1), y, st, None))
                y = body._conv(y, st)
            calls.append(("mod%d.b%d.c%d" % (mi + 2, bi + 1, len(steps)), y, steps[-1], res))
            t = body._conv(y, steps[-1], residual=res)
    seen = {}
    total_t, total_f = 0.0, 0.0
    print("%-16s %-34s %8s %9s %8s %5s" % ("layer", "shape (P x Cout x K)", "us", "TFLOP/s", "GFLOP", "calls"))
    for name, inp, st, res in calls:
        n, h, w, c = inp.shape
        ho = (h + 2 * st.pad - st.kh) // st.stride + 1
        wo = (w + 2 * st.pad - st.kw) // st.stride + 1
        key = (tuple(inp.shape), st.kh, st.stride, st.c_out, res is not None)
        P = n * ho * wo
        flops = 2.0 * P * st.c_out * st.kh * st.kw * (3 if name == "stem" else c)
        if key not in seen:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
            for _ in range(3):
                body._conv(inp, st, residual=res)
            for a, b in ev:
                a.record()
                body._conv(inp, st, residual=res)
                b.record()
            torch.cuda.synchronize()
            ts = sorted(a.elapsed_time(b) for a, b in ev)
            seen[key] = [ts[len(ts) // 2] * 1e3, flops, 0, name, "%d x %d x %d(k%ds%d)" % (P, st.c_out, st.kh * st.kw * c, st.kh, st.stride)]
        seen[key][2] += 1
    for us, flops, cnt, name, shape in seen.values():
        print("%-16s %-34s %8.1f %9.1f %8.2f %5d" % (name, shape, us, flops / us / 1e6, flops / 1e9, cnt))
        total_t += us * cnt
        total_f += flops * cnt
    print("TOTAL conv time %.3f ms, %.1f GFLOP, %.1f TFLOP/s" % (total_t / 1e3, total_f / 1e9, total_f / total_t / 1e6))


if __name__ == "__main__":
    main()
