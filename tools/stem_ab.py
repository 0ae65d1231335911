"""A/B timing of the fused stem variants (RR_TUNE_STEM modes) at the bench shape:
B x 3 x 768 x 1024 float32 and uint8 images, HIP events, modes alternated.
Developer tool (not part of the product path).

    python tools/stem_ab.py [--batch 128 --modes 2,5 --reps 10]
"""

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--height", type=int, default=768)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--modes", default="2,5")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--dtype", default="fp16")
    args = ap.parse_args()
    from cirtorch import _engine as E
    from cirtorch import _ops
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[args.dtype]
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.rand(args.batch, 3, args.height, args.width, generator=g, device="cuda")
    xu = (x * 255).to(torch.uint8)
    w = torch.randn(64, 3, 7, 7, generator=g, device="cuda") * 0.1
    scale = torch.rand(64, generator=g, device="cuda") + 0.5
    shift = torch.randn(64, generator=g, device="cuda") * 0.1
    wpk = _ops.pack_stem_weights(w, dt)
    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    modes = [int(m) for m in args.modes.split(",")]
    res = {m: {"f32": [], "u8": []} for m in modes}
    outs = {}
    ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        # warm-up of every mode and input first: the first timed loop of a process
        # otherwise runs ~15 % slow (clocks / first touch), whichever mode it is
        for m in modes:
            E.check(E.lib().rr_set_tuning(11, m), "rr_set_tuning")
            for inp in (x, xu):
                for _ in range(5):
                    _ops.stem_conv_pool(inp, wpk, scale, shift, mean=mean, std=std)
        torch.cuda.synchronize()
        for rnd in range(args.rounds):
            for m in modes:
                E.check(E.lib().rr_set_tuning(11, m), "rr_set_tuning")
                for name, inp in (("f32", x), ("u8", xu)):
                    y = _ops.stem_conv_pool(inp, wpk, scale, shift, mean=mean, std=std)
                    torch.cuda.synchronize()
                    ea.record()
                    for _ in range(args.reps):
                        y = _ops.stem_conv_pool(inp, wpk, scale, shift, mean=mean, std=std)
                    eb.record()
                    torch.cuda.synchronize()
                    res[m][name].append(ea.elapsed_time(eb) / args.reps * 1e3)
                    if rnd == 0:
                        outs[(m, name)] = y.float()
    finally:
        E.lib().rr_set_tuning(11, 2)
    cmp = {}
    for m in modes[1:]:
        for name in ("f32", "u8"):
            a, b = outs[(modes[0], name)], outs[(m, name)]
            d = (a - b).abs()
            cmp["%d_vs_%d_%s" % (m, modes[0], name)] = {"max_abs": d.max().item(), "frac_equal": (d == 0).float().mean().item(),
                                                       "max_ref": a.abs().max().item()}
    print(json.dumps({"us_per_launch": res, "compare": cmp, "batch": args.batch, "dtype": args.dtype}))


if __name__ == "__main__":
    main()
