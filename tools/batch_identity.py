"""Does image 0 of a B-image chain give the same bits as the same image alone?
Compares the body's stage maps, then replays every conv step of the first
differing stage on both (the batched stage input and its first image) and
prints the first step whose outputs differ, with its launch shape.

  python tools/batch_identity.py [--batch 8] [--precision bf16] [--h 768 --w 1024]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "image-retrieval-for-image-based-localization_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--h", type=int, default=768)
    ap.add_argument("--w", type=int, default=1024)
    args = ap.parse_args()
    from cirtorch.models.GF_net import make_net
    from cirtorch.models.init import random_init_
    dev = torch.device("cuda", 0)
    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    net = random_init_(make_net(args.arch, precision=args.precision, mean=mean, std=std), 1).to(dev).eval()
    body = net.body
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 256, (args.batch, 3, args.h, args.w), generator=g, dtype=torch.uint8).to(dev)
    with torch.no_grad():
        ob = body(x, normalize=(mean, std))
        o1 = body(x[:1].clone(), normalize=(mean, std))
        first = None
        for k in ob:
            a, b = ob[k][:1].float(), o1[k].float()
            eq = torch.equal(a, b)
            print("%-5s %-22s equal=%s maxdiff=%.3g" % (k, tuple(ob[k].shape), eq, (a - b).abs().max().item()))
            if not eq and first is None:
                first = k
        if first is None:
            d1 = net.extract(x[:1].clone())
            db = net.extract(x)[:, :1]
            print("descriptor equal=%s" % torch.equal(d1, db))
            return
        plan = body._plan
        mod_id = int(first[3:]) - 2
        if mod_id < 0:
            print("stem differs")
            return
        prev = "mod%d" % (mod_id + 1)
        tb = ob[prev].permute(0, 2, 3, 1)  # back to the NHWC storage
        t1 = tb[:1].contiguous()
        for bi, (steps, proj) in enumerate(plan["mods"][mod_id]):
            resb = tb if proj is None else body._conv(tb, proj)
            res1 = t1 if proj is None else body._conv(t1, proj)
            if proj is not None and not torch.equal(resb[:1], res1):
                print("block %d proj differs: k%d s%d kp %d cout %d P1 %d" % (bi, proj.kh, proj.stride, proj.w.shape[1],
                                                                             proj.c_out, res1.shape[1] * res1.shape[2]))
                return
            yb, y1 = tb, t1
            for j, st in enumerate(steps):
                last = j + 1 == len(steps)
                yb = body._conv(yb, st, residual=resb if last else None)
                y1 = body._conv(y1, st, residual=res1 if last else None)
                if not torch.equal(yb[:1], y1):
                    d = (yb[:1].float() - y1.float()).abs().max().item()
                    print("block %d step %d differs (maxdiff %.3g): k%d s%d kp %d cout %d in %s out %s" % (
                        bi, j, d, st.kh, st.stride, st.w.shape[1], st.c_out, tuple(t1.shape), tuple(y1.shape)))
                    return
            tb, t1 = yb, y1
        print("unfused replay of %s is identical: the fused boundary kernels differ" % first)


if __name__ == "__main__":
    main()
