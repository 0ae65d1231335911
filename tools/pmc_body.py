"""Workload for the HBM-traffic counter passes of the extractor body (the
bench's dominant kernel family): warm up, then run ITERS forwards of the body
(R50, bf16, B x 3 x H x W) between two marker kernels so the parser can pick
exactly the body's dispatches out of the rocprofv3 counter CSV.

    rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- python3 tools/pmc_body.py
    rocprofv3 --pmc WRITE_SIZE -d DIR -o run --output-format csv -- python3 tools/pmc_body.py
    python3 tools/pmc_parse.py DIR_FETCH DIR_WRITE --iters 3 --batch 32 > profiles/<round>_pmc_traffic.json

Developer tool (not part of the product path)."""

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
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--height", type=int, default=768)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--precision", default="fp16")
    args = ap.parse_args()
    from cirtorch import _ops
    from cirtorch.models.GF_net import make_net
    from cirtorch.models.init import random_init_

    net = make_net(args.arch, precision=args.precision, mean=[0.485, 0.456, 0.406], std=[0.229, 0.224, 0.225])
    random_init_(net, seed=0)
    net = net.cuda().eval()
    x = torch.rand(args.batch, 3, args.height, args.width, device="cuda")
    marker = torch.zeros(64, device="cuda")
    with torch.no_grad():
        for _ in range(2):
            net.body(x, normalize=net._normalizer())
        torch.cuda.synchronize()
        _ops.l2n_rows(marker.view(1, 64))          # marker: body dispatches follow
        for _ in range(args.iters):
            net.body(x, normalize=net._normalizer())
        _ops.l2n_rows(marker.view(1, 64))          # marker: end
        torch.cuda.synchronize()
    print("done", args.iters, "forwards of", args.arch, "B=%d" % args.batch)


if __name__ == "__main__":
    main()
