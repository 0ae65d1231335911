"""Time bench.py's drop-in sub-benchmark (extract_vectors on PNG files and on
decoded pixels) alone.  Developer tool.   python tools/dropin_probe.py [reps]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    import bench
    from cirtorch.models.GF_net import make_net
    from cirtorch.models.init import random_init_
    dev = torch.device("cuda:0")
    net = make_net("resnet50", precision="bf16", mean=[0.485, 0.456, 0.406], std=[0.229, 0.224, 0.225])
    random_init_(net, seed=0)
    net = net.to(dev).eval()
    with torch.no_grad():
        for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
            r = bench.bench_dropin(net, 768, 1024, dev)
            print(json.dumps({k: v for k, v in r.items() if k != "note"}), flush=True)


if __name__ == "__main__":
    main()
