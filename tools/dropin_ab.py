"""extract_vectors on 128 same-size 1024x768 JPEGs, warm call then 3 timed calls
(developer A/B of the drop-in scheduling knobs, RR_EV_* env).  python tools/dropin_ab.py"""
import json
import os
import shutil
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from PIL import Image
    from cirtorch.models import GF_net as G
    from cirtorch.models.init import random_init_
    H, W, n = 768, 1024, 128
    net = G.make_net("resnet50", precision="bf16", mean=[0.485, 0.456, 0.406], std=[0.229, 0.224, 0.225])
    random_init_(net, seed=0)
    net = net.cuda().eval()
    d = tempfile.mkdtemp(prefix="rr_dab_")
    try:
        r = np.random.default_rng(3)
        paths = []
        for i in range(16):
            field = r.random((6, 8, 3))
            up = np.kron(field, np.ones((H // 6 + 1, W // 8 + 1, 1)))[:H, :W]
            arr = (np.clip(0.8 * up + 0.2 * r.random((H, W, 3)), 0, 1) * 255).astype(np.uint8)
            p = os.path.join(d, "im%02d.jpg" % i)
            Image.fromarray(arr).save(p, quality=90)
            paths.append(p)
        ps = [paths[i % 16] for i in range(n)]
        G.extract_vectors(net, ps, None)
        rates = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            G.extract_vectors(net, ps, None)
            rates.append(n / (time.perf_counter() - t0))
        env = {k: v for k, v in os.environ.items() if k.startswith("RR_EV_") or k == "RR_DECODE_PROCS"}
        print(json.dumps({"env": env, "jpg_img_s": [round(x, 1) for x in rates]}), flush=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
