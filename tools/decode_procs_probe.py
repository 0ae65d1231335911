"""Process-decoder probe (developer tool): is the shared-memory ring page-locked
(registered, torch sees it pinned), how fast do 16 worker processes decode
1024x768 JPEGs into it, and how fast do the ring views copy to the GPU.
    python tools/decode_procs_probe.py"""
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
    from cirtorch.utils import decode_procs
    H, W, n = 768, 1024, 128
    d = tempfile.mkdtemp(prefix="rr_dprobe_")
    out = {}
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
        workers = G._default_workers()
        t0 = time.perf_counter()
        dec = decode_procs.get(workers, 2 * n + 8)
        out["startup_s"] = time.perf_counter() - t0
        out["registered"] = dec.registered
        for rep in range(2):
            t0 = time.perf_counter()
            pend = []
            for i in range(0, n, 4):
                pend += dec.submit_group([(p, None, None) for p in ps[i:i + 4]])
            views = [q.result() for q in pend]
            out["decode_img_s_%d" % rep] = n / (time.perf_counter() - t0)
            out["view_is_pinned"] = bool(views[0].is_pinned())
            xh = torch.empty((n,) + tuple(views[0].shape), dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for j, v in enumerate(views):
                xh[j].copy_(v, non_blocking=True)
            t_issue = time.perf_counter() - t0
            torch.cuda.synchronize()
            out["h2d_gbs_%d" % rep] = xh.numel() / (time.perf_counter() - t0) / 1e9
            out["h2d_issue_ms_%d" % rep] = t_issue * 1e3
            ev = torch.cuda.Event()
            ev.record()
            dec.release(views, ev)
        print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
