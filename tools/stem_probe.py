"""Run the fused stem (rr_stem_conv_pool) repeatedly on a 32 x 3 x 768 x 1024
batch, for rocprofv3 counter passes.  Developer tool."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune", default="", help="rr_set_tuning pairs key=value[,key=value]")
    ap.add_argument("--u8", action="store_true", help="uint8 pixels (rr_stem_conv_pool_u8)")
    args = ap.parse_args()
    from cirtorch import _ops
    from cirtorch import _engine as E
    for kv in filter(None, args.tune.split(",")):
        k_, v_ = kv.split("=")
        E.check(E.lib().rr_set_tuning(int(k_), int(v_)), "rr_set_tuning")
    x = torch.rand(32, 3, 768, 1024, device="cuda")
    if args.u8:
        x = (x * 255).to(torch.uint8)
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    wp = _ops.pack_stem_weights(w)
    sc, sh = torch.rand(64, device="cuda") + 0.5, torch.randn(64, device="cuda") * 0.1
    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    for _ in range(3):
        _ops.stem_conv_pool(x, wp, sc, sh, mean=mean, std=std)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        _ops.stem_conv_pool(x, wp, sc, sh, mean=mean, std=std)
    b.record()
    torch.cuda.synchronize()
    print("stem %s %s: %.1f us/launch (32 images)" % (args.tune, "u8" if args.u8 else "f32", a.elapsed_time(b) * 100))


if __name__ == "__main__":
    main()
