"""PMC workload: the 8-phase GEMM (k_gemm8, 1x1 conv, fp16) on one shape, ITERS launches, for
rocprofv3 --pmc passes (tools/g8_pmc.sh).  Developer tool."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    from cirtorch import _ops as ops
    p, c, k = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (4096, 4096, 4096)))
    dt = torch.float16
    g = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.rand(1, 1, p, k, generator=g, device="cuda") * 2 - 1).to(dt)
    wt = (torch.rand(c, k, 1, 1, generator=g, device="cuda") * 2 - 1) / k ** 0.5
    wp = ops.pack_conv_weights(wt, k, dt, perm32=True)
    one, zero = torch.ones(c, device="cuda"), torch.zeros(c, device="cuda")
    for _ in range(12):
        ops.conv2d_fused(x, wp, 1, 1, 1, 0, c, one, zero, leaky=False, perm32=True)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
