"""PMC workload: torch.matmul (hipBLASLt) and k_gemm8 (through a PERM32 1x1 conv) on one fp16 shape,
12 launches each, for a GRBM_GUI_ACTIVE + kernel-trace pass (held clock per kernel: tools/body_clock.py).
    python3 tools/lab/blaslt_pmc_work.py P C K"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
import torch  # noqa: E402


def main():
    from cirtorch import _ops as ops
    p, c, k = (int(v) for v in sys.argv[1:4])
    dt = torch.float16
    g = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.rand(1, 1, p, k, generator=g, device="cuda") * 2 - 1).to(dt)
    wt = (torch.rand(c, k, 1, 1, generator=g, device="cuda") * 2 - 1) / k ** 0.5
    wp = ops.pack_conv_weights(wt, k, dt, perm32=True)
    one, zero = torch.ones(c, device="cuda"), torch.zeros(c, device="cuda")
    a, b = x.view(p, k), wt.view(c, k).to(dt).t()
    for _ in range(12):
        torch.matmul(a, b)
    for _ in range(12):
        ops.conv2d_fused(x, wp, 1, 1, 1, 0, c, one, zero, leaky=False, perm32=True)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
