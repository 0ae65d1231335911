"""PMC workload: the lab copy of k_gemm8's schedule (tools/lab/libg8lab.so) in one diagnostic
mode on one shape, 12 launches, for rocprofv3 --pmc passes (tools/lab/g8lab_pmc.sh).
    python3 tools/lab/g8lab_pmc_work.py MODE P C K"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
import torch  # noqa: E402


def main():
    from cirtorch import _ops as ops
    mode, p, c, k = (int(v) for v in sys.argv[1:5])
    lab8 = ctypes.CDLL(os.path.join(HERE, "libg8lab.so"))
    lab8.lab_g8.restype = ctypes.c_int
    lab8.lab_g8.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int] * 4 + [ctypes.c_void_p]
    dt = torch.float16
    g = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.rand(1, 1, p, k, generator=g, device="cuda") * 2 - 1).to(dt)
    wt = (torch.rand(c, k, 1, 1, generator=g, device="cuda") * 2 - 1) / k ** 0.5
    wp = ops.pack_conv_weights(wt, k, dt, perm32=True)
    one, zero = torch.ones(c, device="cuda"), torch.zeros(c, device="cuda")
    y = torch.empty(p, c, dtype=dt, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(12):
        rc = lab8.lab_g8(x.data_ptr(), wp.data_ptr(), one.data_ptr(), zero.data_ptr(), y.data_ptr(), p, c, k, mode, st)
        assert rc == 0, rc
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
