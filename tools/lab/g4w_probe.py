"""LAB driver: the 4-wave 256x256 GEMM prototype (tools/lab/k_gemm4w.hip -> tools/lab/libg4w.so)
against k_gemm8 (through a PERM32 1x1 conv) and torch.matmul (hipBLASLt) on the same operands:
bit-identity with k_gemm8, then TF/s of each (HIP events).  Developer tool, not a test.

    python3 tools/lab/g4w_probe.py            (env VARIANTS=0,1  SHAPES=PxCxK,...  G8=<RR_TUNE_GEMM8>)
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    from cirtorch import _ops as ops
    from cirtorch import _engine as E
    lab = ctypes.CDLL(os.path.join(HERE, "libg4w.so"))
    lab.lab_gemm4w.restype = ctypes.c_int
    lab.lab_gemm4w.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int] * 3 + [ctypes.c_float, ctypes.c_int,
                                                                          ctypes.c_void_p]
    g8modes = [int(v) for v in os.environ.get("G8MODES", "").split(",") if v]
    if g8modes:
        lab8 = ctypes.CDLL(os.path.join(HERE, "libg8lab.so"))
        lab8.lab_g8.restype = ctypes.c_int
        lab8.lab_g8.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int] * 4 + [ctypes.c_void_p]
    if os.environ.get("G8"):
        E.check(E.lib().rr_set_tuning(8, int(os.environ["G8"])), "rr_set_tuning")
    variants = [int(v) for v in os.environ.get("VARIANTS", "0").split(",") if v]
    shapes = ((16384, 4096, 2048), (8192, 8192, 8192), (131072, 1024, 2048), (393216, 256, 1024),
              (100352, 2048, 512))
    if os.environ.get("SHAPES"):
        shapes = [tuple(int(v) for v in s.split("x")) for s in os.environ["SHAPES"].split(",")]
    dt = torch.float16
    g = torch.Generator(device="cuda").manual_seed(1)
    for (p, c, k) in shapes:
        x = (torch.rand(1, 1, p, k, generator=g, device="cuda") * 2 - 1).to(dt)
        wt = (torch.rand(c, k, 1, 1, generator=g, device="cuda") * 2 - 1) / k ** 0.5
        wp = ops.pack_conv_weights(wt, k, dt, perm32=True)
        one, zero = torch.ones(c, device="cuda"), torch.zeros(c, device="cuda")
        f8 = lambda: ops.conv2d_fused(x, wp, 1, 1, 1, 0, c, one, zero, leaky=False, perm32=True)  # noqa: E731
        y8 = f8()
        a, b = x.view(p, k), wt.view(c, k).to(dt).t()
        fl = 2.0 * p * c * k
        line = "P=%d C=%d K=%d: k_gemm8 %.1f" % (p, c, k, fl / timed(f8) / 1e12)
        line += " hipBLASLt %.1f" % (fl / timed(lambda: torch.matmul(a, b)) / 1e12)
        st = torch.cuda.current_stream().cuda_stream
        for v in variants:
            y4 = torch.empty_like(y8)

            def f4():
                rc = lab.lab_gemm4w(x.data_ptr(), wp.data_ptr(), one.data_ptr(), zero.data_ptr(), y4.data_ptr(),
                                    p, c, k, 1.0, v, st)
                assert rc == 0, rc
            f4()
            torch.cuda.synchronize()
            same = torch.equal(y4.view(torch.int16), y8.view(torch.int16))
            err = (y4.float() - y8.float()).abs().max().item()
            line += " | v%d %.1f TF/s %s(maxdiff %.3g)" % (v, fl / timed(f4) / 1e12, "bit-identical " if same else "DIFFERS ",
                                                       err)
        for md in g8modes:
            y4 = torch.empty_like(y8)

            def f8l():
                rc = lab8.lab_g8(x.data_ptr(), wp.data_ptr(), one.data_ptr(), zero.data_ptr(), y4.data_ptr(), p, c, k, md, st)
                assert rc == 0, rc
            f8l()
            torch.cuda.synchronize()
            same = torch.equal(y4.view(torch.int16), y8.view(torch.int16))
            line += " | g8lab m%d %.1f %s" % (md, fl / timed(f8l) / 1e12, "bit-identical" if same else "differs")
        print(line + " TF/s", flush=True)
        del x, wp, a, b, y8


if __name__ == "__main__":
    main()
