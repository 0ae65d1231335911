"""LAB: the clock the chip holds inside the lab copy of k_gemm8's schedule (tools/lab/k_g8lab.hip) per
diagnostic mode: wave 0 of every block stamps s_memtime (shader clock) and s_memrealtime (constant
100 MHz) before the prologue and after the K-loop; clock = d(memtime) / d(memrealtime) x 100 MHz,
beside the event-timed rate of the same launches.  Developer tool.
    python3 tools/lab/g8lab_clock.py   (env MODES=0,1,2,7  SHAPES=PxCxK,...)"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
import torch  # noqa: E402


def main():
    from cirtorch import _ops as ops
    lab8 = ctypes.CDLL(os.path.join(HERE, "libg8lab.so"))
    lab8.lab_g8s.restype = ctypes.c_int
    lab8.lab_g8s.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_void_p]
    modes = [int(v) for v in os.environ.get("MODES", "0,1,2,7").split(",") if v]
    lab4 = ctypes.CDLL(os.path.join(HERE, "libg4w.so"))
    lab4.lab_gemm4ws.restype = ctypes.c_int
    lab4.lab_gemm4ws.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int] * 3 + [ctypes.c_float, ctypes.c_int,
                                                                           ctypes.c_void_p, ctypes.c_void_p]
    # 4-wave variants with stamps (variant 1 family: 15 = one-state DMA issue, 11 = no DMA in the K-loop)
    variants = [int(v) for v in os.environ.get("VARIANTS", "").split(",") if v]
    shapes = [tuple(int(v) for v in s.split("x")) for s in
              os.environ.get("SHAPES", "16384x4096x2048,393216x256x1024").split(",")]
    dt = torch.float16
    g = torch.Generator(device="cuda").manual_seed(1)
    for (p, c, k) in shapes:
        x = (torch.rand(1, 1, p, k, generator=g, device="cuda") * 2 - 1).to(dt)
        wt = (torch.rand(c, k, 1, 1, generator=g, device="cuda") * 2 - 1) / k ** 0.5
        wp = ops.pack_conv_weights(wt, k, dt, perm32=True)
        one, zero = torch.ones(c, device="cuda"), torch.zeros(c, device="cuda")
        y = torch.empty(p, c, dtype=dt, device="cuda")
        ntiles = ((p + 255) // 256) * ((c + 255) // 256)
        st_buf = torch.zeros(ntiles * 4, dtype=torch.int64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        fl = 2.0 * p * c * k
        line = "P=%d C=%d K=%d:" % (p, c, k)
        for m in modes:
            def run(stamps):
                rc = lab8.lab_g8s(x.data_ptr(), wp.data_ptr(), one.data_ptr(), zero.data_ptr(), y.data_ptr(), p, c, k,
                                  m, st, stamps)
                assert rc == 0, rc
            for _ in range(3):
                run(None)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run(st_buf.data_ptr())
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 10 * 1e-3
            s = st_buf.view(ntiles, 4).cpu().double()
            dt_clk, dt_ref = s[:, 2] - s[:, 0], s[:, 3] - s[:, 1]
            ok = dt_ref > 0
            ghz = (dt_clk[ok] / dt_ref[ok] * 0.1).median().item()
            line += " | m%d %.1f TF/s, %.2f GHz" % (m, fl / t / 1e12, ghz)
        for v in variants:
            def run4(stamps):
                rc = lab4.lab_gemm4ws(x.data_ptr(), wp.data_ptr(), one.data_ptr(), zero.data_ptr(), y.data_ptr(), p, c,
                                      k, 1.0, v, st, stamps)
                assert rc == 0, rc
            for _ in range(3):
                run4(None)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run4(st_buf.data_ptr())
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 10 * 1e-3
            s = st_buf.view(ntiles, 4).cpu().double()
            dt_clk, dt_ref = s[:, 2] - s[:, 0], s[:, 3] - s[:, 1]
            ok = dt_ref > 0
            ghz = (dt_clk[ok] / dt_ref[ok] * 0.1).median().item()
            line += " | 4w-v%d %.1f TF/s, %.2f GHz" % (v, fl / t / 1e12, ghz)
        print(line, flush=True)
        del x, wp, y


if __name__ == "__main__":
    main()
