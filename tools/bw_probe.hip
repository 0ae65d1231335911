// HBM bandwidth probe for the access shapes of the 1x1-conv kernels.
// Developer tool (not part of librr.so):
//   hipcc --offload-arch=gfx950 -O3 tools/bw_probe.hip -o /tmp/bw_probe && /tmp/bw_probe
// Shapes (bf16 NHWC rows of C channels):
//   line  : a wave-instruction reads/writes 1 KiB of consecutive bytes (full 128-B lines)
//   frag  : a wave-instruction covers 16 rows x 64 B (the MFMA B-fragment shape:
//           lane (r16, kq) -> row r16, bytes 16*kq .. of a 64-B half line)
// Each variant: read R bytes and write W bytes per "pixel" in the ratio of a layer.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// full-line copy-like stream: each thread moves 16 B; rin/wout bytes per row
__global__ void k_line(const uint4* __restrict__ in, uint4* __restrict__ out, long long nin, long long nout) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long stride = (long long)gridDim.x * blockDim.x;
    long long n = nin > nout ? nin : nout;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (; i < n; i += stride) {
        uint4 v = i < nin ? in[i] : acc;
        acc.x ^= v.x;
        if (i < nout) out[i] = v;
    }
    if (acc.x == 0x12345678u) out[0] = acc;
}

// fragment-shaped: row = 128 B (64 bf16 ch); a wave handles 16 rows per step:
// lane (r16 = lane & 15, kq = lane >> 4) loads 16 B at row r16, byte 16*kq (+64 for the 2nd half)
__global__ void k_frag(const uint4* __restrict__ in, uint4* __restrict__ out, long long rows_in, int wmul) {
    const int lane = threadIdx.x & 63;
    const int r16 = lane & 15, kq = lane >> 4;
    long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    for (long long s = wave; s * 16 < rows_in; s += nw) {
        long long row = s * 16 + r16;
        const uint4* src = in + row * 8;       // 8 x 16 B per row
        uint4 a = src[kq], b = src[4 + kq];
        // write wmul x the row bytes in the same fragment shape
        for (int m = 0; m < wmul; ++m) {
            uint4* dst = out + (row * wmul + m) * 8;
            dst[kq] = a;
            dst[4 + kq] = b;
        }
    }
}

int main() {
    const long long rows = 1572864LL * 32 / 32;  // pixels (mod2 at B=32)
    const long long bytes_row = 128;             // 64 bf16 channels
    const int wmul = 4;                          // 64 -> 256 channels
    size_t in_b = rows * bytes_row, out_b = rows * bytes_row * wmul;
    void *in, *out;
    CK(hipMalloc(&in, in_b));
    CK(hipMalloc(&out, out_b));
    CK(hipMemset(in, 1, in_b));
    CK(hipMemset(out, 0, out_b));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch, double bytes) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        const int reps = 20;
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-40s %8.1f us  %6.2f TB/s\n", name, ms * 1e3 / reps, bytes / (ms * 1e-3 / reps) / 1e12);
        return 0;
    };
    const int blocks = 256 * 8;
    long long nin = in_b / 16, nout = out_b / 16;
    run("line: read only (201 MB)", [&] { hipLaunchKernelGGL(k_line, dim3(blocks), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, nin, 0ll); }, (double)in_b);
    run("line: write only (805 MB)", [&] { hipLaunchKernelGGL(k_line, dim3(blocks), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, 0ll, nout); }, (double)out_b);
    run("line: read 201 MB + write 805 MB", [&] { hipLaunchKernelGGL(k_line, dim3(blocks), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, nin, nout); }, (double)(in_b + out_b));
    run("line: copy 805 MB (read=write)", [&] { hipLaunchKernelGGL(k_line, dim3(blocks), dim3(256), 0, 0, (const uint4*)out, (uint4*)in, nout / 4, nout / 4); }, (double)(in_b * 2));
    run("frag: read 201 MB + write 805 MB", [&] { hipLaunchKernelGGL(k_frag, dim3(blocks), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, rows, wmul); }, (double)(in_b + out_b));
    for (int nb : {64, 128, 256}) {
        for (int thr : {256, 1024}) {
            char nm[96];
            snprintf(nm, sizeof nm, "line: read 201+write 805, %d blocks x %d", nb, thr);
            run(nm, [&] { hipLaunchKernelGGL(k_line, dim3(nb), dim3(thr), 0, 0, (const uint4*)in, (uint4*)out, nin, nout); }, (double)(in_b + out_b));
            snprintf(nm, sizeof nm, "line: read only 805, %d blocks x %d", nb, thr);
            run(nm, [&] { hipLaunchKernelGGL(k_line, dim3(nb), dim3(thr), 0, 0, (const uint4*)out, (uint4*)in, nout, 0ll); }, (double)out_b);
        }
    }
    run("frag: read 201 MB + write 201 MB", [&] { hipLaunchKernelGGL(k_frag, dim3(blocks), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, rows, 1); }, (double)(2 * in_b));
    return 0;
}
