// DRAM-locality probe for the Q <= 128 kNN score GEMM (developer tool, not product).
// Reads a 1M x 2048 bf16 database (4.1 GB) in k_gemm8s's access pattern and in two
// alternatives, with the same per-wave bytes in flight, and prints GB/s for each:
//   kstep : row-major DB, a K-step reads 128 B from each of a 256-row tile's rows
//           (lane (r16, kq) of wave w: row 32 w + 16 g + r16, bytes kq*16 + 64 hs)
//   kmajor: the same fragments from a K-step-major copy ([tile][K-step][256 x 128 B])
//   rows  : row-major DB, each wave streams whole 4 KiB rows (contiguous)
// hipcc --offload-arch=gfx950 -O3 -o tools/dram_locality_probe tools/dram_locality_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int ROWS = 1 << 20, KP = 2048, ESZ = 2, NK = KP / 64, R = 8;
constexpr long long ROWB = (long long)KP * ESZ;  // 4 KiB

// mode 0: kstep, 1: kmajor, 2: rows.  Persistent over XCD-contiguous tile ranges.
template <int MODE>
__global__ void __launch_bounds__(512, 1) probe(const char* __restrict__ db, unsigned* out, int ntiles) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nwg = gridDim.x, bx = blockIdx.x, xcd = bx & 7;
    const int nt8 = ntiles >> 3, rt8 = ntiles & 7;
    const int s_x = xcd < rt8 ? xcd * (nt8 + 1) : rt8 * (nt8 + 1) + (xcd - rt8) * nt8;
    const int n_x = nt8 + (xcd < rt8 ? 1 : 0);
    const int nb_x = (nwg >> 3) + (xcd < (nwg & 7) ? 1 : 0);
    const int li = bx >> 3;
    const int r16 = lane & 15, kq = lane >> 4;
    uint4 x = {0u, 0u, 0u, 0u};
    for (int t = s_x + li; t < s_x + n_x; t += nb_x) {
        const char* tile = db + (long long)t * 256 * ROWB;
        for (int k0 = 0; k0 < NK; k0 += R) {
            uint4 v[R][2][2];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int ki = min(k0 + u, NK - 1);
#pragma unroll
                for (int g = 0; g < 2; ++g)
#pragma unroll
                    for (int hs = 0; hs < 2; ++hs) {
                        const int row = 32 * wave + 16 * g + r16;
                        long long off;
                        if (MODE == 0) off = (long long)row * ROWB + ki * 128 + kq * 16 + hs * 64;
                        else if (MODE == 1) off = (long long)ki * 32768 + row * 128 + kq * 16 + hs * 64;
                        else {  // wave streams its 32 rows; the 4 x 16 B pieces of a lane are 1 KiB apart
                            const int q = ki * 4 + g * 2 + hs;  // 0..127 pieces of 1 KiB per wave
                            off = (long long)(32 * wave + (q >> 2)) * ROWB + (q & 3) * 1024 + lane * 16;
                        }
                        v[u][g][hs] = *reinterpret_cast<const uint4*>(tile + off);
                    }
            }
#pragma unroll
            for (int u = 0; u < R; ++u)
#pragma unroll
                for (int g = 0; g < 2; ++g)
#pragma unroll
                    for (int hs = 0; hs < 2; ++hs) {
                        if (k0 + u >= NK) continue;
                        x.x ^= v[u][g][hs].x; x.y ^= v[u][g][hs].y; x.z ^= v[u][g][hs].z; x.w ^= v[u][g][hs].w;
                    }
        }
    }
    out[(long long)bx * 512 + tid] = x.x ^ x.y ^ x.z ^ x.w;
}

int main() {
    const long long bytes = (long long)ROWS * ROWB;
    const int ntiles = ROWS / 256, grid = 256;
    char* db;
    unsigned* out;
    CK(hipMalloc(&db, bytes));
    CK(hipMalloc(&out, (size_t)grid * 512 * 4));
    CK(hipMemset(db, 1, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[3] = {"kstep", "kmajor", "rows"};
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 3; ++mode) {
            auto launch = [&]() {
                if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(512), 0, 0, db, out, ntiles);
                else if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(512), 0, 0, db, out, ntiles);
                else hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(512), 0, 0, db, out, ntiles);
            };
            launch();
            CK(hipDeviceSynchronize());
            const int n = 10;
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < n; ++i) launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("{\"pattern\": \"%s\", \"rep\": %d, \"ms\": %.4f, \"gbs\": %.1f}\n", names[mode], rep, ms / n,
                   bytes / (ms / n * 1e-3) / 1e9);
            fflush(stdout);
        }
    CK(hipFree(db));
    CK(hipFree(out));
    return 0;
}
