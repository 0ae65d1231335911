// Probe: does a hipMemsetAsync captured into a hipGraph replay in stream
// order before the kernel captured after it?  (the kNN's running
// threshold tau was reset with hipMemsetAsync and a captured search returned
// empty rows; the reset is now a kernel.)  Pure HIP, no torch.
//
//   hipcc --offload-arch=gfx950 -O2 tools/graph_memset_probe.hip -o tools/graph_memset_probe
//   ./tools/graph_memset_probe
//
// Each case: poison buf with 0xFFFFFFFF by a kernel OUTSIDE the graph, replay
// the graph {memset(buf, 0) ; copy buf -> out ; mark kernel}, check out == 0.
// Cases vary the byte count (24 B = the 6-query tau of a small search, 32 B,
// 4 KiB), the buffer offset inside a larger allocation (the tau slice of the
// kNN workspace), the capture mode and the stream flags.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(2); } } while (0)

__global__ void k_poison(unsigned* p, int n) { int i = blockIdx.x * blockDim.x + threadIdx.x; if (i < n) p[i] = 0xFFFFFFFFu; }
__global__ void k_copy(const unsigned* p, unsigned* o, int n) { int i = blockIdx.x * blockDim.x + threadIdx.x; if (i < n) o[i] = p[i]; }
__global__ void k_atomic_use(unsigned* p, int n, unsigned* o) {
    // like k_chunk_select: read tau, then raise it with atomicMax
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { o[i] = __atomic_load_n(p + i, __ATOMIC_RELAXED); atomicMax(p + i, 5u); }
}

static int run_case(int nwords, size_t offset_bytes, hipStreamCaptureMode mode, unsigned flags, bool d32, bool atomic_use,
                    int reps) {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, flags));
    char* base;
    CK(hipMalloc(&base, offset_bytes + nwords * 4 + 4096));
    unsigned* buf = (unsigned*)(base + offset_bytes);
    unsigned* out;
    CK(hipMalloc(&out, nwords * 4));
    hipGraph_t g;
    hipGraphExec_t ge;
    // warm (eager), like GraphedForward's warm-up calls
    hipLaunchKernelGGL(k_poison, dim3((nwords + 255) / 256), dim3(256), 0, s, buf, nwords);
    if (d32) CK(hipMemsetD32Async((hipDeviceptr_t)buf, 0, nwords, s));
    else CK(hipMemsetAsync(buf, 0, nwords * 4, s));
    CK(hipStreamSynchronize(s));
    CK(hipStreamBeginCapture(s, mode));
    if (d32) CK(hipMemsetD32Async((hipDeviceptr_t)buf, 0, nwords, s));
    else CK(hipMemsetAsync(buf, 0, nwords * 4, s));
    if (atomic_use) hipLaunchKernelGGL(k_atomic_use, dim3((nwords + 255) / 256), dim3(256), 0, s, buf, nwords, out);
    else hipLaunchKernelGGL(k_copy, dim3((nwords + 255) / 256), dim3(256), 0, s, buf, out, nwords);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    std::vector<unsigned> h(nwords);
    int bad_reps = 0;
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_poison, dim3((nwords + 255) / 256), dim3(256), 0, s, buf, nwords);
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), out, nwords * 4, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < nwords; ++i) bad += h[i] != 0u;
        bad_reps += bad != 0;
    }
    printf("words=%5d offset=%6zu mode=%d flags=%u %s %s nodes=%zu : %d / %d replays saw a non-zero word\n", nwords,
           offset_bytes, (int)mode, flags, d32 ? "memsetD32" : "memset   ", atomic_use ? "atomic" : "copy  ", nn,
           bad_reps, reps);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipFree(base));
    CK(hipFree(out));
    CK(hipStreamDestroy(s));
    return bad_reps;
}

int main() {
    int total = 0;
    const int words[] = {6, 8, 1024};
    const size_t offs[] = {0, 256, 1048576 + 768};
    const hipStreamCaptureMode modes[] = {hipStreamCaptureModeGlobal, hipStreamCaptureModeThreadLocal,
                                          hipStreamCaptureModeRelaxed};
    for (int w : words)
        for (size_t o : offs)
            for (auto m : modes)
                for (unsigned f : {0u, (unsigned)hipStreamNonBlocking})
                    for (int d32 = 0; d32 < 2; ++d32)
                        for (int at = 0; at < 2; ++at) total += run_case(w, o, m, f, d32, at, 20);
    printf("TOTAL bad cases: %d\n", total);
    return 0;
}
