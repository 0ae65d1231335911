// Range-check probe (developer tool): does a raw-buffer 8-B load that straddles
// num_records return its in-range dword, or 0 for the whole access?
//   hipcc --offload-arch=gfx950 -O3 tools/oob_probe.hip -o /tmp/oob_probe && /tmp/oob_probe
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* in, unsigned* out) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, 12, 0x00020000);
    const int offs[4] = {0, 4, 8, 12};
    for (int i = 0; i < 4; ++i) {
        const uint2 v = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, offs[i], 0, 0));
        out[2 * i] = v.x;
        out[2 * i + 1] = v.y;
    }
}
int main() {
    float h[8] = {1, 2, 3, 4, 5, 6, 7, 8};
    float* d; unsigned* o; unsigned r[8];
    hipMalloc(&d, sizeof h); hipMalloc(&o, sizeof r);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    k<<<1, 1>>>(d, o);
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    for (int i = 0; i < 4; ++i) printf("offset %2d: %g %g\n", 4 * i, *(float*)&r[2 * i], *(float*)&r[2 * i + 1]);
    return 0;
}
