// librr.so — local-descriptor head:
//   desc = normalize(Linear(grid_sample(x, kpts)))
// Replaces cirtorch/modules/heads/local_head.py:43-71 (localHead.forward):
//   functional.grid_sample(x, kpts.unsqueeze(2), mode="bilinear",
//                          padding_mode="zeros")         (align_corners=False)
//   -> permute -> nn.Linear(dim, E) -> functional.normalize(dim=2)
// and the mutual-nearest-neighbour check of the HPatches matcher
// (cirtorch/utils/evaluation/HPatchesEval.py:31-43) on top of rr_knn_topk.
//
// Layout: feature map NHWC (any of the extractor's stage maps, bf16/fp16/f32),
// keypoints [n][npts][2] float32 in grid_sample's normalised (x, y) in [-1, 1].
// Sampling: one wave per keypoint, lanes over channels (16-B loads of 8 bf16 /
// 4 f32 channels), the four bilinear taps in torch's order (nw, ne, sw, se),
// zero padding per tap.  Linear on the exact-f32 MFMA (rr_linear_rows), then
// x / max(||x||_2, 1e-12) per descriptor.
#include "rr_internal.h"

namespace rr {

namespace {

template <typename T> struct LVec;
template <> struct LVec<bf16_t> {
    static constexpr int N = 8;
    static __device__ __forceinline__ void load(const bf16_t* p, float* v) {
        const uint4 q = *reinterpret_cast<const uint4*>(p);
        const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            v[2 * e] = __uint_as_float(w[e] << 16);
            v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
        }
    }
};
template <> struct LVec<f16_t> {
    static constexpr int N = 8;
    static __device__ __forceinline__ void load(const f16_t* p, float* v) {
        typedef __attribute__((ext_vector_type(8))) _Float16 h8;
        const h8 q = *reinterpret_cast<const h8*>(p);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (float)q[e];
    }
};
template <> struct LVec<float> {
    static constexpr int N = 4;
    static __device__ __forceinline__ void load(const float* p, float* v) {
        const float4 q = *reinterpret_cast<const float4*>(p);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    }
};

// out[kp][c] = bilinear sample of x[img][:, :, c] at keypoint kp (grid_sample, zeros, align_corners=False)
template <typename T>
__global__ void __launch_bounds__(256) k_grid_sample_nhwc(const T* __restrict__ x, int h, int w, int c,
                                                          const float* __restrict__ kpts, int npts, long long nkp,
                                                          float* __restrict__ out) {
    constexpr int V = LVec<T>::N;
    const long long kp = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (kp >= nkp) return;
    const long long img = kp / npts;
    const float gx = kpts[kp * 2], gy = kpts[kp * 2 + 1];
    // grid_sampler_unnormalize(align_corners=False): ((g + 1) * size - 1) / 2
    const float ix = ((gx + 1.f) * w - 1.f) / 2.f;
    const float iy = ((gy + 1.f) * h - 1.f) / 2.f;
    const float fx = floorf(ix), fy = floorf(iy);
    const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
    const float wnw = ((float)x1 - ix) * ((float)y1 - iy);
    const float wne = (ix - (float)x0) * ((float)y1 - iy);
    const float wsw = ((float)x1 - ix) * (iy - (float)y0);
    const float wse = (ix - (float)x0) * (iy - (float)y0);
    const bool in_nw = x0 >= 0 && x0 < w && y0 >= 0 && y0 < h;
    const bool in_ne = x1 >= 0 && x1 < w && y0 >= 0 && y0 < h;
    const bool in_sw = x0 >= 0 && x0 < w && y1 >= 0 && y1 < h;
    const bool in_se = x1 >= 0 && x1 < w && y1 >= 0 && y1 < h;
    const T* base = x + img * h * w * c;
    float* o = out + kp * c;
    for (int c0 = lane * V; c0 < c; c0 += 64 * V) {
        float acc[V];
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] = 0.f;
        float v[V];
        if (in_nw) {
            LVec<T>::load(base + ((long long)y0 * w + x0) * c + c0, v);
#pragma unroll
            for (int e = 0; e < V; ++e) acc[e] += v[e] * wnw;
        }
        if (in_ne) {
            LVec<T>::load(base + ((long long)y0 * w + x1) * c + c0, v);
#pragma unroll
            for (int e = 0; e < V; ++e) acc[e] += v[e] * wne;
        }
        if (in_sw) {
            LVec<T>::load(base + ((long long)y1 * w + x0) * c + c0, v);
#pragma unroll
            for (int e = 0; e < V; ++e) acc[e] += v[e] * wsw;
        }
        if (in_se) {
            LVec<T>::load(base + ((long long)y1 * w + x1) * c + c0, v);
#pragma unroll
            for (int e = 0; e < V; ++e) acc[e] += v[e] * wse;
        }
#pragma unroll
        for (int e = 0; e < V; ++e) o[c0 + e] = acc[e];
    }
}

// y = x / max(||x||_2, eps) per row (torch.nn.functional.normalize), one wave per row
__global__ void __launch_bounds__(256) k_normalize_rows(const float* __restrict__ x, long long rows, int dim,
                                                        float eps, float* __restrict__ y) {
    const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    const float* xr = x + r * dim;
    float ss = 0.f;
    for (int i = lane; i < dim; i += 64) ss += xr[i] * xr[i];
    ss = wave_sum(ss);
    const float d = fmaxf(sqrtf(ss), eps);
    for (int i = lane; i < dim; i += 64) y[r * dim + i] = xr[i] / d;
}

// match[i] = nn12[i] if nn21[nn12[i]] == i else -1 (HPatchesEval.py:31-43)
__global__ void k_mutual(const long long* __restrict__ nn12, int n1, const long long* __restrict__ nn21, int n2,
                         long long* __restrict__ match) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n1) return;
    const long long j = nn12[i];
    match[i] = (j >= 0 && j < n2 && nn21[j] == i) ? j : -1;
}

}  // namespace

}  // namespace rr

using namespace rr;

extern "C" {

size_t rr_local_head_workspace_bytes(long long nkp, int c, int e) {
    return (size_t)nkp * ((size_t)c + (size_t)e) * sizeof(float) + 256;
}

int rr_local_head(const void* x, int n, int h, int w, int c, int dtype, const float* kpts, int npts,
                  const float* weight, const float* bias, int e, float* out, void* workspace,
                  size_t workspace_bytes, void* stream) {
    if (!x || !kpts || !weight || !out) return fail(RR_EINVAL, "rr_local_head: null pointer");
    if (n <= 0 || h <= 0 || w <= 0 || c <= 0 || npts <= 0 || e <= 0) return fail(RR_EINVAL, "rr_local_head: empty");
    const int vec = dtype == RR_F32 ? 4 : 8;
    if (dtype != RR_BF16 && dtype != RR_F16 && dtype != RR_F32) return fail(RR_EINVAL, "rr_local_head: dtype");
    if (c % vec || (((uintptr_t)x) & 15)) return fail(RR_EINVAL, "rr_local_head: c must fill 16-byte lanes");
    if (c % 4) return fail(RR_EINVAL, "rr_local_head: c % 4 != 0");
    const long long nkp = (long long)n * npts;
    if (!workspace || workspace_bytes < rr_local_head_workspace_bytes(nkp, c, e))
        return fail(RR_ENOSPACE, "rr_local_head: workspace too small");
    if (nkp > 0x7fffffffll) return fail(RR_EINVAL, "rr_local_head: too many keypoints");
    hipStream_t s = as_stream(stream);
    float* samp = (float*)workspace;
    float* lin = samp + nkp * c;
    const unsigned g = (unsigned)((nkp + 3) / 4);
    if (dtype == RR_BF16)
        hipLaunchKernelGGL(k_grid_sample_nhwc<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)x, h, w, c, kpts, npts,
                           nkp, samp);
    else if (dtype == RR_F16)
        hipLaunchKernelGGL(k_grid_sample_nhwc<f16_t>, dim3(g), dim3(256), 0, s, (const f16_t*)x, h, w, c, kpts, npts,
                           nkp, samp);
    else
        hipLaunchKernelGGL(k_grid_sample_nhwc<float>, dim3(g), dim3(256), 0, s, (const float*)x, h, w, c, kpts, npts,
                           nkp, samp);
    int rc = check_launch("rr_local_head: sample");
    if (rc) return rc;
    rc = rr_linear_rows(samp, (int)nkp, c, weight, bias, e, lin, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_normalize_rows, dim3(g), dim3(256), 0, s, lin, nkp, e, 1e-12f, out);
    return check_launch("rr_local_head: normalize");
}

int rr_mutual_nn(const long long* nn12, int n1, const long long* nn21, int n2, long long* match, void* stream) {
    if (!nn12 || !nn21 || !match || n1 < 0 || n2 < 0) return fail(RR_EINVAL, "rr_mutual_nn: bad arguments");
    if (n1 == 0) return RR_OK;
    hipLaunchKernelGGL(k_mutual, dim3((n1 + 255) / 256), dim3(256), 0, as_stream(stream), nn12, n1, nn21, n2, match);
    return check_launch("rr_mutual_nn");
}

}  // extern "C"
