// librr.so — descriptor head: global pooling (GeM / MAC / SPoC), L2N, the
// whitening Linear, and the fused globalHead tail.  All HBM-/L2-bound:
// coalesced 8-16 B loads, f32 accumulation, wave shuffles + LDS partials.
//
// Reference: cirtorch/modules/pools.py:10-38 (MAC, SPoC, GeM),
// cirtorch/modules/normalizations.py:9-16 (L2N),
// cirtorch/modules/heads/global_head.py:52-67 (pool -> L2N -> Linear -> L2N).
#include "rr_internal.h"

namespace rr {

// GeM power: exact repeated product for the common integer p (the reference
// evaluates torch.pow with a tensor exponent; for p = 3 both are the cube).
__device__ __forceinline__ float powp(float x, float p, int ip) {
    if (ip == 3) return x * x * x;
    if (ip == 2) return x * x;
    if (ip == 1) return x;
    return __powf(x, p);
}

// NHWC: [n][hw][c].  Block = 256 threads = 4 waves; each lane owns 4 channels
// (one 16-B f32 / 8-B bf16 load per pixel), each wave a quarter of the pixels;
// the 4 partial sums are combined through LDS.  grid = (ceil(c/256), n).
template <typename T>
__global__ void __launch_bounds__(256) k_pool_nhwc(const T* __restrict__ x, int c, int hw, int mode, float p,
                                                   int ip, float eps, float* __restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ch = blockIdx.x * 256 + lane * 4;
    const long long img = blockIdx.y;
    __shared__ float part[4][256];
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (mode == RR_POOL_MAC) acc[0] = acc[1] = acc[2] = acc[3] = -INFINITY;
    if (ch < c) {
        const T* base = x + img * hw * c + ch;
        for (int i = wave; i < hw; i += 4) {
            float v[4];
            const T* q = base + (long long)i * c;
            if constexpr (sizeof(T) == 4) {
                float4 t = *reinterpret_cast<const float4*>(q);
                v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
            } else {
                ushort4 t = *reinterpret_cast<const ushort4*>(q);
                v[0] = bf2f(t.x); v[1] = bf2f(t.y); v[2] = bf2f(t.z); v[3] = bf2f(t.w);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (mode == RR_POOL_GEM) acc[r] += powp(fmaxf(v[r], eps), p, ip);
                else if (mode == RR_POOL_MAC) acc[r] = fmaxf(acc[r], v[r]);
                else acc[r] += v[r];
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) part[wave][lane * 4 + r] = acc[r];
    __syncthreads();
    if (wave == 0 && ch < c) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int j = lane * 4 + r;
            float v;
            if (mode == RR_POOL_MAC) {
                v = fmaxf(fmaxf(part[0][j], part[1][j]), fmaxf(part[2][j], part[3][j]));
            } else {
                v = ((part[0][j] + part[1][j]) + (part[2][j] + part[3][j])) / (float)hw;
                if (mode == RR_POOL_GEM) v = __powf(v, 1.0f / p);
            }
            out[img * c + ch + r] = v;
        }
    }
}

// NCHW: one wave per (image, channel) plane of hw contiguous values.
template <typename T>
__global__ void __launch_bounds__(256) k_pool_nchw(const T* __restrict__ x, long long planes, int hw, int mode,
                                                   float p, int ip, float eps, float* __restrict__ out) {
    const long long plane = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (plane >= planes) return;
    const T* base = x + plane * hw;
    float acc = mode == RR_POOL_MAC ? -INFINITY : 0.f;
    for (int i = lane; i < hw; i += 64) {
        float v = DT<T>::to_f(base[i]);
        if (mode == RR_POOL_GEM) acc += powp(fmaxf(v, eps), p, ip);
        else if (mode == RR_POOL_MAC) acc = fmaxf(acc, v);
        else acc += v;
    }
    acc = mode == RR_POOL_MAC ? wave_max(acc) : wave_sum(acc);
    if (lane == 0) {
        float v = acc;
        if (mode != RR_POOL_MAC) {
            v = v / (float)hw;
            if (mode == RR_POOL_GEM) v = __powf(v, 1.0f / p);
        }
        out[plane] = v;
    }
}

// Row L2N: one 256-thread block per row.
__global__ void __launch_bounds__(256) k_l2n_rows(const float* __restrict__ x, int dim, float eps,
                                                  float* __restrict__ y) {
    const long long row = blockIdx.x;
    const float* xr = x + row * dim;
    __shared__ float red[4];
    float ss = 0.f;
    for (int i = threadIdx.x; i < dim; i += 256) ss += xr[i] * xr[i];
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    const float nrm = sqrtf((red[0] + red[1]) + (red[2] + red[3])) + eps;
    for (int i = threadIdx.x; i < dim; i += 256) y[row * dim + i] = xr[i] / nrm;
}

// Dense layer, one wave per output o: the wave keeps W[o][:] in registers
// (float4 chunks lane, lane+64, ...) and streams every input row through it.
// in_dim % 4 == 0, in_dim <= 4096.
constexpr int LIN_MAXV = 16;  // float4 per lane -> in_dim <= 64*4*16 = 4096
__global__ void __launch_bounds__(256) k_linear_rows(const float* __restrict__ x, int rows, int in_dim,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     int out_dim, float* __restrict__ y) {
    const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (o >= out_dim) return;
    const int n4 = in_dim / 4;
    float4 wr[LIN_MAXV];
    const float4* wrow = reinterpret_cast<const float4*>(w + (long long)o * in_dim);
#pragma unroll
    for (int t = 0; t < LIN_MAXV; ++t) {
        const int j = lane + 64 * t;
        wr[t] = j < n4 ? wrow[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float bias = b ? b[o] : 0.f;
    for (int r = 0; r < rows; ++r) {
        const float4* xr = reinterpret_cast<const float4*>(x + (long long)r * in_dim);
        float s = 0.f;
#pragma unroll
        for (int t = 0; t < LIN_MAXV; ++t) {
            const int j = lane + 64 * t;
            if (j < n4) {
                float4 v = xr[j];
                s += wr[t].x * v.x + wr[t].y * v.y + wr[t].z * v.z + wr[t].w * v.w;
            }
        }
        s = wave_sum(s);
        if (lane == 0) y[(long long)r * out_dim + o] = s + bias;
    }
}

}  // namespace rr

using namespace rr;

extern "C" {

int rr_global_pool(const void* x, int n, int c, int hw, int layout, int mode, float p, float eps, float* out,
                   int dtype, void* stream) {
    if (n <= 0 || c <= 0 || hw <= 0) return fail(RR_EINVAL, "rr_global_pool: empty input");
    if (mode < 0 || mode > 2) return fail(RR_EINVAL, "rr_global_pool: mode");
    if (mode == RR_POOL_GEM && !(p > 0.f)) return fail(RR_EINVAL, "rr_global_pool: GeM p must be > 0");
    int ip = (p == 3.f) ? 3 : (p == 2.f) ? 2 : (p == 1.f) ? 1 : 0;
    hipStream_t s = as_stream(stream);
    if (layout == RR_NHWC) {
        if (c % 4) return fail(RR_EINVAL, "rr_global_pool: NHWC needs c % 4 == 0");
        dim3 grid((c + 255) / 256, n);
        if (dtype == RR_BF16)
            hipLaunchKernelGGL(k_pool_nhwc<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, c, hw, mode, p, ip, eps, out);
        else if (dtype == RR_F32)
            hipLaunchKernelGGL(k_pool_nhwc<float>, grid, dim3(256), 0, s, (const float*)x, c, hw, mode, p, ip, eps, out);
        else
            return fail(RR_EINVAL, "rr_global_pool: dtype");
    } else if (layout == RR_NCHW) {
        long long planes = (long long)n * c;
        dim3 grid((unsigned)((planes + 3) / 4));
        if (dtype == RR_BF16)
            hipLaunchKernelGGL(k_pool_nchw<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, planes, hw, mode, p, ip, eps, out);
        else if (dtype == RR_F32)
            hipLaunchKernelGGL(k_pool_nchw<float>, grid, dim3(256), 0, s, (const float*)x, planes, hw, mode, p, ip, eps, out);
        else
            return fail(RR_EINVAL, "rr_global_pool: dtype");
    } else {
        return fail(RR_EINVAL, "rr_global_pool: layout");
    }
    return check_launch("rr_global_pool");
}

int rr_l2n_rows(const float* x, int rows, int dim, float eps, float* y, void* stream) {
    if (rows <= 0 || dim <= 0) return fail(RR_EINVAL, "rr_l2n_rows: empty");
    hipLaunchKernelGGL(k_l2n_rows, dim3(rows), dim3(256), 0, as_stream(stream), x, dim, eps, y);
    return check_launch("rr_l2n_rows");
}

int rr_linear_rows(const float* x, int rows, int in_dim, const float* w, const float* b, int out_dim, float* y,
                   void* stream) {
    if (rows <= 0 || out_dim <= 0) return fail(RR_EINVAL, "rr_linear_rows: empty");
    if (in_dim % 4 || in_dim <= 0 || in_dim > 64 * 4 * LIN_MAXV)
        return fail(RR_EINVAL, "rr_linear_rows: in_dim must be a multiple of 4, <= 4096");
    hipLaunchKernelGGL(k_linear_rows, dim3((out_dim + 3) / 4), dim3(256), 0, as_stream(stream), x, rows, in_dim, w, b,
                       out_dim, y);
    return check_launch("rr_linear_rows");
}

size_t rr_head_workspace_bytes(int rows, int dim) { return (size_t)2 * rows * dim * sizeof(float); }

int rr_head_l2n_whiten_l2n(const float* x, int rows, int dim, const float* w, const float* b, int whiten, float eps,
                           float* y, void* workspace, void* stream) {
    if (!whiten) return rr_l2n_rows(x, rows, dim, eps, y, stream);
    if (!workspace) return fail(RR_EINVAL, "rr_head_l2n_whiten_l2n: workspace required");
    float* t0 = (float*)workspace;
    float* t1 = t0 + (size_t)rows * dim;
    int rc = rr_l2n_rows(x, rows, dim, eps, t0, stream);
    if (rc) return rc;
    rc = rr_linear_rows(t0, rows, dim, w, b, dim, t1, stream);
    if (rc) return rc;
    return rr_l2n_rows(t1, rows, dim, eps, y, stream);
}

}  // extern "C"
