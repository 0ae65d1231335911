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

// NaN-propagating clamp / max, the semantics of torch.clamp(min=eps) and
// torch.max the reference pools use (pools.py:10-38): a NaN activation (an
// overflowed fp16 chain) must reach the descriptor, where extract_vectors sees
// it, instead of being replaced by eps (fmaxf drops a NaN operand).
__device__ __forceinline__ float clamp_min_nan(float v, float eps) { return v < eps ? eps : v; }
__device__ __forceinline__ float max_nan(float a, float b) { return (a > b || a != a) ? a : b; }

// The exponent of a GeM parameter living in device memory (a learnable
// ``pool.p``, pools.py:34) is read by the kernel itself: no host read-back, so
// any update of the parameter (load_state_dict, optimizer step, in-place
// ``p.data.fill_``) is seen by the next launch and a forward stays
// graph-capturable.  pdev == nullptr: the host value p is used.
__device__ __forceinline__ void gem_exponent(const float* pdev, float& p, int& ip) {
    if (pdev) {
        p = *pdev;
        ip = (p == 3.f) ? 3 : (p == 2.f) ? 2 : (p == 1.f) ? 1 : 0;
    }
}

// NHWC: [n][hw][c].  Block = 256 threads = 4 waves; each lane owns 4 channels
// (one 16-B f32 / 8-B bf16 load per pixel), each wave a quarter of the pixels;
// the 4 partial sums are combined through LDS.  grid = (ceil(c/256), n).
template <typename T>
__global__ void __launch_bounds__(256) k_pool_nhwc(const T* __restrict__ x, int c, int hw, int mode, float p,
                                                   int ip, const float* __restrict__ pdev, float eps,
                                                   float* __restrict__ out) {
    gem_exponent(pdev, p, ip);
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
            } else if constexpr (std::is_same<T, f16_t>::value) {
                typedef __attribute__((ext_vector_type(4))) _Float16 h4;
                const h4 t = *reinterpret_cast<const h4*>(q);
                v[0] = (float)t.x; v[1] = (float)t.y; v[2] = (float)t.z; v[3] = (float)t.w;
            } else {
                ushort4 t = *reinterpret_cast<const ushort4*>(q);
                v[0] = bf2f(t.x); v[1] = bf2f(t.y); v[2] = bf2f(t.z); v[3] = bf2f(t.w);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (mode == RR_POOL_GEM) acc[r] += powp(clamp_min_nan(v[r], eps), p, ip);
                else if (mode == RR_POOL_MAC) acc[r] = max_nan(acc[r], v[r]);
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
                v = max_nan(max_nan(part[0][j], part[1][j]), max_nan(part[2][j], part[3][j]));
            } else {
                v = ((part[0][j] + part[1][j]) + (part[2][j] + part[3][j])) / (float)hw;
                if (mode == RR_POOL_GEM) v = __powf(v, 1.0f / p);
            }
            out[img * c + ch + r] = v;
        }
    }
}

// NHWC bf16 with c % 8 == 0 (the extractor's stage maps): one 16-B load = 8
// channels per lane, a wave covers 512 channels of one pixel, the block's 16
// waves split the pixels (4 loads in flight per lane); the 16 partials are
// combined through LDS in a fixed order.  grid = (ceil(c/512), n).
template <typename H>
__global__ void __launch_bounds__(1024) k_pool_nhwc_h16x8(const uint4* __restrict__ x, int c, int hw, int mode,
                                                           float p, int ip, const float* __restrict__ pdev,
                                                           float eps, float* __restrict__ out) {
    gem_exponent(pdev, p, ip);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c8 = c >> 3;
    const int g = blockIdx.x * 64 + lane;  // this lane's 8-channel group
    const long long img = blockIdx.y;
    __shared__ float part[16][512];
    const bool mac = mode == RR_POOL_MAC;
    float acc[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = mac ? -INFINITY : 0.f;
    auto add = [&](uint4 q) {
        const unsigned u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float v0 = H16<H>::lo(u[e]), v1 = H16<H>::hi(u[e]);
            if (mode == RR_POOL_GEM) {
                acc[2 * e] += powp(clamp_min_nan(v0, eps), p, ip);
                acc[2 * e + 1] += powp(clamp_min_nan(v1, eps), p, ip);
            } else if (mac) {
                acc[2 * e] = max_nan(acc[2 * e], v0);
                acc[2 * e + 1] = max_nan(acc[2 * e + 1], v1);
            } else {
                acc[2 * e] += v0;
                acc[2 * e + 1] += v1;
            }
        }
    };
    if (g < c8) {
        const uint4* base = x + img * hw * c8 + g;
        int i = wave;
        for (; i + 48 < hw; i += 64) {
            const uint4 q0 = base[(long long)i * c8], q1 = base[(long long)(i + 16) * c8];
            const uint4 q2 = base[(long long)(i + 32) * c8], q3 = base[(long long)(i + 48) * c8];
            add(q0); add(q1); add(q2); add(q3);
        }
        for (; i < hw; i += 16) add(base[(long long)i * c8]);
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) part[wave][lane * 8 + r] = acc[r];
    __syncthreads();
    if (threadIdx.x < 512) {
        const int ch = blockIdx.x * 512 + threadIdx.x;
        if (ch < c) {
            float v = part[0][threadIdx.x];
            for (int w = 1; w < 16; ++w) v = mac ? max_nan(v, part[w][threadIdx.x]) : v + part[w][threadIdx.x];
            if (!mac) {
                v = v / (float)hw;
                if (mode == RR_POOL_GEM) v = __powf(v, 1.0f / p);
            }
            out[img * c + ch] = v;
        }
    }
}

// NCHW: one wave per (image, channel) plane of hw contiguous values.
template <typename T>
__global__ void __launch_bounds__(256) k_pool_nchw(const T* __restrict__ x, long long planes, int hw, int mode,
                                                   float p, int ip, const float* __restrict__ pdev, float eps,
                                                   float* __restrict__ out) {
    gem_exponent(pdev, p, ip);
    const long long plane = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (plane >= planes) return;
    const T* base = x + plane * hw;
    float acc = mode == RR_POOL_MAC ? -INFINITY : 0.f;
    for (int i = lane; i < hw; i += 64) {
        float v = DT<T>::to_f(base[i]);
        if (mode == RR_POOL_GEM) acc += powp(clamp_min_nan(v, eps), p, ip);
        else if (mode == RR_POOL_MAC) acc = max_nan(acc, v);
        else acc += v;
    }
    if (mode == RR_POOL_MAC) {
        for (int o = 32; o > 0; o >>= 1) acc = max_nan(acc, __shfl_xor(acc, o, 64));
    } else {
        acc = wave_sum(acc);
    }
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

// Dense layer on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32): a block of 8
// waves owns 16 outputs x 64 rows; wave w takes the K-slices kb = w, w+8, ...
// of 16 inputs.  Lane (r = lane & 15, g = lane >> 4) loads W[o0+r][16kb+4g..+3]
// and x[row+r][16kb+4g..+3] as float4; MFMA e of the four uses component e, so
// each instruction sums k = 16kb + 4g + e over g — every k exactly once.  The
// 8 partial tiles are reduced through LDS in a fixed order.  W is read once per
// 64 rows (the old one-wave-per-output form re-read x per output: ~100x the
// L2 traffic).  in_dim % 4 == 0.  grid = (ceil(out/16), ceil(rows/64)).
typedef __attribute__((ext_vector_type(4))) float lf32x4_t;
__global__ void __launch_bounds__(512) k_linear_mfma(const float* __restrict__ x, int rows, int in_dim,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     int out_dim, float* __restrict__ y) {
    constexpr int RG = 4;  // 16-row groups per block
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int o0 = blockIdx.x * 16, row0 = blockIdx.y * 16 * RG;
    __shared__ float part[8][RG][64][4];
    lf32x4_t acc[RG];
#pragma unroll
    for (int j = 0; j < RG; ++j) acc[j] = (lf32x4_t){0.f, 0.f, 0.f, 0.f};
    const int nkb = (in_dim + 15) / 16;
    const bool orow = o0 + r < out_dim;
    const float* wr = w + (long long)(orow ? o0 + r : 0) * in_dim;
    for (int kb = wave; kb < nkb; kb += 8) {
        const int k = kb * 16 + g * 4;
        const bool kin = k < in_dim;
        const float4 a = (orow && kin) ? *reinterpret_cast<const float4*>(wr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 bx[RG];
#pragma unroll
        for (int j = 0; j < RG; ++j) {
            const int row = row0 + j * 16 + r;
            bx[j] = (row < rows && kin) ? *reinterpret_cast<const float4*>(x + (long long)row * in_dim + k)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < RG; ++j) {
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bx[j].x, acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bx[j].y, acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bx[j].z, acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bx[j].w, acc[j], 0, 0, 0);
        }
    }
#pragma unroll
    for (int j = 0; j < RG; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) part[wave][j][lane][e] = acc[j][e];
    __syncthreads();
    // lane L of the tile holds D[o = 4*(L>>4) + e][row = L & 15]
    for (int t = threadIdx.x; t < RG * 64 * 4; t += 512) {
        const int j = t >> 8, L = (t >> 2) & 63, e = t & 3;
        float v = part[0][j][L][e];
#pragma unroll
        for (int q = 1; q < 8; ++q) v += part[q][j][L][e];
        const int o = o0 + 4 * (L >> 4) + e, row = row0 + j * 16 + (L & 15);
        if (o < out_dim && row < rows) y[(long long)row * out_dim + o] = v + (b ? b[o] : 0.f);
    }
}


// Post-hoc learned whitening (cirtorch/utils/whiten.py:4-12, applied by
// scripts/test.py:253-254) in the reference's arithmetic type: numpy promotes
// the float32 descriptors to float64 against the float64 (m, P) of
// whitenlearn, so y = P[:d] (x - m) and the L2 norm run in float64 here too,
// on the f64 MFMA (v_mfma_f64_16x16x4_f64).  Whitening matrices amplify
// directions of small variance, so a float32 GEMM loses ~1e-3 absolute on
// the output; float64 keeps it at the final float32 rounding.
// Block = 8 waves, 16 outputs x 64 rows; wave w takes the K-slices kb = w,
// w + 8, ... of 16 inputs; lane (r = lane & 15, g = lane >> 4) loads
// P[o0 + r][16 kb + 4 g .. + 3] and x[row + r][...] (centred in f64), MFMA e
// of the four uses component e.  f64 C/D layout: col = lane & 15,
// row = (lane >> 4) + 4 e.  Partial tiles reduced through LDS in fixed order.
typedef __attribute__((ext_vector_type(4))) double lf64x4_t;
__global__ void __launch_bounds__(512) k_whiten_f64(const float* __restrict__ x, int rows, int dim,
                                                    const double* __restrict__ m, const double* __restrict__ P,
                                                    int d_out, double* __restrict__ y) {
    constexpr int RG = 4;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int o0 = blockIdx.x * 16, row0 = blockIdx.y * 16 * RG;
    __shared__ double part[8][RG][64][4];
    lf64x4_t acc[RG];
#pragma unroll
    for (int j = 0; j < RG; ++j) acc[j] = (lf64x4_t){0.0, 0.0, 0.0, 0.0};
    const int nkb = dim / 16;
    const bool orow = o0 + r < d_out;
    const double* pr = P + (long long)(orow ? o0 + r : 0) * dim;
    for (int kb = wave; kb < nkb; kb += 8) {
        const int k = kb * 16 + g * 4;
        double a[4];
        if (orow) {
            const double2 a01 = *reinterpret_cast<const double2*>(pr + k);
            const double2 a23 = *reinterpret_cast<const double2*>(pr + k + 2);
            a[0] = a01.x; a[1] = a01.y; a[2] = a23.x; a[3] = a23.y;
        } else {
            a[0] = a[1] = a[2] = a[3] = 0.0;
        }
        const double2 m01 = *reinterpret_cast<const double2*>(m + k);
        const double2 m23 = *reinterpret_cast<const double2*>(m + k + 2);
        double b[RG][4];
#pragma unroll
        for (int j = 0; j < RG; ++j) {
            const int row = row0 + j * 16 + r;
            if (row < rows) {
                const float4 v = *reinterpret_cast<const float4*>(x + (long long)row * dim + k);
                b[j][0] = (double)v.x - m01.x; b[j][1] = (double)v.y - m01.y;
                b[j][2] = (double)v.z - m23.x; b[j][3] = (double)v.w - m23.y;
            } else {
                b[j][0] = b[j][1] = b[j][2] = b[j][3] = 0.0;
            }
        }
#pragma unroll
        for (int j = 0; j < RG; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[e], b[j][e], acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < RG; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) part[wave][j][lane][e] = acc[j][e];
    __syncthreads();
    for (int t = threadIdx.x; t < RG * 64 * 4; t += 512) {
        const int j = t >> 8, L = (t >> 2) & 63, e = t & 3;
        double v = part[0][j][L][e];
#pragma unroll
        for (int q = 1; q < 8; ++q) v += part[q][j][L][e];
        const int o = o0 + (L >> 4) + 4 * e, row = row0 + j * 16 + (L & 15);
        if (o < d_out && row < rows) y[(long long)row * d_out + o] = v;
    }
}

// y32 = y / (||y||_2 + eps) per row, norm in float64 (whiten.py:10), fixed order.
__global__ void __launch_bounds__(256) k_l2n_rows_f64(const double* __restrict__ y, int dim, double eps,
                                                      float* __restrict__ out) {
    const long long row = blockIdx.x;
    const double* yr = y + row * dim;
    __shared__ double red[4];
    double ss = 0.0;
    for (int i = threadIdx.x; i < dim; i += 256) ss = fma(yr[i], yr[i], ss);
    ss = wave_sum_d(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    const double nrm = sqrt((red[0] + red[1]) + (red[2] + red[3])) + eps;
    for (int i = threadIdx.x; i < dim; i += 256) out[row * dim + i] = (float)(yr[i] / nrm);
}

}  // namespace rr

using namespace rr;

extern "C" {

int rr_global_pool(const void* x, int n, int c, int hw, int layout, int mode, float p, float eps, float* out,
                   int dtype, void* stream) {
    if (mode == RR_POOL_GEM && !(p > 0.f)) return fail(RR_EINVAL, "rr_global_pool: GeM p must be > 0");
    return rr_global_pool_pdev(x, n, c, hw, layout, mode, p, nullptr, eps, out, dtype, stream);
}

int rr_global_pool_pdev(const void* x, int n, int c, int hw, int layout, int mode, float p, const float* p_dev,
                        float eps, float* out, int dtype, void* stream) {
    if (n <= 0 || c <= 0 || hw <= 0) return fail(RR_EINVAL, "rr_global_pool: empty input");
    if (mode < 0 || mode > 2) return fail(RR_EINVAL, "rr_global_pool: mode");
    // the host exponent is validated here; a device exponent (p_dev) is read by the kernel
    if (mode == RR_POOL_GEM && !p_dev && !(p > 0.f)) return fail(RR_EINVAL, "rr_global_pool: GeM p must be > 0");
    const float* pdev = mode == RR_POOL_GEM ? p_dev : nullptr;
    int ip = (p == 3.f) ? 3 : (p == 2.f) ? 2 : (p == 1.f) ? 1 : 0;
    hipStream_t s = as_stream(stream);
    if (layout == RR_NHWC) {
        if (c % 4) return fail(RR_EINVAL, "rr_global_pool: NHWC needs c % 4 == 0");
        dim3 grid((c + 255) / 256, n);
        if (dtype == RR_BF16 && c % 8 == 0 && ((uintptr_t)x & 15) == 0)
            hipLaunchKernelGGL(k_pool_nhwc_h16x8<bf16_t>, dim3((c + 511) / 512, n), dim3(1024), 0, s, (const uint4*)x, c, hw,
                               mode, p, ip, pdev, eps, out);
        else if (dtype == RR_F16 && c % 8 == 0 && ((uintptr_t)x & 15) == 0)
            hipLaunchKernelGGL(k_pool_nhwc_h16x8<f16_t>, dim3((c + 511) / 512, n), dim3(1024), 0, s, (const uint4*)x, c,
                               hw, mode, p, ip, pdev, eps, out);
        else if (dtype == RR_BF16)
            hipLaunchKernelGGL(k_pool_nhwc<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, c, hw, mode, p, ip, pdev, eps, out);
        else if (dtype == RR_F16)
            hipLaunchKernelGGL(k_pool_nhwc<f16_t>, grid, dim3(256), 0, s, (const f16_t*)x, c, hw, mode, p, ip, pdev, eps, out);
        else if (dtype == RR_F32)
            hipLaunchKernelGGL(k_pool_nhwc<float>, grid, dim3(256), 0, s, (const float*)x, c, hw, mode, p, ip, pdev, eps, out);
        else
            return fail(RR_EINVAL, "rr_global_pool: dtype");
    } else if (layout == RR_NCHW) {
        long long planes = (long long)n * c;
        dim3 grid((unsigned)((planes + 3) / 4));
        if (dtype == RR_BF16)
            hipLaunchKernelGGL(k_pool_nchw<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, planes, hw, mode, p, ip, pdev, eps, out);
        else if (dtype == RR_F16)
            hipLaunchKernelGGL(k_pool_nchw<f16_t>, grid, dim3(256), 0, s, (const f16_t*)x, planes, hw, mode, p, ip, pdev, eps, out);
        else if (dtype == RR_F32)
            hipLaunchKernelGGL(k_pool_nchw<float>, grid, dim3(256), 0, s, (const float*)x, planes, hw, mode, p, ip, pdev, eps, out);
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
    if (in_dim % 4 || in_dim <= 0) return fail(RR_EINVAL, "rr_linear_rows: in_dim must be a positive multiple of 4");
    if ((((uintptr_t)x) | ((uintptr_t)w)) & 15) return fail(RR_EINVAL, "rr_linear_rows: x and w must be 16-byte aligned");
    hipLaunchKernelGGL(k_linear_mfma, dim3((out_dim + 15) / 16, (rows + 63) / 64), dim3(512), 0, as_stream(stream), x,
                       rows, in_dim, w, b, out_dim, y);
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

size_t rr_whiten_workspace_bytes(int rows, int d_out) { return (size_t)rows * d_out * sizeof(double); }

int rr_whitenapply(const float* x, int rows, int dim, const double* m, const double* P, int d_out, float* y,
                   void* workspace, size_t workspace_bytes, void* stream) {
    if (rows <= 0 || dim <= 0 || d_out <= 0) return fail(RR_EINVAL, "rr_whitenapply: empty");
    if (dim % 16) return fail(RR_EINVAL, "rr_whitenapply: dim must be a multiple of 16");
    if (d_out > dim) return fail(RR_EINVAL, "rr_whitenapply: d_out > dim");
    if ((((uintptr_t)x) | ((uintptr_t)m) | ((uintptr_t)P)) & 15)
        return fail(RR_EINVAL, "rr_whitenapply: x, m and P must be 16-byte aligned");
    if (!workspace || workspace_bytes < rr_whiten_workspace_bytes(rows, d_out))
        return fail(RR_ENOSPACE, "rr_whitenapply: workspace too small");
    hipStream_t s = as_stream(stream);
    double* t = (double*)workspace;
    for (int r0 = 0; r0 < rows; r0 += 1 << 20) {  // <= 16384 row blocks per launch
        const int n = rows - r0 < (1 << 20) ? rows - r0 : (1 << 20);
        hipLaunchKernelGGL(k_whiten_f64, dim3((d_out + 15) / 16, (n + 63) / 64), dim3(512), 0, s,
                           x + (long long)r0 * dim, n, dim, m, P, d_out, t + (long long)r0 * d_out);
    }
    hipLaunchKernelGGL(k_l2n_rows_f64, dim3(rows), dim3(256), 0, s, t, d_out, 1e-6, y);
    return check_launch("rr_whitenapply");
}

}  // extern "C"
