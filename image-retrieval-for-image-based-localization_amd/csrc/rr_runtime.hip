// librr.so — runtime helpers and the small memory-bound extractor ops:
// error state, image normalise + NCHW->NHWC, max-pool, bilinear resize,
// synthetic-row generator, f32->bf16 cast.  gfx950 only.
#include "rr_internal.h"

#include <cstring>

namespace rr {

static thread_local std::string g_err;

int g_grid_cap = 0;
static int g_dev_cus = 0;

int grid_cus() {
    if (g_dev_cus == 0) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        g_dev_cus = cus;
    }
    return (g_grid_cap > 0 && g_grid_cap < g_dev_cus) ? g_grid_cap : g_dev_cus;
}

void set_error(const std::string& msg) { g_err = msg; }
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// ------------------------------------------------------------------ normalise
struct NormParams {
    float mean[4];
    float stdv[4];
};

// One thread per output pixel: reads c planes (coalesced along w), writes c_pad
// contiguous channels (16 B for bf16 x 8 / f32 x 4).  (x - mean) / std is
// evaluated as in cirtorch/utils/image.py:125 ((x - m) / s, true division).
template <typename T>
__global__ void k_image_to_nhwc(const float* __restrict__ src, int n, int c, int hw, NormParams np,
                                int do_norm, T* __restrict__ dst, int c_pad) {
    long long pix = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long total = (long long)n * hw;
    if (pix >= total) return;
    long long img = pix / hw;
    long long off = pix - img * hw;
    const float* s = src + img * c * hw + off;
    T* d = dst + pix * c_pad;
    for (int ch = 0; ch < c_pad; ++ch) {
        float v = 0.f;
        if (ch < c) {
            v = s[(long long)ch * hw];
            if (do_norm) v = (v - np.mean[ch]) / np.stdv[ch];
        }
        d[ch] = DT<T>::from_f(v);
    }
}

// bf16, c = 3, c_pad = 8: one thread per pixel, one 16-B store; reads are
// coalesced along w within each of the 3 planes.
__global__ void k_image_to_nhwc_bf16x8(const float* __restrict__ src, long long npix, int hw, NormParams np,
                                       int do_norm, uint4* __restrict__ dst) {
    const long long pix = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= npix) return;
    const long long img = pix / hw;
    const long long off = pix - img * hw;
    const float* s = src + img * 3 * hw + off;
    float v[3];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        v[ch] = s[(long long)ch * hw];
        if (do_norm) v[ch] = (v[ch] - np.mean[ch]) / np.stdv[ch];
    }
    uint4 o;
    o.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
    o.y = (unsigned)f2bf(v[2]);
    o.z = 0u;
    o.w = 0u;
    dst[pix] = o;
}

// Ragged batch -> NHWC: one thread per pixel of the h x w batch map; image i's
// planes are read at its own address (row stride w_i), map pixels outside its
// extent read 0 and are then normalised like any other pixel (the pad-then-
// normalise order of random_augmentation.py:102,174).  u8: x / 255 in IEEE
// division (== to_tensor, == the LUT of pixels_to_unit).
template <typename T, bool U8>
__global__ void k_image_to_nhwc_ragged(RaggedTab rt, int c, int h, int w, NormParams np, int do_norm,
                                       T* __restrict__ dst, int c_pad) {
    const int hw = h * w;
    const int img = blockIdx.y;
    const int pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= hw) return;
    const int y = pix / w, x = pix - y * w;
    const int hi = rt.h[img], wi = rt.w[img];
    const bool in = y < hi && x < wi;
    const long long plane = (long long)hi * wi, o = (long long)y * wi + x;
    T* d = dst + ((long long)img * hw + pix) * c_pad;
    for (int ch = 0; ch < c_pad; ++ch) {
        float v = 0.f;
        if (ch < c) {
            if (in) {
                if constexpr (U8) v = (float)((const unsigned char*)rt.p[img])[ch * plane + o] / 255.f;
                else v = ((const float*)rt.p[img])[ch * plane + o];
            }
            if (do_norm) v = (v - np.mean[ch]) / np.stdv[ch];
        }
        d[ch] = DT<T>::from_f(v);
    }
}

// pad_packed_images on the device: [n][c][h][w] elements of type E, image i's
// [c][h_i][w_i] at the top-left, `pad` elsewhere.  One thread per output
// element of one image (blockIdx.y), reads coalesced along each image row.
template <typename E>
__global__ void k_pad_images(RaggedTab rt, int c, int h, int w, E pad, E* __restrict__ dst) {
    const int img = blockIdx.y;
    const long long per = (long long)c * h * w;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= per) return;
    const int x = (int)(i % w);
    const long long r = i / w;
    const int y = (int)(r % h), ch = (int)(r / h);
    const int hi = rt.h[img], wi = rt.w[img];
    E v = pad;
    if (y < hi && x < wi) v = ((const E*)rt.p[img])[((long long)ch * hi + y) * wi + x];
    dst[img * per + i] = v;
}

const char* ragged_fill(RaggedTab& t, const void* const* srcs, const int* extents, int i0, int cnt, int h, int w) {
    for (int j = 0; j < cnt; ++j) {
        const int hi = extents[2 * (i0 + j)], wi = extents[2 * (i0 + j) + 1];
        if (hi < 0 || wi < 0 || hi > h || wi > w) return "image extent outside the batch map";
        if ((hi == 0) != (wi == 0)) return "image extent: both sides must be 0 (a None entry) or positive";
        if (hi > 0 && !srcs[i0 + j]) return "null image pointer with a non-empty extent";
        t.p[j] = hi > 0 ? srcs[i0 + j] : nullptr;
        t.h[j] = hi;
        t.w[j] = wi;
    }
    return nullptr;
}

// NHWC max-pool, 8 channels (16 B of bf16) per thread.
__global__ void k_maxpool_nhwc_bf16x8(const uint4* __restrict__ x, int n, int h, int w, int c8, int k, int stride,
                                      int pad, uint4* __restrict__ y, int ho, int wo) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)n * ho * wo * c8;
    if (i >= total) return;
    const int cc = (int)(i % c8);
    long long r = i / c8;
    const int ow = (int)(r % wo);
    r /= wo;
    const int oh = (int)(r % ho);
    const int img = (int)(r / ho);
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
    const int h0 = oh * stride - pad, w0 = ow * stride - pad;
    for (int a = 0; a < k; ++a) {
        const int hh = h0 + a;
        if (hh < 0 || hh >= h) continue;
        for (int b = 0; b < k; ++b) {
            const int ww = w0 + b;
            if (ww < 0 || ww >= w) continue;
            const uint4 q = x[(((long long)img * h + hh) * w + ww) * c8 + cc];
            const unsigned u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                m[2 * e] = fmaxf(m[2 * e], __uint_as_float(u[e] << 16));
                m[2 * e + 1] = fmaxf(m[2 * e + 1], __uint_as_float(u[e] & 0xffff0000u));
            }
        }
    }
    uint4 o;
    o.x = (unsigned)f2bf(m[0]) | ((unsigned)f2bf(m[1]) << 16);
    o.y = (unsigned)f2bf(m[2]) | ((unsigned)f2bf(m[3]) << 16);
    o.z = (unsigned)f2bf(m[4]) | ((unsigned)f2bf(m[5]) << 16);
    o.w = (unsigned)f2bf(m[6]) | ((unsigned)f2bf(m[7]) << 16);
    y[i] = o;
}

// ------------------------------------------------------------------ max-pool
template <typename T>
__global__ void k_maxpool_nhwc(const T* __restrict__ x, int n, int h, int w, int c, int k, int stride,
                               int pad, T* __restrict__ y, int ho, int wo) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long total = (long long)n * ho * wo * c;
    if (i >= total) return;
    int ch = (int)(i % c);
    long long r = i / c;
    int ow = (int)(r % wo);
    r /= wo;
    int oh = (int)(r % ho);
    int img = (int)(r / ho);
    float m = -INFINITY;
    int h0 = oh * stride - pad, w0 = ow * stride - pad;
    for (int a = 0; a < k; ++a) {
        int hh = h0 + a;
        if (hh < 0 || hh >= h) continue;
        for (int b = 0; b < k; ++b) {
            int ww = w0 + b;
            if (ww < 0 || ww >= w) continue;
            m = fmaxf(m, DT<T>::to_f(x[(((long long)img * h + hh) * w + ww) * c + ch]));
        }
    }
    y[i] = DT<T>::from_f(m);
}

// ------------------------------------------------------------ bilinear resize
// align_corners=False source index, as torch's area_pixel_compute_source_index
// for linear modes: src = scale*(dst+0.5)-0.5 clamped at 0.
__global__ void k_resize_bilinear(const float* __restrict__ src, int c, int h, int w, float* __restrict__ dst,
                                  int ho, int wo, float sh, float sw) {
    const long long total = (long long)c * ho * wo;
    const long long step = (long long)gridDim.x * blockDim.x;   // grid-stride: batches of any size
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += step) {
    int ox = (int)(i % wo);
    long long r = i / wo;
    int oy = (int)(r % ho);
    int ch = (int)(r / ho);
    float fy = fmaxf(sh * (oy + 0.5f) - 0.5f, 0.f);
    float fx = fmaxf(sw * (ox + 0.5f) - 0.5f, 0.f);
    int y0 = (int)fy, x0 = (int)fx;
    int y1 = y0 + (y0 < h - 1 ? 1 : 0);
    int x1 = x0 + (x0 < w - 1 ? 1 : 0);
    float ly1 = fy - y0, ly0 = 1.f - ly1;
    float lx1 = fx - x0, lx0 = 1.f - lx1;
    const float* p = src + (long long)ch * h * w;
    float v = ly0 * (lx0 * p[(long long)y0 * w + x0] + lx1 * p[(long long)y0 * w + x1]) +
              ly1 * (lx0 * p[(long long)y1 * w + x0] + lx1 * p[(long long)y1 * w + x1]);
    dst[i] = v;
    }
}

// ------------------------------------------------------------ synthetic rows
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// One block (256 threads) per row; Box-Muller on 2 x 24-bit uniforms per pair.
__global__ void __launch_bounds__(256) k_fill_unit_rows(float* __restrict__ out, int d, uint64_t seed,
                                                        long long row0) {
    long long row = blockIdx.x;
    uint64_t base = splitmix64(seed ^ (uint64_t)(row0 + row) * 0xD1B54A32D192ED03ull);
    __shared__ double red[4];
    float vals[16];
    double ss = 0.0;
    int per = (d + 255) / 256;  // <= 16 (d <= 4096)
    for (int t = 0; t < per; t += 2) {
        int j = (threadIdx.x + 256 * t);
        uint64_t h = splitmix64(base + (uint64_t)j);
        float u1 = ((h >> 40) + 1) * (1.0f / 16777217.0f);
        float u2 = ((h >> 16) & 0xFFFFFF) * (1.0f / 16777216.0f);
        float r = sqrtf(-2.f * logf(u1));
        float s, c;
        sincosf(6.28318530717958647f * u2, &s, &c);
        vals[t] = r * c;
        if (t + 1 < per) vals[t + 1] = r * s;
    }
    for (int t = 0; t < per; ++t) {
        int j = threadIdx.x + 256 * t;
        if (j < d) ss += (double)vals[t] * vals[t];
    }
    ss = wave_sum_d(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    double tot = red[0] + red[1] + red[2] + red[3];
    float inv = (float)(1.0 / sqrt(tot));
    for (int t = 0; t < per; ++t) {
        int j = threadIdx.x + 256 * t;
        if (j < d) out[row * d + j] = vals[t] * inv;
    }
}

// Grid-stride casts: a dispatch holds < 2^32 work-items, so a 10M x 2048
// database (2e10 elements, config 5) is covered by a capped grid looping.
__global__ void k_cast_f32_f16(const float* __restrict__ x, f16_t* __restrict__ y, long long n) {
    const long long step = (long long)gridDim.x * blockDim.x * 4;
    for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += step) {
        if (i + 3 < n) {
            const float4 v = *reinterpret_cast<const float4*>(x + i);
            y[i] = (f16_t)v.x; y[i + 1] = (f16_t)v.y; y[i + 2] = (f16_t)v.z; y[i + 3] = (f16_t)v.w;
        } else {
            for (long long j = i; j < n; ++j) y[j] = (f16_t)x[j];
        }
    }
}

__global__ void k_cast_f32_bf16(const float* __restrict__ x, bf16_t* __restrict__ y, long long n) {
    const long long step = (long long)gridDim.x * blockDim.x * 4;
    for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += step) {
        if (i + 3 < n) {
            float4 v = *reinterpret_cast<const float4*>(x + i);
            ushort4 o;
            o.x = f2bf(v.x); o.y = f2bf(v.y); o.z = f2bf(v.z); o.w = f2bf(v.w);
            *reinterpret_cast<ushort4*>(y + i) = o;
        } else {
            for (long long j = i; j < n; ++j) y[j] = f2bf(x[j]);
        }
    }
}

// int8 screening copy (rr_quantize_i8): amax = max |x| (non-negative floats order
// like their bit patterns: one unsigned atomicMax per block), then
// y = clamp(rint(x * 127 / amax), -127, 127) with the scale read on the device.
__global__ void k_amax_reset(unsigned* amax) { *amax = 0u; }

__global__ void __launch_bounds__(256) k_absmax(const float* __restrict__ x, long long n, unsigned* __restrict__ amax) {
    const long long step = (long long)gridDim.x * blockDim.x * 4;
    float m = 0.f;
    for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += step) {
        if (i + 3 < n) {
            const float4 v = *reinterpret_cast<const float4*>(x + i);
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        } else {
            for (long long j = i; j < n; ++j) m = fmaxf(m, fabsf(x[j]));
        }
    }
    m = wave_max(m);
    __shared__ float red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(amax, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

__global__ void __launch_bounds__(256) k_cast_f32_i8(const float* __restrict__ x, long long n,
                                                     const unsigned* __restrict__ amax, int8_t* __restrict__ y) {
    const float am = __uint_as_float(*amax);
    const float sc = am > 0.f ? 127.f / am : 1.f;
    auto q = [&](float v) { return (int)fminf(fmaxf(rintf(v * sc), -127.f), 127.f); };
    const long long step = (long long)gridDim.x * blockDim.x * 4;
    for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += step) {
        if (i + 3 < n) {
            const float4 v = *reinterpret_cast<const float4*>(x + i);
            const unsigned w = (unsigned)(q(v.x) & 255) | ((unsigned)(q(v.y) & 255) << 8) |
                               ((unsigned)(q(v.z) & 255) << 16) | ((unsigned)(q(v.w) & 255) << 24);
            *reinterpret_cast<unsigned*>(y + i) = w;
        } else {
            for (long long j = i; j < n; ++j) y[j] = (int8_t)q(x[j]);
        }
    }
}

// Per-row int8 screening copy (queries): one wave per row, amax_rows[r] = max |x_r|,
// y_r = clamp(rint(x_r * 127 / amax_rows[r]), -127, 127).  A positive per-row
// scale leaves each query's ranking unchanged, so a query's screened candidates
// no longer depend on the other queries of its batch.
__global__ void __launch_bounds__(256) k_quantize_i8_rows(const float* __restrict__ x, int rows, int d,
                                                          int8_t* __restrict__ y, float* __restrict__ amax_rows) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    const float* xr = x + (long long)r * d;
    float m = 0.f;
    for (int i = lane * 4; i < d; i += 256) {
        const float4 v = *reinterpret_cast<const float4*>(xr + i);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    m = wave_max(m);
    const float sc = m > 0.f ? 127.f / m : 1.f;
    auto q = [&](float v) { return (int)fminf(fmaxf(rintf(v * sc), -127.f), 127.f); };
    for (int i = lane * 4; i < d; i += 256) {
        const float4 v = *reinterpret_cast<const float4*>(xr + i);
        const unsigned w = (unsigned)(q(v.x) & 255) | ((unsigned)(q(v.y) & 255) << 8) |
                           ((unsigned)(q(v.z) & 255) << 16) | ((unsigned)(q(v.w) & 255) << 24);
        *reinterpret_cast<unsigned*>(y + (long long)r * d + i) = w;
    }
    if (lane == 0) amax_rows[r] = m;
}

static inline unsigned cast_blocks(long long n) {
    const long long b = (n + 1023) / 1024;       // 256 threads x 4 elements
    return (unsigned)(b < (1ll << 20) ? (b > 0 ? b : 1) : (1ll << 20));
}

static inline unsigned nblk(long long total, int b) { return (unsigned)((total + b - 1) / b); }

}  // namespace rr

using namespace rr;

extern "C" {

int rr_version(void) { return 1; }

const char* rr_last_error(void) { return g_err.c_str(); }

int rr_device_arch(char* buf, int buflen) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail(RR_EHIP, "hipGetDevice failed");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return fail(RR_EHIP, "hipGetDeviceProperties failed");
    std::strncpy(buf, prop.gcnArchName, buflen - 1);
    buf[buflen - 1] = 0;
    return RR_OK;
}

int rr_image_to_nhwc(const float* src, int n, int c, int h, int w, const float* mean_host,
                     const float* std_host, int do_normalize, void* dst, int c_pad, int dtype,
                     void* stream) {
    if (c > 4 || c_pad < c || n <= 0 || h <= 0 || w <= 0) return fail(RR_EINVAL, "rr_image_to_nhwc: bad shape");
    NormParams np{};
    for (int i = 0; i < c; ++i) {
        np.mean[i] = do_normalize ? mean_host[i] : 0.f;
        np.stdv[i] = do_normalize ? std_host[i] : 1.f;  // divisor (true division in kernel)
    }
    long long total = (long long)n * h * w;
    if (dtype == RR_BF16 && c == 3 && c_pad == 8 && (((uintptr_t)dst) & 15) == 0)
        hipLaunchKernelGGL(k_image_to_nhwc_bf16x8, dim3(nblk(total, 256)), dim3(256), 0, as_stream(stream), src,
                           total, h * w, np, do_normalize, (uint4*)dst);
    else if (dtype == RR_BF16)
        hipLaunchKernelGGL(k_image_to_nhwc<bf16_t>, dim3(nblk(total, 256)), dim3(256), 0, as_stream(stream), src, n,
                           c, h * w, np, do_normalize, (bf16_t*)dst, c_pad);
    else if (dtype == RR_F16)
        hipLaunchKernelGGL(k_image_to_nhwc<f16_t>, dim3(nblk(total, 256)), dim3(256), 0, as_stream(stream), src, n,
                           c, h * w, np, do_normalize, (f16_t*)dst, c_pad);
    else if (dtype == RR_F32)
        hipLaunchKernelGGL(k_image_to_nhwc<float>, dim3(nblk(total, 256)), dim3(256), 0, as_stream(stream), src, n, c,
                           h * w, np, do_normalize, (float*)dst, c_pad);
    else
        return fail(RR_EINVAL, "rr_image_to_nhwc: dtype");
    return check_launch("rr_image_to_nhwc");
}

int rr_image_to_nhwc_ragged(const void* const* srcs, const int* extents, int n, int c, int h, int w, int u8,
                            const float* mean_host, const float* std_host, int do_normalize, void* dst, int c_pad,
                            int dtype, void* stream) {
    if (!srcs || !extents || !dst) return fail(RR_EINVAL, "rr_image_to_nhwc_ragged: null pointer");
    if (c <= 0 || c > 4 || c_pad < c || n <= 0 || h <= 0 || w <= 0 || (long long)h * w >= (1ll << 31))
        return fail(RR_EINVAL, "rr_image_to_nhwc_ragged: bad shape");
    NormParams np{};
    for (int i = 0; i < c; ++i) {
        np.mean[i] = do_normalize ? mean_host[i] : 0.f;
        np.stdv[i] = do_normalize ? std_host[i] : 1.f;
    }
    const int esz = dtype == RR_F32 ? 4 : 2;
    if (dtype != RR_F32 && dtype != RR_BF16 && dtype != RR_F16) return fail(RR_EINVAL, "rr_image_to_nhwc_ragged: dtype");
    for (int i0 = 0; i0 < n; i0 += RAGGED_MAX) {
        const int cnt = n - i0 < RAGGED_MAX ? n - i0 : RAGGED_MAX;
        RaggedTab t;
        if (const char* e = ragged_fill(t, srcs, extents, i0, cnt, h, w))
            return fail(RR_EINVAL, std::string("rr_image_to_nhwc_ragged: ") + e);
        char* d = (char*)dst + (long long)i0 * h * w * c_pad * esz;
        const dim3 grid(nblk((long long)h * w, 256), cnt);
        auto launch = [&](auto kern, auto* out) {
            hipLaunchKernelGGL(kern, grid, dim3(256), 0, as_stream(stream), t, c, h, w, np, do_normalize, out, c_pad);
        };
        if (dtype == RR_F32) {
            if (u8) launch(k_image_to_nhwc_ragged<float, true>, (float*)d);
            else launch(k_image_to_nhwc_ragged<float, false>, (float*)d);
        } else if (dtype == RR_BF16) {
            if (u8) launch(k_image_to_nhwc_ragged<bf16_t, true>, (bf16_t*)d);
            else launch(k_image_to_nhwc_ragged<bf16_t, false>, (bf16_t*)d);
        } else {
            if (u8) launch(k_image_to_nhwc_ragged<f16_t, true>, (f16_t*)d);
            else launch(k_image_to_nhwc_ragged<f16_t, false>, (f16_t*)d);
        }
    }
    return check_launch("rr_image_to_nhwc_ragged");
}

int rr_pad_images(const void* const* srcs, const int* extents, int n, int c, int h, int w, int elem_bytes,
                  const void* pad_value_host, void* dst, void* stream) {
    if (!srcs || !extents || !dst || !pad_value_host) return fail(RR_EINVAL, "rr_pad_images: null pointer");
    if (n <= 0 || c <= 0 || h <= 0 || w <= 0 || (long long)c * h * w >= (1ll << 40))
        return fail(RR_EINVAL, "rr_pad_images: bad shape");
    if (elem_bytes != 1 && elem_bytes != 2 && elem_bytes != 4 && elem_bytes != 8)
        return fail(RR_EINVAL, "rr_pad_images: elem_bytes must be 1, 2, 4 or 8");
    const long long per = (long long)c * h * w;
    if ((per + 255) / 256 >= (1ll << 31)) return fail(RR_EINVAL, "rr_pad_images: image too large");
    for (int i0 = 0; i0 < n; i0 += RAGGED_MAX) {
        const int cnt = n - i0 < RAGGED_MAX ? n - i0 : RAGGED_MAX;
        RaggedTab t;
        if (const char* e = ragged_fill(t, srcs, extents, i0, cnt, h, w))
            return fail(RR_EINVAL, std::string("rr_pad_images: ") + e);
        char* d = (char*)dst + (long long)i0 * per * elem_bytes;
        const dim3 grid(nblk(per, 256), cnt);
        auto launch = [&](auto pad) {
            typedef decltype(pad) E;
            hipLaunchKernelGGL(k_pad_images<E>, grid, dim3(256), 0, as_stream(stream), t, c, h, w, pad, (E*)d);
        };
        if (elem_bytes == 1) launch(*(const uint8_t*)pad_value_host);
        else if (elem_bytes == 2) launch(*(const uint16_t*)pad_value_host);
        else if (elem_bytes == 4) launch(*(const uint32_t*)pad_value_host);
        else launch(*(const uint64_t*)pad_value_host);
    }
    return check_launch("rr_pad_images");
}

int rr_maxpool2d(const void* x, int n, int h, int w, int c, int k, int stride, int pad, void* y, int ho, int wo,
                 int dtype, void* stream) {
    long long total = (long long)n * ho * wo * c;
    if (total <= 0) return fail(RR_EINVAL, "rr_maxpool2d: empty");
    if (dtype == RR_BF16 && c % 8 == 0 && (((uintptr_t)x | (uintptr_t)y) & 15) == 0)
        hipLaunchKernelGGL(k_maxpool_nhwc_bf16x8, dim3(nblk(total / 8, 256)), dim3(256), 0, as_stream(stream),
                           (const uint4*)x, n, h, w, c / 8, k, stride, pad, (uint4*)y, ho, wo);
    else if (dtype == RR_BF16)
        hipLaunchKernelGGL(k_maxpool_nhwc<bf16_t>, dim3(nblk(total, 256)), dim3(256), 0, as_stream(stream),
                           (const bf16_t*)x, n, h, w, c, k, stride, pad, (bf16_t*)y, ho, wo);
    else if (dtype == RR_F16)
        hipLaunchKernelGGL(k_maxpool_nhwc<f16_t>, dim3(nblk(total, 256)), dim3(256), 0, as_stream(stream),
                           (const f16_t*)x, n, h, w, c, k, stride, pad, (f16_t*)y, ho, wo);
    else if (dtype == RR_F32)
        hipLaunchKernelGGL(k_maxpool_nhwc<float>, dim3(nblk(total, 256)), dim3(256), 0, as_stream(stream),
                           (const float*)x, n, h, w, c, k, stride, pad, (float*)y, ho, wo);
    else
        return fail(RR_EINVAL, "rr_maxpool2d: dtype");
    return check_launch("rr_maxpool2d");
}

int rr_resize_bilinear(const float* src, int c, int h, int w, float* dst, int ho, int wo, double scale_h,
                       double scale_w, void* stream) {
    long long total = (long long)c * ho * wo;
    if (total <= 0) return fail(RR_EINVAL, "rr_resize_bilinear: empty");
    const long long nb = (total + 255) / 256;
    hipLaunchKernelGGL(k_resize_bilinear, dim3((unsigned)(nb < (1ll << 22) ? nb : (1ll << 22))), dim3(256), 0,
                       as_stream(stream), src, c, h, w, dst,
                       ho, wo, (float)scale_h, (float)scale_w);
    return check_launch("rr_resize_bilinear");
}

int rr_fill_unit_rows(float* out, long long rows, int d, unsigned long long seed, long long row0, void* stream) {
    if (d <= 0 || d > 4096 || rows <= 0) return fail(RR_EINVAL, "rr_fill_unit_rows: d must be in (0, 4096]");
    const long long maxgrid = 1ll << 23;  // 2^23 blocks x 256 threads: a dispatch holds < 2^32 work-items
    for (long long r = 0; r < rows; r += maxgrid) {
        long long cnt = rows - r < maxgrid ? rows - r : maxgrid;
        hipLaunchKernelGGL(k_fill_unit_rows, dim3((unsigned)cnt), dim3(256), 0, as_stream(stream), out + r * d, d,
                           (uint64_t)seed, row0 + r);
    }
    return check_launch("rr_fill_unit_rows");
}

int rr_cast_f32_f16(const float* x, void* y, long long n, void* stream) {
    if (n <= 0) return RR_OK;
    if (!x || !y) return fail(RR_EINVAL, "rr_cast_f32_f16: null pointer");
    hipLaunchKernelGGL(k_cast_f32_f16, dim3(cast_blocks(n)), dim3(256), 0, as_stream(stream), x,
                       (f16_t*)y, n);
    return check_launch("rr_cast_f32_f16");
}

int rr_quantize_i8(const float* x, long long n, void* y, float* amax_dev, void* stream) {
    if (n <= 0) return RR_OK;
    if (!x || !y || !amax_dev) return fail(RR_EINVAL, "rr_quantize_i8: null pointer");
    if (n % 4 || ((uintptr_t)x & 15) || ((uintptr_t)y & 3)) return fail(RR_EINVAL, "rr_quantize_i8: n % 4, alignment");
    hipStream_t s = as_stream(stream);
    const unsigned g = cast_blocks(n) < 4096u ? cast_blocks(n) : 4096u;
    hipLaunchKernelGGL(k_amax_reset, dim3(1), dim3(1), 0, s, (unsigned*)amax_dev);
    hipLaunchKernelGGL(k_absmax, dim3(g), dim3(256), 0, s, x, n, (unsigned*)amax_dev);
    hipLaunchKernelGGL(k_cast_f32_i8, dim3(cast_blocks(n)), dim3(256), 0, s, x, n, (const unsigned*)amax_dev,
                       (int8_t*)y);
    return check_launch("rr_quantize_i8");
}

int rr_quantize_i8_rows(const float* x, int rows, int d, void* y, float* amax_rows, void* stream) {
    if (rows <= 0) return RR_OK;
    if (!x || !y || !amax_rows) return fail(RR_EINVAL, "rr_quantize_i8_rows: null pointer");
    if (d <= 0 || d % 4 || ((uintptr_t)x & 15) || ((uintptr_t)y & 3))
        return fail(RR_EINVAL, "rr_quantize_i8_rows: d % 4, alignment");
    hipLaunchKernelGGL(k_quantize_i8_rows, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, as_stream(stream), x, rows,
                       d, (int8_t*)y, amax_rows);
    return check_launch("rr_quantize_i8_rows");
}

int rr_cast_f32_bf16(const float* x, void* y, long long n, void* stream) {
    if (n <= 0) return RR_OK;
    hipLaunchKernelGGL(k_cast_f32_bf16, dim3(cast_blocks(n)), dim3(256), 0, as_stream(stream), x,
                       (bf16_t*)y, n);
    return check_launch("rr_cast_f32_bf16");
}

}  // extern "C"
