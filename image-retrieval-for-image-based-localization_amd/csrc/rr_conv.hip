// librr.so — implicit-GEMM convolution on CDNA4 MFMA with a fused epilogue.
//
// GEMM view (NHWC activations, [c_out][k] packed weights):
//   rows  = output channels c      (A operand: weight rows, K-contiguous)
//   cols  = output pixels  p       (B operand: im2col rows, K-contiguous)
//   D[c][p] = sum_k W[c][k] * X[p][k],  k = (kh*KW + kw)*c_in + ci
// so every operand tile is a set of 64-byte K-runs that are contiguous in HBM
// (one 16-B chunk = 8 bf16 / 4 f32 channels of one input pixel).
//
// Each lane of a 16x16 MFMA output tile holds 4 consecutive channels of one
// pixel, which is exactly the NHWC store granule: the BN scale/shift,
// residual read and activation are applied in registers and written once.
//
// bf16 : v_mfma_f32_16x16x32_bf16 (K = 32 per instruction, f32 accumulate)
// f32  : v_mfma_f32_16x16x4_f32   (exact f32 fma chain, the parity mode)
//
// LDS: double-buffered A/B tiles of 64-B rows, chunk XOR-swizzle
// phys = chunk ^ (((row >> 3) & 1) * 3) makes every ds_read_b128 lane group
// (16 lanes: rows r..r+15 of one chunk column pair) hit 16 distinct 16-B slots.
//
// Reference ops replaced: nn.Conv2d (cirtorch/backbones/resnet.py:61,
// backbones/misc.py:166-180) + ABN eval BN/leaky_relu (utils/misc.py:175-235)
// + residual add/activation (backbones/misc.py:184-203); also the score GEMM
// of the kNN (scripts/test.py:247).
#include "rr_internal.h"

#include <cstdlib>

namespace rr {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;


template <typename T> struct Vec;
template <> struct Vec<bf16_t> { static constexpr int N = 8; };
template <> struct Vec<float> { static constexpr int N = 4; };

__device__ __forceinline__ int lds_off(int row, int chunk) {
    return row * 64 + ((chunk ^ (((row >> 3) & 1) * 3)) << 4);
}

template <typename TO> struct Store4;
template <> struct Store4<float> {
    static __device__ __forceinline__ void st(float* p, const float* v) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
    static __device__ __forceinline__ void ld(const float* p, float* v) {
        float4 t = *reinterpret_cast<const float4*>(p);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    }
};
template <> struct Store4<bf16_t> {
    static __device__ __forceinline__ void st(bf16_t* p, const float* v) {
        ushort4 o;
        o.x = f2bf(v[0]); o.y = f2bf(v[1]); o.z = f2bf(v[2]); o.w = f2bf(v[3]);
        *reinterpret_cast<ushort4*>(p) = o;
    }
    static __device__ __forceinline__ void ld(const bf16_t* p, float* v) {
        ushort4 t = *reinterpret_cast<const ushort4*>(p);
        v[0] = bf2f(t.x); v[1] = bf2f(t.y); v[2] = bf2f(t.z); v[3] = bf2f(t.w);
    }
};

template <typename T, typename TO, int TC, int TP, int WC, int WP, bool K1>
__global__ void __launch_bounds__(256) k_conv(ConvArgs a) {
    constexpr int VEC = Vec<T>::N;
    constexpr int BK = 4 * VEC;  // elements per K-step: 64 bytes per row
    constexpr int CA = TC * 4, CB = TP * 4;
    constexpr int NA = (CA + 255) / 256, NB = (CB + 255) / 256;
    constexpr int FM = TC / WC / 16, FN = TP / WP / 16;
    static_assert(WC * WP == 4, "4 waves");
    static_assert(FM >= 1 && FN >= 1, "tile too small");

    __shared__ __attribute__((aligned(16))) char smem[2 * (TC + TP) * 64];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wc = wave % WC, wp = wave / WC;
    const int c0 = blockIdx.y * TC, p0 = blockIdx.x * TP;
    const T* __restrict__ X = (const T*)a.x;
    const T* __restrict__ Wt = (const T*)a.w;
    const int H = a.h, W = a.w_, Cin = a.cin;

    // ---- per-thread staging descriptors
    long long a_base[NA];
    bool a_ok[NA];
    int a_off[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        int q = tid + i * 256;
        int row = q >> 2, kc = q & 3;
        a_ok[i] = (q < CA) && (c0 + row < a.cout);
        a_base[i] = (long long)(c0 + row) * a.kp + kc * VEC;
        a_off[i] = lds_off(row, kc);
    }
    long long b_base[NB];
    int b_hi[NB], b_wi[NB], b_kc[NB], b_off[NB];
    bool b_ok[NB], b_in[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        int q = tid + i * 256;
        int row = q >> 2, kc = q & 3;
        int p = p0 + row;
        b_in[i] = q < CB;
        b_ok[i] = b_in[i] && p < a.P;
        int pp = b_ok[i] ? p : 0;
        int img = pp / (a.ho * a.wo);
        int rem = pp - img * (a.ho * a.wo);
        int oh = rem / a.wo, ow = rem - oh * a.wo;
        b_hi[i] = oh * a.stride - a.pad;
        b_wi[i] = ow * a.stride - a.pad;
        b_kc[i] = kc;
        b_base[i] = (long long)img * H * W * Cin;
        if (K1) b_base[i] += ((long long)b_hi[i] * W + b_wi[i]) * Cin + kc * VEC;
        b_off[i] = lds_off(row, kc);
    }

    uint4 ra[NA], rb[NB];
    const uint4 zero4 = make_uint4(0, 0, 0, 0);

    auto gload = [&](int k0) {
#pragma unroll
        for (int i = 0; i < NA; ++i)
            ra[i] = a_ok[i] ? *reinterpret_cast<const uint4*>(Wt + a_base[i] + k0) : zero4;
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            if (K1) {
                rb[i] = b_ok[i] ? *reinterpret_cast<const uint4*>(X + b_base[i] + k0) : zero4;
            } else {
                int k = k0 + b_kc[i] * VEC;
                int tap = k >> a.lc;
                int ci = k & (Cin - 1);
                int kh = tap / a.kw;
                int kw = tap - kh * a.kw;
                int hi = b_hi[i] + kh * a.dil, wi = b_wi[i] + kw * a.dil;
                bool ok = b_ok[i] && kh < a.kh && hi >= 0 && hi < H && wi >= 0 && wi < W;
                rb[i] = ok ? *reinterpret_cast<const uint4*>(X + b_base[i] + ((long long)hi * W + wi) * Cin + ci)
                           : zero4;
            }
        }
    };
    auto sstore = [&](int buf) {
        char* As = smem + buf * (TC + TP) * 64;
        char* Bs = As + TC * 64;
#pragma unroll
        for (int i = 0; i < NA; ++i)
            if (tid + i * 256 < CA) *reinterpret_cast<uint4*>(As + a_off[i]) = ra[i];
#pragma unroll
        for (int i = 0; i < NB; ++i)
            if (b_in[i]) *reinterpret_cast<uint4*>(Bs + b_off[i]) = rb[i];
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const int nk = a.kp / BK;
    const int r16 = lane & 15, kq = lane >> 4;
    int fa_off[FM], fb_off[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) fa_off[i] = lds_off(wc * (TC / WC) + i * 16 + r16, kq);
#pragma unroll
    for (int j = 0; j < FN; ++j) fb_off[j] = lds_off(wp * (TP / WP) + j * 16 + r16, kq);

    gload(0);
    sstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) gload((kt + 1) * BK);
        const char* As = smem + cur * (TC + TP) * 64;
        const char* Bs = As + TC * 64;
        uint4 fa[FM], fb[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[i] = *reinterpret_cast<const uint4*>(As + fa_off[i]);
#pragma unroll
        for (int j = 0; j < FN; ++j) fb[j] = *reinterpret_cast<const uint4*>(Bs + fb_off[j]);
        if constexpr (VEC == 8) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        __builtin_bit_cast(bf16x8, fa[i]), __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        float av = __uint_as_float(s == 0 ? fa[i].x : s == 1 ? fa[i].y : s == 2 ? fa[i].z : fa[i].w);
                        float bv = __uint_as_float(s == 0 ? fb[j].x : s == 1 ? fb[j].y : s == 2 ? fb[j].z : fb[j].w);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[i][j], 0, 0, 0);
                    }
        }
        if (kt + 1 < nk) sstore(cur ^ 1);
        __syncthreads();
    }

    // ---- fused epilogue: 4 consecutive channels of one pixel per lane
    TO* __restrict__ Y = (TO*)a.y;
    const TO* __restrict__ R = (const TO*)a.res;
    const bool affine = a.flags & RR_CONV_AFFINE;
    const bool resid = a.flags & RR_CONV_RESIDUAL;
    const bool leaky = a.act == RR_ACT_LEAKY;
    if (a.flags & RR_CONV_PERM32) {  // rows are permuted: scalar path through perm32_channel
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int p = p0 + wp * (TP / WP) + j * 16 + r16;
                if (p >= a.P) continue;
                for (int r = 0; r < 4; ++r) {
                    const int row = c0 + wc * (TC / WC) + i * 16 + 4 * kq + r;
                    if (row >= a.cout) continue;
                    const int c = perm32_channel(row);
                    const long long o = (long long)p * a.ldy + c;
                    float t = acc[i][j][r];
                    if (affine) t = t * a.scale[c] + a.shift[c];
                    if (resid) t += DT<TO>::to_f(R[o]);
                    if (leaky) t = t > 0.f ? t : t * a.slope;
                    Y[o] = DT<TO>::from_f(t);
                }
            }
        return;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        const int c = c0 + wc * (TC / WC) + i * 16 + 4 * kq;
        if (c >= a.cout) continue;
        float sc[4] = {1.f, 1.f, 1.f, 1.f}, sh[4] = {0.f, 0.f, 0.f, 0.f};
        const bool full = (c + 3 < a.cout);
        if (affine) {
            if (full) {
                Store4<float>::ld(a.scale + c, sc);
                Store4<float>::ld(a.shift + c, sh);
            } else {
                for (int r = 0; r < 4; ++r)
                    if (c + r < a.cout) { sc[r] = a.scale[c + r]; sh[r] = a.shift[c + r]; }
            }
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int p = p0 + wp * (TP / WP) + j * 16 + r16;
            if (p >= a.P) continue;
            float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
            const long long o = (long long)p * a.ldy + c;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = v[r] * sc[r] + sh[r];
            if (full) {
                if (resid) {
                    float rv[4];
                    Store4<TO>::ld(R + o, rv);
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] += rv[r];
                }
                if (leaky) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
                }
                Store4<TO>::st(Y + o, v);
            } else {
                for (int r = 0; r < 4; ++r) {
                    if (c + r >= a.cout) break;
                    float t = v[r];
                    if (resid) t += DT<TO>::to_f(R[o + r]);
                    if (leaky) t = t > 0.f ? t : t * a.slope;
                    Y[o + r] = DT<TO>::from_f(t);
                }
            }
        }
    }
}

template <typename T, typename TO, int TC, int TP, int WC, int WP>
static void launch_cfg(const ConvArgs& a, bool k1, hipStream_t s) {
    dim3 grid((a.P + TP - 1) / TP, (a.cout + TC - 1) / TC);
    if (k1)
        hipLaunchKernelGGL((k_conv<T, TO, TC, TP, WC, WP, true>), grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((k_conv<T, TO, TC, TP, WC, WP, false>), grid, dim3(256), 0, s, a);
}

template <typename T, typename TO>
static void launch(const ConvArgs& a, bool k1, hipStream_t s) {
    if (a.P <= 32)
        launch_cfg<T, TO, 256, 32, 4, 1>(a, k1, s);
    else if (a.P <= 64)
        launch_cfg<T, TO, 256, 64, 4, 1>(a, k1, s);
    else if (a.cout <= 64)
        launch_cfg<T, TO, 64, 256, 1, 4>(a, k1, s);
    else
        launch_cfg<T, TO, 128, 128, 2, 2>(a, k1, s);
}

template <typename T, typename TO> void launch_gemm2(const ConvArgs& a, bool k1, hipStream_t s);
extern int g_knn_fused;  // rr_knn.hip
bool launch_stream1x1(const ConvArgs& a, hipStream_t s, bool f16);  // rr_stream.hip
bool launch_conv3x3(const ConvArgs& a, hipStream_t s, bool f16);    // rr_conv3.hip
extern int g_stream_mode;
extern int g_conv3_mode;
extern int g_conv3_pipe;
extern int g_stem_mode;
extern int g_stream_xcd;
extern int g_conv3s;
extern int g_wres;
extern int g_pair_mid;
extern int g_wres_ring;

// out[R][k] = w[chan(R)][ci][kh][kw] with k = (kh*KW + kw)*cin_pad + ci, zeros elsewhere.
template <typename T>
__global__ void k_pack_conv(const float* __restrict__ w, int cout, int cin, int kh, int kw, int cin_pad, int kp,
                            int perm, T* __restrict__ out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)cout * kp) return;
    const int R = (int)(i / kp), k = (int)(i - (long long)R * kp);
    const int co = perm ? perm32_channel(R) : R;
    const int tap = k / cin_pad, ci = k - tap * cin_pad;
    float v = 0.f;
    if (tap < kh * kw && ci < cin) {
        const int y = tap / kw, x = tap - y * kw;
        v = w[(((long long)co * cin + ci) * kh + y) * kw + x];
    }
    out[i] = DT<T>::from_f(v);
}

// v2 (LDS-DMA) engine eligibility: 128-byte K-steps and 31-bit buffer offsets.
static bool use_v2(const ConvArgs& a, int dtype) {
    static int forced = -1;
    if (forced < 0) {
        const char* e = getenv("RR_GEMM_V1");
        forced = (e && e[0] == '1') ? 1 : 0;
    }
    if (forced == 1) return false;
    const int esz = dtype == RR_F32 ? 4 : 2;
    const long long xbytes = (long long)a.n * a.h * a.w_ * a.cin * esz;
    return (a.kp * esz) % 128 == 0 && xbytes < (1ll << 31) && (long long)256 * a.kp * esz < (1ll << 31);
}

template <typename T, typename TO>
static int dispatch(const ConvArgs& a, bool k1, int dtype, hipStream_t s) {
    if constexpr (sizeof(T) == 2 && std::is_same<T, TO>::value) {  // bf16 / fp16 fused kernels
        constexpr bool f16 = std::is_same<T, f16_t>::value;
        if (k1 && launch_stream1x1(a, s, f16)) return RR_OK;
        if (!k1 && launch_conv3x3(a, s, f16)) return RR_OK;
    }
    if constexpr (std::is_same<T, f16_t>::value) {  // fp16: the LDS-DMA engine only
        if ((a.kp * 2) % 128 || 256ll * a.kp * 2 >= (1ll << 31))
            return fail(RR_EINVAL, "rr_conv2d_fused: fp16 needs 128-byte K-steps (k_packed % 64 == 0)");
        // the engine addresses x through a 31-bit buffer offset: split the batch
        // into image groups below 2 GiB of input (y / residual are plain pointers)
        const long long img_bytes = (long long)a.h * a.w_ * a.cin * 2;
        if (img_bytes >= (1ll << 31)) return fail(RR_EINVAL, "rr_conv2d_fused: one fp16 input image exceeds 2 GiB");
        const int per = (int)(((1ll << 31) - 1) / img_bytes);
        const long long opx = (long long)a.ho * a.wo;
        for (int n0 = 0; n0 < a.n; n0 += per) {
            ConvArgs c = a;
            c.n = a.n - n0 < per ? a.n - n0 : per;
            c.x = (const char*)a.x + n0 * img_bytes;
            c.y = (char*)a.y + n0 * opx * a.ldy * (long long)sizeof(TO);
            if (a.res) c.res = (const char*)a.res + n0 * opx * a.ldy * (long long)sizeof(TO);
            c.P = (int)(c.n * opx);
            launch_gemm2<T, TO>(c, k1, s);
        }
    } else {
        if (use_v2(a, dtype)) launch_gemm2<T, TO>(a, k1, s);
        else launch<T, TO>(a, k1, s);
    }
    return RR_OK;
}

void gemm_scores(const ConvArgs& a, int dtype, hipStream_t s) {
    if (dtype == RR_BF16) dispatch<bf16_t, float>(a, true, dtype, s);
    else if (dtype == RR_F16) dispatch<f16_t, float>(a, true, dtype, s);  // d >= 64: 128-B K-steps
    else dispatch<float, float>(a, true, dtype, s);
}

}  // namespace rr

using namespace rr;

extern "C" int rr_conv2d_fused(const void* x, const void* w, const float* scale, const float* shift,
                               const void* residual, void* y, const rr_conv_desc* d, int dtype, int out_dtype,
                               void* stream) {
    if (!d) return fail(RR_EINVAL, "rr_conv2d_fused: null desc");
    if (d->c_in <= 0 || (d->c_in & (d->c_in - 1))) return fail(RR_EINVAL, "rr_conv2d_fused: c_in must be a power of two");
    const int vec = dtype == RR_F32 ? 4 : 8;
    if (d->c_in < vec) return fail(RR_EINVAL, "rr_conv2d_fused: c_in below one 16-byte chunk");
    if (d->k_packed % (4 * vec) != 0 || d->k_packed < d->kh * d->kw * d->c_in)
        return fail(RR_EINVAL, "rr_conv2d_fused: k_packed must cover kh*kw*c_in and be a multiple of 64 bytes");
    if (d->ldy < d->c_out || (d->ldy % 4) != 0) return fail(RR_EINVAL, "rr_conv2d_fused: ldy");
    if ((d->flags & RR_CONV_AFFINE) && (!scale || !shift)) return fail(RR_EINVAL, "rr_conv2d_fused: affine needs scale/shift");
    if ((d->flags & RR_CONV_RESIDUAL) && !residual) return fail(RR_EINVAL, "rr_conv2d_fused: residual pointer");
    const long long P = (long long)d->n * d->ho * d->wo;
    if (P <= 0 || P > 0x7fffffffll) return fail(RR_EINVAL, "rr_conv2d_fused: pixel count");
    if ((long long)(d->c_out + 255) / 256 > 65535) return fail(RR_EINVAL, "rr_conv2d_fused: c_out too large");
    if (d->ho != (d->h + 2 * d->pad - d->dil * (d->kh - 1) - 1) / d->stride + 1 ||
        d->wo != (d->w + 2 * d->pad - d->dil * (d->kw - 1) - 1) / d->stride + 1)
        return fail(RR_EINVAL, "rr_conv2d_fused: output size inconsistent with kernel/stride/pad");

    ConvArgs a{};
    a.x = x; a.w = w; a.scale = scale; a.shift = shift; a.res = residual; a.y = y;
    a.n = d->n; a.h = d->h; a.w_ = d->w; a.cin = d->c_in; a.ho = d->ho; a.wo = d->wo; a.cout = d->c_out;
    a.kh = d->kh; a.kw = d->kw; a.stride = d->stride; a.pad = d->pad; a.dil = d->dil; a.kp = d->k_packed;
    a.ldy = d->ldy; a.act = d->act; a.flags = d->flags; a.slope = d->slope;
    a.lc = __builtin_ctz((unsigned)d->c_in);
    a.P = (int)P;
    // 1x1 / pad 0: every K-run of a pixel is contiguous -> no im2col index math.
    const bool k1 = d->kh == 1 && d->kw == 1 && d->pad == 0 && d->k_packed == d->c_in;
    hipStream_t s = as_stream(stream);
    int rc;
    if (dtype == RR_BF16 && out_dtype == RR_BF16) rc = dispatch<bf16_t, bf16_t>(a, k1, dtype, s);
    else if (dtype == RR_BF16 && out_dtype == RR_F32) rc = dispatch<bf16_t, float>(a, k1, dtype, s);
    else if (dtype == RR_F16 && out_dtype == RR_F16) rc = dispatch<f16_t, f16_t>(a, k1, dtype, s);
    else if (dtype == RR_F16 && out_dtype == RR_F32) rc = dispatch<f16_t, float>(a, k1, dtype, s);
    else if (dtype == RR_F32 && out_dtype == RR_F32) rc = dispatch<float, float>(a, k1, dtype, s);
    else return fail(RR_EINVAL, "rr_conv2d_fused: unsupported dtype pair");
    if (rc) return rc;
    return check_launch("rr_conv2d_fused");
}

extern "C" int rr_pack_conv_weights(const float* w, int c_out, int c_in, int kh, int kw, int c_in_pad, int k_packed,
                                    int perm32, void* out, int dtype, void* stream) {
    if (c_out <= 0 || c_in <= 0 || c_in_pad < c_in || k_packed < kh * kw * c_in_pad)
        return fail(RR_EINVAL, "rr_pack_conv_weights: bad shape");
    if (perm32 && (c_out % 32)) return fail(RR_EINVAL, "rr_pack_conv_weights: perm32 needs c_out % 32 == 0");
    const long long total = (long long)c_out * k_packed;
    const unsigned blocks = (unsigned)((total + 255) / 256);
    if (dtype == RR_BF16)
        hipLaunchKernelGGL(k_pack_conv<bf16_t>, dim3(blocks), dim3(256), 0, as_stream(stream), w, c_out, c_in, kh, kw,
                           c_in_pad, k_packed, perm32, (bf16_t*)out);
    else if (dtype == RR_F16)
        hipLaunchKernelGGL(k_pack_conv<f16_t>, dim3(blocks), dim3(256), 0, as_stream(stream), w, c_out, c_in, kh, kw,
                           c_in_pad, k_packed, perm32, (f16_t*)out);
    else if (dtype == RR_F32)
        hipLaunchKernelGGL(k_pack_conv<float>, dim3(blocks), dim3(256), 0, as_stream(stream), w, c_out, c_in, kh, kw,
                           c_in_pad, k_packed, perm32, (float*)out);
    else
        return fail(RR_EINVAL, "rr_pack_conv_weights: dtype");
    return check_launch("rr_pack_conv_weights");
}

namespace rr {
void set_gemm_tuning(int key, int value);
}
extern "C" int rr_set_tuning(int key, int value) {
    if (key < 0 || key > 16) return fail(RR_EINVAL, "rr_set_tuning: unknown key");
    if (key == RR_TUNE_KNN_FUSED) {
        rr::g_knn_fused = value != 0;
        return RR_OK;
    }
    if (key == RR_TUNE_GRID_CUS) {
        if (value < 0) return fail(RR_EINVAL, "rr_set_tuning: RR_TUNE_GRID_CUS must be >= 0");
        rr::g_grid_cap = value;
        return RR_OK;
    }
    if (key == RR_TUNE_STREAM_1X1) rr::g_stream_mode = value;
    else if (key == RR_TUNE_CONV3X3) rr::g_conv3_mode = value;
    else if (key == RR_TUNE_CONV3_PIPE) rr::g_conv3_pipe = value;
    else if (key == RR_TUNE_STEM) rr::g_stem_mode = value;
    else if (key == RR_TUNE_STREAM_XCD) rr::g_stream_xcd = value;
    else if (key == RR_TUNE_CONV3S) rr::g_conv3s = value;
    else if (key == RR_TUNE_WRES) rr::g_wres = value;
    else if (key == RR_TUNE_PAIR_MID) rr::g_pair_mid = value;
    else if (key == RR_TUNE_WRES_RING) rr::g_wres_ring = value;
    else rr::set_gemm_tuning(key, value);
    return RR_OK;
}
