// librr.so — fused ResNet stem (bf16): normalise + conv1 7x7/s2/p3 (3 -> 64)
// + BN affine + activation + max-pool 3x3/s2/p1, one kernel.
//
// Replaces the reference's mod1 = Sequential(conv1, bn1, pool1)
// (cirtorch/backbones/resnet.py:59-66) fed by utils/image.py:125 `normalize`.
// The unfused path moves the 64-channel stride-2 map through HBM twice
// (conv write + pool read: 4x the pooled bytes) and runs the 7x7 im2col
// through the generic LDS-DMA engine at 8 padded channels per tap.
//
// Layout of the work, per block (one per CU, persistent over tiles):
//   * pooled tile PH x PW  <-  stem tile (2PH+1) x (2PW+1)  <-  input patch
//     (4PH+7) x (4PW+8) pixels of the fp32 NCHW image, normalised on the fly
//     and staged in LDS as bf16 [row][col][4 ch] (8 B / pixel, channel 3 = 0);
//     the next tile's patch is fetched into VGPRs while this tile computes;
//   * K = 7 kh x 8 kw x 4 ch = 224 (kw = 7 and ch = 3 carry zero weights), so
//     an MFMA K-step is one kernel row and a lane's 8 k-values are two
//     horizontally adjacent input pixels: one aligned 16-B ds_read;
//   * weights (PERM32 row order, [64][256] bf16) live in VGPRs for the whole
//     launch (4 channel fragments x 7 K-steps);
//   * epilogue: BN + activation -> bf16 stem tile in LDS (-inf outside the
//     stem map, i.e. max-pool padding), then the 3x3/s2 max, 16-B stores.
// Results equal the unfused path up to fp32 summation order inside the conv
// (the max-pool is exact on the same bf16 values).
#include "rr_internal.h"

#include <type_traits>

namespace rr {

namespace {

typedef __attribute__((ext_vector_type(4))) float tf32x4_t;

struct StemArgs {
    const void* x;    // [n][3][h][w] float32, or uint8 pixels (value / 255, torchvision ToTensor)
    const uint4* w;   // [64][256] bf16 (as 16-B chunks), PERM32 rows, k = kh*32 + kw*4 + ci
    const float* scale;
    const float* shift;
    bf16_t* y;        // [n][hp][wp][64]
    int n, h, w_, ho, wo, hp, wp;
    float mean[3], rstd[3];  // rstd = 1 / std (rounded once on the host)
    int do_norm, leaky;
    float slope;
};

constexpr int NT = 512;  // threads per block (8 waves)
// packed stem weights: [64 rows (PERM32)][448] 16-bit = 56 x 16-B chunks per row:
// k < 256: kernel-row layout (k = kh*32 + kw*4 + ci) of v1-v3; k in [256, 448):
// the space-to-depth layout of v4 (k' = kr*48 + kc*12 + a*6 + b*3 + ci, kh = 2kr + a,
// kw = 2kc + b)
constexpr int WROW = 56, W4OFF = 32;

typedef __attribute__((ext_vector_type(2))) short short2v;

// Two packed bf16 -> order-preserving int16 keys (and back: the map is an
// involution): negative values get their magnitude bits flipped, so signed
// 16-bit order == float order; max-pool then runs on v_pk_max_i16.
__device__ __forceinline__ unsigned bf16_key2(unsigned w) {
    const unsigned neg = (w >> 15) & 0x00010001u;
    return w ^ (neg * 0x7FFFu);
}

template <int PH, int PW, typename HT, bool U8 = false, typename TAB = NoTab>
__global__ void __launch_bounds__(NT) k_stem_pool(StemArgs a, TAB rt, int tiles_w, int tiles_hw, int ntiles) {
    constexpr bool RG = std::is_same<TAB, RaggedTab>::value;
    constexpr int SR = 2 * PH + 1, SC = 2 * PW + 1, NP = SR * SC, NF = (NP + 15) / 16;
    constexpr unsigned KNI = H16<HT>::NEG_INF ^ 0x7FFFu;  // order key of -inf (pool padding)
    constexpr unsigned KNI2 = KNI | (KNI << 16);
    constexpr int IR = 2 * (SR - 1) + 7, IC = 2 * (SC - 1) + 8;  // IC even: 16-B aligned pixel pairs
    constexpr int NSLOT = IR * IC, SPT = (NSLOT + NT - 1) / NT;
    constexpr int PATCH = NSLOT * 8;
    static_assert(IC % 2 == 0, "pixel pairs");
    __shared__ __attribute__((aligned(16))) char sP[2][PATCH];
    __shared__ __attribute__((aligned(16))) char sO[NF * 16 * 128];
    __shared__ __attribute__((aligned(16))) float sS[64], sH[64];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int H = a.h, W = a.w_;
    const long long plane = (long long)H * W;

    if (tid < 64) {
        sS[tid] = a.scale[tid];
        sH[tid] = a.shift[tid];
    }
    // weights -> VGPRs: fragment i (packed rows 16i..16i+15), K-step m
    uint4 areg[4][7];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int m = 0; m < 7; ++m) areg[i][m] = a.w[(i * 16 + r16) * WROW + m * 4 + q];

    auto tile_origin = [&](int t, int& img, int& ph0, int& pw0) {
        img = t / tiles_hw;
        const int rem = t - img * tiles_hw;
        const int th = rem / tiles_w;
        ph0 = th * PH;
        pw0 = (rem - th * tiles_w) * PW;
    };

    float pf[SPT][3];
    auto fill_load = [&](int t) {
        int img, ph0, pw0;
        tile_origin(t, img, ph0, pw0);
        const int ir0 = 4 * ph0 - 5, ic0 = 4 * pw0 - 5;  // = 2 * (2 * p0 - 1) - 3
        // the image's own extent (ragged: its pixels at its own address; map pixels
        // past it read 0 -- the batch pad, normalised in fill_store)
        const void* ib = a.x;
        int hi = H, wi = W;
        long long ibase = (long long)img * 3 * plane, iplane = plane;
        if constexpr (RG) {
            ib = rt.p[img];
            hi = rt.h[img];
            wi = rt.w[img];
            ibase = 0;
            iplane = (long long)hi * wi;
        }
#pragma unroll
        for (int u = 0; u < SPT; ++u) {
            const int slot = tid + NT * u;
            const int r = slot / IC, c = slot - r * IC;
            const int ih = ir0 + r, iw = ic0 + c;
            const bool ok = slot < NSLOT && (unsigned)ih < (unsigned)hi && (unsigned)iw < (unsigned)wi;
            const long long o = ok ? (long long)ih * wi + iw : 0;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                if constexpr (U8)  // IEEE division: the same float as torch's / numpy's x / 255
                    pf[u][ch] = ok ? (float)((const unsigned char*)ib)[ibase + ch * iplane + o] / 255.f : 0.f;
                else
                    pf[u][ch] = ok ? ((const float*)ib)[ibase + ch * iplane + o] : 0.f;
            }
        }
    };
    auto fill_store = [&](int t, int buf) {
        int img, ph0, pw0;
        tile_origin(t, img, ph0, pw0);
        const int ir0 = 4 * ph0 - 5, ic0 = 4 * pw0 - 5;
#pragma unroll
        for (int u = 0; u < SPT; ++u) {
            const int slot = tid + NT * u;
            if (slot >= NSLOT) continue;
            const int r = slot / IC, c = slot - r * IC;
            const bool ok = (unsigned)(ir0 + r) < (unsigned)H && (unsigned)(ic0 + c) < (unsigned)W;
            float v[3];
#pragma unroll
            for (int ch = 0; ch < 3; ++ch)  // zero padding is applied AFTER normalisation
                v[ch] = (ok && a.do_norm) ? (pf[u][ch] - a.mean[ch]) * a.rstd[ch] : pf[u][ch];
            uint2 o;
            o.x = H16<HT>::pack2(v[0], v[1]);
            o.y = H16<HT>::pack2(v[2], 0.f);
            *reinterpret_cast<uint2*>(sP[buf] + slot * 8) = o;
        }
    };

    int t = blockIdx.x;
    if (t >= ntiles) return;
    fill_load(t);
    fill_store(t, 0);
    __syncthreads();
    int cur = 0;
    for (; t < ntiles; t += gridDim.x, cur ^= 1) {
        const int tn = t + gridDim.x;
        if (tn < ntiles) fill_load(tn);
        int img, ph0, pw0;
        tile_origin(t, img, ph0, pw0);
        const int sr0 = 2 * ph0 - 1, sc0 = 2 * pw0 - 1;
        const char* patch = sP[cur];
        for (int f = wave; f < NF; f += NT / 64) {
            const int n = f * 16 + r16;
            const int nn = n < NP ? n : NP - 1;
            const int sr = nn / SC, sc = nn - sr * SC;
            const char* pb = patch + ((2 * sr) * IC + 2 * sc + 2 * q) * 8;
            tf32x4_t acc[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] = (tf32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int m = 0; m < 7; ++m) {
                const uint4 b = *reinterpret_cast<const uint4*>(pb + m * IC * 8);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[i] = H16<HT>::mfma(areg[i][m], b, acc[i]);
            }
            const bool valid = (unsigned)(sr0 + sr) < (unsigned)a.ho && (unsigned)(sc0 + sc) < (unsigned)a.wo;
            if (n < NP) {
#pragma unroll
                for (int i2 = 0; i2 < 2; ++i2) {
                    const int cl = 32 * i2 + 8 * q;  // 8 consecutive channels (PERM32 rows)
                    float v[8];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] = acc[2 * i2][r] * sS[cl + r] + sH[cl + r];
                        v[4 + r] = acc[2 * i2 + 1][r] * sS[cl + 4 + r] + sH[cl + 4 + r];
                    }
                    if (a.leaky) {  // slope in [0, 1] (host-checked): leaky(v) = max(v, slope * v)
#pragma unroll
                        for (int r = 0; r < 8; ++r) v[r] = fmaxf(v[r], v[r] * a.slope);
                    }
                    uint4 o;
                    if (valid) {
                        o.x = bf16_key2(H16<HT>::pack2(v[0], v[1]));
                        o.y = bf16_key2(H16<HT>::pack2(v[2], v[3]));
                        o.z = bf16_key2(H16<HT>::pack2(v[4], v[5]));
                        o.w = bf16_key2(H16<HT>::pack2(v[6], v[7]));
                    } else {
                        o = make_uint4(KNI2, KNI2, KNI2, KNI2);  // key(-inf): pool padding
                    }
                    const int chunk = 4 * i2 + q;
                    *reinterpret_cast<uint4*>(sO + n * 128 + ((chunk ^ (n & 7)) << 4)) = o;
                }
            }
        }
        if (tn < ntiles) fill_store(tn, cur ^ 1);
        __syncthreads();
        // 3x3 / s2 max over the stem tile; item = (pooled pixel, 8-channel chunk)
#pragma unroll
        for (int it = 0; it < (PH * PW * 8 + NT - 1) / NT; ++it) {
            const int item = tid + NT * it;
            if (item >= PH * PW * 8) break;
            const int c = item & 7, pp = item >> 3;
            const int pr = pp / PW, pc = pp - pr * PW;
            if (ph0 + pr >= a.hp || pw0 + pc >= a.wp) continue;
            // max over the 9 taps on order-preserving int16 keys of the bf16 values,
            // two channels per v_pk_max_i16
            short2v mx[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) mx[j] = (short2v){(short)KNI, (short)KNI};
#pragma unroll
            for (int dr = 0; dr < 3; ++dr)
#pragma unroll
                for (int dc = 0; dc < 3; ++dc) {
                    const int n = (2 * pr + dr) * SC + 2 * pc + dc;
                    const uint4 v = *reinterpret_cast<const uint4*>(sO + n * 128 + ((c ^ (n & 7)) << 4));
                    mx[0] = __builtin_elementwise_max(mx[0], __builtin_bit_cast(short2v, v.x));
                    mx[1] = __builtin_elementwise_max(mx[1], __builtin_bit_cast(short2v, v.y));
                    mx[2] = __builtin_elementwise_max(mx[2], __builtin_bit_cast(short2v, v.z));
                    mx[3] = __builtin_elementwise_max(mx[3], __builtin_bit_cast(short2v, v.w));
                }
            uint4 o;
            o.x = bf16_key2(__builtin_bit_cast(unsigned, mx[0]));
            o.y = bf16_key2(__builtin_bit_cast(unsigned, mx[1]));
            o.z = bf16_key2(__builtin_bit_cast(unsigned, mx[2]));
            o.w = bf16_key2(__builtin_bit_cast(unsigned, mx[3]));
            *reinterpret_cast<uint4*>(a.y + (((long long)img * a.hp + ph0 + pr) * a.wp + pw0 + pc) * 64 + 8 * c) = o;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Stem v2: pool BEFORE the epilogue.  f(v) = round16(act(|s| * v + h)) is
// non-decreasing in v (fma with |s| >= 0, leaky with slope in [0, 1], RNE),
// so max-pool(f(conv)) == f(max-pool(conv)) exactly.  Output channels whose
// BN scale is negative get their weight rows negated when the fragments are
// loaded (bf16/fp16 negation and the MFMA sum are sign-symmetric, so the
// accumulator is exactly -conv) and use |s|: every value equals the select-
// form result of k_stem_pool bit for bit, and BN + activation + packing run
// on the 4x fewer pooled pixels only.
// Work layout: a tile is PH = 8 pooled rows x PW = 56 pooled cols; wave w
// owns stem columns 14w .. 14w + 15 (one 16-pixel B fragment per stem row,
// 2 columns of overlap: 7 pooled columns) and walks the 17 stem rows top to
// bottom: the vertical 3-max of each pooled row is a per-lane max3 over the
// accumulators of 3 consecutive stem rows (kept in VGPRs), the horizontal
// 3-max two DPP row shifts (lane i <- lanes i+1, i+2 of the 16-pixel row).
// No LDS round trip and no barrier for the pooling; one barrier per tile for
// the double-buffered input patch (normalised fp32 -> packed 16-bit,
// [row][col][4 ch], 39 x 234 pixels).
template <typename HT, bool U8>
__global__ void __launch_bounds__(NT) k_stem_pool2(StemArgs a, int tiles_w, int tiles_hw, int ntiles) {
    constexpr int PH = 8, PW = 56, SRN = 2 * PH + 1, CB = 14;
    constexpr int IR = 2 * (SRN - 1) + 7;            // 39 input rows
    constexpr int SCN = CB * 7 + 16;                 // 114 stem columns
    constexpr int IC = 2 * (SCN - 1) + 8;            // 234 input columns (even: 16-B pixel pairs)
    constexpr int HIC = IC / 2;
    constexpr int NPAIR = IR * HIC, PPT = (NPAIR + NT - 1) / NT;
    constexpr int PATCH = IR * IC * 8;
    static_assert(PW == 7 * (NT / 64), "one 7-pooled-column block per wave");
    __shared__ __attribute__((aligned(16))) char sP[2][PATCH];
    __shared__ __attribute__((aligned(16))) float sS[64], sH[64];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int H = a.h, W = a.w_;
    const long long plane = (long long)H * W;

    if (tid < 64) {
        sS[tid] = fabsf(a.scale[tid]);
        sH[tid] = a.shift[tid];
    }
    // weights -> VGPRs (fragment i = packed rows 16i .. 16i+15, K-step m = kernel row),
    // rows of negative-scale channels negated (sign bit of every 16-bit element)
    uint4 areg[4][7];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const unsigned flip = a.scale[perm32_channel(i * 16 + r16)] < 0.f ? 0x80008000u : 0u;
#pragma unroll
        for (int m = 0; m < 7; ++m) {
            uint4 w = a.w[(i * 16 + r16) * WROW + m * 4 + q];
            w.x ^= flip; w.y ^= flip; w.z ^= flip; w.w ^= flip;
            areg[i][m] = w;
        }
    }

    auto tile_origin = [&](int t, int& img, int& ph0, int& pw0) {
        img = t / tiles_hw;
        const int rem = t - img * tiles_hw;
        const int th = rem / tiles_w;
        ph0 = th * PH;
        pw0 = (rem - th * tiles_w) * PW;
    };

    // patch fill: pixel pairs (2 adjacent input columns) -> one 16-B LDS store;
    // in two halves (pairs u < PH1, u >= PH1) so only half the raw pixels are
    // live in VGPRs while the MFMAs run
    constexpr int PH1 = (PPT + 1) / 2;
    float pf[PH1][6];
    auto fill_load = [&](int t, int half) {
        int img, ph0, pw0;
        tile_origin(t, img, ph0, pw0);
        const int ir0 = 4 * ph0 - 5, ic0 = 4 * pw0 - 5;
        // one raw buffer per image (3 planes) with 32-bit offsets; a pixel outside
        // the image gets an offset past the buffer (reads 0) -- never a negative
        // one -- and is zeroed after normalisation in fill_store anyway
        constexpr int ESZ = U8 ? 1 : 4;
        constexpr unsigned OOBO = 0x80000000u;
        const char* ib = (const char*)a.x + (long long)img * 3 * plane * ESZ;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)ib, (short)0, (int)(3 * plane * ESZ), 0x00020000);
#pragma unroll
        for (int uu = 0; uu < PH1; ++uu) {
            const int u = half * PH1 + uu;
            if (u >= PPT) break;
            const int k = tid + NT * u;
            const int kk = k < NPAIR ? k : NPAIR - 1;
            const int r = kk / HIC, c = 2 * (kk - r * HIC);
            const int ih = ir0 + r, iw = ic0 + c;
            const bool rok = (unsigned)ih < (unsigned)H;
            const int o = (ih * W + iw) * ESZ;
            const unsigned off0 = rok && (unsigned)iw < (unsigned)W ? (unsigned)o : OOBO;
            const unsigned off1 = rok && (unsigned)(iw + 1) < (unsigned)W ? (unsigned)(o + ESZ) : OOBO;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                const unsigned po = (unsigned)(ch * (int)plane * ESZ);
                if constexpr (U8) {  // IEEE division: the same float as torch's / numpy's x / 255
                    pf[uu][2 * ch] = (float)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)(off0 + po), 0, 0) / 255.f;
                    pf[uu][2 * ch + 1] = (float)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)(off1 + po), 0, 0) / 255.f;
                } else {
                    pf[uu][2 * ch] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(off0 + po), 0, 0));
                    pf[uu][2 * ch + 1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(off1 + po), 0, 0));
                }
            }
        }
    };
    auto fill_store = [&](int t, int buf, int half) {
        int img, ph0, pw0;
        tile_origin(t, img, ph0, pw0);
        const int ir0 = 4 * ph0 - 5, ic0 = 4 * pw0 - 5;
#pragma unroll
        for (int uu = 0; uu < PH1; ++uu) {
            const int u = half * PH1 + uu;
            if (u >= PPT) break;
            const int k = tid + NT * u;
            if (k >= NPAIR) continue;
            const int r = k / HIC, c = 2 * (k - r * HIC);
            const bool rok = (unsigned)(ir0 + r) < (unsigned)H;
            const bool ok0 = rok && (unsigned)(ic0 + c) < (unsigned)W;
            const bool ok1 = rok && (unsigned)(ic0 + c + 1) < (unsigned)W;
            float v[6];
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {  // zero padding is applied AFTER normalisation
                const float x0 = pf[uu][2 * ch], x1 = pf[uu][2 * ch + 1];
                v[2 * ch] = ok0 ? (a.do_norm ? (x0 - a.mean[ch]) * a.rstd[ch] : x0) : 0.f;
                v[2 * ch + 1] = ok1 ? (a.do_norm ? (x1 - a.mean[ch]) * a.rstd[ch] : x1) : 0.f;
            }
            uint4 o;
            o.x = H16<HT>::pack2(v[0], v[2]);
            o.y = H16<HT>::pack2(v[4], 0.f);
            o.z = H16<HT>::pack2(v[1], v[3]);
            o.w = H16<HT>::pack2(v[5], 0.f);
            *reinterpret_cast<uint4*>(sP[buf] + (r * IC + c) * 8) = o;
        }
    };

    const float slope = a.leaky ? a.slope : 1.f;  // identity == leaky with slope 1
    const float NINF = -__builtin_inff();
    int t = blockIdx.x;
    if (t >= ntiles) return;
    fill_load(t, 0);
    fill_store(t, 0, 0);
    fill_load(t, 1);
    fill_store(t, 0, 1);
    __syncthreads();
    int cur = 0;
    for (; t < ntiles; t += gridDim.x, cur ^= 1) {
        const int tn = t + gridDim.x;
        if (tn < ntiles) fill_load(tn, 0);
        int img, ph0, pw0;
        tile_origin(t, img, ph0, pw0);
        const int cb = CB * wave;
        const char* pb = sP[cur] + (2 * (cb + r16) + 2 * q) * 8;
        // this wave's pooled columns: skip the wave when all of them lie past the map
        const bool active = pw0 + 7 * wave < a.wp;
        // even stem dims (host-checked): the only stem pixels outside the map that
        // feed stored outputs are row -1 (top tiles) and column -1 (left tiles,
        // wave 0, lane 0)
        const bool left = pw0 == 0 && wave == 0;
        auto pool_out = [&](int pr, const h16_f32x4_t (&m)[4]) {
            float hv[4][4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float v = m[i][e];
                    const float v1 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x101, 0xF, 0xF, false));
                    const float v2 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x102, 0xF, 0xF, false));
                    hv[i][e] = fmaxf(fmaxf(v, v1), v2);
                }
            const int pc = 7 * wave + (r16 >> 1);
            if ((r16 & 1) == 0 && r16 < 14 && ph0 + pr < a.hp && pw0 + pc < a.wp) {
                bf16_t* dst = a.y + (((long long)img * a.hp + ph0 + pr) * a.wp + pw0 + pc) * 64;
#pragma unroll
                for (int i2 = 0; i2 < 2; ++i2) {
                    const int cl = 32 * i2 + 8 * q;  // 8 consecutive channels (PERM32 rows)
                    float v[8];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] = hv[2 * i2][r] * sS[cl + r] + sH[cl + r];
                        v[4 + r] = hv[2 * i2 + 1][r] * sS[cl + 4 + r] + sH[cl + 4 + r];
                    }
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[r] = fmaxf(v[r], v[r] * slope);
                    uint4 o;
                    o.x = H16<HT>::pack2(v[0], v[1]);
                    o.y = H16<HT>::pack2(v[2], v[3]);
                    o.z = H16<HT>::pack2(v[4], v[5]);
                    o.w = H16<HT>::pack2(v[6], v[7]);
                    *reinterpret_cast<uint4*>(dst + cl) = o;
                }
            }
        };
        auto stem_row = [&](int r, h16_f32x4_t (&acc)[4]) {
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] = (h16_f32x4_t){0.f, 0.f, 0.f, 0.f};
            const char* rb = pb + r * (2 * IC * 8);
#pragma unroll
            for (int m = 0; m < 7; ++m) {
                const uint4 b = *reinterpret_cast<const uint4*>(rb + m * IC * 8);
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] = H16<HT>::mfma(areg[i][m], b, acc[i]);
            }
        };
        h16_f32x4_t A[4];
        if (active) {
            stem_row(0, A);
            if (ph0 == 0) {  // stem row -1: max-pool padding
#pragma unroll
                for (int i = 0; i < 4; ++i) A[i] = (h16_f32x4_t){NINF, NINF, NINF, NINF};
            }
        }
        for (int pr = 0; pr < PH; ++pr) {
            if (pr == PH / 2 && tn < ntiles) {  // first half of the next patch -> LDS, second half in flight
                fill_store(tn, cur ^ 1, 0);
                fill_load(tn, 1);
            }
            if (active) {
                h16_f32x4_t B[4], C[4], m3[4];
                stem_row(2 * pr + 1, B);
                stem_row(2 * pr + 2, C);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int e = 0; e < 4; ++e) m3[i][e] = fmaxf(fmaxf(A[i][e], B[i][e]), C[i][e]);
                if (left) {  // stem column -1 (lane 0 of wave 0): max-pool padding; the DPP
                             // shifts in pool_out then run with every lane active
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int e = 0; e < 4; ++e) m3[i][e] = r16 == 0 ? NINF : m3[i][e];
                }
                pool_out(pr, m3);
#pragma unroll
                for (int i = 0; i < 4; ++i) A[i] = C[i];
            }
        }
        if (tn < ntiles) fill_store(tn, cur ^ 1, 1);
        __syncthreads();
    }
}


// ---------------------------------------------------------------------------
// Stem v3: the v2 tile and pool-before-epilogue, with the MFMA operands
// swapped so pooling and the epilogue run lane-locally on useful values only.
// A = 16 stem pixels (rows), B = 16 output channels (columns): lane (j, q)
// holds pixels 4q..4q+3 of output channel 4j + f in fragment f.  The wave's
// 16 pixels are stem columns 14w + 4q + e: group q pools pooled columns
// 7w + 2q (its pixels e = 0,1,2) and 7w + 2q + 1 (e = 2,3 and pixel e = 0 of
// group q + 1, one ds_bpermute from lane + 16; group 3's second column belongs
// to the next wave and is dropped).  Per pooled row a lane runs 16 + 8 max3,
// BN + activation on 8 values (4 consecutive channels of 2 pooled pixels) and
// two 8-B stores -- v2 shifted 32 values by DPP and ran the epilogue on every
// lane of which 7 of 16 stored.  Per-lane channel constants live in VGPRs.
// Patch fill: float pixels are normalised as packed pairs (v_pk_add/mul_f32,
// the same IEEE operations); uint8 pixels go through a per-channel LDS table
// of the normalised value of each byte (x / 255 in IEEE division, then the
// same normalisation), computed once per block.  Same values as v2 bit for
// bit when the swapped MFMA accumulates in the same order.
// first pixel of the 8-B load that carries pixel pair (iw, iw + 1) of an image
// row of wi pixels: the pair itself inside the row, the row's first / last two
// pixels where the pair overhangs it (so a pair load never leaves its row when
// wi >= 2; a 1-pixel row loads its pixel and the next element)
__device__ __forceinline__ int pair_base(int iw, int wi) { return max(min(iw, wi - 2), 0); }

// FF (fast fill): a wave-instruction of the patch fill whose pixel pairs all lie inside the
// image row and the batch map (every pair of an interior tile, most of a border tile's) skips
// the border selects: the same values, ~1/4 of the vector instructions per pair.
template <typename HT, bool U8, int NPART, typename TAB = NoTab, bool FF = false>
__global__ void __launch_bounds__(NT) k_stem_pool3(StemArgs a, TAB rt, int tiles_w, int tiles_hw, int ntiles) {
    constexpr bool RG = std::is_same<TAB, RaggedTab>::value;
    constexpr int PH = 8, PW = 56, SRN = 2 * PH + 1, CB = 14;
    constexpr int IR = 2 * (SRN - 1) + 7;            // 39 input rows
    constexpr int SCN = CB * 7 + 16;                 // 114 stem columns
    constexpr int IC = 2 * (SCN - 1) + 8;            // 234 input columns (even: 16-B pixel pairs)
    constexpr int HIC = IC / 2;
    constexpr int NPAIR = IR * HIC, PPT = (NPAIR + NT - 1) / NT;
    constexpr int PATCH = IR * IC * 8;
    static_assert(PW == 7 * (NT / 64), "one 7-pooled-column block per wave");
    constexpr int NPRE = 2;  // K-steps of the next odd stem row read ahead (of 7)
    typedef __attribute__((ext_vector_type(2))) float f2;
    __shared__ __attribute__((aligned(16))) char sP[2][PATCH];
    __shared__ float sL[U8 ? 3 * 256 : 1];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int H = a.h, W = a.w_;
    const long long plane = (long long)H * W;

    if constexpr (U8) {
        for (int i = tid; i < 3 * 256; i += NT) {
            const int ch = i >> 8;
            const float x = (float)(i & 255) / 255.f;  // IEEE division = to_tensor
            sL[i] = a.do_norm ? (x - a.mean[ch]) * a.rstd[ch] : x;
        }
    }
    // B fragments: channel 4 * r16 + f of fragment f, K-step m = kernel row m;
    // negative-scale channels negated (pool before the epilogue, see v2)
    uint4 breg[4][7];
    float sc[4], sh[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
        const int c = 4 * r16 + f;
        const int R = (c & ~31) | (((c >> 2) & 1) << 4) | (((c >> 3) & 3) << 2) | (c & 3);  // perm32_channel^-1
        const float s = a.scale[c];
        sc[f] = fabsf(s);
        sh[f] = a.shift[c];
        const unsigned flip = s < 0.f ? 0x80008000u : 0u;
#pragma unroll
        for (int m = 0; m < 7; ++m) {
            uint4 w = a.w[R * WROW + m * 4 + q];
            w.x ^= flip; w.y ^= flip; w.z ^= flip; w.w ^= flip;
            breg[f][m] = w;
        }
    }

    auto tile_origin = [&](int t, int& img, int& ph0, int& pw0) {
        img = t / tiles_hw;
        const int rem = t - img * tiles_hw;
        const int th = rem / tiles_w;
        ph0 = th * PH;
        pw0 = (rem - th * tiles_w) * PW;
    };

    // patch fill in NPART parts, so only a third of the raw pixels is live in
    // VGPRs while the MFMAs run (v2's halves spilled ~30 VGPRs)
    constexpr int PH1 = (PPT + NPART - 1) / NPART;
    typedef typename std::conditional<U8, int, float>::type PT;
    PT pf[PH1][6];
    auto fill_load = [&](int t, int half) {
        int img, ph0, pw0;
        tile_origin(t, img, ph0, pw0);
        const int ir0 = 4 * ph0 - 5, ic0 = 4 * pw0 - 5;
        constexpr int ESZ = U8 ? 1 : 4;
        constexpr unsigned OOBO = 0x80000000u;
        // the image's own extent and planes (ragged: at its own address; map
        // pixels past its extent read 0 -- the batch pad, normalised in fill_store)
        const char* ib;
        int hi = H, wi = W;
        if constexpr (RG) {
            ib = (const char*)rt.p[img];
            hi = rt.h[img];
            wi = rt.w[img];
        } else {
            ib = (const char*)a.x + (long long)img * 3 * plane * ESZ;
        }
        const int iplane = hi * wi;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)ib, (short)0, (int)(3 * iplane * ESZ), 0x00020000);
#pragma unroll
        for (int uu = 0; uu < PH1; ++uu) {
            const int u = half * PH1 + uu;
            if (u >= PPT) break;
            int k = tid + NT * u;
            asm volatile("" : "+v"(k));  // offsets computed here, not hoisted into live VGPRs
            const int kk = k < NPAIR ? k : NPAIR - 1;
            const int r = kk / HIC, c = 2 * (kk - r * HIC);
            const int ih = ir0 + r, iw = ic0 + c;
            const bool rok = (unsigned)ih < (unsigned)hi;
            if constexpr (U8) {  // one byte load per pixel (out of the image: raw 0)
                const int o = (ih * wi + iw) * ESZ;
                const unsigned off0 = rok && (unsigned)iw < (unsigned)wi ? (unsigned)o : OOBO;
                const unsigned off1 = rok && (unsigned)(iw + 1) < (unsigned)wi ? (unsigned)(o + ESZ) : OOBO;
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
                    const unsigned po = (unsigned)(ch * iplane * ESZ);
                    pf[uu][2 * ch] = ch * 256 + (int)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)(off0 + po), 0, 0);
                    pf[uu][2 * ch + 1] = ch * 256 + (int)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)(off1 + po), 0, 0);
                }
            } else {
                // float pixels: one 8-B load per pixel pair at pair_base (fill_store
                // picks the pair's values); for a 1-pixel row the second dword may
                // pass the buffer end, which the per-dword range check reads as 0
                // (tools/oob_probe.hip) -- that value is never used
                const int bw = pair_base(iw, wi);
                const unsigned offp = rok ? (unsigned)((ih * wi + bw) * ESZ) : OOBO;
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
                    const unsigned po = (unsigned)(ch * iplane * ESZ);
                    const uint2 v2 = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(offp + po), 0, 0));
                    pf[uu][2 * ch] = __builtin_bit_cast(float, v2.x);
                    pf[uu][2 * ch + 1] = __builtin_bit_cast(float, v2.y);
                }
            }
        }
    };
    auto fill_store = [&](int t, int buf, int half) {
        int img, ph0, pw0;
        tile_origin(t, img, ph0, pw0);
        const int ir0 = 4 * ph0 - 5, ic0 = 4 * pw0 - 5;
#pragma unroll
        for (int uu = 0; uu < PH1; ++uu) {
            const int u = half * PH1 + uu;
            if (u >= PPT) break;
            int k = tid + NT * u;
            asm volatile("" : "+v"(k));
            if (k >= NPAIR) continue;
            const int r = k / HIC, c = 2 * (k - r * HIC);
            const bool rok = (unsigned)(ir0 + r) < (unsigned)H;
            const bool ok0 = rok && (unsigned)(ic0 + c) < (unsigned)W;
            const bool ok1 = rok && (unsigned)(ic0 + c + 1) < (unsigned)W;
            // float pixels (fill_load's pair loads): which loaded value is which
            // pixel; pixels outside the image row read raw 0 (the ragged batch pad)
            const int iw = ic0 + c;
            int wi = W;
            if constexpr (RG) wi = rt.w[img];
            if constexpr (FF) {
                // both pixels inside the map row and (float) inside the image row, so
                // pair_base(iw, wi) == iw: ok0 = ok1 = in0 = in1 = true, no shift --
                // the general path below reduces to exactly these operations
                const bool inner = rok && iw >= 0 && iw + 1 < (U8 ? W : wi);
                if (__builtin_amdgcn_ballot_w64(!inner) == 0) {  // every active lane (wave-uniform)
                    f2 v[3];
#pragma unroll
                    for (int ch = 0; ch < 3; ++ch) {
                        if constexpr (U8) {
                            v[ch] = (f2){sL[pf[uu][2 * ch]], sL[pf[uu][2 * ch + 1]]};
                        } else {
                            v[ch] = (f2){pf[uu][2 * ch], pf[uu][2 * ch + 1]};
                            if (a.do_norm) v[ch] = (v[ch] - (f2){a.mean[ch], a.mean[ch]}) * (f2){a.rstd[ch], a.rstd[ch]};
                        }
                    }
                    uint4 o;
                    o.x = H16<HT>::pack2(v[0].x, v[1].x);
                    o.y = H16<HT>::pack2(v[2].x, 0.f);
                    o.z = H16<HT>::pack2(v[0].y, v[1].y);
                    o.w = H16<HT>::pack2(v[2].y, 0.f);
                    *reinterpret_cast<uint4*>(sP[buf] + (r * IC + c) * 8) = o;
                    continue;
                }
            }
            const int sh = iw - pair_base(iw, wi);  // -1 / 0 / +1 where a pixel is in the row
            const bool in0 = (unsigned)iw < (unsigned)wi, in1 = (unsigned)(iw + 1) < (unsigned)wi;
            f2 v[3];
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {  // zero padding is applied AFTER normalisation
                f2 x;
                if constexpr (U8) {
                    x = (f2){sL[pf[uu][2 * ch]], sL[pf[uu][2 * ch + 1]]};
                } else {
                    const float q0 = pf[uu][2 * ch], q1 = pf[uu][2 * ch + 1];
                    x = (f2){in0 ? (sh > 0 ? q1 : q0) : 0.f, in1 ? (sh < 0 ? q0 : q1) : 0.f};
                    if (a.do_norm) x = (x - (f2){a.mean[ch], a.mean[ch]}) * (f2){a.rstd[ch], a.rstd[ch]};
                }
                v[ch] = (f2){ok0 ? x.x : 0.f, ok1 ? x.y : 0.f};
            }
            uint4 o;
            o.x = H16<HT>::pack2(v[0].x, v[1].x);
            o.y = H16<HT>::pack2(v[2].x, 0.f);
            o.z = H16<HT>::pack2(v[0].y, v[1].y);
            o.w = H16<HT>::pack2(v[2].y, 0.f);
            *reinterpret_cast<uint4*>(sP[buf] + (r * IC + c) * 8) = o;
        }
    };

    const float slope = a.leaky ? a.slope : 1.f;  // identity == leaky with slope 1
    const float NINF = -__builtin_inff();
    int t = blockIdx.x;
    if (t >= ntiles) return;
    if constexpr (U8) __syncthreads();  // byte table
#pragma unroll
    for (int part = 0; part < NPART; ++part) {
        fill_load(t, part);
        fill_store(t, 0, part);
    }
    __syncthreads();
    const int nb_addr = ((lane + 16) & 63) * 4;
    int cur = 0;
    for (; t < ntiles; t += gridDim.x, cur ^= 1) {
        const int tn = t + gridDim.x;
        if (tn < ntiles) fill_load(tn, 0);
        int img, ph0, pw0;
        tile_origin(t, img, ph0, pw0);
        const char* pb = sP[cur] + (2 * (CB * wave + r16) + 2 * q) * 8;
        const bool active = pw0 + 7 * wave < a.wp;
        // even stem dims (host-checked): the only stem pixels outside the map that
        // feed stored outputs are row -1 (top tiles) and column -1 (left tiles:
        // wave 0, pixel 0 = lanes of group 0, element 0)
        const bool left = pw0 == 0 && wave == 0;
        const int pc0 = 7 * wave + 2 * q;
        const bool st0 = pw0 + pc0 < a.wp, st1 = q < 3 && pw0 + pc0 + 1 < a.wp;
        // the first NPRE K-steps' patch fragments of the next odd stem row are read
        // before the pooling tail of the current pooled row: their LDS latency
        // overlaps the tail instead of opening the next row's MFMAs
        uint4 pre[NPRE];
        auto preload = [&](int r) {
            const char* rb = pb + r * (2 * IC * 8);
#pragma unroll
            for (int m = 0; m < NPRE; ++m) pre[m] = *reinterpret_cast<const uint4*>(rb + m * IC * 8);
        };
        auto stem_row = [&](int r, h16_f32x4_t (&acc)[4], bool use_pre) {
#pragma unroll
            for (int f = 0; f < 4; ++f) acc[f] = (h16_f32x4_t){0.f, 0.f, 0.f, 0.f};
            const char* rb = pb + r * (2 * IC * 8);
#pragma unroll
            for (int m = 0; m < 7; ++m) {
                const uint4 px = use_pre && m < NPRE ? pre[m] : *reinterpret_cast<const uint4*>(rb + m * IC * 8);
#pragma unroll
                for (int f = 0; f < 4; ++f) acc[f] = H16<HT>::mfma(px, breg[f][m], acc[f]);
            }
        };
        h16_f32x4_t A[4];
        if (active) {
            stem_row(0, A, false);
            preload(1);
            if (ph0 == 0) {  // stem row -1: max-pool padding
#pragma unroll
                for (int f = 0; f < 4; ++f) A[f] = (h16_f32x4_t){NINF, NINF, NINF, NINF};
            }
        }
        for (int pr = 0; pr < PH; ++pr) {
#pragma unroll
            for (int part = 1; part < NPART; ++part)
                if (pr == part * PH / NPART && tn < ntiles) {  // part - 1 of the next patch -> LDS, part in flight
                    fill_store(tn, cur ^ 1, part - 1);
                    fill_load(tn, part);
                }
            if (active) {
                h16_f32x4_t B[4];
                stem_row(2 * pr + 1, B, true);
#pragma unroll
                for (int f = 0; f < 4; ++f)
#pragma unroll
                    for (int e = 0; e < 4; ++e) A[f][e] = fmaxf(A[f][e], B[f][e]);  // rows 2pr, 2pr+1
                h16_f32x4_t C[4];
                stem_row(2 * pr + 2, C, false);
                if (pr + 1 < PH) preload(2 * pr + 3);
                float p0[4], p1[4];
#pragma unroll
                for (int f = 0; f < 4; ++f) {
                    float m3[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) m3[e] = fmaxf(A[f][e], C[f][e]);
                    if (left && q == 0) m3[0] = NINF;  // stem column -1: max-pool padding
                    const float nb = __int_as_float(__builtin_amdgcn_ds_bpermute(nb_addr, __float_as_int(m3[0])));
                    p0[f] = fmaxf(fmaxf(m3[0], m3[1]), m3[2]);
                    p1[f] = fmaxf(fmaxf(m3[2], m3[3]), nb);
                    A[f] = C[f];
                }
                if (ph0 + pr < a.hp) {
                    bf16_t* dst = a.y + (((long long)img * a.hp + ph0 + pr) * a.wp + pw0 + pc0) * 64 + 4 * r16;
                    auto epi = [&](const float (&p)[4]) {
                        float v[4];
#pragma unroll
                        for (int f = 0; f < 4; ++f) {
                            v[f] = p[f] * sc[f] + sh[f];
                            v[f] = fmaxf(v[f], v[f] * slope);
                        }
                        return make_uint2(H16<HT>::pack2(v[0], v[1]), H16<HT>::pack2(v[2], v[3]));
                    };
                    if (st0) *reinterpret_cast<uint2*>(dst) = epi(p0);
                    if (st1) *reinterpret_cast<uint2*>(dst + 64) = epi(p1);
                }
            }
        }
        if (tn < ntiles) fill_store(tn, cur ^ 1, NPART - 1);
        __syncthreads();
    }
}


// ---------------------------------------------------------------------------
// Stem v4: v3's tile, wave layout, lane-local pooling and epilogue, with the
// conv's K in space-to-depth form.  The stride-2 7x7 conv on 3 channels is a
// stride-1 4x4 conv on 12-channel "s2d pixels" (2x2 input pixels x 3 channels,
// the 8x8-padded kernel: kh = 7 / kw = 7 carry zero weights): K = 4 x 4 x 12 =
// 192 = 6 MFMA K-steps of 32 instead of v3's 7 (7 kernel rows x 8 pixels x 4
// channels, 66 % of it useful; here 77 %).  The patch sits in LDS as s2d pixels
// of 24 B ([s2d row][s2d col][a][b][ci], a / b = row / column in the pair): the 4
// s2d pixels of one kernel row are 48 contiguous values, so a lane's 8 values of
// a K-step (k0 = 32 m + 8 q; a kernel row holds 48, a multiple of 8) are 16
// contiguous bytes at an 8-B aligned address: two ds_read_b64.  The tile's s2d
// rows and columns start one before its first stem row / column (stem pixel c
// uses s2d columns c - 1 .. c + 2); the patch (20 x 117 s2d pixels, 56 KiB) covers
// the same input rectangle as v3's (4 ph0 - 5 .., 4 pw0 - 5 ..), plus the one input
// row under the zero kh = 7 weights.  Same value per tap as v3 (normalised,
// rounded to 16 bits, zero padding after normalisation); only the f32 summation
// order of the 147 products differs.
template <typename HT, bool U8, int NPART, typename TAB = NoTab>
__global__ void __launch_bounds__(NT) k_stem_pool4(StemArgs a, TAB rt, int tiles_w, int tiles_hw, int ntiles) {
    constexpr bool RG = std::is_same<TAB, RaggedTab>::value;
    constexpr int PH = 8, PW = 56, SRN = 2 * PH + 1, CB = 14;
    constexpr int SCN = CB * 7 + 16;                 // 114 stem columns
    constexpr int PR = SRN + 3, PC = SCN + 3;        // 20 x 117 s2d pixels
    constexpr int SP = 24;                           // bytes per s2d pixel (12 x 16-bit)
    constexpr int NPIX = PR * PC, PPT = (NPIX + NT - 1) / NT;
    constexpr int PATCH = NPIX * SP;
    static_assert(PW == 7 * (NT / 64), "one 7-pooled-column block per wave");
    __shared__ __attribute__((aligned(16))) char sP[2][PATCH];
    __shared__ float sL[U8 ? 3 * 256 : 1];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int H = a.h, W = a.w_;
    const long long plane = (long long)H * W;

    if constexpr (U8) {
        for (int i = tid; i < 3 * 256; i += NT) {
            const int ch = i >> 8;
            const float x = (float)(i & 255) / 255.f;  // IEEE division = to_tensor
            sL[i] = a.do_norm ? (x - a.mean[ch]) * a.rstd[ch] : x;
        }
    }
    // B fragments (channel 4 * r16 + f of fragment f, s2d K-step m), negative-scale
    // channels negated (pool before the epilogue, see v2)
    uint4 breg[4][6];
    float sc[4], sh[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
        const int c = 4 * r16 + f;
        const int R = (c & ~31) | (((c >> 2) & 1) << 4) | (((c >> 3) & 3) << 2) | (c & 3);  // perm32_channel^-1
        const float s = a.scale[c];
        sc[f] = fabsf(s);
        sh[f] = a.shift[c];
        const unsigned flip = s < 0.f ? 0x80008000u : 0u;
#pragma unroll
        for (int m = 0; m < 6; ++m) {
            uint4 w = a.w[R * WROW + W4OFF + m * 4 + q];
            w.x ^= flip; w.y ^= flip; w.z ^= flip; w.w ^= flip;
            breg[f][m] = w;
        }
    }
    // this lane's byte offset of K-step m inside the 4 x 4 s2d window of its pixel
    int koff[6];
#pragma unroll
    for (int m = 0; m < 6; ++m) {
        const int k0 = 32 * m + 8 * q;
        koff[m] = (k0 / 48) * (PC * SP) + (k0 % 48) * 2;
    }

    auto tile_origin = [&](int t, int& img, int& ph0, int& pw0) {
        img = t / tiles_hw;
        const int rem = t - img * tiles_hw;
        const int th = rem / tiles_w;
        ph0 = th * PH;
        pw0 = (rem - th * tiles_w) * PW;
    };

    // patch fill in NPART parts: work item = one s2d pixel (2 input rows x 2 columns x 3 channels)
    constexpr int PH1 = (PPT + NPART - 1) / NPART;
    typedef typename std::conditional<U8, int, float>::type PT;
    PT pf[PH1][12];
    auto fill_load = [&](int t, int part) {
        int img, ph0, pw0;
        tile_origin(t, img, ph0, pw0);
        const int ir0 = 4 * ph0 - 5, ic0 = 4 * pw0 - 5;
        constexpr int ESZ = U8 ? 1 : 4;
        constexpr unsigned OOBO = 0x80000000u;
        const char* ib;
        int hi = H, wi = W;
        if constexpr (RG) {
            ib = (const char*)rt.p[img];
            hi = rt.h[img];
            wi = rt.w[img];
        } else {
            ib = (const char*)a.x + (long long)img * 3 * plane * ESZ;
        }
        const int iplane = hi * wi;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)ib, (short)0, (int)(3 * iplane * ESZ), 0x00020000);
#pragma unroll
        for (int uu = 0; uu < PH1; ++uu) {
            const int u = part * PH1 + uu;
            if (u >= PPT) break;
            int k = tid + NT * u;
            asm volatile("" : "+v"(k));  // offsets computed here, not hoisted into live VGPRs
            const int kk = k < NPIX ? k : NPIX - 1;
            const int r = kk / PC, c = kk - r * PC;
            const int ih = ir0 + 2 * r, iw = ic0 + 2 * c;
            unsigned off[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {  // e = a * 2 + b
                const int y = ih + (e >> 1), x = iw + (e & 1);
                off[e] = ((unsigned)y < (unsigned)hi && (unsigned)x < (unsigned)wi) ? (unsigned)((y * wi + x) * ESZ)
                                                                                     : OOBO;
            }
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                const unsigned po = (unsigned)(ch * iplane * ESZ);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if constexpr (U8)
                        pf[uu][e * 3 + ch] = ch * 256 + (int)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)(off[e] + po), 0, 0);
                    else
                        pf[uu][e * 3 + ch] =
                            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(off[e] + po), 0, 0));
                }
            }
        }
    };
    auto fill_store = [&](int t, int buf, int part) {
        int img, ph0, pw0;
        tile_origin(t, img, ph0, pw0);
        const int ir0 = 4 * ph0 - 5, ic0 = 4 * pw0 - 5;
#pragma unroll
        for (int uu = 0; uu < PH1; ++uu) {
            const int u = part * PH1 + uu;
            if (u >= PPT) break;
            int k = tid + NT * u;
            asm volatile("" : "+v"(k));
            if (k >= NPIX) continue;
            const int r = k / PC, c = k - r * PC;
            float v[12];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const bool ok = (unsigned)(ir0 + 2 * r + (e >> 1)) < (unsigned)H &&
                                (unsigned)(ic0 + 2 * c + (e & 1)) < (unsigned)W;
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {  // zero padding is applied AFTER normalisation
                    float x;
                    if constexpr (U8) x = sL[pf[uu][e * 3 + ch]];
                    else x = a.do_norm ? (pf[uu][e * 3 + ch] - a.mean[ch]) * a.rstd[ch] : pf[uu][e * 3 + ch];
                    v[e * 3 + ch] = ok ? x : 0.f;
                }
            }
            char* dst = sP[buf] + k * SP;
            *reinterpret_cast<uint2*>(dst) = make_uint2(H16<HT>::pack2(v[0], v[1]), H16<HT>::pack2(v[2], v[3]));
            *reinterpret_cast<uint2*>(dst + 8) = make_uint2(H16<HT>::pack2(v[4], v[5]), H16<HT>::pack2(v[6], v[7]));
            *reinterpret_cast<uint2*>(dst + 16) = make_uint2(H16<HT>::pack2(v[8], v[9]), H16<HT>::pack2(v[10], v[11]));
        }
    };

    const float slope = a.leaky ? a.slope : 1.f;  // identity == leaky with slope 1
    const float NINF = -__builtin_inff();
    int t = blockIdx.x;
    if (t >= ntiles) return;
    if constexpr (U8) __syncthreads();  // byte table
#pragma unroll
    for (int part = 0; part < NPART; ++part) {
        fill_load(t, part);
        fill_store(t, 0, part);
    }
    __syncthreads();
    const int nb_addr = ((lane + 16) & 63) * 4;
    int cur = 0;
    for (; t < ntiles; t += gridDim.x, cur ^= 1) {
        const int tn = t + gridDim.x;
        if (tn < ntiles) fill_load(tn, 0);
        int img, ph0, pw0;
        tile_origin(t, img, ph0, pw0);
        const char* pb = sP[cur] + (CB * wave + r16) * SP;
        const bool active = pw0 + 7 * wave < a.wp;
        const bool left = pw0 == 0 && wave == 0;
        const int pc0 = 7 * wave + 2 * q;
        const bool st0 = pw0 + pc0 < a.wp, st1 = q < 3 && pw0 + pc0 + 1 < a.wp;
        auto stem_row = [&](int r, h16_f32x4_t (&acc)[4]) {
#pragma unroll
            for (int f = 0; f < 4; ++f) acc[f] = (h16_f32x4_t){0.f, 0.f, 0.f, 0.f};
            const char* rb = pb + r * (PC * SP);
#pragma unroll
            for (int m = 0; m < 6; ++m) {
                const uint2 lo = *reinterpret_cast<const uint2*>(rb + koff[m]);
                const uint2 hi = *reinterpret_cast<const uint2*>(rb + koff[m] + 8);
                const uint4 px = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
                for (int f = 0; f < 4; ++f) acc[f] = H16<HT>::mfma(px, breg[f][m], acc[f]);
            }
        };
        h16_f32x4_t A[4];
        if (active) {
            stem_row(0, A);
            if (ph0 == 0) {  // stem row -1: max-pool padding
#pragma unroll
                for (int f = 0; f < 4; ++f) A[f] = (h16_f32x4_t){NINF, NINF, NINF, NINF};
            }
        }
        for (int pr = 0; pr < PH; ++pr) {
#pragma unroll
            for (int part = 1; part < NPART; ++part)
                if (pr == part * PH / NPART && tn < ntiles) {  // part - 1 of the next patch -> LDS, part in flight
                    fill_store(tn, cur ^ 1, part - 1);
                    fill_load(tn, part);
                }
            if (active) {
                h16_f32x4_t B[4];
                stem_row(2 * pr + 1, B);
#pragma unroll
                for (int f = 0; f < 4; ++f)
#pragma unroll
                    for (int e = 0; e < 4; ++e) A[f][e] = fmaxf(A[f][e], B[f][e]);  // rows 2pr, 2pr+1
                h16_f32x4_t C[4];
                stem_row(2 * pr + 2, C);
                float p0[4], p1[4];
#pragma unroll
                for (int f = 0; f < 4; ++f) {
                    float m3[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) m3[e] = fmaxf(A[f][e], C[f][e]);
                    if (left && q == 0) m3[0] = NINF;  // stem column -1: max-pool padding
                    const float nb = __int_as_float(__builtin_amdgcn_ds_bpermute(nb_addr, __float_as_int(m3[0])));
                    p0[f] = fmaxf(fmaxf(m3[0], m3[1]), m3[2]);
                    p1[f] = fmaxf(fmaxf(m3[2], m3[3]), nb);
                    A[f] = C[f];
                }
                if (ph0 + pr < a.hp) {
                    bf16_t* dst = a.y + (((long long)img * a.hp + ph0 + pr) * a.wp + pw0 + pc0) * 64 + 4 * r16;
                    auto epi = [&](const float (&p)[4]) {
                        float v[4];
#pragma unroll
                        for (int f = 0; f < 4; ++f) {
                            v[f] = p[f] * sc[f] + sh[f];
                            v[f] = fmaxf(v[f], v[f] * slope);
                        }
                        return make_uint2(H16<HT>::pack2(v[0], v[1]), H16<HT>::pack2(v[2], v[3]));
                    };
                    if (st0) *reinterpret_cast<uint2*>(dst) = epi(p0);
                    if (st1) *reinterpret_cast<uint2*>(dst + 64) = epi(p1);
                }
            }
        }
        if (tn < ntiles) fill_store(tn, cur ^ 1, NPART - 1);
        __syncthreads();
    }
}


// out[R][k], R packed row (PERM32), k < 256: k = kh*32 + kw*4 + ci (kh < 7, kw < 7,
// ci < 3 real; rest 0); k in [256, 448): the s2d order of v4 (see WROW)
template <typename HT>
__global__ void k_stem_pack(const float* __restrict__ w, HT* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 64 * 448) return;
    const int R = i / 448, k = i - R * 448;
    const int co = perm32_channel(R);
    int kh, kw, ci;
    if (k < 256) {
        kh = k >> 5; kw = (k >> 2) & 7; ci = k & 3;
    } else {
        const int kk = k - 256, kr = kk / 48, kc = (kk % 48) / 12, j = kk % 12;
        kh = 2 * kr + j / 6; kw = 2 * kc + (j % 6) / 3; ci = j % 3;
    }
    float v = 0.f;
    if (kh < 7 && kw < 7 && ci < 3) v = w[((co * 3 + ci) * 7 + kh) * 7 + kw];
    out[i] = DT<HT>::from_f(v);
}


}  // namespace

}  // namespace rr

using namespace rr;

extern "C" int rr_stem_pack_weights(const float* w, int c_out, int c_in, int kh, int kw, void* out, int dtype,
                                    void* stream) {
    if (dtype != RR_BF16 && dtype != RR_F16) return fail(RR_EINVAL, "rr_stem_pack_weights: bf16 / fp16 only");
    if (!w || !out) return fail(RR_EINVAL, "rr_stem_pack_weights: null pointer");
    if (c_out != 64 || c_in != 3 || kh != 7 || kw != 7)
        return fail(RR_EINVAL, "rr_stem_pack_weights: the fused stem is the 3->64 7x7 conv1");
    if (dtype == RR_F16)
        hipLaunchKernelGGL(k_stem_pack<f16_t>, dim3(112), dim3(256), 0, as_stream(stream), w, (f16_t*)out);
    else
        hipLaunchKernelGGL(k_stem_pack<bf16_t>, dim3(112), dim3(256), 0, as_stream(stream), w, (bf16_t*)out);
    return check_launch("rr_stem_pack_weights");
}

namespace rr {
int g_stem_mode = 2;  // rr_set_tuning(RR_TUNE_STEM): 5 space-to-depth K (v4), 2 swapped-operand lane-local
                      // pooling (v3; 3 / 4: 2 / 5 fill parts), 1 pool-before-epilogue kernel (v2), 0 k_stem_pool
}

// One launch over a same-size batch (TAB = NoTab, a.x = the [n][3][h][w] buffer)
// or over <= RAGGED_MAX images of a ragged batch (TAB = RaggedTab).
template <bool U8, typename TAB>
static void stem_launch(const StemArgs& a, const TAB& rt, int dtype, hipStream_t st) {
    constexpr bool RG = std::is_same<TAB, RaggedTab>::value;
    const int g_stem_cus = grid_cus();
    if (g_stem_mode >= 1 && a.ho % 2 == 0 && a.wo % 2 == 0) {  // v2/v3 handle the even stem maps (borders top / left)
        constexpr int PH = 8, PW = 56;
        const int tiles_w = (a.wp + PW - 1) / PW, tiles_h = (a.hp + PH - 1) / PH;
        const int ntiles = a.n * tiles_h * tiles_w;
        const int grid = ntiles < g_stem_cus ? ntiles : g_stem_cus;
        if (g_stem_mode >= 2 || RG) {  // 2: patch fill in 3 parts (default), 3: 2 parts, 4: 5 parts
            auto launch = [&](auto kern) {
                hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), 0, st, a, rt, tiles_w, tiles_w * tiles_h, ntiles);
            };
            if (g_stem_mode == 5) {
                if (dtype == RR_F16) launch(k_stem_pool4<f16_t, U8, 3, TAB>);
                else launch(k_stem_pool4<bf16_t, U8, 3, TAB>);
            } else if (dtype == RR_F16) {
                if (g_stem_mode == 3) launch(k_stem_pool3<f16_t, U8, 2, TAB>);
                else if (g_stem_mode == 4) launch(k_stem_pool3<f16_t, U8, 5, TAB>);
                else if (g_stem_mode == 6) launch(k_stem_pool3<f16_t, U8, 3, TAB, true>);
                else launch(k_stem_pool3<f16_t, U8, 3, TAB>);
            } else {
                if (g_stem_mode == 3) launch(k_stem_pool3<bf16_t, U8, 2, TAB>);
                else if (g_stem_mode == 4) launch(k_stem_pool3<bf16_t, U8, 5, TAB>);
                else if (g_stem_mode == 6) launch(k_stem_pool3<bf16_t, U8, 3, TAB, true>);
                else launch(k_stem_pool3<bf16_t, U8, 3, TAB>);
            }
            return;
        }
        if constexpr (!RG) {
            if (dtype == RR_F16)
                hipLaunchKernelGGL((k_stem_pool2<f16_t, U8>), dim3(grid), dim3(NT), 0, st, a, tiles_w,
                                   tiles_w * tiles_h, ntiles);
            else
                hipLaunchKernelGGL((k_stem_pool2<bf16_t, U8>), dim3(grid), dim3(NT), 0, st, a, tiles_w,
                                   tiles_w * tiles_h, ntiles);
        }
        return;
    }
    constexpr int PH = 4, PW = 32;
    const int tiles_w = (a.wp + PW - 1) / PW, tiles_h = (a.hp + PH - 1) / PH;
    const int ntiles = a.n * tiles_h * tiles_w;
    const int grid = ntiles < g_stem_cus ? ntiles : g_stem_cus;
    if (dtype == RR_F16)
        hipLaunchKernelGGL((k_stem_pool<PH, PW, f16_t, U8, TAB>), dim3(grid), dim3(NT), 0, st, a, rt, tiles_w,
                           tiles_w * tiles_h, ntiles);
    else
        hipLaunchKernelGGL((k_stem_pool<PH, PW, bf16_t, U8, TAB>), dim3(grid), dim3(NT), 0, st, a, rt, tiles_w,
                           tiles_w * tiles_h, ntiles);
}

// x: a same-size [n][3][h][w] batch, or (srcs != nullptr) a ragged batch whose
// image i is [3][extents[2i]][extents[2i+1]] at srcs[i], padded to h x w.
template <bool U8>
static int stem_conv_pool(const void* x, const void* const* srcs, const int* extents, int n, int h, int w,
                          const float* mean_host, const float* std_host, int do_normalize, const void* wpk,
                          const float* scale, const float* shift, int act, float slope, void* y, int hp, int wp,
                          int dtype, void* stream) {
    const char* fn = srcs ? "rr_stem_conv_pool_ragged" : "rr_stem_conv_pool";
    auto err = [&](const char* m) { return fail(RR_EINVAL, std::string(fn) + ": " + m); };
    if (dtype != RR_BF16 && dtype != RR_F16) return err("bf16 / fp16 only");
    if ((!x && !srcs) || (srcs && !extents) || !wpk || !scale || !shift || !y) return err("null pointer");
    if (n <= 0 || h <= 0 || w <= 0) return err("bad shape");
    const int ho = (h + 2 * 3 - 7) / 2 + 1, wo = (w + 2 * 3 - 7) / 2 + 1;
    if (ho <= 0 || wo <= 0) return err("image smaller than the kernel");
    if (hp != (ho + 2 - 3) / 2 + 1 || wp != (wo + 2 - 3) / 2 + 1)
        return err("output size must be the 3x3/s2/p1 pool of the stem map");
    if ((long long)3 * h * w * (U8 ? 1 : 4) >= (1ll << 31)) return err("image too large (32-bit buffer offsets)");
    if ((long long)n * ((hp + 3) / 4) * ((wp + 31) / 32) >= (1ll << 31)) return err("too many tiles");
    if (act != RR_ACT_IDENTITY && act != RR_ACT_LEAKY) return err("act");
    StemArgs a;
    a.x = x;
    a.w = (const uint4*)wpk;
    a.scale = scale;
    a.shift = shift;
    a.y = (bf16_t*)y;
    a.n = n; a.h = h; a.w_ = w; a.ho = ho; a.wo = wo; a.hp = hp; a.wp = wp;
    a.do_norm = do_normalize ? 1 : 0;
    for (int c = 0; c < 3; ++c) {
        a.mean[c] = do_normalize ? mean_host[c] : 0.f;
        a.rstd[c] = do_normalize ? (float)(1.0 / (double)std_host[c]) : 1.f;
    }
    a.leaky = act == RR_ACT_LEAKY;
    if (a.leaky && !(slope >= 0.f && slope <= 1.f)) return err("leaky slope must be in [0, 1]");
    a.slope = slope;
    if (!srcs) {
        stem_launch<U8>(a, NoTab{}, dtype, as_stream(stream));
        return check_launch(fn);
    }
    for (int i0 = 0; i0 < n; i0 += RAGGED_MAX) {
        const int cnt = n - i0 < RAGGED_MAX ? n - i0 : RAGGED_MAX;
        RaggedTab t;
        if (const char* e = ragged_fill(t, srcs, extents, i0, cnt, h, w)) return err(e);
        StemArgs ac = a;
        ac.x = nullptr;
        ac.n = cnt;
        ac.y = (bf16_t*)y + (long long)i0 * hp * wp * 64;
        stem_launch<U8>(ac, t, dtype, as_stream(stream));
    }
    return check_launch(fn);
}

extern "C" int rr_stem_conv_pool(const float* x, int n, int h, int w, const float* mean_host, const float* std_host,
                                 int do_normalize, const void* wpk, const float* scale, const float* shift, int act,
                                 float slope, void* y, int hp, int wp, int dtype, void* stream) {
    return stem_conv_pool<false>(x, nullptr, nullptr, n, h, w, mean_host, std_host, do_normalize, wpk, scale, shift,
                                 act, slope, y, hp, wp, dtype, stream);
}

extern "C" int rr_stem_conv_pool_u8(const unsigned char* x, int n, int h, int w, const float* mean_host,
                                    const float* std_host, int do_normalize, const void* wpk, const float* scale,
                                    const float* shift, int act, float slope, void* y, int hp, int wp, int dtype,
                                    void* stream) {
    return stem_conv_pool<true>(x, nullptr, nullptr, n, h, w, mean_host, std_host, do_normalize, wpk, scale, shift,
                                act, slope, y, hp, wp, dtype, stream);
}

extern "C" int rr_stem_conv_pool_ragged(const void* const* srcs, const int* extents, int n, int h, int w, int u8,
                                        const float* mean_host, const float* std_host, int do_normalize,
                                        const void* wpk, const float* scale, const float* shift, int act, float slope,
                                        void* y, int hp, int wp, int dtype, void* stream) {
    if (!srcs) return fail(RR_EINVAL, "rr_stem_conv_pool_ragged: null image table");
    return u8 ? stem_conv_pool<true>(nullptr, srcs, extents, n, h, w, mean_host, std_host, do_normalize, wpk, scale,
                                     shift, act, slope, y, hp, wp, dtype, stream)
              : stem_conv_pool<false>(nullptr, srcs, extents, n, h, w, mean_host, std_host, do_normalize, wpk, scale,
                                      shift, act, slope, y, hp, wp, dtype, stream);
}
