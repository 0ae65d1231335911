// librr.so — streaming 1x1 conv for the HBM-bound bottleneck layers (bf16 or
// fp16 operands: H16<H> picks the MFMA and the packing; 16-bit storage is
// moved as raw bits).
//
// The 1x1 convolutions of a bottleneck (conv1 / conv3 / projection) have
// K = 64..512: a few MFMAs per byte, so they are bound by HBM, not by the
// matrix cores (ResNet-50 @ 32 x 1024x768: ~60 % of conv time).  The tiled
// LDS-DMA engine (rr_gemm.hip) loses there because one wave's vmcnt counts
// its epilogue stores together with its next tile's DMA: every tile waits for
// its own stores to drain, which serialises the memory pipeline.
//
// This kernel is weight-stationary and barrier-free after the prologue:
//   * a block holds one slice of TC output channels x all K input channels of
//     the (PERM32-packed) weights in LDS, loaded once;
//   * every wave then streams its own 16*FN-pixel strips: activations go
//     HBM -> VGPR directly in the MFMA B-operand layout (no LDS round trip),
//     D strips deep (rotating register sets, compiler-tracked vmcnt — all
//     VMEM traffic is visible to the compiler, so a wait for strip j's
//     operands never waits for the stores of strips < j);
//   * the residual rows are prefetched the same way, D strips ahead;
//   * fused epilogue: BN scale/shift (from LDS), + residual, leaky ReLU,
//     bf16 pack, one 16-B store per (fragment pair, pixel).
// HBM traffic = x once (per channel slice) + residual once + y once.
#include "rr_internal.h"

namespace rr {

namespace {

typedef __attribute__((ext_vector_type(4))) float sf32x4_t;

// LDS image of the weight slice: row r (packed output channel), 16-B chunk c
// lives at r*K*2 + ((c ^ f(r)) * 16); f makes every ds_read_b128 lane group of
// an A-fragment read hit 16 distinct 4-bank groups (checked for K = 64..1024).
template <int K>
__device__ __forceinline__ int wswz(int row, int chunk) {
    const int f = K == 64 ? ((row >> 1) & 7) : (row & 15);
    return row * (K * 2) + ((chunk ^ f) << 4);
}

template <int TC, int K, int FN, int D, int NW, bool RES, typename H>
__global__ void __launch_bounds__(64 * NW) k_stream1x1(ConvArgs a, int nslices, int xmap) {
    constexpr int NI = TC / 16;   // accumulator fragments (channels) per wave
    constexpr int NK = K / 32;    // MFMA K-steps
    constexpr int NR = TC / 32;   // 16-B epilogue vectors per pixel
    constexpr int SP = 16 * FN;   // pixels per strip
    constexpr bool AREG = NI * NK * 4 <= 32;  // small slices keep A in VGPRs
    __shared__ __attribute__((aligned(16))) char sA[TC * K * 2];
    __shared__ __attribute__((aligned(16))) float sS[TC], sH[TC];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // xmap (grid a multiple of 8 x nslices): blocks b, b + 8, b + 16, ... share
    // an XCD (workgroups go round-robin over the 8 XCDs), so the nslices blocks
    // that stream the same strips for different channel slices are put there:
    // a strip's input is fetched into one XCD's L2 and re-read from it, not
    // fetched by nslices XCDs from HBM
    const int b = (int)blockIdx.x;
    const int slice = xmap ? (b >> 3) % nslices : b % nslices;
    const int bi = xmap ? ((b >> 3) / nslices) * 8 + (b & 7) : b / nslices;
    const int G = (int)gridDim.x / nslices;
    const int c0 = slice * TC;

    // ---- prologue: weight slice + affine into LDS (once per block)
    {
        const char* wsrc = (const char*)a.w + (long long)c0 * K * 2;
        constexpr int CH = TC * K / 8;  // 16-B chunks
        for (int i = tid; i < CH; i += 64 * NW) {
            const int r = i / (K / 8), c = i - r * (K / 8);
            *reinterpret_cast<uint4*>(sA + wswz<K>(r, c)) = *reinterpret_cast<const uint4*>(wsrc + (long long)i * 16);
        }
        const bool affine = a.flags & RR_CONV_AFFINE;
        for (int i = tid; i < TC; i += 64 * NW) {
            sS[i] = affine ? a.scale[c0 + i] : 1.f;
            sH[i] = affine ? a.shift[c0 + i] : 0.f;
        }
    }
    __syncthreads();

    const int r16 = lane & 15, kq = lane >> 4;
    const long long P = a.P;
    const int nstrips = (int)((P + SP - 1) / SP);
    const int gw = bi * NW + wave, GW = G * NW;
    const int nmine = gw < nstrips ? (nstrips - gw + GW - 1) / GW : 0;
    if (nmine == 0) return;
    const int niter = (nmine + D - 1) / D * D;
    const int hw = a.ho * a.wo;
    const bf16_t* __restrict__ X = (const bf16_t*)a.x;
    const bf16_t* __restrict__ R = (const bf16_t*)a.res;
    bf16_t* __restrict__ Y = (bf16_t*)a.y;
    const bool leaky = a.act == RR_ACT_LEAKY;
    const float slope = a.slope;

    // strip i of this wave (clamped past the end: loads stay in range, stores are skipped)
    auto strip_of = [&](int i) { return gw + (i < nmine ? i : nmine - 1) * GW; };
    auto pix = [&](int s, int j) {  // this lane's pixel in fragment j of strip s (clamped)
        long long p = (long long)s * SP + j * 16 + r16;
        return p < P ? p : P - 1;
    };
    auto x_off = [&](long long p) {  // element offset of pixel p's input row
        const long long img = p / hw;
        const int rem = (int)(p - img * hw);
        const int oh = rem / a.wo, ow = rem - oh * a.wo;
        return ((img * a.h + (long long)oh * a.stride) * a.w_ + (long long)ow * a.stride) * K;
    };

    uint4 bq[D][FN][NK];
    uint4 rq[RES ? D : 1][RES ? FN : 1][RES ? NR : 1];
    auto load_b = [&](uint4 (&dst)[FN][NK], int s) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const bf16_t* src = X + x_off(pix(s, j)) + 8 * kq;
#pragma unroll
            for (int kk = 0; kk < NK; ++kk) dst[j][kk] = *reinterpret_cast<const uint4*>(src + kk * 32);
        }
    };
    auto load_r = [&](uint4 (&dst)[RES ? FN : 1][RES ? NR : 1], int s) {
        if constexpr (RES) {
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const bf16_t* src = R + pix(s, j) * a.ldy + c0 + 8 * kq;
#pragma unroll
                for (int i2 = 0; i2 < NR; ++i2) dst[j][i2] = ld16_once(src + 32 * i2);  // residual: read once
            }
        }
    };

    uint4 areg[AREG ? NI : 1][AREG ? NK : 1];
    if constexpr (AREG) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int kk = 0; kk < NK; ++kk)
                areg[i][kk] = *reinterpret_cast<const uint4*>(sA + wswz<K>(i * 16 + r16, kk * 4 + kq));
    }

#pragma unroll
    for (int d = 0; d < D; ++d) {
        load_b(bq[d], strip_of(d));
        load_r(rq[RES ? d : 0], strip_of(d));
    }

    for (int it = 0; it < niter; it += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int i = it + d;
            const int s = strip_of(i);
            const bool live = i < nmine;
            // one 32-channel group at a time: 2 x FN accumulators, epilogue right away
#pragma unroll
            for (int i2 = 0; i2 < NR; ++i2) {
                // opaque LDS base: keeps the compiler from hoisting every A fragment of
                // the (loop-invariant) weight slice into VGPRs, which would spill
                int abase = 0;
                asm volatile("" : "+v"(abase));
                sf32x4_t acc[2][FN];
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int j = 0; j < FN; ++j) acc[h][j] = (sf32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kk = 0; kk < NK; ++kk)
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int ii = 2 * i2 + h;
                        const uint4 av = AREG ? areg[AREG ? ii : 0][AREG ? kk : 0]
                                              : *reinterpret_cast<const uint4*>(sA + abase + wswz<K>(ii * 16 + r16, kk * 4 + kq));
#pragma unroll
                        for (int j = 0; j < FN; ++j)
                            acc[h][j] = H16<H>::mfma(av, bq[d][j][kk], acc[h][j]);
                    }
                if (live) {
                    const int cl = 32 * i2 + 8 * kq;  // 8 consecutive channels of this lane
                    const float4 sc0 = *reinterpret_cast<const float4*>(sS + cl);
                    const float4 sc1 = *reinterpret_cast<const float4*>(sS + cl + 4);
                    const float4 sh0 = *reinterpret_cast<const float4*>(sH + cl);
                    const float4 sh1 = *reinterpret_cast<const float4*>(sH + cl + 4);
                    const float sc[8] = {sc0.x, sc0.y, sc0.z, sc0.w, sc1.x, sc1.y, sc1.z, sc1.w};
                    const float sh[8] = {sh0.x, sh0.y, sh0.z, sh0.w, sh1.x, sh1.y, sh1.z, sh1.w};
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        const long long p = (long long)s * SP + j * 16 + r16;
                        float v[8];
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            v[r] = acc[0][j][r] * sc[r] + sh[r];
                            v[4 + r] = acc[1][j][r] * sc[4 + r] + sh[4 + r];
                        }
                        if constexpr (RES) {
                            const uint4 q = rq[d][j][i2];
                            const unsigned w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                v[2 * r] += H16<H>::lo(w4[r]);
                                v[2 * r + 1] += H16<H>::hi(w4[r]);
                            }
                        }
                        if (leaky) {
#pragma unroll
                            for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * slope;
                        }
                        uint4 o;
                        o.x = H16<H>::pack2(v[0], v[1]);
                        o.y = H16<H>::pack2(v[2], v[3]);
                        o.z = H16<H>::pack2(v[4], v[5]);
                        o.w = H16<H>::pack2(v[6], v[7]);
                        if (p < P) st16_once(Y + p * a.ldy + c0 + cl, o);
                    }
                }
            }
            load_b(bq[d], strip_of(i + D));  // refill: strip i + D
            load_r(rq[RES ? d : 0], strip_of(i + D));
        }
    }
}

// ---------------------------------------------------------------------------
// Fused bottleneck boundary (bf16, the 64/256-channel stage of ResNet-50/101/
// 152): block i's conv3 (1x1, 64 -> 256, BN, + residual, activation) and block
// i+1's conv1 (1x1, 256 -> C1, BN, activation) in one pass.
//   y = act3(W3 . x * s3 + h3 + r)   is stored once and, still in registers,
//   z = act1(W1 . y * s1 + h1)       consumes it as the second GEMM's B operand:
// with PERM32 rows a lane's accumulator pair holds 8 consecutive y channels of
// one pixel, which is exactly an MFMA B fragment (k = channel), so y is never
// re-read from HBM (-2 B x 256 per pixel vs two launches).  Both weight slices
// (32 KiB + C1 x 512 B) and the affines stay in LDS; activations stream
// HBM -> VGPR D strips deep as in k_stream1x1.
// PROJ: the first block of the stage, whose shortcut is the projection
// proj_bn(proj_conv(x_in)) (1x1, stride 1, 64 -> 256): it is computed in the
// same pass from the block input (a third GEMM into its own accumulators), so
// the 256-channel projection map is neither written nor read back.
struct PairArgs {
    const bf16_t* x;   // [P][64]
    const bf16_t* w3;  // [256][64]  PERM32 rows
    const float *s3, *h3;
    const bf16_t* res; // [P][256] (!PROJ)
    const bf16_t* xp;  // [P][64]  block input (PROJ)
    const bf16_t* wp;  // [256][64] PERM32 rows (PROJ)
    const float *sp, *hp;
    const bf16_t* w1;  // [C1][256]  PERM32 rows
    const float *s1, *h1;
    bf16_t* y;         // [P][256]
    bf16_t* z;         // [P][C1]
    long long P;
    int act3, act1;
    float slope3, slope1;
};

template <int C1, int D, bool PROJ, typename H>
__global__ void __launch_bounds__(512) k_stream_pair(PairArgs a) {
    constexpr int K3 = 64, C3 = 256, NW = 8;
    constexpr int NK3 = K3 / 32, NR3 = C3 / 32, NF1 = C1 / 16, NK1 = C3 / 32;
    __shared__ __attribute__((aligned(16))) char sW3[C3 * K3 * 2];
    __shared__ __attribute__((aligned(16))) char sW1[C1 * C3 * 2];
    __shared__ __attribute__((aligned(16))) float sS3[C3], sH3[C3], sS1[C1], sH1[C1];
    __shared__ __attribute__((aligned(16))) char sWp[PROJ ? C3 * K3 * 2 : 16];
    __shared__ __attribute__((aligned(16))) float sSp[PROJ ? C3 : 1], sHp[PROJ ? C3 : 1];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < C3 * K3 / 8; i += 64 * NW) {
        const int r = i / (K3 / 8), c = i - r * (K3 / 8);
        *reinterpret_cast<uint4*>(sW3 + wswz<K3>(r, c)) = reinterpret_cast<const uint4*>(a.w3)[i];
    }
    for (int i = tid; i < C1 * C3 / 8; i += 64 * NW) {
        const int r = i / (C3 / 8), c = i - r * (C3 / 8);
        *reinterpret_cast<uint4*>(sW1 + wswz<C3>(r, c)) = reinterpret_cast<const uint4*>(a.w1)[i];
    }
    for (int i = tid; i < C3; i += 64 * NW) {
        sS3[i] = a.s3[i];
        sH3[i] = a.h3[i];
    }
    for (int i = tid; i < C1; i += 64 * NW) {
        sS1[i] = a.s1[i];
        sH1[i] = a.h1[i];
    }
    if constexpr (PROJ) {
        for (int i = tid; i < C3 * K3 / 8; i += 64 * NW) {
            const int r = i / (K3 / 8), c = i - r * (K3 / 8);
            *reinterpret_cast<uint4*>(sWp + wswz<K3>(r, c)) = reinterpret_cast<const uint4*>(a.wp)[i];
        }
        for (int i = tid; i < C3; i += 64 * NW) {
            sSp[i] = a.sp[i];
            sHp[i] = a.hp[i];
        }
    }
    __syncthreads();

    const int r16 = lane & 15, kq = lane >> 4;
    const long long P = a.P;
    const int nstrips = (int)((P + 15) / 16);
    const int gw = (int)blockIdx.x * NW + wave, GW = (int)gridDim.x * NW;
    const int nmine = gw < nstrips ? (nstrips - gw + GW - 1) / GW : 0;
    if (nmine == 0) return;
    const int niter = (nmine + D - 1) / D * D;
    const bool leaky3 = a.act3 == RR_ACT_LEAKY, leaky1 = a.act1 == RR_ACT_LEAKY;
    auto strip_of = [&](int i) { return gw + (i < nmine ? i : nmine - 1) * GW; };
    auto pix = [&](int s) {
        const long long p = (long long)s * 16 + r16;
        return p < P ? p : P - 1;
    };

    uint4 bq[D][NK3], rq[D][PROJ ? NK3 : NR3];  // PROJ: rq holds the block input's B fragments
    auto load = [&](int d, int s) {
        const long long p = pix(s);
        const bf16_t* xs = a.x + p * K3 + 8 * kq;
#pragma unroll
        for (int kk = 0; kk < NK3; ++kk) bq[d][kk] = ld16_once(xs + kk * 32);
        if constexpr (PROJ) {
            const bf16_t* ps = a.xp + p * K3 + 8 * kq;
#pragma unroll
            for (int kk = 0; kk < NK3; ++kk) rq[d][kk] = ld16_once(ps + kk * 32);
        } else {
            const bf16_t* rs = a.res + p * C3 + 8 * kq;
#pragma unroll
            for (int i2 = 0; i2 < NR3; ++i2) rq[d][i2] = ld16_once(rs + 32 * i2);
        }
    };
#pragma unroll
    for (int d = 0; d < D; ++d) load(d, strip_of(d));

    for (int it = 0; it < niter; it += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int i = it + d;
            const long long p = (long long)strip_of(i) * 16 + r16;
            const bool st = i < nmine && p < P;
            uint4 yq[NR3];
            // ---- y = act3(W3 x * s3 + h3 + r): one 32-channel pair at a time
#pragma unroll
            for (int i2 = 0; i2 < NR3; ++i2) {
                int abase = 0;
                asm volatile("" : "+v"(abase));  // keep the weight fragments in LDS (no hoisting into VGPRs)
                sf32x4_t acc[2] = {(sf32x4_t){0.f, 0.f, 0.f, 0.f}, (sf32x4_t){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
                for (int kk = 0; kk < NK3; ++kk)
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const uint4 av = *reinterpret_cast<const uint4*>(sW3 + abase + wswz<K3>((2 * i2 + h) * 16 + r16, kk * 4 + kq));
                        acc[h] = H16<H>::mfma(av, bq[d][kk], acc[h]);
                    }
                const int c = 32 * i2 + 8 * kq;
                float v[8];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[0][r] * sS3[c + r] + sH3[c + r];
                    v[4 + r] = acc[1][r] * sS3[c + 4 + r] + sH3[c + 4 + r];
                }
                if constexpr (PROJ) {  // shortcut = proj_bn(proj_conv(x_in)), kept in f32
                    sf32x4_t pacc[2] = {(sf32x4_t){0.f, 0.f, 0.f, 0.f}, (sf32x4_t){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
                    for (int kk = 0; kk < NK3; ++kk)
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const uint4 av = *reinterpret_cast<const uint4*>(sWp + abase + wswz<K3>((2 * i2 + h) * 16 + r16, kk * 4 + kq));
                            pacc[h] = H16<H>::mfma(av, rq[d][kk], pacc[h]);
                        }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] += pacc[0][r] * sSp[c + r] + sHp[c + r];
                        v[4 + r] += pacc[1][r] * sSp[c + 4 + r] + sHp[c + 4 + r];
                    }
                } else {
                    const uint4 q = rq[d][i2];
                    const unsigned w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[2 * r] += H16<H>::lo(w4[r]);
                        v[2 * r + 1] += H16<H>::hi(w4[r]);
                    }
                }
                if (leaky3) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope3;
                }
                yq[i2].x = H16<H>::pack2(v[0], v[1]);
                yq[i2].y = H16<H>::pack2(v[2], v[3]);
                yq[i2].z = H16<H>::pack2(v[4], v[5]);
                yq[i2].w = H16<H>::pack2(v[6], v[7]);
                if (st) st16_once(a.y + p * C3 + c, yq[i2]);
            }
            load(d, strip_of(i + D));  // refill this slot: strip i + D
            // ---- z = act1(W1 y * s1 + h1), y straight from registers
            sf32x4_t zacc[NF1];
#pragma unroll
            for (int o = 0; o < NF1; ++o) zacc[o] = (sf32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < NK1; ++kk) {
                int abase = 0;
                asm volatile("" : "+v"(abase));
#pragma unroll
                for (int o = 0; o < NF1; ++o) {
                    const uint4 av = *reinterpret_cast<const uint4*>(sW1 + abase + wswz<C3>(o * 16 + r16, kk * 4 + kq));
                    zacc[o] = H16<H>::mfma(av, yq[kk], zacc[o]);
                }
            }
#pragma unroll
            for (int o2 = 0; o2 < NF1 / 2; ++o2) {
                const int c = 32 * o2 + 8 * kq;
                float v[8];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = zacc[2 * o2][r] * sS1[c + r] + sH1[c + r];
                    v[4 + r] = zacc[2 * o2 + 1][r] * sS1[c + 4 + r] + sH1[c + 4 + r];
                }
                if (leaky1) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope1;
                }
                uint4 o;
                o.x = H16<H>::pack2(v[0], v[1]);
                o.y = H16<H>::pack2(v[2], v[3]);
                o.z = H16<H>::pack2(v[4], v[5]);
                o.w = H16<H>::pack2(v[6], v[7]);
                if (st) st16_once(a.z + p * C1 + c, o);
            }
        }
    }
}


// ---------------------------------------------------------------------------
// Fused bottleneck boundary of the 128/512-channel stage (ResNet-50/101/152
// mod3): block i's conv3 (1x1, 128 -> 512, BN, + residual, activation) and
// block i+1's conv1 (1x1, 512 -> 128, BN, activation) in one pass, so the
// 512-channel map y is written once and never read back (-1 KiB per pixel).
// The weights (128 KiB + 128 KiB) do not fit in LDS beside the tiles, so they
// live in VGPRs for the whole launch: wave w holds W3 rows 64w..64w+63 (4 x 4
// fragments) and W1 rows 16w..16w+15 (16 fragments), 128 VGPRs.  Per tile of
// TP = 64 pixels (persistent blocks, one per CU):
//   * x tile [64][128] (16 KiB) and residual tile [64][512] (64 KiB) arrive by
//     LDS-DMA (buffer_load ... lds), the residual one tile ahead into the
//     second of two buffers, x during stage 2 of the previous tile;
//   * stage 1: y = act3(W3 x * s3 + h3 + r) per wave for its 64 channels; y
//     goes to HBM and, in place of the residual, into the LDS tile;
//   * stage 2: z = act1(W1 y * s1 + h1) with y read back from LDS (K = 512).
// LDS images are [pixel][16-B chunk] with the chunk XOR (pixel & 15) swizzle
// (applied on the DMA source side): every ds_read_b128 lane group of a B
// fragment hits 16 distinct 16-B bank groups.  MFMA accumulation order per
// element equals the two unfused k_stream1x1 launches (K-steps in order), so
// y and z are bit-identical to them.
typedef __attribute__((ext_vector_type(4))) int si32x4_t;

// A value loaded once before a loop (weights kept in VGPRs): passing it through an
// empty asm makes the asm its producer, so the compiler's wait for the load sits
// before the loop instead of (counted against the loop's own LDS-DMA / stores,
// which it cannot see) in front of every use inside it.
__device__ __forceinline__ void pin_loaded(uint4& v) {
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
}

__device__ __forceinline__ void sdma16(si32x4_t rsrc, unsigned voff, unsigned lds_addr) {
    unsigned keep;
    lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"  // M0 write -> LDS-DMA: 1 wait state (descriptor: fenced in the rsrc maker)
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(lds_addr)
        : "memory");
}
__device__ __forceinline__ si32x4_t srsrc(const void* base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)base;
    si32x4_t r;
    r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)b);
    r.y = __builtin_amdgcn_readfirstlane((int)((unsigned)(b >> 32) & 0xFFFFu));
    r.z = __builtin_amdgcn_readfirstlane((int)bytes);  // reads past the end return zeros
    r.w = 0x00020000;
    // VALU (readfirstlane) SGPR write -> LDS-DMA descriptor read: 5 wait states, tied to the
    // registers so no use of the descriptor is scheduled above it (tools/dma_audit.py checks)
    int x = r.x, y = r.y, z = r.z;
    asm volatile("s_nop 4" : "+s"(x), "+s"(y), "+s"(z));
    r.x = x;
    r.y = y;
    r.z = z;
    return r;
}

struct PairMidArgs {
    const bf16_t* x;    // [P][128]
    const bf16_t* w3;   // [512][128] PERM32 rows
    const float *s3, *h3;
    const bf16_t* res;  // [P][512]
    const bf16_t* w1;   // [128][512] PERM32 rows
    const float *s1, *h1;
    bf16_t* y;          // [P][512]
    bf16_t* z;          // [P][128]
    long long P;
    int act3, act1;
    float slope3, slope1;
};

template <typename H>
__global__ void __launch_bounds__(512, 1) k_pair_mid(PairMidArgs a) {
    constexpr int K3 = 128, C3 = 512, C1 = 128, TP = 64;
    constexpr int XB = TP * K3 * 2, RB = TP * C3 * 2;  // 16 KiB, 64 KiB
    __shared__ __attribute__((aligned(1024))) char smem[2 * RB + XB];
    __shared__ __attribute__((aligned(16))) float sS3[C3], sH3[C3], sS1[C1], sH1[C1];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, kq = lane >> 4;
    for (int i = tid; i < C3; i += 512) {
        sS3[i] = a.s3[i];
        sH3[i] = a.h3[i];
    }
    if (tid < C1) {
        sS1[tid] = a.s1[tid];
        sH1[tid] = a.h1[tid];
    }
    // weight fragments -> VGPRs (A operand: lane holds k = 32 kk + 8 kq .. + 7 of row r16)
    uint4 a3[4][4], a1[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            a3[i][kk] = *reinterpret_cast<const uint4*>(a.w3 + (long long)(64 * wave + 16 * i + r16) * K3 + 32 * kk + 8 * kq);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
        a1[kk] = *reinterpret_cast<const uint4*>(a.w1 + (long long)(16 * wave + r16) * C3 + 32 * kk + 8 * kq);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) pin_loaded(a3[i][kk]);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) pin_loaded(a1[kk]);
    __syncthreads();

    const long long P = a.P;
    const int ntiles = (int)((P + TP - 1) / TP);
    const int t0 = (int)blockIdx.x, G = (int)gridDim.x;
    if (t0 >= ntiles) return;
    const si32x4_t rsX = srsrc(a.x, (unsigned)(P * K3 * 2));
    const si32x4_t rsR = srsrc(a.res, (unsigned)(P * C3 * 2));
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    const unsigned ldsX = lds0 + 2 * RB;
    // x tile: 16 wave-instructions of 4 pixels x 256 B (2 per wave)
    auto dma_x = [&](int t) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int d = 2 * wave + u, px = 4 * d + (lane >> 4), slot = lane & 15;
            const unsigned off = (unsigned)(((long long)t * TP + px) * (K3 * 2)) + (unsigned)((slot ^ (px & 15)) << 4);
            sdma16(rsX, off, ldsX + d * 1024);
        }
    };
    // residual tile: 64 wave-instructions of one pixel x 1 KiB (8 per wave)
    auto dma_r = [&](int t, int buf) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int px = 8 * wave + u;
            const unsigned off = (unsigned)(((long long)t * TP + px) * (C3 * 2)) + (unsigned)((lane ^ (px & 15)) << 4);
            sdma16(rsR, off, lds0 + buf * RB + px * 1024);
        }
    };
    const bool leaky3 = a.act3 == RR_ACT_LEAKY, leaky1 = a.act1 == RR_ACT_LEAKY;

    dma_r(t0, 0);
    dma_x(t0);
    for (int k = 0, t = t0; t < ntiles; ++k, t += G) {
        const int cur = k & 1;
        const bool more = t + G < ntiles;
        // x(t), r(t) landed; only the previous tile's 4 z stores may stay in flight
        if (k == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
        if (more) dma_r(t + G, cur ^ 1);
        const char* X = smem + 2 * RB;
        char* RY = smem + cur * RB;
        // ---- stage 1: y = act3(W3 x * s3 + h3 + r), one 32-channel pair at a time
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2) {
            h16_f32x4_t acc[2][4];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[h][j] = (h16_f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                uint4 bx[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int px = 16 * j + r16;
                    bx[j] = *reinterpret_cast<const uint4*>(X + px * (K3 * 2) + ((((4 * kk + kq) ^ (px & 15))) << 4));
                }
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[h][j] = H16<H>::mfma(a3[2 * i2 + h][kk], bx[j], acc[h][j]);
            }
            const int c = 64 * wave + 32 * i2 + 8 * kq;  // 8 consecutive channels of this lane (PERM32)
            const int chunk = c >> 3;
            const float4 sc0 = *reinterpret_cast<const float4*>(sS3 + c);
            const float4 sc1 = *reinterpret_cast<const float4*>(sS3 + c + 4);
            const float4 sh0 = *reinterpret_cast<const float4*>(sH3 + c);
            const float4 sh1 = *reinterpret_cast<const float4*>(sH3 + c + 4);
            const float sc[8] = {sc0.x, sc0.y, sc0.z, sc0.w, sc1.x, sc1.y, sc1.z, sc1.w};
            const float sh[8] = {sh0.x, sh0.y, sh0.z, sh0.w, sh1.x, sh1.y, sh1.z, sh1.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int px = 16 * j + r16;
                uint4* slot = reinterpret_cast<uint4*>(RY + px * (C3 * 2) + ((chunk ^ (px & 15)) << 4));
                const uint4 q = *slot;
                const unsigned w4[4] = {q.x, q.y, q.z, q.w};
                float v[8];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[0][j][r] * sc[r] + sh[r];
                    v[4 + r] = acc[1][j][r] * sc[4 + r] + sh[4 + r];
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[2 * r] += H16<H>::lo(w4[r]);
                    v[2 * r + 1] += H16<H>::hi(w4[r]);
                }
                if (leaky3) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope3;
                }
                uint4 o;
                o.x = H16<H>::pack2(v[0], v[1]);
                o.y = H16<H>::pack2(v[2], v[3]);
                o.z = H16<H>::pack2(v[4], v[5]);
                o.w = H16<H>::pack2(v[6], v[7]);
                *slot = o;
                const long long p = (long long)t * TP + px;
                if (p < P) st16_once(a.y + p * C3 + c, o);
            }
        }
        // y tile complete in LDS; x buffer free
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (more) dma_x(t + G);
        // ---- stage 2: z = act1(W1 y * s1 + h1), K = 512 from the LDS y tile
        h16_f32x4_t zacc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) zacc[j] = (h16_f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
            uint4 by[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int px = 16 * j + r16;
                by[j] = *reinterpret_cast<const uint4*>(RY + px * (C3 * 2) + ((((4 * kk + kq) ^ (px & 15))) << 4));
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) zacc[j] = H16<H>::mfma(a1[kk], by[j], zacc[j]);
        }
        {
            // packed rows 16w + 4kq + r = channels 32 (w >> 1) + 8 kq + 4 (w & 1) + r
            const int c = 32 * (wave >> 1) + 8 * kq + 4 * (wave & 1);
            const float4 sc = *reinterpret_cast<const float4*>(sS1 + c);
            const float4 sh = *reinterpret_cast<const float4*>(sH1 + c);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v[4] = {zacc[j][0] * sc.x + sh.x, zacc[j][1] * sc.y + sh.y, zacc[j][2] * sc.z + sh.z,
                              zacc[j][3] * sc.w + sh.w};
                if (leaky1) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope1;
                }
                uint2 o;
                o.x = H16<H>::pack2(v[0], v[1]);
                o.y = H16<H>::pack2(v[2], v[3]);
                const long long p = (long long)t * TP + 16 * j + r16;
                if (p < P) st8_once(a.z + p * C1 + c, o);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The same boundary with a deeper HBM stream (round 6, the default; RR_TUNE_PAIR_MID = 0 runs
// k_pair_mid above).  k_pair_mid's 64-pixel tiles leave one residual tile (64 KiB) in flight
// per CU, issued at the tile start and landed long before the tile ends, and its x tile
// is issued after stage 1, so the next tile's wait also drains the y stores: the read
// stream idles for part of every tile (4.6 TB/s of algorithmic traffic in the bench step).
// Here tiles are TP = 32 pixels, the residual tiles sit in a 4-slot ring (3 tiles ahead: up
// to 96 KiB of reads in flight per CU) and x is double buffered (one tile ahead), both
// issued at the top of the tile, before its stores: the counted wait at the next top covers
// only the loads it needs, never the stores.  Per tile (iteration k, tile t_k):
//   top: vmcnt(10) = x(t_k) and r(t_k) have landed (younger: r(t_{k+2}) 4, y(t_{k-1}) 4,
//        z(t_{k-1}) 2 per lane), barrier; issue x(t_{k+1}) (1 per lane), r(t_{k+3}) (4);
//   stage 1 / barrier / stage 2 as in k_pair_mid on 32 pixels (same fragments and K order
//   per element: bit-identical).
// DMAs of tiles past the end are issued anyway (their offsets read past the buffer: zeros),
// so every lane's count is the same on every tile.
template <typename H>
__global__ void __launch_bounds__(512, 1) k_pair_mid_ring(PairMidArgs a) {
    constexpr int K3 = 128, C3 = 512, C1 = 128, TP = 32, NR = 4;
    constexpr int XB = TP * K3 * 2, RB = TP * C3 * 2;  // 8 KiB, 32 KiB
    __shared__ __attribute__((aligned(1024))) char smem[NR * RB + 2 * XB];
    __shared__ __attribute__((aligned(16))) float sS3[C3], sH3[C3], sS1[C1], sH1[C1];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, kq = lane >> 4;
    for (int i = tid; i < C3; i += 512) {
        sS3[i] = a.s3[i];
        sH3[i] = a.h3[i];
    }
    if (tid < C1) {
        sS1[tid] = a.s1[tid];
        sH1[tid] = a.h1[tid];
    }
    uint4 a3[4][4], a1[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            a3[i][kk] = *reinterpret_cast<const uint4*>(a.w3 + (long long)(64 * wave + 16 * i + r16) * K3 + 32 * kk + 8 * kq);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
        a1[kk] = *reinterpret_cast<const uint4*>(a.w1 + (long long)(16 * wave + r16) * C3 + 32 * kk + 8 * kq);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) pin_loaded(a3[i][kk]);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) pin_loaded(a1[kk]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the weights: the counted waits below see only DMA / stores
    __syncthreads();

    const long long P = a.P;
    const int ntiles = (int)((P + TP - 1) / TP);
    const int t0 = (int)blockIdx.x, G = (int)gridDim.x;
    if (t0 >= ntiles) return;
    const si32x4_t rsX = srsrc(a.x, (unsigned)(P * K3 * 2));
    const si32x4_t rsR = srsrc(a.res, (unsigned)(P * C3 * 2));
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    const unsigned ldsX = lds0 + NR * RB;
    // x tile: 8 wave-instructions of 4 pixels x 256 B (one per wave)
    auto dma_x = [&](int t, int xb) {
        const int px = 4 * wave + (lane >> 4), slot = lane & 15;
        const unsigned off = (unsigned)(((long long)t * TP + px) * (K3 * 2)) + (unsigned)((slot ^ (px & 15)) << 4);
        sdma16(rsX, off, ldsX + xb * XB + wave * 1024);
    };
    // residual tile: 32 wave-instructions of one pixel x 1 KiB (4 per wave)
    auto dma_r = [&](int t, int buf) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int px = 4 * wave + u;
            const unsigned off = (unsigned)(((long long)t * TP + px) * (C3 * 2)) + (unsigned)((lane ^ (px & 15)) << 4);
            sdma16(rsR, off, lds0 + buf * RB + px * 1024);
        }
    };
    const bool leaky3 = a.act3 == RR_ACT_LEAKY, leaky1 = a.act1 == RR_ACT_LEAKY;

    dma_x(t0, 0);
    dma_r(t0, 0);
    dma_r(t0 + G, 1);
    dma_r(t0 + 2 * G, 2);
    for (int k = 0, t = t0; t < ntiles; ++k, t += G) {
        const int cur = k & 3, xc = k & 1;
        if (k == 0) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(10)\n\ts_barrier" ::: "memory");
        dma_x(t + G, xc ^ 1);
        dma_r(t + 3 * G, (k + 3) & 3);
        const char* X = smem + NR * RB + xc * XB;
        char* RY = smem + cur * RB;
        // ---- stage 1: y = act3(W3 x * s3 + h3 + r), one 32-channel pair at a time
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2) {
            h16_f32x4_t acc[2][2];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[h][j] = (h16_f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                uint4 bx[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int px = 16 * j + r16;
                    bx[j] = *reinterpret_cast<const uint4*>(X + px * (K3 * 2) + ((((4 * kk + kq) ^ (px & 15))) << 4));
                }
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[h][j] = H16<H>::mfma(a3[2 * i2 + h][kk], bx[j], acc[h][j]);
            }
            const int c = 64 * wave + 32 * i2 + 8 * kq;  // 8 consecutive channels of this lane (PERM32)
            const int chunk = c >> 3;
            const float4 sc0 = *reinterpret_cast<const float4*>(sS3 + c);
            const float4 sc1 = *reinterpret_cast<const float4*>(sS3 + c + 4);
            const float4 sh0 = *reinterpret_cast<const float4*>(sH3 + c);
            const float4 sh1 = *reinterpret_cast<const float4*>(sH3 + c + 4);
            const float sc[8] = {sc0.x, sc0.y, sc0.z, sc0.w, sc1.x, sc1.y, sc1.z, sc1.w};
            const float sh[8] = {sh0.x, sh0.y, sh0.z, sh0.w, sh1.x, sh1.y, sh1.z, sh1.w};
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int px = 16 * j + r16;
                uint4* slot = reinterpret_cast<uint4*>(RY + px * (C3 * 2) + ((chunk ^ (px & 15)) << 4));
                const uint4 q = *slot;
                const unsigned w4[4] = {q.x, q.y, q.z, q.w};
                float v[8];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[0][j][r] * sc[r] + sh[r];
                    v[4 + r] = acc[1][j][r] * sc[4 + r] + sh[4 + r];
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[2 * r] += H16<H>::lo(w4[r]);
                    v[2 * r + 1] += H16<H>::hi(w4[r]);
                }
                if (leaky3) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope3;
                }
                uint4 o;
                o.x = H16<H>::pack2(v[0], v[1]);
                o.y = H16<H>::pack2(v[2], v[3]);
                o.z = H16<H>::pack2(v[4], v[5]);
                o.w = H16<H>::pack2(v[6], v[7]);
                *slot = o;
                const long long p = (long long)t * TP + px;
                if (p < P) st16_once(a.y + p * C3 + c, o);
            }
        }
        // y tile complete in LDS; the x buffer of this tile is free
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // ---- stage 2: z = act1(W1 y * s1 + h1), K = 512 from the LDS y tile
        h16_f32x4_t zacc[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) zacc[j] = (h16_f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
            uint4 by[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int px = 16 * j + r16;
                by[j] = *reinterpret_cast<const uint4*>(RY + px * (C3 * 2) + ((((4 * kk + kq) ^ (px & 15))) << 4));
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) zacc[j] = H16<H>::mfma(a1[kk], by[j], zacc[j]);
        }
        {
            const int c = 32 * (wave >> 1) + 8 * kq + 4 * (wave & 1);
            const float4 sc = *reinterpret_cast<const float4*>(sS1 + c);
            const float4 sh = *reinterpret_cast<const float4*>(sH1 + c);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                float v[4] = {zacc[j][0] * sc.x + sh.x, zacc[j][1] * sc.y + sh.y, zacc[j][2] * sc.z + sh.z,
                              zacc[j][3] * sc.w + sh.w};
                if (leaky1) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope1;
                }
                uint2 o;
                o.x = H16<H>::pack2(v[0], v[1]);
                o.y = H16<H>::pack2(v[2], v[3]);
                const long long p = (long long)t * TP + 16 * j + r16;
                if (p < P) st8_once(a.z + p * C1 + c, o);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// ---------------------------------------------------------------------------
// Weight-stationary 1x1 with the weights in VGPRs (the bottleneck conv3 of
// mod4 / mod5: 256 -> 1024 and 512 -> 2048, BN, + residual, activation; the
// K = 256 / 512 projections and the mod4 block-1 conv1, without residual,
// strided or not).
// k_stream1x1 keeps the weight slice in LDS and streams the activations into
// VGPRs, so every MFMA re-reads a 1 KiB A fragment from LDS: at K = 512 the
// LDS port, not the matrix cores, sets its pace (~600 TFLOP/s).  Here the
// roles flip:
//   * each wave holds its CW output channels x all K of the PERM32 weights in
//     VGPRs for the whole launch (CW / 16 x K / 32 fragments = 128 VGPRs);
//     a block (8 waves, one per CU, persistent) owns BC = 8 CW channels;
//   * activation tiles [TP pixels][K] (RES: and the residual tile [TP][BC])
//     arrive by LDS-DMA into one of three buffers, two tiles ahead (~100 KiB
//     in flight per CU), swizzled (16-B chunk XOR pixel & 15) on the source
//     side; a strided conv gathers its input rows in the DMA offsets;
//   * a B fragment read from LDS feeds CW / 16 MFMAs (4 at K = 256, 2 at
//     K = 512, vs 1 in k_stream1x1); the residual is read from LDS in the
//     epilogue.
// The nslices channel slices of one pixel tile run on one XCD (block b of
// the XCD-contiguous map), so the activation tile is fetched from HBM once
// and re-read from that XCD's L2.  MFMA accumulation order per element
// (K-steps 0..K/32-1 from zero) equals k_stream1x1's: outputs are
// bit-identical to it.
struct WresArgs {
    const bf16_t* x;    // [n][h][w][K]
    const bf16_t* w;    // [C][K] PERM32 rows
    const float *scale, *shift;
    const bf16_t* res;  // [P][ldy] (RES)
    bf16_t* y;          // [P][ldy]
    long long P;
    int ldy, nslices, xmap, act;
    float slope;
    int h, w_, ho, wo, stride;
};

template <int K, int CW, bool RES, typename H, bool DEEP = true>
__global__ void __launch_bounds__(512, 1) k_wres1x1(WresArgs a) {
    constexpr int TP = 32, NJ = TP / 16, NI = CW / 16, NK = K / 32, BC = 8 * CW;
    constexpr int XRB = K * 2, RRB = RES ? BC * 2 : 0;  // row bytes of the two tiles
    constexpr int XB = TP * XRB, RB = TP * RRB;         // tile bytes
    // buffers: 3 (two tiles ahead) where the residual tile fills the LDS; the non-residual forms
    // (16 / 32 KiB tiles) keep 5 / 3 tiles ahead (round 6: the strided mod3 projection streamed
    // at 4.7 TB/s two tiles ahead)
    constexpr int BUF = XB + RB, NBUF = RES || !DEEP ? 3 : (BUF <= 16384 ? 6 : 4), DA = NBUF - 1;
    constexpr int NDX = XB / 1024 / 8, NDR = RB / 1024 / 8;  // DMA instructions per wave
    constexpr int ND = NDX + NDR, NST = (CW / 32) * NJ;      // ... and stores per wave per tile
    static_assert(NI * NK <= 32 && XB % 8192 == 0 && RB % 8192 == 0, "tile shape");
    static_assert(XRB <= 1024 && RRB <= 1024, "row fits one DMA instruction");
    __shared__ __attribute__((aligned(1024))) char smem[NBUF * BUF];
    __shared__ __attribute__((aligned(16))) float sS[BC], sH[BC];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, kq = lane >> 4;
    const int b = (int)blockIdx.x, ns = a.nslices;
    const int slice = a.xmap ? (b >> 3) % ns : b % ns;
    const int bi = a.xmap ? ((b >> 3) / ns) * 8 + (b & 7) : b / ns;
    const int G = (int)gridDim.x / ns;
    const int c0 = slice * BC, cw0 = c0 + CW * wave;

    const bool affine = a.scale != nullptr;
    for (int i = tid; i < BC; i += 512) {
        sS[i] = affine ? a.scale[c0 + i] : 1.f;
        sH[i] = affine ? a.shift[c0 + i] : 0.f;
    }
    uint4 areg[NI][NK];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int kk = 0; kk < NK; ++kk)
            areg[i][kk] = *reinterpret_cast<const uint4*>(a.w + (long long)(cw0 + 16 * i + r16) * K + 32 * kk + 8 * kq);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) pin_loaded(areg[i][kk]);
    __syncthreads();

    const long long P = a.P;
    const int ntiles = (int)((P + TP - 1) / TP);
    if (bi >= ntiles) return;
    const long long nimg = P / ((long long)a.ho * a.wo);
    const si32x4_t rsX = srsrc(a.x, (unsigned)(nimg * a.h * a.w_ * XRB));
    si32x4_t rsR = rsX;
    if constexpr (RES) rsR = srsrc(a.res + c0, (unsigned)(P * a.ldy * 2 - (long long)c0 * 2));
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    const int hw = a.ho * a.wo;
    auto x_row = [&](unsigned p) -> unsigned {  // input row of output pixel p (past the end: past the buffer)
        if (a.stride == 1) return p;
        const unsigned img = p / (unsigned)hw, rem = p - img * (unsigned)hw;
        const unsigned oh = rem / (unsigned)a.wo, ow = rem - oh * (unsigned)a.wo;
        return (img * (unsigned)a.h + oh * (unsigned)a.stride) * (unsigned)a.w_ + ow * (unsigned)a.stride;
    };
    // instruction d of a tile moves LDS bytes [1 KiB d, 1 KiB (d + 1)): 1024 / row-bytes pixels
    auto dma = [&](int t, int buf) {
#pragma unroll
        for (int u = 0; u < NDX; ++u) {
            constexpr int CPR = XRB / 16;
            const int d = NDX * wave + u, px = d * (1024 / XRB) + lane / CPR, slot = lane % CPR;
            const unsigned off = x_row((unsigned)(t * TP + px)) * XRB + (unsigned)((slot ^ (px & 15)) << 4);
            sdma16(rsX, off, lds0 + buf * BUF + d * 1024);
        }
        if constexpr (RES) {
#pragma unroll
            for (int u = 0; u < NDR; ++u) {
                constexpr int CPR = RRB / 16;
                const int d = NDR * wave + u, px = d * (1024 / RRB) + lane / CPR, slot = lane % CPR;
                const unsigned off = (unsigned)(((long long)t * TP + px) * a.ldy * 2) + (unsigned)((slot ^ (px & 15)) << 4);
                sdma16(rsR, off, lds0 + buf * BUF + XB + d * 1024);
            }
        }
    };
    const bool leaky = a.act == RR_ACT_LEAKY;

    if constexpr (DA == 2) {
        dma(bi, 0);
        if (bi + G < ntiles) dma(bi + G, 1);
    } else {
        // DA tiles ahead, issued whether or not they exist (past the end: offsets past the
        // buffers, zeros), so every wave's vmcnt count is the same on every tile
#pragma unroll
        for (int j = 0; j < DA; ++j) dma(bi + j * G, j);
    }
    for (int k = 0, t = bi; t < ntiles; ++k, t += G) {
        const int cur = k % NBUF;
        if constexpr (DA == 2) {
            // tile t's DMA landed: still in flight after it may be tile t + G's DMA and
            // (k > 0) this wave's stores of tile t - G, issued in that order
            if (t + G < ntiles) {
                if (k == 0) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(ND) : "memory");
                else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(ND + NST) : "memory");
            } else {
                if (k == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(NST) : "memory");
            }
            // every wave is past tile t - G: its buffer takes tile t + 2G
            if (t + 2 * G < ntiles) dma(t + 2 * G, (k + 2) % NBUF);
        } else {
            // tile t's DMA landed: younger are tiles t + G .. t + (DA - 1) G and (k > 0) the
            // stores of tile t - G (older stores are waited for too: an over-wait, safe)
            if (k == 0) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((DA - 1) * ND) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((DA - 1) * ND + NST) : "memory");
            // every wave is past tile t - G: its buffer takes tile t + DA G
            dma(t + DA * G, (k + DA) % NBUF);
        }
        const char* X = smem + cur * BUF;
        const char* Rt = X + XB;
        h16_f32x4_t acc[NI][NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = (h16_f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
            uint4 bx[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int px = 16 * j + r16;
                bx[j] = *reinterpret_cast<const uint4*>(X + px * XRB + (((4 * kk + kq) ^ (px & 15)) << 4));
            }
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[i][j] = H16<H>::mfma(areg[i][kk], bx[j], acc[i][j]);
        }
#pragma unroll
        for (int i2 = 0; i2 < CW / 32; ++i2) {
            const int cl = CW * wave + 32 * i2 + 8 * kq;  // 8 consecutive channels of this lane (PERM32)
            const float4 sc0 = *reinterpret_cast<const float4*>(sS + cl);
            const float4 sc1 = *reinterpret_cast<const float4*>(sS + cl + 4);
            const float4 sh0 = *reinterpret_cast<const float4*>(sH + cl);
            const float4 sh1 = *reinterpret_cast<const float4*>(sH + cl + 4);
            const float sc[8] = {sc0.x, sc0.y, sc0.z, sc0.w, sc1.x, sc1.y, sc1.z, sc1.w};
            const float sh[8] = {sh0.x, sh0.y, sh0.z, sh0.w, sh1.x, sh1.y, sh1.z, sh1.w};
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int px = 16 * j + r16;
                float v[8];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[2 * i2][j][r] * sc[r] + sh[r];
                    v[4 + r] = acc[2 * i2 + 1][j][r] * sc[4 + r] + sh[4 + r];
                }
                if constexpr (RES) {
                    const uint4 q = *reinterpret_cast<const uint4*>(Rt + px * RRB + (((cl >> 3) ^ (px & 15)) << 4));
                    const unsigned w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[2 * r] += H16<H>::lo(w4[r]);
                        v[2 * r + 1] += H16<H>::hi(w4[r]);
                    }
                }
                if (leaky) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
                }
                uint4 o;
                o.x = H16<H>::pack2(v[0], v[1]);
                o.y = H16<H>::pack2(v[2], v[3]);
                o.z = H16<H>::pack2(v[4], v[5]);
                o.w = H16<H>::pack2(v[6], v[7]);
                const long long p = (long long)t * TP + px;
                if (p < P) st16_once(a.y + p * a.ldy + c0 + cl, o);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


}  // namespace
int g_stream_xcd = 1;  // rr_set_tuning(RR_TUNE_STREAM_XCD): channel slices of one strip on one XCD
namespace {

template <int TC, int K, int FN, int D, int NW, typename H>
void launch_s_t(const ConvArgs& a, hipStream_t s) {
    const int g_stream_cus = grid_cus();
    constexpr int LDS = TC * K * 2 + TC * 8;
    constexpr int PER_CU = (160 * 1024 / LDS) >= 2 && NW <= 8 ? (NW <= 4 ? 4 : 2) : 1;
    const int nslices = a.cout / TC;
    const long long nstrips = ((long long)a.P + 16 * FN - 1) / (16 * FN);
    long long per_slice = (long long)PER_CU * g_stream_cus / nslices;
    if (per_slice < 1) per_slice = 1;
    const long long need = (nstrips + NW - 1) / NW;
    if (per_slice > need) per_slice = need;
    const int grid = (int)(per_slice * nslices);
    const int xmap = g_stream_xcd && nslices > 1 && grid % (8 * nslices) == 0;
    if (a.flags & RR_CONV_RESIDUAL)
        hipLaunchKernelGGL((k_stream1x1<TC, K, FN, D, NW, true, H>), dim3(grid), dim3(64 * NW), 0, s, a, nslices, xmap);
    else
        hipLaunchKernelGGL((k_stream1x1<TC, K, FN, D, NW, false, H>), dim3(grid), dim3(64 * NW), 0, s, a, nslices, xmap);
}

}  // namespace

int g_stream_mode = 1;  // rr_set_tuning(RR_TUNE_STREAM_1X1): 0 off, 1 auto, 2 / 3 see launch_stream1x1
int g_wres = 2;         // rr_set_tuning(RR_TUNE_WRES)
int g_pair_mid = 1;     // rr_set_tuning(RR_TUNE_PAIR_MID): 1 k_pair_mid_ring (default), 0 k_pair_mid
int g_wres_ring = 1;    // rr_set_tuning(RR_TUNE_WRES_RING): 1 deep rings for the non-residual k_wres1x1, 0 two ahead

namespace {
template <int K, int CW>
void launch_wres(const ConvArgs& a, hipStream_t s, bool f16) {
    constexpr int BC = 8 * CW;
    const bool res = a.flags & RR_CONV_RESIDUAL;
    WresArgs w;
    w.w = (const bf16_t*)a.w;
    const bool affine = a.flags & RR_CONV_AFFINE;
    w.scale = affine ? a.scale : nullptr;
    w.shift = affine ? a.shift : nullptr;
    w.ldy = a.ldy;
    w.act = a.act;
    w.slope = a.slope;
    w.h = a.h; w.w_ = a.w_; w.ho = a.ho; w.wo = a.wo; w.stride = a.stride;
    w.nslices = a.cout / BC;
    int per = grid_cus() / w.nslices;
    if (per < 1) per = 1;
    // whole-image chunks whose input and residual / output stay inside 31-bit buffer offsets
    const long long in_img = (long long)a.h * a.w_ * K * 2, out_img = (long long)a.ho * a.wo * a.ldy * 2;
    long long ich = (1ll << 31) / (in_img > out_img ? in_img : out_img);
    if (ich < 1) ich = 1;
    const long long hw = (long long)a.ho * a.wo;
    for (long long i0 = 0; i0 < a.n; i0 += ich) {
        const long long ni = a.n - i0 < ich ? a.n - i0 : ich;
        w.x = (const bf16_t*)a.x + i0 * a.h * a.w_ * K;
        w.res = res ? (const bf16_t*)a.res + i0 * hw * a.ldy : nullptr;
        w.y = (bf16_t*)a.y + i0 * hw * a.ldy;
        w.P = ni * hw;
        const long long ntiles = (w.P + 31) / 32;
        const int ps = (int)(per < ntiles ? per : ntiles);
        const int grid = ps * w.nslices;
        w.xmap = w.nslices > 1 && grid % (8 * w.nslices) == 0;
        auto go = [&](auto h) {
            using H = decltype(h);
            if (res) hipLaunchKernelGGL((k_wres1x1<K, CW, true, H>), dim3(grid), dim3(512), 0, s, w);
            else if (g_wres_ring) hipLaunchKernelGGL((k_wres1x1<K, CW, false, H>), dim3(grid), dim3(512), 0, s, w);
            else hipLaunchKernelGGL((k_wres1x1<K, CW, false, H, false>), dim3(grid), dim3(512), 0, s, w);
        };
        if (f16) go(f16_t{});
        else go(bf16_t{});
    }
}
}  // namespace

// bf16 1x1 (pad 0, any stride), PERM32 weights, bf16 out: returns false when the
// shape is not one the streaming kernel is built for (caller uses the tiled engine).
template <int TC, int K, int FN, int D, int NW>
void launch_s(const ConvArgs& a, hipStream_t s, bool f16) {
    if (f16) launch_s_t<TC, K, FN, D, NW, f16_t>(a, s);
    else launch_s_t<TC, K, FN, D, NW, bf16_t>(a, s);
}

bool gemm8_eligible(const ConvArgs& a, bool k1, int esz);  // rr_gemm.hip

bool launch_stream1x1(const ConvArgs& a, hipStream_t s, bool f16) {
    if (g_stream_mode == 0) return false;
    if (!(a.flags & RR_CONV_PERM32) || a.kh != 1 || a.kw != 1 || a.pad != 0 || a.kp != a.cin) return false;
    if (a.P < 4096 || (long long)a.n * a.h * a.w_ * a.cin >= (1ll << 31)) return false;
    const bool res = a.flags & RR_CONV_RESIDUAL;
    const int K = a.cin, C = a.cout;
    if (g_wres && (a.ldy & 7) == 0 && (a.stride == 1 ? a.h == a.ho && a.w_ == a.wo : !res)) {
        if (K == 512 && C == 2048 && res) { launch_wres<512, 32>(a, s, f16); return true; }
        if (K == 256 && C == 1024 && res) { launch_wres<256, 64>(a, s, f16); return true; }
        // the mod3 block-1 conv3 (128 -> 512 + the projection shortcut): one 512-channel slice,
        // so its input is read once (the streaming kernel's two slices re-read it)
        if (K == 128 && C == 512 && res) { launch_wres<128, 64>(a, s, f16); return true; }
        if (g_wres >= 2) {  // the non-residual K = 256 / 512 1x1s (projections, mod4 block-1 conv1)
            if (K == 512 && (C == 256 || C == 1024 || C == 2048) && !res) { launch_wres<512, 32>(a, s, f16); return true; }
            if (K == 256 && (C == 512 || C == 1024) && !res) { launch_wres<256, 64>(a, s, f16); return true; }
        }
    }
    // mode 2: the residual 512 -> 2048 1x1 (mod5 conv3) on the 8-phase GEMM;
    // mode 3: also the residual 256 -> 1024 1x1 (mod4 conv3)
    if (g_stream_mode >= 2 && K == 512 && C == 2048 && res && gemm8_eligible(a, true, 2)) return false;
    if (g_stream_mode >= 3 && K == 256 && C == 1024 && res && gemm8_eligible(a, true, 2)) return false;
    if (K == 64 && C == 64) { launch_s<64, 64, 2, 4, 8>(a, s, f16); return true; }
    if (K == 64 && C == 256) { launch_s<256, 64, 1, 2, 8>(a, s, f16); return true; }
    if (K == 256 && C == 64) { launch_s<64, 256, 1, 4, 8>(a, s, f16); return true; }
    if (K == 256 && C == 128) { launch_s<128, 256, 1, 3, 8>(a, s, f16); return true; }
    if (K == 128 && C == 512) { launch_s<256, 128, 1, 3, 8>(a, s, f16); return true; }
    if (K == 512 && C == 128) { launch_s<128, 512, 1, 2, 8>(a, s, f16); return true; }
    if (K == 256 && C == 1024 && res) { launch_s<256, 256, 1, 2, 8>(a, s, f16); return true; }
    if (K == 256 && C == 512 && !res) { launch_s<256, 256, 1, 2, 8>(a, s, f16); return true; }
    // 128-channel slices of a 512-deep panel: the input is re-read per slice
    // (from L2 / Infinity Cache: slices of one strip run side by side), the
    // output and residual stream once (mod5 conv3 461 -> 600, mod4 conv1
    // 606 -> 673, mod4 projection 632 -> 695 TFLOP/s at 128 images vs the
    // tiled engine).  K = 1024 does not fit: one strip's B operand alone is
    // 128 VGPRs, and a single-strip-deep stream measured 395-410 vs 712-720.
    if (K == 512 && C == 2048 && res) { launch_s<128, 512, 1, 2, 8>(a, s, f16); return true; }
    // K = 512 without residual into 256 / 1024 channels (mod4 conv1 of block 1, the
    // strided mod4 projection): the 8-phase GEMM is faster where it applies
    // (587 vs 623, 548 vs 598 us at 128 images)
    if (K == 512 && !res && (C == 256 || C == 1024) && gemm8_eligible(a, true, 2)) return false;
    if (K == 512 && C == 256 && !res) { launch_s<128, 512, 1, 2, 8>(a, s, f16); return true; }
    if (K == 512 && C == 1024 && !res) { launch_s<128, 512, 1, 2, 8>(a, s, f16); return true; }
    return false;
}


}  // namespace rr

using namespace rr;

extern "C" int rr_conv1x1_pair(const void* x, long long p, int c_in, const void* w3, const float* scale3,
                               const float* shift3, int c_mid, const void* residual, const void* xp, const void* wp,
                               const float* scalep, const float* shiftp, int act3, float slope3, const void* w1,
                               const float* scale1, const float* shift1, int c_out, int act1, float slope1, void* y,
                               void* z, int dtype, void* stream) {
    if (dtype != RR_BF16 && dtype != RR_F16) return fail(RR_EINVAL, "rr_conv1x1_pair: bf16 / fp16 only");
    const bool stage2 = c_in == 64 && c_mid == 256 && (c_out == 64 || c_out == 128);
    const bool stage3 = c_in == 128 && c_mid == 512 && c_out == 128;
    if (!stage2 && !stage3)
        return fail(RR_EINVAL, "rr_conv1x1_pair: shapes (c_in 64, c_mid 256, c_out 64|128) or (128, 512, 128) only");
    if (!x || !w3 || !scale3 || !shift3 || !w1 || !scale1 || !shift1 || !y || !z)
        return fail(RR_EINVAL, "rr_conv1x1_pair: null pointer");
    const bool proj = residual == nullptr;
    if (proj && stage3) return fail(RR_EINVAL, "rr_conv1x1_pair: the 128/512 boundary needs a residual");
    if (proj && (!xp || !wp || !scalep || !shiftp))
        return fail(RR_EINVAL, "rr_conv1x1_pair: either residual or the projection (xp, wp, scalep, shiftp) is required");
    if (proj && ((((uintptr_t)xp) | ((uintptr_t)wp)) & 15))
        return fail(RR_EINVAL, "rr_conv1x1_pair: 16-byte alignment required");
    if (p <= 0) return fail(RR_EINVAL, "rr_conv1x1_pair: empty");
    if ((((uintptr_t)x) | ((uintptr_t)residual) | ((uintptr_t)y) | ((uintptr_t)z) | ((uintptr_t)w3) |
         ((uintptr_t)w1)) & 15)
        return fail(RR_EINVAL, "rr_conv1x1_pair: 16-byte alignment required");
    if (act3 != RR_ACT_IDENTITY && act3 != RR_ACT_LEAKY) return fail(RR_EINVAL, "rr_conv1x1_pair: act3");
    if (act1 != RR_ACT_IDENTITY && act1 != RR_ACT_LEAKY) return fail(RR_EINVAL, "rr_conv1x1_pair: act1");
    const int g_pair_cus = grid_cus();
    hipStream_t s = as_stream(stream);
    if (stage3) {
        // pixel chunks of 2^20 (the residual buffer resource addresses 1 GiB with 32-bit offsets)
        constexpr long long CH = 1ll << 20;
        for (long long p0 = 0; p0 < p; p0 += CH) {
            PairMidArgs m;
            const long long pn = p - p0 < CH ? p - p0 : CH;
            m.x = (const bf16_t*)x + p0 * 128; m.w3 = (const bf16_t*)w3; m.s3 = scale3; m.h3 = shift3;
            m.res = (const bf16_t*)residual + p0 * 512; m.w1 = (const bf16_t*)w1; m.s1 = scale1; m.h1 = shift1;
            m.y = (bf16_t*)y + p0 * 512; m.z = (bf16_t*)z + p0 * 128; m.P = pn;
            m.act3 = act3; m.act1 = act1; m.slope3 = slope3; m.slope1 = slope1;
            const long long ntiles = (pn + (g_pair_mid ? 31 : 63)) / (g_pair_mid ? 32 : 64);
            const int grid = (int)(ntiles < g_pair_cus ? ntiles : g_pair_cus);
            if (g_pair_mid) {
                if (dtype == RR_F16) hipLaunchKernelGGL(k_pair_mid_ring<f16_t>, dim3(grid), dim3(512), 0, s, m);
                else hipLaunchKernelGGL(k_pair_mid_ring<bf16_t>, dim3(grid), dim3(512), 0, s, m);
            } else {
                if (dtype == RR_F16) hipLaunchKernelGGL(k_pair_mid<f16_t>, dim3(grid), dim3(512), 0, s, m);
                else hipLaunchKernelGGL(k_pair_mid<bf16_t>, dim3(grid), dim3(512), 0, s, m);
            }
        }
        return check_launch("rr_conv1x1_pair");
    }
    PairArgs a;
    a.x = (const bf16_t*)x; a.w3 = (const bf16_t*)w3; a.s3 = scale3; a.h3 = shift3; a.res = (const bf16_t*)residual;
    a.w1 = (const bf16_t*)w1; a.s1 = scale1; a.h1 = shift1; a.y = (bf16_t*)y; a.z = (bf16_t*)z; a.P = p;
    a.act3 = act3; a.act1 = act1; a.slope3 = slope3; a.slope1 = slope1;
    a.xp = (const bf16_t*)xp; a.wp = (const bf16_t*)wp; a.sp = scalep; a.hp = shiftp;
    const long long nstrips = (p + 15) / 16;
    long long grid = (nstrips + 7) / 8;
    if (grid > g_pair_cus) grid = g_pair_cus;
    const dim3 g((unsigned)grid), b(512);
    auto go = [&](auto h) {
        using H = decltype(h);
        if (c_out == 64 && !proj) hipLaunchKernelGGL((k_stream_pair<64, 2, false, H>), g, b, 0, s, a);
        else if (c_out == 64) hipLaunchKernelGGL((k_stream_pair<64, 2, true, H>), g, b, 0, s, a);
        else if (!proj) hipLaunchKernelGGL((k_stream_pair<128, 2, false, H>), g, b, 0, s, a);
        else hipLaunchKernelGGL((k_stream_pair<128, 2, true, H>), g, b, 0, s, a);
    };
    if (dtype == RR_F16) go(f16_t{});
    else go(bf16_t{});
    return check_launch("rr_conv1x1_pair");
}
