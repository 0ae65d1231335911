// librr.so — direct 3x3 convolution (stride 1, pad 1, bf16) with the input
// halo patch staged ONCE in LDS.
//
// The implicit-GEMM engine (rr_gemm.hip) stages an im2col B tile per K-step,
// so every input pixel crosses the L2 -> LDS path 9 times (once per tap): the
// 3x3 layers of the bottleneck blocks run at 50-100 FLOP per staged byte and
// are bound by that path, not by the matrix cores.  Here a block owns an
// output tile of TH x TW pixels of one image x TC output channels; per
// 64-channel input chunk it stages the (TH+2) x (TW+2) halo patch once and
// reads the 9 taps out of LDS by address offset (6x fewer staged bytes at
// 8 x 32 tiles).  With 64 input channels the block's whole weight slice
// (9 taps x TC rows x 128 B) also stays resident in LDS ("A-stationary");
// otherwise the 128-B weight K-steps stream through a 2-stage ring and the
// next chunk's patch is fetched one 1-KiB piece per tap behind them.
//
// K order per output tile: (input chunk cc, tap, 64 channels).  The standard
// packed weight row (k = tap*c_in + ci, RR_CONV_PERM32 rows) is read at
// k0 = tap*c_in + cc*64, so no special packing is needed.
// LDS images: weight K-step [TC rows][128 B], patch [pixel][128 B]; both with
// the 16-B chunk XOR swizzle (chunk ^ (row & 7)) applied on the DMA source, so
// every ds_read_b128 lane group of a fragment read hits distinct slots.
// Synchronisation: LDS-DMA (buffer_load ... lds) tracked by counted vmcnt +
// raw s_barrier; the epilogue reads BN scale/shift from LDS, so no
// compiler-visible global load ever drains the DMA queue.
//
// Replaces the 3x3 nn.Conv2d of ResidualBlock (cirtorch/backbones/misc.py:
// 166-172, stride on this conv; here the stride-1 blocks) + the ABN eval BN +
// leaky_relu (cirtorch/utils/misc.py:175-235).
#include "rr_internal.h"

#include <type_traits>

namespace rr {

namespace {

typedef __attribute__((ext_vector_type(4))) float pf32x4_t;
typedef __attribute__((ext_vector_type(4))) int pi32x4_t;

constexpr unsigned POOB = 0x80000000u;  // voffset beyond every buffer: the DMA writes zeros

// One 16-B-per-lane LDS-DMA wave-instruction: LDS[lds_addr + lane*16] = buf[voff].
__device__ __forceinline__ void pdma16(pi32x4_t rsrc, unsigned voff, unsigned lds_addr) {
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

template <int N>
__device__ __forceinline__ void pwait_barrier() {
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(N) : "memory");
}
// vmcnt(n) + barrier for a wave-uniform runtime n <= N (a chain of scalar
// compares picks the exact immediate).
template <int N>
__device__ __forceinline__ void pwait_barrier_n(int n) {
    if constexpr (N == 0) {
        pwait_barrier<0>();
    } else {
        if (n >= N) pwait_barrier<N>();
        else pwait_barrier_n<N - 1>(n);
    }
}

__device__ __forceinline__ pi32x4_t prsrc(const void* base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)base;
    pi32x4_t r;
    r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)b);
    r.y = __builtin_amdgcn_readfirstlane((int)((unsigned)(b >> 32) & 0xFFFFu));
    r.z = __builtin_amdgcn_readfirstlane((int)bytes);
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

struct TileC {
    int ct, img, oh0, ow0;
};

template <int TC, int TH, int TW, int WC, int WP, bool ARES, int NSA, typename HT>
__global__ void __launch_bounds__(64 * WC * WP) k_conv3x3(ConvArgs a, int tiles_w, int tiles_hw, int tiles_c,
                                                         int ntiles, int g_pipe) {
    constexpr int NW = WC * WP, NT = 64 * NW;
    constexpr int TP = TH * TW;
    constexpr int PC = TW + 2, NPIX = (TH + 2) * PC;
    constexpr int NDP = (NPIX + 7) / 8;          // patch wave-instructions (8 pixels x 128 B each)
    constexpr int NDPW = (NDP + NW - 1) / NW;    // ... per wave (ring mode: one per tap)
    constexpr int PBYTES = (ARES ? NDP : NDPW * NW) * 1024;
    constexpr int NIA = TC / (8 * NW);           // weight wave-instructions per wave per K-step
    constexpr int AST = TC * 128;                // one weight K-step in LDS
    constexpr int ABYTES = (ARES ? 9 : NSA) * AST;
    constexpr int MAXC = ARES ? TC : 512;        // BN scale/shift of every output channel
    constexpr int FM = TC / WC / 16, FN = TP / WP / 16;
    constexpr int NST = (FM / 2) * FN;           // epilogue stores per wave (full tiles only)
    static_assert(TC % (8 * NW) == 0 && FM % 2 == 0 && TW % 16 == 0 && (TP / WP) % 16 == 0, "tile shape");
    static_assert(ARES || NDPW <= 8, "ring mode fetches the next patch one piece per tap (taps 0..7)");
    static_assert(NST >= 2, "vmcnt immediates below assume NST > 1");
    static_assert(NSA == 2 || NSA == 3, "weight ring depth");
    __shared__ __attribute__((aligned(1024))) char smem[ABYTES + 2 * PBYTES + 2 * MAXC * 4];
    float* sS = reinterpret_cast<float*>(smem + ABYTES + 2 * PBYTES);
    float* sH = sS + MAXC;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wc = wave % WC, wp = wave / WC;
    const int H = a.h, W = a.w_, Cin = a.cin, nck = Cin >> 6;
    const pi32x4_t rsX = prsrc(a.x, (unsigned)((long long)a.n * H * W * Cin * 2));
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    const int lrow = lane >> 3, lch = lane & 7;

    {
        const bool aff = a.flags & RR_CONV_AFFINE;
        for (int i = tid; i < a.cout; i += NT) {
            sS[i] = aff ? a.scale[i] : 1.f;
            sH[i] = aff ? a.shift[i] : 0.f;
        }
    }
    __syncthreads();  // affine visible to every wave (read into VGPRs by the overlapped epilogue)
    const int my_tiles = (int)blockIdx.x < ntiles ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    if (my_tiles == 0) return;

    auto tile_of = [&](int lt) {
        const int t = (int)blockIdx.x + lt * (int)gridDim.x;
        TileC c;
        c.ct = t % tiles_c;
        const int pt = t / tiles_c;
        c.img = pt / tiles_hw;
        const int rem = pt - c.img * tiles_hw;
        const int th = rem / tiles_w;
        c.oh0 = th * TH;
        c.ow0 = (rem - th * tiles_w) * TW;
        return c;
    };

    // wave-instruction d of the patch of (tile, chunk cc) -> patch buffer `buf`:
    // patch pixels 8d .. 8d+7 (origin (oh0-1, ow0-1)); outside the image -> zeros
    auto patch_dma = [&](TileC tc, int cc, int buf, int d) {
        const int q = d * 8 + lrow;
        const int pr = q / PC, pc = q - pr * PC;
        const int hh = tc.oh0 - 1 + pr, ww = tc.ow0 - 1 + pc;
        unsigned off = POOB;
        if (q < NPIX && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
            off = (unsigned)(((((long long)tc.img * H + hh) * W + ww) * Cin + cc * 64 + ((lch ^ lrow) << 3)) * 2);
        pdma16(rsX, off, lds0 + ABYTES + buf * PBYTES + d * 1024);
    };
    // weight K-step (tap, chunk cc) of channel tile ct -> LDS dst ([TC rows][128 B], swizzled)
    auto w_dma = [&](int ct, int tap, int cc, unsigned dst) {
        const pi32x4_t rsW = prsrc((const char*)a.w + (long long)ct * TC * a.kp * 2, (unsigned)(TC * a.kp * 2));
        const unsigned k0b = (unsigned)((tap * Cin + cc * 64) * 2);
#pragma unroll
        for (int i = 0; i < NIA; ++i) {
            const int row = (wave + NW * i) * 8 + lrow;
            pdma16(rsW, (unsigned)(row * a.kp * 2) + k0b + (unsigned)((lch ^ lrow) << 4), dst + (wave + NW * i) * 1024);
        }
    };

    const int r16 = lane & 15, kq = lane >> 4;
    const int arow0 = wc * (TC / WC) + r16;
    int bq[FN];  // patch pixel read by this lane for fragment j at tap (0, 0)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        const int p = wp * (TP / WP) + j * 16;
        bq[j] = (p / TW) * PC + (p % TW) + r16;
    }

    pf32x4_t acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = (pf32x4_t){0.f, 0.f, 0.f, 0.f};

    // A / B fragments of half-step hs (channels 32*hs .. +31 of the 64-channel
    // K-step) at tap offset toff, and the FM x FN MFMAs on them
    auto frag_load = [&](const char* As, const char* Ps, int toff, int hs, uint4 (&fa)[FM], uint4 (&fb)[FN]) {
        const int ch = kq + 4 * hs;
#pragma unroll
        for (int i = 0; i < FM; ++i)
            fa[i] = *reinterpret_cast<const uint4*>(As + (arow0 + i * 16) * 128 + ((ch ^ (r16 & 7)) << 4));
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int q = bq[j] + toff;
            fb[j] = *reinterpret_cast<const uint4*>(Ps + q * 128 + ((ch ^ (q & 7)) << 4));
        }
    };
    auto frag_mfma = [&](const uint4 (&fa)[FM], const uint4 (&fb)[FN]) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
                acc[i][j] = H16<HT>::mfma(fa[i], fb[j], acc[i][j]);
    };
    auto mfma_step = [&](const char* As, const char* Ps, int toff) {
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) {
            uint4 fa[FM], fb[FN];
            frag_load(As, Ps, toff, hs, fa, fb);
            frag_mfma(fa, fb);
        }
    };
    bf16_t* __restrict__ Y = (bf16_t*)a.y;
    const bool leaky = a.act == RR_ACT_LEAKY;
    const float slope = a.slope;
    // PERM32 rows: a lane's fragment pair (2*i2, 2*i2+1) holds 8 consecutive
    // output channels of one pixel -> one 16-B store; exactly NST stores.
    // one 16-B store of the epilogue: fragment pair (2*i2, 2*i2+1) x pixel
    // fragment j of accumulators `ac`, BN affine (sc, sh: this lane's 8 channels)
    auto store_one = [&](const TileC& tc, const pf32x4_t (&ac)[FM][FN], int i2, int j, const float (&sc)[8],
                         const float (&sh)[8]) {
        const int c = tc.ct * TC + wc * (TC / WC) + 32 * i2 + 8 * kq;
        const int p = wp * (TP / WP) + j * 16 + r16;
        const long long pix = ((long long)tc.img * H + tc.oh0 + p / TW) * W + tc.ow0 + p % TW;
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            v[r] = ac[2 * i2][j][r] * sc[r] + sh[r];
            v[4 + r] = ac[2 * i2 + 1][j][r] * sc[4 + r] + sh[4 + r];
        }
        if (leaky) {
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * slope;
        }
        uint4 o;
        o.x = H16<HT>::pack2(v[0], v[1]);
        o.y = H16<HT>::pack2(v[2], v[3]);
        o.z = H16<HT>::pack2(v[4], v[5]);
        o.w = H16<HT>::pack2(v[6], v[7]);
        *reinterpret_cast<uint4*>(Y + pix * a.ldy + c) = o;
    };
    auto load_affine = [&](int ct, int i2, float (&sc)[8], float (&sh)[8]) {
        const int c = ct * TC + wc * (TC / WC) + 32 * i2 + 8 * kq;
        const float4 s0 = *reinterpret_cast<const float4*>(sS + c);
        const float4 s1 = *reinterpret_cast<const float4*>(sS + c + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(sH + c);
        const float4 h1 = *reinterpret_cast<const float4*>(sH + c + 4);
        sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w; sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
        sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w; sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
    };
    // PERM32 rows: a lane's fragment pair (2*i2, 2*i2+1) holds 8 consecutive
    // output channels of one pixel -> one 16-B store; exactly NST stores.
    auto epilogue = [&](const TileC& tc) {
#pragma unroll
        for (int i2 = 0; i2 < FM / 2; ++i2) {
            float sc[8], sh[8];
            load_affine(tc.ct, i2, sc, sh);
#pragma unroll
            for (int j = 0; j < FN; ++j) store_one(tc, acc, i2, j, sc, sh);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = (pf32x4_t){0.f, 0.f, 0.f, 0.f};
    };

    TileC cur = tile_of(0);
    if constexpr (ARES) {
        // c_in = 64, one channel tile: weights for all 9 taps stay resident; per
        // tile one barrier, the next tile's patch in flight during this one.
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) w_dma(0, tap, 0, lds0 + tap * AST);
        for (int d = wave; d < NDP; d += NW) patch_dma(cur, 0, 0, d);
        if (g_pipe) {
            // Epilogue overlap: tile lt's stores are computed from a copy of its
            // accumulators (accP) during tile lt + 1's MFMAs, one store after
            // every few half-steps, so the VALU / store issue of the epilogue
            // hides under the matrix pipe instead of idling it between tiles
            // (all waves reach the epilogue together: one barrier per tile).
            // Branch-free activation: leaky(v) = max(v, slope * v) for slope in
            // [0, 1] (host-checked; identity = slope 1), bit-equal to the select form.
            pf32x4_t accP[FM][FN];
            float esc[FM / 2][8], esh[FM / 2][8];  // one channel tile: the affine stays in VGPRs
            const float sl = leaky ? slope : 1.f;
            auto store_bf = [&](const TileC& tc, int i2, int j) {
                const int c = wc * (TC / WC) + 32 * i2 + 8 * kq;
                const int p = wp * (TP / WP) + j * 16 + r16;
                const long long pix = ((long long)tc.img * H + tc.oh0 + p / TW) * W + tc.ow0 + p % TW;
                float v[8];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = accP[2 * i2][j][r] * esc[i2][r] + esh[i2][r];
                    v[4 + r] = accP[2 * i2 + 1][j][r] * esc[i2][4 + r] + esh[i2][4 + r];
                }
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] = fmaxf(v[r], v[r] * sl);
                uint4 o;
                o.x = H16<HT>::pack2(v[0], v[1]);
                o.y = H16<HT>::pack2(v[2], v[3]);
                o.z = H16<HT>::pack2(v[4], v[5]);
                o.w = H16<HT>::pack2(v[6], v[7]);
                *reinterpret_cast<uint4*>(Y + pix * a.ldy + c) = o;
            };
            TileC prev = cur;
            auto tile_body = [&](auto has_prev, int lt) {
                const char* Ps = smem + ABYTES + (lt & 1) * PBYTES;
                constexpr int GAP = 18 / NST > 0 ? 18 / NST : 1;
                // per-tile opaque copies of the patch pixel indices: the 18 x FN fragment
                // addresses are derived inside the tile instead of being hoisted out of
                // the tile loop as loop invariants (they would not fit beside accP)
                int bql[FN];
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    bql[j] = bq[j];
                    asm volatile("" : "+v"(bql[j]));
                }
#pragma unroll
                for (int s = 0; s < 18; ++s) {
                    const int tap = s >> 1;
                    uint4 fa[FM], fb[FN];
                    {
                        const int ch = kq + 4 * (s & 1), toff = (tap / 3) * PC + tap % 3;
                        const char* As = smem + tap * AST;
#pragma unroll
                        for (int i = 0; i < FM; ++i)
                            fa[i] = *reinterpret_cast<const uint4*>(As + (arow0 + i * 16) * 128 + ((ch ^ (r16 & 7)) << 4));
#pragma unroll
                        for (int j = 0; j < FN; ++j) {
                            const int q = bql[j] + toff;
                            fb[j] = *reinterpret_cast<const uint4*>(Ps + q * 128 + ((ch ^ (q & 7)) << 4));
                        }
                    }
                    frag_mfma(fa, fb);
                    if constexpr (decltype(has_prev)::value) {
                        if (s % GAP == GAP - 1 && s / GAP < NST) store_bf(prev, (s / GAP) / FN, (s / GAP) % FN);
                    }
                }
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        accP[i][j] = acc[i][j];
                        acc[i][j] = (pf32x4_t){0.f, 0.f, 0.f, 0.f};
                    }
            };
            for (int lt = 0; lt < my_tiles; ++lt) {
                // patch(lt) landed; from lt = 2 on the NST stores of tile lt - 2 (issued
                // during tile lt - 1, after patch(lt)'s DMA) may stay in flight
                if (lt <= 1) pwait_barrier<0>();
                else pwait_barrier<NST>();
                if (lt == 0) {
#pragma unroll
                    for (int i2 = 0; i2 < FM / 2; ++i2) load_affine(0, i2, esc[i2], esh[i2]);
                }
                if (lt + 1 < my_tiles) {
                    const TileC nxt = tile_of(lt + 1);
                    for (int d = wave; d < NDP; d += NW) patch_dma(nxt, 0, (lt + 1) & 1, d);
                }
                if (lt == 0) tile_body(std::false_type{}, lt);
                else tile_body(std::true_type{}, lt);
                prev = cur;
                if (lt + 1 < my_tiles) cur = tile_of(lt + 1);
            }
#pragma unroll
            for (int e = 0; e < NST; ++e) store_bf(prev, e / FN, e % FN);
        } else {
            for (int lt = 0; lt < my_tiles; ++lt) {
                // patch(lt) landed (older than the previous tile's NST epilogue stores)
                if (lt == 0) pwait_barrier<0>();
                else pwait_barrier<NST>();
                if (lt + 1 < my_tiles) {
                    const TileC nxt = tile_of(lt + 1);
                    for (int d = wave; d < NDP; d += NW) patch_dma(nxt, 0, (lt + 1) & 1, d);
                }
                const char* Ps = smem + ABYTES + (lt & 1) * PBYTES;
#pragma unroll
                for (int tap = 0; tap < 9; ++tap) mfma_step(smem + tap * AST, Ps, (tap / 3) * PC + tap % 3);
                epilogue(cur);
                if (lt + 1 < my_tiles) cur = tile_of(lt + 1);
            }
        }
    } else {
        // steps (tile, chunk, tap); weight K-steps through an NSA-stage ring, one
        // barrier per step; the next (tile, chunk) patch arrives piecewise.
        const int total = my_tiles * nck * 9;
        TileC nxt = my_tiles > 1 ? tile_of(1) : cur;
        auto adv = [&](int& t_, int& c_, int& l_) {
            if (++t_ == 9) {
                t_ = 0;
                if (++c_ == nck) { c_ = 0; ++l_; }
            }
        };
        for (int d = wave; d < NDP; d += NW) patch_dma(cur, 0, 0, d);
        int ptap = 0, pcc = 0, plt = 0;  // next weight K-step to fetch
        for (int i = 0; i < NSA - 1 && i < total; ++i) {
            w_dma(plt == 0 ? cur.ct : nxt.ct, ptap, pcc, lds0 + i * AST);
            adv(ptap, pcc, plt);
        }
        int lt = 0, cc = 0, tap = 0, grp = 0;
        int tm1 = 0, tm2 = 0, am1 = 0;  // VMEM ops after the weight fetch of steps s-1, s-2; weight ops of s-1
        for (int s = 0; s < total; ++s) {
            // A(s) landed; only the younger VMEM ops (later weight steps, patch
            // pieces, the previous tile's epilogue stores) may stay in flight
            if (s == 0) pwait_barrier<0>();
            else if constexpr (NSA == 2) pwait_barrier_n<NST + 1>(tm1);
            else pwait_barrier_n<NIA + NST + 2>(tm2 + am1 + tm1);
            int ntap = tap, ncc = cc, nlt = lt;
            adv(ntap, ncc, nlt);
            int a_now = 0, t_now = 0;
            if (s + NSA - 1 < total) {  // weight K-step s + NSA - 1 into the slot step s - 1 used
                w_dma(plt == lt ? cur.ct : nxt.ct, ptap, pcc, lds0 + ((s + NSA - 1) % NSA) * AST);
                adv(ptap, pcc, plt);
                a_now = NIA;
            }
            if (tap < NDPW) {  // piece `tap` of the next group's patch
                const bool same = cc + 1 < nck;
                if (same || lt + 1 < my_tiles) {
                    TileC g;  // field-wise select (a selected reference would live in scratch)
                    g.ct = same ? cur.ct : nxt.ct;
                    g.img = same ? cur.img : nxt.img;
                    g.oh0 = same ? cur.oh0 : nxt.oh0;
                    g.ow0 = same ? cur.ow0 : nxt.ow0;
                    patch_dma(g, same ? cc + 1 : 0, (grp + 1) & 1, wave + NW * tap);
                    t_now = 1;
                }
            }
            mfma_step(smem + (s % NSA) * AST, smem + ABYTES + (grp & 1) * PBYTES, (tap / 3) * PC + tap % 3);
            if (ntap == 0) {
                ++grp;
                if (ncc == 0) {
                    epilogue(cur);
                    t_now += NST;
                    cur = nxt;
                    if (nlt + 1 < my_tiles) nxt = tile_of(nlt + 1);
                }
            }
            tm2 = tm1;
            tm1 = t_now;
            am1 = a_now;
            tap = ntap;
            cc = ncc;
            lt = nlt;
        }
    }
}

// ---------------------------------------------------------------------------
// mod2 3x3 (c_in = c_out = 64) with the weights in VGPRs.  k_conv3x3's
// A-stationary form reads both operands from LDS: per MFMA 0.75 KiB (2 A + 4 B
// fragments per 8 MFMAs), and the 72 KiB weight image leaves room for only two
// halo patches.  Here each wave keeps its 32 output channels x all 576 K of
// the PERM32 weights in VGPRs (2 x 18 fragments, 144 VGPRs) for the whole
// launch, so a B fragment read from LDS feeds 2 MFMAs and nothing else is
// read; the LDS holds three 8x32-tile halo patches, prefetched two tiles ahead
// by LDS-DMA.  The patch rows are laid out 40 pixel slots apart (34 used): a
// multiple of 8, so the chunk swizzle (chunk ^ (slot & 7)) is the same on
// every patch row and the 18 K-steps' fragment addresses are 24 per-lane
// bases (pixel fragment x tap column x half-step) plus immediate row offsets
// — no address arithmetic between the MFMAs.
// Persistent block per CU, 8 waves = 2 channel halves x 4 pixel quarters;
// tiles walked XCD-contiguously (the 32 tiles an XCD holds at once are 4 tile
// rows of one image: vertical halo re-reads hit its L2).  Accumulation order
// (tap, half-step) equals k_conv3x3's: bit-identical outputs.
// A value loaded once before a loop (weights kept in VGPRs): passing it through an
// empty asm makes the asm its producer, so the compiler's wait for the load sits
// before the loop instead of (counted against the loop's own LDS-DMA / stores,
// which it cannot see) in front of every use inside it.
__device__ __forceinline__ void pin_loaded(uint4& v) {
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
}

template <typename HT>
__global__ void __launch_bounds__(512, 1) k_c3w64(ConvArgs a, int tiles_w, int tiles_hw, int ntiles) {
    constexpr int TH = 8, TW = 32, TP = TH * TW, PCW = TW + 2, PITCH = 40;  // 34 patch columns, 40 slots
    constexpr int NSLOT = (TH + 2) * PITCH, NP = NSLOT / 8;                 // 400 slots, 50 pieces of 8
    constexpr int PBYTES = NP * 1024;
    constexpr int NBUF = 3, FN = TP / 4 / 16, NST = FN;  // per wave: 4 pixel fragments, 4 epilogue stores
    static_assert(PITCH % 8 == 0 && NSLOT % 8 == 0, "row-invariant swizzle");
    __shared__ __attribute__((aligned(1024))) char smem[NBUF * PBYTES];
    __shared__ __attribute__((aligned(16))) float sS[64], sH[64];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wc = wave & 1, wp = wave >> 1;
    const int r16 = lane & 15, kq = lane >> 4, lrow = lane >> 3, lch = lane & 7;
    const int H = a.h, W = a.w_;
    if (tid < 64) {
        const bool aff = a.flags & RR_CONV_AFFINE;
        sS[tid] = aff ? a.scale[tid] : 1.f;
        sH[tid] = aff ? a.shift[tid] : 0.f;
    }
    uint4 areg[2][18];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int s = 0; s < 18; ++s)
            areg[i][s] = *reinterpret_cast<const uint4*>((const bf16_t*)a.w + (long long)(32 * wc + 16 * i + r16) * 576 +
                                                         (s >> 1) * 64 + 32 * (s & 1) + 8 * kq);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int s = 0; s < 18; ++s) pin_loaded(areg[i][s]);
    __syncthreads();

    // XCD-contiguous walk: round i, XCD x = b & 7 takes tiles [i G + x G/8, ... + G/8)
    const int b = (int)blockIdx.x, G = (int)gridDim.x;
    auto tile_id = [&](int i) { return i * G + (b & 7) * (G >> 3) + (b >> 3); };
    const pi32x4_t rsX = prsrc(a.x, (unsigned)((long long)a.n * H * W * 64 * 2));
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    // pieces d = wave + 8 u (50 per patch: waves 0-1 issue 7, the others 6)
    const int nd = (NP - wave + 7) / 8;
    auto patch_dma = [&](int t, int buf) {
        const int img = t / tiles_hw, rem = t - img * tiles_hw, th = rem / tiles_w;
        const int oh0 = th * TH, ow0 = (rem - th * tiles_w) * TW;
#pragma unroll
        for (int u = 0; u < 7; ++u) {
            const int d = wave + 8 * u, q = d * 8 + lrow;
            if (d >= NP) break;  // wave-uniform
            const int pr = q / PITCH, pc = q - pr * PITCH;
            const int hh = oh0 - 1 + pr, ww = ow0 - 1 + pc;
            unsigned off = POOB;
            if (t < ntiles && pc < PCW && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
                off = (unsigned)(((((long long)img * H + hh) * W + ww) * 64 + ((lch ^ lrow) << 3)) * 2);
            pdma16(rsX, off, lds0 + buf * PBYTES + d * 1024);
        }
    };
    // per-lane fragment address bases: pixel fragment j, tap column dx, half-step hs
    int rel[FN][3][2];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        const int p = wp * (TP / 4) + j * 16;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
            const int q = (p / TW) * PITCH + (p % TW) + r16 + dx;
#pragma unroll
            for (int hs = 0; hs < 2; ++hs) rel[j][dx][hs] = q * 128 + (((kq + 4 * hs) ^ (q & 7)) << 4);
        }
    }
    bf16_t* __restrict__ Y = (bf16_t*)a.y;
    const bool leaky = a.act == RR_ACT_LEAKY;
    const float slope = a.slope;
    const int nmine = (ntiles - 1 - (b >> 3) - (b & 7) * (G >> 3)) >= 0
                          ? (ntiles - 1 - (b & 7) * (G >> 3) - (b >> 3)) / G + 1 : 0;
    if (nmine == 0) return;
    // a wave issues the same nd pieces for every patch (past the last tile: zeros),
    // so its counted waits are fixed: nd for the next patch (+ NST stores)
    patch_dma(tile_id(0), 0);
    patch_dma(tile_id(1), 1);
    for (int i = 0; i < nmine; ++i) {
        // patch(i) landed: younger are patch(i + 1) and tile i - 1's stores
        if (nd == 7) {
            if (i == 0) pwait_barrier<7>();
            else pwait_barrier<7 + NST>();
        } else {
            if (i == 0) pwait_barrier<6>();
            else pwait_barrier<6 + NST>();
        }
        patch_dma(tile_id(i + 2), (i + 2) % NBUF);
        const char* Ps = smem + (i % NBUF) * PBYTES;
        const char* base[FN][3][2];
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
#pragma unroll
                for (int hs = 0; hs < 2; ++hs) {
                    int r = rel[j][dx][hs];
                    asm volatile("" : "+v"(r));  // per-tile opaque copy: bases stay 24 VGPRs
                    base[j][dx][hs] = Ps + r;
                }
        pf32x4_t acc[2][FN];
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[ii][j] = (pf32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 18; ++s) {
            const int tap = s >> 1, hs = s & 1, dy = tap / 3, dx = tap % 3;
            uint4 fb[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) fb[j] = *reinterpret_cast<const uint4*>(base[j][dx][hs] + dy * PITCH * 128);
#pragma unroll
            for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[ii][j] = H16<HT>::mfma(areg[ii][s], fb[j], acc[ii][j]);
        }
        const int t = tile_id(i);
        const int img = t / tiles_hw, rem = t - img * tiles_hw, th = rem / tiles_w;
        const int oh0 = th * TH, ow0 = (rem - th * tiles_w) * TW;
        const int c = 32 * wc + 8 * kq;
        const float4 s0 = *reinterpret_cast<const float4*>(sS + c), s1 = *reinterpret_cast<const float4*>(sS + c + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(sH + c), h1 = *reinterpret_cast<const float4*>(sH + c + 4);
        const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int p = wp * (TP / 4) + j * 16 + r16;
            const long long pix = ((long long)img * H + oh0 + p / TW) * W + ow0 + p % TW;
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[0][j][r] * sc[r] + sh[r];
                v[4 + r] = acc[1][j][r] * sc[4 + r] + sh[4 + r];
            }
            if (leaky) {
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * slope;
            }
            uint4 o;
            o.x = H16<HT>::pack2(v[0], v[1]);
            o.y = H16<HT>::pack2(v[2], v[3]);
            o.z = H16<HT>::pack2(v[4], v[5]);
            o.w = H16<HT>::pack2(v[6], v[7]);
            *reinterpret_cast<uint4*>(Y + pix * a.ldy + c) = o;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace
int g_conv3_pipe = 1;  // rr_set_tuning(RR_TUNE_CONV3_PIPE): 1 software-pipelined A-stationary tiles, 0 compiler schedule
namespace {

template <int TC, int TH, int TW, int WC, int WP, bool ARES, int NSA = 2>
void launch_c3(const ConvArgs& a, hipStream_t s, bool f16) {
    const int tiles_w = a.w_ / TW, tiles_h = a.h / TH, tiles_c = a.cout / TC;
    const long long ntl = (long long)a.n * tiles_h * tiles_w * tiles_c;
    const int cus = grid_cus();
    const int grid = (int)(ntl < cus ? ntl : cus);
    // the overlapped epilogue's branch-free activation needs slope in [0, 1]
    const int pipe = g_conv3_pipe && (a.act != RR_ACT_LEAKY || (a.slope >= 0.f && a.slope <= 1.f));
    if (f16)
        hipLaunchKernelGGL((k_conv3x3<TC, TH, TW, WC, WP, ARES, NSA, f16_t>), dim3(grid), dim3(64 * WC * WP), 0, s, a,
                           tiles_w, tiles_w * tiles_h, tiles_c, (int)ntl, pipe);
    else
        hipLaunchKernelGGL((k_conv3x3<TC, TH, TW, WC, WP, ARES, NSA, bf16_t>), dim3(grid), dim3(64 * WC * WP), 0, s, a,
                           tiles_w, tiles_w * tiles_h, tiles_c, (int)ntl, pipe);
}

}  // namespace

int g_c3w64 = 1;       // mod2 3x3 on k_c3w64 under RR_TUNE_CONV3X3 = 1 (9 forces it)
int g_conv3_mode = 1;  // rr_set_tuning(RR_TUNE_CONV3X3): 0 off, 1 auto, 2 / 3 prefer 8x32 / 4x32 tiles,
                       // 4 / 6 A-stationary with 1x8 / 1x4 waves (auto: 2x4), 7 3-stage weight ring,
                       // 8 256-channel x 6x32 tiles (auto where c_out % 256 == 0 and h % 6 == 0)

// bf16 3x3 / stride 1 / pad 1 with PERM32 weights, bf16 out, no residual, and
// image sizes the tiles divide; returns false otherwise (caller falls back to
// the implicit-GEMM engine).
bool gemm8_eligible(const ConvArgs& a, bool k1, int esz);  // rr_gemm.hip
bool launch_conv3s(const ConvArgs& a, hipStream_t s, bool f16);  // rr_conv3s.hip

bool launch_conv3x3(const ConvArgs& a, hipStream_t s, bool f16) {
    if (g_conv3_mode == 0) return false;
    // the staggered two-wave-group kernel (c_out = 128, or c_in = c_out = 64)
    if (g_conv3_mode == 1 && launch_conv3s(a, s, f16)) return true;
    if (a.kh != 3 || a.kw != 3 || a.stride != 1 || a.pad != 1 || a.dil != 1) return false;
    if (!(a.flags & RR_CONV_PERM32) || (a.flags & RR_CONV_RESIDUAL) || a.ldy != a.cout) return false;
    if (a.cin % 64 || a.kp != 9 * a.cin || a.w_ % 32) return false;
    if ((long long)a.n * a.h * a.w_ * a.cin * 2 >= (1ll << 31)) return false;
    if ((long long)a.n * a.h * a.w_ >= (1ll << 31) / 2) return false;
    // 256-multiple output channels on a chip-filling problem (mod4 / mod5 3x3 at
    // 128 images): the 8-phase GEMM on tap-uniform im2col beats the direct
    // kernel (420 vs 479, 392 vs 455 us) — the taps re-read from L2
    if (a.cout % 256 == 0 && g_conv3_mode == 1 && gemm8_eligible(a, false, 2)) return false;
    const int g_c3_cus = grid_cus();
    if (a.cin == 64 && a.cout == 64 && a.h % 8 == 0 && (g_conv3_mode == 9 || (g_conv3_mode == 1 && g_c3w64))) {
        const int tiles_w = a.w_ / 32, tiles_hw = tiles_w * (a.h / 8);
        const long long ntl = (long long)a.n * tiles_hw;
        int grid = (int)(ntl < g_c3_cus ? ntl : g_c3_cus) & ~7;
        if (grid < 8) grid = 8;
        if (f16) hipLaunchKernelGGL(k_c3w64<f16_t>, dim3(grid), dim3(512), 0, s, a, tiles_w, tiles_hw, (int)ntl);
        else hipLaunchKernelGGL(k_c3w64<bf16_t>, dim3(grid), dim3(512), 0, s, a, tiles_w, tiles_hw, (int)ntl);
        return true;
    }
    if (a.cin == 64 && a.cout == 64 && a.h % 8 == 0) {
        // 8 waves (2 per SIMD) measured fastest: 125 us vs 146 (4 waves) at 32 x 192x256x64
        if (g_conv3_mode == 4) launch_c3<64, 8, 32, 1, 8, true>(a, s, f16);
        else if (g_conv3_mode == 6) launch_c3<64, 8, 32, 1, 4, true>(a, s, f16);
        else launch_c3<64, 8, 32, 2, 4, true>(a, s, f16);
        return true;
    }
    if (a.cout % 128 == 0 && a.cout <= 512) {
        // 8 x 32 tiles when they still give every CU two or more tiles, else 4 x 32
        // (tuning modes 2 / 3 force one of them where the image height allows)
        const long long t8 = a.h % 8 == 0 ? (long long)a.n * (a.h / 8) * (a.w_ / 32) * (a.cout / 128) : 0;
        const bool want8 = g_conv3_mode == 2 || (g_conv3_mode != 3 && t8 >= 2 * g_c3_cus);
        // 256-channel tiles x 6 x 32 pixels (half the patch re-reads across channel
        // tiles, 48 MFMAs per wave between barriers) for c_out % 256 == 0
        // (measured at 128 x R50: mod4 c2 505 -> 461 us, mod5 c2 472 -> 416 us; default where it applies)
        if ((g_conv3_mode == 1 || g_conv3_mode == 8) && a.cout % 256 == 0 && a.h % 6 == 0) {
            launch_c3<256, 6, 32, 4, 2, false>(a, s, f16);
            return true;
        }
        const bool deep = g_conv3_mode == 7;  // 3-stage weight ring
        if (t8 > 0 && (want8 || a.h % 4 != 0)) {
            if (deep) launch_c3<128, 8, 32, 2, 4, false, 3>(a, s, f16);
            else launch_c3<128, 8, 32, 2, 4, false>(a, s, f16);
            return true;
        }
        if (a.h % 4 == 0) {
            if (deep) launch_c3<128, 4, 32, 2, 4, false, 3>(a, s, f16);
            else launch_c3<128, 4, 32, 2, 4, false>(a, s, f16);
            return true;
        }
    }
    return false;
}

}  // namespace rr
