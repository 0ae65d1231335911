// librr.so — one whole ResNet bottleneck block of the 256-channel stage (mod2) in one launch:
//   t2 = act(bn2(conv3x3(t1)))                         3x3, 64 -> 64, stride 1   (MFMA-bound)
//   y  = act(bn3(conv1x1(t2)) + shortcut)              64 -> 256                 (HBM-bound)
//   z  = act(bn1'(conv1x1(y)))                         256 -> C1, next block's conv1
// i.e. conv2 .. conv3 + residual of ResidualBlock i and conv1 of block i + 1
// (cirtorch/backbones/misc.py:163-203), where the unfused chain runs k_c3w64 (the 3x3, ~0.5 ms
// per 128 images, MFMA-bound) and then k_stream_pair (conv3 + conv1, ~1.6 ms, HBM-bound) — the
// matrix work of the first sits beside nothing, the second waits on HBM.  Here the two run at
// the same time on every CU, split by wave role, so the 3x3 hides under the boundary's HBM
// time and t2 never touches HBM (-256 B per pixel):
//   * waves 0-3 ("3x3 role") are k_c3w64's waves on a 4 x 32-pixel tile: each keeps 32 output
//     channels x all 576 K of the PERM32 weights in VGPRs (2 channel halves x 2 pixel halves),
//     the t1 halo patch (6 x 34 pixels, 40-slot pitch, chunk ^ (slot & 7)) arrives by LDS-DMA,
//     and the (tap, half-step) MFMA order is k_c3w64's: t2 is bit-identical to it;
//   * waves 4-7 ("pair role") are k_stream_pair's waves: W3 / W1 (/ Wp) in LDS, one 16-pixel
//     strip per phase, the strip's t2 read from an LDS tile instead of HBM, the residual (or
//     the projection's input) prefetched two phases ahead into registers, issue priority 1;
//     same MFMA order, so y and z are bit-identical to the unfused launches;
//   * two phases per tile, both roles meet at 2 barriers per tile: in phase A the pair role
//     runs strips 0-3 of tile s while the 3x3 role computes tile s + 1 (its lower pixel half
//     having first stored tile s's strips 4-7); in phase B the pair role runs strips 4-7 and
//     the 3x3 role stores tile s + 1's strips 0-3 and loads the patch of tile s + 2 — one
//     patch buffer and one t2 tile suffice (LDS <= 150 KB with the projection or C1 = 128).
// Persistent, one 512-thread block per CU; XCD x's blocks take tiles of the XCD's contiguous
// range from a per-XCD atomic counter (or, with no counter array, a static walk).  Optional
// (CONV1, the stage's first block): the block's own conv1 (1x1 64 -> 64) applied to the patch
// in LDS, so the launch reads the block input instead of t1.
#include "rr_internal.h"

#ifndef C3P_IG2
#define C3P_IG2 1
#endif

namespace rr {

namespace {

typedef __attribute__((ext_vector_type(4))) float cf32x4_t;
typedef __attribute__((ext_vector_type(4))) int ci32x4_t;

constexpr unsigned COOB = 0x80000000u;  // voffset beyond every buffer: the DMA writes zeros

__device__ __forceinline__ void cdma16(ci32x4_t rsrc, unsigned voff, unsigned lds_addr) {
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

__device__ __forceinline__ ci32x4_t crsrc(const void* base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)base;
    ci32x4_t r;
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

// t2 reaches the LDS by ds_write (not DMA): its writes must be done before the barrier
__device__ __forceinline__ void cbar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// k_stream_pair's weight image swizzle (every ds_read_b128 lane group of an A fragment hits
// 16 distinct 4-bank groups)
template <int K>
__device__ __forceinline__ int cwswz(int row, int chunk) {
    const int f = K == 64 ? ((row >> 1) & 7) : (row & 15);
    return row * (K * 2) + ((chunk ^ f) << 4);
}

__device__ __forceinline__ void cpin(uint4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }

}  // namespace

struct C3PairArgs {
    const bf16_t* t1;          // [n][h][w][64]: conv1 output of block i (CONV1: the block input)
    const bf16_t* w0;          // CONV1: conv1 of block i, [64][64] PERM32 rows
    const float *s0, *h0;      // CONV1: folded bn1
    const bf16_t* w33;         // [64][576] PERM32 rows, k = tap * 64 + ci
    const float *s33, *h33;    // folded bn2
    const bf16_t* w3;          // [256][64] PERM32 rows
    const float *s3, *h3;
    const bf16_t* res;         // [P][256] shortcut (!PROJ)
    const bf16_t* xp;          // [P][64] block input (PROJ: shortcut = proj_bn(proj_conv(xp)))
    const bf16_t* wp;          // [256][64] PERM32 rows
    const float *sp, *hp;
    const bf16_t* w1;          // [C1][256] PERM32 rows (conv1 of block i + 1)
    const float *s1, *h1;
    bf16_t* y;                 // [P][256]
    bf16_t* z;                 // [P][C1]
    int* queue;                // 8 zeroed per-XCD tile counters (dynamic walk) or NULL (static)
    int n, h, w;
    int act2, act3, act1, act0;
    float slope2, slope3, slope1, slope0;
};

namespace {

// CONV1 (the stage's first block, PROJ): the patch DMA brings the block input x, and the 3x3
// role turns it into t1 = act0(W0 x s0 + h0) in place (k_stream1x1's K order and rounding;
// slots outside the image back to the 3x3's zero padding) before its 3x3 — one more barrier
// per tile, and conv1's own launch (x read, t1 written and re-read) is gone.
template <int C1, bool PROJ, typename HT, bool CONV1 = false>
__global__ void __launch_bounds__(512, 1) k_c3pair(C3PairArgs a, int tiles_w, int tiles_hw, int ntiles) {
    static_assert(!CONV1 || PROJ, "conv1 in the launch: the stage's first block only");
    constexpr int TH = 4, TW = 32, TP = TH * TW, PITCH = 40;     // 4 x 32 tile; patch rows 40 slots apart
    constexpr int NSLOT = (TH + 2) * PITCH, NP = NSLOT / 8;      // 240 slots, 30 pieces of 8 slots (1 KiB)
    constexpr int PCW = TW + 2;                                  // 34 patch columns used
    constexpr int FN = 4;                                        // 3x3 wave: 4 pixel fragments (64 px)
    constexpr int K3 = 64, C3 = 256, NK3 = K3 / 32, NR3 = C3 / 32, NF1 = C1 / 16, NK1 = C3 / 32;
    static_assert(NSLOT % 8 == 0 && PITCH % 8 == 0, "row-invariant patch swizzle");
    __shared__ __attribute__((aligned(1024))) char sPatch[NSLOT * 128];
    __shared__ __attribute__((aligned(16))) char sT2[TP * 128];
    __shared__ __attribute__((aligned(16))) char sW3[C3 * K3 * 2];
    __shared__ __attribute__((aligned(16))) char sW1[C1 * C3 * 2];
    __shared__ __attribute__((aligned(16))) char sWp[PROJ ? C3 * K3 * 2 : 16];
    __shared__ __attribute__((aligned(16))) float sS3[C3], sH3[C3], sS1[C1], sH1[C1], sS2[64], sH2[64];
    __shared__ __attribute__((aligned(16))) float sSp[PROJ ? C3 : 4], sHp[PROJ ? C3 : 4];
    __shared__ __attribute__((aligned(16))) char sW0[CONV1 ? 64 * 64 * 2 : 16];
    __shared__ __attribute__((aligned(16))) float sS0[CONV1 ? 64 : 4], sH0[CONV1 ? 64 : 4];
    __shared__ int sTile[4];  // tile of step s in slot s & 3 (-1: none), fetched three steps ahead

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool role3 = wave < 4;                  // 3x3 role (waves 0-3) / pair role (4-7)
    const int r16 = lane & 15, kq = lane >> 4, lrow = lane >> 3, lch = lane & 7;
    const int H = a.h, W = a.w;

    // ---- LDS weights and affines (all waves), 3x3 weights to the VGPRs of the 3x3 role
    for (int i = tid; i < C3 * K3 / 8; i += 512) {
        const int r = i / (K3 / 8), c = i - r * (K3 / 8);
        *reinterpret_cast<uint4*>(sW3 + cwswz<K3>(r, c)) = reinterpret_cast<const uint4*>(a.w3)[i];
        if constexpr (PROJ) *reinterpret_cast<uint4*>(sWp + cwswz<K3>(r, c)) = reinterpret_cast<const uint4*>(a.wp)[i];
    }
    for (int i = tid; i < C1 * C3 / 8; i += 512) {
        const int r = i / (C3 / 8), c = i - r * (C3 / 8);
        *reinterpret_cast<uint4*>(sW1 + cwswz<C3>(r, c)) = reinterpret_cast<const uint4*>(a.w1)[i];
    }
    for (int i = tid; i < C3; i += 512) {
        sS3[i] = a.s3[i];
        sH3[i] = a.h3[i];
        if constexpr (PROJ) {
            sSp[i] = a.sp[i];
            sHp[i] = a.hp[i];
        }
    }
    for (int i = tid; i < C1; i += 512) {
        sS1[i] = a.s1[i];
        sH1[i] = a.h1[i];
    }
    if (tid < 64) {
        sS2[tid] = a.s33[tid];
        sH2[tid] = a.h33[tid];
        if constexpr (CONV1) {
            sS0[tid] = a.s0[tid];
            sH0[tid] = a.h0[tid];
        }
    }
    if constexpr (CONV1)
        for (int i = tid; i < 64 * 64 / 8; i += 512) {
            const int r = i / 8, c = i - r * 8;
            *reinterpret_cast<uint4*>(sW0 + cwswz<64>(r, c)) = reinterpret_cast<const uint4*>(a.w0)[i];
        }
    const int wc = wave & 1, wpx = (wave >> 1) & 1;  // 3x3 role: channel half, pixel half

    // ---- this block's tiles.  Static: k_c3w64's XCD-contiguous walk.  Dynamic (a.queue):
    // XCD x = blockIdx & 7 owns the contiguous tile range [s_x, s_x + n_x) and its blocks take
    // the next tile from the XCD's counter, so a block that starts late (its CU still held by
    // another stream's kernel) takes fewer tiles instead of finishing its fixed share late.
    // Thread 0 fetches step s's tile during step s - 3 into sTile (both roles read it after
    // the barriers that follow).
    const int b = (int)blockIdx.x, G = (int)gridDim.x, xcd = b & 7;
    const int nt8 = ntiles >> 3, rt8 = ntiles & 7;
    const int s_x = xcd < rt8 ? xcd * (nt8 + 1) : rt8 * (nt8 + 1) + (xcd - rt8) * nt8;
    const int n_x = nt8 + (xcd < rt8 ? 1 : 0);
    auto fetch_tile = [&](int i) __attribute__((always_inline)) {
        if (a.queue) {
            const int v = atomicAdd(a.queue + xcd, 1);
            return v < n_x ? s_x + v : -1;
        }
        const int t = i * G + xcd * (G >> 3) + (b >> 3);
        return t < ntiles ? t : -1;
    };
    if (tid == 0) {
        sTile[0] = fetch_tile(0);
        sTile[1] = fetch_tile(1);
        sTile[2] = fetch_tile(2);
    }
    __syncthreads();
    auto tile_id = [&](int i) __attribute__((always_inline)) { return sTile[i & 3]; };
    if (tile_id(0) < 0) return;  // block-uniform
    auto tile_org = [&](int t, int& img, int& oh0, int& ow0) __attribute__((always_inline)) {
        img = t / tiles_hw;
        const int rem = t - img * tiles_hw, th = rem / tiles_w;
        oh0 = th * TH;
        ow0 = (rem - th * tiles_w) * TW;
    };

    // ================================================================= 3x3 role state
    const ci32x4_t rsX = crsrc(a.t1, (unsigned)((long long)a.n * H * W * 64 * 2));
    const unsigned ldsP = (unsigned)(unsigned long long)sPatch;
    // patch pieces d = wave + 4 u (30 per patch: waves 0-1 issue 8, waves 2-3 issue 7)
    auto patch_dma = [&](int t, bool live) __attribute__((always_inline)) {
        int img = 0, oh0 = 0, ow0 = 0;
        if (live) tile_org(t, img, oh0, ow0);
        // the pieces' per-lane slot values derived per call from an opaque copy of the lane's
        // row: hoisted out of the tile walk they were spilled, and each reload's vmcnt(0)
        // serialised the DMA pieces behind it
        int lr = lrow;
        asm volatile("" : "+v"(lr));
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int d = wave + 4 * u, q = d * 8 + lr;
            if (d >= NP) break;  // wave-uniform
            const int pr = q / PITCH, pc = q - pr * PITCH;
            const int hh = oh0 - 1 + pr, ww = ow0 - 1 + pc;
            unsigned off = COOB;
            if (live && pc < PCW && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
                off = (unsigned)(((((long long)img * H + hh) * W + ww) * 64 + ((lch ^ lr) << 3)) * 2);
            cdma16(rsX, off, ldsP + d * 1024);
        }
    };
    h16_f32x4_t acc[2][FN];
    // the tile's 3x3 (k_c3w64's K-step loop: 18 x (4 fragment reads, 8 MFMAs))
    auto conv3x3 = [&](const uint4 (&areg)[2][18]) __attribute__((always_inline)) {
        // fragment address bases (pixel fragment j, tap column dx, half-step hs), derived per
        // tile from an opaque copy of the lane's column: live only across this loop (24 VGPRs),
        // not across the whole tile walk beside the 144 weight VGPRs
        int lc;  // the lane's column, recomputed per tile (not a register live across the walk)
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lc));
        lc &= 15;
        const char* base[FN][3][2];
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
#pragma unroll
                for (int hs = 0; hs < 2; ++hs) {
                    const int q = (wpx * 2 + (j >> 1)) * PITCH + (j & 1) * 16 + lc + dx;  // tile pixel wpx*64 + j*16
                    base[j][dx][hs] = sPatch + q * 128 + (((kq + 4 * hs) ^ (q & 7)) << 4);
                }
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[ii][j] = (h16_f32x4_t){0.f, 0.f, 0.f, 0.f};
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
    };
    // CONV1: the patch (block input x) -> t1 in place, one 16-slot fragment per step, fragments
    // wave, wave + 4, ... (15 per patch): t1 = act0(W0 x s0 + h0) with k_stream1x1's MFMA order
    // (K-steps 0, 1; channel pairs 32 i2 + 8 kq) and rounding; slots outside the image (and
    // the unused pitch columns) get 0, the 3x3's zero padding
    auto convert_patch = [&](int t) __attribute__((always_inline)) {
        if constexpr (CONV1) {
            int img, oh0, ow0;
            tile_org(t, img, oh0, ow0);
            const bool leaky0 = a.act0 == RR_ACT_LEAKY;
            for (int f = wave; f < NP * 8 / 16; f += 4) {
                int q = f * 16 + r16;
                asm volatile("" : "+v"(q));
                const int pr = q / PITCH, pc = q - pr * PITCH;
                const int hh = oh0 - 1 + pr, ww = ow0 - 1 + pc;
                const bool valid = pc < PCW && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
                char* slot = sPatch + q * 128;
                uint4 bx[2];
#pragma unroll
                for (int kk = 0; kk < 2; ++kk)
                    bx[kk] = *reinterpret_cast<const uint4*>(slot + (((4 * kk + kq) ^ (q & 7)) << 4));
                h16_f32x4_t c0[4];
#pragma unroll
                for (int ii = 0; ii < 4; ++ii) c0[ii] = (h16_f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                    for (int ii = 0; ii < 4; ++ii) {
                        const uint4 av = *reinterpret_cast<const uint4*>(sW0 + cwswz<64>(ii * 16 + r16, kk * 4 + kq));
                        c0[ii] = H16<HT>::mfma(av, bx[kk], c0[ii]);
                    }
#pragma unroll
                for (int i2 = 0; i2 < 2; ++i2) {
                    const int c = 32 * i2 + 8 * kq;
                    float v[8];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] = c0[2 * i2][r] * sS0[c + r] + sH0[c + r];
                        v[4 + r] = c0[2 * i2 + 1][r] * sS0[c + 4 + r] + sH0[c + 4 + r];
                    }
                    if (leaky0) {
#pragma unroll
                        for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope0;
                    }
                    uint4 o = make_uint4(0u, 0u, 0u, 0u);
                    if (valid) {
                        o.x = H16<HT>::pack2(v[0], v[1]);
                        o.y = H16<HT>::pack2(v[2], v[3]);
                        o.z = H16<HT>::pack2(v[4], v[5]);
                        o.w = H16<HT>::pack2(v[6], v[7]);
                    }
                    *reinterpret_cast<uint4*>(slot + (((4 * i2 + kq) ^ (q & 7)) << 4)) = o;
                }
            }
        }
    };
    // bn2 + act, 8 consecutive channels per lane -> the t2 tile (16-B chunk ^ (pixel & 7))
    auto store_t2 = [&]() __attribute__((always_inline)) {
        const int c = 32 * wc + 8 * kq;
        float sc[8], sh[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            sc[r] = sS2[c + r];
            sh[r] = sH2[c + r];
        }
        const bool leaky2 = a.act2 == RR_ACT_LEAKY;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int p = wpx * (TP / 2) + j * 16 + r16;  // tile-local pixel
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[0][j][r] * sc[r] + sh[r];
                v[4 + r] = acc[1][j][r] * sc[4 + r] + sh[4 + r];
            }
            if (leaky2) {
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope2;
            }
            uint4 o;
            o.x = H16<HT>::pack2(v[0], v[1]);
            o.y = H16<HT>::pack2(v[2], v[3]);
            o.z = H16<HT>::pack2(v[4], v[5]);
            o.w = H16<HT>::pack2(v[6], v[7]);
            *reinterpret_cast<uint4*>(sT2 + p * 128 + (((4 * wc + kq) ^ (p & 7)) << 4)) = o;
        }
    };

    // ================================================================= pair role state
    const int pw = wave - 4;
    const bool leaky3 = a.act3 == RR_ACT_LEAKY, leaky1 = a.act1 == RR_ACT_LEAKY;
    constexpr int NRQ = PROJ ? NK3 : NR3;  // shortcut (or projection input) fragments of a strip
    auto strip_pixel = [&](int t, int k) __attribute__((always_inline)) {  // global pixel of lane r16 in local strip k of tile t
        int img, oh0, ow0;
        tile_org(t, img, oh0, ow0);
        return ((long long)img * H + oh0 + (k >> 1)) * W + ow0 + (k & 1) * 16 + r16;
    };
    auto load_rq = [&](uint4 (&dst)[NRQ], long long p) __attribute__((always_inline)) {
        if constexpr (PROJ) {
            const bf16_t* ps = a.xp + p * K3 + 8 * kq;
#pragma unroll
            for (int kk = 0; kk < NK3; ++kk) dst[kk] = ld16_once(ps + kk * 32);
        } else {
            const bf16_t* rs = a.res + p * C3 + 8 * kq;
#pragma unroll
            for (int i2 = 0; i2 < NR3; ++i2) dst[i2] = ld16_once(rs + 32 * i2);
        }
    };
    // one 16-pixel strip: y = act3(W3 t2 s3 + h3 + shortcut) -> HBM, z = act1(W1 y s1 + h1) -> HBM
    // (k_stream_pair's strip body, t2 from the LDS tile)
    auto pair_strip = [&](int k, long long p, const uint4 (&rv)[NRQ]) __attribute__((always_inline)) {
        uint4 bq[NK3];
        {
            const int q = k * 16 + r16;
#pragma unroll
            for (int kk = 0; kk < NK3; ++kk)
                bq[kk] = *reinterpret_cast<const uint4*>(sT2 + q * 128 + (((4 * kk + kq) ^ (q & 7)) << 4));
        }
        uint4 yq[NR3];
        // IG 32-channel groups per step: four independent W3 (and Wp) accumulator chains in
        // flight instead of two (measured -2 % projection form, -1 % residual forms)
        constexpr int IG = C3P_IG2 ? 2 : 1;
#pragma unroll
        for (int i0 = 0; i0 < NR3; i0 += IG) {
            int abase = 0;
            asm volatile("" : "+v"(abase));  // keep the weight fragments in LDS (no hoisting into VGPRs)
            h16_f32x4_t acc3[IG][2], pacc[IG][2];
#pragma unroll
            for (int g = 0; g < IG; ++g)
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) acc3[g][hh] = pacc[g][hh] = (h16_f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < NK3; ++kk)
#pragma unroll
                for (int g = 0; g < IG; ++g)
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh) {
                        const uint4 av = *reinterpret_cast<const uint4*>(sW3 + abase + cwswz<K3>((2 * (i0 + g) + hh) * 16 + r16, kk * 4 + kq));
                        acc3[g][hh] = H16<HT>::mfma(av, bq[kk], acc3[g][hh]);
                    }
            if constexpr (PROJ) {  // shortcut = proj_bn(proj_conv(x_in)), kept in f32
#pragma unroll
                for (int kk = 0; kk < NK3; ++kk)
#pragma unroll
                    for (int g = 0; g < IG; ++g)
#pragma unroll
                        for (int hh = 0; hh < 2; ++hh) {
                            const uint4 av = *reinterpret_cast<const uint4*>(sWp + abase + cwswz<K3>((2 * (i0 + g) + hh) * 16 + r16, kk * 4 + kq));
                            pacc[g][hh] = H16<HT>::mfma(av, rv[kk], pacc[g][hh]);
                        }
            }
#pragma unroll
            for (int g = 0; g < IG; ++g) {
                const int i2 = i0 + g;
                const int c = 32 * i2 + 8 * kq;
                float v[8];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc3[g][0][r] * sS3[c + r] + sH3[c + r];
                    v[4 + r] = acc3[g][1][r] * sS3[c + 4 + r] + sH3[c + 4 + r];
                }
                if constexpr (PROJ) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] += pacc[g][0][r] * sSp[c + r] + sHp[c + r];
                        v[4 + r] += pacc[g][1][r] * sSp[c + 4 + r] + sHp[c + 4 + r];
                    }
                } else {
                    const uint4 qv = rv[i2];
                    const unsigned w4[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[2 * r] += H16<HT>::lo(w4[r]);
                        v[2 * r + 1] += H16<HT>::hi(w4[r]);
                    }
                }
                if (leaky3) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope3;
                }
                yq[i2].x = H16<HT>::pack2(v[0], v[1]);
                yq[i2].y = H16<HT>::pack2(v[2], v[3]);
                yq[i2].z = H16<HT>::pack2(v[4], v[5]);
                yq[i2].w = H16<HT>::pack2(v[6], v[7]);
                st16_once(a.y + p * C3 + c, yq[i2]);
            }
        }
        h16_f32x4_t zacc[NF1];
#pragma unroll
        for (int o = 0; o < NF1; ++o) zacc[o] = (h16_f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < NK1; ++kk) {
            int abase = 0;
            asm volatile("" : "+v"(abase));
#pragma unroll
            for (int o = 0; o < NF1; ++o) {
                const uint4 av = *reinterpret_cast<const uint4*>(sW1 + abase + cwswz<C3>(o * 16 + r16, kk * 4 + kq));
                zacc[o] = H16<HT>::mfma(av, yq[kk], zacc[o]);
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
            o.x = H16<HT>::pack2(v[0], v[1]);
            o.y = H16<HT>::pack2(v[2], v[3]);
            o.z = H16<HT>::pack2(v[4], v[5]);
            o.w = H16<HT>::pack2(v[6], v[7]);
            st16_once(a.z + p * C1 + c, o);
        }
    };

    // ================================================================= the two roles
    // Each role runs its own loop (so the registers of one are dead in the other: the 3x3
    // role's 144 weight VGPRs never sit beside the pair role's shortcut prefetch), both
    // meeting at the same barriers: 3 in the prologue, 2 per tile.
    if (role3) {
        uint4 areg[2][18];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int ks = 0; ks < 18; ++ks)
                areg[i][ks] = *reinterpret_cast<const uint4*>(a.w33 + (long long)(32 * wc + 16 * i + r16) * 576 +
                                                              (ks >> 1) * 64 + 32 * (ks & 1) + 8 * kq);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int ks = 0; ks < 18; ++ks) cpin(areg[i][ks]);
        auto conv = [&]() __attribute__((always_inline)) { conv3x3(areg); };
        // prologue: tile 0's 3x3 (strips 0-3 stored now, 4-7 at the start of step 0), tile 1's patch
        patch_dma(tile_id(0), true);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        cbar();
        if constexpr (CONV1) {
            convert_patch(tile_id(0));
            cbar();
        }
        conv();
        if (wpx == 0) store_t2();
        cbar();  // every 3x3 wave is done with patch 0
        patch_dma(tile_id(1), tile_id(1) >= 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        cbar();
        for (int s = 0; tile_id(s) >= 0; ++s) {
            const bool more = tile_id(s + 1) >= 0;
            // phase A: tile s's strips 4-7 (lower pixel half), then tile s + 1's 3x3
            if (wpx == 1) store_t2();
            if constexpr (CONV1) {
                if (more) convert_patch(tile_id(s + 1));
                cbar();
            }
            if (more) conv();
            cbar();
            // phase B: tile s + 1's strips 0-3 (upper pixel half), tile s + 2's patch
            if (more) {
                if (wpx == 0) store_t2();
                const int t2i = tile_id(s + 2);
                patch_dma(t2i, t2i >= 0);
                // step s + 3's tile into the slot step s - 1 used (read by no one after step s - 1)
                if (tid == 0) sTile[(s + 3) & 3] = t2i >= 0 ? fetch_tile(s + 3) : -1;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            cbar();
        }
    } else {
        // the HBM stream issues ahead of the 3x3 role's MFMA run on the same SIMD
        // (measured: setprio 1 -2 % per block vs none; 2 the same as 1)
        __builtin_amdgcn_s_setprio(1);
        // shortcut fragments two phases ahead (4 buffers: phases A / B of two tiles), so a
        // pair wave keeps ~16 KiB of loads in flight across the barriers
        uint4 rq[4][NRQ];
        load_rq(rq[0], strip_pixel(tile_id(0), pw));
        load_rq(rq[1], strip_pixel(tile_id(0), 4 + pw));
        cbar();
        if constexpr (CONV1) cbar();  // the 3x3 role's conv1 of patch 0
        cbar();
        cbar();
        for (int s = 0; tile_id(s) >= 0; s += 2) {
            {  // tile s from buffers 0 / 1, tile s + 1's into 2 / 3
                const int t = tile_id(s);
                const bool n1 = tile_id(s + 1) >= 0;
                if (n1) load_rq(rq[2], strip_pixel(tile_id(s + 1), pw));
                if constexpr (CONV1) cbar();  // the 3x3 role's conv1 of the next patch
                pair_strip(pw, strip_pixel(t, pw), rq[0]);
                cbar();
                if (n1) load_rq(rq[3], strip_pixel(tile_id(s + 1), 4 + pw));
                pair_strip(4 + pw, strip_pixel(t, 4 + pw), rq[1]);
                cbar();
            }
            if (tile_id(s + 1) >= 0) {  // tile s + 1 from buffers 2 / 3, tile s + 2's into 0 / 1
                const int t = tile_id(s + 1);
                const bool n2 = tile_id(s + 2) >= 0;
                if (n2) load_rq(rq[0], strip_pixel(tile_id(s + 2), pw));
                if constexpr (CONV1) cbar();
                pair_strip(pw, strip_pixel(t, pw), rq[2]);
                cbar();
                if (n2) load_rq(rq[1], strip_pixel(tile_id(s + 2), 4 + pw));
                pair_strip(4 + pw, strip_pixel(t, 4 + pw), rq[3]);
                cbar();
            }
        }
    }
}

}  // namespace

}  // namespace rr

using namespace rr;

extern "C" int rr_conv3x3_pair(const void* t1, int n, int h, int w, const void* w0, const float* scale0,
                               const float* shift0, int act0, float slope0, const void* w33, const float* scale2,
                               const float* shift2, int act2, float slope2, const void* w3, const float* scale3,
                               const float* shift3, const void* residual, const void* xp, const void* wp,
                               const float* scalep, const float* shiftp, int act3, float slope3, const void* w1,
                               const float* scale1, const float* shift1, int c_out, int act1, float slope1, void* y,
                               void* z, int* tile_queue, int dtype, void* stream) {
    if (dtype != RR_BF16 && dtype != RR_F16) return fail(RR_EINVAL, "rr_conv3x3_pair: dtype (bf16 / fp16)");
    if (!t1 || !w33 || !scale2 || !shift2 || !w3 || !scale3 || !shift3 || !w1 || !scale1 || !shift1 || !y || !z)
        return fail(RR_EINVAL, "rr_conv3x3_pair: null pointer");
    const bool proj = residual == nullptr;
    if (proj && (!xp || !wp || !scalep || !shiftp))
        return fail(RR_EINVAL, "rr_conv3x3_pair: either residual or the projection (xp, wp, scalep, shiftp)");
    if (c_out != 64 && c_out != 128) return fail(RR_EINVAL, "rr_conv3x3_pair: c_out 64 or 128");
    if (proj && c_out != 64) return fail(RR_EINVAL, "rr_conv3x3_pair: the projection form takes c_out = 64");
    const bool conv1 = w0 != nullptr;
    if (conv1 && (!proj || !scale0 || !shift0 || ((uintptr_t)w0 & 15)))
        return fail(RR_EINVAL, "rr_conv3x3_pair: conv1 in the launch (w0) needs the projection form, scale0, shift0");
    if (conv1 && act0 != RR_ACT_IDENTITY && act0 != RR_ACT_LEAKY) return fail(RR_EINVAL, "rr_conv3x3_pair: act0");
    if (n <= 0 || h <= 0 || w <= 0 || h % 4 || w % 32) return fail(RR_EINVAL, "rr_conv3x3_pair: h % 4, w % 32");
    if ((long long)n * h * w * 64 * 2 >= (1ll << 31)) return fail(RR_EINVAL, "rr_conv3x3_pair: t1 over 2 GiB (split the batch)");
    for (const void* p : {t1, w33, w3, residual, xp, wp, w1, (const void*)y, (const void*)z})
        if ((uintptr_t)p & 15) return fail(RR_EINVAL, "rr_conv3x3_pair: 16-byte alignment required");
    if ((uintptr_t)tile_queue & 3) return fail(RR_EINVAL, "rr_conv3x3_pair: tile_queue alignment");
    for (int act : {act2, act3, act1})
        if (act != RR_ACT_IDENTITY && act != RR_ACT_LEAKY) return fail(RR_EINVAL, "rr_conv3x3_pair: activation");
    C3PairArgs a;
    a.t1 = (const bf16_t*)t1; a.w33 = (const bf16_t*)w33; a.s33 = scale2; a.h33 = shift2;
    a.w3 = (const bf16_t*)w3; a.s3 = scale3; a.h3 = shift3; a.res = (const bf16_t*)residual;
    a.xp = (const bf16_t*)xp; a.wp = (const bf16_t*)wp; a.sp = scalep; a.hp = shiftp;
    a.w1 = (const bf16_t*)w1; a.s1 = scale1; a.h1 = shift1; a.y = (bf16_t*)y; a.z = (bf16_t*)z;
    a.n = n; a.h = h; a.w = w; a.act2 = act2; a.act3 = act3; a.act1 = act1;
    a.slope2 = slope2; a.slope3 = slope3; a.slope1 = slope1; a.queue = tile_queue;
    a.w0 = (const bf16_t*)w0; a.s0 = scale0; a.h0 = shift0; a.act0 = act0; a.slope0 = slope0;
    const int tiles_w = w / 32, tiles_hw = (h / 4) * tiles_w;
    const long long ntl = (long long)n * tiles_hw;
    if (ntl >= (1ll << 31)) return fail(RR_EINVAL, "rr_conv3x3_pair: too many tiles");
    const int cus = grid_cus();
    int grid = (int)(ntl < cus ? ntl : cus) & ~7;
    if (grid < 8) grid = 8;
    const dim3 g((unsigned)grid), b(512);
    hipStream_t s = as_stream(stream);
    auto go = [&](auto hv) {
        using H = decltype(hv);
        if (conv1) hipLaunchKernelGGL((k_c3pair<64, true, H, true>), g, b, 0, s, a, tiles_w, tiles_hw, (int)ntl);
        else if (proj) hipLaunchKernelGGL((k_c3pair<64, true, H>), g, b, 0, s, a, tiles_w, tiles_hw, (int)ntl);
        else if (c_out == 64) hipLaunchKernelGGL((k_c3pair<64, false, H>), g, b, 0, s, a, tiles_w, tiles_hw, (int)ntl);
        else hipLaunchKernelGGL((k_c3pair<128, false, H>), g, b, 0, s, a, tiles_w, tiles_hw, (int)ntl);
    };
    if (dtype == RR_F16) go(f16_t{});
    else go(bf16_t{});
    return check_launch("rr_conv3x3_pair");
}
