// librr.so — direct 3x3 convolution (stride 1, pad 1, 16-bit) on the
// staggered two-wave-group schedule of k_gemm8 (rr_gemm.hip).
//
// k_conv3x3 (rr_conv3.hip) stages the input halo patch once in LDS and reads
// the 9 taps by address offset, but every wave of a block reaches the same
// barrier, reads its fragments and then issues its MFMAs in lock step: the
// LDS reads of all 8 waves sit in front of the matrix pipe (MFMA busy 0.37 on
// the mod3 3x3, 0.47 on mod2).  Here a block is persistent over a contiguous
// range of output tiles of one XCD and runs the k_gemm8 phase structure:
//   * phase = every wave does one 64-channel x 32-pixel x 64-deep sub-block
//     (16 v_mfma_f32_16x16x32) between two s_barriers; two phases per K-step
//     (the two pixel halves of the tile), the A (weight) fragments read once
//     per K-step and kept in registers for the second phase: 16 KiB of LDS
//     reads per 32 MFMAs per wave (half the CU's LDS rate at full MFMA rate);
//   * waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave
//     reads LDS / issues DMA while its partner runs its MFMA cluster;
//   * operands arrive by LDS-DMA (buffer_load ... lds) tracked by counted
//     vmcnt, each LDS region overwritten no earlier than two phases after its
//     last read (the rule that keeps the lagging group's reads safe).
// Two variants (mod3 / mod2 of R50; measured 442-454 vs 532 us and 533-554 vs
// 525 us at 128 images, so only the first is on by default):
//   k_c3s_w128  c_out = 128, c_in = 64 * nck (mod3: 128): 8 x 32 output tile;
//               per 64-channel input chunk a (8+2) x (32+2) halo patch
//               (128 B per pixel) double-buffered by chunk — the next chunk
//               (or the next tile's first) arrives one 1-KiB piece per phase
//               while the current one is read; 128-row weight K-steps through
//               a 3-stage ring (tap-major inside a chunk, k = tap * c_in + ci);
//   k_c3s_w64   c_in = c_out = 64 (mod2): 16 x 32 output tile, the 64 input
//               channels split into two 32-channel chunks of 64 B per pixel
//               (additive 16-B chunk swizzle (c + 2 * ((q >> 2) & 1)) & 3 keeps
//               every ds_read_b128 lane group on distinct banks), all 18
//               32-deep weight K-steps resident in LDS, a K-step pair per phase.
// Epilogue: folded BN scale / shift (kept in VGPRs) + leaky / identity, one
// 16-B store per PERM32 fragment pair; the stores of tile t stay in flight
// across the first phases of tile t + 1 (counted waits).
//
// Replaces the stride-1 3x3 nn.Conv2d of ResidualBlock (cirtorch/backbones/
// misc.py:166-172) + the ABN eval BN + leaky_relu (cirtorch/utils/misc.py:175-235).
#include "rr_internal.h"

namespace rr {

namespace {

typedef __attribute__((ext_vector_type(4))) float sf32x4_t;
typedef __attribute__((ext_vector_type(4))) int si32x4_t;

constexpr unsigned SOOB = 0x80000000u;  // voffset beyond every buffer: the DMA writes zeros

// One 16-B-per-lane LDS-DMA wave-instruction: LDS[lds_addr + lane*16] = buf[voff].
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

template <int N>
__device__ __forceinline__ void svm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

__device__ __forceinline__ si32x4_t srsrc(const void* base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)base;
    si32x4_t r;
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

__device__ __forceinline__ void sbar() { asm volatile("s_barrier" ::: "memory"); }

struct TileS {
    int img, oh0, ow0;
};

// XCD-contiguous persistent tile range of this block (blocks are dealt
// round-robin over the 8 XCDs): XCD x owns [s_x, s_x + n_x), its nb_x blocks
// stride through it, so the tiles in flight on one XCD are raster neighbours
// whose halo rows are L2 hits.
struct TileRange {
    int s_x, n_x, nb_x, li;
};
__device__ __forceinline__ TileRange tile_range(int ntiles) {
    const int nwg = (int)gridDim.x, bx = (int)blockIdx.x, xcd = bx & 7;
    const int nt8 = ntiles >> 3, rt8 = ntiles & 7;
    TileRange r;
    r.s_x = xcd < rt8 ? xcd * (nt8 + 1) : rt8 * (nt8 + 1) + (xcd - rt8) * nt8;
    r.n_x = nt8 + (xcd < rt8 ? 1 : 0);
    r.nb_x = (nwg >> 3) + (xcd < (nwg & 7) ? 1 : 0);
    r.li = bx >> 3;
    return r;
}

// BN scale / shift of this lane's 2 x 8 output channels c0 + 32 * i2 + 8 * kq + r,
// loaded once, waited for here and made opaque, so that no compiler-inserted
// vmcnt wait for them can land inside the DMA-counted main loop.
__device__ __forceinline__ void load_affine_regs(const ConvArgs& a, int c0, int kq, float (&sc)[2][8],
                                                 float (&sh)[2][8]) {
    const bool aff = a.flags & RR_CONV_AFFINE;
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2) {
        const int c = c0 + 32 * i2 + 8 * kq;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            sc[i2][r] = aff ? a.scale[c + r] : 1.f;
            sh[i2][r] = aff ? a.shift[c + r] : 0.f;
        }
    }
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(sc[i2][r]), "+v"(sh[i2][r]));
}

// one 16-B epilogue store: fragment pair (acc[2 i2], acc[2 i2 + 1]) of pixel fragment j
template <typename HT>
__device__ __forceinline__ void store8(HT* __restrict__ Y, long long o, const sf32x4_t& a0, const sf32x4_t& a1,
                                       const float (&sc)[8], const float (&sh)[8], float sl) {
    float v[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        v[r] = a0[r] * sc[r] + sh[r];
        v[4 + r] = a1[r] * sc[4 + r] + sh[4 + r];
    }
    // leaky(v) = max(v, slope * v) for slope in [0, 1] (host-checked; identity: slope 1)
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = fmaxf(v[r], v[r] * sl);
    uint4 q;
    q.x = H16<HT>::pack2(v[0], v[1]);
    q.y = H16<HT>::pack2(v[2], v[3]);
    q.z = H16<HT>::pack2(v[4], v[5]);
    q.w = H16<HT>::pack2(v[6], v[7]);
    *reinterpret_cast<uint4*>(Y + o) = q;
}

// ---------------------------------------------------------------------------
// c_out = 128, c_in = 64 * nck.  LDS: 3 weight stages x 16 KiB + 2 patch buffers x 44 KiB.
template <typename HT>
__global__ void __launch_bounds__(512, 1) k_c3s_w128(ConvArgs a, int tiles_w, int tiles_hw, int ntiles) {
    constexpr int TW = 32, PC = TW + 2, NPIX = 10 * PC;  // 8 x 32 tile, (8+2) x (32+2) patch
    constexpr int NPC = (NPIX + 7) / 8;                   // 43 pieces of 8 pixels x 128 B
    constexpr int WST = 128 * 128, PB = 44 * 1024, WBYTES = 3 * WST;
    __shared__ __attribute__((aligned(1024))) char smem[WBYTES + 2 * PB];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wn = wave & 3;
    TileRange tr = tile_range(ntiles);
    if (tr.li >= tr.n_x) return;
    const int H = a.h, W = a.w_, Cin = a.cin, nck = Cin >> 6, KS = 9 * nck;
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    const int lrow = lane >> 3, lch = lane & 7, r16 = lane & 15, kq = lane >> 4;
    const si32x4_t rsX = srsrc(a.x, (unsigned)((long long)a.n * H * W * Cin * 2));
    const si32x4_t rsW = srsrc(a.w, (unsigned)(128ll * a.kp * 2));

    float esc[2][8], esh[2][8];
    load_affine_regs(a, grp * 64, kq, esc, esh);
    const float sl = a.act == RR_ACT_LEAKY ? a.slope : 1.f;

    auto tile_of = [&](int t) {
        TileS c;
        c.img = t / tiles_hw;
        const int rem = t - c.img * tiles_hw;
        const int th = rem / tiles_w;
        c.oh0 = th * 8;
        c.ow0 = (rem - th * tiles_w) * TW;
        return c;
    };
    // patch piece i (0..5) of (tile, chunk cc) into patch buffer `buf`; live = false: zeros
    auto piece = [&](const TileS& tc, int cc, int buf, int i, bool live) {
        const int d = min(wave + 8 * i, NPC - 1);  // pieces past the last repeat it (same bytes)
        const int q = d * 8 + lrow;
        const int pr = q / PC, pcol = q - pr * PC;
        const int hh = tc.oh0 - 1 + pr, ww = tc.ow0 - 1 + pcol;
        unsigned off = SOOB;
        if (live && q < NPIX && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
            off = (unsigned)(((((long long)tc.img * H + hh) * W + ww) * Cin + cc * 64 + ((lch ^ lrow) << 3)) * 2);
        sdma16(rsX, off, lds0 + WBYTES + buf * PB + d * 1024);
    };
    // weight K-step ks (chunk ks / 9, tap ks % 9) into ring stage ks % 3: 128 rows x 128 B
    auto wstep = [&](int ks) {
        const int cc = ks / 9, tap = ks - cc * 9;
        const unsigned k0b = (unsigned)((tap * Cin + cc * 64) * 2);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int row = (wave + 8 * i) * 8 + lrow;
            sdma16(rsW, (unsigned)(row * a.kp * 2) + k0b + (unsigned)((lch ^ lrow) << 4),
                   lds0 + (ks % 3) * WST + (wave + 8 * i) * 1024);
        }
    };

    int bq[2][2];  // patch pixel of (pixel half h, fragment j) at tap (0, 0)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 2; ++j) bq[h][j] = (h * 4 + wn) * PC + j * 16 + r16;

    sf32x4_t acc[2][4][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[h][i][j] = (sf32x4_t){0.f, 0.f, 0.f, 0.f};
    uint4 fa[4][2], fb[2][2];
    const int arow0 = grp * 64 + r16;

    auto mfma_h = [&](int h) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int hs = 0; hs < 2; ++hs)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[h][i][j] = H16<HT>::mfma(fa[i][hs], fb[j][hs], acc[h][i][j]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    HT* __restrict__ Y = (HT*)a.y;

    // ---- prologue: weight K-steps 0, 1 and chunk 0 of the first tile
    TileS cur = tile_of(tr.s_x + tr.li);
    int pb = 0;  // patch buffer of the current chunk
    wstep(0);
    wstep(1 % KS);
#pragma unroll
    for (int i = 0; i < 6; ++i) piece(cur, 0, 0, i, true);
    svm_wait<0>();
    sbar();
    if (grp == 1) sbar();  // stagger: group 1 runs one barrier behind group 0

    for (;;) {
        const int li_next = tr.li + tr.nb_x;
        const bool more = li_next < tr.n_x;
        const TileS nxt = more ? tile_of(tr.s_x + li_next) : cur;
        for (int cc = 0; cc < nck; ++cc) {
            const bool last_chunk = cc + 1 == nck;
            const char* Ps = smem + WBYTES + pb * PB;
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int ks = cc * 9 + tap;
                const int toff = (tap / 3) * PC + tap % 3;
                // phase A: pixel half 0; A fragments of K-step ks (kept for phase B)
                {
                    const char* Ws = smem + (ks % 3) * WST;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int hs = 0; hs < 2; ++hs)
                            fa[i][hs] = *reinterpret_cast<const uint4*>(
                                Ws + (arow0 + i * 16) * 128 + (((kq + 4 * hs) ^ (r16 & 7)) << 4));
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        // opaque per-phase copy: the 36 tap x fragment addresses are derived
                        // here instead of being hoisted (and spilled) as loop invariants
                        int qj = bq[0][j];
                        asm volatile("" : "+v"(qj));
                        const int q = qj + toff;
#pragma unroll
                        for (int hs = 0; hs < 2; ++hs)
                            fb[j][hs] = *reinterpret_cast<const uint4*>(Ps + q * 128 + (((kq + 4 * hs) ^ (q & 7)) << 4));
                    }
                    // weight K-step ks + 2 into the stage K-step ks - 1 used (read two phases ago)
                    int k2 = ks + 2;
                    if (k2 >= KS) k2 -= KS;
                    wstep(k2);
                    sbar();
                    mfma_h(0);
                    sbar();
                }
                // phase B: pixel half 1; piece `tap` of the next chunk into the other buffer
                {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        int qj = bq[1][j];
                        asm volatile("" : "+v"(qj));
                        const int q = qj + toff;
#pragma unroll
                        for (int hs = 0; hs < 2; ++hs)
                            fb[j][hs] = *reinterpret_cast<const uint4*>(Ps + q * 128 + (((kq + 4 * hs) ^ (q & 7)) << 4));
                    }
                    if (tap <= 5) {
                        if (!last_chunk) piece(cur, cc + 1, pb ^ 1, tap, true);
                        else piece(nxt, 0, pb ^ 1, tap, more);
                    }
                    // weight K-step ks + 1 (issued in phase A of ks - 1) has landed: only the
                    // younger ops may stay in flight (the previous tile's 8 epilogue stores too at ks = 0)
                    if (tap == 0) {
                        if (cc == 0) svm_wait<11>();
                        else svm_wait<3>();
                    } else if (tap <= 5) {
                        svm_wait<4>();
                    } else if (tap == 6) {
                        svm_wait<3>();
                    } else {
                        svm_wait<2>();
                    }
                    sbar();
                    mfma_h(1);
                    sbar();
                }
            }
            pb ^= 1;
        }
        // ---- epilogue: 8 stores per lane (the tile's stores stay in flight across the next phases)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const long long pix = ((long long)cur.img * H + cur.oh0 + h * 4 + wn) * W + cur.ow0 + j * 16 + r16;
#pragma unroll
                for (int i2 = 0; i2 < 2; ++i2)
                    store8<HT>(Y, pix * a.ldy + grp * 64 + 32 * i2 + 8 * kq, acc[h][2 * i2][j], acc[h][2 * i2 + 1][j],
                               esc[i2], esh[i2], sl);
            }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[h][i][j] = (sf32x4_t){0.f, 0.f, 0.f, 0.f};
        if (!more) break;
        tr.li = li_next;
        cur = nxt;
    }
    if (grp == 0) sbar();  // equal barrier counts for both groups
    svm_wait<0>();
}

// ---------------------------------------------------------------------------
// c_in = c_out = 64.  LDS: 18 resident weight K-steps x 4 KiB + 2 chunk patches x 39 KiB.
// 64-B pixel rows: logical 16-B chunk c of LDS pixel / weight row q sits at
// physical chunk (c + ((q >> 1) & 2)) & 3.
__device__ __forceinline__ int sw64(int c, int q) { return (c + ((q >> 1) & 2)) & 3; }

template <typename HT>
__global__ void __launch_bounds__(512, 1) k_c3s_w64(ConvArgs a, int tiles_w, int tiles_hw, int ntiles) {
    constexpr int TW = 32, PC = TW + 2, NPIX = 18 * PC;  // 16 x 32 tile, (16+2) x (32+2) patch
    constexpr int NPC = (NPIX + 15) / 16;                 // 39 pieces of 16 pixels x 64 B
    constexpr int KST = 64 * 64, WBYTES = 18 * KST, PB = NPC * 1024;
    __shared__ __attribute__((aligned(1024))) char smem[WBYTES + 2 * PB];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2;
    TileRange tr = tile_range(ntiles);
    if (tr.li >= tr.n_x) return;
    const int H = a.h, W = a.w_;
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    const int r16 = lane & 15, kq = lane >> 4;
    const si32x4_t rsX = srsrc(a.x, (unsigned)((long long)a.n * H * W * 64 * 2));

    float esc[2][8], esh[2][8];
    load_affine_regs(a, 0, kq, esc, esh);
    const float sl = a.act == RR_ACT_LEAKY ? a.slope : 1.f;

    auto tile_of = [&](int t) {
        TileS c;
        c.img = t / tiles_hw;
        const int rem = t - c.img * tiles_hw;
        const int th = rem / tiles_w;
        c.oh0 = th * 16;
        c.ow0 = (rem - th * tiles_w) * TW;
        return c;
    };
    // patch piece i (0..4) of (tile, 32-channel chunk cc) into buffer cc; live = false: zeros
    auto piece = [&](const TileS& tc, int cc, int i, bool live) {
        const int d = min(wave + 8 * i, NPC - 1);
        const int q = d * 16 + (lane >> 2);
        const int lc = (lane - ((q >> 1) & 2)) & 3;  // logical chunk whose physical slot this lane fills
        const int pr = q / PC, pcol = q - pr * PC;
        const int hh = tc.oh0 - 1 + pr, ww = tc.ow0 - 1 + pcol;
        unsigned off = SOOB;
        if (live && q < NPIX && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
            off = (unsigned)(((((long long)tc.img * H + hh) * W + ww) * 64 + cc * 32 + lc * 8) * 2);
        sdma16(rsX, off, lds0 + WBYTES + cc * PB + d * 1024);
    };

    int bq[2][2];  // patch pixel of (pixel half h, fragment j) at tap (0, 0)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 2; ++j) bq[h][j] = (h * 8 + wave) * PC + j * 16 + r16;

    sf32x4_t acc[2][4][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[h][i][j] = (sf32x4_t){0.f, 0.f, 0.f, 0.f};
    uint4 fa[4][2], fb[2][2];

    auto mfma_h = [&](int h) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int hs = 0; hs < 2; ++hs)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[h][i][j] = H16<HT>::mfma(fa[i][hs], fb[j][hs], acc[h][i][j]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    // fragments of 32-deep K-step ks (chunk ks / 9, tap ks % 9) into slot hs
    auto read_a = [&](int ks, int hs) {
        const char* Ws = smem + ks * KST;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = i * 16 + r16;
            fa[i][hs] = *reinterpret_cast<const uint4*>(Ws + row * 64 + (sw64(kq, row) << 4));
        }
    };
    auto read_b = [&](int ks, int h, int hs) {
        const int cc = ks / 9, tap = ks - cc * 9;
        const char* Ps = smem + WBYTES + cc * PB;
        const int toff = (tap / 3) * PC + tap % 3;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            int qj = bq[h][j];
            asm volatile("" : "+v"(qj));  // derived per phase, not hoisted as loop invariants
            const int q = qj + toff;
            fb[j][hs] = *reinterpret_cast<const uint4*>(Ps + q * 64 + (sw64(kq, q) << 4));
        }
    };
    HT* __restrict__ Y = (HT*)a.y;

    // ---- prologue: all 18 weight K-steps (9 instructions per wave) + chunk 0 of the first tile
    {
        const si32x4_t rsW = srsrc(a.w, (unsigned)(64ll * a.kp * 2));
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int u = wave + 8 * i;  // instruction u: K-step u / 4, rows (u % 4) * 16 .. + 15
            const int ks = u >> 2, cc = ks / 9, tap = ks - cc * 9;
            const int row = (u & 3) * 16 + (lane >> 2);
            const int lc = (lane - ((row >> 1) & 2)) & 3;
            sdma16(rsW, (unsigned)((row * a.kp + tap * 64 + cc * 32 + lc * 8) * 2), lds0 + ks * KST + (u & 3) * 1024);
        }
    }
    TileS cur = tile_of(tr.s_x + tr.li);
#pragma unroll
    for (int i = 0; i < 5; ++i) piece(cur, 0, i, true);
    svm_wait<0>();
    sbar();
    if (grp == 1) sbar();  // stagger: group 1 runs one barrier behind group 0

    for (;;) {
        const int li_next = tr.li + tr.nb_x;
        const bool more = li_next < tr.n_x;
        const TileS nxt = more ? tile_of(tr.s_x + li_next) : cur;
#pragma unroll
        for (int m = 0; m < 9; ++m) {
            // phase A: K-steps 2m, 2m + 1 on pixel half 0 (A fragments kept for phase B)
            read_a(2 * m, 0);
            read_a(2 * m + 1, 1);
            read_b(2 * m, 0, 0);
            read_b(2 * m + 1, 0, 1);
            // chunk 1 of this tile (buffer 1, last read two phases ago) in phases 1-3,
            // chunk 0 of the next tile (buffer 0) in phases 11-13
            if (m == 1) { piece(cur, 1, 2, true); piece(cur, 1, 3, true); }
            if (m == 6) { piece(nxt, 0, 2, more); piece(nxt, 0, 3, more); }
            sbar();
            mfma_h(0);
            sbar();
            // phase B: pixel half 1
            read_b(2 * m, 1, 0);
            read_b(2 * m + 1, 1, 1);
            if (m == 0) { piece(cur, 1, 0, true); piece(cur, 1, 1, true); }
            if (m == 1) piece(cur, 1, 4, true);
            if (m == 5) { piece(nxt, 0, 0, more); piece(nxt, 0, 1, more); }
            if (m == 6) piece(nxt, 0, 4, more);
            // chunk 1 is read from K-step 9 (m = 4), the next tile's chunk 0 from m = 0
            if (m == 3 || m == 8) svm_wait<0>();
            sbar();
            mfma_h(1);
            sbar();
        }
        // ---- epilogue: 8 stores per lane
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const long long pix = ((long long)cur.img * H + cur.oh0 + h * 8 + wave) * W + cur.ow0 + j * 16 + r16;
#pragma unroll
                for (int i2 = 0; i2 < 2; ++i2)
                    store8<HT>(Y, pix * a.ldy + 32 * i2 + 8 * kq, acc[h][2 * i2][j], acc[h][2 * i2 + 1][j], esc[i2],
                               esh[i2], sl);
            }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[h][i][j] = (sf32x4_t){0.f, 0.f, 0.f, 0.f};
        if (!more) break;
        tr.li = li_next;
        cur = nxt;
    }
    if (grp == 0) sbar();  // equal barrier counts for both groups
    svm_wait<0>();
}

}  // namespace

int g_conv3s = 1;  // rr_set_tuning(RR_TUNE_CONV3S): 0 off, 1 auto (default): the c_out = 128 form;
                   // 2 also the c_in = c_out = 64 form (measured 533-554 vs 525 us for k_conv3x3
                   // at 128 x R50 mod2: HBM-latency bound there, see DESIGN)

// bf16 / fp16 3x3 / stride 1 / pad 1, PERM32 weights, no residual, one
// channel tile (c_out = 128 with c_in % 64 == 0, or c_in = c_out = 64), image
// sizes the tiles divide, 31-bit buffer offsets; false: caller falls back.
bool launch_conv3s(const ConvArgs& a, hipStream_t s, bool f16) {
    if (!g_conv3s) return false;
    if (a.kh != 3 || a.kw != 3 || a.stride != 1 || a.pad != 1 || a.dil != 1) return false;
    if (!(a.flags & RR_CONV_PERM32) || (a.flags & RR_CONV_RESIDUAL) || a.ldy % 8) return false;
    if (a.act == RR_ACT_LEAKY && !(a.slope >= 0.f && a.slope <= 1.f)) return false;
    if (a.kp != 9 * a.cin || a.w_ % 32) return false;
    if ((long long)a.n * a.h * a.w_ * a.cin * 2 >= (1ll << 31) || (long long)a.cout * a.kp * 2 >= (1ll << 31)) return false;
    const bool w64 = g_conv3s == 2 && a.cin == 64 && a.cout == 64 && a.h % 16 == 0;
    const bool w128 = a.cout == 128 && a.cin % 64 == 0 && a.h % 8 == 0;
    if (!w64 && !w128) return false;
    const int th = w64 ? 16 : 8;
    const int tiles_w = a.w_ / 32, tiles_hw = (a.h / th) * tiles_w;
    const long long ntl = (long long)a.n * tiles_hw;
    const int cus = grid_cus();
    // at least two tiles per block, and a grid of >= 8 blocks (one per XCD range)
    if (ntl < 2ll * cus || cus < 8 || ntl >= (1ll << 31)) return false;
    const dim3 g((unsigned)cus), b(512);
    if (w64) {
        if (f16) hipLaunchKernelGGL((k_c3s_w64<f16_t>), g, b, 0, s, a, tiles_w, tiles_hw, (int)ntl);
        else hipLaunchKernelGGL((k_c3s_w64<bf16_t>), g, b, 0, s, a, tiles_w, tiles_hw, (int)ntl);
    } else {
        if (f16) hipLaunchKernelGGL((k_c3s_w128<f16_t>), g, b, 0, s, a, tiles_w, tiles_hw, (int)ntl);
        else hipLaunchKernelGGL((k_c3s_w128<bf16_t>), g, b, 0, s, a, tiles_w, tiles_hw, (int)ntl);
    }
    return true;
}

}  // namespace rr
