// librr.so — implicit-GEMM engine v2: LDS-DMA staging (buffer_load ... lds),
// 128-byte K-steps, counted vmcnt across raw barriers.
//
// Same GEMM view as rr_conv.hip (rows = output channels / database rows,
// cols = output pixels / queries, K-contiguous operands, NHWC epilogue), but:
//   * each K-step moves 128 B per row (64 bf16 / 32 f32) straight from HBM
//     into LDS with buffer_load_dwordx4 ... lds: one wave-instruction writes
//     8 whole rows (1 KiB) — no VGPR staging, no ds_write;
//   * im2col zero padding and out-of-range rows come for free: an invalid
//     lane gets a voffset beyond the buffer's num_records and the hardware
//     range check returns zeros;
//   * the bank-conflict swizzle lives on the SOURCE address: lane l of a
//     wave-instruction lands at LDS row 8j + l/8, physical chunk l%8, and
//     fetches logical chunk (l%8) ^ (row%8); fragment reads apply the same
//     XOR, which makes every ds_read_b128 lane group hit 16 distinct slots;
//   * two LDS stages, the next K-step's DMA issued before the current
//     step's MFMAs, waited with a counted s_waitcnt vmcnt(N) + raw s_barrier
//     (never __syncthreads(), whose fence would drain the prefetch).
#include "rr_internal.h"

#include <cstdlib>
#include <type_traits>

namespace rr {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

template <typename T> struct Vec2;
template <> struct Vec2<bf16_t> { static constexpr int N = 8; };
template <> struct Vec2<f16_t> { static constexpr int N = 8; };
template <> struct Vec2<float> { static constexpr int N = 4; };

constexpr unsigned OOB = 0x80000000u;  // voffset beyond every buffer: reads as 0

// One 16-B-per-lane LDS-DMA wave-instruction: LDS[m0 + lane*16] = buf[voff].
// Issued from inline asm so hipcc neither counts it nor inserts a blanket
// vmcnt(0) before later ds_reads (which it does for compiler-visible LDS-DMA):
// completion is tracked by the explicit vmcnt(N) below.  M0 is saved/restored.
typedef __attribute__((ext_vector_type(4))) int i32x4_t;
__device__ __forceinline__ void dma16(i32x4_t rsrc, unsigned voff, unsigned lds_addr) {
    unsigned keep;
    lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);  // wave-uniform by construction; make it provable
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
__device__ __forceinline__ void wait_vm_barrier() {
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(N) : "memory");
}
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ i32x4_t make_rsrc(const void* base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)base;
    i32x4_t r;
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

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

template <typename TO> struct St4;
template <> struct St4<float> {
    static __device__ __forceinline__ void st(float* p, const float* v) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
    static __device__ __forceinline__ void ld(const float* p, float* v) {
        float4 t = *reinterpret_cast<const float4*>(p);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    }
};
template <> struct St4<bf16_t> {
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

template <> struct St4<f16_t> {
    static __device__ __forceinline__ void st(f16_t* p, const float* v) {
        typedef __attribute__((ext_vector_type(4))) _Float16 h4;
        *reinterpret_cast<h4*>(p) = (h4){(f16_t)v[0], (f16_t)v[1], (f16_t)v[2], (f16_t)v[3]};
    }
    static __device__ __forceinline__ void ld(const f16_t* p, float* v) {
        typedef __attribute__((ext_vector_type(4))) _Float16 h4;
        const h4 t = *reinterpret_cast<const h4*>(p);
        v[0] = (float)t.x; v[1] = (float)t.y; v[2] = (float)t.z; v[3] = (float)t.w;
    }
};

// Persistent tile loop: block b walks tiles t = b, b + grid, ... as one
// flattened stream of (tile, K-step) steps, so the LDS-DMA of the next tile's
// first K-step is in flight while the current tile's epilogue runs.
// PERM: weight rows are stored in the 32-row MFMA-interleaved order
// (packed row g*32 + i*16 + 4*q + r  <->  channel g*32 + 8*q + 4*i + r), so a
// lane's two accumulator fragments hold 8 CONSECUTIVE output channels:
// one 16-B bf16 store / residual load per (fragment pair, pixel).
// AK > 0 ("A-stationary"): the layer has a single output-channel tile
// (c_out <= TC) and at most AK K-steps, so the whole weight slice is fetched
// into LDS once per block and only the activation tile streams through the
// ring — the per-CU LDS-DMA volume drops to the B operand alone.
// KM (operand-B addressing): 1 = 1x1 / pad 0 (K1), 2 = im2col with c_in a multiple of the
// 128-B K-step (every step inside one filter tap: wave-uniform tap, TAPU), 0 = generic im2col.
template <typename T, typename TO, int TC, int TP, int WC, int WP, int KM, bool PERM, int NS, int AK>
__global__ void __launch_bounds__(64 * WC * WP, ((NS == 2 && AK * TC <= 256) || WC * WP == 8 ? 2 : 1)) k_igemm(ConvArgs a, int tiles_p, int ntiles, int xmap) {
    constexpr bool K1 = KM == 1, tapu = KM == 2;
    constexpr int VEC = Vec2<T>::N;
    constexpr int BK = 8 * VEC;               // elements per K-step (128 B per row)
    constexpr int ESZ = sizeof(T);
    constexpr int NW = WC * WP;                  // waves per block (4 or 8)
    constexpr int NIA = TC / (8 * NW), NIB = TP / (8 * NW);  // LDS-DMA instructions per wave per stage
    constexpr int NLD = NIA + NIB;
    constexpr int FM = TC / WC / 16, FN = TP / WP / 16;
    constexpr int STAGE = (AK ? TP : TC + TP) * 128;
    constexpr int ABYTES = AK * TC * 128;
    static_assert(AK == 0 || NS == 2, "A-stationary uses the 2-stage ring");
    static_assert((NW == 4 || NW == 8) && TC % (8 * NW) == 0 && TP % (8 * NW) == 0, "tile");
    static_assert(!PERM || FM % 2 == 0, "PERM pairs fragments");

    static_assert(NS >= 2 && NS <= 4 && (NS - 1) * NLD < 64, "stages");
    __shared__ __attribute__((aligned(1024))) char smem[ABYTES + NS * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wc = wave % WC, wp = wave / WC;
    const int H = a.h, W = a.w_, Cin = a.cin;
    const unsigned tap_magic = tapu_magic(a.kh * a.kw);  // tapu_k0
    const long long xbytes = (long long)a.n * H * W * Cin * ESZ;
    const i32x4_t rsB = make_rsrc(a.x, (unsigned)xbytes);
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    const int lrow = lane >> 3;                 // row within an 8-row wave-instruction
    const int lchunk = (lane & 7) ^ (lrow & 7); // logical chunk fetched by this lane (source swizzle)
    const int nk = a.kp / BK;
    const int my_tiles = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    const int total = my_tiles * nk;
    // XCD-aware tile order: workgroups are placed round-robin over the 8 XCDs
    // (blockIdx % 8), so logical tile t runs on XCD t % 8.  Re-map it so each
    // XCD sweeps a contiguous range of pixel tiles: the im2col taps a tile
    // shares with its neighbours (rows above / below) are then L2 hits on the
    // same XCD instead of Infinity-Cache reads.  A bijection on [0, ntiles).
    // Within an XCD's range the order is pixel-tile-major, so the channel tiles
    // of one pixel tile run side by side and share its activations in L2.
    // xmap bit 1: static priority for the second half of the waves (the
    // arbitration loser of each SIMD pair), bit 0: XCD-contiguous tile order
    if ((xmap & 2) && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    xmap &= 1;
    const int n8 = xmap ? ntiles & ~7 : 0, per8 = n8 >> 3;
    const int tiles_c = ntiles / tiles_p;
    auto tile_at = [&](int lt) {  // -> channel-major tile index (c0 = t / tiles_p)
        const int t = (int)blockIdx.x + lt * (int)gridDim.x;
        if (!xmap) return t;
        const int q = t < n8 ? (t & 7) * per8 + (t >> 3) : t;
        return (q % tiles_c) * tiles_p + q / tiles_c;
    };

    // ---- issue-side state (tile whose K-steps are being fetched)
    i32x4_t rsA;
    unsigned a_off[NIA];
    int b_hi[NIB], b_wi[NIB];
    unsigned b_base[NIB];
    int is_tile = 0, is_k = 0;

    auto setup_tile = [&](int t) {
        const int c0 = (t / tiles_p) * TC, p0 = (t % tiles_p) * TP;
        const long long arows = (long long)min(TC, a.cout - c0);
        rsA = make_rsrc((const char*)a.w + (long long)c0 * a.kp * ESZ, (unsigned)(arows * a.kp * ESZ));
#pragma unroll
        for (int i = 0; i < NIA; ++i) {
            const int row = (wave + NW * i) * 8 + lrow;
            a_off[i] = row < arows ? (unsigned)(((long long)row * a.kp + lchunk * VEC) * ESZ) : OOB;
        }
#pragma unroll
        for (int i = 0; i < NIB; ++i) {
            const int row = (wave + NW * i) * 8 + lrow;
            const int p = p0 + row;
            if (p < a.P) {
                const int img = p / (a.ho * a.wo);
                const int rem = p - img * (a.ho * a.wo);
                const int oh = rem / a.wo, ow = rem - oh * a.wo;
                b_hi[i] = oh * a.stride - a.pad;
                b_wi[i] = ow * a.stride - a.pad;
                long long base = (long long)img * H * W * Cin;
                if (K1 || tapu) base += ((long long)b_hi[i] * W + b_wi[i]) * Cin + lchunk * VEC;
                b_base[i] = (unsigned)base;  // tapu: may wrap below 0; taps add back mod 2^32
            } else {
                b_hi[i] = b_wi[i] = -(1 << 28);  // fails every tap's bounds check
                b_base[i] = OOB;
            }
        }
    };

    auto issue = [&](int stage) {  // fetch step (is_tile, is_k) into `stage`, then advance
        if (is_k == 0) setup_tile(tile_at(is_tile));
        const int k0 = tapu ? tapu_k0(is_k, a.kh * a.kw, tap_magic, Cin / BK, Cin, BK) : is_k * BK;
        const unsigned As = lds0 + stage * STAGE;
        const unsigned Bs = AK ? lds0 + ABYTES + stage * STAGE : As + TC * 128;
        if constexpr (AK > 0) {
            if (is_tile == 0 && is_k == 0) {  // whole weight slice, once per block
                for (int kk = 0; kk < nk; ++kk)
#pragma unroll
                    for (int i = 0; i < NIA; ++i) {
                        const int kk0 = tapu ? tapu_k0(kk, a.kh * a.kw, tap_magic, Cin / BK, Cin, BK) : kk * BK;
                        const unsigned off = a_off[i] == OOB ? OOB : a_off[i] + (unsigned)(kk0 * ESZ);
                        dma16(rsA, off, lds0 + kk * TC * 128 + (wave + NW * i) * 1024);
                    }
            }
        } else {
#pragma unroll
            for (int i = 0; i < NIA; ++i) {
                const unsigned off = a_off[i] == OOB ? OOB : a_off[i] + (unsigned)(k0 * ESZ);
                dma16(rsA, off, As + (wave + NW * i) * 1024);
            }
        }
        int tap_dh = 0, tap_dw = 0, tap_add = 0;
        if constexpr (tapu) {
            const int tap = k0 >> a.lc, ci0 = k0 & (Cin - 1);
            const int kh = tap / a.kw, kw = tap - kh * a.kw;
            tap_dh = kh * a.dil;
            tap_dw = kw * a.dil;
            tap_add = (tap_dh * W + tap_dw) * Cin + ci0;
        }
#pragma unroll
        for (int i = 0; i < NIB; ++i) {
            unsigned off;
            if (K1) {
                off = b_base[i] == OOB ? OOB : (b_base[i] + (unsigned)k0) * ESZ;
            } else if constexpr (tapu) {
                // c_in is a multiple of the 128-B K-step: the step lies inside one tap, so
                // (kh, kw, ci0) are wave-uniform and a lane only re-checks its row's bounds
                const int hi = b_hi[i] + tap_dh, wi = b_wi[i] + tap_dw;
                const bool ok = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
                off = ok ? (b_base[i] + (unsigned)tap_add) * ESZ : OOB;
            } else {
                const int k = k0 + lchunk * VEC;
                const int tap = k >> a.lc;
                const int ci = k & (Cin - 1);
                const int kh = tap / a.kw;
                const int kw = tap - kh * a.kw;
                const int hi = b_hi[i] + kh * a.dil, wi = b_wi[i] + kw * a.dil;
                const bool ok = b_base[i] != OOB && kh < a.kh && hi >= 0 && hi < H && wi >= 0 && wi < W;
                off = ok ? (unsigned)((b_base[i] + ((long long)hi * W + wi) * Cin + ci) * ESZ) : OOB;
            }
            dma16(rsB, off, Bs + (wave + NW * i) * 1024);
        }
        if (++is_k == nk) { is_k = 0; ++is_tile; }
    };

    f32x4_t acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    const int r16 = lane & 15, kq = lane >> 4;
    const int arow0 = wc * (TC / WC) + r16, brow0 = wp * (TP / WP) + r16;
    TO* __restrict__ Y = (TO*)a.y;
    const TO* __restrict__ R = (const TO*)a.res;
    const bool affine = a.flags & RR_CONV_AFFINE;
    const bool resid = a.flags & RR_CONV_RESIDUAL;
    const bool leaky = a.act == RR_ACT_LEAKY;

    // bf16 PERM epilogue: the residual rows of the tile (8 channels = 16 B per
    // (fragment pair, pixel)) are fetched into registers while the tile's last
    // K-step is still on the MFMAs, so the epilogue does not wait on HBM.
    // With a 2-stage ring (XPREF) the fetch is issued one tile ahead, together
    // with that tile's first LDS-DMA, into the other of two register buffers,
    // so even single-K-step (K = 64) layers overlap the residual read.
    // (residual convs are the 1x1 conv3 of a block: K1 only; register budget: no spills at 64x64/wave)
    constexpr bool PREF = PERM && K1 && sizeof(TO) == 2 && FM * FN <= 16;
    constexpr bool XPREF = PREF && NS == 2;
    uint4 rres[XPREF ? 2 : 1][PREF ? FM / 2 : 1][PREF ? FN : 1];
    auto prefetch_res = [&](auto bsel, int t) {
        constexpr int BUF = decltype(bsel)::value;
        if constexpr (PREF) {
            if (!resid) return;
            const int c0 = (t / tiles_p) * TC, p0 = (t % tiles_p) * TP;
#pragma unroll
            for (int i2 = 0; i2 < FM / 2; ++i2)
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int c = c0 + wc * (TC / WC) + 32 * i2 + 8 * kq;
                    const int p = p0 + wp * (TP / WP) + j * 16 + r16;
                    rres[BUF][i2][j] = (c < a.cout && p < a.P)
                                      ? *reinterpret_cast<const uint4*>(R + (long long)p * a.ldy + c)
                                      : make_uint4(0, 0, 0, 0);
                }
        }
    };

    auto epilogue = [&](auto bsel, int t) {
        constexpr int BUF = decltype(bsel)::value;
        const int c0 = (t / tiles_p) * TC, p0 = (t % tiles_p) * TP;
        if constexpr (PERM) {
            float sc[FM / 2][8], sh[FM / 2][8];
#pragma unroll
            for (int i2 = 0; i2 < FM / 2; ++i2) {
                const int c = min(c0 + wc * (TC / WC) + 32 * i2 + 8 * kq, a.cout - 8);
                if (affine) {
                    St4<float>::ld(a.scale + c, sc[i2]);
                    St4<float>::ld(a.scale + c + 4, sc[i2] + 4);
                    St4<float>::ld(a.shift + c, sh[i2]);
                    St4<float>::ld(a.shift + c + 4, sh[i2] + 4);
                } else {
#pragma unroll
                    for (int r = 0; r < 8; ++r) { sc[i2][r] = 1.f; sh[i2][r] = 0.f; }
                }
            }
#pragma unroll
            for (int i2 = 0; i2 < FM / 2; ++i2) {
                const int c = c0 + wc * (TC / WC) + 32 * i2 + 8 * kq;  // 8 consecutive channels
                if (c >= a.cout) continue;                             // cout % 32 == 0 under PERM
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int p = p0 + wp * (TP / WP) + j * 16 + r16;
                    if (p >= a.P) continue;
                    float v[8];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] = acc[2 * i2][j][r] * sc[i2][r] + sh[i2][r];
                        v[4 + r] = acc[2 * i2 + 1][j][r] * sc[i2][4 + r] + sh[i2][4 + r];
                    }
                    const long long o = (long long)p * a.ldy + c;
                    if (resid) {
                        float rv[8];
                        if constexpr (PREF) {
                            const uint4 q = rres[BUF][i2][j];
                            const unsigned w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                rv[2 * r] = H16<TO>::lo(w4[r]);
                                rv[2 * r + 1] = H16<TO>::hi(w4[r]);
                            }
                        } else {
                            St4<TO>::ld(R + o, rv);
                            St4<TO>::ld(R + o + 4, rv + 4);
                        }
#pragma unroll
                        for (int r = 0; r < 8; ++r) v[r] += rv[r];
                    }
                    if (leaky) {
#pragma unroll
                        for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
                    }
                    if constexpr (sizeof(TO) == 2) {
                        uint4 q;
                        q.x = H16<TO>::pack2(v[0], v[1]);
                        q.y = H16<TO>::pack2(v[2], v[3]);
                        q.z = H16<TO>::pack2(v[4], v[5]);
                        q.w = H16<TO>::pack2(v[6], v[7]);
                        *reinterpret_cast<uint4*>(Y + o) = q;
                    } else {
                        St4<TO>::st(Y + o, v);
                        St4<TO>::st(Y + o + 4, v + 4);
                    }
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int c = c0 + wc * (TC / WC) + i * 16 + 4 * kq;
                if (c >= a.cout) continue;
                float sc[4] = {1.f, 1.f, 1.f, 1.f}, sh[4] = {0.f, 0.f, 0.f, 0.f};
                const bool full = (c + 3 < a.cout);
                if (affine) {
                    if (full) {
                        St4<float>::ld(a.scale + c, sc);
                        St4<float>::ld(a.shift + c, sh);
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
                    if constexpr (sizeof(TO) == 4) {
                        if (a.scr_k) {  // kNN screen: append survivors, store nothing
                            screen_append(a, v, c, a.cout, p, a.scr_tau[p]);
                            continue;
                        }
                    }
                    if (full) {
                        if (resid) {
                            float rv[4];
                            St4<TO>::ld(R + o, rv);
#pragma unroll
                            for (int r = 0; r < 4; ++r) v[r] += rv[r];
                        }
                        if (leaky) {
#pragma unroll
                            for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
                        }
                        St4<TO>::st(Y + o, v);
                    } else {
                        for (int r = 0; r < 4; ++r) {
                            if (c + r >= a.cout) break;
                            float tt = v[r];
                            if (resid) tt += DT<TO>::to_f(R[o + r]);
                            if (leaky) tt = tt > 0.f ? tt : tt * a.slope;
                            Y[o + r] = DT<TO>::from_f(tt);
                        }
                    }
                }
            }
        }
    };

    if (total == 0) return;
    // NS-stage ring: steps s+1 .. s+NS-1 are in flight while step s computes.
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    auto xprefetch = [&]() {  // after issue(): the issued step opened tile `is_tile - 1`
        if constexpr (XPREF) {
            if (is_k == 1 % nk || nk == 1) {
                const int lt = is_k == 0 ? is_tile - 1 : is_tile;  // local index of the tile just opened
                const int t = tile_at(lt);
                if (lt & 1) prefetch_res(B1{}, t);
                else prefetch_res(B0{}, t);
            }
        }
    };
    int issued = 0;
#pragma unroll
    for (int i = 0; i < NS - 1; ++i)
        if (issued < total) { issue(issued++ % NS); xprefetch(); }
    int ck = 0, ctile = 0;
    for (int s = 0; s < total; ++s) {
        const int cur = s % NS;
        if constexpr (NS == 2) {
            if (issued < total) { issue(issued++ % NS); xprefetch(); }
        }
        // wait until this wave's step-s DMA is done (younger steps may stay in
        // flight; older epilogue VMEM ops are drained too), then barrier: everyone's.
        const int ahead = issued - s - 1;
        if (NS >= 4 && ahead >= 3) wait_vm_barrier<(NS >= 4 ? 3 : 0) * NLD>();
        else if (NS >= 3 && ahead == 2) wait_vm_barrier<(NS >= 3 ? 2 : 0) * NLD>();
        else if (ahead == 1) wait_vm_barrier<AK ? NIB : NLD>();  // AK: a step issues B only (A's one-time load is older)
        else wait_vm_barrier<0>();
        // NS >= 3: ONE barrier per K-step.  The refill is issued after it, into
        // stage (s + NS - 1) % NS == (s - 1) % NS, which every wave finished
        // reading in step s - 1 (all of them have passed this barrier), so the
        // end-of-step LDS barrier of the 2-stage ring is not needed; NS - 2
        // steps stay in flight across the wait.
        if constexpr (NS >= 3) {
            if (issued < total) { issue(issued++ % NS); xprefetch(); }
        }
        if constexpr (!XPREF) {
            if (ck == nk - 1) prefetch_res(B0{}, tile_at(ctile));
        }
        const char* As = AK ? smem + ck * TC * 128 : smem + cur * STAGE;
        const char* Bs = AK ? smem + ABYTES + cur * STAGE : As + TC * 128;
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) {
            uint4 fa[FM], fb[FN];
#pragma unroll
            for (int i = 0; i < FM; ++i) fa[i] = *reinterpret_cast<const uint4*>(As + swz(arow0 + i * 16, kq + 4 * hs));
#pragma unroll
            for (int j = 0; j < FN; ++j) fb[j] = *reinterpret_cast<const uint4*>(Bs + swz(brow0 + j * 16, kq + 4 * hs));
            if constexpr (std::is_same<T, f16_t>::value) {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, fa[i]),
                                                                           __builtin_bit_cast(f16x8_t, fb[j]),
                                                                           acc[i][j], 0, 0, 0);
            } else if constexpr (VEC == 8) {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[i]),
                                                                            __builtin_bit_cast(bf16x8_t, fb[j]),
                                                                            acc[i][j], 0, 0, 0);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int j = 0; j < FN; ++j) {
                            const unsigned av = e == 0 ? fa[i].x : e == 1 ? fa[i].y : e == 2 ? fa[i].z : fa[i].w;
                            const unsigned bv = e == 0 ? fb[j].x : e == 1 ? fb[j].y : e == 2 ? fb[j].z : fb[j].w;
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av), __uint_as_float(bv),
                                                                             acc[i][j], 0, 0, 0);
                        }
            }
        }
        if constexpr (NS == 2) lds_barrier();  // every wave finished reading stage `cur` before it is refilled
        if (++ck == nk) {
            const int t = tile_at(ctile);
            if constexpr (XPREF) {
                if (ctile & 1) epilogue(B1{}, t);
                else epilogue(B0{}, t);
            } else {
                epilogue(B0{}, t);
            }
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
            ck = 0;
            ++ctile;
        }
    }
}

static int g_stages = 0;
static bool g_wide = true;
static bool g_ast = false;
static bool g_xmap = false;
static bool g_prio = false;
static bool g_env_done = false;

static int num_cus() {
    if (!g_env_done) {
        const char* e = getenv("RR_GEMM_STAGES");
        g_stages = (e && (e[0] == '3')) ? 3 : 2;
        const char* w = getenv("RR_GEMM_WIDE");
        g_wide = !(w && w[0] == '0');
        const char* pr = getenv("RR_GEMM_PRIO");
        g_prio = pr && pr[0] == '1';
        g_env_done = true;
    }
    return grid_cus();
}

template <typename T, typename TO, int TC, int TP, int WC, int WP, int NS, int AK = 0>
static void launch_ns(const ConvArgs& a, bool k1, bool perm, hipStream_t s) {
    constexpr int LDS = AK * TC * 128 + NS * (AK ? TP : TC + TP) * 128;
    constexpr int PER_CU = ((160 * 1024) / LDS >= 2 && WC * WP == 4) ? 2 : 1;
    const int tiles_p = (a.P + TP - 1) / TP;
    const int tiles_c = (a.cout + TC - 1) / TC;
    const int ntiles = tiles_p * tiles_c;
    const int cap = PER_CU * num_cus();
    const int grid = ntiles < cap ? ntiles : cap;
    const int km = k1 ? 1 : ((a.cin * (int)sizeof(T)) % 128 == 0 && tapu_ok(a.kh * a.kw, (long long)a.kp * (int)sizeof(T) / 128)) ? 2 : 0;
#define RR_L3(PV)                                                                                                    \
    do {                                                                                                             \
        if (km == 1)                                                                                                 \
            hipLaunchKernelGGL((k_igemm<T, TO, TC, TP, WC, WP, 1, PV, NS, AK>), dim3(grid), dim3(64 * WC * WP), 0, s, \
                               a, tiles_p, ntiles, (g_xmap ? 1 : 0) | (g_prio ? 2 : 0));                                                  \
        else if (km == 2)                                                                                            \
            hipLaunchKernelGGL((k_igemm<T, TO, TC, TP, WC, WP, 2, PV, NS, AK>), dim3(grid), dim3(64 * WC * WP), 0, s, \
                               a, tiles_p, ntiles, (g_xmap ? 1 : 0) | (g_prio ? 2 : 0));                                                  \
        else                                                                                                         \
            hipLaunchKernelGGL((k_igemm<T, TO, TC, TP, WC, WP, 0, PV, NS, AK>), dim3(grid), dim3(64 * WC * WP), 0, s, \
                               a, tiles_p, ntiles, (g_xmap ? 1 : 0) | (g_prio ? 2 : 0));                                                  \
    } while (0)
    if constexpr (std::is_same<T, TO>::value && (TC / WC / 16) % 2 == 0) {
        if (perm) {
            RR_L3(true);
            return;
        }
    }
    RR_L3(false);
#undef RR_L3
}

template <typename T, typename TO, int TC, int TP, int WC, int WP>
static void launch_cfg3(const ConvArgs& a, bool k1, bool perm, hipStream_t s) {
    num_cus();
    if constexpr (3 * (TC + TP) * 128 <= 160 * 1024 && WC * WP == 4) {
        if (g_stages == 3) {
            launch_ns<T, TO, TC, TP, WC, WP, 3>(a, k1, perm, s);
            return;
        }
    }
    launch_ns<T, TO, TC, TP, WC, WP, 2>(a, k1, perm, s);
}


// ---------------------------------------------------------------------------
// 8-phase 256 x 256 tile with staggered wave groups (16-bit operands).
//
// The k_igemm ring above keeps ONE K-step in flight across each barrier pair,
// so every 64-deep step waits on its own LDS-DMA (MFMA busy ~40 %).  Here the
// 256 x 256 x 64 step is split into four 128 x 128 quadrants and the operand
// tiles into half-tiles (A0 / A1 = channel rows 0-127 / 128-255, B0 / B1 =
// pixel rows 0-127 / 128-255; 128 rows x 128 B = 16 KiB each), double
// buffered (E: even K-steps, O: odd; 128 KiB of LDS):
//   * a phase = one quadrant x K 64: the block's 8 waves each do a 64 x 32
//     sub-block (16 MFMAs), reading only the half-tiles of that quadrant;
//     quadrant order (0,0) (0,1) (1,1) (1,0) reuses the A or B fragments of
//     the previous phase from registers;
//   * every phase issues ONE half-tile LDS-DMA (2 per lane), into the
//     half-tile whose last read was two phases earlier, for the K-step that
//     buffer holds next: each load has 4-7 phases to land;
//   * s_waitcnt vmcnt(4) once per K-step (phases 4 and 8) retires the loads
//     the next four phases read; raw s_barrier, never vmcnt(0) in the loop;
//   * waves 4-7 run one barrier behind waves 0-3 (each SIMD holds one wave
//     of each group): while one group runs its MFMA cluster the other reads
//     LDS / issues DMA, so the matrix pipe of every SIMD alternates between
//     two instruction streams.  The two-phase restage distance and the wait
//     placement (before the first barrier of the phase preceding the reads)
//     are what keep both hazards closed under that one-barrier skew.
// Tiles are assigned XCD-contiguously (bijective remap): the pixel tiles of
// one channel tile (e.g. the query tiles of one database tile in the kNN
// score GEMM) share their A rows in one XCD's L2.  One tile per block.
// T = int8_t: the kNN screening GEMM on int8-quantised rows (v_mfma_i32_16x16x64_i8,
// twice the bf16 MFMA rate, half the bytes per row): a 128-B K-step is 128 elements
// (two 64-deep MFMAs), the accumulators are exact int32 and the epilogue converts
// them to float (K1, natural row order, float out only).
template <typename T, typename TO, int KM, bool PERM>
__global__ void __launch_bounds__(512, 1) k_gemm8(ConvArgs a, int tiles_p, int ntiles, int pmajor) {
    constexpr bool I8 = std::is_same<T, int8_t>::value;
    static_assert(sizeof(T) == 2 || (I8 && KM == 1 && !PERM && sizeof(TO) == 4), "16-bit operands / int8 scores");
    constexpr bool K1 = KM == 1, tapu = KM == 2;
    constexpr int ESZ = sizeof(T), VEC = 16 / ESZ, KSE = 128 / ESZ, HT = 16384, SS_MAX = 2048;
    // [buf E/O][A0, A1, B0, B1] + folded BN scale / shift of up to 2048 channels
    __shared__ __attribute__((aligned(1024))) char smem[8 * HT + 2 * SS_MAX * 4];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2;              // wave group; also the 64-row half of each quadrant
    // The epilogue reads scale / shift from LDS, so it issues no global load: a
    // load there would wait (vmcnt is in order) for the next tile's prologue DMA.
    float* const lds_sc = reinterpret_cast<float*>(smem + 8 * HT);
    float* const lds_sh = lds_sc + SS_MAX;
    const bool ss_lds = PERM && (a.flags & RR_CONV_AFFINE) && a.cout <= SS_MAX;
    if (ss_lds) {
        for (int c = tid; c < a.cout; c += 512) {
            lds_sc[c] = a.scale[c];
            lds_sh[c] = a.shift[c];
        }
    }
    // kNN screening (float out, natural order): the same region holds the queries'
    // thresholds (<= 1024) and the 8 waves' survivor lists (ScreenStage)
    uint32_t* const lds_tau = reinterpret_cast<uint32_t*>(smem + 8 * HT);
    uint32_t* const lds_stage = lds_tau + 1024;
    static_assert(4 * (1024 + 8 * 3 * ScreenStage::CAP) <= 2 * SS_MAX * 4, "screen staging fits the region");
    const bool tau_lds = !PERM && sizeof(TO) == 4 && a.scr_k && a.P <= 1024;
    if (tau_lds) {
        for (int q = tid; q < a.P; q += 512) lds_tau[q] = a.scr_tau[q];
        __syncthreads();  // visible to every wave before any epilogue reads it
    }
    const int wn = wave & 3;                // 32-column quarter of each quadrant
    // XCD-contiguous bijective tile order (blocks are dispatched round-robin over 8 XCDs)
    // Persistent blocks over an XCD-contiguous tile order: XCD x (blocks are
    // dispatched round-robin over the 8 XCDs) owns the contiguous tile range
    // [s_x, s_x + n_x) and its nb_x blocks stride through it, so the tiles in
    // flight on one XCD share A / B rows in its L2.  With one block per tile
    // (grid = ntiles) this is the plain bijective remap.
    const int nwg = (int)gridDim.x, bx = (int)blockIdx.x, xcd = bx & 7;
    const int nt8 = ntiles >> 3, rt8 = ntiles & 7;
    const int s_x = xcd < rt8 ? xcd * (nt8 + 1) : rt8 * (nt8 + 1) + (xcd - rt8) * nt8;
    const int n_x = nt8 + (xcd < rt8 ? 1 : 0);
    const int nb_x = (nwg >> 3) + (xcd < (nwg & 7) ? 1 : 0);
    int li = bx >> 3;  // this block's local tile index on its XCD
    if (li >= n_x) return;
    const int H = a.h, W = a.w_, Cin = a.cin;
    const unsigned tap_magic = tapu_magic(a.kh * a.kw);  // tapu_k0
    const int nk = a.kp / KSE;
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    const int lrow = lane >> 3, lchunk = (lane & 7) ^ (lrow & 7);

    // ---- per-tile LDS-DMA descriptors: half-tile h, instruction i covers rows (wave + 8 i) * 8 + lrow
    const i32x4_t rsB = make_rsrc(a.x, (unsigned)((long long)a.n * H * W * Cin * ESZ));
    int c0 = 0, p0 = 0;
    i32x4_t rsA;
    unsigned a_off[2][2], b_base[2][2];
    int b_hi[2][2], b_wi[2][2];
    // tile order: channel-major (the pixel tiles of one channel tile consecutive: the kNN
    // score GEMM's query tiles of one database tile share its rows in one XCD's L2) or
    // pixel-major (pmajor: the channel tiles of one pixel tile consecutive, so a conv's
    // input tile is fetched into one XCD's L2 once for all its channel tiles)
    const int tiles_c = ntiles / tiles_p;
    auto setup = [&](int t) {
        c0 = (pmajor ? t % tiles_c : t / tiles_p) * 256;
        p0 = (pmajor ? t / tiles_c : t % tiles_p) * 256;
        const long long arows = min(256, a.cout - c0);
        rsA = make_rsrc((const char*)a.w + (long long)c0 * a.kp * ESZ, (unsigned)(arows * a.kp * ESZ));
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int row = h * 128 + (wave + 8 * i) * 8 + lrow;
                a_off[h][i] = row < arows ? (unsigned)(((long long)row * a.kp + lchunk * VEC) * ESZ) : OOB;
                const int p = p0 + row;
                if (p < a.P) {
                    const int img = p / (a.ho * a.wo);
                    const int rem = p - img * (a.ho * a.wo);
                    const int oh = rem / a.wo, ow = rem - oh * a.wo;
                    b_hi[h][i] = oh * a.stride - a.pad;
                    b_wi[h][i] = ow * a.stride - a.pad;
                    b_base[h][i] = (unsigned)((long long)img * H * W * Cin +
                                              ((long long)b_hi[h][i] * W + b_wi[h][i]) * Cin + lchunk * VEC);
                } else {
                    b_hi[h][i] = b_wi[h][i] = -(1 << 28);
                    b_base[h][i] = OOB;
                }
            }
    };
    setup(s_x + li);
    // K-step descriptor, computed once per K-step (not per half-tile issue): the
    // DMA-issue slots sit between the barriers of the staggered schedule, so
    // every instruction there delays the partner group's matrix pipe.  The tap
    // split uses magic multiplies (no integer division on the issue path).
    const unsigned kw_magic = tapu_magic(a.kw);
    struct KD {
        int k0, dh, dw, add;
        bool live;
    };
    auto kdesc = [&](int kt) {
        KD d;
        d.live = kt < nk;
        d.k0 = tapu ? tapu_k0(kt, a.kh * a.kw, tap_magic, Cin >> 6, Cin, 64) : kt * KSE;
        d.dh = d.dw = d.add = 0;
        if constexpr (tapu) {
            const int tap = d.k0 >> a.lc, ci0 = d.k0 & (Cin - 1);
            const int kh = (int)(((unsigned)tap * kw_magic) >> 16), kw = tap - kh * a.kw;
            d.dh = kh * a.dil;
            d.dw = kw * a.dil;
            d.add = (d.dh * W + d.dw) * Cin + ci0;
        }
        return d;
    };
    // half-tile X (0 A0, 1 A1, 2 B0, 3 B1) of K-step d into buffer buf; K-steps >= nk load zeros
    auto issue = [&](int X, const KD& d, int buf) {
        const unsigned dst = lds0 + (buf * 4 + X) * HT;
        if (X < 2) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const unsigned off = (d.live && a_off[X][i] != OOB) ? a_off[X][i] + (unsigned)(d.k0 * ESZ) : OOB;
                dma16(rsA, off, dst + (wave + 8 * i) * 1024);
            }
        } else {
            const int h = X - 2;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                unsigned off = OOB;
                if (d.live && b_base[h][i] != OOB) {
                    if constexpr (K1) {
                        off = (b_base[h][i] + (unsigned)d.k0) * ESZ;
                    } else {
                        const int hi = b_hi[h][i] + d.dh, wi = b_wi[h][i] + d.dw;
                        if ((unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W)
                            off = (b_base[h][i] + (unsigned)d.add) * ESZ;
                    }
                }
                dma16(rsB, off, dst + (wave + 8 * i) * 1024);
            }
        }
    };
    const KD kd0 = kdesc(0), kd1 = kdesc(1);

    f32x4_t acc[2][2][4][2];
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[qa][qb][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    const int r16 = lane & 15, kq = lane >> 4;
    uint4 fa[4][2], fb[2][2];
    auto read_a = [&](int buf, int h) {
        const char* base = smem + (buf * 4 + h) * HT;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int hs = 0; hs < 2; ++hs)
                fa[i][hs] = *reinterpret_cast<const uint4*>(base + swz(grp * 64 + i * 16 + r16, kq + 4 * hs));
    };
    auto read_b = [&](int buf, int h) {
        const char* base = smem + (buf * 4 + 2 + h) * HT;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int hs = 0; hs < 2; ++hs)
                fb[j][hs] = *reinterpret_cast<const uint4*>(base + swz(wn * 32 + j * 16 + r16, kq + 4 * hs));
    };
    auto mfma_q = [&](int qa, int qb) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int hs = 0; hs < 2; ++hs)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if constexpr (I8)
                        acc[qa][qb][i][j] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_mfma_i32_16x16x64_i8(
                            __builtin_bit_cast(i32x4_t, fa[i][hs]), __builtin_bit_cast(i32x4_t, fb[j][hs]),
                            __builtin_bit_cast(i32x4_t, acc[qa][qb][i][j]), 0, 0, 0));
                    else if constexpr (std::is_same<T, f16_t>::value)
                        acc[qa][qb][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                            __builtin_bit_cast(f16x8_t, fa[i][hs]), __builtin_bit_cast(f16x8_t, fb[j][hs]),
                            acc[qa][qb][i][j], 0, 0, 0);
                    else
                        acc[qa][qb][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8_t, fa[i][hs]), __builtin_bit_cast(bf16x8_t, fb[j][hs]),
                            acc[qa][qb][i][j], 0, 0, 0);
                }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto bar = []() { asm volatile("s_barrier" ::: "memory"); };

    // ---- prologue: K-step 0 into E (A0 B1 A1 B0), K-step 1's A0 / B1 into O
    auto prologue = [&]() {
        issue(0, kd0, 0);
        issue(3, kd0, 0);
        issue(1, kd0, 0);
        issue(2, kd0, 0);
        issue(0, kd1, 1);
        issue(3, kd1, 1);
    };
    prologue();
    const int nit = (nk + 1) >> 1;
    // the previous tile's epilogue issued exactly ST_FULL stores and nothing else
    // (a full tile, no residual load); they are younger than this tile's prologue
    constexpr int ST_FULL = 16;
    static_assert(4 + ST_FULL == 20, "the counted wait below");
    bool prev_full = false;
    for (;;) {
        // K-step 0 has landed: only the 4 youngest DMAs (K-step 1's A0 / B1) and
        // the previous tile's epilogue stores (issued after this tile's prologue)
        // may still be in flight; an epilogue with a data-dependent store count
        // is waited for entirely
        if (prev_full) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");  // 4 + ST_FULL
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        bar();
        if (grp == 1) bar();  // stagger: group 1 runs one barrier behind group 0

    KD dto = kd1;  // descriptor of K-step `to`, carried from the previous iteration's to + 2
    for (int it = 0; it < nit; ++it) {
        const int te = 2 * it, to = 2 * it + 1;
        const KD de2 = kdesc(te + 2), do2 = kdesc(to + 2);
        // phases 1-4: K-step te from E; loads: A1-O(to), B0-O(to), A0-E(te+2), B1-E(te+2)
        read_a(0, 0); read_b(0, 0); issue(1, dto, 1);
        bar(); mfma_q(0, 0); bar();
        read_b(0, 1); issue(2, dto, 1);
        bar(); mfma_q(0, 1); bar();
        read_a(0, 1); issue(0, de2, 0);
        bar(); mfma_q(1, 1); bar();
        read_b(0, 0); issue(3, de2, 0);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // K-step `to` (buffer O) has landed
        bar(); mfma_q(1, 0); bar();
        // phases 5-8: K-step to from O; loads: A1-E(te+2), B0-E(te+2), A0-O(to+2), B1-O(to+2)
        read_a(1, 0); read_b(1, 0); issue(1, de2, 0);
        bar(); mfma_q(0, 0); bar();
        read_b(1, 1); issue(2, de2, 0);
        bar(); mfma_q(0, 1); bar();
        read_a(1, 1); issue(0, do2, 1);
        bar(); mfma_q(1, 1); bar();
        read_b(1, 0); issue(3, do2, 1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // K-step te + 2 (buffer E) has landed
        bar(); mfma_q(1, 0); bar();
        dto = do2;
    }
    if (grp == 0) bar();  // equal barrier counts for both groups: every wave's LDS reads are done
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing (zero) K-step DMAs have landed

    // the next tile's prologue DMA flies while this tile's epilogue runs
    const int ec0 = c0, ep0 = p0;
    li += nb_x;
    const bool more = li < n_x;
    TO* __restrict__ Y = (TO*)a.y;
    const TO* __restrict__ R = (const TO*)a.res;
    const bool affine = a.flags & RR_CONV_AFFINE;
    const bool resid = a.flags & RR_CONV_RESIDUAL;
    const bool leaky = a.act == RR_ACT_LEAKY;
    if (more) {
        setup(s_x + li);
        prologue();
    }
    // ---- epilogue: folded BN scale / shift, residual, activation, NHWC store
    if constexpr (PERM && sizeof(TO) == 2)
        prev_full = !resid && (ss_lds || !affine) && ec0 + 256 <= a.cout && ep0 + 256 <= a.P;
    bool screened = false;
    if constexpr (!PERM && sizeof(TO) == 4) {
        if (a.scr_k) {  // kNN screen: stage the survivors, append them in batches, store nothing
            screened = true;
            ScreenStage st{lds_stage + wave * 3 * ScreenStage::CAP, 0};
#pragma unroll
            for (int qa = 0; qa < 2; ++qa)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            const int c = ec0 + qa * 128 + grp * 64 + i * 16 + 4 * kq;
                            const int p = ep0 + qb * 128 + wn * 32 + j * 16 + r16;
                            const bool ok = p < a.P;
                            uint32_t tau = 0xffffffffu;
                            if (ok) tau = tau_lds ? lds_tau[p] : a.scr_tau[p];
                            float v[4];
#pragma unroll
                            for (int r = 0; r < 4; ++r)  // (as the affine-free store path)
                                v[r] = I8 ? (float)__builtin_bit_cast(i32x4_t, acc[qa][qb][i][j])[r]
                                          : acc[qa][qb][i][j][r] * 1.f + 0.f;
                            st.add(a, v, c, a.cout, p, ok, tau);
                        }
            st.flush(a);
        }
    }
#pragma unroll
    for (int qa = 0; qa < 2 && !screened; ++qa) {
        if constexpr (PERM) {
#pragma unroll
            for (int i2 = 0; i2 < 2; ++i2) {
                const int c = ec0 + qa * 128 + grp * 64 + 32 * i2 + 8 * kq;  // 8 consecutive channels
                if (c >= a.cout) continue;
                float sc[8], sh[8];
                if (ss_lds) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) { sc[r] = lds_sc[c + r]; sh[r] = lds_sh[c + r]; }
                } else if (affine) {
                    St4<float>::ld(a.scale + c, sc);
                    St4<float>::ld(a.scale + c + 4, sc + 4);
                    St4<float>::ld(a.shift + c, sh);
                    St4<float>::ld(a.shift + c + 4, sh + 4);
                } else {
#pragma unroll
                    for (int r = 0; r < 8; ++r) { sc[r] = 1.f; sh[r] = 0.f; }
                }
#pragma unroll
                for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int p = ep0 + qb * 128 + wn * 32 + j * 16 + r16;
                        if (p >= a.P) continue;
                        float v[8];
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            v[r] = acc[qa][qb][2 * i2][j][r] * sc[r] + sh[r];
                            v[4 + r] = acc[qa][qb][2 * i2 + 1][j][r] * sc[4 + r] + sh[4 + r];
                        }
                        const long long o = (long long)p * a.ldy + c;
                        if (resid) {
                            float rv[8];
                            St4<TO>::ld(R + o, rv);
                            St4<TO>::ld(R + o + 4, rv + 4);
#pragma unroll
                            for (int r = 0; r < 8; ++r) v[r] += rv[r];
                        }
                        if (leaky) {
#pragma unroll
                            for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
                        }
                        if constexpr (sizeof(TO) == 2) {
                            uint4 q;
                            q.x = H16<TO>::pack2(v[0], v[1]);
                            q.y = H16<TO>::pack2(v[2], v[3]);
                            q.z = H16<TO>::pack2(v[4], v[5]);
                            q.w = H16<TO>::pack2(v[6], v[7]);
                            *reinterpret_cast<uint4*>(Y + o) = q;
                        } else {
                            St4<TO>::st(Y + o, v);
                            St4<TO>::st(Y + o + 4, v + 4);
                        }
                    }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c = ec0 + qa * 128 + grp * 64 + i * 16 + 4 * kq;
                if (c >= a.cout) continue;
                float sc[4] = {1.f, 1.f, 1.f, 1.f}, sh[4] = {0.f, 0.f, 0.f, 0.f};
                const bool full = c + 3 < a.cout;
                if (affine) {
                    for (int r = 0; r < 4; ++r)
                        if (c + r < a.cout) { sc[r] = a.scale[c + r]; sh[r] = a.shift[c + r]; }
                }
#pragma unroll
                for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int p = ep0 + qb * 128 + wn * 32 + j * 16 + r16;
                        if (p >= a.P) continue;
                        float v[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            v[r] = I8 ? (float)__builtin_bit_cast(i32x4_t, acc[qa][qb][i][j])[r]
                                      : acc[qa][qb][i][j][r] * sc[r] + sh[r];
                        if constexpr (sizeof(TO) == 4) {
                            if (a.scr_k) {  // kNN screen: append survivors, store nothing
                                screen_append(a, v, c, a.cout, p, a.scr_tau[p]);
                                continue;
                            }
                        }
                        const long long o = (long long)p * a.ldy + c;
                        if (full) {
                            if (resid) {
                                float rv[4];
                                St4<TO>::ld(R + o, rv);
#pragma unroll
                                for (int r = 0; r < 4; ++r) v[r] += rv[r];
                            }
                            if (leaky) {
#pragma unroll
                                for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
                            }
                            St4<TO>::st(Y + o, v);
                        } else {
                            for (int r = 0; r < 4; ++r) {
                                if (c + r >= a.cout) break;
                                float tt = v[r];
                                if (resid) tt += DT<TO>::to_f(R[o + r]);
                                if (leaky) tt = tt > 0.f ? tt : tt * a.slope;
                                Y[o + r] = DT<TO>::from_f(tt);
                            }
                        }
                    }
            }
        }
    }
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[qa][qb][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    if (!more) break;
    }  // persistent tile loop
}

// ---------------------------------------------------------------------------
// Half-width 8-phase variant for the kNN score GEMM at <= 128 queries: a
// 256 (database rows, A) x 128 (queries, B) tile, so no MFMA runs on empty
// query rows (k_gemm8's 256-wide pixel tile would waste half of them).
// Same wave layout, quadrant phases and one-barrier wave-group stagger as
// k_gemm8, with two phases per 64-deep K-step (A0 x B0, A1 x B0; the B
// fragments stay in registers for the second) and a 3-stage ring of
// {A0, A1, B0} half-tiles (144 KiB): K-step t + 2's A0 / B0 are issued in
// phase A of t and its A1 in phase B of t, into the stage K-step t - 1 used --
// every half-tile is overwritten two phases after its last read (the k_gemm8
// rule that keeps the skewed group's reads safe) and has four phases to land.
// Counted waits (2 DMA instructions per half-tile and lane): phase A waits for
// this K-step's A1 (10 younger), phase B for the next K-step's A0 / B0 (8).
template <typename T>
__global__ void __launch_bounds__(512, 1) k_gemm8h(ConvArgs a, int ntiles) {
    static_assert(sizeof(T) == 2, "16-bit operands");
    constexpr int VEC = 8, ESZ = 2, HT = 16384, ST = 3 * HT;  // stage = [A0, A1, B0]
    __shared__ __attribute__((aligned(1024))) char smem[3 * ST];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wn = wave & 3;
    // XCD-contiguous bijective tile order (one block per tile)
    const int bx = (int)blockIdx.x, xcd = bx & 7;
    const int nt8 = ntiles >> 3, rt8 = ntiles & 7;
    const int t = (xcd < rt8 ? xcd * (nt8 + 1) : rt8 * (nt8 + 1) + (xcd - rt8) * nt8) + (bx >> 3);
    if (t >= ntiles) return;
    const int nk = a.kp / 64;
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    const int lrow = lane >> 3, lchunk = (lane & 7) ^ (lrow & 7);

    const int c0 = t * 256;
    const long long arows = min(256, a.cout - c0);
    const i32x4_t rsA = make_rsrc((const char*)a.w + (long long)c0 * a.kp * ESZ, (unsigned)(arows * a.kp * ESZ));
    const i32x4_t rsB = make_rsrc(a.x, (unsigned)((long long)a.P * a.cin * ESZ));
    unsigned a_off[2][2], b_off[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int row = h * 128 + (wave + 8 * i) * 8 + lrow;
            a_off[h][i] = row < arows ? (unsigned)(((long long)row * a.kp + lchunk * VEC) * ESZ) : OOB;
        }
        const int p = (wave + 8 * i) * 8 + lrow;
        b_off[i] = p < a.P ? (unsigned)(((long long)p * a.cin + lchunk * VEC) * ESZ) : OOB;
    }
    // half-tile X (0 A0, 1 A1, 2 B0) of K-step kt into its ring stage; K-steps >= nk load zeros
    auto issue = [&](int X, int kt) {
        const unsigned dst = lds0 + (kt % 3) * ST + X * HT;
        const bool live = kt < nk;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const unsigned base = X < 2 ? a_off[X][i] : b_off[i];
            const unsigned off = (live && base != OOB) ? base + (unsigned)(kt * 128) : OOB;
            dma16(X < 2 ? rsA : rsB, off, dst + (wave + 8 * i) * 1024);
        }
    };

    f32x4_t acc[2][4][2];
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[qa][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int r16 = lane & 15, kq = lane >> 4;
    uint4 fa[4][2], fb[2][2];
    auto read_a = [&](int kt, int h) {
        const char* base = smem + (kt % 3) * ST + h * HT;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int hs = 0; hs < 2; ++hs)
                fa[i][hs] = *reinterpret_cast<const uint4*>(base + swz(grp * 64 + i * 16 + r16, kq + 4 * hs));
    };
    auto read_b = [&](int kt) {
        const char* base = smem + (kt % 3) * ST + 2 * HT;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int hs = 0; hs < 2; ++hs)
                fb[j][hs] = *reinterpret_cast<const uint4*>(base + swz(wn * 32 + j * 16 + r16, kq + 4 * hs));
    };
    auto mfma_q = [&](int qa) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int hs = 0; hs < 2; ++hs)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if constexpr (std::is_same<T, f16_t>::value)
                        acc[qa][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                            __builtin_bit_cast(f16x8_t, fa[i][hs]), __builtin_bit_cast(f16x8_t, fb[j][hs]),
                            acc[qa][i][j], 0, 0, 0);
                    else
                        acc[qa][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8_t, fa[i][hs]), __builtin_bit_cast(bf16x8_t, fb[j][hs]),
                            acc[qa][i][j], 0, 0, 0);
                }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto bar = []() { asm volatile("s_barrier" ::: "memory"); };

    // prologue: K-steps 0 and 1 (A0, B0, A1 each); K-step 0's A0 / B0 landed
    issue(0, 0); issue(2, 0); issue(1, 0);
    issue(0, 1); issue(2, 1); issue(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    bar();
    if (grp == 1) bar();  // stagger: group 1 runs one barrier behind group 0
    for (int kt = 0; kt < nk; ++kt) {
        // phase A: A0 x B0 of K-step kt; K-step kt + 2's A0 / B0 into the stage kt - 1 used
        read_a(kt, 0); read_b(kt);
        issue(0, kt + 2); issue(2, kt + 2);
        asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // K-step kt's A1 has landed
        bar(); mfma_q(0); bar();
        // phase B: A1 x B0 (B fragments from registers); K-step kt + 2's A1
        read_a(kt, 1);
        issue(1, kt + 2);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // K-step kt + 1's A0 / B0 have landed
        bar(); mfma_q(1); bar();
    }
    if (grp == 0) bar();  // equal barrier counts: every wave's LDS reads are done
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- epilogue: scores (database row c, query p) -> kNN screen or the f32 slab
    float* __restrict__ Y = (float*)a.y;
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = c0 + qa * 128 + grp * 64 + i * 16 + 4 * kq;
            if (c >= a.cout) continue;
            const bool full = c + 3 < a.cout;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int p = wn * 32 + j * 16 + r16;
                if (p >= a.P) continue;
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = acc[qa][i][j][r];
                if (a.scr_k) {  // kNN screen: append survivors, store nothing
                    screen_append(a, v, c, a.cout, p, a.scr_tau[p]);
                    continue;
                }
                const long long o = (long long)p * a.ldy + c;
                if (full) {
                    St4<float>::st(Y + o, v);
                } else {
                    for (int r = 0; r < 4; ++r)
                        if (c + r < a.cout) Y[o + r] = v[r];
                }
            }
        }
}

// ---------------------------------------------------------------------------
// Streaming form of the <= 128-query kNN score GEMM (k_gemm8s).  At 128 queries
// a DB byte feeds only 128 MACs, so k_gemm8h is bound by how many DB bytes it
// keeps in flight, and its LDS ring (3 stages x 48 KiB) gives a DMA only about
// two K-steps (~1 us) to land.  Here the DB rows bypass LDS: each wave owns 32
// rows of a 256-row tile and loads their A fragments straight into registers,
// R K-steps ahead (R x 4 KiB per wave, 8 x R x 4 KiB per CU in flight); only the
// queries -- shared by all 8 waves -- go through an LDS ring of R + 1 K-steps
// (16 KiB each, LDS-DMA).  Blocks are persistent over an XCD-contiguous tile
// range and the K-step stream runs on across tiles, so the next tile's rows are
// already in flight during a tile's epilogue.  Per element the MFMA operands, K
// order and accumulation order are k_gemm8h's (16x16x32, K-steps in order, the
// two 32-deep halves in order), so the scores -- and k_slot_fixup's recomputed
// keys -- are bit-identical to it.
// vmcnt: per stream position the block issues 2 query DMAs (asm, not counted
// by the compiler) and then 4 DB loads (compiler-visible); position f's query
// stage is complete once at most 6 (R - 1) + 4 younger operations remain.
// T = int8_t: int8-quantised rows on v_mfma_i32_16x16x64_i8 (see k_gemm8): the same
// 128-B K-steps carry 128 elements, accumulators are exact int32, scores float(acc).
template <typename T, int R>
__global__ void __launch_bounds__(512, 1) k_gemm8s(ConvArgs a, int ntiles) {
    constexpr bool I8 = std::is_same<T, int8_t>::value;
    static_assert((sizeof(T) == 2 || I8) && 6 * (R - 1) + 4 <= 63, "16-bit / int8 operands, vmcnt range");
    constexpr int ESZ = sizeof(T), VEC = 16 / ESZ, HT = 16384, NB = R + 1;
    // query stages + the queries' thresholds (<= 128) + 8 survivor lists (ScreenStage)
    __shared__ __attribute__((aligned(1024))) char smem[NB * HT + 4 * (128 + 8 * 3 * ScreenStage::CAP)];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwg = (int)gridDim.x, bx = (int)blockIdx.x, xcd = bx & 7;
    const int nt8 = ntiles >> 3, rt8 = ntiles & 7;
    const int s_x = xcd < rt8 ? xcd * (nt8 + 1) : rt8 * (nt8 + 1) + (xcd - rt8) * nt8;
    const int n_x = nt8 + (xcd < rt8 ? 1 : 0);
    const int nb_x = (nwg >> 3) + (xcd < (nwg & 7) ? 1 : 0);
    const int li = bx >> 3;
    if (li >= n_x) return;
    const int my = (n_x - li + nb_x - 1) / nb_x;  // tiles of this block: s_x + li + m * nb_x
    const int nk = a.kp * ESZ / 128;
    const int F = my * nk;                        // (tile, K-step) stream of this block
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    const int lrow = lane >> 3, lchunk = (lane & 7) ^ (lrow & 7);
    const int r16 = lane & 15, kq = lane >> 4;

    const i32x4_t rsB = make_rsrc(a.x, (unsigned)((long long)a.P * a.cin * ESZ));
    unsigned b_off[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int p = (wave + 8 * i) * 8 + lrow;
        b_off[i] = p < a.P ? (unsigned)(((long long)p * a.cin + lchunk * VEC) * ESZ) : OOB;
    }
    uint32_t* const lds_tau = reinterpret_cast<uint32_t*>(smem + NB * HT);
    uint32_t* const lds_stage = lds_tau + 128;
    if (a.scr_k) {
        for (int q = tid; q < a.P; q += 512) lds_tau[q] = a.scr_tau[q];
        // visible to every wave before any epilogue reads it: with one K-step per
        // tile (D = 64) the first epilogue comes before a second block barrier
        __syncthreads();
    }
    // issue side: stream position (mi, ki); this lane's two DB rows of tile mi
    // (positions past the block's stream re-read its last tile: same count of
    // operations in flight, results unused)
    int mi = 0, ki = 0;
    const char* arow[2];
    auto set_rows = [&](int m) {
        const int t = s_x + li + min(m, my - 1) * nb_x;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const int row = min(t * 256 + 32 * wave + 16 * g + r16, a.cout - 1);
            arow[g] = (const char*)a.w + (long long)row * a.kp * ESZ + kq * 16;
        }
    };
    set_rows(0);
    uint4 ar[R][2][2];  // [ring slot][row group][32-deep half]
    int bst = 0;        // query stage of the next issue
    auto issue = [&](uint4 (&dst)[2][2]) {
        const bool live = mi < my;
        const unsigned dstl = lds0 + bst * HT;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            dma16(rsB, (live && b_off[i] != OOB) ? b_off[i] + (unsigned)(ki * 128) : OOB, dstl + (wave + 8 * i) * 1024);
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int hs = 0; hs < 2; ++hs)
                dst[g][hs] = *reinterpret_cast<const uint4*>(arow[g] + ki * 128 + hs * 64);
        bst = bst + 1 == NB ? 0 : bst + 1;
        if (++ki == nk) {
            ki = 0;
            ++mi;
            set_rows(mi);
        }
    };
#pragma unroll
    for (int u = 0; u < R; ++u) issue(ar[u]);

    f32x4_t acc[2][8];
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[g][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    int cst = 0;     // query stage of the position being consumed
    int m = 0, kc = 0;
    for (int f0 = 0; f0 < F; f0 += R) {
#pragma unroll
        for (int u = 0; u < R; ++u) {
            if (f0 + u >= F) break;
            // this position's query stage has landed (6 (R - 1) + 4 younger ops) in
            // every wave, and every wave has read the stage the next DMA overwrites
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(6 * (R - 1) + 4) : "memory");
            const char* Bs = smem + cst * HT;
            cst = cst + 1 == NB ? 0 : cst + 1;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                uint4 fb[2];
#pragma unroll
                for (int hs = 0; hs < 2; ++hs)
                    fb[hs] = *reinterpret_cast<const uint4*>(Bs + swz(j * 16 + r16, kq + 4 * hs));
#pragma unroll
                for (int hs = 0; hs < 2; ++hs)
#pragma unroll
                    for (int g = 0; g < 2; ++g) {
                        if constexpr (I8)
                            acc[g][j] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_mfma_i32_16x16x64_i8(
                                __builtin_bit_cast(i32x4_t, ar[u][g][hs]), __builtin_bit_cast(i32x4_t, fb[hs]),
                                __builtin_bit_cast(i32x4_t, acc[g][j]), 0, 0, 0));
                        else if constexpr (std::is_same<T, f16_t>::value)
                            acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                                __builtin_bit_cast(f16x8_t, ar[u][g][hs]), __builtin_bit_cast(f16x8_t, fb[hs]),
                                acc[g][j], 0, 0, 0);
                        else
                            acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                __builtin_bit_cast(bf16x8_t, ar[u][g][hs]), __builtin_bit_cast(bf16x8_t, fb[hs]),
                                acc[g][j], 0, 0, 0);
                    }
            }
            issue(ar[u]);  // position f + R into the ring slot just consumed
            if (++kc == nk) {
                // ---- tile epilogue: scores (database row c + r, query p)
                const int c0 = (s_x + li + m * nb_x) * 256;
                float* __restrict__ Y = (float*)a.y;
                if (a.scr_k) {  // stage the survivors, append them in batches (full-wave control flow)
                    ScreenStage st{lds_stage + wave * 3 * ScreenStage::CAP, 0};
#pragma unroll
                    for (int g = 0; g < 2; ++g)
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const int p = j * 16 + r16;
                            const bool ok = p < a.P;
                            float v[4];
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                v[r] = I8 ? (float)__builtin_bit_cast(i32x4_t, acc[g][j])[r] : acc[g][j][r];
                            st.add(a, v, c0 + 32 * wave + 16 * g + 4 * kq, a.cout, p, ok, ok ? lds_tau[p] : 0xffffffffu);
                        }
                    st.flush(a);
                }
#pragma unroll
                for (int g = 0; g < 2 && !a.scr_k; ++g) {
                    const int c = c0 + 32 * wave + 16 * g + 4 * kq;
                    if (c >= a.cout) continue;
                    const bool full = c + 3 < a.cout;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int p = j * 16 + r16;
                        if (p >= a.P) continue;
                        float v[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            v[r] = I8 ? (float)__builtin_bit_cast(i32x4_t, acc[g][j])[r] : acc[g][j][r];
                        acc[g][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
                        const long long o = (long long)p * a.ldy + c;
                        if (full) {
                            St4<float>::st(Y + o, v);
                        } else {
                            for (int r = 0; r < 4; ++r)
                                if (c + r < a.cout) Y[o + r] = v[r];
                        }
                    }
                }
#pragma unroll
                for (int g = 0; g < 2; ++g)
#pragma unroll
                    for (int j = 0; j < 8; ++j) acc[g][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
                kc = 0;
                ++m;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing positions' operations
}

// ---------------------------------------------------------------------------
// The mirror of k_gemm8h for 128-channel convs (auto: the strided mod3 3x3,
// 699 vs 775 us on k_igemm at 128 images; the stride-1 mod3 3x3 stays on the
// direct k_conv3x3, 550 vs 664 us on this kernel):
// a 128 (output channels, A) x 256 (pixels, B) tile, phases A0 x B0 and
// A0 x B1 (the A fragments stay in registers for the second), the same
// 3-stage {A0, B0, B1} ring / issue distances / counted waits, k_gemm8's
// operand-B addressing (1x1 or tap-uniform im2col) and PERM32 epilogue
// (folded BN, residual, activation, one 16-B store per fragment pair).
template <typename T, int KM>
__global__ void __launch_bounds__(512, 1) k_gemm8a(ConvArgs a, int tiles_p, int ntiles) {
    static_assert(sizeof(T) == 2, "16-bit operands");
    constexpr bool K1 = KM == 1, tapu = KM == 2;
    constexpr int VEC = 8, ESZ = 2, HT = 16384, ST = 3 * HT;  // stage = [A0, B0, B1]
    __shared__ __attribute__((aligned(1024))) char smem[3 * ST];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wn = wave & 3;
    // persistent blocks over an XCD-contiguous tile range (k_gemm8's walk): XCD x owns
    // [s_x, s_x + n_x), its nb_x blocks stride through it; grid = ntiles is one tile per block
    const int nwg = (int)gridDim.x, bx = (int)blockIdx.x, xcd = bx & 7;
    const int nt8 = ntiles >> 3, rt8 = ntiles & 7;
    const int s_x = xcd < rt8 ? xcd * (nt8 + 1) : rt8 * (nt8 + 1) + (xcd - rt8) * nt8;
    const int n_x = nt8 + (xcd < rt8 ? 1 : 0);
    const int nb_x = (nwg >> 3) + (xcd < (nwg & 7) ? 1 : 0);
    int li = bx >> 3;
    if (li >= n_x) return;
    const int H = a.h, W = a.w_, Cin = a.cin;
    const unsigned tap_magic = tapu_magic(a.kh * a.kw);  // tapu_k0
    const int nk = a.kp / 64;
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    const int lrow = lane >> 3, lchunk = (lane & 7) ^ (lrow & 7);
    const int r16 = lane & 15, kq = lane >> 4;

    // c_out = 128 (gemm8a_eligible): one channel tile, so this lane's 2 x 8 BN scale / shift
    // stay in registers for every tile (the epilogue issues no global load: a load there
    // would wait, vmcnt being in order, for the next tile's prologue DMA)
    const bool affine = a.flags & RR_CONV_AFFINE;
    float esc[2][8], esh[2][8];
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2) {
        const int c = grp * 64 + 32 * i2 + 8 * kq;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            esc[i2][r] = affine ? a.scale[c + r] : 1.f;
            esh[i2][r] = affine ? a.shift[c + r] : 0.f;
        }
    }
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(esc[i2][r]), "+v"(esh[i2][r]));

    int p0 = 0;
    const i32x4_t rsA = make_rsrc((const char*)a.w, (unsigned)(128ll * a.kp * ESZ));
    const i32x4_t rsB = make_rsrc(a.x, (unsigned)((long long)a.n * H * W * Cin * ESZ));
    unsigned a_off[2], b_base[2][2];
    int b_hi[2][2], b_wi[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int arow = (wave + 8 * i) * 8 + lrow;
        a_off[i] = (unsigned)(((long long)arow * a.kp + lchunk * VEC) * ESZ);
    }
    auto setup = [&](int t) {
        p0 = t * 256;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int p = p0 + h * 128 + (wave + 8 * i) * 8 + lrow;
                if (p < a.P) {
                    const int img = p / (a.ho * a.wo);
                    const int rem = p - img * (a.ho * a.wo);
                    const int oh = rem / a.wo, ow = rem - oh * a.wo;
                    b_hi[h][i] = oh * a.stride - a.pad;
                    b_wi[h][i] = ow * a.stride - a.pad;
                    b_base[h][i] = (unsigned)((long long)img * H * W * Cin +
                                              ((long long)b_hi[h][i] * W + b_wi[h][i]) * Cin + lchunk * VEC);
                } else {
                    b_hi[h][i] = b_wi[h][i] = -(1 << 28);
                    b_base[h][i] = OOB;
                }
            }
    };
    setup(s_x + li);
    // K-step descriptor, once per K-step (k_gemm8's KD: no division on the issue path)
    const unsigned kw_magic = tapu_magic(a.kw);
    struct KD {
        int k0, dh, dw, add, stage;
        bool live;
    };
    auto kdesc = [&](int kt) {
        KD d;
        d.live = kt < nk;
        d.stage = kt % 3;
        d.k0 = tapu ? tapu_k0(kt, a.kh * a.kw, tap_magic, Cin >> 6, Cin, 64) : kt * 64;
        d.dh = d.dw = d.add = 0;
        if constexpr (tapu) {
            const int tap = d.k0 >> a.lc, ci0 = d.k0 & (Cin - 1);
            const int kh = (int)(((unsigned)tap * kw_magic) >> 16), kw = tap - kh * a.kw;
            d.dh = kh * a.dil;
            d.dw = kw * a.dil;
            d.add = (d.dh * W + d.dw) * Cin + ci0;
        }
        return d;
    };
    // half-tile X (0 A0, 1 B0, 2 B1) of K-step d into its ring stage; K-steps >= nk load zeros
    auto issue = [&](int X, const KD& d) {
        const unsigned dst = lds0 + d.stage * ST + X * HT;
        if (X == 0) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const unsigned off = d.live ? a_off[i] + (unsigned)(d.k0 * 2) : OOB;
                dma16(rsA, off, dst + (wave + 8 * i) * 1024);
            }
        } else {
            const int h = X - 1;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                unsigned off = OOB;
                if (d.live && b_base[h][i] != OOB) {
                    if constexpr (K1) {
                        off = (b_base[h][i] + (unsigned)d.k0) * ESZ;
                    } else {
                        const int hi = b_hi[h][i] + d.dh, wi = b_wi[h][i] + d.dw;
                        if ((unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W)
                            off = (b_base[h][i] + (unsigned)d.add) * ESZ;
                    }
                }
                dma16(rsB, off, dst + (wave + 8 * i) * 1024);
            }
        }
    };

    f32x4_t acc[2][4][2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[qb][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    uint4 fa[4][2], fb[2][2];
    auto read_a = [&](int kt) {
        const char* base = smem + (kt % 3) * ST;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int hs = 0; hs < 2; ++hs)
                fa[i][hs] = *reinterpret_cast<const uint4*>(base + swz(grp * 64 + i * 16 + r16, kq + 4 * hs));
    };
    auto read_b = [&](int kt, int h) {
        const char* base = smem + (kt % 3) * ST + (1 + h) * HT;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int hs = 0; hs < 2; ++hs)
                fb[j][hs] = *reinterpret_cast<const uint4*>(base + swz(wn * 32 + j * 16 + r16, kq + 4 * hs));
    };
    auto mfma_q = [&](int qb) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int hs = 0; hs < 2; ++hs)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if constexpr (std::is_same<T, f16_t>::value)
                        acc[qb][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                            __builtin_bit_cast(f16x8_t, fa[i][hs]), __builtin_bit_cast(f16x8_t, fb[j][hs]),
                            acc[qb][i][j], 0, 0, 0);
                    else
                        acc[qb][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8_t, fa[i][hs]), __builtin_bit_cast(bf16x8_t, fb[j][hs]),
                            acc[qb][i][j], 0, 0, 0);
                }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto bar = []() { asm volatile("s_barrier" ::: "memory"); };
    auto prologue = [&]() {
        const KD d0 = kdesc(0), d1 = kdesc(1);
        issue(0, d0); issue(1, d0); issue(2, d0);
        issue(0, d1); issue(1, d1); issue(2, d1);
    };

    T* __restrict__ Y = (T*)a.y;
    const T* __restrict__ R = (const T*)a.res;
    const bool resid = a.flags & RR_CONV_RESIDUAL;
    const bool leaky = a.act == RR_ACT_LEAKY;
    prologue();
    // the previous tile's epilogue issued exactly ST_FULL stores and nothing else (a full
    // tile, no residual load); they are younger than this tile's prologue
    constexpr int ST_FULL = 8;
    bool prev_full = false;
    for (;;) {
        // K-step 0's A0 / B0 have landed: younger are its B1, K-step 1 (8) and the
        // previous tile's epilogue stores; an epilogue with loads / fewer stores is
        // waited for with it
        if (prev_full) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // 8 + ST_FULL
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        static_assert(8 + ST_FULL == 16, "the counted wait above");
        bar();
        if (grp == 1) bar();
        for (int kt = 0; kt < nk; ++kt) {
            const KD d2 = kdesc(kt + 2);
            // phase A: A0 x B0 of K-step kt; K-step kt + 2's A0 / B0
            read_a(kt); read_b(kt, 0);
            issue(0, d2); issue(1, d2);
            asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // K-step kt's B1 has landed
            bar(); mfma_q(0); bar();
            // phase B: A0 (registers) x B1; K-step kt + 2's B1
            read_b(kt, 1);
            issue(2, d2);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // K-step kt + 1's A0 / B0 have landed
            bar(); mfma_q(1); bar();
        }
        if (grp == 0) bar();  // equal barrier counts: every wave's LDS reads of this tile are done
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing (zero) K-step DMAs have landed

        // the next tile's prologue DMA flies while this tile's epilogue runs
        const int ep0 = p0;
        li += nb_x;
        const bool more = li < n_x;
        if (more) {
            setup(s_x + li);
            prologue();
        }
        prev_full = !resid && ep0 + 256 <= a.P;
        // ---- epilogue (PERM32 rows): folded BN scale / shift, residual, activation, NHWC store
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2) {
            const int c = grp * 64 + 32 * i2 + 8 * kq;  // 8 consecutive channels
#pragma unroll
            for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int p = ep0 + qb * 128 + wn * 32 + j * 16 + r16;
                    if (p >= a.P) continue;
                    float v[8];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] = acc[qb][2 * i2][j][r] * esc[i2][r] + esh[i2][r];
                        v[4 + r] = acc[qb][2 * i2 + 1][j][r] * esc[i2][4 + r] + esh[i2][4 + r];
                    }
                    const long long o = (long long)p * a.ldy + c;
                    if (resid) {
                        float rv[8];
                        St4<T>::ld(R + o, rv);
                        St4<T>::ld(R + o + 4, rv + 4);
#pragma unroll
                        for (int r = 0; r < 8; ++r) v[r] += rv[r];
                    }
                    if (leaky) {
#pragma unroll
                        for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
                    }
                    uint4 q;
                    q.x = H16<T>::pack2(v[0], v[1]);
                    q.y = H16<T>::pack2(v[2], v[3]);
                    q.z = H16<T>::pack2(v[4], v[5]);
                    q.w = H16<T>::pack2(v[6], v[7]);
                    *reinterpret_cast<uint4*>(Y + o) = q;
                }
        }
        if (!more) break;
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[qb][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

static int g_gemm8 = -1;  // rr_set_tuning(RR_TUNE_GEMM8) / RR_GEMM8: 0 off, 1 auto (default), 2 force where legal
static bool g_gemm8_tile = false;  // RR_TUNE_GEMM8 value | 4: one block per tile instead of persistent blocks
static bool g_gemm8_pmajor = true;  // RR_TUNE_GEMM8 value | 64: conv tiles channel-major
static bool g_gemm8_short_persist = true;  // RR_TUNE_GEMM8 value | 512: short-K 1x1 convs one block per tile

// 16-bit operands, 1x1 or tap-uniform im2col, an even number of 64-deep
// K-steps, 31-bit operand offsets, and (auto) enough 256 x 256 tiles to fill
// the chip twice with no half-empty channel tile (c_out = 128 would waste
// half the MFMAs).
bool gemm8_eligible(const ConvArgs& a, bool k1, int esz) {
    if (g_gemm8 < 0) {
        const char* e = getenv("RR_GEMM8");
        g_gemm8 = (e && e[0] == '0') ? 0 : 1;
    }
    if (!g_gemm8 || esz != 2) return false;
    const int km = k1 ? 1 : ((a.cin * 2) % 128 == 0 && tapu_ok(a.kh * a.kw, a.kp / 64)) ? 2 : 0;
    const int nk = a.kp / 64;
    if (km == 0 || nk < 2 || (nk & 1) || a.kp % 64) return false;
    if ((long long)a.n * a.h * a.w_ * a.cin * 2 >= (1ll << 31) || 256ll * a.kp * 2 >= (1ll << 31)) return false;
    if ((a.flags & RR_CONV_PERM32) && a.cout % 32) return false;
    const long long ntiles = (long long)((a.P + 255) / 256) * ((a.cout + 255) / 256);
    // (a partial last channel tile is negligible for long channel dims, e.g. the
    // database rows of the kNN score GEMM)
    if (g_gemm8 == 1 && (a.P < 256 || ntiles < 2 * grid_cus() || (a.cout % 256 && a.cout < 4096))) return false;
    return true;
}

template <typename T, typename TO>
static bool try_gemm8(const ConvArgs& a, bool k1, bool perm, hipStream_t s) {
    if constexpr (sizeof(T) != 2) {
        return false;
    } else {
        if (!gemm8_eligible(a, k1, 2)) return false;
        const int km = k1 ? 1 : 2;
        const int tiles_p = (a.P + 255) / 256, tiles_c = (a.cout + 255) / 256;
        const long long ntiles = (long long)tiles_p * tiles_c;
        // persistent blocks (one per CU walks its XCD's tile range, the next tile's
        // prologue DMA overlapping this tile's epilogue) for the kNN score GEMM
        // (Q = 1024: 5.386 / 5.390 -> 5.356 / 5.339 ms, same-box A/B); one block per
        // tile for the convs, where persistence measured -0.3 % on the body
        // (25.69 / 25.73 vs 25.77 / 26.13 ms).  RR_TUNE_GEMM8 = 2 forces persistence
        // everywhere, | 4 forces one block per tile.
        const long long cus = grid_cus();
        // Short-K 1x1 convs without a residual (<= 16 K-steps per tile) are persistent
        // too: their epilogue reads BN scale / shift from LDS and its stores are counted
        // into the next tile's first wait, so the next prologue lands under the epilogue
        // (128 x R50 layers, same box: K = 512 540 -> 521 / 579 -> 552 us, K = 1024
        // neutral to -8 us; K = 2048 and the 3x3s measured slower, so they stay one block
        // per tile).
        const bool short_k1 = g_gemm8_short_persist && k1 && a.kp / 64 <= 16 && !(a.flags & RR_CONV_RESIDUAL);
        const bool persist = !g_gemm8_tile && (g_gemm8 == 2 || !std::is_same<T, TO>::value ||
                                               (std::is_same<T, TO>::value && short_k1));
        // (a grid below 8 blocks would leave some XCD's tile range without a block)
        const dim3 g((unsigned)(!persist || cus < 8 || ntiles < cus ? ntiles : cus)), b(512);
        // conv GEMMs (16-bit out) walk their tiles pixel-major (RR_TUNE_GEMM8 | 64: channel-major)
        const int pmajor = std::is_same<T, TO>::value && g_gemm8_pmajor && tiles_c > 1;
#define RR_G8(KMV, PV) hipLaunchKernelGGL((k_gemm8<T, TO, KMV, PV>), g, b, 0, s, a, tiles_p, (int)ntiles, pmajor)
        if constexpr (std::is_same<T, TO>::value) {
            if (perm) {
                if (km == 1) RR_G8(1, true);
                else RR_G8(2, true);
                return true;
            }
        }
        if (km == 1) RR_G8(1, false);
        else RR_G8(2, false);
#undef RR_G8
        return true;
    }
}

static int g_gemm8h = 1;  // rr_set_tuning(RR_TUNE_GEMM8, value | 8): k_gemm8h off
static int g_gemm8s = 1;  // rr_set_tuning(RR_TUNE_GEMM8, value | 32): k_gemm8h instead of k_gemm8s

// k_gemm8h: 16-bit 1x1 score GEMM (float out, natural row order, no affine /
// residual / activation) with <= 128 "pixels" (queries), long channel dim.
template <typename T, typename TO>
static bool try_gemm8h(const ConvArgs& a, bool k1, bool perm, hipStream_t s) {
    if constexpr (sizeof(T) != 2 || !std::is_same<TO, float>::value) {
        return false;
    } else {
        if (!g_gemm8h || !k1 || perm || a.kp % 64 || a.kp != a.cin || a.kp / 64 < 2) return false;
        if (a.flags & (RR_CONV_AFFINE | RR_CONV_RESIDUAL) || a.act != RR_ACT_IDENTITY) return false;
        if (a.P < 1 || a.P > 128 || (long long)a.P * a.cin * 2 >= (1ll << 31) || 256ll * a.kp * 2 >= (1ll << 31))
            return false;
        const long long ntiles = ((long long)a.cout + 255) / 256;
        if (ntiles >= (1ll << 31)) return false;
        if (g_gemm8s) {
            // persistent streaming form: one block per CU (a grid below 8 blocks
            // would leave some XCD's tile range without a block)
            const long long cus = grid_cus();
            const unsigned g = (unsigned)(cus < 8 || ntiles < cus ? ntiles : cus);
            // K-steps in flight per wave: 4 (Q = 128 vs 1M rows: 1.13 / 1.12 ms vs 1.15 / 1.14 at 6,
            // 1.28 at 8, profiles/r03_ab/r03ac_gemm8s_depth_ab.txt); RR_GEMM8S_R = 3 or 6: A/B
            static const int rdepth = getenv("RR_GEMM8S_R") ? atoi(getenv("RR_GEMM8S_R")) : 4;
            if (rdepth == 6)
                hipLaunchKernelGGL((k_gemm8s<T, 6>), dim3(g), dim3(512), 0, s, a, (int)ntiles);
            else if (rdepth == 3)
                hipLaunchKernelGGL((k_gemm8s<T, 3>), dim3(g), dim3(512), 0, s, a, (int)ntiles);
            else
                hipLaunchKernelGGL((k_gemm8s<T, 4>), dim3(g), dim3(512), 0, s, a, (int)ntiles);
        } else {
            hipLaunchKernelGGL((k_gemm8h<T>), dim3((unsigned)ntiles), dim3(512), 0, s, a, (int)ntiles);
        }
        return true;
    }
}

static int g_gemm8a = 1;  // rr_set_tuning(RR_TUNE_GEMM8, value | 16): k_gemm8a off
static bool g_gemm8a_tile = false;  // RR_TUNE_GEMM8 value | 128: k_gemm8a one block per tile

// k_gemm8a: 16-bit PERM32 convs with 128-multiple c_out below 256 (1x1 or
// tap-uniform im2col), enough 128 x 256 tiles to fill the chip twice.
bool gemm8a_eligible(const ConvArgs& a, bool k1) {
    if (!g_gemm8a || !(a.flags & RR_CONV_PERM32) || a.cout % 128 || a.cout >= 256) return false;
    const int km = k1 ? 1 : ((a.cin * 2) % 128 == 0 && tapu_ok(a.kh * a.kw, a.kp / 64)) ? 2 : 0;
    if (km == 0 || a.kp % 64 || a.kp / 64 < 2) return false;
    if ((long long)a.n * a.h * a.w_ * a.cin * 2 >= (1ll << 31) || 128ll * a.kp * 2 >= (1ll << 31)) return false;
    const long long ntiles = (long long)((a.P + 255) / 256) * (a.cout / 128);
    return ntiles >= 2 * grid_cus() && ntiles < (1ll << 31);
}

template <typename T, typename TO>
static bool try_gemm8a(const ConvArgs& a, bool k1, bool perm, hipStream_t s) {
    if constexpr (sizeof(T) != 2 || !std::is_same<T, TO>::value) {
        return false;
    } else {
        if (!perm || !gemm8a_eligible(a, k1)) return false;
        const int tiles_p = (a.P + 255) / 256;
        const int ntiles = tiles_p;  // c_out = 128: one channel tile
        // persistent (RR_TUNE_GEMM8 value | 128: one block per tile)
        // (a grid below 8 blocks would leave some XCD's tile range without a block)
        const int cus = grid_cus();
        const int grid = g_gemm8a_tile || cus < 8 || ntiles < cus ? ntiles : cus;
        if (k1) hipLaunchKernelGGL((k_gemm8a<T, 1>), dim3(grid), dim3(512), 0, s, a, tiles_p, ntiles);
        else hipLaunchKernelGGL((k_gemm8a<T, 2>), dim3(grid), dim3(512), 0, s, a, tiles_p, ntiles);
        return true;
    }
}

// kNN score GEMM on int8-quantised rows (float scores = exact int32 dot products):
// k_gemm8s at <= 128 queries (streaming the database), persistent k_gemm8 above.
// Needs 128-B K-steps (d % 128 == 0) and, for k_gemm8, an even K-step count.
int gemm_scores_i8(const ConvArgs& a, hipStream_t s) {
    if (a.kp != a.cin || a.kp % 128 || a.P < 1 || (long long)a.P * a.cin >= (1ll << 31) ||
        256ll * a.kp >= (1ll << 31))
        return fail(RR_EINVAL, "int8 score GEMM: d must be a multiple of 128 (rows and queries below 2 GiB)");
    const long long cus = grid_cus();
    if (a.P <= 128) {
        const long long ntiles = ((long long)a.cout + 255) / 256;
        const unsigned g = (unsigned)(cus < 8 || ntiles < cus ? ntiles : cus);
        hipLaunchKernelGGL((k_gemm8s<int8_t, 4>), dim3(g), dim3(512), 0, s, a, (int)ntiles);
        return RR_OK;
    }
    if ((a.kp / 128) & 1) return fail(RR_EINVAL, "int8 score GEMM above 128 queries: d must be a multiple of 256");
    const int tiles_p = (a.P + 255) / 256;
    const long long ntiles = (long long)tiles_p * ((a.cout + 255) / 256);
    if (ntiles >= (1ll << 31)) return fail(RR_EINVAL, "int8 score GEMM: too many tiles");
    const dim3 g((unsigned)(cus < 8 || ntiles < cus ? ntiles : cus));
    hipLaunchKernelGGL((k_gemm8<int8_t, float, 1, false>), g, dim3(512), 0, s, a, tiles_p, (int)ntiles, 0);
    return RR_OK;
}

int g_force_cfg = 0;  // rr_set_tuning(RR_TUNE_GEMM_CONFIG, ...)

template <typename T, typename TO>
void launch_gemm2(const ConvArgs& a, bool k1, hipStream_t s) {
    const bool perm = (a.flags & RR_CONV_PERM32) != 0;
    const bool resid = (a.flags & RR_CONV_RESIDUAL) != 0;
    num_cus();
    switch (g_force_cfg) {
        case 1: launch_cfg3<T, TO, 128, 128, 2, 2>(a, k1, perm, s); return;
        case 2: launch_cfg3<T, TO, 64, 256, 1, 4>(a, k1, perm, s); return;
        case 3: launch_cfg3<T, TO, 256, 128, 4, 2>(a, k1, perm, s); return;
        case 4: launch_cfg3<T, TO, 256, 256, 4, 2>(a, k1, perm, s); return;
        case 5: launch_cfg3<T, TO, 256, 64, 4, 1>(a, k1, perm, s); return;
        case 7: launch_ns<T, TO, 256, 128, 4, 2, 3>(a, k1, perm, s); return;  // 8 waves, 3-stage ring (144 KiB)
        case 8: launch_ns<T, TO, 128, 256, 2, 4, 3>(a, k1, perm, s); return;  // 8 waves, 3-stage ring (144 KiB)
        default: break;
    }
    if (g_force_cfg == 0 && try_gemm8<T, TO>(a, k1, perm, s)) return;
    if (g_force_cfg == 0 && try_gemm8a<T, TO>(a, k1, perm, s)) return;
    // A-stationary variants (single output-channel tile, short K)
    const int nk = a.kp / (sizeof(T) == 2 ? 64 : 32);
    if (g_force_cfg == 6 || (g_force_cfg == 0 && g_ast)) {
        if (a.cout > 128 && a.cout <= 256 && nk <= 1 && a.P > 64) {
            launch_ns<T, TO, 256, 64, 4, 1, 2, 1>(a, k1, perm, s);
            return;
        }
    }
    // Automatic choice (per-shape sweep, tools/tune_layers.py, R50 @ 32 x 768x1024):
    //  * small P: one row of pixel tiles, channel-wide
    //  * c_out = 64: 64x256; c_out = 128: 128x128
    //  * residual 1x1 into 256 channels with one K-step: A-stationary 256x64
    //  * residual, K < 512: 256x128 (8 waves); everything else >= 256 channels: 256x256 (8 waves)
    if (a.P <= 32)
        launch_cfg3<T, TO, 256, 32, 4, 1>(a, k1, perm, s);
    else if (a.P <= 64)
        launch_cfg3<T, TO, 256, 64, 4, 1>(a, k1, perm, s);
    else if (a.P <= 128 && a.cout >= 4096 && try_gemm8h<T, TO>(a, k1, perm, s))  // kNN score GEMM at 65..128 queries
        return;
    else if (a.P <= 128 && a.cout >= 4096)  // kNN score GEMM at 65..128 queries: no half-empty 256-wide pixel tiles;
        // 128 x 128 (4 waves, 64 KiB: two blocks per CU) measured 1.296 / 1.306 vs 1.328 / 1.335 ms for the
        // Q = 128 search against 1M x 2048 with 256 x 128 (tools/knn_cfg_ab.sh)
        launch_cfg3<T, TO, 128, 128, 2, 2>(a, k1, perm, s);
    else if (a.cout <= 64)
        launch_cfg3<T, TO, 64, 256, 1, 4>(a, k1, perm, s);
    else if (a.cout <= 128 || !g_wide)
        launch_cfg3<T, TO, 128, 128, 2, 2>(a, k1, perm, s);
    else if (resid && a.cout <= 256 && nk <= 1)
        launch_ns<T, TO, 256, 64, 4, 1, 2, 1>(a, k1, perm, s);
    else if (resid && a.kp < 512)
        launch_cfg3<T, TO, 256, 128, 4, 2>(a, k1, perm, s);
    else if (resid && a.cout >= 2048 && a.P >= 65536)  // mod5 conv3 at >= 64 images: 256x64 tiles, -13 % (tune_layers)
        launch_cfg3<T, TO, 256, 64, 4, 1>(a, k1, perm, s);
    else
        launch_cfg3<T, TO, 256, 256, 4, 2>(a, k1, perm, s);
}

void set_gemm_tuning(int key, int value) {
    num_cus();
    if (key == RR_TUNE_GEMM_CONFIG) g_force_cfg = value;
    else if (key == RR_TUNE_GEMM_STAGES) g_stages = value == 3 ? 3 : 2;
    else if (key == RR_TUNE_GEMM_WIDE) g_wide = value != 0;
    else if (key == RR_TUNE_GEMM_ASTAT) g_ast = value != 0;
    else if (key == RR_TUNE_GEMM_XCD_MAP) g_xmap = value != 0;
    else if (key == RR_TUNE_GEMM8) {
        g_gemm8h = !(value >= 0 && (value & 8));
        g_gemm8a = !(value >= 0 && (value & 16));
        g_gemm8s = !(value >= 0 && (value & 32));
        g_gemm8_tile = value >= 0 && (value & 4);
        g_gemm8_pmajor = !(value >= 0 && (value & 64));
        g_gemm8_short_persist = !(value >= 0 && (value & 512));
        g_gemm8a_tile = value >= 0 && (value & 128);
        value = value < 0 ? 0 : value & 3;
        g_gemm8 = value > 2 ? 2 : value;
    }
}

template void launch_gemm2<bf16_t, bf16_t>(const ConvArgs&, bool, hipStream_t);
template void launch_gemm2<bf16_t, float>(const ConvArgs&, bool, hipStream_t);
template void launch_gemm2<f16_t, float>(const ConvArgs&, bool, hipStream_t);
template void launch_gemm2<f16_t, f16_t>(const ConvArgs&, bool, hipStream_t);
template void launch_gemm2<float, float>(const ConvArgs&, bool, hipStream_t);

}  // namespace rr
