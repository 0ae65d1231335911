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
        "s_nop 4\n\t"
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
        const int k0 = is_k * BK;
        const unsigned As = lds0 + stage * STAGE;
        const unsigned Bs = AK ? lds0 + ABYTES + stage * STAGE : As + TC * 128;
        if constexpr (AK > 0) {
            if (is_tile == 0 && is_k == 0) {  // whole weight slice, once per block
                for (int kk = 0; kk < nk; ++kk)
#pragma unroll
                    for (int i = 0; i < NIA; ++i) {
                        const unsigned off = a_off[i] == OOB ? OOB : a_off[i] + (unsigned)(kk * BK * ESZ);
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
    const int km = k1 ? 1 : (a.cin * (int)sizeof(T)) % 128 == 0 ? 2 : 0;
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
    else if (a.P <= 128 && a.cout >= 4096)  // kNN score GEMM at 65..128 queries: no half-empty 256-wide pixel tiles
        launch_cfg3<T, TO, 256, 128, 4, 2>(a, k1, perm, s);
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
}

template void launch_gemm2<bf16_t, bf16_t>(const ConvArgs&, bool, hipStream_t);
template void launch_gemm2<bf16_t, float>(const ConvArgs&, bool, hipStream_t);
template void launch_gemm2<f16_t, float>(const ConvArgs&, bool, hipStream_t);
template void launch_gemm2<f16_t, f16_t>(const ConvArgs&, bool, hipStream_t);
template void launch_gemm2<float, float>(const ConvArgs&, bool, hipStream_t);

}  // namespace rr
