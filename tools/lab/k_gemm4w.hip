// LAB (developer experiment, not part of librr.so): a 4-wave 256x256 GEMM tile, one wave per SIMD,
// each wave a 128 x 128 sub-tile (8 x 8 accumulator fragments of 16x16, 256 registers), the
// structure of the library GEMM that beats k_gemm8 by 14-18 % on plain shapes
// (profiles/r06_ab/r06j_gemm8_vs_hipblaslt_square.txt: 4 waves, MT256x256x64, MI16x16, 130 KiB LDS).
// y[p][c] = act(sum_k x[p][k] w[c][k] * scale[c] + shift[c]), fp16 in / out, PERM32 weight rows,
// the same LDS half-tile image, DMA and K order as k_gemm8 (so results are bit-identical to it).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC tools/lab/k_gemm4w.hip -o tools/lab/libg4w.so
#include "../../image-retrieval-for-image-based-localization_amd/csrc/rr_internal.h"

namespace lab {
using rr::f16_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) int i32x4_t;
constexpr unsigned OOB = 0x80000000u;

__device__ __forceinline__ void dma16(i32x4_t rsrc, unsigned voff, unsigned lds_addr) {
    unsigned keep;
    lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
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
// the same LDS-DMA without the m0 save / restore (m0 declared clobbered) and one wait state
__device__ __forceinline__ void dma16f(i32x4_t rsrc, unsigned voff, unsigned lds_addr) {
    lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
    asm volatile(
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %0, %1, 0 offen lds"
        :
        : "v"(voff), "s"(rsrc), "s"(lds_addr)
        : "memory", "m0");
}
// m0 saved / restored, one wait state
__device__ __forceinline__ void dma16s(i32x4_t rsrc, unsigned voff, unsigned lds_addr) {
    unsigned keep;
    lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(lds_addr)
        : "memory");
}
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

struct G4Args {
    const f16_t* x;   // [P][K]
    const f16_t* w;   // [C][K] PERM32 rows
    const float *scale, *shift;
    f16_t* y;         // [P][C]
    int P, C, K;
    float slope;
    unsigned long long* stamps;  // optional clock stamps [block][4] (variant 1 only)
};

// VARIANT 0: 2 stages of a whole 64-deep K-step (4 half-tiles A0 A1 B0 B1, 64 KiB each); per
// K-step: wait for its DMA, one barrier, issue the next K-step's DMA (16 per wave), then the
// fragment reads and 128 MFMAs of this K-step.
template <int VARIANT>
__global__ void __launch_bounds__(256, 1) k_gemm4w(G4Args a, int tiles_c, int ntiles) {
    constexpr int HT = 16384, ST = 4 * HT;
    __shared__ __attribute__((aligned(1024))) char smem[2 * ST];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wcl = wave & 1;
    const int r16 = lane & 15, kq = lane >> 4;
    const int lrow = lane >> 3, lchunk = (lane & 7) ^ (lrow & 7);
    // XCD-contiguous bijective tile order, pixel-major (the channel tiles of a pixel tile adjacent)
    const int bx = (int)blockIdx.x, xcd = bx & 7, nt8 = ntiles >> 3, rt8 = ntiles & 7;
    const int t = (xcd < rt8 ? xcd * (nt8 + 1) : rt8 * (nt8 + 1) + (xcd - rt8) * nt8) + (bx >> 3);
    const int c0 = (t % tiles_c) * 256, p0 = (t / tiles_c) * 256;
    const int K = a.K, nk = K / 64;
    const int arows = min(256, a.C - c0);
    const i32x4_t rsA = make_rsrc(a.w + (long long)c0 * K, (unsigned)((long long)arows * K * 2));
    const i32x4_t rsB = make_rsrc(a.x, (unsigned)((long long)a.P * K * 2));
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    // per lane: the row offsets of its 16 DMA pieces (X = A0 A1 B0 B1, i = 0..3: rows (wave + 4 i) 8 + lrow)
    unsigned off[4][4];
#pragma unroll
    for (int X = 0; X < 4; ++X)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = (X & 1) * 128 + (wave + 4 * i) * 8 + lrow;
            if (X < 2) off[X][i] = row < arows ? (unsigned)(((long long)row * K + lchunk * 8) * 2) : OOB;
            else off[X][i] = p0 + row < a.P ? (unsigned)(((long long)(p0 + row) * K + lchunk * 8) * 2) : OOB;
        }
    auto issue = [&](int kt, int s) {
        const bool live = kt < nk;
#pragma unroll
        for (int X = 0; X < 4; ++X)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const unsigned o = live && off[X][i] != OOB ? off[X][i] + (unsigned)(kt * 128) : OOB;
                dma16(X < 2 ? rsA : rsB, o, lds0 + s * ST + X * HT + (wave + 4 * i) * 1024);
            }
    };
    f32x4_t acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    issue(0, 0);
    for (int kt = 0; kt < nk; ++kt) {
        const int s = kt & 1;
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        issue(kt + 1, s ^ 1);
        const char* A = smem + s * ST + wr * HT;
        const char* B = smem + s * ST + (2 + wcl) * HT;
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) {
            uint4 fa[8], fb[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) fa[i] = *reinterpret_cast<const uint4*>(A + swz(i * 16 + r16, kq + 4 * hs));
#pragma unroll
            for (int j = 0; j < 8; ++j) fb[j] = *reinterpret_cast<const uint4*>(B + swz(j * 16 + r16, kq + 4 * hs));
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, fa[i]),
                                                                       __builtin_bit_cast(f16x8_t, fb[j]), acc[i][j], 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // epilogue: PERM32 rows -> a lane's fragment pair (2 i2, 2 i2 + 1) holds 8 consecutive channels
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) {
        const int c = c0 + wr * 128 + 32 * i2 + 8 * kq;
        if (c >= a.C) continue;
        float sc[8], sh[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) { sc[r] = a.scale[c + r]; sh[r] = a.shift[c + r]; }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int p = p0 + wcl * 128 + j * 16 + r16;
            if (p >= a.P) continue;
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[2 * i2][j][r] * sc[r] + sh[r];
                v[4 + r] = acc[2 * i2 + 1][j][r] * sc[4 + r] + sh[4 + r];
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
            typedef __attribute__((ext_vector_type(8))) _Float16 h8;
            *reinterpret_cast<h8*>(a.y + (long long)p * a.C + c) =
                (h8){(f16_t)v[0], (f16_t)v[1], (f16_t)v[2], (f16_t)v[3], (f16_t)v[4], (f16_t)v[5], (f16_t)v[6], (f16_t)v[7]};
        }
    }
}


// VARIANT 1: the same tile, two register sets of fragments (R0 = half-step 0, R1 = half-step 1
// of a K-step) so every LDS read lands a half-step before its MFMAs:
//   phase A of K-step kt: read R1 (kt, hs 1) from stage kt&1  ||  64 MFMAs on R0
//   mid: lgkmcnt(0) (stage kt&1 fully read) + vmcnt(0) (K-step kt+1 landed) + barrier
//   phase B: DMA K-step kt+2 into stage kt&1, read R0 (kt+1, hs 0) from stage (kt+1)&1  ||  64 MFMAs on R1
// Each phase is 16 pinned groups {(DMA piece), 1 fragment read, 4 MFMAs}.
// MODE (diagnostic): 0 normal, 1 no DMA inside the K-loop, 2 no fragment reads inside the K-loop,
// 3 no wait for the DMA at mid-step (wrong results: latency probe), 4 the short DMA sequence
template <int MODE>
__global__ void __launch_bounds__(256, 1) k_gemm4w_v1(G4Args a, int tiles_c, int ntiles) {
    constexpr int HT = 16384, ST = 4 * HT;
    __shared__ __attribute__((aligned(1024))) char smem[2 * ST];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wcl = wave & 1;
    const int r16 = lane & 15, kq = lane >> 4;
    const int lrow = lane >> 3, lchunk = (lane & 7) ^ (lrow & 7);
    const int bx = (int)blockIdx.x, xcd = bx & 7, nt8 = ntiles >> 3, rt8 = ntiles & 7;
    const int t = (xcd < rt8 ? xcd * (nt8 + 1) : rt8 * (nt8 + 1) + (xcd - rt8) * nt8) + (bx >> 3);
    const int c0 = (t % tiles_c) * 256, p0 = (t / tiles_c) * 256;
    const int K = a.K, nk = K / 64;
    const int arows = min(256, a.C - c0);
    const i32x4_t rsA = make_rsrc(a.w + (long long)c0 * K, (unsigned)((long long)arows * K * 2));
    const i32x4_t rsB = make_rsrc(a.x, (unsigned)((long long)a.P * K * 2));
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    unsigned long long t0 = 0, r0s = 0;
    if (a.stamps && wave == 0) {
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r0s)::"memory");
    }
    unsigned off[4][4];
#pragma unroll
    for (int X = 0; X < 4; ++X)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = (X & 1) * 128 + (wave + 4 * i) * 8 + lrow;
            if (X < 2) off[X][i] = row < arows ? (unsigned)(((long long)row * K + lchunk * 8) * 2) : OOB;
            else off[X][i] = p0 + row < a.P ? (unsigned)(((long long)(p0 + row) * K + lchunk * 8) * 2) : OOB;
        }
    auto dma = [&](int X, int i, int kt, int s) {
        const unsigned o = kt < nk && off[X][i] != OOB ? off[X][i] + (unsigned)(kt * 128) : OOB;
        if (MODE == 5) dma16s(X < 2 ? rsA : rsB, o, lds0 + s * ST + X * HT + (wave + 4 * i) * 1024);
        else if (MODE == 4) dma16f(X < 2 ? rsA : rsB, o, lds0 + s * ST + X * HT + (wave + 4 * i) * 1024);
        else dma16(X < 2 ? rsA : rsB, o, lds0 + s * ST + X * HT + (wave + 4 * i) * 1024);
    };
    f32x4_t acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    uint4 R0[16], R1[16];  // [0..7] A fragments (rows i*16), [8..15] B fragments (cols j*16)
    auto rd1 = [&](uint4* R, int g, int s, int hs) {
        const char* base = smem + s * ST + (g < 8 ? wr : 2 + wcl) * HT;
        R[g] = *reinterpret_cast<const uint4*>(base + swz((g & 7) * 16 + r16, kq + 4 * hs));
    };
    auto mm4 = [&](const uint4* R, int g) {  // MFMAs (i = g / 2, j = 4 (g & 1) .. + 3)
        const int i = g >> 1;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * (g & 1) + jj;
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, R[i]),
                                                               __builtin_bit_cast(f16x8_t, R[8 + j]), acc[i][j], 0, 0, 0);
        }
    };
#pragma unroll
    for (int X = 0; X < 4; ++X)
#pragma unroll
        for (int i = 0; i < 4; ++i) dma(X, i, 0, 0);
#pragma unroll
    for (int X = 0; X < 4; ++X)
#pragma unroll
        for (int i = 0; i < 4; ++i) dma(X, i, 1, 1);
    asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int g = 0; g < 16; ++g) rd1(R0, g, 0, 0);
    for (int kt = 0; kt < nk; ++kt) {
        const int s = kt & 1;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            __builtin_amdgcn_sched_barrier(0);
            if (MODE != 2) rd1(R1, g, s, 1);
            mm4(R0, g);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (MODE == 3) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            __builtin_amdgcn_sched_barrier(0);
            if (MODE != 1) dma(g >> 2, g & 3, kt + 2, s);
            if (MODE != 2) rd1(R0, g, s ^ 1, 0);
            mm4(R1, g);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.stamps && wave == 0) {
        unsigned long long t1, r1;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r1)::"memory");
        if (lane == 0) {
            unsigned long long* st = a.stamps + 4ll * blockIdx.x;
            st[0] = t0;
            st[1] = r0s;
            st[2] = t1;
            st[3] = r1;
        }
    }
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) {
        const int c = c0 + wr * 128 + 32 * i2 + 8 * kq;
        if (c >= a.C) continue;
        float sc[8], sh[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) { sc[r] = a.scale[c + r]; sh[r] = a.shift[c + r]; }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int p = p0 + wcl * 128 + j * 16 + r16;
            if (p >= a.P) continue;
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[2 * i2][j][r] * sc[r] + sh[r];
                v[4 + r] = acc[2 * i2 + 1][j][r] * sc[4 + r] + sh[4 + r];
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
            typedef __attribute__((ext_vector_type(8))) _Float16 h8;
            *reinterpret_cast<h8*>(a.y + (long long)p * a.C + c) =
                (h8){(f16_t)v[0], (f16_t)v[1], (f16_t)v[2], (f16_t)v[3], (f16_t)v[4], (f16_t)v[5], (f16_t)v[6], (f16_t)v[7]};
        }
    }
}

// VARIANT 2: half-step stages (K 32: A 256 x 64 B + B 256 x 64 B = 32 KiB), 4 of them (128 KiB),
// so an LDS-DMA has three phases (1.5 K-steps) to land instead of one.  64-B rows: chunk kq of
// row r sits at slot kq ^ g[(r >> 2) & 3], g = {0, 2, 3, 1} (conflict-free for the four
// ds_read_b128 lane groups).  Phase h (one half-step, 64 MFMAs per wave): groups 0-7 read two
// fragments of R(h+1) from stage (h+1)&3, groups 8-15 issue one DMA piece of half-step h+4 into
// stage h&3 (last read in phase h-1); every group 4 MFMAs on R(h).  End of phase: lgkmcnt(0) +
// vmcnt(16) (half-step h+2 landed) + barrier.
__device__ __forceinline__ int g4(int b) { return (0x1320 >> (4 * (b & 3))) & 3; }  // g = {0, 2, 3, 1}

__global__ void __launch_bounds__(256, 1) k_gemm4w_v2(G4Args a, int tiles_c, int ntiles) {
    constexpr int SS = 32768, HALF = 16384;
    __shared__ __attribute__((aligned(1024))) char smem[4 * SS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wcl = wave & 1;
    const int r16 = lane & 15, kq = lane >> 4;
    const int bx = (int)blockIdx.x, xcd = bx & 7, nt8 = ntiles >> 3, rt8 = ntiles & 7;
    const int t = (xcd < rt8 ? xcd * (nt8 + 1) : rt8 * (nt8 + 1) + (xcd - rt8) * nt8) + (bx >> 3);
    const int c0 = (t % tiles_c) * 256, p0 = (t / tiles_c) * 256;
    const int K = a.K, nh = K / 32;
    const int arows = min(256, a.C - c0);
    const i32x4_t rsA = make_rsrc(a.w + (long long)c0 * K, (unsigned)((long long)arows * K * 2));
    const i32x4_t rsB = make_rsrc(a.x, (unsigned)((long long)a.P * K * 2));
    const unsigned lds0 = (unsigned)(unsigned long long)smem;
    // DMA pieces: wave w issues pieces w + 4 q (q = 0..7) of a stage; piece p < 16: A rows 16 p ..,
    // else B rows 16 (p - 16) ..; lane l: row 16 p' + (l >> 2), physical chunk l & 3
    unsigned off[8];
    const int lr = lane >> 2, lc = (lane & 3) ^ g4(lane >> 4);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int pc = wave + 4 * q;
        const int row = (pc & 15) * 16 + lr;
        if (pc < 16) off[q] = row < arows ? (unsigned)(((long long)row * K + lc * 8) * 2) : OOB;
        else off[q] = p0 + row < a.P ? (unsigned)(((long long)(p0 + row) * K + lc * 8) * 2) : OOB;
    }
    auto dma = [&](int q, int h) {
        const unsigned o = h < nh && off[q] != OOB ? off[q] + (unsigned)(h * 64) : OOB;
        dma16(q < 4 ? rsA : rsB, o, lds0 + (h & 3) * SS + (wave + 4 * q) * 1024);
    };
    // fragment reads: A rows wr*128 + i*16 + r16, B rows wcl*128 + j*16 + r16; slot kq ^ g
    const int rdo = r16 * 64 + 16 * (kq ^ g4(r16 >> 2));
    const int rdA = wr * 128 * 64 + rdo, rdB = HALF + wcl * 128 * 64 + rdo;
    f32x4_t acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    uint4 R[2][16];
    auto rd1 = [&](uint4* Rx, int f, int h) {  // fragment f (0..7 A rows f*16, 8..15 B rows)
        const char* base = smem + (h & 3) * SS + (f < 8 ? rdA : rdB) + (f & 7) * 1024;
        Rx[f] = *reinterpret_cast<const uint4*>(base);
    };
    auto mm4 = [&](const uint4* Rx, int g) {
        const int i = g >> 1;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * (g & 1) + jj;
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, Rx[i]),
                                                               __builtin_bit_cast(f16x8_t, Rx[8 + j]), acc[i][j], 0, 0, 0);
        }
    };
    auto phase = [&](uint4* Rc, uint4* Rn, int h) {
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            __builtin_amdgcn_sched_barrier(0);
            if (g < 8) {
                rd1(Rn, 2 * g, h + 1);
                rd1(Rn, 2 * g + 1, h + 1);
            } else {
                dma(g - 8, h + 4);
            }
            mm4(Rc, g);
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int q = 0; q < 8; ++q) dma(q, h);
    asm volatile("s_waitcnt vmcnt(24)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int f = 0; f < 16; ++f) rd1(R[0], f, 0);
    asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
    for (int h = 0; h < nh; h += 2) {
        phase(R[0], R[1], h);
        phase(R[1], R[0], h + 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) {
        const int c = c0 + wr * 128 + 32 * i2 + 8 * kq;
        if (c >= a.C) continue;
        float sc[8], sh[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) { sc[r] = a.scale[c + r]; sh[r] = a.shift[c + r]; }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int p = p0 + wcl * 128 + j * 16 + r16;
            if (p >= a.P) continue;
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[2 * i2][j][r] * sc[r] + sh[r];
                v[4 + r] = acc[2 * i2 + 1][j][r] * sc[4 + r] + sh[4 + r];
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
            typedef __attribute__((ext_vector_type(8))) _Float16 h8;
            *reinterpret_cast<h8*>(a.y + (long long)p * a.C + c) =
                (h8){(f16_t)v[0], (f16_t)v[1], (f16_t)v[2], (f16_t)v[3], (f16_t)v[4], (f16_t)v[5], (f16_t)v[6], (f16_t)v[7]};
        }
    }
}

// VARIANT 3: register-staged loads instead of LDS-DMA, so the LDS writes happen where the schedule
// puts them (phase A's first half) rather than whenever the DMA data arrives.  Per K-step kt:
//   phase A: 16 groups {ds_write one staged 1-KiB piece of K-step kt+1 (groups 0-7: two), then the
//            buffer loads of K-step kt+2 into the freed staging registers (groups 8-15: two),
//            read one fragment of R1 (kt, hs 1), 4 MFMAs on R0}
//   mid: lgkmcnt(0) + barrier (stage (kt+1)&1 written, stage kt&1 read)
//   phase B: 16 groups {read one fragment of R0 (kt+1, hs 0) from stage (kt+1)&1, 4 MFMAs on R1}
// The staging loads are compiler-visible (raw buffer loads), so hipcc places their vmcnt waits.
__global__ void __launch_bounds__(256, 1) k_gemm4w_v3(G4Args a, int tiles_c, int ntiles) {
    constexpr int HT = 16384, ST = 4 * HT;
    __shared__ __attribute__((aligned(1024))) char smem[2 * ST];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wcl = wave & 1;
    const int r16 = lane & 15, kq = lane >> 4;
    const int lrow = lane >> 3, lch = lane & 7;
    const int bx = (int)blockIdx.x, xcd = bx & 7, nt8 = ntiles >> 3, rt8 = ntiles & 7;
    const int t = (xcd < rt8 ? xcd * (nt8 + 1) : rt8 * (nt8 + 1) + (xcd - rt8) * nt8) + (bx >> 3);
    const int c0 = (t % tiles_c) * 256, p0 = (t / tiles_c) * 256;
    const int K = a.K, nk = K / 64;
    const int arows = min(256, a.C - c0);
    __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)(a.w + (long long)c0 * K), (short)0,
                                                                   arows * K * 2, 0x00020000);
    __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.P * K * 2, 0x00020000);
    // piece q (0..15) of a wave: half-tile X = q >> 2, rows (wave + 4 (q & 3)) * 8 + lrow, logical chunk lch
    unsigned off[16];
    int wofs[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int X = q >> 2, i = q & 3;
        const int row = (X & 1) * 128 + (wave + 4 * i) * 8 + lrow;
        if (X < 2) off[q] = row < arows ? (unsigned)((row * K + lch * 8) * 2) : OOB;
        else off[q] = p0 + row < a.P ? (unsigned)(((p0 + row) * K + lch * 8) * 2) : OOB;
        wofs[q] = X * HT + swz(row & 127, lch);
    }
    uint4 stg[16];
    auto gload = [&](int q, int kt) {
        const unsigned o = kt < nk && off[q] != OOB ? off[q] + (unsigned)(kt * 128) : OOB;
        stg[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(q < 8 ? rsA : rsB, o, 0, 0));
    };
    auto swrite = [&](int q, int s) { *reinterpret_cast<uint4*>(smem + s * ST + wofs[q]) = stg[q]; };
    f32x4_t acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    uint4 R0[16], R1[16];
    auto rd1 = [&](uint4* R, int g, int s, int hs) {
        const char* base = smem + s * ST + (g < 8 ? wr : 2 + wcl) * HT;
        R[g] = *reinterpret_cast<const uint4*>(base + swz((g & 7) * 16 + r16, kq + 4 * hs));
    };
    auto mm4 = [&](const uint4* R, int g) {
        const int i = g >> 1;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * (g & 1) + jj;
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, R[i]),
                                                               __builtin_bit_cast(f16x8_t, R[8 + j]), acc[i][j], 0, 0, 0);
        }
    };
    // prologue: K-step 0 staged and written to stage 0, K-step 1 staged
#pragma unroll
    for (int q = 0; q < 16; ++q) gload(q, 0);
#pragma unroll
    for (int q = 0; q < 16; ++q) swrite(q, 0);
#pragma unroll
    for (int q = 0; q < 16; ++q) gload(q, 1);
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 16; ++g) rd1(R0, g, 0, 0);
    for (int kt = 0; kt < nk; ++kt) {
        const int s = kt & 1;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            __builtin_amdgcn_sched_barrier(0);
            if (g < 8) {
                swrite(2 * g, s ^ 1);
                swrite(2 * g + 1, s ^ 1);
            } else {
                gload(2 * (g - 8), kt + 2);
                gload(2 * (g - 8) + 1, kt + 2);
            }
            rd1(R1, g, s, 1);
            mm4(R0, g);
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            __builtin_amdgcn_sched_barrier(0);
            rd1(R0, g, s ^ 1, 0);
            mm4(R1, g);
        }
        __builtin_amdgcn_sched_barrier(0);
        // the next phase A overwrites stage s (read in phase A above, fragments R1): every wave's
        // reads of it are done (lgkmcnt(0) before the barrier above); stage s^1 (read in phase B)
        // is written again only after the next mid barrier
    }
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) {
        const int c = c0 + wr * 128 + 32 * i2 + 8 * kq;
        if (c >= a.C) continue;
        float sc[8], sh[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) { sc[r] = a.scale[c + r]; sh[r] = a.shift[c + r]; }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int p = p0 + wcl * 128 + j * 16 + r16;
            if (p >= a.P) continue;
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[2 * i2][j][r] * sc[r] + sh[r];
                v[4 + r] = acc[2 * i2 + 1][j][r] * sc[4 + r] + sh[4 + r];
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * a.slope;
            typedef __attribute__((ext_vector_type(8))) _Float16 h8;
            *reinterpret_cast<h8*>(a.y + (long long)p * a.C + c) =
                (h8){(f16_t)v[0], (f16_t)v[1], (f16_t)v[2], (f16_t)v[3], (f16_t)v[4], (f16_t)v[5], (f16_t)v[6], (f16_t)v[7]};
        }
    }
}

}  // namespace lab

extern "C" int lab_gemm4ws(const void* x, const void* w, const float* scale, const float* shift, void* y, int P,
                           int C, int K, float slope, int variant, void* stream, unsigned long long* stamps);
extern "C" int lab_gemm4w(const void* x, const void* w, const float* scale, const float* shift, void* y, int P, int C,
                          int K, float slope, int variant, void* stream) {
    return lab_gemm4ws(x, w, scale, shift, y, P, C, K, slope, variant, stream, nullptr);
}
extern "C" int lab_gemm4ws(const void* x, const void* w, const float* scale, const float* shift, void* y, int P,
                           int C, int K, float slope, int variant, void* stream, unsigned long long* stamps) {
    if (K % 64 || C % 32 || P <= 0) return -1;
    lab::G4Args a{(const rr::f16_t*)x, (const rr::f16_t*)w, scale, shift, (rr::f16_t*)y, P, C, K, slope, stamps};
    const int tiles_c = (C + 255) / 256, tiles_p = (P + 255) / 256, ntiles = tiles_c * tiles_p;
    hipStream_t s = (hipStream_t)stream;
    if (variant == 0) hipLaunchKernelGGL((lab::k_gemm4w<0>), dim3(ntiles), dim3(256), 0, s, a, tiles_c, ntiles);
    else if (variant == 1) hipLaunchKernelGGL(lab::k_gemm4w_v1<0>, dim3(ntiles), dim3(256), 0, s, a, tiles_c, ntiles);
    else if (variant == 2) hipLaunchKernelGGL(lab::k_gemm4w_v2, dim3(ntiles), dim3(256), 0, s, a, tiles_c, ntiles);
    else if (variant == 11) hipLaunchKernelGGL(lab::k_gemm4w_v1<1>, dim3(ntiles), dim3(256), 0, s, a, tiles_c, ntiles);
    else if (variant == 12) hipLaunchKernelGGL(lab::k_gemm4w_v1<2>, dim3(ntiles), dim3(256), 0, s, a, tiles_c, ntiles);
    else if (variant == 13) hipLaunchKernelGGL(lab::k_gemm4w_v1<3>, dim3(ntiles), dim3(256), 0, s, a, tiles_c, ntiles);
    else if (variant == 14) hipLaunchKernelGGL(lab::k_gemm4w_v1<4>, dim3(ntiles), dim3(256), 0, s, a, tiles_c, ntiles);
    else if (variant == 15) hipLaunchKernelGGL(lab::k_gemm4w_v1<5>, dim3(ntiles), dim3(256), 0, s, a, tiles_c, ntiles);
    else if (variant == 3) hipLaunchKernelGGL(lab::k_gemm4w_v3, dim3(ntiles), dim3(256), 0, s, a, tiles_c, ntiles);
    else return -2;
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
