// LAB (developer experiment, not part of librr.so): the 8-wave, 8-phase staggered 256x256 GEMM
// schedule of k_gemm8 (csrc/rr_gemm.hip) reduced to the 1x1 fp16 PERM32 case, one tile per
// block, with diagnostic modes that drop one ingredient of the K-loop at a time, to find what
// holds its MFMA pipe at ~0.58 busy on plain GEMM shapes (results are wrong in modes 1-3).
//   MODE 0: the schedule as in the library (must be bit-identical to k_gemm8)
//   MODE 1: no LDS-DMA inside the K-loop        MODE 2: no fragment reads inside the K-loop
//   MODE 3: no barriers inside the K-loop       MODE 4: no s_setprio around the MFMA clusters
//   MODE 5: both B halves' fragments held in registers: quadrant (1,0) reuses B0 instead of re-reading it
//           (24 instead of 28 fragment reads per wave and K-step; bit-identical)
//   MODE 6: the DMA issued but never waited for inside the K-loop (latency probe; wrong results)
//   MODE 7: the K-loop's DMA issued with out-of-range offsets (issue + LDS writes of zeros, no memory reads)
//   MODE 8: every LDS-DMA with the nt bit, MODE 9: with sc1 (both bypass the CU's L1; bit-identical)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC tools/lab/k_g8lab.hip -o tools/lab/libg8lab.so
#include "../../image-retrieval-for-image-based-localization_amd/csrc/rr_internal.h"

namespace lab8 {
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
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(lds_addr)
        : "memory");
}
template <int POL>
__device__ __forceinline__ void dma16p(i32x4_t rsrc, unsigned voff, unsigned lds_addr) {
    if constexpr (POL == 0) {
        dma16(rsrc, voff, lds_addr);
    } else {
        unsigned keep;
        lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
        if constexpr (POL == 1)
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds\n\t"
                         "s_mov_b32 m0, %0" : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds_addr) : "memory");
        else
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen sc1 lds\n\t"
                         "s_mov_b32 m0, %0" : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds_addr) : "memory");
    }
}
__device__ __forceinline__ i32x4_t make_rsrc(const void* base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)base;
    int x = __builtin_amdgcn_readfirstlane((int)(unsigned)b);
    int y = __builtin_amdgcn_readfirstlane((int)((unsigned)(b >> 32) & 0xFFFFu));
    int z = __builtin_amdgcn_readfirstlane((int)bytes);
    asm volatile("s_nop 4" : "+s"(x), "+s"(y), "+s"(z));
    i32x4_t r;
    r.x = x;
    r.y = y;
    r.z = z;
    r.w = 0x00020000;
    return r;
}
__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

struct G8Args {
    const f16_t* x;  // [P][K]
    const f16_t* w;  // [C][K] PERM32 rows
    const float *scale, *shift;
    f16_t* y;        // [P][C]
    int P, C, K;
    unsigned long long* stamps;  // optional clock stamps [block][4]: memtime / memrealtime at start and end
};

template <int MODE>
__global__ void __launch_bounds__(512, 1) k_g8lab(G8Args a, int tiles_c, int ntiles) {
    constexpr int HT = 16384;
    __shared__ __attribute__((aligned(1024))) char smem[8 * HT];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wn = wave & 3;
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
    // clock stamps (diagnostic, separate buffer): wave 0 reads the shader clock and the constant
    // reference clock before the prologue and after the K-loop
    unsigned long long t0 = 0, r0 = 0;
    if (a.stamps && wave == 0) {
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r0)::"memory");
    }
    unsigned a_off[2][2], b_off[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int row = h * 128 + (wave + 8 * i) * 8 + lrow;
            a_off[h][i] = row < arows ? (unsigned)(((long long)row * K + lchunk * 8) * 2) : OOB;
            b_off[h][i] = p0 + row < a.P ? (unsigned)(((long long)(p0 + row) * K + lchunk * 8) * 2) : OOB;
        }
    // half-tile X (0 A0, 1 A1, 2 B0, 3 B1) of K-step kt into buffer buf
    auto issue = [&](int X, int kt, int buf) {
        if (MODE == 1) return;
        const unsigned dst = lds0 + (buf * 4 + X) * HT;
        const bool live = kt < nk;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const unsigned o = X < 2 ? a_off[X][i] : b_off[X - 2][i];
            dma16p<MODE == 8 ? 1 : MODE == 9 ? 2 : 0>(X < 2 ? rsA : rsB, MODE != 7 && live && o != OOB ? o + (unsigned)(kt * 128) : OOB, dst + (wave + 8 * i) * 1024);
        }
    };
    f32x4_t acc[2][2][4][2];
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[qa][qb][i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    uint4 fa[4][2], fbh[2][2][2];  // fbh[h]: B half h (MODE 5 keeps both; otherwise only fbh[0] is used)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) fa[i][hs] = fbh[0][i & 1][hs] = fbh[1][i & 1][hs] = make_uint4(0, 0, 0, 0);
    auto read_a = [&](int buf, int h) {
        if (MODE == 2) return;
        const char* base = smem + (buf * 4 + h) * HT;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int hs = 0; hs < 2; ++hs)
                fa[i][hs] = *reinterpret_cast<const uint4*>(base + swz(grp * 64 + i * 16 + r16, kq + 4 * hs));
    };
    auto read_b = [&](int buf, int h) {
        if (MODE == 2) return;
        const char* base = smem + ((buf & 1) * 4 + 2 + h) * HT;
        auto& fb = fbh[MODE == 5 ? h : 0];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int hs = 0; hs < 2; ++hs)
                fb[j][hs] = *reinterpret_cast<const uint4*>(base + swz(wn * 32 + j * 16 + r16, kq + 4 * hs));
    };
    auto mfma_q = [&](int qa, int qb) {
        auto& fb = fbh[MODE == 5 ? qb : 0];
        __builtin_amdgcn_sched_barrier(0);
        if (MODE != 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int hs = 0; hs < 2; ++hs)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[qa][qb][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                        __builtin_bit_cast(f16x8_t, fa[i][hs]), __builtin_bit_cast(f16x8_t, fb[j][hs]), acc[qa][qb][i][j],
                        0, 0, 0);
        if (MODE != 4) __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto bar = []() {
        if (MODE != 3) asm volatile("s_barrier" ::: "memory");
    };
    auto vm4 = []() {
        if (MODE != 1 && MODE != 6) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    };
    // prologue: K-step 0 into E (A0 B1 A1 B0), K-step 1's A0 / B1 into O
    {
        const int X0[4] = {0, 3, 1, 2};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int X = X0[q];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const unsigned o = X < 2 ? a_off[X][i] : b_off[X - 2][i];
                dma16(X < 2 ? rsA : rsB, o, lds0 + X * HT + (wave + 8 * i) * 1024);
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int X = X0[q];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const unsigned o = X < 2 ? a_off[X][i] : b_off[X - 2][i];
                dma16(X < 2 ? rsA : rsB, nk > 1 && o != OOB ? o + 128u : OOB, lds0 + (4 + X) * HT + (wave + 8 * i) * 1024);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    if (grp == 1) asm volatile("s_barrier" ::: "memory");
    const int nit = (nk + 1) >> 1;
    for (int it = 0; it < nit; ++it) {
        const int te = 2 * it, to = 2 * it + 1;
        read_a(0, 0); read_b(0, 0); issue(1, to, 1);
        bar(); mfma_q(0, 0); bar();
        read_b(0, 1); issue(2, to, 1);
        bar(); mfma_q(0, 1); bar();
        read_a(0, 1); issue(0, te + 2, 0);
        bar(); mfma_q(1, 1); bar();
        if (MODE != 5) read_b(0, 0);
        issue(3, te + 2, 0);
        vm4();
        bar(); mfma_q(1, 0); bar();
        read_a(1, 0); read_b(1, 0); issue(1, te + 2, 0);
        bar(); mfma_q(0, 0); bar();
        read_b(1, 1); issue(2, te + 2, 0);
        bar(); mfma_q(0, 1); bar();
        read_a(1, 1); issue(0, to + 2, 1);
        bar(); mfma_q(1, 1); bar();
        if (MODE != 5) read_b(1, 0);
        issue(3, to + 2, 1);
        vm4();
        bar(); mfma_q(1, 0); bar();
    }
    if (grp == 0) asm volatile("s_barrier" ::: "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.stamps && wave == 0) {
        unsigned long long t1, r1;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r1)::"memory");
        if (lane == 0) {
            unsigned long long* st = a.stamps + 4ll * blockIdx.x;
            st[0] = t0;
            st[1] = r0;
            st[2] = t1;
            st[3] = r1;
        }
    }
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2) {
            const int c = c0 + qa * 128 + grp * 64 + 32 * i2 + 8 * kq;
            if (c >= a.C) continue;
            float sc[8], sh[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) { sc[r] = a.scale[c + r]; sh[r] = a.shift[c + r]; }
#pragma unroll
            for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int p = p0 + qb * 128 + wn * 32 + j * 16 + r16;
                    if (p >= a.P) continue;
                    float v[8];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] = acc[qa][qb][2 * i2][j][r] * sc[r] + sh[r];
                        v[4 + r] = acc[qa][qb][2 * i2 + 1][j][r] * sc[4 + r] + sh[4 + r];
                    }
                    typedef __attribute__((ext_vector_type(8))) _Float16 h8;
                    *reinterpret_cast<h8*>(a.y + (long long)p * a.C + c) = (h8){(f16_t)v[0], (f16_t)v[1], (f16_t)v[2],
                                                                                (f16_t)v[3], (f16_t)v[4], (f16_t)v[5],
                                                                                (f16_t)v[6], (f16_t)v[7]};
                }
        }
}

}  // namespace lab8

extern "C" int lab_g8s(const void* x, const void* w, const float* scale, const float* shift, void* y, int P, int C,
                       int K, int mode, void* stream, unsigned long long* stamps);
extern "C" int lab_g8(const void* x, const void* w, const float* scale, const float* shift, void* y, int P, int C,
                      int K, int mode, void* stream) {
    return lab_g8s(x, w, scale, shift, y, P, C, K, mode, stream, nullptr);
}
extern "C" int lab_g8s(const void* x, const void* w, const float* scale, const float* shift, void* y, int P, int C,
                       int K, int mode, void* stream, unsigned long long* stamps) {
    if (K % 128 || C % 32 || P <= 0) return -1;
    lab8::G8Args a{(const rr::f16_t*)x, (const rr::f16_t*)w, scale, shift, (rr::f16_t*)y, P, C, K, stamps};
    const int tiles_c = (C + 255) / 256, tiles_p = (P + 255) / 256, ntiles = tiles_c * tiles_p;
    hipStream_t s = (hipStream_t)stream;
    switch (mode) {
        case 0: hipLaunchKernelGGL(lab8::k_g8lab<0>, dim3(ntiles), dim3(512), 0, s, a, tiles_c, ntiles); break;
        case 1: hipLaunchKernelGGL(lab8::k_g8lab<1>, dim3(ntiles), dim3(512), 0, s, a, tiles_c, ntiles); break;
        case 2: hipLaunchKernelGGL(lab8::k_g8lab<2>, dim3(ntiles), dim3(512), 0, s, a, tiles_c, ntiles); break;
        case 3: hipLaunchKernelGGL(lab8::k_g8lab<3>, dim3(ntiles), dim3(512), 0, s, a, tiles_c, ntiles); break;
        case 4: hipLaunchKernelGGL(lab8::k_g8lab<4>, dim3(ntiles), dim3(512), 0, s, a, tiles_c, ntiles); break;
        case 5: hipLaunchKernelGGL(lab8::k_g8lab<5>, dim3(ntiles), dim3(512), 0, s, a, tiles_c, ntiles); break;
        case 6: hipLaunchKernelGGL(lab8::k_g8lab<6>, dim3(ntiles), dim3(512), 0, s, a, tiles_c, ntiles); break;
        case 7: hipLaunchKernelGGL(lab8::k_g8lab<7>, dim3(ntiles), dim3(512), 0, s, a, tiles_c, ntiles); break;
        case 8: hipLaunchKernelGGL(lab8::k_g8lab<8>, dim3(ntiles), dim3(512), 0, s, a, tiles_c, ntiles); break;
        case 9: hipLaunchKernelGGL(lab8::k_g8lab<9>, dim3(ntiles), dim3(512), 0, s, a, tiles_c, ntiles); break;
        default: return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
