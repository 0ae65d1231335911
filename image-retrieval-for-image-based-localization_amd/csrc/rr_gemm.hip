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

namespace rr {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((address_space(3))) void lds_void;

template <typename T> struct Vec2;
template <> struct Vec2<bf16_t> { static constexpr int N = 8; };
template <> struct Vec2<float> { static constexpr int N = 4; };

constexpr unsigned OOB = 0x80000000u;  // voffset beyond every buffer: reads as 0

// s_waitcnt vmcnt(n) (gfx9 encoding: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt[5:4]<<14)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}

// One 16-B-per-lane LDS-DMA wave-instruction: LDS[m0 + lane*16] = buf[voff].
// Issued from inline asm so hipcc neither counts it nor inserts a blanket
// vmcnt(0) before later ds_reads (which it does for compiler-visible LDS-DMA):
// completion is tracked by the explicit vmcnt(N) below.  M0 is saved/restored.
typedef __attribute__((ext_vector_type(4))) int i32x4_t;
__device__ __forceinline__ void dma16(i32x4_t rsrc, unsigned voff, unsigned lds_addr) {
    unsigned keep;
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

template <typename T, typename TO, int TC, int TP, int WC, int WP, bool K1>
__global__ void __launch_bounds__(256, 2) k_gemm2(ConvArgs a) {
    constexpr int VEC = Vec2<T>::N;
    constexpr int BK = 8 * VEC;               // elements per K-step (128 B per row)
    constexpr int ESZ = sizeof(T);
    constexpr int NIA = TC / 32, NIB = TP / 32;  // LDS-DMA instructions per wave per stage
    constexpr int NLD = NIA + NIB;
    constexpr int FM = TC / WC / 16, FN = TP / WP / 16;
    constexpr int STAGE = (TC + TP) * 128;
    static_assert(WC * WP == 4 && TC % 32 == 0 && TP % 32 == 0, "tile");

    __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wc = wave % WC, wp = wave / WC;
    const int c0 = blockIdx.y * TC, p0 = blockIdx.x * TP;
    const int H = a.h, W = a.w_, Cin = a.cin;

    // ---- buffer resources: A = this block's weight rows, B = whole input
    const long long arows = (long long)min(TC, a.cout - c0);
    const i32x4_t rsA = make_rsrc((const char*)a.w + (long long)c0 * a.kp * ESZ, (unsigned)(arows * a.kp * ESZ));
    const long long xbytes = (long long)a.n * H * W * Cin * ESZ;
    const i32x4_t rsB = make_rsrc(a.x, (unsigned)xbytes);
    const unsigned lds0 = (unsigned)(unsigned long long)smem;

    // ---- per-lane DMA descriptors
    const int lrow = lane >> 3;                 // row within an 8-row wave-instruction
    const int lchunk = (lane & 7) ^ (lrow & 7); // logical chunk fetched by this lane (source swizzle)
    unsigned a_off[NIA];
#pragma unroll
    for (int i = 0; i < NIA; ++i) {
        const int row = (wave + 4 * i) * 8 + lrow;
        a_off[i] = row < arows ? (unsigned)(((long long)row * a.kp + lchunk * VEC) * ESZ) : OOB;
    }
    int b_hi[NIB], b_wi[NIB];
    unsigned b_base[NIB];  // element offset of the pixel's (img, hi0, wi0) origin, or OOB
#pragma unroll
    for (int i = 0; i < NIB; ++i) {
        const int row = (wave + 4 * i) * 8 + lrow;
        const int p = p0 + row;
        if (p < a.P) {
            const int img = p / (a.ho * a.wo);
            const int rem = p - img * (a.ho * a.wo);
            const int oh = rem / a.wo, ow = rem - oh * a.wo;
            b_hi[i] = oh * a.stride - a.pad;
            b_wi[i] = ow * a.stride - a.pad;
            long long base = (long long)img * H * W * Cin;
            if (K1) base += ((long long)b_hi[i] * W + b_wi[i]) * Cin + lchunk * VEC;
            b_base[i] = (unsigned)base;
        } else {
            b_hi[i] = b_wi[i] = 0;
            b_base[i] = OOB;
        }
    }

    auto issue = [&](int stage, int k0) {
        const unsigned As = lds0 + stage * STAGE;
        const unsigned Bs = As + TC * 128;
#pragma unroll
        for (int i = 0; i < NIA; ++i) {
            const unsigned off = a_off[i] == OOB ? OOB : a_off[i] + (unsigned)(k0 * ESZ);
            dma16(rsA, off, As + (wave + 4 * i) * 1024);
        }
#pragma unroll
        for (int i = 0; i < NIB; ++i) {
            unsigned off;
            if (K1) {
                off = b_base[i] == OOB ? OOB : (b_base[i] + (unsigned)k0) * ESZ;
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
            dma16(rsB, off, Bs + (wave + 4 * i) * 1024);
        }
    };

    f32x4_t acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    const int r16 = lane & 15, kq = lane >> 4;
    const int arow0 = wc * (TC / WC) + r16, brow0 = wp * (TP / WP) + r16;
    const int nk = a.kp / BK;

    issue(0, 0);
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) {
            issue(cur ^ 1, (kt + 1) * BK);
            wait_vm_barrier<NLD>();   // this wave's stage-kt DMA done; barrier: everyone's
        } else {
            wait_vm_barrier<0>();
        }
        const char* As = smem + cur * STAGE;
        const char* Bs = As + TC * 128;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            uint4 fa[FM], fb[FN];
#pragma unroll
            for (int i = 0; i < FM; ++i) fa[i] = *reinterpret_cast<const uint4*>(As + swz(arow0 + i * 16, kq + 4 * s));
#pragma unroll
            for (int j = 0; j < FN; ++j) fb[j] = *reinterpret_cast<const uint4*>(Bs + swz(brow0 + j * 16, kq + 4 * s));
            if constexpr (VEC == 8) {
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
        lds_barrier();  // every wave finished reading stage `cur` before it is refilled
    }

    // ---- fused epilogue (4 consecutive channels of one pixel per lane)
    TO* __restrict__ Y = (TO*)a.y;
    const TO* __restrict__ R = (const TO*)a.res;
    const bool affine = a.flags & RR_CONV_AFFINE;
    const bool resid = a.flags & RR_CONV_RESIDUAL;
    const bool leaky = a.act == RR_ACT_LEAKY;
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
static void launch2_cfg(const ConvArgs& a, bool k1, hipStream_t s) {
    dim3 grid((a.P + TP - 1) / TP, (a.cout + TC - 1) / TC);
    if (k1)
        hipLaunchKernelGGL((k_gemm2<T, TO, TC, TP, WC, WP, true>), grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((k_gemm2<T, TO, TC, TP, WC, WP, false>), grid, dim3(256), 0, s, a);
}

template <typename T, typename TO>
void launch_gemm2(const ConvArgs& a, bool k1, hipStream_t s) {
    if (a.P <= 32)
        launch2_cfg<T, TO, 256, 32, 4, 1>(a, k1, s);
    else if (a.P <= 64)
        launch2_cfg<T, TO, 256, 64, 4, 1>(a, k1, s);
    else if (a.cout <= 64)
        launch2_cfg<T, TO, 64, 256, 1, 4>(a, k1, s);
    else
        launch2_cfg<T, TO, 128, 128, 2, 2>(a, k1, s);
}

template void launch_gemm2<bf16_t, bf16_t>(const ConvArgs&, bool, hipStream_t);
template void launch_gemm2<bf16_t, float>(const ConvArgs&, bool, hipStream_t);
template void launch_gemm2<float, float>(const ConvArgs&, bool, hipStream_t);

}  // namespace rr
