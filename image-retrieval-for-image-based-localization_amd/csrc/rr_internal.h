// Internal helpers shared by the librr.so translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <string>

#include "../../include/rr.h"

namespace rr {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// CUs one persistent launch may spread over: the device's CU count, capped by
// rr_set_tuning(RR_TUNE_GRID_CUS, n) (0 = no cap) so that launches on two
// streams can share the chip (rr_runtime.hip).
int grid_cus();
extern int g_grid_cap;

// A ragged image batch (a cirtorch PackedSequence at the model boundary,
// utils/parallel/packed_sequence.py:8-96): image i of a launch is [c][h_i][w_i]
// at its own device address and the batch map is the max extent H x W.  Map
// pixels outside image i's extent read as 0 -- the zero fill of
// pad_packed_images (utils/sequence.py:51) -- BEFORE normalisation (the in-tree
// order: random_augmentation.py:102 pads, :174 normalises), so no padded copy
// of the batch is ever written.  Passed by value in the kernel arguments (one
// 1-KiB table, graph-capturable, no host->device copy); the host splits a
// longer batch into launches of at most RAGGED_MAX images.
constexpr int RAGGED_MAX = 64;
struct RaggedTab {
    const void* p[RAGGED_MAX];
    int h[RAGGED_MAX];
    int w[RAGGED_MAX];
};
struct NoTab {};  // a same-size batch: one [n][c][H][W] buffer

// Fill a table for images [i0, i0 + cnt) of a host (pointer, extent) list;
// returns an error message or nullptr.
const char* ragged_fill(RaggedTab& t, const void* const* srcs, const int* extents, int i0, int cnt, int h, int w);

// Launch-error check: every entry point ends with this.
inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(RR_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    return RR_OK;
}

// bf16 stored as raw uint16 bits.
typedef uint16_t bf16_t;
typedef _Float16 f16_t;  // IEEE binary16 (kNN screening copies)

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even float -> bf16, NaN kept NaN.  On the device this is
// the gfx950 v_cvt_pk_bf16_f32 instruction (branch-free; the bit-twiddling
// form compiles to an exec-masked branch per element); the host form is the
// same rounding in integer arithmetic.
typedef __attribute__((ext_vector_type(2))) float f32x2_cvt_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_cvt_t;
__device__ __host__ __forceinline__ bf16_t f2bf(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bit_cast(bf16_t, (__bf16)f);
#else
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (bf16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (bf16_t)(u >> 16);
#endif
}
// two floats -> packed bf16x2 (lo in bits 0..15), one v_cvt_pk_bf16_f32.
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_cvt_t){lo, hi}, bf16x2_cvt_t));
}

template <typename T> struct DT;
template <> struct DT<float> {
    static __device__ __forceinline__ float load(const float* p) { return *p; }
    static __device__ __forceinline__ float to_f(float v) { return v; }
    static __device__ __forceinline__ float from_f(float v) { return v; }
};
template <> struct DT<bf16_t> {
    static __device__ __forceinline__ float to_f(bf16_t v) { return bf2f(v); }
    static __device__ __forceinline__ bf16_t from_f(float v) { return f2bf(v); }
};
// 16-bit MFMA operand types of the fused kernels (bf16 or IEEE fp16): one
// v_mfma_f32_16x16x32_{bf16,f16} on 8 packed values per lane, packing of two
// floats (round to nearest even) and unpacking of a packed pair.
typedef __attribute__((ext_vector_type(4))) float h16_f32x4_t;
template <typename H> struct H16;
template <> struct H16<bf16_t> {
    typedef __attribute__((ext_vector_type(8))) __bf16 v8;
    static __device__ __forceinline__ h16_f32x4_t mfma(uint4 a, uint4 b, h16_f32x4_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8, a), __builtin_bit_cast(v8, b), c, 0, 0, 0);
    }
    static __device__ __forceinline__ uint32_t pack2(float lo, float hi) { return pack_bf16x2(lo, hi); }
    static __device__ __forceinline__ float lo(uint32_t w) { return __uint_as_float(w << 16); }
    static __device__ __forceinline__ float hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
    static constexpr uint32_t NEG_INF = 0xFF80u;
};
template <> struct H16<f16_t> {
    typedef __attribute__((ext_vector_type(8))) _Float16 v8;
    typedef __attribute__((ext_vector_type(2))) _Float16 v2;
    static __device__ __forceinline__ h16_f32x4_t mfma(uint4 a, uint4 b, h16_f32x4_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8, a), __builtin_bit_cast(v8, b), c, 0, 0, 0);
    }
    static __device__ __forceinline__ uint32_t pack2(float lo, float hi) {
        return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_cvt_t){lo, hi}, v2));
    }
    static __device__ __forceinline__ float lo(uint32_t w) { return (float)__builtin_bit_cast(v2, w).x; }
    static __device__ __forceinline__ float hi(uint32_t w) { return (float)__builtin_bit_cast(v2, w).y; }
    static constexpr uint32_t NEG_INF = 0xFC00u;
};

template <> struct DT<f16_t> {  // IEEE binary16, round to nearest even
    static __device__ __forceinline__ float to_f(f16_t v) { return (float)v; }
    static __device__ __forceinline__ f16_t from_f(float v) { return (f16_t)v; }
};

// 16-B / 8-B global accesses of the streaming kernels (rr_stream.hip): data
// read or written exactly once per launch.  (Marking them nontemporal -- nt
// stores, nt loads and nt LDS-DMA -- measured 7 % slower on the body: 27.2-27.3
// vs 25.4 ms per 128-image forward, same box; kept plain.)
__device__ __forceinline__ void st16_once(void* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }
__device__ __forceinline__ void st8_once(void* p, uint2 v) { *reinterpret_cast<uint2*>(p) = v; }
__device__ __forceinline__ uint4 ld16_once(const void* p) { return *reinterpret_cast<const uint4*>(p); }

// Packed-k offset (elements) of K-step kt of a tap-uniform im2col conv (c_in a
// multiple of the bk-deep K-step, k = tap * c_in + ci in the packed row), in
// (input chunk, tap) order: every conv kernel of the engine -- the direct 3x3s
// (rr_conv3.hip / rr_conv3s.hip) and the im2col GEMMs -- accumulates a filter in
// the same (chunk, tap, 32-channel half) order, so the kernel a layer runs on,
// which depends on the batch size, never changes a bit of its output.  K-steps
// past ntap * nchunk (a zero-padded k_packed tail) stay linear.
// magic = ceil(2^16 / ntap): the chunk index (kt * magic) >> 16 equals
// kt / ntap for every kt < 2^16 / ntap (checked on the host: tapu_ok), two
// scalar integer instructions on the DMA issue path instead of a division.
__host__ __device__ __forceinline__ unsigned tapu_magic(int ntap) { return (65536u + (unsigned)ntap - 1u) / (unsigned)ntap; }
// every K-step index of a conv with ntap taps and nsteps tap-uniform K-steps is in that range
__host__ __device__ __forceinline__ bool tapu_ok(int ntap, long long nsteps) { return nsteps * (ntap - 1) < 65536; }
__device__ __forceinline__ int tapu_k0(int kt, int ntap, unsigned magic, int nchunk, int cin, int bk) {
#ifdef RR_TAPU_LINEAR  // timing experiments only: the linear (tap, chunk) order
    return kt * bk;
#endif
    if (kt >= ntap * nchunk) return kt * bk;
    const int cc = (int)(((unsigned)kt * magic) >> 16), tap = kt - cc * ntap;
    return tap * cin + cc * bk;
}

// Arguments of the MFMA implicit-GEMM engine (rr_conv.hip); also drives the
// kNN score GEMM (rr_knn.hip).
struct ConvArgs {
    const void* x;
    const void* w;
    const float* scale;
    const float* shift;
    const void* res;
    void* y;
    int n, h, w_, cin, ho, wo, cout, kh, kw, stride, pad, dil, kp, ldy, act, flags;
    float slope;
    int lc;  // log2(cin)
    int P;   // n*ho*wo
    // kNN screening epilogue of the score GEMM (rr_knn.hip), float output only:
    // when scr_k != nullptr nothing is stored to y; every score whose key is
    // >= scr_tau[query] is appended to the (query, chunk) candidate slot
    // (chunk = (scr_row0 + row) / scr_L, KC entries, scr_cnt counts appends).
    uint32_t* scr_tau;
    int* scr_cnt;
    uint32_t* scr_k;
    int* scr_i;
    int scr_L, scr_nchunks, scr_KC, scr_row0;
};

// monotone uint32 key of a float score (larger score <-> larger key; 0 = sentinel)
__device__ __forceinline__ uint32_t score_key(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Screening epilogue: 4 consecutive database rows c..c+3 (valid: < rows) of query p.
__device__ __forceinline__ void screen_append(const ConvArgs& a, const float* v, int c, int rows, int p,
                                              uint32_t tau) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        if (c + r >= rows) break;
        const uint32_t key = score_key(v[r]);
        if (key >= tau) {
            const int grow = a.scr_row0 + c + r;
            const int chunk = grow / a.scr_L;
            const long long slot = (long long)p * a.scr_nchunks + chunk;
            const int pos = atomicAdd(a.scr_cnt + slot, 1);
            if (pos < a.scr_KC) {
                a.scr_k[slot * a.scr_KC + pos] = key;
                a.scr_i[slot * a.scr_KC + pos] = grow;
            }
        }
    }
}
// Staged screening epilogue (k_gemm8 / k_gemm8s): the survivors of a wave are
// first compacted into a wave-private LDS list (ballot + mbcnt: no atomics, no
// waits), and appended to their (query, chunk) slots in batches of 64, one
// lane per survivor, so a wave waits for one round of atomic returns per 64
// survivors instead of one per fragment that holds a survivor.  Which KC of an
// overflowing slot's survivors are stored does not matter: k_slot_fixup
// rebuilds every slot whose count exceeds KC, and a slot's candidates are a set
// (the final select orders them by key, then row).  Every lane of the wave must
// call add() / flush() (full-wave control flow): validity goes in `ok`.
struct ScreenStage {
    static constexpr int CAP = 128;  // entries per wave: key, global row, query (3 words each)
    uint32_t* e;                     // this wave's LDS list
    int n;                           // staged entries (wave-uniform)
    __device__ __forceinline__ void flush(const ConvArgs& a) {
        const int lane = threadIdx.x & 63;
        for (int b = 0; b < n; b += 64) {
            const int k = b + lane;
            if (k < n) {
                const uint32_t key = e[3 * k], grow = e[3 * k + 1], p = e[3 * k + 2];
                const long long slot = (long long)p * a.scr_nchunks + (int)grow / a.scr_L;
                const int pos = atomicAdd(a.scr_cnt + slot, 1);
                if (pos < a.scr_KC) {
                    a.scr_k[slot * a.scr_KC + pos] = key;
                    a.scr_i[slot * a.scr_KC + pos] = (int)grow;
                }
            }
        }
        n = 0;
    }
    // scores v[0..3] of database rows c..c+3 (valid: < rows) and query p (valid: ok)
    __device__ __forceinline__ void add(const ConvArgs& a, const float* v, int c, int rows, int p, bool ok,
                                        uint32_t tau) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t key = score_key(v[r]);
            const bool s = ok && c + r < rows && key >= tau;
            const unsigned long long m = __ballot(s);
            if (m == 0ull) continue;  // wave-uniform
            if (n + 64 > CAP) flush(a);
            if (s) {
                const int k = n + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                e[3 * k] = key;
                e[3 * k + 1] = (uint32_t)(a.scr_row0 + c + r);
                e[3 * k + 2] = (uint32_t)p;
            }
            n += __popcll(m);
        }
    }
};
// scores[p][c] (f32, row stride ldy) = x[p][:] . w[c][:], 1x1 GEMM, dtype in.
void gemm_scores(const ConvArgs& a, int dtype, hipStream_t s);
// the same on int8-quantised rows (rr_gemm.hip): float(exact int32 dot product)
int gemm_scores_i8(const ConvArgs& a, hipStream_t s);

// RR_CONV_PERM32 row order: packed row g*32 + i*16 + 4q + r holds channel g*32 + 8q + 4i + r.
__host__ __device__ __forceinline__ int perm32_channel(int packed_row) {
    return (packed_row & ~31) | (((packed_row & 15) >> 2) << 3) | (((packed_row >> 4) & 1) << 2) | (packed_row & 3);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

}  // namespace rr
