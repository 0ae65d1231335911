// librr.so — full ranking: the GPU form of
//     scores = np.dot(vecs.T, qvecs); ranks = np.argsort(-scores, axis=0)
// (scripts/test.py:247-248, train_globalF.py:733-734) for any database size
// (rr_knn_topk sorts its candidates in LDS, so it covers k <= 8192 only; a
// revisited-dataset evaluation with distractors ranks every database item).
//
// Order: score descending, database index ascending — the order rr_knn_topk
// emits, with the SAME float64 score: the exact float64 products of the
// float32 rows summed in k_rescore's order (lane l accumulates t = 4l + 256s
// + e, then the xor butterfly 32, 16, .., 1), so the first k ranks here are
// bit-identical to a top-k search.
//
//  k_rank_scores   one wave per (2 database rows, 16 queries): the queries
//                  staged in LDS (float32), float64 FMAs, butterfly per pair;
//                  writes the radix key ~order(score) (ascending key = score
//                  descending) and the row index
//  k_radix_hist / k_radix_scan / k_radix_scatter
//                  stable LSD radix sort of the 64-bit keys per query, 8
//                  passes of 8-bit digits over 4096-element tiles; the stable
//                  scatter keeps equal keys in index order (the input is in
//                  index order), which is the (score desc, index asc) rule.
#include "rr_internal.h"

#include <utility>

namespace rr {

namespace {

constexpr int RQG = 16;          // queries per score wave
constexpr int RTILE = 4096;      // radix tile (elements)
constexpr int RT = 256;          // radix threads per block
constexpr int RROUNDS = RTILE / RT;

__device__ __forceinline__ unsigned long long order_key_desc(double s) {
    unsigned long long u = __double_as_longlong(s);
    u = (u >> 63) ? ~u : (u | 0x8000000000000000ull);  // ascending u <-> ascending score
    return ~u;                                         // ascending key <-> descending score
}

// grid (blocks, ceil(nq / 16)), 512 threads: persistent over row pairs (8 waves x 2 rows
// per block step), the block's 16 queries staged once in LDS; d % 256 == 0
__global__ void __launch_bounds__(512) k_rank_scores(const float* __restrict__ db32, long long n,
                                                     const float* __restrict__ q32, int nq, int d,
                                                     unsigned long long* __restrict__ keys,
                                                     unsigned* __restrict__ idx) {
    extern __shared__ __attribute__((aligned(16))) float sq[];  // [RQG][d]
    const int q0 = blockIdx.y * RQG;
    const int nqg = min(RQG, nq - q0);
    for (int i = threadIdx.x * 4; i < RQG * d; i += 512 * 4) {
        const int qq = i / d, t = i - qq * d;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (qq < nqg) v = *reinterpret_cast<const float4*>(q32 + (long long)(q0 + qq) * d + t);
        *reinterpret_cast<float4*>(sq + i) = v;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (long long r0 = ((long long)blockIdx.x * 8 + wave) * 2; r0 < n; r0 += (long long)gridDim.x * 16) {
        double acc[2][RQG];
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int qq = 0; qq < RQG; ++qq) acc[r][qq] = 0.0;
        const float* d0 = db32 + r0 * d;
        const float* d1 = db32 + (r0 + 1 < n ? r0 + 1 : r0) * d;
        for (int t = lane * 4; t < d; t += 256) {
            const float4 x0 = *reinterpret_cast<const float4*>(d0 + t);
            const float4 x1 = *reinterpret_cast<const float4*>(d1 + t);
#pragma unroll
            for (int qq = 0; qq < RQG; ++qq) {
                const float4 y = *reinterpret_cast<const float4*>(sq + qq * d + t);
                acc[0][qq] = fma((double)x0.x, (double)y.x, acc[0][qq]);
                acc[0][qq] = fma((double)x0.y, (double)y.y, acc[0][qq]);
                acc[0][qq] = fma((double)x0.z, (double)y.z, acc[0][qq]);
                acc[0][qq] = fma((double)x0.w, (double)y.w, acc[0][qq]);
                acc[1][qq] = fma((double)x1.x, (double)y.x, acc[1][qq]);
                acc[1][qq] = fma((double)x1.y, (double)y.y, acc[1][qq]);
                acc[1][qq] = fma((double)x1.z, (double)y.z, acc[1][qq]);
                acc[1][qq] = fma((double)x1.w, (double)y.w, acc[1][qq]);
            }
        }
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int qq = 0; qq < RQG; ++qq) {
                const double sc = wave_sum_d(acc[r][qq]);  // k_rescore's butterfly
                const long long row = r0 + r;
                if (lane == qq && qq < nqg && row < n) {
                    keys[(long long)(q0 + qq) * n + row] = order_key_desc(sc);
                    idx[(long long)(q0 + qq) * n + row] = (unsigned)row;
                }
            }
    }
}

// digit histogram of tile blockIdx.x of query blockIdx.y -> hist[q][digit][tile]
__global__ void __launch_bounds__(RT) k_radix_hist(const unsigned long long* __restrict__ keys, long long n,
                                                   int ntiles, int shift, unsigned* __restrict__ hist) {
    __shared__ unsigned h[256];
    const int q = blockIdx.y, tile = blockIdx.x;
    h[threadIdx.x] = 0;
    __syncthreads();
    const unsigned long long* k = keys + (long long)q * n;
    const long long e0 = (long long)tile * RTILE;
    for (int r = 0; r < RROUNDS; ++r) {
        const long long e = e0 + r * RT + threadIdx.x;
        if (e < n) atomicAdd(&h[(unsigned)(k[e] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[((long long)q * 256 + threadIdx.x) * ntiles + tile] = h[threadIdx.x];
}

// exclusive scan of hist[q][*][*] (digit-major) in place; one block per query
__global__ void __launch_bounds__(1024) k_radix_scan(unsigned* __restrict__ hist, int ntiles) {
    __shared__ unsigned part[1024];
    const int q = blockIdx.x;
    unsigned* h = hist + (long long)q * 256 * ntiles;
    const long long m = 256ll * ntiles;
    const long long per = (m + 1023) / 1024;
    const long long b = threadIdx.x * per, e = min(m, b + per);
    unsigned s = 0;
    for (long long i = b; i < e; ++i) s += h[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan of the thread sums
        const unsigned v = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    unsigned run = threadIdx.x ? part[threadIdx.x - 1] : 0u;
    for (long long i = b; i < e; ++i) {
        const unsigned c = h[i];
        h[i] = run;
        run += c;
    }
}

// stable scatter of tile blockIdx.x of query blockIdx.y by the digit at `shift`;
// out_idx64 != nullptr (last pass): write the row indices as int64 ranks
__global__ void __launch_bounds__(RT) k_radix_scatter(const unsigned long long* __restrict__ kin,
                                                      const unsigned* __restrict__ iin, long long n, int ntiles,
                                                      int shift, const unsigned* __restrict__ offs,
                                                      unsigned long long* __restrict__ kout,
                                                      unsigned* __restrict__ iout, long long* __restrict__ out_idx64) {
    __shared__ unsigned base[256], run[256], cnt[RT / 64][256];
    const int q = blockIdx.y, tile = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    base[tid] = offs[((long long)q * 256 + tid) * ntiles + tile];
    run[tid] = 0;
    const long long qo = (long long)q * n;
    const long long e0 = (long long)tile * RTILE;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int r = 0; r < RROUNDS; ++r) {
        for (int w = 0; w < RT / 64; ++w) cnt[w][tid] = 0;
        __syncthreads();
        const long long e = e0 + r * RT + tid;
        const bool live = e < n;
        unsigned long long key = live ? kin[qo + e] : 0ull;
        const unsigned id = live ? iin[qo + e] : 0u;
        const unsigned dg = (unsigned)(key >> shift) & 255u;
        // lanes of this wave with the same digit (live ones only)
        unsigned long long same = __ballot(live);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const unsigned long long bb = __ballot((dg >> bit) & 1u);
            same &= ((dg >> bit) & 1u) ? bb : ~bb;
        }
        const unsigned wrank = __popcll(same & lt);
        if (live && wrank == 0) cnt[wave][dg] = __popcll(same);
        __syncthreads();
        if (live) {
            unsigned pre = 0;
            for (int w = 0; w < wave; ++w) pre += cnt[w][dg];
            const long long pos = qo + base[dg] + run[dg] + pre + wrank;
            if (out_idx64) out_idx64[pos] = (long long)id;
            else {
                kout[pos] = key;
                iout[pos] = id;
            }
        }
        __syncthreads();
        unsigned tot = 0;
        for (int w = 0; w < RT / 64; ++w) tot += cnt[w][tid];
        run[tid] += tot;
    }
}

struct RankPlan {
    int ntiles;
    size_t keys_bytes, idx_bytes, hist_bytes, total;
};

RankPlan rank_plan(long long n, int nq) {
    RankPlan p;
    p.ntiles = (int)((n + RTILE - 1) / RTILE);
    p.keys_bytes = ((size_t)nq * n * 8 + 255) / 256 * 256;
    p.idx_bytes = ((size_t)nq * n * 4 + 255) / 256 * 256;
    p.hist_bytes = ((size_t)nq * 256 * p.ntiles * 4 + 255) / 256 * 256;
    p.total = 2 * p.keys_bytes + 2 * p.idx_bytes + p.hist_bytes;
    return p;
}

}  // namespace
}  // namespace rr

using namespace rr;

extern "C" {

size_t rr_rank_workspace_bytes(long long n, int nq) {
    if (n <= 0 || nq <= 0) return 0;
    return rank_plan(n, nq).total;
}

int rr_rank_full(const float* db_f32, long long n, const float* q_f32, int nq, int d, long long* out_idx,
                 void* workspace, size_t workspace_bytes, void* stream) {
    if (n <= 0 || nq <= 0) return fail(RR_EINVAL, "rr_rank_full: empty problem");
    if (n > 0xffffffffll) return fail(RR_EINVAL, "rr_rank_full: more than 2^32 rows");
    if (d <= 0 || d % 256) return fail(RR_EINVAL, "rr_rank_full: d must be a multiple of 256 (zero-pad)");
    if ((size_t)RQG * d * 4 > 160 * 1024) return fail(RR_EINVAL, "rr_rank_full: d too large for the LDS query tile");
    const RankPlan p = rank_plan(n, nq);
    if (!workspace || workspace_bytes < p.total) return fail(RR_ENOSPACE, "rr_rank_full: workspace too small");
    if (nq > 65535) return fail(RR_EINVAL, "rr_rank_full: more than 65535 queries per call (grid y); split them");
    if ((long long)nq * p.ntiles > 0x7fffffffll)
        return fail(RR_EINVAL, "rr_rank_full: problem too large");
    hipStream_t s = as_stream(stream);
    char* ws = (char*)workspace;
    unsigned long long* k0 = (unsigned long long*)ws;
    unsigned long long* k1 = (unsigned long long*)(ws + p.keys_bytes);
    unsigned* i0 = (unsigned*)(ws + 2 * p.keys_bytes);
    unsigned* i1 = (unsigned*)(ws + 2 * p.keys_bytes + p.idx_bytes);
    unsigned* hist = (unsigned*)(ws + 2 * p.keys_bytes + 2 * p.idx_bytes);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_rank_scores, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    const long long pairs = (n + 15) / 16;
    const unsigned gx = (unsigned)(pairs < 4ll * grid_cus() ? pairs : 4ll * grid_cus());
    hipLaunchKernelGGL(k_rank_scores, dim3(gx, (unsigned)((nq + RQG - 1) / RQG)), dim3(512), (size_t)RQG * d * 4, s,
                       db_f32, n, q_f32, nq, d, k0, i0);
    const dim3 g((unsigned)p.ntiles, (unsigned)nq);
    for (int pass = 0; pass < 8; ++pass) {
        const int shift = pass * 8;
        hipLaunchKernelGGL(k_radix_hist, g, dim3(RT), 0, s, k0, n, p.ntiles, shift, hist);
        hipLaunchKernelGGL(k_radix_scan, dim3(nq), dim3(1024), 0, s, hist, p.ntiles);
        hipLaunchKernelGGL(k_radix_scatter, g, dim3(RT), 0, s, k0, i0, n, p.ntiles, shift, hist, k1, i1,
                           pass == 7 ? out_idx : (long long*)nullptr);
        std::swap(k0, k1);
        std::swap(i0, i1);
    }
    return check_launch("rr_rank_full");
}

}  // extern "C"
