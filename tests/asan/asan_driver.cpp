// Host half of librr under AddressSanitizer (SURVEY §5 "Race detection /
// sanitizers").  Built by `make -C <csrc> asan` against librr_asan.so (every
// .hip compiled host-only with -fsanitize=address: no device code objects, so
// a launch that gets past the host checks fails with a HIP error instead of
// running).  Drives, on a host without a GPU:
//  * the workspace sizing of every entry point that has one, over a grid of sizes;
//  * the argument checks of the entry points (null / negative / unsupported
//    arguments must return RR_EINVAL / RR_ENOSPACE with a message, never touch memory);
//  * the ragged-batch table packing (> 64 images -> several launches, host arrays
//    of pointers and extents read in full);
//  * rr_set_tuning, rr_last_error, rr_comm_unique_id (RCCL dlopen'ed).
// Exit status 0 and the last line "ASAN-DRIVER OK" when nothing was reported.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/rr.h"

static int g_fail = 0;
#define EXPECT(cond)                                                               \
    do {                                                                           \
        if (!(cond)) {                                                             \
            std::fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond, \
                         rr_last_error());                                         \
            ++g_fail;                                                              \
        }                                                                          \
    } while (0)

// a non-null, never-dereferenced stand-in for a device address
static void* fake(size_t off = 0) { return reinterpret_cast<void*>(static_cast<uintptr_t>(0x100000000ull + off)); }

int main() {
    EXPECT(rr_version() > 0);
    EXPECT(rr_last_error() != nullptr);

    // --- workspace sizing
    for (long long n : {1ll, 1000ll, 65536ll, 1000000ll, 10000000ll})
        for (int nq : {1, 70, 128, 1024})
            for (int dt : {RR_F32, RR_BF16, RR_F16, RR_I8}) {
                const size_t b = rr_knn_workspace_bytes(n, nq, 2048, 100, 0, dt);
                EXPECT(b > 0);
                EXPECT(rr_knn_workspace_bytes(n, nq, 2048, 100, 4096, dt) >= b);
            }
    EXPECT(rr_knn_workspace_bytes(0, 10, 2048, 10, 0, RR_F32) == 0);
    for (int rows : {1, 5, 128, 5063}) {
        EXPECT(rr_head_workspace_bytes(rows, 2048) > 0);
        EXPECT(rr_whiten_workspace_bytes(rows, 2048) > 0);
    }
    for (int r : {1, 2, 8}) EXPECT(rr_topk_allgather_workspace_bytes(r, 1024, 100) >= (size_t)r * 1024 * 100 * 16);
    EXPECT(rr_rank_workspace_bytes(5000, 70) > 0);
    EXPECT(rr_local_head_workspace_bytes(8 * 2048, 1024, 128) > 0);

    // --- argument checks (each must fail cleanly)
    double s[4];
    long long ix[4];
    EXPECT(rr_knn_topk(nullptr, nullptr, 0, nullptr, nullptr, 1, 64, 1, 0, 0, s, ix, nullptr, 0, RR_F32, nullptr) ==
           RR_EINVAL);
    EXPECT(rr_knn_topk(fake(), (const float*)fake(), 100, fake(), (const float*)fake(), 1, 48, 1, 0, 0, s, ix,
                       fake(), 1 << 20, RR_F32, nullptr) == RR_EINVAL);          // d not a power of two
    EXPECT(rr_knn_topk(fake(), (const float*)fake(), 100, fake(), (const float*)fake(), 1, 64, 1, 0, 0, s, ix,
                       fake(), 1 << 20, 7, nullptr) == RR_EINVAL);               // dtype
    EXPECT(rr_knn_topk(fake(), (const float*)fake(), 100, fake(), (const float*)fake(), 200, 128, 1, 0, 0, s, ix,
                       fake(), 1 << 30, RR_I8, nullptr) == RR_EINVAL);           // int8 d = 128 above 128 queries
    EXPECT(rr_knn_topk(fake(), (const float*)fake(), 100, fake(), (const float*)fake(), 1, 64, 5, 3, 0, s, ix,
                       fake(), 1 << 20, RR_F32, nullptr) == RR_EINVAL);          // cand < k
    EXPECT(rr_knn_topk(fake(), (const float*)fake(), 100000, fake(), (const float*)fake(), 4, 256, 10, 0, 0, s, ix,
                       fake(), 16, RR_BF16, nullptr) == RR_ENOSPACE);            // workspace too small
    EXPECT(rr_knn_topk_checked_i8(fake(), (const float*)fake(), 100, fake(), (const float*)fake(), 1, 256, 1, 0, 0,
                                  s, ix, fake(), 1 << 20, 1.f, nullptr, 1, nullptr, nullptr, nullptr) == RR_EINVAL);
    EXPECT(rr_topk_merge(nullptr, nullptr, 0, 1, 1, 1, s, ix, nullptr) == RR_EINVAL);
    EXPECT(rr_topk_merge((const double*)fake(), (const long long*)fake(), 8, 1, 4096, 10, s, ix, nullptr) == RR_EINVAL);
    EXPECT(rr_quantize_i8(nullptr, 16, fake(), (float*)fake(), nullptr) == RR_EINVAL);
    EXPECT(rr_quantize_i8((const float*)fake(), 15, fake(), (float*)fake(), nullptr) == RR_EINVAL);
    EXPECT(rr_quantize_i8_rows(nullptr, 4, 16, fake(), (float*)fake(), nullptr) == RR_EINVAL);
    EXPECT(rr_quantize_i8_rows((const float*)fake(), 4, 18, fake(), (float*)fake(), nullptr) == RR_EINVAL);
    EXPECT(rr_quantize_i8_rows((const float*)fake(), 0, 18, fake(), (float*)fake(), nullptr) == RR_OK);

    rr_conv_desc d;
    std::memset(&d, 0, sizeof d);
    d.n = 1; d.h = 8; d.w = 8; d.c_in = 48;  // c_in not a power of two
    d.ho = 8; d.wo = 8; d.c_out = 64; d.kh = d.kw = 1; d.stride = 1; d.dil = 1; d.k_packed = 64; d.ldy = 64;
    EXPECT(rr_conv2d_fused(fake(), fake(), (const float*)fake(), (const float*)fake(), nullptr, fake(), &d, RR_BF16,
                           RR_BF16, nullptr) != RR_OK);
    EXPECT(rr_conv2d_fused(fake(), fake(), nullptr, nullptr, nullptr, fake(), nullptr, RR_BF16, RR_BF16, nullptr) !=
           RR_OK);
    EXPECT(rr_conv1x1_pair(fake(), 100, 32, fake(), nullptr, nullptr, 256, nullptr, nullptr, nullptr, nullptr,
                           nullptr, 1, 0.01f, fake(), nullptr, nullptr, 64, 1, 0.01f, fake(), fake(), RR_BF16,
                           nullptr) == RR_EINVAL);                                // c_in 32: no fused form
    const float* ff = (const float*)fake();
    EXPECT(rr_conv3x3_pair(fake(), 2, 18, 64, nullptr, nullptr, nullptr, 0, 0.f, fake(), ff, ff, 1, 0.01f, fake(), ff, ff, fake(), nullptr, nullptr,
                           nullptr, nullptr, 1, 0.01f, fake(), ff, ff, 64, 1, 0.01f, fake(), fake(), nullptr, RR_BF16,
                           nullptr) == RR_EINVAL);                                // h % 4
    EXPECT(rr_conv3x3_pair(fake(), 2, 16, 64, nullptr, nullptr, nullptr, 0, 0.f, fake(), ff, ff, 1, 0.01f, fake(), ff, ff, nullptr, fake(), fake(),
                           ff, ff, 1, 0.01f, fake(), ff, ff, 128, 1, 0.01f, fake(), fake(), nullptr, RR_F16,
                           nullptr) == RR_EINVAL);                                // projection form with c_out 128
    EXPECT(rr_conv3x3_pair(fake(), 2, 16, 64, nullptr, nullptr, nullptr, 0, 0.f, fake(), ff, ff, 1, 0.01f, fake(), ff, ff, fake(), nullptr, nullptr,
                           nullptr, nullptr, 1, 0.01f, fake(), ff, ff, 64, 1, 0.01f, fake(), fake(), nullptr, RR_F32,
                           nullptr) == RR_EINVAL);                                // 16-bit only

    // --- ragged batches: 150 images (3 launches of <= 64), host tables read in full
    const int n = 150;
    std::vector<const void*> srcs(n);
    std::vector<int> ext(2 * n);
    for (int i = 0; i < n; ++i) {
        srcs[i] = (i % 17 == 5) ? nullptr : fake((size_t)i << 24);
        ext[2 * i] = (i % 17 == 5) ? 0 : 64 + (i * 7) % 64;
        ext[2 * i + 1] = (i % 17 == 5) ? 0 : 96 + (i * 13) % 32;
    }
    const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
    // no device code in this build: each call gets through its table packing, then the launch fails
    const int r1 = rr_image_to_nhwc_ragged(srcs.data(), ext.data(), n, 3, 128, 128, 0, mean, stdv, 1, fake(), 4,
                                           RR_BF16, nullptr);
    EXPECT(r1 != RR_OK);
    const int r2 = rr_stem_conv_pool_ragged(srcs.data(), ext.data(), n, 128, 128, 1, mean, stdv, 1, fake(),
                                            (const float*)fake(), (const float*)fake(), RR_ACT_LEAKY, 0.01f, fake(),
                                            32, 32, RR_F16, nullptr);
    EXPECT(r2 != RR_OK);
    const float pad0 = 0.f;
    const int r3 = rr_pad_images(srcs.data(), ext.data(), n, 3, 128, 128, 4, &pad0, fake(), nullptr);
    EXPECT(r3 != RR_OK);
    ext[3] = 129;  // an extent larger than the batch map
    EXPECT(rr_image_to_nhwc_ragged(srcs.data(), ext.data(), n, 3, 128, 128, 0, mean, stdv, 1, fake(), 4, RR_BF16,
                                   nullptr) == RR_EINVAL);
    EXPECT(rr_pad_images(srcs.data(), ext.data(), n, 3, 128, 128, 3, &pad0, fake(), nullptr) == RR_EINVAL);

    // --- tuning knobs
    EXPECT(rr_set_tuning(7, 64) == RR_OK);
    EXPECT(rr_set_tuning(7, 0) == RR_OK);
    EXPECT(rr_set_tuning(-1, 0) != RR_OK);
    EXPECT(rr_set_tuning(1 << 20, 0) != RR_OK);

    // --- RCCL id (librccl dlopen'ed; any outcome is fine, it must not corrupt memory)
    char id[256];
    const int rc = rr_comm_unique_id(id, 256);
    std::printf("rr_comm_unique_id -> %d (%s)\n", rc, rc ? rr_last_error() : "ok");
    EXPECT(rr_comm_unique_id(id, 16) == RR_EINVAL);

    std::printf("%d check(s) failed\n", g_fail);
    if (g_fail) return 1;
    std::printf("ASAN-DRIVER OK\n");
    return 0;
}
