/*
 * rr.h — C ABI of librr.so, the MI355X (gfx950) extract-and-match engine.
 *
 * The reference (Tarekbouamer/Image-Retrieval-for-Image-Based-Localization,
 * package `cirtorch`) is pure Python: its hot path is a chain of torch
 * nn.Modules plus two numpy calls.  Each entry point below replaces one
 * reference operator; the Python host package `cirtorch` (same module names,
 * same argument meaning) binds them with ctypes — see INTEGRATION.md.
 *
 * Conventions
 *   - every function returns 0 on success, a negative code on error;
 *     rr_last_error() returns the message (thread-local).
 *   - all tensor pointers are DEVICE pointers; nothing here allocates:
 *     scratch is caller-provided and sized by the matching *_workspace_bytes.
 *   - `stream` is a hipStream_t (NULL = default stream); every call only
 *     enqueues work (no host synchronisation), so calls are graph-capturable.
 *   - activations are NHWC ("channels_last"); dtype codes below.
 *   - re-entrant; one process per GPU.
 */
#ifndef RR_H_
#define RR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 16-bit types: every conv kernel; RR_F16 also kNN screening; RR_I8: kNN screening only (rr_quantize_i8) */
enum rr_dtype { RR_F32 = 0, RR_BF16 = 1, RR_F16 = 2, RR_I8 = 3 };
enum rr_act { RR_ACT_IDENTITY = 0, RR_ACT_LEAKY = 1 };
enum rr_pool_mode { RR_POOL_GEM = 0, RR_POOL_MAC = 1, RR_POOL_SPOC = 2 };
enum rr_conv_flags { RR_CONV_AFFINE = 1, RR_CONV_RESIDUAL = 2, RR_CONV_PERM32 = 4 };
enum rr_layout { RR_NHWC = 0, RR_NCHW = 1 };

#define RR_OK 0
#define RR_EINVAL -1
#define RR_EHIP -2
#define RR_ENOSPACE -3

/* ------------------------------------------------------------------ runtime */
int rr_version(void);
/* "source_digest=<12 hex> arch=gfx950": the sha1 digest of the csrc .hip / .h sources and this
 * header the library was built from (tools/src_digest.py), for the provenance of a prebuilt
 * librr.so. */
const char* rr_build_info(void);
const char* rr_last_error(void);
/* Device architecture name of the current device (e.g. "gfx950"). */
int rr_device_arch(char* buf, int buflen);

/* ------------------------------------------------------------ extractor ops */

/* NCHW float32 image batch -> NHWC `dtype` with `c_pad` channels (zeros in the
 * pad channels), optionally (x - mean_c) / std_c.
 * Replaces cirtorch/utils/image.py:86-127 `normalize` (called from
 * datasets/augmentation/random_augmentation.py:174) fused with the layout
 * change the conv stack needs.  mean/std are HOST arrays of c floats. */
int rr_image_to_nhwc(const float* src, int n, int c, int h, int w,
                     const float* mean_host, const float* std_host, int do_normalize,
                     void* dst, int c_pad, int dtype, void* stream);

/* Implicit-GEMM convolution on MFMA with a fused epilogue:
 *   y = act( conv(x, w) * scale[c] + shift[c] (+ residual) )
 * Replaces nn.Conv2d (cirtorch/backbones/resnet.py:61, backbones/misc.py:166-180)
 * followed by the inplace_abn ABN eval BN + leaky_relu / identity
 * (utils/misc.py:175-235) and the residual add + activation of
 * ResidualBlock.forward (backbones/misc.py:184-203).
 *   x  : [n][h][w][c_in]            (dtype)
 *   w  : [c_out][k_packed]          (dtype) k = (kh*KW + kw)*c_in + ci, zero padded
 *   y  : [n*ho*wo][ldy]             (out_dtype), channel c at column c
 *   residual : same layout/dtype as y (flag RR_CONV_RESIDUAL)
 *   RR_CONV_PERM32: w rows are in the 32-row MFMA-interleaved order written by
 *   rr_pack_conv_weights(perm32=1) (c_out % 32 == 0); y is still in natural
 *   channel order.  scale/shift are always indexed by the natural channel.
 * Also used as the score GEMM of the kNN (1x1, ldy = slab width). */
typedef struct rr_conv_desc {
    int n, h, w, c_in;     /* input; c_in = channel stride, power of two */
    int ho, wo, c_out;     /* output */
    int kh, kw, stride, pad, dil;
    int k_packed;          /* weight row length, multiple of 32 */
    int ldy;               /* output row stride in elements (>= c_out) */
    int act;               /* rr_act */
    float slope;           /* leaky slope */
    int flags;             /* rr_conv_flags */
} rr_conv_desc;

int rr_conv2d_fused(const void* x, const void* w, const float* scale, const float* shift,
                    const void* residual, void* y, const rr_conv_desc* desc,
                    int dtype, int out_dtype, void* stream);

/* Pack nn.Conv2d weights w[c_out][c_in][kh][kw] (float32, the reference
 * state-dict layout, cirtorch/backbones/resnet.py:61) into the engine layout
 * out[c_out][k_packed] (`dtype`), k = (kh*KW + kw)*c_in_pad + ci, zero padded
 * channels and K tail; perm32 != 0 stores rows in the RR_CONV_PERM32 order. */
int rr_pack_conv_weights(const float* w, int c_out, int c_in, int kh, int kw, int c_in_pad,
                         int k_packed, int perm32, void* out, int dtype, void* stream);

/* Fused bottleneck boundary, bf16 or fp16 (dtype), PERM32-packed weights (1x1 convs):
 *   y = act3(conv1x1(x, w3) * scale3 + shift3 + shortcut)      [p][c_mid]
 *   z = act1(conv1x1(y, w1) * scale1 + shift1)                 [p][c_out]
 * i.e. conv3 + bn3 + residual add + activation of ResidualBlock i and conv1 +
 * bn1 + activation of block i + 1 (cirtorch/backbones/misc.py:166-203), in one
 * pass that never re-reads y.  shortcut = residual ([p][c_mid]) when given;
 * with residual == NULL it is the block's projection proj_bn(proj_conv(xp))
 * (1x1 stride 1, xp [p][c_in], wp [c_mid][c_in], scalep/shiftp; misc.py:179-182)
 * computed in the same pass.  p = pixels (n*h*w, stride 1).  Shapes: c_in 64,
 * c_mid 256, c_out 64 or 128 (the 256-channel stage); anything else returns
 * RR_EINVAL and the caller runs separate rr_conv2d_fused launches instead. */
int rr_conv1x1_pair(const void* x, long long p, int c_in, const void* w3, const float* scale3,
                    const float* shift3, int c_mid, const void* residual, const void* xp, const void* wp,
                    const float* scalep, const float* shiftp, int act3, float slope3, const void* w1,
                    const float* scale1, const float* shift1, int c_out, int act1, float slope1, void* y,
                    void* z, int dtype, void* stream);

/* One bottleneck block of the 256-channel stage fused (bf16 or fp16 dtype, PERM32 weights):
 *   t2 = act2(conv3x3(t1, w33) * scale2 + shift2)                 3x3 / s1 / p1, 64 -> 64
 *   y  = act3(conv1x1(t2, w3) * scale3 + shift3 + shortcut)       64 -> 256
 *   z  = act1(conv1x1(y, w1) * scale1 + shift1)                   256 -> c_out (64 or 128)
 * conv2 .. conv3 + residual of ResidualBlock i and conv1 of block i + 1
 * (cirtorch/backbones/misc.py:163-203) in one pass: t2 never reaches HBM and the 3x3's
 * matrix work runs beside the boundary's memory traffic.  shortcut = residual ([p][256]) or,
 * with residual == NULL, the projection proj_bn(proj_conv(xp)) (c_out 64).  t1 [n][h][w][64],
 * h % 4 == 0, w % 32 == 0; y / z bit-identical to the unfused launches (the 3x3 kernel +
 * rr_conv1x1_pair).  RR_EINVAL for other shapes (the caller runs those launches instead).
 * w0 (PERM32 [64][64]) or NULL: with w0 (projection form only) t1 is the block's input x and
 * conv1 + bn1 + act0 of the block (t1 = act0(conv1x1(x, w0) * scale0 + shift0)) runs in the
 * same launch; pass x as xp too.  Bit-identical to rr_conv2d_fused of conv1 first.
 * tile_queue: 8 ints, zero on entry, used as per-XCD tile counters (blocks that start late
 * take fewer tiles; the kernel leaves them non-zero, so one zeroed array per launch), or
 * NULL for the static tile walk; the results do not depend on it. */
int rr_conv3x3_pair(const void* t1, int n, int h, int w, const void* w0, const float* scale0,
                    const float* shift0, int act0, float slope0, const void* w33, const float* scale2,
                    const float* shift2, int act2, float slope2, const void* w3, const float* scale3,
                    const float* shift3, const void* residual, const void* xp, const void* wp,
                    const float* scalep, const float* shiftp, int act3, float slope3, const void* w1,
                    const float* scale1, const float* shift1, int c_out, int act1, float slope1, void* y,
                    void* z, int* tile_queue, int dtype, void* stream);

/* 3x3/s2/p1 style max pooling, NHWC.  Replaces nn.MaxPool2d(3, stride=2,
 * padding=1) of the stem (cirtorch/backbones/resnet.py:65). */
int rr_maxpool2d(const void* x, int n, int h, int w, int c, int k, int stride, int pad,
                 void* y, int ho, int wo, int dtype, void* stream);

/* Fused ResNet stem, bf16 or fp16 (dtype): normalise + conv1 7x7/s2/p3 (3 -> 64) + BN affine
 * + activation + max-pool 3x3/s2/p1 in one kernel.  Replaces mod1 =
 * Sequential(conv1, bn1, pool1) of cirtorch/backbones/resnet.py:59-66 applied
 * to the output of utils/image.py:125 `normalize`.
 *   x     : [n][3][h][w] float32 (raw pixels when do_normalize, mean/std HOST arrays of 3)
 *   wpk   : rr_stem_pack_weights output, [64][448] (dtype): the kernel-row layout (k < 256) and the
 *           space-to-depth layout (k >= 256) of the two stem kernel families
 *   scale, shift : [64] float32 (folded BN), act RR_ACT_*, slope for leaky
 *   y     : [n][hp][wp][64] (dtype), hp/wp = the pool of the (h+1)/2 x (w+1)/2 stem map */
int rr_stem_pack_weights(const float* w, int c_out, int c_in, int kh, int kw, void* out, int dtype, void* stream);
int rr_stem_conv_pool(const float* x, int n, int h, int w, const float* mean_host, const float* std_host,
                      int do_normalize, const void* wpk, const float* scale, const float* shift, int act,
                      float slope, void* y, int hp, int wp, int dtype, void* stream);
/* Same, on uint8 pixels [n][3][h][w]: each value is x / 255 in float32 (the
 * torchvision ToTensor the reference's loaders apply, datasets/generic/
 * transform.py:128), so the result equals rr_stem_conv_pool on x / 255.
 * A decoded image crosses PCIe as 1 B per channel instead of 4. */
int rr_stem_conv_pool_u8(const unsigned char* x, int n, int h, int w, const float* mean_host,
                         const float* std_host, int do_normalize, const void* wpk, const float* scale,
                         const float* shift, int act, float slope, void* y, int hp, int wp, int dtype,
                         void* stream);

/* ---- ragged image batches (a PackedSequence of different-size images) ----
 * Replace pad_packed_images (cirtorch/utils/sequence.py:4-67) + normalize
 * (utils/image.py:125) on a cirtorch.utils.parallel.PackedSequence
 * (utils/parallel/packed_sequence.py:8-96) feeding the body: image i is
 * [c][h_i][w_i] at its own DEVICE address srcs[i] (NULL with h_i = w_i = 0 for
 * a None entry); `extents` is a HOST array {h_0, w_0, h_1, w_1, ...}; the
 * batch map is h x w (>= every extent).  Map pixels outside image i read as 0
 * (the reference's top-left zero pad) BEFORE normalisation -- in-tree order,
 * random_augmentation.py:102 then :174 -- so a pad becomes -mean/std when
 * do_normalize.  No padded copy of the batch is written; `srcs` are read
 * directly.  u8: srcs are uint8 pixels read as x / 255 (to_tensor), else
 * float32.  Any n (split internally into launches of <= 64 images). */
int rr_image_to_nhwc_ragged(const void* const* srcs, const int* extents, int n, int c, int h, int w, int u8,
                            const float* mean_host, const float* std_host, int do_normalize,
                            void* dst, int c_pad, int dtype, void* stream);
/* The fused stem (rr_stem_conv_pool) on a ragged batch; y is [n][hp][wp][64]
 * of the h x w batch map.  Results equal rr_stem_conv_pool(_u8) on the padded
 * batch bit for bit. */
int rr_stem_conv_pool_ragged(const void* const* srcs, const int* extents, int n, int h, int w, int u8,
                             const float* mean_host, const float* std_host, int do_normalize, const void* wpk,
                             const float* scale, const float* shift, int act, float slope, void* y, int hp, int wp,
                             int dtype, void* stream);
/* pad_packed_images itself (utils/sequence.py:4-67) for device tensors: one
 * launch writes the [n][c][h][w] padded batch (elements of elem_bytes = 1, 2,
 * 4 or 8 bytes; pad_value points to one HOST element) from the ragged list. */
int rr_pad_images(const void* const* srcs, const int* extents, int n, int c, int h, int w, int elem_bytes,
                  const void* pad_value_host, void* dst, void* stream);

/* Bilinear resize, align_corners=False, NCHW float32 (one image).
 * Replaces nn.functional.interpolate(scale_factor=s, mode='bilinear',
 * align_corners=False) of the multi-scale pyramid (cirtorch/models/GF_net.py:32-35). */
int rr_resize_bilinear(const float* src, int c, int h, int w, float* dst, int ho, int wo,
                       double scale_h, double scale_w, void* stream);

/* Global pooling to out[n][c] float32.
 * GeM: (mean_hw max(x,eps)^p)^(1/p)  — cirtorch/modules/pools.py:30-38
 * MAC: max_hw x                      — pools.py:10-16
 * SPoC: mean_hw x                    — pools.py:20-26
 * x layout RR_NHWC ([n][hw][c], any dtype) or RR_NCHW ([n][c][hw]). */
int rr_global_pool(const void* x, int n, int c, int hw, int layout, int mode,
                   float p, float eps, float* out, int dtype, void* stream);
/* Same, GeM exponent read by the kernel from DEVICE memory when p_dev != NULL
 * (the learnable scalar `pool.p` Parameter, pools.py:34): no host read-back,
 * so every update of the parameter is seen and the call stays graph-capturable. */
int rr_global_pool_pdev(const void* x, int n, int c, int hw, int layout, int mode,
                        float p, const float* p_dev, float eps, float* out, int dtype, void* stream);

/* Row L2 normalisation y = x / (||x||_2 + eps) over `dim` contiguous floats.
 * Replaces cirtorch/modules/normalizations.py:9-16 (L2N). In-place allowed. */
int rr_l2n_rows(const float* x, int rows, int dim, float eps, float* y, void* stream);

/* Dense layer y[r][o] = sum_i x[r][i] * W[o][i] + b[o] (b may be NULL), fp32.
 * Replaces the nn.Linear "learned whitening" of globalHead
 * (cirtorch/modules/heads/global_head.py:26,63). */
int rr_linear_rows(const float* x, int rows, int in_dim, const float* w, const float* b,
                   int out_dim, float* y, void* stream);

/* Fused globalHead tail: y = L2N(W . L2N(x) + b) (whiten != 0) or L2N(x).
 * x: pooled [rows][dim] f32.  Replaces global_head.py:52-67 after the pool.
 * workspace: rr_head_workspace_bytes(rows, dim). */
size_t rr_head_workspace_bytes(int rows, int dim);
int rr_head_l2n_whiten_l2n(const float* x, int rows, int dim, const float* w, const float* b,
                           int whiten, float eps, float* y, void* workspace, void* stream);

/* Post-hoc learned whitening, y = L2N(P[:d_out] (x - m)) per row, computed in
 * float64 on the f64 MFMA like the reference (cirtorch/utils/whiten.py:4-12:
 * numpy promotes the float32 vectors to the float64 m, P of whitenlearn;
 * applied at scripts/test.py:253-254).  x [rows][dim] float32 (dim % 16 == 0),
 * m [dim] float64, P [>= d_out][dim] float64 row-major, y [rows][d_out]
 * float32 (the float64 result rounded once).  L2N adds 1e-6 to the norm.
 * workspace: rr_whiten_workspace_bytes(rows, d_out). */
size_t rr_whiten_workspace_bytes(int rows, int d_out);
int rr_whitenapply(const float* x, int rows, int dim, const double* m, const double* P, int d_out,
                   float* y, void* workspace, size_t workspace_bytes, void* stream);

/* --------------------------------------------------------------- matching */

/* Brute-force cosine kNN with exact ordering.
 * Replaces `scores = np.dot(vecs.T, qvecs); ranks = np.argsort(-scores, axis=0)`
 * (scripts/test.py:247-248, scripts/train_globalF.py:733-734), returning only
 * the first k ranks.  Candidates are screened with an MFMA score GEMM in
 * `dtype` (db/q: RR_F32, RR_BF16, or RR_F16 — the fp16 database of SURVEY
 * §8d config 5; d >= 64 for the 16-bit types), then re-scored in float64
 * from the float32 copies and ordered by (score desc, index asc).
 *   db      : [n_db][d] (dtype)      db_f32 : [n_db][d] float32 (re-rank)
 *   q       : [nq][d]   (dtype)      q_f32  : [nq][d]   float32
 *   out_scores : [nq][k] float64     out_idx : [nq][k] int64 (+ idx_offset)
 * `cand` = candidates kept per query (>= k); 0 picks the default for dtype. */
size_t rr_knn_workspace_bytes(long long n_db, int nq, int d, int k, int cand, int dtype);
int rr_knn_topk(const void* db, const float* db_f32, long long n_db,
                const void* q, const float* q_f32, int nq, int d, int k, int cand,
                long long idx_offset, double* out_scores, long long* out_idx,
                void* workspace, size_t workspace_bytes, int dtype, void* stream);

/* Same, with a certificate: out_uncertain[q] = 0 when the screening margin
 * provably covers query q (every row outside the candidates has exact score
 * below the returned k-th score: screening key + error bound, the bound from
 * the screening dtype, d, ||q|| and db_norm_max = max ||db row||), 1 when a
 * cluster tighter than the screening error straddles the candidate cut —
 * re-search such queries with RR_F32 screening / more candidates
 * (cirtorch.search.KnnIndex.search(verify=True) does). */
int rr_knn_topk_checked(const void* db, const float* db_f32, long long n_db,
                        const void* q, const float* q_f32, int nq, int d, int k, int cand,
                        long long idx_offset, double* out_scores, long long* out_idx,
                        void* workspace, size_t workspace_bytes, int dtype, float db_norm_max,
                        int* out_uncertain, void* stream);

/* The certificate for int8 screening (rr_quantize_i8 database, rr_quantize_i8_rows
 * or rr_quantize_i8 queries): q_amax = the queries' max |x| (one per row when
 * q_amax_per_row, else one for all), db_amax = the database's; the bound is the
 * quantisation residual bound s E (||q8|| + ||x8|| + E), s = aq ax / 127^2,
 * E = sqrt(d) / 2 — ~0.02 at d = 2048, so on dense random data most queries stay
 * uncertified (re-search them), while well-separated top-k certify. */
int rr_knn_topk_checked_i8(const void* db, const float* db_f32, long long n_db,
                           const void* q, const float* q_f32, int nq, int d, int k, int cand,
                           long long idx_offset, double* out_scores, long long* out_idx,
                           void* workspace, size_t workspace_bytes, float db_norm_max,
                           const float* q_amax, int q_amax_per_row, const float* db_amax,
                           int* out_uncertain, void* stream);

/* Merge R per-shard top-k lists per query into one top-k by (score desc,
 * index asc).  in_*: [R][nq][k_in]; out_*: [nq][k].  Used after the RCCL
 * all-gather of per-shard results.  k_in*R <= 4096. */
int rr_topk_merge(const double* in_scores, const long long* in_idx, int r, int nq, int k_in,
                  int k, double* out_scores, long long* out_idx, void* stream);

/* ------------------------------------------------------ sharded search (RCCL) */
/* For a non-Python host of the sharded search (one process per GPU; the Python
 * host uses torch.distributed, cirtorch/search.py ShardedIndex).  RCCL is
 * dlopen'ed on first use.  Rank 0 creates the id, the host sends it to every
 * rank out of band, each rank calls rr_comm_init with its GPU current.  Then
 * per search: rr_knn_topk on the local rows (idx_offset = the shard's first
 * global row) -> rr_topk_allgather_merge = RCCL all-gather of the [nq][k]
 * (score f64, index i64) lists over xGMI + rr_topk_merge, bit-identical to a
 * 1-GPU search of the whole database.  Replaces the missing per-rank gather
 * of scripts/train_globalF.py:667-730. */
int rr_comm_unique_id(void* id_out, int id_bytes);                 /* id_bytes >= 128 */
int rr_comm_init(void** comm, int nranks, const void* id, int id_bytes, int rank);
int rr_comm_destroy(void* comm);
size_t rr_topk_allgather_workspace_bytes(int nranks, int nq, int k);
int rr_topk_allgather_merge(void* comm, const double* scores, const long long* idx, int nq, int k,
                            double* out_scores, long long* out_idx, void* workspace, size_t workspace_bytes,
                            void* stream);

/* ------------------------------------------------------- local descriptors */
/* Local-descriptor head (config 5): desc = normalize(W . grid_sample(x, kpts) + b).
 * Replaces cirtorch/modules/heads/local_head.py:43-71 (localHead.forward:
 * functional.grid_sample(mode="bilinear", padding_mode="zeros",
 * align_corners=False) -> nn.Linear(dim, e) -> functional.normalize(dim=2)).
 *   x    : [n][h][w][c] NHWC feature map (dtype), c a multiple of 8 (bf16) / 4 (f32)
 *   kpts : [n][npts][2] float32 normalised (x, y) in [-1, 1] (grid_sample grid)
 *   weight [e][c], bias [e] (may be NULL) float32;  out [n][npts][e] float32
 * workspace: rr_local_head_workspace_bytes(n*npts, c, e). */
size_t rr_local_head_workspace_bytes(long long nkp, int c, int e);
int rr_local_head(const void* x, int n, int h, int w, int c, int dtype, const float* kpts, int npts,
                  const float* weight, const float* bias, int e, float* out, void* workspace,
                  size_t workspace_bytes, void* stream);
/* Mutual nearest neighbours from the two directions' top-1 lists (int64):
 * match[i] = nn12[i] if nn21[nn12[i]] == i else -1.  Replaces the
 * np.argmin/argmin mutual check of HPatchesEval.py:31-43 (nn12/nn21 from
 * rr_knn_topk with k = 1: exact order, ties -> lower index like np.argmin). */
int rr_mutual_nn(const long long* nn12, int n1, const long long* nn21, int n2, long long* match, void* stream);

/* Full ranking for any database size: out_idx[q][r] = the r-th database row of
 * query q by (float64 score desc, index asc) — np.argsort(-np.dot(vecs.T, qvecs),
 * axis=0) of scripts/test.py:247-248 as [nq][n] (rr_knn_topk ranks k <= 8192).
 * The float64 score is rr_knn_topk's re-score (same summation order), so the
 * first k ranks equal a top-k search.  db_f32 [n][d], q_f32 [nq][d] float32,
 * d a multiple of 256 (zero-pad); workspace >= rr_rank_workspace_bytes
 * (24 B x nq x n + histograms). */
size_t rr_rank_workspace_bytes(long long n, int nq);
int rr_rank_full(const float* db_f32, long long n, const float* q_f32, int nq, int d, long long* out_idx,
                 void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------ tuning */
/* Engine tuning knobs (process-wide; for benchmarking / autotuning tools):
 *   RR_TUNE_GEMM_CONFIG  0 = automatic tile choice, 1 = 128x128, 2 = 64x256,
 *                        3 = 256x128 (8 waves), 4 = 256x256 (8 waves), 5 = 256x64,
 *                        7 / 8 = 256x128 / 128x256 (8 waves, 3-stage ring)
 *                        6 = A-stationary (weights resident in LDS) where eligible
 *   RR_TUNE_GEMM_STAGES  2 or 3 LDS stages (3: one resident block per CU)
 *   RR_TUNE_GEMM_WIDE    0/1 allow the 8-wave tiles in the automatic choice
 *   RR_TUNE_GEMM_ASTAT   0/1 allow the A-stationary tiles in the automatic choice
 *   RR_TUNE_GEMM_XCD_MAP 0/1 XCD-contiguous tile order (default 0)
 *   RR_TUNE_STREAM_1X1   0/1 weight-stationary streaming kernel for the
 *                        HBM-bound bf16 1x1 convs (default 1); 2 / 3 also route the
 *                        residual 512->2048 / 256->1024 1x1s to the 8-phase GEMM (A/B only)
 *   RR_TUNE_CONV3X3      0 off, 1 auto (default): direct 3x3 kernel with LDS
 *                        halo patches for the bf16 stride-1 3x3 convs;
 *                        2 / 3 prefer its 8x32 / 4x32 pixel tiles, 4 / 6 use
 *                        1x8 / 1x4 waves for the c_in = 64 A-stationary form,
 *                        7 a 3-stage weight ring, 8 256-channel x 6x32 tiles,
 *                        9 the c_in = c_out = 64 form with the weights in VGPRs
 *                        (k_c3w64; also what 1 picks for that shape)
 *   RR_TUNE_GRID_CUS     cap on the CUs one persistent launch spreads over
 *                        (0 = all; e.g. half the chip for two concurrent streams)
 *   RR_TUNE_GEMM8        0 off, 1 auto, 2 forced: the 8-phase staggered 256x256 GEMM for eligible
 *                        16-bit 1x1 / tap-uniform convs and score GEMMs (default 1: persistent
 *                        blocks for the kNN score GEMM, one block per tile for convs; 2: also
 *                        persistent everywhere; | 4: one block per tile everywhere; | 8: no
 *                        k_gemm8h / k_gemm8s; | 16: no k_gemm8a; | 32: k_gemm8h instead of the streaming
 *                        k_gemm8s for the <= 128-query score GEMM; | 64: conv tiles walked
 *                        channel-major instead of pixel-major; | 128: k_gemm8a one block per
 *                        tile instead of persistent blocks)
 *   RR_TUNE_KNN_FUSED    0/1 kNN screening in the score-GEMM epilogue after a 4-chunk
 *                        prefix (default 1); 0 = every chunk through the score slab
 *   RR_TUNE_CONV3_PIPE   1 (default): the direct 3x3 kernel reads the operands of its next
 *                        half-step while the current one's MFMAs issue; 0: compiler schedule
 *   RR_TUNE_STEM         2 (default): fused stem v3 (pixels x channels MFMA, lane-local
 *                        pooling; 3 / 4: patch fill in 2 / 5 parts); 1: v2 (pools the raw
 *                        conv before BN/activation, exact by monotonicity); 0: v1 (BN/activation
 *                        on every stem pixel).  Odd stem maps always take v1.
 *   RR_TUNE_STREAM_XCD   1 (default): the streaming 1x1's channel-slice blocks of one pixel
 *                        strip run on one XCD (the strip's input is re-read from that L2)
 *   RR_TUNE_CONV3S       1 (default): the staggered two-wave-group direct 3x3 (persistent,
 *                        chunk-double-buffered halo patches) for the stride-1 3x3s with
 *                        c_out = 128 under RR_TUNE_CONV3X3 = 1; 2: also c_in = c_out = 64; 0 off
 *   RR_TUNE_WRES         1: the residual 256 -> 1024 / 512 -> 2048 1x1s (bottleneck conv3 of
 *                        mod4 / mod5) on the weight-stationary k_wres1x1 (weights in VGPRs,
 *                        activation + residual tiles by LDS-DMA); 2: also the non-residual
 *                        K = 256 / 512 1x1s (projections, strided or not; mod4 block-1 conv1;
 *                        default); 0: the streaming 1x1 / 8-phase GEMM
 *   RR_TUNE_PAIR_MID     1 (default): the 128/512 boundary of rr_conv1x1_pair on 32-pixel tiles
 *                        with a 4-slot residual ring (3 tiles ahead); 0: 64-pixel tiles, one ahead
 *                        (same results bit for bit)
 *   RR_TUNE_WRES_RING    1 (default): the non-residual k_wres1x1 forms (projections, mod4 block-1
 *                        conv1) keep 5 (K = 256) / 3 (K = 512) activation tiles in flight; 0: two
 *                        (same results bit for bit) */
enum rr_tune_key { RR_TUNE_GEMM_CONFIG = 0, RR_TUNE_GEMM_STAGES = 1, RR_TUNE_GEMM_WIDE = 2,
                   RR_TUNE_GEMM_ASTAT = 3, RR_TUNE_GEMM_XCD_MAP = 4, RR_TUNE_STREAM_1X1 = 5,
                   RR_TUNE_CONV3X3 = 6, RR_TUNE_GRID_CUS = 7, RR_TUNE_GEMM8 = 8,
                   RR_TUNE_KNN_FUSED = 9, RR_TUNE_CONV3_PIPE = 10,
                   RR_TUNE_STEM = 11, RR_TUNE_STREAM_XCD = 12, RR_TUNE_CONV3S = 13,
                   RR_TUNE_WRES = 14, RR_TUNE_PAIR_MID = 15, RR_TUNE_WRES_RING = 16 };
int rr_set_tuning(int key, int value);

/* ----------------------------------------------------------- data helpers */
/* Counter-based N(0,1) rows, each L2-normalised: row i of the global matrix
 * depends only on (seed, i0 + i), so shards generate identical rows. */
int rr_fill_unit_rows(float* out, long long rows, int d, unsigned long long seed,
                      long long row0, void* stream);
/* int8 screening copy of float32 rows for rr_knn_topk(dtype RR_I8): y = clamp(rint(x * 127 / amax),
 * -127, 127) with amax = max |x| over all n elements, reduced on the device into amax_dev (one float of
 * caller scratch; no host synchronisation).  The screening scores are then exact int32 dot products of
 * the quantised rows (v_mfma_i32_16x16x64_i8, twice the bf16 MFMA rate, half the bf16 bytes); the final
 * top-k is the exact float64 re-score of the candidates, as for every screening dtype. */
int rr_quantize_i8(const float* x, long long n, void* y, float* amax_dev, void* stream);
/* Per-row int8 copy (queries): amax_rows[r] = max |x_r|, y_r = clamp(rint(x_r * 127 / amax_rows[r]),
 * -127, 127); x [rows][d] float32, d % 4 == 0.  A query's screened candidates then do not depend on
 * the other queries of its batch. */
int rr_quantize_i8_rows(const float* x, int rows, int d, void* y, float* amax_rows, void* stream);
/* float32 -> bf16 (round to nearest even). */
int rr_cast_f32_bf16(const float* x, void* y, long long n, void* stream);
/* float32 -> fp16 (IEEE binary16, round to nearest even). */
int rr_cast_f32_f16(const float* x, void* y, long long n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RR_H_ */
