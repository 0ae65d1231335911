"""numpy / torch-CPU restatement of the hot-path operators (TEST INFRASTRUCTURE ONLY).

References (upstream paths):
  gem / mac / spoc   ``cirtorch/modules/pools.py:10-38``
  l2n                ``cirtorch/modules/normalizations.py:9-16``
  head               ``cirtorch/modules/heads/global_head.py:52-67``
  rank               ``scripts/test.py:247-248`` (np.dot + np.argsort(-scores, axis=0))
  compute_map        ``cirtorch/utils/evaluation/ParisOxfordEval.py:4-113``
  whitenapply/learn  ``cirtorch/utils/whiten.py:4-65``
"""

import numpy as np
import torch
import torch.nn.functional as F


# ---------------------------------------------------------------- pooling / norm
def gem(x, p=3.0, eps=1e-6):
    """x: torch N x C x H x W -> N x C x 1 x 1  (``pools.py:38``)."""
    p = torch.as_tensor([p], dtype=x.dtype) if not torch.is_tensor(p) else p
    return F.avg_pool2d(x.clamp(min=eps).pow(p), (x.size(-2), x.size(-1))).pow(1.0 / p)


def mac(x):
    return F.max_pool2d(x, (x.size(-2), x.size(-1)))  # ``pools.py:16``


def spoc(x):
    return F.avg_pool2d(x, (x.size(-2), x.size(-1)))  # ``pools.py:26``


def l2n(x, eps=1e-6):
    return x / (torch.norm(x, p=2, dim=1, keepdim=True) + eps).expand_as(x)  # ``normalizations.py:16``


def head(x, p, w, b, whiten=True):
    """globalHead.forward: x N x C x h x w -> D x N."""
    y = l2n(gem(x, p)).squeeze(-1).squeeze(-1)
    if whiten:
        y = l2n(F.linear(y, w, b))
    return y.permute(1, 0)


# ---------------------------------------------------------------- matching
def rank_reference(db_rows, q_rows):
    """The reference match, verbatim in numpy (``scripts/test.py:247-248``):
    vecs = D x N (columns = db), qvecs = D x Q  ->  ranks N x Q.
    Our inputs are row-major [N][D] / [Q][D] == vecs.T / qvecs.T."""
    scores = np.dot(db_rows, q_rows.T)          # == np.dot(vecs.T, qvecs)
    ranks = np.argsort(-scores, axis=0)
    return scores, ranks


def topk_exact(db_rows, q_rows, k):
    """Top-k per query with the tie rule of the build (score desc, index asc),
    scores computed in float64 (exact products of fp32 inputs).
    Returns (scores64 [Q][k], idx int64 [Q][k])."""
    s = np.dot(q_rows.astype(np.float64), db_rows.astype(np.float64).T)  # Q x N
    n = s.shape[1]
    k = min(k, n)
    # lexsort: last key primary -> (-score, index)
    out_i = np.empty((s.shape[0], k), dtype=np.int64)
    out_s = np.empty((s.shape[0], k), dtype=np.float64)
    idx = np.arange(n)
    for qi in range(s.shape[0]):
        part = np.argpartition(-s[qi], k - 1)[:k] if k < n else idx
        thr = s[qi, part].min()
        cand = np.nonzero(s[qi] >= thr)[0]
        order = np.lexsort((cand, -s[qi, cand]))[:k]
        out_i[qi] = cand[order]
        out_s[qi] = s[qi, out_i[qi]]
    return out_s, out_i


def topk_from_fp32_ranks(db_rows, q_rows, k):
    """Top-k from the reference fp32 scores with a stable sort (ties -> lower index)."""
    scores = np.dot(db_rows, q_rows.T)
    ranks = np.argsort(-scores, axis=0, kind="stable")[:k]
    return np.take_along_axis(scores, ranks, axis=0).T, ranks.T.astype(np.int64)


# ---------------------------------------------------------------- mAP
def compute_ap(ranks, nres):
    """``ParisOxfordEval.py:4-38`` (trapezoidal AP over positive ranks)."""
    ap = 0.0
    recall_step = 1.0 / nres
    for j in np.arange(len(ranks)):
        rank = ranks[j]
        precision_0 = 1.0 if rank == 0 else float(j) / rank
        precision_1 = float(j + 1) / (rank + 1)
        ap += (precision_0 + precision_1) * recall_step / 2.0
    return ap


def compute_map(ranks, gnd, kappas=()):
    """``ParisOxfordEval.py:41-113`` (np.in1d -> np.isin, same semantics)."""
    mAP = 0.0
    nq = len(gnd)
    aps = np.zeros(nq)
    pr = np.zeros(len(kappas))
    prs = np.zeros((nq, len(kappas)))
    nempty = 0
    for i in np.arange(nq):
        qgnd = np.array(gnd[i]["ok"])
        if qgnd.shape[0] == 0:
            aps[i] = float("nan")
            prs[i, :] = float("nan")
            nempty += 1
            continue
        try:
            qgndj = np.array(gnd[i]["junk"])
        except KeyError:
            qgndj = np.empty(0)
        pos = np.arange(ranks.shape[0])[np.isin(ranks[:, i], qgnd)]
        junk = np.arange(ranks.shape[0])[np.isin(ranks[:, i], qgndj)]
        k = 0
        ij = 0
        if len(junk):
            ip = 0
            while ip < len(pos):
                while ij < len(junk) and pos[ip] > junk[ij]:
                    k += 1
                    ij += 1
                pos[ip] = pos[ip] - k
                ip += 1
        ap = compute_ap(pos, len(qgnd))
        mAP = mAP + ap
        aps[i] = ap
        pos += 1
        for j in np.arange(len(kappas)):
            kq = min(max(pos), kappas[j])
            prs[i, j] = (pos <= kq).sum() / kq
        pr = pr + prs[i, :]
    mAP = mAP / (nq - nempty)
    pr = pr / (nq - nempty)
    return mAP, aps, pr, prs


def compute_map_revisited(ranks, gnd, kappas=(1, 5, 10)):
    """E / M / H protocol of ``ParisOxfordEval.py:129-166``; returns dict."""
    def proto(ok_keys, junk_keys):
        g = [{"ok": np.concatenate([q[k] for k in ok_keys]),
              "junk": np.concatenate([q[k] for k in junk_keys])} for q in gnd]
        return compute_map(ranks, g, list(kappas))
    mapE, _, mprE, _ = proto(["easy"], ["junk", "hard"])
    mapM, _, mprM, _ = proto(["easy", "hard"], ["junk"])
    mapH, _, mprH, _ = proto(["hard"], ["junk", "easy"])
    return {"mapE": mapE, "mapM": mapM, "mapH": mapH,
            "mprE": mprE, "mprM": mprM, "mprH": mprH}


# ---------------------------------------------------------------- whitening
def whitenapply(X, m, P, dimensions=None):
    """``whiten.py:4-12``; X is D x N."""
    if not dimensions:
        dimensions = P.shape[0]
    X = np.dot(P[:dimensions, :], X - m)
    return X / (np.linalg.norm(X, ord=2, axis=0, keepdims=True) + 1e-6)


def _cholesky(S):
    """``whiten.py:50-65`` (diagonal loading until PD)."""
    alpha = 0.0
    while True:
        try:
            return np.linalg.cholesky(S + alpha * np.eye(*S.shape))
        except np.linalg.LinAlgError:
            alpha = 1e-10 if alpha == 0 else alpha * 10


def whitenlearn(X, qidxs, pidxs):
    """``whiten.py:32-48``."""
    m = X[:, qidxs].mean(axis=1, keepdims=True)
    df = X[:, qidxs] - X[:, pidxs]
    S = np.dot(df, df.T) / df.shape[1]
    P = np.linalg.inv(_cholesky(S))
    df = np.dot(P, X - m)
    D = np.dot(df, df.T)
    eigval, eigvec = np.linalg.eig(D)
    order = eigval.argsort()[::-1]
    eigvec = eigvec[:, order]
    return m, np.dot(eigvec.T, P)


def pcawhitenlearn(X):
    """``whiten.py:14-30``."""
    N = X.shape[1]
    m = X.mean(axis=1, keepdims=True)
    Xc = X - m
    Xcov = np.dot(Xc, Xc.T)
    Xcov = (Xcov + Xcov.T) / (2 * N)
    eigval, eigvec = np.linalg.eig(Xcov)
    order = eigval.argsort()[::-1]
    eigval = eigval[order]
    eigvec = eigvec[:, order]
    return m, np.dot(np.linalg.inv(np.sqrt(np.diag(eigval))), eigvec.T)


def local_head(x, kpts, w, b):
    """localHead.forward (cirtorch/modules/heads/local_head.py:43-71): bilinear
    grid_sample (zeros, align_corners=False; local_head.py:51) -> permute ->
    Linear (:67) -> functional.normalize(dim=2) (:69).  x [B,C,H,W], kpts [B,N,2]."""
    import torch.nn.functional as F
    d = F.grid_sample(x, kpts.unsqueeze(2), mode="bilinear", padding_mode="zeros", align_corners=False)
    d = d.squeeze(-1).permute(0, 2, 1)
    return F.normalize(F.linear(d, w, b), dim=2)


def nn_matcher(desc1, desc2):
    """Mutual-NN matcher of HPatchesEval.py:23-43 (get_desc_dist + nn_matcher),
    restated: L2 distance matrix, argmin both ways, -1 where not mutual.
    (The reference module imports cv2, absent here: parity unpinned by a
    reference run; the restatement is five numpy lines of the same calls.)"""
    dist = np.linalg.norm(desc1[:, None] - desc2[None], axis=2)
    n1 = np.argmin(dist, axis=1)
    n2 = np.argmin(dist, axis=0)
    n1 = n1.copy()
    n1[n2[n1] != np.arange(len(n1))] = -1
    return n1


# ---------------------------------------------------------------- upstream multi-scale rule
def extract_ms_upstream(net, x, ms, msp, whiten):
    """One image through the upstream ``extract_vectors(ms, msp)`` rule that
    ``scripts/test.py:200,236-238`` calls: for every scale s the image (already
    normalised, C x H x W) is bilinearly resized (align_corners=False; s = 1 ->
    as is), its descriptor f_s is raised to msp, the mean over scales is taken to
    the power 1 / msp and the result is L2-normalised.  The upstream source
    (cirtorch/networks/imageretrievalnet.py of cnnimageretrieval-pytorch) is not
    in /root/reference: PARITY UNPINNED for this rule (restated from its
    published description).  net: an oracle.backbone.OracleNet; returns D."""
    acc = None
    for s in ms:
        xs = x[None] if s == 1 else F.interpolate(x[None], scale_factor=s, mode="bilinear", align_corners=False)
        v = net.head(net.body(xs)["mod5"], whiten=whiten)[:, 0].pow(msp)
        acc = v if acc is None else acc + v
    v = (acc / len(ms)).pow(1.0 / msp)
    return v / v.norm()
