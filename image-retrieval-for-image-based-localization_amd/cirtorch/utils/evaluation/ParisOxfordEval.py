"""mAP / mP@k over ranked lists — the evaluation of
``cirtorch/utils/evaluation/ParisOxfordEval.py:4-195`` (old Oxford/Paris
protocol and the revisited Easy / Medium / Hard protocol).

Formulation (vectorised per query, no per-rank Python loop):
  * the rank position of every database item comes from ONE inverse
    permutation of the query's ranked list (a scatter; done on the GPU when
    ``ranks`` is a GPU tensor from ``cirtorch.search.rank``);
  * the positions of the positives / junk items are gathers from it,
    sorted (``np.isin`` over the ranked list yields the same ascending set);
  * junk removal: each positive's position drops by the number of junk
    items ranked above it (``np.searchsorted``);
  * AP is the trapezoid over the positives' recall steps,
    ``sum_j ((j / r_j or 1 if r_j == 0) + (j + 1) / (r_j + 1)) / (2 n)``,
    accumulated left to right (``np.cumsum``) in float64 — the same IEEE
    operations in the same order as a scalar loop, so results are
    bit-identical to the reference's (pinned by ``tests/golden/map.npz``).
"""

import numpy as np

try:  # GPU inverse permutation when the ranks live on the GPU
    import torch
except ImportError:  # pragma: no cover
    torch = None


def _positions(ranks):
    """ranks [N_ranked, Q] (numpy or torch) -> posof [Q, N_db] int64 with the rank
    position of each database item (-1 where an item is not in the list).
    Negative entries (the -1 fill of unfilled kNN slots, k > N) are ignored:
    they scatter into a dummy column that is dropped."""
    if torch is not None and torch.is_tensor(ranks):
        r = ranks.long()
        n, q = r.shape
        ndb = max(int(r.max().item()) + 1, 0) if r.numel() else 0
        r = torch.where(r < 0, torch.full_like(r, ndb), r)
        pos = torch.full((q, ndb + 1), -1, dtype=torch.int64, device=r.device)
        pos.scatter_(1, r.t().contiguous(), torch.arange(n, device=r.device).expand(q, n).contiguous())
        return pos[:, :ndb].cpu().numpy()
    r = np.asarray(ranks).astype(np.int64, copy=False)
    n, q = r.shape
    ndb = max(int(r.max()) + 1, 0) if r.size else 0
    r = np.where(r < 0, ndb, r)
    pos = np.full((q, ndb + 1), -1, dtype=np.int64)
    pos[np.arange(q)[:, None], r.T] = np.arange(n)[None, :]
    return pos[:, :ndb]


def _ranked(posq, items):
    """ascending rank positions of `items` present in the ranked list"""
    items = np.asarray(items, dtype=np.int64).reshape(-1)
    items = items[(items >= 0) & (items < posq.shape[0])]
    p = np.unique(posq[items])
    return p[p >= 0]


def compute_ap(ranks, nres):
    """AP of one query from the 0-based positions of its positives (ascending,
    junk already removed) and the number of positives (``ParisOxfordEval.py:4-38``)."""
    r = np.asarray(ranks, dtype=np.float64)
    if r.size == 0:
        return 0.0
    j = np.arange(r.size, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        p0 = np.where(r == 0, 1.0, j / r)
    p1 = (j + 1.0) / (r + 1.0)
    terms = (p0 + p1) * (1.0 / nres) / 2.0
    return float(np.cumsum(terms)[-1])


def _map_from_positions(posof, gnd, kappas):
    nq = len(gnd)
    aps = np.zeros(nq)
    prs = np.zeros((nq, len(kappas)))
    pr = np.zeros(len(kappas))
    total = 0.0
    nempty = 0
    for i in range(nq):
        qgnd = np.array(gnd[i]["ok"])
        if qgnd.shape[0] == 0:
            aps[i] = float("nan")
            prs[i, :] = float("nan")
            nempty += 1
            continue
        pos = _ranked(posof[i], qgnd)
        junk = _ranked(posof[i], gnd[i]["junk"]) if "junk" in gnd[i] else np.empty(0, dtype=np.int64)
        if len(junk):
            pos = pos - np.searchsorted(junk, pos, side="left")
        ap = compute_ap(pos, len(qgnd))
        total = total + ap
        aps[i] = ap
        pos = pos + 1
        for j, kap in enumerate(kappas):
            kq = min(int(pos.max()), kap) if pos.size else kap
            prs[i, j] = (pos <= kq).sum() / kq
        pr = pr + prs[i, :]
    return total / (nq - nempty), aps, pr / (nq - nempty), prs


def compute_map(ranks, gnd, kappas=[]):
    """(mAP, per-query AP, mP@k, per-query P@k) over `ranks` [N, Q] for gnd
    dicts with "ok" (and optional "junk") item lists (``ParisOxfordEval.py:41-113``)."""
    return _map_from_positions(_positions(ranks), gnd, kappas)


def _print(*args):
    print(args[0] % tuple(args[1:]) if len(args) > 1 else args[0])


_PROTOCOLS = (("E", ["easy"], ["junk", "hard"]), ("M", ["easy", "hard"], ["junk"]), ("H", ["hard"], ["junk", "easy"]))


def compute_map_and_print(dataset, ranks, gnd, log_info=_print, kappas=[1, 5, 10]):
    """Old protocol (oxford5k / paris6k) or revisited E / M / H (roxford5k /
    rparis6k), logged like ``ParisOxfordEval.py:116-195``; returns the score
    dict (``mAP`` = (M + H) / 2 for the revisited datasets)."""
    if dataset.startswith("oxford5k") or dataset.startswith("paris6k"):
        mAP, _, _, _ = compute_map(ranks, gnd)
        log_info("{%s}: mAP = {%f}", dataset, np.around(mAP * 100, decimals=2))
        return {"mAP": 100 * mAP}
    if dataset.startswith("roxford5k") or dataset.startswith("rparis6k"):
        posof = _positions(ranks)    # one inverse permutation serves all three protocols
        res = {}
        for proto, okk, jk in _PROTOCOLS:
            g2 = [{"ok": np.concatenate([g[k] for k in okk]), "junk": np.concatenate([g[k] for k in jk])}
                  for g in gnd]
            res[proto] = _map_from_positions(posof, g2, kappas)
        mapE, mapM, mapH = res["E"][0], res["M"][0], res["H"][0]
        log_info("{%s}: mAP E: {%f}, M: {%f}, H: {%f}", dataset, np.around(mapE * 100, decimals=2),
                 np.around(mapM * 100, decimals=2), np.around(mapH * 100, decimals=2))
        for j in range(len(kappas)):
            log_info("{%s}: mP@k{%f} E: {%f}, M: {%f}, H: {%f}", dataset, kappas[j],
                     np.around(res["E"][2] * 100, decimals=2)[j], np.around(res["M"][2] * 100, decimals=2)[j],
                     np.around(res["H"][2] * 100, decimals=2)[j])
        return {"mAP": 100 * (mapM + mapH) / 2.0, "mapE": mapE, "mapM": mapM, "mapH": mapH}
    raise ValueError("unknown dataset %s" % dataset)
