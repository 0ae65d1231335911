"""mAP / mP@k over full ranks (reference
``cirtorch/utils/evaluation/ParisOxfordEval.py:4-195``; ``np.in1d`` -> ``np.isin``).
Ranks may be a numpy array or a torch tensor (e.g. from ``cirtorch.search.rank``)."""

import numpy as np


def compute_ap(ranks, nres):
    nimgranks = len(ranks)
    ap = 0.0
    recall_step = 1.0 / nres
    for j in np.arange(nimgranks):
        rank = ranks[j]
        precision_0 = 1.0 if rank == 0 else float(j) / rank
        precision_1 = float(j + 1) / (rank + 1)
        ap += (precision_0 + precision_1) * recall_step / 2.0
    return ap


def _np(ranks):
    if hasattr(ranks, "detach"):
        ranks = ranks.detach().cpu().numpy()
    return np.asarray(ranks)


def compute_map(ranks, gnd, kappas=[]):
    ranks = _np(ranks)
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
        qgndj = np.array(gnd[i]["junk"]) if "junk" in gnd[i] else np.empty(0)
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


def _print(*args):
    print(args[0] % tuple(args[1:]) if len(args) > 1 else args[0])


def compute_map_and_print(dataset, ranks, gnd, log_info=_print, kappas=[1, 5, 10]):
    if dataset.startswith("oxford5k") or dataset.startswith("paris6k"):
        mAP, aps, _, _ = compute_map(ranks, gnd)
        log_info("{%s}: mAP = {%f}", dataset, np.around(mAP * 100, decimals=2))
        return {"mAP": 100 * mAP}
    if dataset.startswith("roxford5k") or dataset.startswith("rparis6k"):
        res = {}
        for proto, okk, jk in (("E", ["easy"], ["junk", "hard"]), ("M", ["easy", "hard"], ["junk"]),
                               ("H", ["hard"], ["junk", "easy"])):
            g2 = [{"ok": np.concatenate([g[k] for k in okk]), "junk": np.concatenate([g[k] for k in jk])}
                  for g in gnd]
            res[proto] = compute_map(ranks, g2, kappas)
        mapE, mapM, mapH = res["E"][0], res["M"][0], res["H"][0]
        log_info("{%s}: mAP E: {%f}, M: {%f}, H: {%f}", dataset, np.around(mapE * 100, decimals=2),
                 np.around(mapM * 100, decimals=2), np.around(mapH * 100, decimals=2))
        for j in range(len(kappas)):
            log_info("{%s}: mP@k{%f} E: {%f}, M: {%f}, H: {%f}", dataset, kappas[j],
                     np.around(res["E"][2] * 100, decimals=2)[j], np.around(res["M"][2] * 100, decimals=2)[j],
                     np.around(res["H"][2] * 100, decimals=2)[j])
        return {"mAP": 100 * (mapM + mapH) / 2.0, "mapE": mapE, "mapM": mapM, "mapH": mapH}
    raise ValueError("unknown dataset %s" % dataset)
