"""Learned whitening (reference ``cirtorch/utils/whiten.py:4-65``).

``whitenlearn`` / ``pcawhitenlearn`` solve a small D x D eigenproblem once on
the host (numpy, exactly as the reference).  ``whitenapply`` — applied to every
database and query vector — runs on the GPU engine: Y = P[:d] (X - m), then
column L2 normalisation with +1e-6 on the norm (``whiten.py:10``)."""

import os

import numpy as np
import torch

from .. import _ops


def whitenapply(X, m, P, dimensions=None):
    """X: D x N (numpy or torch).  Returns the same kind it was given."""
    was_numpy = not torch.is_tensor(X)
    if not dimensions:
        dimensions = P.shape[0]
    Xt = torch.as_tensor(np.asarray(X) if was_numpy else X)
    out_dtype = Xt.dtype
    Xt = Xt.cuda().float()
    mt = torch.as_tensor(np.asarray(m) if not torch.is_tensor(m) else m).cuda().float().reshape(-1)
    Pt = torch.as_tensor(np.asarray(P) if not torch.is_tensor(P) else P).cuda().float()[:dimensions].contiguous()
    rows = (Xt.t() - mt[None, :]).contiguous()           # [N, D] centred rows
    y = _ops.linear_rows(rows, Pt, None)                  # [N, d]
    y = _ops.l2n_rows(y, 1e-6)
    Y = y.t()
    if was_numpy:
        return Y.cpu().numpy().astype(np.asarray(X).dtype, copy=False)
    return Y.to(out_dtype)


def pcawhitenlearn(X):
    N = X.shape[1]
    m = X.mean(axis=1, keepdims=True)
    Xc = X - m
    Xcov = np.dot(Xc, Xc.T)
    Xcov = (Xcov + Xcov.T) / (2 * N)
    eigval, eigvec = np.linalg.eig(Xcov)
    order = eigval.argsort()[::-1]
    eigval = eigval[order]
    eigvec = eigvec[:, order]
    P = np.dot(np.linalg.inv(np.sqrt(np.diag(eigval))), eigvec.T)
    return m, P


def whitenlearn(X, qidxs, pidxs):
    m = X[:, qidxs].mean(axis=1, keepdims=True)
    df = X[:, qidxs] - X[:, pidxs]
    S = np.dot(df, df.T) / df.shape[1]
    P = np.linalg.inv(cholesky(S))
    df = np.dot(P, X - m)
    D = np.dot(df, df.T)
    eigval, eigvec = np.linalg.eig(D)
    order = eigval.argsort()[::-1]
    eigvec = eigvec[:, order]
    P = np.dot(eigvec.T, P)
    return m, P


def cholesky(S):
    alpha = 0
    while True:
        try:
            return np.linalg.cholesky(S + alpha * np.eye(*S.shape))
        except np.linalg.LinAlgError:
            alpha = 1e-10 if alpha == 0 else alpha * 10
            print(">>>> {}::cholesky: Matrix is not positive definite, adding {:.0e} on the diagonal"
                  .format(os.path.basename(__file__), alpha))
