"""Learned whitening (reference ``cirtorch/utils/whiten.py:4-65``).

``whitenlearn`` / ``pcawhitenlearn`` solve a small D x D eigenproblem once on
the host (numpy, exactly as the reference).  ``whitenapply`` — applied to every
database and query vector — runs on the GPU engine: Y = P[:d] (X - m), then
column L2 normalisation with +1e-6 on the norm (``whiten.py:10``)."""

import os
import sys

import numpy as np
import torch

from .. import _ops


def whitenapply(X, m, P, dimensions=None):
    """X: D x N (numpy or torch) -> P[:dimensions] (X - m), columns L2-normalised
    (+1e-6 on the norm, ``whiten.py:10``).  The arithmetic is float64, as in
    the reference (numpy promotes the float32 vectors to the float64 m, P of
    whitenlearn), on the GPU's f64 MFMA (``rr_whitenapply``); the result is
    float32 columns (numpy input -> numpy output)."""
    was_numpy = not torch.is_tensor(X)
    if not dimensions:
        dimensions = P.shape[0]
    Xt = torch.as_tensor(np.asarray(X) if was_numpy else X)
    dev = Xt.device if Xt.is_cuda else torch.device("cuda")
    rows = Xt.t().to(dev).float().contiguous()                                    # [N, D]
    mt = torch.as_tensor(np.asarray(m) if not torch.is_tensor(m) else m).to(dev).double().reshape(-1)
    if not torch.is_tensor(P) and np.iscomplexobj(P):
        # np.linalg.eig of a numerically non-symmetric D can return a negligible
        # imaginary part; a real one means degenerate training pairs
        if np.abs(P.imag).max() > 1e-9 * max(np.abs(P.real).max(), 1e-300):
            raise ValueError("whitenapply: complex whitening matrix (degenerate whitenlearn input)")
        P = P.real
    Pt = torch.as_tensor(np.asarray(P) if not torch.is_tensor(P) else P).to(dev).double()
    y = _ops.whitenapply_rows(rows, mt, Pt, int(dimensions))                       # [N, d]
    Y = y.t()
    if was_numpy:
        return Y.cpu().numpy()
    return Y


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
                  .format(os.path.basename(__file__), alpha), file=sys.stderr)
