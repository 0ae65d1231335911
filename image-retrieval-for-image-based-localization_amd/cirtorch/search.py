"""GPU matching: the replacement for the reference's host-side rank
``scores = np.dot(vecs.T, qvecs); ranks = np.argsort(-scores, axis=0)``
(``scripts/test.py:247-248``, ``scripts/train_globalF.py:733-734``).

* ``knn(vecs, qvecs, k)``  -> first k ranks (k x Q, int64) and their scores,
  exactly ordered by (score desc, index asc); scores re-computed in float64.
* ``rank(vecs, qvecs)``     -> full ranks (N x Q) for mAP evaluation, any N.
* ``KnnIndex``              -> a resident database (float32 rows + optional
  bf16 or fp16 screening copy) queried many times.
* ``ShardedIndex``          -> database rows split over the ranks of a
  torch.distributed group (RCCL on ROCm), per-shard top-k, all-gather of the
  (score, index) lists, on-GPU merge — bit-identical to the 1-GPU result.

Layouts: the reference keeps descriptors as D x N columns; the engine reads
row-major [N][D].  ``vecs.t()`` of a D x N column matrix produced by
``globalHead`` is already a contiguous [N][D] view (no copy).
"""

import torch
import torch.distributed as dist

from . import _ops

# screening precision of the score GEMM (the final top-k is always the exact float64
# re-score): int8 = database rows quantised with one scale per tensor, queries with one
# per row, exact int32 dot products on v_mfma_i32_16x16x64_i8 (twice the bf16 rate, half
# the bytes).  Certificates (verify): fp16 / bf16 / fp32 from the rounding error bound,
# int8 from the quantisation residual bound (~0.02 at D = 2048: on dense random data most
# int8 queries stay uncertified and are re-searched, so fp16 is the certified default)
_PREC = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16, "bfloat16": torch.bfloat16,
         "fp16": torch.float16, "float16": torch.float16, "int8": torch.int8}


def _rows(cols):
    """D x N column matrix (torch or numpy) -> contiguous float32 [N][D] on GPU."""
    if not torch.is_tensor(cols):
        cols = torch.from_numpy(cols)
    rows = cols.t()
    if not rows.is_cuda:
        rows = rows.cuda()
    return rows.float().contiguous()


def _padded_dim(d, dtype):
    """The engine's score GEMM takes power-of-two D >= 32 (>= 64 for fp16,
    >= 256 for int8 screening); other D are zero-padded, which changes no dot
    product."""
    p = 64 if dtype == torch.float16 else 256 if dtype == torch.int8 else 32
    while p < d:
        p <<= 1
    return p


def _pad_cols(x, d_pad):
    if x.shape[1] == d_pad:
        return x
    return torch.nn.functional.pad(x, (0, d_pad - x.shape[1])).contiguous()


class KnnIndex:
    def __init__(self, db_rows, precision="fp32", cand=0, idx_offset=0):
        """db_rows: [N, D] float32 on the GPU (kept by reference, not copied,
        when D is a power of two >= 32; zero-padded otherwise)."""
        self.dtype = _PREC[precision]
        self.dim = db_rows.shape[1]
        self.d_pad = _padded_dim(self.dim, self.dtype)
        self.db32 = _pad_cols(db_rows.float().contiguous(), self.d_pad)
        self.db_amax = None   # int8: the database's quantisation scale (max |x|), kept for the certificate
        if self.dtype == torch.int8 and self.db32.shape[0]:
            self.db, self.db_amax = _ops.quantize_i8(self.db32, with_scale=True)
        else:
            self.db = _ops.cast_screen(self.db32, self.dtype) if self.db32.shape[0] else self.db32.to(self.dtype)
        self.cand = cand
        self.idx_offset = idx_offset
        self._ws = {}   # scratch per stream: searches on different streams never share a slab
        # the certificate's max row norm, read once here so that no search (and no
        # profile of one) pays for the norm pass over the database
        self._norm_max = float(self.db32.norm(dim=1).max().item()) if self.ntotal else 0.0

    @property
    def ntotal(self):
        return self.db32.shape[0]

    def _workspace(self, need, device):
        """Scratch of the current stream.  A buffer is only ever used by the
        stream it was allocated on, so concurrent searches of one index on two
        streams do not race; a replaced buffer is freed in that stream's order."""
        stream = torch.cuda.current_stream(device)
        ws = self._ws.get(stream.cuda_stream)
        if ws is None or ws.numel() < need:
            ws = torch.empty(need, dtype=torch.uint8, device=device)
            self._ws[stream.cuda_stream] = ws
        return ws

    def norm_max(self):
        """largest database row norm (computed when the index is built)"""
        return self._norm_max

    def _screen_queries(self, q32):
        """float32 query rows -> (screening copy, int8 per-row scales or None)"""
        if self.dtype == torch.int8:
            return _ops.quantize_i8(q32, per_row=True, with_scale=True)
        return _ops.cast_screen(q32, self.dtype), None

    def search(self, q_rows, k, verify=True):
        """q_rows [Q, D] -> (scores float64 [Q, k], idx int64 [Q, k]) on the current stream.
        An empty shard (ntotal == 0) returns k (-inf, -1) entries per query, which
        the sharded merge drops.

        verify=True (the default: the reference ranks exactly, scripts/test.py:247-248)
        certifies the screening margin of every query (the rows left out are provably
        below the returned k-th score given the screening dtype's error bound) and
        re-searches uncertain queries — clusters of near-duplicates tighter than the
        screening error — with float32 screening and more candidates; this costs one
        device->host read per search, so it cannot be captured in a graph.

        verify=False is the explicit opt-out: the screened candidate pool re-ranked in
        float64, no certificate (exact unless near-ties straddle the screening cut);
        graph-capturable.

        verify="deferred" returns (scores, idx, pending): the same certificate,
        copied to pinned host memory without a synchronisation; pending.resolve()
        (later, e.g. once the next batch's work is queued) waits for it and
        re-searches the uncertain queries in place, returning how many there were."""
        if q_rows.shape[1] != self.dim:
            raise RuntimeError("KnnIndex.search: queries have D=%d, the database D=%d" % (q_rows.shape[1], self.dim))
        q32 = _pad_cols(q_rows.float().contiguous(), self.d_pad)
        if verify is True and q32.is_cuda and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("KnnIndex.search: verify=True reads the certificate back and cannot run "
                               "inside a graph capture; capture with verify=False (or 'deferred' outside)")
        if self.ntotal == 0 or q32.shape[0] == 0:
            s = torch.full((q32.shape[0], k), float("-inf"), dtype=torch.float64, device=q32.device)
            i = torch.full((q32.shape[0], k), -1, dtype=torch.int64, device=q32.device)
            return (s, i, Pending.done()) if verify == "deferred" else (s, i)
        if verify:
            s, i, unc = self.search_checked(q32, k)
            pend = Pending(unc, lambda bad: self._research(q32, bad, k), s, i)
            if verify == "deferred":
                return s, i, pend
            pend.resolve()
            return s, i
        q, _ = self._screen_queries(q32)
        need = _ops.knn_workspace_bytes(self.ntotal, q.shape[0], q.shape[1], k, self.cand, self.dtype)
        return _ops.knn_topk(self.db, self.db32, q, q32, k, cand=self.cand, idx_offset=self.idx_offset,
                             workspace=self._workspace(need, q.device))

    def search_checked(self, q_rows, k):
        """queries [Q, D] -> (scores, idx, int32 [Q] uncertain flags), no synchronisation"""
        q32 = _pad_cols(q_rows.float().contiguous(), self.d_pad)
        q, qa = self._screen_queries(q32)
        need = _ops.knn_workspace_bytes(self.ntotal, q.shape[0], q.shape[1], k, self.cand, self.dtype)
        return _ops.knn_topk(self.db, self.db32, q, q32, k, cand=self.cand, idx_offset=self.idx_offset,
                             workspace=self._workspace(need, q.device), db_norm_max=self.norm_max(),
                             i8_scales=None if qa is None else (qa, self.db_amax))

    def _research(self, q32, bad, k):
        """exact top-k of the queries q32[bad] (int64 [n] on the device): float32
        screening (error ~d 2^-24), then the largest candidate pool"""
        s, i = None, None
        sel = torch.arange(bad.numel(), device=bad.device)
        for cand in (0, min(8192, max(1024, 8 * k))):
            qb = q32[bad[sel]].contiguous()
            need = _ops.knn_workspace_bytes(self.ntotal, qb.shape[0], qb.shape[1], k, cand, torch.float32)
            s2, i2, u2 = _ops.knn_topk(self.db32, self.db32, qb, qb, k, cand=cand, idx_offset=self.idx_offset,
                                       workspace=self._workspace(need, qb.device), db_norm_max=self.norm_max())
            if s is None:
                s, i = s2, i2
            else:
                s[sel], i[sel] = s2, i2
            keep = torch.nonzero(u2).flatten()
            if keep.numel() == 0:
                return s, i
            sel = sel[keep]
        # more than 8192 rows within the float32 screening error of the k-th score
        # (exact duplicates of it, say): the full exact ranking of those queries
        s[sel], i[sel] = self._exact_by_rank(q32[bad[sel]].contiguous(), k)
        return s, i

    def _exact_by_rank(self, q32, k):
        """top-k of every row's float64 score by (score desc, index asc) -- rr_rank_full
        (the k_rescore summation order, stable radix sort), no screening at all; the
        scores are the same rows re-scored by the top-k pipeline over just those rows
        (gathered in index order, so its tie order is the global one)"""
        n, kk = self.ntotal, min(k, self.ntotal)
        d256 = (self.d_pad + 255) // 256 * 256
        db = _pad_cols(self.db32, d256)
        q = _pad_cols(q32, d256)
        per = max(1, min(65535, RANK_BYTES_MAX // (32 * n)))
        top = torch.cat([_ops.rank_full(db, q[j:j + per].contiguous())[:, :kk] for j in range(0, q.shape[0], per)])
        s = torch.full((q32.shape[0], k), float("-inf"), dtype=torch.float64, device=q32.device)
        i = torch.full((q32.shape[0], k), -1, dtype=torch.int64, device=q32.device)
        for r in range(q32.shape[0]):
            rows = torch.sort(top[r]).values
            sub = KnnIndex(self.db32[rows], "fp32", cand=max(kk, 32))
            sr, ir = sub.search(q32[r:r + 1], kk, verify=False)   # every row is a candidate
            s[r, :kk], i[r, :kk] = sr[0], rows[ir[0]] + self.idx_offset
        return s, i


class Pending:
    """The certificate of a search, read back later: the int32 flags are copied to
    pinned host memory on the search's stream and an event is recorded, so the
    caller is not synchronised until resolve().  resolve() waits for the event and,
    for the flagged queries, calls research(bad) -> (scores, idx) and writes them
    into the returned rows; it returns the number of re-searched queries."""

    def __init__(self, unc, research, s, i):
        self.s, self.i, self.research, self.unc = s, i, research, unc
        self.ev = None
        if unc.is_cuda:
            self.host = torch.empty(unc.shape, dtype=unc.dtype, pin_memory=True)
            self.host.copy_(unc, non_blocking=True)
            self.ev = torch.cuda.Event()
            self.ev.record()
        else:
            self.host = unc.clone()
        self.count = None

    @classmethod
    def done(cls):
        p = cls.__new__(cls)
        p.count = 0
        return p

    def resolve(self):
        if self.count is not None:
            return self.count
        if self.ev is not None:
            self.ev.synchronize()
        bad = torch.nonzero(self.host).flatten()
        self.count = int(bad.numel())
        if self.count:
            bad = bad.to(self.s.device)
            s2, i2 = self.research(bad)
            self.s[bad], self.i[bad] = s2, i2
        return self.count


def knn(vecs, qvecs, k, precision="fp32", cand=0, verify=True):
    """vecs D x N, qvecs D x Q (reference layout) -> (ranks k x Q int64, scores k x Q float64),
    certified exact by default (verify=False: the uncertified screen, see KnnIndex.search)."""
    db = _rows(vecs)
    q = _rows(qvecs)
    s, i = KnnIndex(db, precision, cand).search(q, k, verify=verify)
    return i.t(), s.t()


RANK_BYTES_MAX = 2 << 30  # device scratch + output of one rr_rank_full call
RANK_KNN_MAX = 8192  # up to this size the top-k pipeline (LDS bitonic sort of all rows) ranks in one pass


def rank(vecs, qvecs, precision="fp32", method="auto"):
    """Full ranking, the GPU equivalent of ``np.argsort(-np.dot(vecs.T, qvecs), axis=0)``:
    N x Q int64 by (score desc, index asc) on the float64 re-score.  N <= 8192: the
    top-k pipeline with k = N; larger N (revisited datasets with distractors):
    rr_rank_full (float64 scores + a stable radix sort), identical order."""
    n = vecs.shape[1]
    if method == "knn" or (method == "auto" and n <= RANK_KNN_MAX):
        # cand = n: every row is re-scored in float64, nothing is screened out to certify
        ranks, _ = knn(vecs, qvecs, n, precision=precision, cand=n, verify=False)
        return ranks
    db, q = _rows(vecs), _rows(qvecs)
    d_pad = (db.shape[1] + 255) // 256 * 256
    db, q = _pad_cols(db, d_pad), _pad_cols(q, d_pad)
    # ~32 B of scratch + output per (query, row): queries in independent groups that
    # fit RANK_BYTES_MAX (and the kernels' 65535-query grid), each ranked on its own
    per = max(1, min(65535, RANK_BYTES_MAX // (32 * n)))
    if q.shape[0] <= per:
        return _ops.rank_full(db, q).t()
    out = torch.empty((n, q.shape[0]), dtype=torch.int64, device=db.device)
    for j in range(0, q.shape[0], per):
        out[:, j:j + per] = _ops.rank_full(db, q[j:j + per].contiguous()).t()
    return out


def shard_range(n, rank, world):
    """Contiguous row shard of rank r: [r*ceil(n/R), min(n, (r+1)*ceil(n/R)))."""
    per = (n + world - 1) // world
    r0 = min(n, rank * per)
    return r0, max(0, min(per, n - r0))


def all_gather_stacked(t, group=None):
    """[...] per rank -> [R, ...] on every rank.  GPU tensors on an RCCL group
    ("nccl" backend on ROCm): one all_gather_into_tensor over xGMI.  Other
    backends (gloo) gather host copies and the result returns to t's device."""
    world = dist.get_world_size(group)
    if t.is_cuda and dist.get_backend(group) == "nccl":
        out = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=group)
        return out
    host = t.detach().cpu().contiguous()
    out = torch.empty((world,) + tuple(host.shape), dtype=host.dtype)
    dist.all_gather(list(out.unbind(0)), host, group=group)
    return out.to(t.device)


class ShardedIndex:
    """Database rows [row0, row0 + n_local) of a global matrix live on this
    rank; ``search`` expects the same queries on every rank (all-gather them
    first if each rank extracted its own).

    The only exchange is one all-gather of the per-shard (score f64, index i64)
    lists, packed in one buffer — Q x k x 16 bytes per rank — followed by the on-GPU merge with the
    (score desc, index asc) rule, so the merged result is bit-identical to a
    single-GPU search of the whole database."""

    def __init__(self, local_rows, row0, precision="bf16", cand=0, group=None, local_index=None, merge=None):
        self.local = local_index if local_index is not None else KnnIndex(local_rows, precision, cand, idx_offset=row0)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.merge = merge or _ops.topk_merge

    def search(self, q_rows, k, verify=True):
        """merged top-k of the queries (the same on every rank).  verify=True (default) /
        "deferred": every shard certifies its own top-k; the flags travel in the
        same all-gather as the lists, so every rank sees the same uncertain set
        and re-searches it (each shard in float32, then one more exchange) together.
        verify=False: the uncertified screen."""
        if not verify:
            s, i = self.local.search(q_rows, k, verify=False)
            return (s, i) if self.world == 1 else self.exchange(s, i, k)
        if self.world == 1:
            return self.local.search(q_rows, k, verify=verify)
        if self.local.ntotal == 0 or q_rows.shape[0] == 0:
            # an empty shard certifies trivially: (-inf, -1) lists, no flags
            s, i = self.local.search(q_rows, k, verify=False)
            unc = torch.zeros(q_rows.shape[0], dtype=torch.int32, device=s.device)
        else:
            # the flags travel in the all-gather: no per-shard Pending (pinned copy + event)
            s, i, unc = self.local.search_checked(q_rows, k)
        s, i, flags = self.exchange(s, i, k, flags=unc)

        def research(bad):
            s2, i2 = self.local.search(q_rows[bad], k, verify=True)
            return self.exchange(s2, i2, k)

        pend = Pending(flags, research, s, i)
        if verify == "deferred":
            return s, i, pend
        pend.resolve()
        return s, i

    def exchange(self, s, i, k, flags=None):
        """per-shard (score f64, index i64) [Q, k] -> merged [Q, k]: ONE all-gather of
        the two lists packed as int64 pairs [Q, k, 2] (16 B per entry), then the merge.
        flags (int32 [Q], optional) ride along as one more pair per query and come back
        OR-ed over the shards."""
        packed = torch.stack([s.contiguous().view(torch.int64), i], dim=-1)
        if flags is not None:
            extra = torch.zeros((s.shape[0], 1, 2), dtype=torch.int64, device=s.device)
            extra[:, 0, 0] = flags
            packed = torch.cat([packed, extra], dim=1)
        g = all_gather_stacked(packed, self.group)                 # [R, Q, k(+1), 2]
        ms, mi = self.merge(g[:, :, :k, 0].contiguous().view(torch.float64), g[:, :, :k, 1].contiguous(), k)
        if flags is None:
            return ms, mi
        return ms, mi, g[:, :, k, 0].amax(0).to(torch.int32)


def merge_topk(scores, idx, k):
    """[R, Q, k_in] per-shard lists -> [Q, k] by (score desc, index asc)."""
    return _ops.topk_merge(scores, idx, k)


def mutual_nn(desc1, desc2, precision="fp32"):
    """Mutual nearest-neighbour matcher of HPatchesEval.py:31-43 for unit-norm
    descriptors [N1, D] and [N2, D] (rows): nearest by L2 distance == highest
    dot product, exact order with ties to the lower index like np.argmin.
    Returns int64 [N1]: the match in desc2, or -1 where not mutual."""
    a = desc1.float().contiguous()
    b = desc2.float().contiguous()
    _, n12 = KnnIndex(b, precision).search(a, 1, verify=True)
    _, n21 = KnnIndex(a, precision).search(b, 1, verify=True)
    return _ops.mutual_nn(n12[:, 0], n21[:, 0])
