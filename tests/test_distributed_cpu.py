"""World-size-2 gloo test of the sharded matching path (CPU).

The product's sharding / gather / merge plumbing (cirtorch.search.ShardedIndex,
shard_range, all_gather_stacked) runs for real over torch.distributed (gloo);
only the two compute kernels are replaced by CPU stand-ins from the oracle
(the HIP versions are covered by tests/test_gpu_knn.py::test_topk_merge_*)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _CpuLocal:
    def __init__(self, rows, row0):
        self.rows, self.row0 = rows, row0
        self.ntotal = rows.shape[0]

    def search(self, q, k, verify=False):
        from oracle import ops
        s, i = ops.topk_exact(self.rows.numpy(), q.numpy(), k)
        if i.shape[1] < k:  # shard smaller than k: pad like the kernel (-1)
            pad = k - i.shape[1]
            s = np.concatenate([s, np.full((s.shape[0], pad), -np.inf)], 1)
            i = np.concatenate([i, np.full((i.shape[0], pad), -1 - self.row0)], 1)
        return torch.from_numpy(s), torch.from_numpy(i + self.row0)


class _CpuLocalFlaky(_CpuLocal):
    """A shard whose unverified screen misses its best row for some queries and
    flags exactly those (the certificate), so only the verified merge is exact."""

    def search(self, q, k, verify=False):
        s, i = _CpuLocal.search(self, q, k)
        if verify is True:
            return s, i
        return self.search_checked(q, k)[:2]

    def search_checked(self, q, k):
        """(scores, idx, uncertain flags) -- ShardedIndex's certified path"""
        unc = torch.tensor([(j + self.row0) % 3 == 0 for j in range(q.shape[0])], dtype=torch.int32)
        bad_rows = torch.nonzero(unc).flatten()
        s, i = _CpuLocal.search(self, q, k)
        s2, i2 = _CpuLocal.search(self, q, k + 1)
        s, i = s.clone(), i.clone()
        s[bad_rows], i[bad_rows] = s2[bad_rows, 1:], i2[bad_rows, 1:]     # the best row lost
        return s, i, unc


def _cpu_merge(gs, gi, k):
    R, Q, kin = gs.shape
    s = gs.permute(1, 0, 2).reshape(Q, R * kin).numpy()
    i = gi.permute(1, 0, 2).reshape(Q, R * kin).numpy()
    out_s, out_i = np.empty((Q, k)), np.empty((Q, k), dtype=np.int64)
    for q in range(Q):
        valid = i[q] >= 0
        ss, ii = s[q][valid], i[q][valid]
        o = np.lexsort((ii, -ss))[:k]
        out_s[q], out_i[q] = ss[o], ii[o]
    return torch.from_numpy(out_s), torch.from_numpy(out_i)


def _worker(rank, world, port, n, d, q, k, ret, verify=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cirtorch.search import ShardedIndex, shard_range, all_gather_stacked
        from oracle import data
        db = torch.from_numpy(data.unit_rows(n, d, seed=91))
        r0, nl = shard_range(n, rank, world)
        local = (_CpuLocalFlaky if verify else _CpuLocal)(db[r0:r0 + nl], r0)
        idx = ShardedIndex(None, r0, local_index=local, merge=_cpu_merge)
        # each rank "extracts" its own queries, then all-gathers them (bench.py step)
        qs = torch.from_numpy(data.unit_rows(q * world, d, seed=92))[rank * q:(rank + 1) * q]
        qa = all_gather_stacked(qs).reshape(world * q, d)
        if verify == "deferred":
            s, i, pend = idx.search(qa, k, verify="deferred")
            wrong = int((i != torch.from_numpy(idx_exact(db, qa, k))).any(1).sum())
            n_re = pend.resolve()
            ret[rank] = (s.numpy(), i.numpy(), n_re, wrong)
        elif verify:
            s, i = idx.search(qa, k, verify=True)
            ret[rank] = (s.numpy(), i.numpy())
        else:
            s, i = idx.search(qa, k, verify=False)
            ret[rank] = (s.numpy(), i.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_search_equals_single(world):
    n, d, q, k = 3001, 64, 3, 17
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, d, q, k, ret), nprocs=world, join=True)
    from oracle import data, ops
    db = data.unit_rows(n, d, seed=91)
    qa = data.unit_rows(q * world, d, seed=92)
    ref_s, ref_i = ops.topk_exact(db, qa, k)
    for r in range(world):
        s, i = ret[r]
        np.testing.assert_array_equal(i, ref_i)
        np.testing.assert_allclose(s, ref_s, rtol=0, atol=1e-15)


def idx_exact(db, qa, k):
    from oracle import ops
    return ops.topk_exact(db.numpy(), qa.numpy(), k)[1]


@pytest.mark.parametrize("verify", [True, "deferred"])
def test_sharded_verified_search_flags_travel_with_the_lists(verify):
    """verify: every shard certifies its own top-k; the uncertain flags ride in the
    same all-gather as the (score, index) lists, so both ranks see the same
    uncertain set, re-search it and exchange once more -- the merged result is
    exact although each shard's unverified screen missed rows."""
    world, n, d, q, k = 2, 3001, 64, 4, 17
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, d, q, k, ret, verify), nprocs=world, join=True)
    from oracle import data, ops
    db = data.unit_rows(n, d, seed=91)
    qa = data.unit_rows(q * world, d, seed=92)
    ref_s, ref_i = ops.topk_exact(db, qa, k)
    for r in range(world):
        np.testing.assert_array_equal(ret[r][1], ref_i)
        np.testing.assert_allclose(ret[r][0], ref_s, rtol=0, atol=1e-15)
        if verify == "deferred":
            n_re, wrong = ret[r][2], ret[r][3]
            # rank 0 flags queries 0, 3, 6; rank 1 (row0 = 1501) flags 2, 5: the union
            assert n_re == 5 and 0 < wrong <= 5


def test_shard_range_covers_rows():
    from cirtorch.search import shard_range
    for n in (1, 7, 1000, 1_000_000):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert sum(nl for _, nl in spans) == n
            pos = 0
            for r0, nl in spans:
                if nl:
                    assert r0 == pos
                pos += nl
