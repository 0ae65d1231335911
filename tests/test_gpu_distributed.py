"""Sharded matching with the REAL kernels across processes (gloo, world 2 and
3, every rank on cuda:0): per-shard HIP KnnIndex search, all-gather of the
(score, index) lists through host copies, HIP rr_topk_merge — bit-identical
to one search of the whole database (the reference never gathers: scripts/
train_globalF.py:652-657,678,720).  World 3 with a 2-row database leaves one
rank with an empty shard, which must contribute sentinels instead of hanging
the gather."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, d, q, k, prec, ret, verify=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "image-retrieval-for-image-based-localization_amd"),
              os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cirtorch import _ops
        from cirtorch.search import ShardedIndex, shard_range, all_gather_stacked
        dev = torch.device("cuda", 0)
        r0, nl = shard_range(n, rank, world)
        db = _ops.fill_unit_rows(n, d, seed=0x5EED1, device=dev)[r0:r0 + nl].contiguous()
        idx = ShardedIndex(db, r0, precision=prec)
        # each rank extracts its own queries, then all of them are gathered (bench.py step)
        qs = _ops.fill_unit_rows(q * world, d, seed=0x5EED2, device=dev)[rank * q:(rank + 1) * q].contiguous()
        qa = all_gather_stacked(qs).reshape(world * q, d)
        if verify == "deferred":
            s, i, pend = idx.search(qa, k, verify="deferred")
            n_re = pend.resolve()
        else:
            s, i = idx.search(qa, k, verify=verify)
            n_re = -1
        torch.cuda.synchronize()
        ret[rank] = (s.cpu().numpy(), i.cpu().numpy(), n_re)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,prec", [(2, 30000, "bf16"), (2, 20011, "fp16"), (3, 2, "fp32"), (2, 70001, "int8"),
                                          (3, 5, "int8")])
def test_sharded_real_kernels_equal_single_search(cuda, world, n, prec):
    from cirtorch import _ops
    from cirtorch.search import KnnIndex
    d, q, k = 256, 3, 50
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), n, d, q, k, prec, ret), nprocs=world, join=True,
                       start_method="spawn")
    db = _ops.fill_unit_rows(n, d, seed=0x5EED1, device=cuda)
    qa = _ops.fill_unit_rows(q * world, d, seed=0x5EED2, device=cuda)
    s1, i1 = KnnIndex(db, prec).search(qa, k)
    s1, i1 = s1.cpu().numpy(), i1.cpu().numpy()
    for r in range(world):
        s, i, _ = ret[r]
        np.testing.assert_array_equal(i, i1)
        np.testing.assert_array_equal(s, s1)
    if n < k:
        assert (i1[:, n:] == -1).all()


@pytest.mark.parametrize("world,n,prec,verify", [(2, 70001, "fp16", "deferred"), (2, 70001, "int8", "deferred"),
                                                 (3, 40000, "bf16", True)])
def test_sharded_real_kernels_certified(cuda, world, n, prec, verify):
    """The certified sharded search: each shard's certificate travels in the
    top-k all-gather, every rank re-searches the same uncertain queries and
    exchanges again -- the merged result equals the exact oracle on every rank,
    and every rank reports the same re-searched count."""
    from cirtorch import _ops
    from oracle import ops
    d, q, k = 256, 3, 50
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), n, d, q, k, prec, ret, verify), nprocs=world, join=True,
                       start_method="spawn")
    db = _ops.fill_unit_rows(n, d, seed=0x5EED1, device=cuda).cpu().numpy()
    qa = _ops.fill_unit_rows(q * world, d, seed=0x5EED2, device=cuda).cpu().numpy()
    ref_s, ref_i = ops.topk_exact(db, qa, k)
    counts = set()
    for r in range(world):
        s, i, n_re = ret[r]
        np.testing.assert_array_equal(i, ref_i)
        np.testing.assert_allclose(s, ref_s, rtol=0, atol=1e-12)
        counts.add(n_re)
    assert len(counts) == 1


def test_c_abi_rccl_single_rank_merge(cuda):
    """The C-ABI sharded-search exchange (rr_comm_* + rr_topk_allgather_merge,
    RCCL dlopen'ed by librr.so) on a 1-rank communicator: the all-gather +
    merge of one shard's top-k is that shard's top-k, bit for bit, and equals
    the Python ShardedIndex path (world 1)."""
    import ctypes
    from cirtorch import _engine as E
    from cirtorch.search import KnnIndex
    from oracle import data
    lib = E.lib()
    db = torch.from_numpy(data.unit_rows(50000, 256, seed=61)).to(cuda)
    q = torch.from_numpy(data.unit_rows(16, 256, seed=62)).to(cuda)
    k = 20
    s, i = KnnIndex(db, "bf16").search(q, k)
    idbuf = ctypes.create_string_buffer(128)
    E.check(lib.rr_comm_unique_id(idbuf, 128), "rr_comm_unique_id")
    comm = ctypes.c_void_p()
    E.check(lib.rr_comm_init(ctypes.byref(comm), 1, idbuf, 128, 0), "rr_comm_init")
    try:
        nbytes = lib.rr_topk_allgather_workspace_bytes(1, q.shape[0], k)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=cuda)
        os_ = torch.empty_like(s)
        oi = torch.empty_like(i)
        E.check(lib.rr_topk_allgather_merge(comm, E.ptr(s), E.ptr(i), q.shape[0], k, E.ptr(os_), E.ptr(oi),
                                            E.ptr(ws), nbytes, E.stream_ptr(cuda)), "rr_topk_allgather_merge")
        torch.cuda.synchronize()
        assert torch.equal(oi, i) and torch.equal(os_, s)
    finally:
        E.check(lib.rr_comm_destroy(comm), "rr_comm_destroy")
