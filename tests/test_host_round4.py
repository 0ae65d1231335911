"""Round-4 host tests (no GPU): the rewritten ragged-batch surface
(PackedSequence, pad_packed_images / pack_padded_images on host tensors,
htime) against the reference behaviour (cirtorch/utils/parallel/
packed_sequence.py:8-96, utils/sequence.py:4-79, utils/general.py:13-27)."""

import numpy as np
import pytest
import torch


def test_packed_sequence_protocol():
    from cirtorch.utils.parallel import PackedSequence
    a, b, c = torch.rand(3, 5, 7), torch.rand(3, 6, 4), torch.rand(2, 6, 4)
    ps = PackedSequence([a, None, b])
    assert len(ps) == 3 and ps[0] is a and ps[1] is None
    assert isinstance(ps[1:], PackedSequence) and len(ps[1:]) == 2
    assert list(iter(ps))[2] is b
    assert ps.dtype == torch.float32 and ps.device == torch.device("cpu") and not ps.all_none
    assert ps.extents == [(5, 7), (0, 0), (6, 4)] and ps.max_extent == (6, 7)
    assert PackedSequence(a, b)[1] is b                           # varargs form
    assert PackedSequence([None, None]).all_none and PackedSequence([None]).dtype is None
    s = ps + PackedSequence([c])
    assert len(s) == 4 and len(ps) == 3
    ps += PackedSequence([c])
    assert len(ps) == 4 and ps[3] is c
    with pytest.raises(TypeError):
        ps + [c]
    with pytest.raises(TypeError):
        PackedSequence([a, b.double()])
    with pytest.raises(TypeError):
        PackedSequence([a, np.zeros(3)])


def test_packed_sequence_contiguous():
    from cirtorch.utils.parallel import PackedSequence
    a, b = torch.rand(2, 4), torch.rand(3, 4)
    cat, idx = PackedSequence([a, None, b]).contiguous
    assert torch.equal(cat, torch.cat([a, b])) and idx.tolist() == [0, 0, 2, 2, 2]
    assert PackedSequence([None]).contiguous == (None, None)
    with pytest.raises(ValueError):
        PackedSequence([a, torch.rand(1, 5)]).contiguous
    # derived on access: still correct after +=
    ps = PackedSequence([a])
    ps += PackedSequence([torch.rand(1, 5)])
    with pytest.raises(ValueError):
        ps.contiguous


def _ref_pad(entries, pad, snap):
    """the reference semantics written out: top-left, pad elsewhere, sizes"""
    live = [t for t in entries if t is not None]
    h = max(t.shape[-2] for t in live)
    w = max(t.shape[-1] for t in live)
    if snap:
        h, w = (h + snap - 1) // snap * snap, (w + snap - 1) // snap * snap
    out = torch.full((len(entries),) + tuple(live[0].shape[:-2]) + (h, w), pad, dtype=live[0].dtype)
    for i, t in enumerate(entries):
        if t is not None:
            out[i, ..., :t.shape[-2], :t.shape[-1]] = t
    return out


@pytest.mark.parametrize("snap", [None, 8])
@pytest.mark.parametrize("pad", [0.0, -2.5])
def test_pad_packed_images_host(snap, pad):
    from cirtorch.utils.parallel import PackedSequence
    from cirtorch.utils.sequence import pad_packed_images, pack_padded_images
    entries = [torch.rand(3, 5, 7), None, torch.rand(3, 6, 4)]
    padded, sizes = pad_packed_images(PackedSequence(entries), pad_value=pad, snap_size_to=snap)
    assert torch.equal(padded, _ref_pad(entries, pad, snap))
    assert [tuple(s) for s in sizes] == [(5, 7), (0, 0), (6, 4)]
    back = pack_padded_images(padded, sizes)
    assert torch.equal(back[0], entries[0]) and torch.equal(back[2], entries[2]) and back[1].numel() == 0
    e2 = [torch.arange(12).view(3, 4), torch.arange(10).view(5, 2)]
    p2, s2 = pad_packed_images(PackedSequence(e2), pad_value=7)
    assert torch.equal(p2, _ref_pad(e2, 7, None)) and p2.dtype == torch.int64


def test_pad_packed_images_errors():
    from cirtorch.utils.parallel import PackedSequence
    from cirtorch.utils.sequence import pad_packed_images
    with pytest.raises(ValueError):
        pad_packed_images(PackedSequence([None, None]))
    with pytest.raises(ValueError):
        pad_packed_images(PackedSequence([torch.rand(3, 4, 4), torch.rand(1, 4, 4)]))
    with pytest.raises(ValueError):
        pad_packed_images(PackedSequence([torch.rand(3, 4, 4), torch.rand(4, 4)]))
    with pytest.raises(ValueError):
        pad_packed_images(PackedSequence([torch.rand(2, 3, 4, 4)]))


@pytest.mark.parametrize("secs,text", [(0, "0s"), (59.4, "59s"), (60, "1m 0s"), (3725, "1h 2m 5s"),
                                       (3600, "1h 0m 0s"), (90061, "1d 1h 1m 1s"), (86400, "1d 0h 0m 0s")])
def test_htime(secs, text):
    from cirtorch.utils.general import htime
    assert htime(secs) == text
