"""PackedSequence — the ragged image batch at the model boundary.

Surface of the reference ``cirtorch/utils/parallel/packed_sequence.py:8-96``
(constructor from a list or varargs, ``+`` / ``+=``, ``len``, indexing and
slicing, iteration, in-place ``cuda()`` / ``cpu()``, ``all_none`` / ``dtype`` /
``device``, ``contiguous`` -> (concatenation along dim 0, owner index per row)),
the same exception types on bad input.

On the MI355X engine a PackedSequence is never padded on the way into the
body: ``ResNet.forward`` hands the entries to the stem as a ragged table
(per-image device address + extent, ``rr_stem_conv_pool_ragged`` /
``rr_image_to_nhwc_ragged``) and the stem reads the max-extent batch map
on the fly.  ``extents`` / ``max_extent`` describe that table.  Properties are
derived from the current entries on every access, so they stay correct after
``+=``.
"""

import torch


def _distinct(values):
    seen = []
    for v in values:
        if v not in seen:
            seen.append(v)
    return seen


class PackedSequence:
    __slots__ = ("_tensors",)

    def __init__(self, *args):
        entries = args[0] if len(args) == 1 and isinstance(args[0], list) else args
        entries = list(entries)
        live = [t for t in entries if t is not None]
        if not all(isinstance(t, torch.Tensor) for t in live):
            raise TypeError("PackedSequence entries must be torch tensors or None")
        if len(_distinct(t.dtype for t in live)) > 1:
            raise TypeError("PackedSequence entries must share one dtype")
        if len(_distinct(t.device for t in live)) > 1:
            raise TypeError("PackedSequence entries must live on one device")
        self._tensors = entries

    # ------------------------------------------------------------- sequence protocol
    def _check_other(self, other):
        if not isinstance(other, PackedSequence):
            raise TypeError("can only concatenate a PackedSequence to a PackedSequence")

    def __add__(self, other):
        self._check_other(other)
        return PackedSequence(self._tensors + other._tensors)

    def __iadd__(self, other):
        self._check_other(other)
        self._tensors = self._tensors + other._tensors
        return self

    def __len__(self):
        return len(self._tensors)

    def __getitem__(self, item):
        picked = self._tensors[item]
        return PackedSequence(picked) if isinstance(item, slice) else picked

    def __iter__(self):
        return iter(self._tensors)

    # ------------------------------------------------------------- placement (in place)
    def _map(self, fn):
        self._tensors = [None if t is None else fn(t) for t in self._tensors]
        return self

    def cuda(self, device=None, non_blocking=False):
        return self._map(lambda t: t.cuda(device, non_blocking))

    def cpu(self):
        return self._map(lambda t: t.cpu())

    # ------------------------------------------------------------- properties
    def _live(self):
        return [t for t in self._tensors if t is not None]

    @property
    def all_none(self):
        return not self._live()

    @property
    def dtype(self):
        live = self._live()
        return live[0].dtype if live else None

    @property
    def device(self):
        live = self._live()
        return live[0].device if live else None

    @property
    def extents(self):
        """(H_i, W_i) of every entry ((0, 0) for None): the ragged table's extents."""
        return [(0, 0) if t is None else (int(t.shape[-2]), int(t.shape[-1])) for t in self._tensors]

    @property
    def max_extent(self):
        """the batch map (max H, max W) the engine pads the entries to on the fly"""
        ext = [e for e, t in zip(self.extents, self._tensors) if t is not None]
        return (max(h for h, _ in ext), max(w for _, w in ext)) if ext else (0, 0)

    @property
    def contiguous(self):
        """(entries concatenated along dim 0, index of the entry each row came from);
        the entries' trailing dims must agree."""
        live = [(i, t) for i, t in enumerate(self._tensors) if t is not None]
        if len(_distinct(tuple(t.shape[1:]) for _, t in live)) > 1:
            raise ValueError("PackedSequence entries differ beyond dim 0: no contiguous view")
        if not live:
            return None, None
        owners = torch.tensor([i for i, _ in live], dtype=torch.long, device=live[0][1].device)
        rows = torch.tensor([t.shape[0] for _, t in live], dtype=torch.long, device=live[0][1].device)
        return torch.cat([t for _, t in live], dim=0), torch.repeat_interleave(owners, rows)
