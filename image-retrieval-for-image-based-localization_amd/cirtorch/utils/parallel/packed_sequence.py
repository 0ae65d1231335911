"""PackedSequence: a list of variable-size tensors (reference
``cirtorch/utils/parallel/packed_sequence.py:8-96``; same API)."""

import torch


def _all_same(lst):
    return not lst or lst.count(lst[0]) == len(lst)


class PackedSequence:
    def __init__(self, *args):
        tensors = args[0] if len(args) == 1 and isinstance(args[0], list) else list(args)
        for t in tensors:
            if t is not None and not isinstance(t, torch.Tensor):
                raise TypeError("All args must be tensors")
        if not _all_same([t.dtype for t in tensors if t is not None]):
            raise TypeError("All tensors must have the same type")
        if not _all_same([t.device for t in tensors if t is not None]):
            raise TypeError("All tensors must reside on the same device")
        self._tensors = tensors
        self._compatible = _all_same([t.shape[1:] for t in tensors if t is not None])
        self._all_none = all(t is None for t in tensors)

    def __add__(self, other):
        if not isinstance(other, PackedSequence):
            raise TypeError("other must be a PackedSequence")
        return PackedSequence(self._tensors + other._tensors)

    def __iadd__(self, other):
        if not isinstance(other, PackedSequence):
            raise TypeError("other must be a PackedSequence")
        self._tensors += other._tensors
        return self

    def __len__(self):
        return len(self._tensors)

    def __getitem__(self, item):
        if isinstance(item, slice):
            return PackedSequence(*self._tensors[item])
        return self._tensors[item]

    def __iter__(self):
        return iter(self._tensors)

    def cuda(self, device=None, non_blocking=False):
        self._tensors = [t.cuda(device, non_blocking) if t is not None else None for t in self._tensors]
        return self

    def cpu(self):
        self._tensors = [t.cpu() if t is not None else None for t in self._tensors]
        return self

    @property
    def all_none(self):
        return self._all_none

    @property
    def dtype(self):
        return None if self.all_none else next(t.dtype for t in self._tensors if t is not None)

    @property
    def device(self):
        return None if self.all_none else next(t.device for t in self._tensors if t is not None)

    @property
    def contiguous(self):
        if not self._compatible:
            raise ValueError("The tensors in the sequence are not compatible for contiguous view")
        if self.all_none:
            return None, None
        packed, idx = [], []
        for i, t in enumerate(self._tensors):
            if t is not None:
                packed.append(t)
                idx.append(t.new_full((t.size(0),), i, dtype=torch.long))
        return torch.cat(packed, dim=0), torch.cat(idx, dim=0)
