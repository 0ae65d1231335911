from .packed_sequence import PackedSequence  # noqa: F401
