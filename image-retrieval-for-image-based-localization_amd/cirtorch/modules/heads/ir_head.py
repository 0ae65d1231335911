"""Reference keeps a byte-identical copy of globalHead under the old name
(``cirtorch/modules/heads/ir_head.py``)."""
from .global_head import globalHead as ImageRetrievalHead  # noqa: F401
