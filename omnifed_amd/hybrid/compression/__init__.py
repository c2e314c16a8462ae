"""Drop-in for ``src.omnifed.hybrid.compression`` (reference ``__init__.py:3-21``), GPU-backed."""

from .core import (
    Compression,
    ResidualMemory,
    ResidualUpdates,
    layerwise_decompress,
)
from .qsgd import QSGD_COMPRESSION_NAME, QSGD_PACKED_COMPRESSION_NAME, QSGDQuantCompression
from .topk import TOPK_COMPRESSION_NAME, TopKCompression

__all__ = [
    "Compression",
    "ResidualMemory",
    "ResidualUpdates",
    "TopKCompression",
    "TOPK_COMPRESSION_NAME",
    "QSGDQuantCompression",
    "QSGD_COMPRESSION_NAME",
    "QSGD_PACKED_COMPRESSION_NAME",
    "layerwise_decompress",
]
