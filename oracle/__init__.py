"""CPU oracle for the QSGD / Top-K codec path — TEST INFRASTRUCTURE ONLY.

Everything under ``oracle/`` is a checker.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only to check or to time the reference-equivalent CPU codec beside the
GPU number.  The product path (``omnifed_amd``) never imports it and has no CPU
fallback: when the HIP library is missing it raises.

Pinning: the restatement is checked against golden vectors produced by the
real reference (``/root/reference/src/omnifed/hybrid/...``) imported in the
build container by ``tests/golden/gen_golden.py``; see ``tests/test_oracle_golden.py``.
"""

from .qsgd import (  # noqa: F401
    mt19937_uniforms,
    MTStream,
    qsgd_quantize,
    qsgd_dequantize,
    qsgd_encode_dict,
    storage_width,
)
from .philox import philox4x32_10, philox_uniforms  # noqa: F401
from .topk import TopKOracle, topk_k, topk_sparse, topk_desparse  # noqa: F401
from .aggregate import ps_aggregate, layerwise_decompress  # noqa: F401
