"""PS aggregate-after-decode oracle — TEST INFRASTRUCTURE ONLY.

* ``ps_aggregate`` ↔ ``CentralServerServicer._accumulate_model_updates`` +
  ``_apply_model_updates`` (global_grpc_server.py:147-171): ``acc += decoded``
  per client in arrival order (here: the order given), then
  ``acc / total_samples`` (fp32 ÷ int).
* ``layerwise_decompress`` ↔ core.py:62-71: sparse scatter-add of every
  client's (values, indices), then ``/ client_count``.
"""

from __future__ import annotations

from typing import Sequence

import torch


def ps_aggregate(decoded: Sequence[torch.Tensor], total_samples: int, compute_mean: bool = True):
    acc = torch.zeros_like(decoded[0])
    for y in decoded:
        acc += y
    if compute_mean:
        return acc / total_samples
    return acc


def layerwise_decompress(collected_vals, collected_ix, tensor_shape, client_count):
    t = torch.zeros(tensor_shape).view(-1)
    for v, ix in zip(collected_vals, collected_ix):
        t.data[ix] += v
    t /= client_count
    return t.reshape(tensor_shape)
