"""The codec's LayerStates inside the REFERENCE's own generated messages (build container only).

The reference's unchanged client and server put the codec's LayerStates into their own
generated ``global_grpc_pb2.ModelUpdate`` / ``ModelParameters``
(src/omnifed/hybrid/communicator/global_grpc_client.py:75-80, global_grpc_server.py:226-230).
With that module imported (here through gen_golden.py's import shim, in a subprocess so the
shim never leaks into other tests), every LayerState the codec's builders make must be an
instance of the reference's class, construct those messages and round-trip.  Skipped where
the reference tree is absent (the GPU box): tests/test_gpu_r2.py covers the same behaviour
with a stand-in generated module.
"""

import os
import subprocess
import sys

import pytest

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

SCRIPT = r"""
import sys
sys.path.insert(0, {golden!r}); sys.path.insert(0, {root!r})
from gen_golden import _install_shim
_install_shim()
import numpy as np, torch
from src.omnifed.hybrid.communicator import global_grpc_pb2 as ref_pb2
from omnifed_amd.hybrid.communicator import global_grpc_pb2 as ours
from omnifed_amd.hybrid.communicator.global_grpc_compression import (
    _encode_dense_layer, decode_layer_tensor, qsgd_layer_from_payload, topk_layer_from_payload)

assert ours.active_module() is ref_pb2
layers = [qsgd_layer_from_payload("w", (2, 3), bytes([1, 255, 0, 3, 2, 1]), 0.5, 8, 16),
          topk_layer_from_payload("t", (10,), np.array([0.5, -1.0], np.float32), np.array([3, 7])),
          _encode_dense_layer("d", torch.tensor([[1.5, -2.0]]))]
assert all(type(L) is ref_pb2.LayerState for L in layers)
up = ref_pb2.ModelUpdate(client_id="c0", round_number=2, layers=layers, number_samples=48)
mp = ref_pb2.ModelParameters(round_number=2, layers=layers, is_ready=True)
back = ref_pb2.ModelUpdate(); back.ParseFromString(up.SerializeToString())
assert [L.layer_name for L in back.layers] == ["w", "t", "d"]
# the private schema serialises identically
priv = ours.LayerState(); priv.ParseFromString(layers[0].SerializeToString())
assert priv.SerializeToString() == layers[0].SerializeToString()
assert decode_layer_tensor(back.layers[2]).tolist() == [[1.5, -2.0]]
# an injected module wins over the automatic choice; None restores it
ours.set_wire_module(ours)
assert type(qsgd_layer_from_payload("w", (1,), b"\x01", 1.0, 8, 16)) is ours.LayerState
ours.set_wire_module(None)
assert ours.active_module() is ref_pb2
try:
    ref_pb2.ModelUpdate(layers=[ours.LayerState(layer_name="x")])
except TypeError:
    pass
else:
    raise AssertionError("a foreign-pool LayerState was accepted")
print("INTEROP-OK")
"""


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_layer_states_are_the_reference_pb2_classes():
    code = SCRIPT.format(golden=os.path.join(HERE, "golden"), root=os.path.dirname(HERE))
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "INTEROP-OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
