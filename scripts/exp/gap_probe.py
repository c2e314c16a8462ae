"""Which kernels leave an idle gap before the next launch (experiment, for rocprofv3 --kernel-trace):
Llama-400M bracketed encode + decode with the finish launch's fix phase on (polls the norm
granules) or off (omf_plan_set_debug spec bit 8: no fix, no polling)."""
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
spec = int(sys.argv[1]) if len(sys.argv) > 1 else 0
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
plan = codec.Plan(sizes, device=dev)
x = torch.randn(plan.arena_end, device=dev) * 1e-3
q = torch.empty(plan.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(plan.nt, device=dev)
y = torch.empty(plan.arena_end, device=dev)
plan.set_debug(spec=spec)
for i in range(40):
    plan.qsgd_encode(x, 4, q_out=q, norm_out=nr, alpha=2.0, seed=1, offset=i)
    plan.qsgd_decode(q, 8, 16, nr, y_out=y)
torch.cuda.synchronize()
plan.set_debug()
print("ok", flush=True)
