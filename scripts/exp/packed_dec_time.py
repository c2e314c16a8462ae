"""Device-resident timing of the opt-in packed-wire kernels on Llama-400M (s = 4, b = 6):
omf_qsgd_pack, omf_qsgd_decode_packed and, beside them, the int8 arena decode."""
import json
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [int(torch.Size(s).numel()) for _, s in shapes.model_shapes("llama400m")]
plan = codec.Plan(sizes, device=dev)
x = torch.randn(plan.arena_end, device=dev) * 1e-3
q, nn = plan.qsgd_encode(x, 4, seed=1)
pk = plan.qsgd_pack(q, 8, 16)
y = torch.empty(plan.arena_end, device=dev)


def ev_ms(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


res = {"elements": plan.arena_end,
       "pack_ms": ev_ms(lambda: plan.qsgd_pack(q, 8, 16, packed_out=pk)),
       "decode_packed_ms": ev_ms(lambda: plan.qsgd_decode_packed(pk, 16, nn, y_out=y)),
       "decode_int8_ms": ev_ms(lambda: plan.qsgd_decode(q, 8, 16, nn, y_out=y)),
       "decode_packed_acc_ms": ev_ms(lambda: plan.qsgd_decode_packed(pk, 16, nn, y_out=y, accumulate=True))}
n = plan.arena_end
res["decode_packed_GBs"] = round((0.75 * n + 4 * n) / res["decode_packed_ms"] / 1e6, 1)
print(json.dumps({k: round(v, 4) if isinstance(v, float) else v for k, v in res.items()}))
