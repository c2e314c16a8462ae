"""A/B (interleaved, one process): the bracketed encoder with the fused finish (default) vs the
separate finish launch (omf_plan_set_debug spec bit 512), Llama-400M s = 4 by default.
Prints one JSON line: per variant, the median over rounds of the mean encode time (HIP events
around `reps` back-to-back encodes) and of an encode + decode step."""
import json
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "llama400m"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
reps = 20
dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes(cfg)]
plan = codec.Plan.get(sizes, device=dev)
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn(plan.arena_end, device=dev, generator=g) * 1e-3
q = torch.empty(plan.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(plan.nt, device=dev)
y = torch.empty(plan.arena_end, device=dev)
st = torch.cuda.current_stream(dev)


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(0)
    a.record(st)
    for i in range(reps):
        fn(i)
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


res = {"fused": {"enc": [], "step": []}, "legacy": {"enc": [], "step": []}}
for r in range(rounds):
    for name, bits in (("fused", 0), ("legacy", 512)):
        plan.set_debug(spec=bits)
        res[name]["enc"].append(timed(lambda i: plan.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=7, offset=i)))
        res[name]["step"].append(timed(lambda i: (plan.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=7, offset=i),
                                                  plan.qsgd_decode(q, 8, 16, nr, y_out=y))))
        plan.check()
plan.set_debug()
out = {"config": cfg, "rounds": rounds, "reps": reps, "strategy": plan.strategy}
for name, d in res.items():
    for k, v in d.items():
        v = sorted(v)
        out[f"{name}_{k}_ms"] = round(v[len(v) // 2], 4)
        out[f"{name}_{k}_ms_all"] = [round(t, 4) for t in d[k]]
print(json.dumps(out), flush=True)
