"""ResNet-18 / small-arena encoder strategies, interleaved (experiment): encode and encode+decode
per strategy, events around 50 back-to-back calls, median of 7 rounds."""
import json
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
res = {}
for cfg, s in (("resnet18", 3), ("resnet18", 8), ("llama150m", 4)):
    sizes = [shapes.numel(sh) for _, sh in shapes.model_shapes(cfg)]
    plan = codec.Plan(sizes, device=dev)
    x = torch.randn(plan.arena_end, device=dev) * 1e-3
    w = 1 if 2**s <= 127 else 4
    q = torch.empty(plan.payload_elems(8 * w), dtype=torch.int8 if w == 1 else torch.int32, device=dev)
    nr = torch.empty(plan.nt, device=dev)
    y = torch.empty(plan.arena_end, device=dev)
    strategies = ["ring", "grid", "bracket"] if s <= 4 else ["ring", "grid", "ordered"]
    times = {st: {"enc": [], "step": []} for st in strategies}
    for rnd in range(7):
        for st in strategies:
            plan.set_encode_strategy(st)
            for mode in ("enc", "step"):
                for i in range(3):
                    plan.qsgd_encode(x, s, q_out=q, norm_out=nr, alpha=2.0, seed=1, offset=i)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(50):
                    plan.qsgd_encode(x, s, q_out=q, norm_out=nr, alpha=2.0, seed=1, offset=i)
                    if mode == "step":
                        plan.qsgd_decode(q, 8 * w, 2**s, nr, y_out=y)
                e1.record()
                torch.cuda.synchronize()
                times[st][mode].append(e0.elapsed_time(e1) / 50 * 1e3)
            assert plan.check() is not None
    res[f"{cfg}_s{s}"] = {st: {m: round(sorted(v)[3], 2) for m, v in d.items()} for st, d in times.items()}
    print(json.dumps({f"{cfg}_s{s}": res[f"{cfg}_s{s}"]}), flush=True)
