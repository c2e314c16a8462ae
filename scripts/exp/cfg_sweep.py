"""Time every ring configuration on the Llama-400M arena (experiment)."""
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
p = codec.Plan(sizes, device=dev)
x = torch.randn(p.arena_end, device=dev) * 1e-3
q = torch.empty(p.payload_elems(8), dtype=torch.int8, device=dev)
nr = torch.empty(p.nt, device=dev)


def tm(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
nin = nr.clone()
print("flat(norm in)", round(tm(lambda: p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1, norm_in=nin)), 4), flush=True)
cfgs = [int(c) for c in sys.argv[1:]] or [0, 5, 6, 7, 8, 9, 10]
for cfg in cfgs:
    for big in (1, 0):
        p.set_ring(cfg=cfg, big_mode=big)
        t = tm(lambda: p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1))
        ok = p.check()
        info = p.ring_info
        print(f"cfg {cfg} big {big} {t:.4f} ms  two_pass {info['two_pass_tensors']} hold {info['hold_max']} ok {ok}",
              flush=True)
