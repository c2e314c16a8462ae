"""Ring encoder phase pricing (experiment): time with OMF_RING_DBG switches set by the caller."""
import os
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes(sys.argv[1] if len(sys.argv) > 1 else "llama400m")]
p = codec.Plan(sizes, device=dev)
x = torch.randn(p.arena_end, device=dev) * 1e-3
q = torch.empty(p.arena_end, dtype=torch.int8, device=dev)
nr = torch.empty(p.nt, device=dev)
p.set_encode_strategy("ring")
for cfg in (0, 1, 2, 3):
    for bm in (1,):
        p.set_ring(cfg=cfg, big_mode=bm)
        for _ in range(2):
            p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
        e1.record()
        torch.cuda.synchronize()
        print(f"dbg {os.environ.get('OMF_RING_DBG', '0')} cfg {cfg} big {bm}: {e0.elapsed_time(e1) / 10:.4f} ms "
              f"coresident {p.check()}", flush=True)
