"""Stress every ring configuration under the debug timing modes (OMF_RING_DBG set by the caller, applied with Plan.set_debug):
20 launches each on Llama-400M and on a mixed small arena; prints one line per configuration."""
import os
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
cfgs = [int(c) for c in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1, 2, 3, 4]
arenas = {"llama400m": [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")],
          "mixed": [7, 1000, 16384, 40000, 70001, 3, 1 << 20, 5_000_000, 17, 300_000]}
for name, sizes in arenas.items():
    p = codec.Plan(sizes, device=dev)
    p.set_encode_strategy("ring")
    p.set_debug(ring=int(os.environ.get("OMF_RING_DBG", "0")))
    x = torch.randn(p.arena_end, device=dev) * 1e-3
    for cfg in cfgs:
        for hold in (0, 3):
            p.set_ring(cfg=cfg, hold_max=hold)
            for i in range(20):
                p.qsgd_encode(x, 4 if i % 2 else 8, seed=i)
            torch.cuda.synchronize()
            print(f"dbg {os.environ.get('OMF_RING_DBG', '0')} {name} cfg {cfg} hold {hold}: ok coresident {p.check()}",
                  flush=True)
