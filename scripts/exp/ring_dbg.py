"""Ring encoder phase pricing (experiment): time with OMF_RING_DBG switches set by the caller (applied with Plan.set_debug)."""
import os
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
cfgs = [int(c) for c in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0]
p = codec.Plan(sizes, device=dev)
x = torch.randn(p.arena_end, device=dev) * 1e-3
q = torch.empty(p.arena_end, dtype=torch.int8, device=dev)
nr = torch.empty(p.nt, device=dev)
p.set_encode_strategy("ring")
p.set_debug(ring=int(os.environ.get("OMF_RING_DBG", "0")))
for cfg in cfgs:
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

if int(os.environ.get("OMF_RING_DBG", "0")) & 4:
    names = ["L wait free slot", "L load+reduce", "Q wait loaded", "poller resolve", "Q wait norm", "Q tiles",
             "L total", "Q total"]
    for cfg in cfgs:
        if cfg == 3:
            names = ["-", "publish", "resolve norm", "quantise", "-", "-", "total", "-"]
        p.set_ring(cfg=cfg, big_mode=1)
        p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
        p.ring_profile()
        p.qsgd_encode(x, 4, q_out=q, norm_out=nr, seed=1)
        prof = p.ring_profile()
        lw, qw = 8, 8
        waves = {0: lw, 1: lw, 2: qw, 3: 1, 4: qw - 1, 5: qw, 6: lw, 7: qw} if cfg != 3 else {i: 16 for i in range(8)}
        for i, nm in enumerate(names):
            per_wave = prof[i] / (256 * waves[i])
            print(f"  {nm:18s} {per_wave / 2400:10.1f} us/wave (shader cycles / 2.4 GHz)", flush=True)

