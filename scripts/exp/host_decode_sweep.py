"""decode_updates_dict to the CPU (pageable pooled arena, the default) and the host round trip on
Llama-400M QSGD s=4, over D2H ring chunk sizes and copy-thread counts (medians of 3 after a warm-up)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from omnifed_amd import hostio, shapes  # noqa: E402
from omnifed_amd.hybrid.communicator.global_grpc_compression import (  # noqa: E402
    build_global_compressor, decode_updates_dict, encode_updates_dict)

dev = torch.device("cuda", 0)
named = shapes.model_shapes("llama400m")
g = torch.Generator(device=dev).manual_seed(1)
upd = {n: torch.randn(s, device=dev, generator=g) * 1e-3 for n, s in named}
comp = build_global_compressor(enabled=True, scheme="qsgd", bit_width=4, device=dev)
layers = encode_updates_dict(upd, comp)
host = {n: t.cpu().pin_memory() for n, t in upd.items()}


def tm(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(sorted(ts)[len(ts) // 2] * 1e3, 2)


out = []
print(json.dumps({"encode_from_host_ms": tm(lambda: encode_updates_dict(host, comp)),
                  "encode_from_device_ms": tm(lambda: encode_updates_dict(upd, comp))}), flush=True)
for mb in (32, 64, 128):
    hostio.RING_CHUNK_BYTES = mb << 20
    for slots in (None, 8, 4):
        r = {"ring_MB": mb, "slots": slots}
        orig = hostio.D2HRing.__init__.__defaults__
        hostio.D2HRing.__init__.__defaults__ = (orig[0], orig[1], slots)
        r["decode_cpu_ms"] = tm(lambda: decode_updates_dict(layers))
        r["roundtrip_ms"] = tm(lambda: decode_updates_dict(encode_updates_dict(host, comp)))
        hostio.D2HRing.__init__.__defaults__ = orig
        print(json.dumps(r), flush=True)
