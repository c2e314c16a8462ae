"""Encode / step time of one library build (OMF_CODEC_LIB_EXPERIMENT selects a variant): HIP events
around 20 calls, median of 7 rounds.  One JSON line.
usage: enc_time.py [config=llama400m] [bits=4] [strategy=the plan's default] [value_format=0] [u=0]
(value_format 1 bf16 / 2 fp16; u=1: caller uniforms, the parity mode's input)"""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes(sys.argv[1] if len(sys.argv) > 1 else "llama400m")]
p = codec.Plan(sizes, device=dev)
bits = int(sys.argv[2]) if len(sys.argv) > 2 else 4
if len(sys.argv) > 3:
    p.set_encode_strategy(sys.argv[3])
fmt = int(sys.argv[4]) if len(sys.argv) > 4 else 0
use_u = len(sys.argv) > 5 and sys.argv[5] == "1"
L = 2 ** bits
w = 8 if L <= 127 else 32
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn(p.arena_end, device=dev, generator=g) * 1e-3
if fmt:  # the exact fp32 upcast of a half tensor
    x = x.to(torch.bfloat16 if fmt == 1 else torch.float16).float()
u = torch.rand(p.arena_end, device=dev, generator=g) if use_u else None
q = torch.empty(p.payload_elems(w), dtype=torch.int8 if w == 8 else torch.int32, device=dev)
nr = torch.empty(p.nt, device=dev)
y = torch.empty(p.arena_end, device=dev)
st = torch.cuda.current_stream(dev)


def tm(fn, reps=20):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(0)
    a.record(st)
    for i in range(reps):
        fn(i)
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


enc, step = [], []
for _ in range(7):
    enc.append(tm(lambda i: p.qsgd_encode(x, bits, q_out=q, norm_out=nr, seed=7, offset=i, value_format=fmt, u=u)))
    step.append(tm(lambda i: (p.qsgd_encode(x, bits, q_out=q, norm_out=nr, seed=7, offset=i, value_format=fmt, u=u),
                              p.qsgd_decode(q, w, L, nr, y_out=y))))
p.check()
print(json.dumps({"lib": os.path.basename(os.environ.get("OMF_CODEC_LIB_EXPERIMENT", "base")), "bits": bits,
                  "strategy": p.strategy, "value_format": fmt, "u": use_u,
                  "enc_ms": round(sorted(enc)[3], 4), "step_ms": round(sorted(step)[3], 4),
                  "payload_sha": __import__("hashlib").sha256(q.cpu().numpy().tobytes()).hexdigest()[:16]}), flush=True)
