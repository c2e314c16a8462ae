"""Where the QSGD step's time goes beyond encode + decode (Llama-400M, s = 4, bench.py's shapes):
events around K steps, around K encodes, around K decodes, and the wall clock around K steps."""
import sys, time
import torch
sys.path.insert(0, ".")
from omnifed_amd import codec, shapes

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
plan = codec.Plan.get(sizes, device=dev)
g = torch.Generator(device=dev); g.manual_seed(1000)
x = torch.randn(plan.arena_end, device=dev, generator=g) * 1e-3
s = int(sys.argv[1]) if len(sys.argv) > 1 else 4
L = 2 ** s; w = 1 if L <= 127 else 4; width = 8 * w
q = torch.empty(plan.payload_elems(width), dtype=torch.int8 if w == 1 else torch.int32, device=dev)
norms = torch.empty(plan.nt, dtype=torch.float32, device=dev)
y = torch.empty(plan.arena_end, dtype=torch.float32, device=dev)
st = torch.cuda.current_stream(dev)
enc = lambda i: plan.qsgd_encode(x, s, q_out=q, norm_out=norms, alpha=1.0, seed=5, offset=i)
dec = lambda i: plan.qsgd_decode(q, width, L, norms, y_out=y)
def step(i):
    enc(i); dec(i)
def ev(fn, K=20):
    fn(0); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for i in range(K): fn(i)
    b.record(st); torch.cuda.synchronize()
    return a.elapsed_time(b) / K
def wall(fn, K=20):
    fn(0); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K): fn(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / K
def host(fn, K=20):  # host time per call (enqueue only)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K): fn(i)
    t1 = time.perf_counter(); torch.cuda.synchronize()
    return (t1 - t0) * 1e3 / K
for r in range(3):
    print(f"s={s} round {r}: step events {ev(step):.4f} wall {wall(step):.4f} | enc {ev(enc):.4f} dec {ev(dec):.4f} "
          f"| host enqueue step {host(step):.4f} enc {host(enc):.4f} dec {host(dec):.4f} ms", flush=True)

if len(sys.argv) > 2:  # what makes the first timed steps slow: a fresh plan / buffers, or the GPU's clocks?
    plan2 = codec.Plan(sizes, device=dev)  # a fresh plan on the warm GPU
    q2, n2, y2 = torch.empty_like(q), torch.empty_like(norms), torch.empty_like(y)
    def step2(i):
        plan2.qsgd_encode(x, s, q_out=q2, norm_out=n2, alpha=1.0, seed=5, offset=i)
        plan2.qsgd_decode(q2, width, L, n2, y_out=y2)
    print(f"fresh plan on a warm GPU: step events {ev(step2):.4f} then {ev(step2):.4f}", flush=True)
    time.sleep(2.0)  # the GPU idles
    print(f"after 2 s idle: step events {ev(step):.4f} then {ev(step):.4f}", flush=True)
    time.sleep(2.0)
    a = torch.randn(8192, 8192, device=dev)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:
        a = a @ a.T * 1e-4
    torch.cuda.synchronize()
    print(f"after 2 s idle + 100 ms of GEMMs: step events {ev(step):.4f} then {ev(step):.4f}", flush=True)
