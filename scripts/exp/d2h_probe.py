"""Device-to-host of a decoded fp32 arena into CPU tensors (the CPU placement of
decode_updates_dict): the plain pageable `.cpu()`, a ring of pinned chunks drained into a pageable
tensor by worker-thread memmoves, and a pinned destination (torch's caching host allocator).
Llama-400M arena (1.6 GB), medians of 5 after 2 warm-ups."""
import ctypes
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from omnifed_amd import hostio, shapes  # noqa: E402

N = sum(shapes.numel(s) for _, s in shapes.model_shapes("llama400m"))
dev = torch.device("cuda", 0)
y = torch.randn(N, device=dev)
st = torch.cuda.current_stream(dev)
hostio.retain_host_memory()


def plain():
    return y.cpu()


def pinned_dst():
    out = torch.empty(N, dtype=torch.float32, pin_memory=True)
    out.copy_(y, non_blocking=True)
    st.synchronize()
    return out


def ring(limit, slots):
    def run():
        out = torch.empty(N, dtype=torch.float32)
        raw = y.view(torch.uint8)
        dst = out.data_ptr()
        total = raw.numel()
        ex = hostio.pool()
        with hostio.STAGING.lease("probe", slots * limit) as h:
            base = h.buf.data_ptr()
            futs = [None] * slots

            def land(ev, d, s, n):
                ev.synchronize()
                ctypes.memmove(d, s, n)

            for g, a in enumerate(range(0, total, limit)):
                b = min(a + limit, total)
                s = g % slots
                if futs[s] is not None:
                    futs[s].result()
                h.buf[s * limit:s * limit + b - a].copy_(raw[a:b], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
                futs[s] = ex.submit(land, ev, dst + a, base + s * limit, b - a)
            for f in futs:
                if f is not None:
                    f.result()
        return out

    return run


def med(fn, reps=5, warm=2):
    for _ in range(warm):
        r = fn()
        del r
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t0)
        del r
    ts.sort()
    return round(ts[len(ts) // 2] * 1e3, 2)


ref = y.cpu()
res = {"bytes": 4 * N, "workers": hostio.workers(), "plain_cpu_ms": med(plain), "pinned_dst_ms": med(pinned_dst)}
for limit in (8 << 20, 32 << 20):
    for slots in (4, 8, 16):
        fn = ring(limit, slots)
        assert torch.equal(fn(), ref)
        res[f"ring_{limit >> 20}MiB_x{slots}_ms"] = med(fn)
for w in (4, 16):
    hostio.set_workers(w)
    res[f"ring_8MiB_x16_w{w}_ms"] = med(ring(8 << 20, 16))
print(json.dumps(res), flush=True)
