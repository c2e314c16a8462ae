"""How many Top-K candidates does the sampled threshold let through on the bench's error-feedback
workload (Llama-400M, k = 1 %, four rotating gradients, alpha = 1)?  After W warm-up encodes with
the real encoder, t' = r + alpha x of the next call is formed in torch and the kernel's threshold
rule is replayed per tensor (2 Ki random 16-element runs, a 13-bit magnitude-key histogram, the
bin whose suffix reaches m + 6 sqrt(m) + 32 samples): candidates / k per tensor size, in total,
and with a few other margins and bin resolutions."""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
from omnifed_amd import codec, shapes  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [shapes.numel(s) for _, s in shapes.model_shapes("llama400m")]
plan = codec.Plan.get(sizes, device=dev)
g = torch.Generator(device=dev).manual_seed(1000)
xs = [torch.randn(plan.arena_end, device=dev, generator=g) * 1e-3 for _ in range(4)]
res = torch.zeros(plan.arena_end, device=dev)
ks = plan.topk_ks(0.01)
K = sum(ks)
vals = torch.empty(K, device=dev)
idx = torch.empty(K, dtype=torch.int64, device=dev)
W = int(sys.argv[1]) if len(sys.argv) > 1 else 8


def key(t):
    return t.abs().view(torch.int32)  # non-negative fp32 bits, monotone in |t|


out = {"warmup_calls": W, "k_total": K}
for w in range(W):
    plan.topk_encode(xs[w % 4], 0.01, residual=res, residual_mode=1, values=vals, indices=idx, alpha=1.0)
torch.cuda.synchronize()
tp = res + xs[W % 4]
gen = torch.Generator(device=dev).manual_seed(7)
for sbits, z, c0 in ((13, 6.0, 32.0), (13, 4.0, 16.0), (15, 6.0, 32.0), (11, 6.0, 32.0)):
    shift = 31 - sbits
    tot = 0
    by_size = {}
    for t, (o, n) in enumerate(zip(plan.offsets, plan.sizes)):
        kt = ks[t]
        v = key(tp[o:o + n])
        nr = min(2048, max(1, (n + 255) // 256))
        if n >= 16:
            starts = torch.randint(0, n - 15, (nr,), device=dev, generator=gen)
            samp = v[(starts[:, None] + torch.arange(16, device=dev)).reshape(-1)]
        else:
            samp = v
        S = samp.numel()
        m = kt * S / n
        want = m + z * math.sqrt(m) + c0
        if m < 16 or want >= S:
            c = n
        else:
            h = torch.bincount((samp >> shift).long(), minlength=1 << sbits)
            suf = torch.flip(torch.cumsum(torch.flip(h, [0]), 0), [0])
            thr = int(torch.nonzero(suf >= math.ceil(want)).max())
            c = int(((v >> shift) >= thr).sum())
        tot += c
        e = by_size.setdefault(n, [0, 0])
        e[0] += c
        e[1] += kt
    out[f"s{sbits}_z{z:g}_c{c0:g}"] = {"cand_over_k": round(tot / K, 3),
                                       "by_size": {str(n): round(a / b, 3) for n, (a, b) in by_size.items()}}
# the same rule on a fresh gradient (no residual): the Gaussian case
print(json.dumps(out), flush=True)
