#!/usr/bin/env python3
"""Cost of the reference's tie rule on the Llama-400M Top-K encode (tie_order "torch" vs "index").

    python scripts/topk_order_bench.py [out.json] [--verify]

Error-feedback calls with a fresh N(0, 1e-3) gradient each (bench.py's Top-K workload): wall time
of Plan.topk_encode per call with the device order alone and with omf_topk_torch_order after it,
and how many tensors the census rewrote.  --verify checks one torch-order call against the oracle
(torch.topk on the CPU, every tensor: values, indices and residual bytes).
"""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from omnifed_amd import codec, shapes  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else None
    verify = "--verify" in sys.argv
    dev = torch.device("cuda", 0)
    named = shapes.model_shapes("llama400m")
    sizes = [shapes.numel(s) for _, s in named]
    plan = codec.Plan.get(sizes, device=dev)
    g = torch.Generator(device=dev).manual_seed(3)
    res = {"config": "llama400m", "ratio": 0.01, "tensors": len(sizes), "elements": sum(sizes),
           "host_threads": os.cpu_count()}
    for order in ("index", "torch"):
        r = torch.empty(plan.arena_end, device=dev)
        times, reord = [], []
        for call in range(8):
            x = torch.randn(plan.arena_end, device=dev, generator=g) * 1e-3
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            plan.topk_encode(x, 0.01, residual=r, residual_mode=2 if call == 0 else 1, tie_order=order)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
            reord.append(plan.topk_reordered if order == "torch" else 0)
            print(order, call, round(times[-1], 2), reord[-1], flush=True)
        res[order] = {"ms_per_call": times, "median_ms": sorted(times[2:])[len(times[2:]) // 2],
                      "tensors_rewritten": reord}
    if verify:
        import oracle

        r = torch.empty(plan.arena_end, device=dev)
        x = torch.randn(plan.arena_end, device=dev, generator=g) * 1e-3
        v, i, ks = plan.topk_encode(x, 0.01, residual=r, residual_mode=2, tie_order="torch")
        vh, ih, rh, xh = v.cpu(), i.cpu(), r.cpu(), x.cpu()
        K, bad = 0, []
        t0 = time.perf_counter()
        for t, (o, n) in enumerate(zip(plan.offsets, sizes)):
            k = ks[t]
            ov, oi = oracle.topk_sparse(xh[o:o + n], 0.01)
            want = xh[o:o + n].clone()
            want[oi] = 0.0
            if not (ih[K:K + k].numpy().tobytes() == oi.numpy().tobytes()
                    and vh[K:K + k].numpy().tobytes() == ov.numpy().tobytes()
                    and rh[o:o + n].numpy().tobytes() == want.numpy().tobytes()):
                bad.append(t)
            K += k
        res["verify"] = {"tensors": len(sizes), "mismatched": bad, "rewritten": plan.topk_reordered,
                         "oracle_s": round(time.perf_counter() - t0, 1)}
        print("verify", res["verify"], flush=True)
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps({k: (v if not isinstance(v, dict) else {kk: vv for kk, vv in v.items() if kk != "ms_per_call"})
                      for k, v in res.items()}))


if __name__ == "__main__":
    main()
