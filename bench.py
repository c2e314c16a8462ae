#!/usr/bin/env python3
"""Benchmark: device-resident QSGD encode+decode of Llama-400M gradients (BASELINE.json metric).

One step = encode (omf_qsgd_encode: norms + stochastic levels + int8 payload, one launch)
+ decode (omf_qsgd_decode, one launch) of one client's full Llama-400M update arena
(183 tensors, 401 122 304 fp32 elements, synthetic N(0,1)*1e-3, random-init shapes),
bit_width 4 (16 levels, int8 wire — the presets' value), on-device Philox draws.
Inputs are resident in HBM before timing starts.

value = algorithmic bytes of all ranks / time, algorithmic bytes per step = (8 + 2w)·N
(encode reads 4N, writes wN; decode reads wN, writes 4N).

  python bench.py [--gpus N --steps K --warmup W --config llama400m --bits 4]
  N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
Each rank is one synthetic client (weak scaling).  For N > 1 the PS weighted sum over
RCCL is timed after the codec steps and reported beside the metric.
"""

from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist

METRIC = "GB/s device-resident QSGD encode+decode, Llama-400M grads, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
HERE = os.path.dirname(os.path.abspath(__file__))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="llama400m")
    ap.add_argument("--bits", type=int, default=4)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip PCIe-inclusive and PS timings")
    return ap.parse_args()


def init_dist(n):
    if n <= 1 and "RANK" not in os.environ:
        return 0, 1, 0
    # the rank's GPU first: RCCL binds its communicator (and barrier) to the current device
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    torch.cuda.set_device(local)
    dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    rank, world = dist.get_rank(), dist.get_world_size()
    return rank, world, local


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(v, world, dev):
    if world == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(named, bits, budget_elems=100_000_000):
    """Reference-equivalent CPU codec (oracle, kind 'port') on a bounded sample of the same workload."""
    import oracle

    torch.manual_seed(0)
    sample, tot = [], 0
    for name, shape in named:
        n = int(np.prod(shape))
        sample.append(torch.randn(n) * 1e-3)
        tot += n
        if tot >= budget_elems:
            break
    threads = torch.get_num_threads()

    def one():
        payloads = []
        for x in sample:  # encode: reference op sequence + tobytes (global_grpc_compression.py:105-116)
            q, norm, w, lv = oracle.qsgd_quantize(x, bits)
            payloads.append((q.numpy().astype(np.int8 if w == 8 else np.int32).tobytes(), norm, w, lv, x.numel()))
        for b, norm, w, lv, n in payloads:  # decode: frombuffer + decompress_quantized (:173-182)
            q = torch.from_numpy(np.frombuffer(b, dtype=np.int8 if w == 8 else np.int32).copy())
            oracle.qsgd_dequantize(q, norm, lv, (n,))

    one()  # warm-up
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        one()
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    w = 1 if 2**bits <= 127 else 4
    return {
        "value": round((8 + 2 * w) * tot / t / 1e9, 4),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"first {len(sample)} tensors of the same Llama-400M arena ({tot} fp32 elements), "
                  f"QSGD s={bits} encode+decode incl. tobytes/frombuffer, median of 3 after 1 warm-up; "
                  f"fp32-gradient rate {4 * tot / t / 1e9:.4f} GB/s",
        "seconds_per_pass": round(t, 4),
    }


def main():
    args = parse()
    rank, world, local = init_dist(args.gpus)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from omnifed_amd import codec, shapes
    from omnifed_amd.build import build

    if rank == 0:
        build()
    barrier(world)
    named = shapes.model_shapes(args.config)
    sizes = [shapes.numel(s) for _, s in named]
    N = sum(sizes)
    plan = codec.Plan.get(sizes, device=dev, chunk=args.chunk)
    s = args.bits
    L = 2**s
    w = 1 if L <= 127 else 4
    width = 8 * w
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    x = torch.randn(plan.arena_end, device=dev, generator=g) * 1e-3
    q = torch.empty(plan.arena_end, dtype=torch.int8 if w == 1 else torch.int32, device=dev)
    norms = torch.empty(plan.nt, dtype=torch.float32, device=dev)
    y = torch.empty(plan.arena_end, dtype=torch.float32, device=dev)
    seed = 0x5EED + rank

    def step(i):
        plan.qsgd_encode(x, s, q_out=q, norm_out=norms, seed=seed, offset=i)
        plan.qsgd_decode(q, width, L, norms, y_out=y)

    for i in range(args.warmup):
        step(i)
    plan.check()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    dt = max_over_ranks(time.perf_counter() - t0, world, dev)
    plan.check()
    alg_bytes_step = (8 + 2 * w) * N
    value = world * alg_bytes_step * args.steps / dt / 1e9

    # --- dominant-kernel roofline: HIP events on the launch stream around each launch
    st = torch.cuda.current_stream(dev)
    reps = max(args.steps, 10)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    evd = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for i in range(reps):
        ev[i][0].record(st)
        plan.qsgd_encode(x, s, q_out=q, norm_out=norms, seed=seed, offset=10_000 + i)
        ev[i][1].record(st)
        evd[i][0].record(st)
        plan.qsgd_decode(q, width, L, norms, y_out=y)
        evd[i][1].record(st)
    torch.cuda.synchronize()
    enc_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    dec_ms = float(np.mean([a.elapsed_time(b) for a, b in evd]))
    enc_bytes = (4 + w) * N
    dec_bytes = (w + 4) * N
    dom_ms, dom_bytes, dom_name = (enc_ms, enc_bytes, plan.encoder_kernel) if enc_ms >= dec_ms else \
        (dec_ms, dec_bytes, "qsgd_decode_flat")
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic = None
    tpath = os.path.join(HERE, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        try:
            with open(tpath) as f:
                tj = json.load(f)
            if tj.get("config") == args.config and tj.get("bits") == s:
                traffic = tj.get("bytes_per_launch", {}).get(dom_name)
        except (OSError, ValueError):
            traffic = None
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": dom_name,
                "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": round(dom_ms, 4),
                "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
                "encode_GBs": round(enc_bytes / enc_ms / 1e6, 1), "decode_GBs": round(dec_bytes / dec_ms / 1e6, 1)}

    extras = {}
    if not args.no_extras and world == 1:
        # PCIe-inclusive rate: host fp32 in -> device encode -> host payload; host payload -> decode -> host fp32
        xh = torch.empty(plan.arena_end, dtype=torch.float32, pin_memory=True)
        xh.copy_(x, non_blocking=False)
        qh = torch.empty(plan.arena_end, dtype=q.dtype, pin_memory=True)
        yh = torch.empty(plan.arena_end, dtype=torch.float32, pin_memory=True)
        xd = torch.empty_like(x)

        def pcie_step(i):
            xd.copy_(xh, non_blocking=True)
            plan.qsgd_encode(xd, s, q_out=q, norm_out=norms, seed=seed, offset=20_000 + i)
            qh.copy_(q, non_blocking=True)
            q.copy_(qh, non_blocking=True)
            plan.qsgd_decode(q, width, L, norms, y_out=y)
            yh.copy_(y, non_blocking=True)

        pcie_step(0)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(5):
            pcie_step(i)
        torch.cuda.synchronize()
        pt = (time.perf_counter() - t1) / 5
        extras["pcie_inclusive"] = {"ms_per_step": round(pt * 1e3, 3),
                                    "algorithmic_GBs": round(alg_bytes_step / pt / 1e9, 2),
                                    "fp32_gradient_GBs": round(4 * N / pt / 1e9, 2)}
        del xh, qh, yh, xd
    if not args.no_extras and world > 1:
        from omnifed_amd.ps import GpuOps, weighted_sum_gather, weighted_sum_reduce

        ops = GpuOps(plan)
        wgt = float(world * (world + 1) / 2)
        acc = torch.empty_like(y)
        bufs = [(torch.empty_like(q), torch.empty_like(norms)) for _ in range(world)] if rank == 0 else None

        def t_op(fn, reps=5):
            fn()
            torch.cuda.synchronize()
            barrier(world)
            ta = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            barrier(world)
            return max_over_ranks((time.perf_counter() - ta) / reps, world, dev)

        t_red = t_op(lambda: weighted_sum_reduce(y, wgt, ops))
        t_gat = t_op(lambda: weighted_sum_gather(q, norms, width, L, acc, wgt, ops, bufs=bufs))
        extras["ps_weighted_sum"] = {"reduce_fp32_ms": round(t_red * 1e3, 3),
                                     "gather_payload_decode_ms": round(t_gat * 1e3, 3),
                                     "fp32_bytes_per_rank": 4 * N, "payload_bytes_per_rank": w * N}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(named, s)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic N(0,1)*1e-3 gradients of the named shapes (no checkpoints)",
            "config": {"workload": f"{args.config} QSGD encode+decode, bit_width {s} ({L} levels, int{8 * w} wire), "
                                   f"philox draws, one client per GPU",
                       "tensors": len(sizes), "elements_per_client": N, "bit_width": s,
                       "algorithmic_bytes_per_step_per_client": alg_bytes_step,
                       "fp32_gradient_GBs": round(world * 4 * N * args.steps / dt / 1e9, 2),
                       "parallelism": f"clients{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            **extras,
        }
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
