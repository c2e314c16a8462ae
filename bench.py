#!/usr/bin/env python3
"""Benchmark: device-resident QSGD encode+decode of Llama-400M gradients (BASELINE.json metric).

One step = encode (omf_qsgd_encode: norms + stochastic levels + int8 payload, one launch,
the client weighting ``param * batch_samples`` fused as alpha) + decode (omf_qsgd_decode,
one launch) of one client's full Llama-400M update arena (183 tensors, 401 122 304 fp32
elements, synthetic N(0,1)*1e-3, random-init shapes), bit_width 4 (16 levels, int8 wire —
the presets' value), on-device Philox draws.  Inputs are resident in HBM before timing.

value = algorithmic bytes of all ranks / time, algorithmic bytes per step = (8 + 2w)·N
(encode reads 4N, writes wN; decode reads wN, writes 4N).

The same line carries a ``topk`` object: the Top-K codec (k = 1 % per tensor, error
feedback, weighting fused) on the same arena, algorithmic bytes 16N + 24k per step
(§8d), with its own roofline and CPU baseline.  ``--codec topk`` makes Top-K the line.

  python bench.py [--gpus N --steps K --warmup W --config llama400m --bits 4]
  N > 1: either the driver's torchrun (RANK/WORLD_SIZE set) or ``python bench.py --gpus N``,
  which spawns the N rank processes itself (before anything touches a GPU).
Each rank is one synthetic client (weak scaling).  For N > 1 the PS weighted sum over
RCCL (Σ decode(Q(w_i x_i)) / Σ w_i) and the Top-K sparse aggregate are timed after the
codec steps and reported beside the metric.
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

METRIC = "GB/s device-resident QSGD encode+decode, Llama-400M grads, 1/2/4/8 GPUs"
METRIC_TOPK = "GB/s device-resident Top-K k=1% encode+decode (error feedback), Llama-400M grads, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
HERE = os.path.dirname(os.path.abspath(__file__))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="llama400m")
    ap.add_argument("--bits", type=int, default=4)
    ap.add_argument("--ratio", type=float, default=0.01)
    ap.add_argument("--codec", choices=("qsgd", "topk"), default="qsgd")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-topk", action="store_true", help="skip the Top-K object of the QSGD line")
    ap.add_argument("--no-extras", action="store_true", help="skip PCIe-inclusive and PS timings")
    ap.add_argument("--dist", action="store_true",
                    help="N = 1 in a one-rank RCCL group: also runs the PS weighted-sum / Top-K aggregate leg "
                         "(the N > 1 code path; no scaling is implied)")
    return ap.parse_args()


# ---------------------------------------------------------------- launch

def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int) -> int:
    """``--gpus N`` without a launcher: start N rank processes of this script (one per GPU)
    and return the first non-zero exit code.  Nothing here touches a GPU."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    codes = [p.wait() for p in procs]
    return next((c for c in codes if c != 0), 0)


def init_dist(torch, dist, force: bool = False):
    """The rank's process group (RCCL).  ``force`` at world size 1: a one-rank group with a loopback
    rendezvous, so the N > 1 aggregate leg runs on one GPU (``--dist``)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        if force:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            torch.cuda.set_device(0)
            dist.init_process_group(backend="nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        return 0, 1, 0
    # the rank's GPU first: RCCL binds its communicator (and barrier) to the current device
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    torch.cuda.set_device(local)
    dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    return dist.get_rank(), dist.get_world_size(), local


# ---------------------------------------------------------------- CPU baseline

def progress(msg: str) -> None:
    """One line on stderr per leg (long runs stay visibly alive; stdout carries only the JSON line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def affinity_cores() -> int:
    """CPUs in this process's affinity mask (on the GPU box: every CPU of the machine)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - non-Linux
        return os.cpu_count() or 1


def cgroup_cpu_quota(path: str = "/sys/fs/cgroup/cpu.max"):
    """The cgroup v2 CPU quota in whole CPUs (``cpu.max``: quota period), None when unlimited or absent."""
    try:
        with open(path) as f:
            quota, period = f.read().split()[:2]
    except (OSError, ValueError):
        return None
    if quota == "max":
        return None
    return max(1, int(int(quota) // int(period)))


def visible_cores() -> int:
    """CPUs this process can actually use: its affinity mask, capped by its cgroup CPU quota (the GPU
    box's affinity mask shows the whole machine while the job's share is 16 CPUs; torch at 256 threads
    on a 16-CPU quota only thrashes)."""
    q = cgroup_cpu_quota()
    return min(affinity_cores(), q) if q else affinity_cores()


def stratified_sample(named, budget):
    """Every k-th tensor of the arena (a representative mix of shapes) up to ``budget`` elements."""
    sizes = [int(np.prod(s)) for _, s in named]
    stride = max(1, int(np.ceil(sum(sizes) / budget)))
    picked = [i for i in range(0, len(sizes), stride)]
    while sum(sizes[i] for i in picked) > budget and len(picked) > 1:
        picked.pop(int(np.argmax([sizes[i] for i in picked])))
    return picked, sizes


def _median_time(fn, reps=5):
    fn()  # warm-up
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def thread_sweep(torch, fn):
    """Median time of ``fn`` at 1 thread, torch's default (the box sets OMP_NUM_THREADS) and every
    core this process may run on."""
    default = torch.get_num_threads()
    times = {}
    for th in sorted({1, default, visible_cores()}):
        torch.set_num_threads(th)
        times[th] = _median_time(fn)
        progress(f"cpu baseline at {th} threads: {times[th]:.3f} s per sample")
    torch.set_num_threads(default)
    return times


def cpu_baseline(torch, named, bits, budget=40_000_000):
    """The reference's op sequence (oracle, kind 'port') on a stratified sample of the arena, at 1 thread,
    torch's default thread count and every visible core, median of 5 after 1 warm-up; the fastest is the
    value (``cores`` = its thread count); extrapolated per element to the whole arena."""
    import oracle

    picked, sizes = stratified_sample(named, budget)
    torch.manual_seed(0)
    sample = [torch.randn(sizes[i]) * 1e-3 for i in picked]
    tot = sum(x.numel() for x in sample)
    w = 1 if 2**bits <= 127 else 4

    def one():
        payloads = []
        for x in sample:  # encode: reference op sequence + tobytes (global_grpc_compression.py:105-116)
            q, norm, wd, lv = oracle.qsgd_quantize(x, bits)
            payloads.append((q.numpy().astype(np.int8 if wd == 8 else np.int32).tobytes(), norm, wd, lv, x.numel()))
        for b, norm, wd, lv, n in payloads:  # decode: frombuffer + decompress_quantized (:173-182)
            q = torch.from_numpy(np.frombuffer(b, dtype=np.int8 if wd == 8 else np.int32).copy())
            oracle.qsgd_dequantize(q, norm, lv, (n,))

    times = thread_sweep(torch, one)
    N = sum(sizes)
    per = (8 + 2 * w)
    best = min(times, key=lambda k: times[k])
    return {
        "value": round(per * tot / times[best] / 1e9, 4),
        "unit": "GB/s",
        "cores": best,
        "visible_cores": visible_cores(),
        "affinity_cores": affinity_cores(),
        "kind": "port",
        "cpu": cpu_model(),
        "sample": f"{len(picked)} of {len(sizes)} tensors (every {max(1, int(np.ceil(N / budget)))}th; {tot} of {N} "
                  f"fp32 elements) of the same arena, QSGD s={bits} encode+decode incl. tobytes/frombuffer, median of 5 "
                  f"after 1 warm-up, per-element rate extrapolated to the arena",
        "GBs_by_threads": {str(k): round(per * tot / v / 1e9, 4) for k, v in times.items()},
        "seconds_full_arena_by_threads": {str(k): round(v * N / tot, 2) for k, v in times.items()},
    }


def cpu_baseline_topk(torch, named, ratio, budget=12_000_000):
    """The reference Top-K with error feedback (oracle TopKOracle: compensate -> topk -> residual) plus its
    zero-fill decode, on a stratified sample, at the thread counts of thread_sweep, median of 5."""
    import oracle

    picked, sizes = stratified_sample(named, budget)
    torch.manual_seed(0)
    sample = [torch.randn(sizes[i]) * 1e-3 for i in picked]
    tot = sum(x.numel() for x in sample)
    ks = [oracle.topk_k(x.numel(), ratio) for x in sample]
    comp = oracle.TopKOracle(ratio)

    def one():
        for j, x in enumerate(sample):
            (vals, idx), _ = comp.compress(x, f"t{j}")
            oracle.topk_desparse(vals, idx, x.numel())

    times = thread_sweep(torch, one)
    alg = 16 * tot + 24 * sum(ks)
    best = min(times, key=lambda k: times[k])
    return {"value": round(alg / times[best] / 1e9, 4), "unit": "GB/s", "cores": best, "visible_cores": visible_cores(),
            "affinity_cores": affinity_cores(), "kind": "port",
            "cpu": cpu_model(),
            "sample": f"{len(picked)} of {len(sizes)} tensors ({tot} fp32 elements), Top-K k={ratio:g} with error "
                      f"feedback + zero-fill decode, median of 5 after 1 warm-up",
            "GBs_by_threads": {str(k): round(alg / v / 1e9, 4) for k, v in times.items()}}


# ---------------------------------------------------------------- measurement helpers

def pmc_traffic(kernel, config, bits):
    """Per-launch HBM bytes of ``kernel`` from profiles/pmc_traffic.json, if it was measured on these
    exact kernel sources (its source digest); otherwise None."""
    from omnifed_amd.build import source_digest

    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None, "no PMC file"
    run = tj.get("runs", {}).get(f"{config}/s{bits}")
    if run is None:
        return None, f"PMC file has no {config}/s{bits} run"
    if tj.get("source_sha") != source_digest():
        return None, f"PMC file measured on other kernel sources (commit {tj.get('commit')}, {tj.get('date')})"
    return run.get("bytes_per_launch", {}).get(kernel), f"rocprofv3 PMC, commit {tj.get('commit')}, {tj.get('date')}"


SETTLE_S = 0.2  # untimed steps before the first leg's W warm-up steps (see settle)


def settle(torch, step, seconds=SETTLE_S):
    """Run untimed ``step`` calls for ``seconds`` of wall time, then synchronise.  The box's GPU idles
    before the run, and from idle it takes ~10-20 ms of load to reach its steady clocks: measured
    (scripts/exp/step_gap.py), the first 20 QSGD steps after 2 s idle take 0.676-0.680 ms each and
    the next 20 0.631-0.633, while 100 ms of any GPU work first makes the first 20 take 0.639.  The
    W warm-up steps (3.4 ms at the driver's W = 5) do not cover that ramp; this does.  Nothing of it
    is timed or reused: the K timed steps still run every launch of every step."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < seconds:
        step(10_000_000 + i)
        i += 1
        if i % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return i


def event_ms(torch, st, fn, reps):
    """Mean duration of ``fn`` (its launches on stream ``st``) in a back-to-back loop, from two
    HIP events recorded on ``st`` around ``reps`` calls (the steady-state launch duration of
    calls queued back to back)."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(0)  # one untimed call: the loop starts in steady state
    a.record(st)
    for i in range(reps):
        fn(i)
    b.record(st)
    torch.cuda.synchronize()
    return float(a.elapsed_time(b)) / reps


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    # stdout carries the one JSON line only: native libraries print banners to fd 1 (RCCL's version
    # block at process-group init), so fd 1 becomes stderr and the line goes to a duplicate of it
    sys.stdout.flush()
    line_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    rank, world, local = init_dist(torch, dist, args.dist)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from omnifed_amd import codec, shapes
    from omnifed_amd.build import build

    if rank == 0:
        build()
    if world > 1:
        dist.barrier()

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(v):
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed(step, k0, steps):
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(k0 + i)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        return max_over_ranks(time.perf_counter() - t0)

    named = shapes.model_shapes(args.config)
    sizes = [shapes.numel(s) for _, s in named]
    N = sum(sizes)
    plan = codec.Plan.get(sizes, device=dev, chunk=args.chunk)
    weight = float(1 + rank)  # this client's batch_samples (the weighting fused as alpha)
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    x = torch.randn(plan.arena_end, device=dev, generator=g) * 1e-3
    st = torch.cuda.current_stream(dev)

    # ------------------------------------------------------------ QSGD
    s = args.bits
    L = 2**s
    w = 1 if L <= 127 else 4
    width = 8 * w
    q = torch.empty(plan.payload_elems(width), dtype=torch.int8 if w == 1 else torch.int32, device=dev)
    norms = torch.empty(plan.nt, dtype=torch.float32, device=dev)
    y = torch.empty(plan.arena_end, dtype=torch.float32, device=dev)
    seed = 0x5EED + rank

    def q_step(i):
        plan.qsgd_encode(x, s, q_out=q, norm_out=norms, alpha=weight, seed=seed, offset=i)
        plan.qsgd_decode(q, width, L, norms, y_out=y)

    qsgd = None
    settled = 0
    if args.codec == "qsgd":
        progress("qsgd steps")
        settled = settle(torch, q_step)
        for i in range(args.warmup):
            q_step(i)
        plan.check()
        dt = timed(q_step, args.warmup, args.steps)
        plan.check()
        alg_bytes_step = (8 + 2 * w) * N
        reps = max(args.steps, 10)
        enc_ms = event_ms(torch, st, lambda i: plan.qsgd_encode(x, s, q_out=q, norm_out=norms, alpha=weight, seed=seed,
                                                                offset=10_000 + i), reps)
        enc_kernel = plan.last_encoder_kernel  # what the encode launched (the plan's record)
        dec_ms = event_ms(torch, st, lambda i: plan.qsgd_decode(q, width, L, norms, y_out=y), reps)
        plan.check()
        enc_bytes = dec_bytes = (4 + w) * N
        dom_ms, dom_bytes, dom_name = (enc_ms, enc_bytes, enc_kernel) if enc_ms >= dec_ms else \
            (dec_ms, dec_bytes, "qsgd_decode_flat")
        achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
        traffic, tsrc = pmc_traffic(dom_name, args.config, s)
        if dom_name == "qsgd_spec_all":  # the whole bracketed encode call, timed as one unit
            dom_name = ("omf_qsgd_encode = qsgd_spec_bracket + qsgd_spec_quant + qsgd_spec_finish"
                        " (at widths <= 4 the bracket runs as qsgd_spec_quant_fb's first workgroups)")
        qsgd = {
            "value": world * alg_bytes_step * args.steps / dt / 1e9, "ms_per_step": dt / args.steps * 1e3,
            "alg_bytes_step": alg_bytes_step,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
                         "kernel": dom_name, "algorithmic_bytes_per_launch": dom_bytes,
                         "avg_launch_ms": round(dom_ms, 4), "encode_ms": round(enc_ms, 4),
                         "decode_ms": round(dec_ms, 4), "encode_GBs": round(enc_bytes / enc_ms / 1e6, 1),
                         "decode_GBs": round(dec_bytes / dec_ms / 1e6, 1)},
        }

    # ------------------------------------------------------------ Top-K
    topk = None
    if args.codec == "topk" or not args.no_topk:
        progress("topk steps")
        ratio = args.ratio
        ks = plan.topk_ks(ratio)
        K = sum(ks)
        # a fresh gradient every step, as in training (4 resident arenas in rotation): error
        # feedback on one repeated gradient makes every never-selected residual grow in lockstep
        # (r = c x after c steps), a degenerate magnitude distribution no client produces
        xs = [x] + [torch.randn(plan.arena_end, device=dev, generator=g) * 1e-3 for _ in range(3)]
        res = torch.zeros(plan.arena_end, dtype=torch.float32, device=dev)
        vals = torch.empty(K, dtype=torch.float32, device=dev)
        idx = torch.empty(K, dtype=torch.int64, device=dev)
        yt = torch.empty(plan.arena_end, dtype=torch.float32, device=dev)

        def t_enc(i):
            plan.topk_encode(xs[i % len(xs)], ratio, residual=res, residual_mode=1, values=vals, indices=idx,
                             alpha=weight)

        def t_step(i):
            t_enc(i)
            plan.topk_decode_arena(vals, idx, ratio, y=yt, mode=0)

        if args.codec == "topk":
            settled = settle(torch, t_step)
        for i in range(args.warmup):
            t_step(i)
        plan.topk_stats(reset=True)
        steps_t = args.steps if args.codec == "topk" else max(5, args.steps // 2)
        dtt = timed(t_step, args.warmup, steps_t)
        alg_t = 16 * N + 24 * K
        reps = max(steps_t, 5)
        tenc = event_ms(torch, st, t_enc, reps)
        tdec = event_ms(torch, st, lambda i: plan.topk_decode_arena(vals, idx, ratio, y=yt, mode=0), reps)
        enc_alg = 12 * N + 12 * K  # read x, read+write the residual, write values+indices
        ach = enc_alg / (tenc * 1e-3) / 1e9
        t_traffic, t_tsrc = pmc_traffic("topk_encode_all", args.config, s)  # every launch of one encode call
        topk = {"metric": METRIC_TOPK, "value": round(world * alg_t * steps_t / dtt / 1e9, 2), "unit": "GB/s",
                "ms_per_step": round(dtt / steps_t * 1e3, 4), "steps": steps_t, "ratio": ratio, "k_total": K,
                "algorithmic_bytes_per_step_per_client": alg_t,
                "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": t_traffic, "traffic_source": t_tsrc,
                             "kernel": "omf_topk_encode (all launches of one call; stream-asynchronous, no host wait)",
                             "algorithmic_bytes_per_launch": enc_alg, "avg_launch_ms": round(tenc, 4),
                             "decode_ms": round(tdec, 4)},
                "encoder_paths": plan.topk_stats(),  # timed calls: bucket-sort fast path vs fallbacks
                "tie_order": "index"}
        if not args.no_extras:
            # the drop-in's default order (the reference's bytes where magnitudes tie): the device encode,
            # then omf_topk_torch_order's census and host rewrite of the tied tensors; wall clock
            progress("topk torch order")
            tw, nre = [], []
            for i in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                plan.topk_encode(xs[i % len(xs)], ratio, residual=res, residual_mode=1, values=vals, indices=idx,
                                 alpha=weight, tie_order="torch")
                torch.cuda.synchronize()
                tw.append((time.perf_counter() - t0) * 1e3)
                nre.append(plan.topk_reordered)
            topk["torch_order"] = {"ms_per_encode": round(sorted(tw)[1], 2), "tensors_rewritten": nre,
                                   "tensors": plan.nt, "host_threads": min(16, os.cpu_count() or 1)}
        del res, yt, xs

    extras = {}
    if not args.no_extras and world == 1 and qsgd is not None and args.config == "llama400m":
        # the other QSGD configs of BASELINE.json on one GPU: ResNet-18 at "8 levels" (s = 3, int8)
        # and the base default s = 8 (int32 wire), Llama-150M at the presets' s = 4
        progress("other configs")
        others = {}
        for cname, bits in (("resnet18", 3), ("resnet18", 8), ("llama150m", 4)):
            sz = [shapes.numel(sh) for _, sh in shapes.model_shapes(cname)]
            pl = codec.Plan.get(sz, device=dev)
            n_ = sum(sz)
            w_ = 1 if 2**bits <= 127 else 4
            xo = torch.randn(pl.arena_end, device=dev, generator=g) * 1e-3
            qo = torch.empty(pl.payload_elems(8 * w_), dtype=torch.int8 if w_ == 1 else torch.int32, device=dev)
            no = torch.empty(pl.nt, dtype=torch.float32, device=dev)
            yo = torch.empty(pl.arena_end, dtype=torch.float32, device=dev)

            def o_step(i, pl=pl, xo=xo, qo=qo, no=no, yo=yo, bits=bits, w_=w_):
                pl.qsgd_encode(xo, bits, q_out=qo, norm_out=no, alpha=weight, seed=seed, offset=i)
                pl.qsgd_decode(qo, 8 * w_, 2**bits, no, y_out=yo)

            for i in range(3):
                o_step(i)
            reps = 20
            to = timed(o_step, 3, reps) / reps
            pl.check()
            others[f"{cname}_s{bits}"] = {"elements": n_, "tensors": len(sz), "ms_per_step": round(to * 1e3, 4),
                                           "algorithmic_GBs": round((8 + 2 * w_) * n_ / to / 1e9, 1)}
            del xo, qo, no, yo
        extras["other_configs"] = others
    if not args.no_extras and world == 1 and qsgd is not None:
        progress("pcie-inclusive rate")
        # PCIe-inclusive rate: host fp32 in -> device encode -> host payload; host payload -> decode -> host fp32
        xh = torch.empty(plan.arena_end, dtype=torch.float32, pin_memory=True)
        xh.copy_(x, non_blocking=False)
        qh = torch.empty(q.numel(), dtype=q.dtype, pin_memory=True)
        yh = torch.empty(plan.arena_end, dtype=torch.float32, pin_memory=True)
        xd = torch.empty_like(x)

        def pcie_step(i):
            xd.copy_(xh, non_blocking=True)
            plan.qsgd_encode(xd, s, q_out=q, norm_out=norms, alpha=weight, seed=seed, offset=20_000 + i)
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
        # Pipelined: the uplink (x in, encode, payload out) and the downlink (payload in, decode,
        # fp32 out) on two streams, step i's downlink beside step i+1's uplink, so each PCIe
        # direction carries 4 N + w N bytes per step at once (PCIe is full duplex).  Double-buffered
        # device payloads and norms; the downlink of step i waits for its payload's arrival on the host.
        s_up, s_dn = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        q2 = [torch.empty_like(q) for _ in range(2)]
        n2 = [torch.empty_like(norms) for _ in range(2)]
        nh = torch.empty(norms.numel(), dtype=norms.dtype, pin_memory=True)
        qd = torch.empty_like(q)
        nd = torch.empty_like(norms)
        ev_q = [torch.cuda.Event() for _ in range(2)]
        ev_free = [torch.cuda.Event() for _ in range(2)]

        def pipe_step(i):
            b = i & 1
            with torch.cuda.stream(s_up):
                s_up.wait_event(ev_free[b])  # the host payload buffer's previous reader is done
                xd.copy_(xh, non_blocking=True)
                plan.qsgd_encode(xd, s, q_out=q2[b], norm_out=n2[b], alpha=weight, seed=seed, offset=20_000 + i)
                qh.copy_(q2[b], non_blocking=True)
                nh.copy_(n2[b], non_blocking=True)
                ev_q[b].record(s_up)
            with torch.cuda.stream(s_dn):
                s_dn.wait_event(ev_q[b])
                qd.copy_(qh, non_blocking=True)
                nd.copy_(nh, non_blocking=True)
                ev_free[b].record(s_dn)
                plan.qsgd_decode(qd, width, L, nd, y_out=y)
                yh.copy_(y, non_blocking=True)

        for b in range(2):
            ev_free[b].record(torch.cuda.current_stream(dev))
        pipe_step(0)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(1, 9):
            pipe_step(i)
        torch.cuda.synchronize()
        pp = (time.perf_counter() - t1) / 8
        extras["pcie_inclusive"] = {"ms_per_step": round(pt * 1e3, 3),
                                    "algorithmic_GBs": round((8 + 2 * w) * N / pt / 1e9, 2),
                                    "fp32_gradient_GBs": round(4 * N / pt / 1e9, 2),
                                    "serial": "H2D x, encode, D2H payload, H2D payload, decode, D2H y on one stream",
                                    "pipelined_ms_per_step": round(pp * 1e3, 3),
                                    "pipelined_algorithmic_GBs": round((8 + 2 * w) * N / pp / 1e9, 2),
                                    "pipelined": "uplink and downlink on two streams, step i's downlink beside step "
                                                 "i+1's uplink (PCIe full duplex); steady state over 8 steps"}
        del xh, qh, yh, xd, q2, n2, qd, nd
    if not args.no_extras and dist.is_initialized():
        progress("PS aggregates over the process group")
        from omnifed_amd.ps import GpuOps, qsgd_weighted_round, topk_sparse_aggregate, total_weight

        ops = GpuOps(plan, seed=seed)
        total = total_weight(weight, dev)
        acc = torch.empty_like(y)
        bufs = [(torch.empty_like(q), torch.empty_like(norms)) for _ in range(world)] if rank == 0 else None
        ps = {"clients": world, "total_weight": total, "fp32_bytes_per_rank": 4 * N, "payload_bytes_per_rank": w * N}
        for mode in ("gather", "reduce"):
            def ps_step(i, mode=mode):
                qsgd_weighted_round(x, weight, total, ops, s, 30_000 + i, mode=mode, y=y, acc=acc, q=q, norms=norms,
                                    bufs=bufs)
            ps_step(0)
            ps[f"{mode}_ms"] = round(timed(ps_step, 1, 5) / 5 * 1e3, 3)
        extras["ps_weighted_sum"] = ps
        if topk is not None:
            K = topk["k_total"]
            vals = torch.empty(K, dtype=torch.float32, device=dev)
            idx = torch.empty(K, dtype=torch.int64, device=dev)
            plan.topk_encode(x, args.ratio, values=vals, indices=idx, alpha=weight)
            tb = [(torch.empty_like(vals), torch.empty_like(idx)) for _ in range(world)]
            agg = {}
            for name, dst in (("allgather", None), ("gather_root", 0)):
                def tk_step(i, dst=dst):
                    topk_sparse_aggregate(vals, idx, args.ratio, acc, ops, dst=dst, bufs=tb)
                tk_step(0)
                agg[f"{name}_ms"] = round(timed(tk_step, 1, 5) / 5 * 1e3, 3)
            agg["bytes_per_rank"] = 12 * K
            extras["topk_sparse_aggregate"] = agg

    cpu = cpu_t = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if qsgd is not None:
            cpu = cpu_baseline(torch, named, s)
        if topk is not None:
            cpu_t = cpu_baseline_topk(torch, named, args.ratio)
    if topk is not None:
        topk["cpu_baseline"] = cpu_t

    if rank == 0:
        common = {"n_gpus": world, "warmup": args.warmup,
                  "settle": {"seconds": SETTLE_S, "untimed_steps": settled,
                             "why": "GPU clock ramp from idle (bench.settle); before the W warm-up steps"},
                  "higher_is_better": True, "scaling": "weak",
                  "vs_baseline": None, "dtype": "f32",
                  "data": "synthetic N(0,1)*1e-3 gradients of the named shapes (no checkpoints)"}
        if qsgd is not None:
            line = {"metric": METRIC, "value": round(qsgd["value"], 2), "unit": "GB/s", "steps": args.steps,
                    "ms_per_step": round(qsgd["ms_per_step"], 4), **common,
                    "config": {"workload": f"{args.config} QSGD encode+decode, bit_width {s} ({L} levels, int{8 * w} "
                                           f"wire), philox draws, client weighting fused (alpha = batch_samples = "
                                           f"rank + 1), one client per GPU",
                               "tensors": len(sizes), "elements_per_client": N, "bit_width": s,
                               "algorithmic_bytes_per_step_per_client": qsgd["alg_bytes_step"],
                               "fp32_gradient_GBs": round(qsgd["value"] * 4 / (8 + 2 * w), 2),
                               "parallelism": f"clients{world}"},
                    "roofline": qsgd["roofline"], "cpu_baseline": cpu, "topk": topk, **extras}
        else:
            line = {"metric": METRIC_TOPK, "value": topk["value"], "unit": "GB/s", "steps": topk["steps"],
                    "ms_per_step": topk["ms_per_step"], **common,
                    "config": {"workload": f"{args.config} Top-K k={args.ratio:g} per tensor, error feedback, "
                                           f"client weighting fused, arena decode, one client per GPU",
                               "tensors": len(sizes), "elements_per_client": N, "k_total": topk["k_total"],
                               "algorithmic_bytes_per_step_per_client": topk["algorithmic_bytes_per_step_per_client"],
                               "parallelism": f"clients{world}"},
                    "roofline": topk["roofline"], "cpu_baseline": cpu_t, **extras}
        print(json.dumps(line), file=line_out, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
