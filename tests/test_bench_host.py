"""bench.py's host helpers (CPU): the CPU-baseline thread count is the process's affinity mask
capped by its cgroup v2 quota (the GPU box lists 256 CPUs in the mask but grants 16), and the
stratified sample picks every k-th tensor within its budget; the untimed settle before the warm-up."""
import os
import time

import bench


def _cpu_max(tmp_path, text):
    p = tmp_path / "cpu.max"
    p.write_text(text)
    return str(p)


def test_cgroup_cpu_quota_parses_cpu_max(tmp_path):
    assert bench.cgroup_cpu_quota(_cpu_max(tmp_path, "1600000 100000\n")) == 16
    assert bench.cgroup_cpu_quota(_cpu_max(tmp_path, "150000 100000\n")) == 1  # whole CPUs, rounded down
    assert bench.cgroup_cpu_quota(_cpu_max(tmp_path, "50000 100000\n")) == 1   # never below one
    assert bench.cgroup_cpu_quota(_cpu_max(tmp_path, "max 100000\n")) is None  # unlimited
    assert bench.cgroup_cpu_quota(_cpu_max(tmp_path, "garbage\n")) is None
    assert bench.cgroup_cpu_quota(str(tmp_path / "absent")) is None


def test_visible_cores_is_capped_by_the_quota(monkeypatch):
    monkeypatch.setattr(bench, "affinity_cores", lambda: 256)
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: 16)
    assert bench.visible_cores() == 16
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: None)
    assert bench.visible_cores() == 256
    monkeypatch.setattr(bench, "affinity_cores", lambda: 8)
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: 16)
    assert bench.visible_cores() == 8


def test_affinity_cores_matches_the_process_mask():
    assert bench.affinity_cores() == len(os.sched_getaffinity(0))


def test_stratified_sample_stays_within_budget():
    named = [(f"t{i}", (100 * (i + 1),)) for i in range(20)]
    picked, sizes = bench.stratified_sample(named, 1000)
    assert sizes == [100 * (i + 1) for i in range(20)]
    assert picked and sum(sizes[i] for i in picked) <= 1000
    assert picked == sorted(picked) and picked[0] == 0  # every k-th tensor from the first, largest dropped
    one, _ = bench.stratified_sample([("big", (10, 1000))], 10)
    assert one == [0]  # a single tensor is kept even over the budget


def test_settle_runs_untimed_steps_for_its_wall_time():
    """bench.settle: untimed steps for the given wall time (the GPU's clock ramp), synchronising
    every 16 steps and at the end; the steps get offsets far from the timed loop's."""
    calls, syncs = [], []

    class _Cuda:
        @staticmethod
        def synchronize():
            syncs.append(len(calls))

    class _Torch:
        cuda = _Cuda

    def step(i):
        calls.append(i)
        time.sleep(0.001)

    n = bench.settle(_Torch, step, seconds=0.05)
    assert n == len(calls) >= 10
    assert min(calls) >= 10_000_000
    assert syncs[0] == 0 and syncs[-1] == n  # before the first step and after the last
