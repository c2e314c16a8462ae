#!/bin/bash
# Round-3 measurement: Top-K + wire tests, a Top-K bench line, a rocprofv3 kernel-trace of it, the wire path.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_r2.py tests/test_gpu_topk_ps.py \
    tests/test_gpu_wire.py tests/test_gpu_packed_wire.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r3_topk_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --codec topk --no-cpu-baseline --no-extras --steps 20 > gpurun_out/r3_topk_bench.json \
    2> gpurun_out/r3_topk_bench.err || exit 2
rm -rf gpurun_out/r3_topk_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_topk_prof -o run -- \
    python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 10 > gpurun_out/r3_topk_prof.log 2>&1 || exit 3
timeout -k 10 300 python -u scripts/wire_bench.py > gpurun_out/r3_wire.json 2> gpurun_out/r3_wire.err || exit 4
