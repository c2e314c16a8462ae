#!/bin/bash
# Round-3: tiled Top-K decode with a per-sub-tile bitmap (no 32 KiB LDS clear) — tests and timing.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_topk_ps.py tests/test_gpu_r3.py tests/test_gpu_r2.py \
    -x -q --timeout 200 --timeout-method thread -k "decode or topk" > gpurun_out/r3z_tests.log 2>&1 || { tail -30 gpurun_out/r3z_tests.log; exit 1; }
tail -1 gpurun_out/r3z_tests.log
rm -rf gpurun_out/r3z_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3z_prof -o run -- \
    python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 20 > gpurun_out/r3z_prof.log 2>&1 || exit 5
grep '^{' gpurun_out/r3z_prof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['decode_ms'])"
