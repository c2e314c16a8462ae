#!/bin/bash
# Round-3: Top-K with the 1.5-sigma sure margin — every Top-K GPU test, then the Top-K line.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_topk_ps.py tests/test_gpu_r3.py tests/test_gpu_r2.py tests/test_gpu_integration.py \
    -x -q --timeout 200 --timeout-method thread -k "topk or Topk or TopK or sure" > gpurun_out/r3s_tests.log 2>&1 || { tail -30 gpurun_out/r3s_tests.log; exit 1; }
tail -1 gpurun_out/r3s_tests.log
timeout -k 10 300 python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 30 > gpurun_out/r3s_bench.json 2> gpurun_out/r3s_bench.err || exit 4
python3 -c "import json; d=json.load(open('gpurun_out/r3s_bench.json')); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['decode_ms'], d['roofline']['frac'])"
rm -rf gpurun_out/r3s_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s_prof -o run -- \
    python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 20 > gpurun_out/r3s_prof.log 2>&1 || exit 5
