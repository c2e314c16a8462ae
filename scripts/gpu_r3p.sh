#!/bin/bash
# Round-3: bracketed encoder's fix phase with one thread per wave slot — QSGD tests, bench, kernel trace.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_qsgd.py tests/test_gpu_r3.py tests/test_gpu_wire.py \
    tests/test_gpu_r2.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3p_tests.log 2>&1 || { tail -30 gpurun_out/r3p_tests.log; exit 1; }
tail -1 gpurun_out/r3p_tests.log
rm -rf gpurun_out/r3p_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3p_prof -o run -- \
    python3 bench.py --no-topk --no-cpu-baseline --no-extras --steps 20 > gpurun_out/r3p_prof.log 2>&1 || exit 3
timeout -k 10 300 python3 bench.py --no-topk --no-cpu-baseline --no-extras --steps 50 > gpurun_out/r3p_bench.json 2> gpurun_out/r3p_bench.err || exit 4
python3 -c "import json; d=json.load(open('gpurun_out/r3p_bench.json')); print(d['ms_per_step'], d['roofline']['encode_ms'], d['roofline']['decode_ms'], d['roofline']['frac'])"
