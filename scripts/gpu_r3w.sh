#!/bin/bash
# Round-3: ordering events without a system-scope fence — gaps in the traces, the two-stream
# ordering tests, the QSGD bench line with its ResNet-18 / Llama-150M configs.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3w_l400 gpurun_out/r3w_r18
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3w_l400 -o run -- python3 scripts/exp/gap_probe.py 0 > gpurun_out/r3w_l400.log 2>&1 || exit 1
echo "== l400"; python3 scripts/exp/trace_gaps.py gpurun_out/r3w_l400 120
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3w_r18 -o run -- python3 scripts/exp/r18_trace.py - ed > gpurun_out/r3w_r18.log 2>&1 || exit 1
echo "== r18"; python3 scripts/exp/trace_gaps.py gpurun_out/r3w_r18 400
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "stream or order" > gpurun_out/r3w_tests.log 2>&1 || { tail -20 gpurun_out/r3w_tests.log; exit 2; }
tail -1 gpurun_out/r3w_tests.log
timeout -k 10 300 python3 bench.py --no-topk --no-cpu-baseline --steps 50 > gpurun_out/r3w_bench.json 2> gpurun_out/r3w_bench.err || exit 4
python3 -c "import json; d=json.load(open('gpurun_out/r3w_bench.json')); print(d['ms_per_step'], d['roofline']['encode_ms'], d['roofline']['decode_ms'], d['roofline']['frac'], d['other_configs'])"
