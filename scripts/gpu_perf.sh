#!/usr/bin/env bash
# Perf session: chunk sweep + rocprofv3 kernel stats of a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/sweep_chunk.py llama400m ${SWEEP_CHUNKS:-16384,65536,131072,262144} > gpurun_out/sweep.log 2>&1; rc=$?
echo "sweep rc=$rc"; cat gpurun_out/sweep.log | tail -8
[ $rc -eq 0 ] || exit $rc
if [ -n "${PROF:-}" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1; rc=$?
  echo "prof rc=$rc"; tail -2 gpurun_out/prof.log
fi
exit $rc
