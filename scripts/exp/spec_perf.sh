#!/usr/bin/env bash
# Bracketed single-read encoder: interleaved strategy timings on three BASELINE arenas, then a
# rocprofv3 kernel trace of its four launches on Llama-400M (experiment; one gpurun call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in llama400m llama150m resnet18; do
  MODEL=$m timeout -k 10 180 python scripts/exp/ab_strategy.py bracket ordered ring flat >> gpurun_out/spec_perf.log 2>&1 || { echo "ab $m failed"; tail -20 gpurun_out/spec_perf.log; exit 1; }
done
cat gpurun_out/spec_perf.log
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/spec_prof" -o run -- python3 "$R/scripts/exp/ab_strategy.py" bracket > gpurun_out/spec_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/spec_prof.log; exit 1; }
db=$(ls "$R"/gpurun_out/spec_prof/*/*results.db "$R"/gpurun_out/spec_prof/*results.db 2>/dev/null | head -1)
[ -n "$db" ] && python3 scripts/rocpd_stats.py "$db" gpurun_out/spec_kernel_stats.csv
exit 0
