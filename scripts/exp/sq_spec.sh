#!/usr/bin/env bash
# SQ / GRBM counter passes over scripts/exp/spec_only.py (one pass per counter group).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/exp/spec_only.py > gpurun_out/eo.log 2>&1
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/gpurun_out/sq$i" -o run -- \
    python3 "$R/scripts/exp/spec_only.py" > gpurun_out/sq$i.log 2>&1
done
python3 scripts/exp/sq_counters.py gpurun_out/sq1 gpurun_out/sq2
