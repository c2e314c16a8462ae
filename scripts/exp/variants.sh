#!/usr/bin/env bash
# Time the encode phases with prebuilt experiment variants (scripts/exp/_build/*/lib.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for v in base r7 norng nodiv nornd_nodiv; do
  echo "== $v"
  OMF_CODEC_LIB_EXPERIMENT=scripts/exp/_build/$v/lib.so timeout -k 10 200 python scripts/exp/probe.py 2>&1 | grep -v amdgpu.ids | grep -E "encode|quant|norms|decode |Error|error"
done
