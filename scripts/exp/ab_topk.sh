#!/bin/bash
# Interleaved A/B of the Top-K bench line: A = scripts/exp/ab_old.so (OMF_CODEC_LIB_EXPERIMENT),
# B = the in-tree library; two rounds each, one bench.py process per run.
set -o pipefail
cd "$(dirname "$0")/../.." && export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export OMF_CODEC_LIB_EXPERIMENT=$PWD/scripts/exp/ab_old.so; else unset OMF_CODEC_LIB_EXPERIMENT; fi
    timeout -k 10 300 python3 bench.py --codec topk --steps 20 --no-extras --no-cpu-baseline > gpurun_out/ab_$v$r.json 2> gpurun_out/ab_$v$r.err || { tail -5 gpurun_out/ab_$v$r.err; exit 2; }
    python3 -c "import json,sys; b=json.loads(open('gpurun_out/ab_$v$r.json').read().strip().splitlines()[-1]); t=b.get('topk', b); print('$v$r', b['ms_per_step'], t['roofline']['avg_launch_ms'], t['roofline']['decode_ms'])"
  done
done
