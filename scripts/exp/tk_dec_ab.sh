#!/bin/bash
# Experiment (GPU box): the tiled Top-K decode's sub-tile size: 8 Ki elements (the default: 32 KiB
# LDS tile + 2 Ki staged entries, 3 workgroups per CU) against 4 Ki (round 3) and 16 / 32 Ki
# (round 4: 64 / 128 KiB tiles, more stores in flight per barrier phase, 2 / 1 workgroups per CU).
set -o pipefail
cd "$(dirname "$0")/../.." && export TMPDIR=/tmp
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude"
build() {
  local d=/tmp/omf_dec_$1; shift; mkdir -p $d
  for s in omf_runtime.cpp omf_qsgd.hip omf_qsgd_ring.hip omf_qsgd_pack.hip omf_topk.hip; do
    (timeout -k 10 400 hipcc $F "$@" -c omnifed_amd/csrc/$s -o $d/$s.o && echo "$d $s" >> gpurun_out/tkd_progress.txt) &
  done
  wait
  timeout -k 10 200 hipcc --offload-arch=gfx950 -shared -fPIC -o $d/lib.so $d/*.o || exit 1
  echo "built $d" >> gpurun_out/tkd_progress.txt  # a long silent build looks hung to the box
}
VARS="${VARS:-s13 s14 s15}"
for v in $VARS; do
  case $v in
    s13) build s13 -DOMF_DEC_SUB_BITS=13 ;;
    s14) build s14 -DOMF_DEC_SUB_BITS=14 ;;
    s15) build s15 -DOMF_DEC_SUB_BITS=15 ;;
    t1024) build t1024 -DOMF_DEC_SUB_BITS=14 -DOMF_DEC_TILE_THREADS=1024 ;;
    t256) build t256 -DOMF_DEC_SUB_BITS=14 -DOMF_DEC_TILE_THREADS=256 ;;
    k4) build k4 -DOMF_DEC_SUB_BITS=14 -DOMF_DEC_STAGE=4096 ;;
  esac
done
echo built
for rep in 1 2; do
for v in $VARS; do
  o=gpurun_out/tkd_${v}_$rep; rm -rf $o
  OMF_CODEC_LIB_EXPERIMENT=/tmp/omf_dec_$v/lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o run -- \
      python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 20 > $o.log 2>&1 || exit 3
done
done
