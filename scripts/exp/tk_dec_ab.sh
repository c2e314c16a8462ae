#!/bin/bash
# Experiment (GPU box): the tiled Top-K decode's shape, interleaved variants of one build each:
# sub-tile size (s13 / s14 = the default 16 Ki, 64 KiB LDS tile / s15), tile threads (t256 / t1024),
# staged entries (k4), and a bit per element in place of the zeroed tile (m1 / m15).  Variants
# named in CHECK also run the Top-K GPU tests on their build first.
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
    m1) build m1 -DOMF_DEC_SUB_BITS=14 -DOMF_DEC_MASK=1 ;;
    m15) build m15 -DOMF_DEC_SUB_BITS=15 -DOMF_DEC_MASK=1 ;;
  esac
done
echo built
for v in ${CHECK:-}; do
  OMF_CODEC_LIB_EXPERIMENT=/tmp/omf_dec_$v/lib.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 \
      --timeout-method thread -m gpu tests/test_gpu_topk_wire.py tests/test_gpu_topk_ps.py tests/test_gpu_topk_half.py \
      > gpurun_out/tkd_check_$v.log 2>&1 || { tail -30 gpurun_out/tkd_check_$v.log; exit 4; }
  tail -1 gpurun_out/tkd_check_$v.log
done
for rep in 1 2; do
for v in $VARS; do
  o=gpurun_out/tkd_${v}_$rep; rm -rf $o
  OMF_CODEC_LIB_EXPERIMENT=/tmp/omf_dec_$v/lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o run -- \
      python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 20 > $o.log 2>&1 || exit 3
done
done
