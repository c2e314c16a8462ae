# Top-K streaming-pass sub-chunk size A/B: default build (512) against variant libraries.
set -o pipefail
cd $GRAFT_REPO_ROOT
one() {  # tag lib
  OMF_CODEC_LIB_EXPERIMENT=$2 timeout -k 10 120 python3 bench.py --codec topk --no-cpu-baseline --no-extras > gpurun_out/tksub_$1.json 2>/dev/null || exit 3
  python3 -c "import json;d=json.load(open('gpurun_out/tksub_$1.json'));r=d['roofline'];print('$1', d['ms_per_step'], r['avg_launch_ms'], r.get('decode_ms'))"
}
for r in 1 2; do
  one s512_$r ""
  one s1024_$r gpu_exp_libs/tk1024.so
  one s256_$r gpu_exp_libs/tk256.so
done
