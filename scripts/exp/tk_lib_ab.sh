# Interleaved Top-K A/B of the default build against a variant library (bench.py --codec topk lines).
# bash scripts/exp/tk_lib_ab.sh <variant.so>
set -o pipefail
cd $GRAFT_REPO_ROOT
V=$1
one() {  # tag lib
  OMF_CODEC_LIB_EXPERIMENT=$2 timeout -k 10 120 python3 bench.py --codec topk --no-cpu-baseline --no-extras > gpurun_out/tkab_$1.json 2>/dev/null || exit 3
  python3 -c "import json;d=json.load(open('gpurun_out/tkab_$1.json'));r=d['roofline'];print('$1', d['ms_per_step'], r['avg_launch_ms'], r.get('decode_ms'))"
}
for r in 1 2 3; do
  one default_$r ""
  one variant_$r "$V"
done
