# Interleaved A/B of the default build against a variant library: bench.py lines (QSGD only).
# bash scripts/exp/lib_ab.sh <variant.so> [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
V=$1; shift
one() {  # tag lib
  OMF_CODEC_LIB_EXPERIMENT=$2 timeout -k 10 120 python3 bench.py --no-topk --no-cpu-baseline --no-extras "${@:3}" > gpurun_out/ab_$1.json 2>/dev/null || exit 3
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$1.json'));r=d['roofline'];print('$1', d['ms_per_step'], r['encode_ms'], r['decode_ms'])"
}
for r in 1 2 3; do
  one default_$r "" "$@"
  one variant_$r "$V" "$@"
done
