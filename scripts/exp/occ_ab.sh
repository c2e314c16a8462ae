# Occupancy caps by dynamic LDS (experiment knobs OMF_SPEC_LDS, OMF_SPEC_LDS_W, OMF_DEC_LDS,
# OMF_TOPK_LDS): bench.py lines per setting, two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
one() {  # tag env-assignment bench-args...
  local tag=$1 envs=$2; shift 2
  env $envs timeout -k 10 120 python3 bench.py --no-topk --no-cpu-baseline --no-extras "$@" > gpurun_out/occ_$tag.json 2>/dev/null || exit 3
  python3 -c "import json;d=json.load(open('gpurun_out/occ_$tag.json'));r=d['roofline'];print('$tag $envs', d['ms_per_step'], r['encode_ms'], r['decode_ms'])"
}
for r in 1 2; do
  for l in 10240 12288 16384 20480; do one w${l}_$r OMF_SPEC_LDS_W=$l --bits 8; done
  for l in 0 24576 28672; do one d${l}_$r OMF_DEC_LDS=$l; one d8${l}_$r OMF_DEC_LDS=$l --bits 8; done
done
