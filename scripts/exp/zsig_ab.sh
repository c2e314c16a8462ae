# Bracket width (OMF_SPEC_ZSIG sigmas) A/B at s = 4 and s = 8: bench.py lines, two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
one() {  # tag zsig bench-args...
  local tag=$1 z=$2; shift 2
  OMF_SPEC_ZSIG=$z timeout -k 10 120 python3 bench.py --no-topk --no-cpu-baseline --no-extras "$@" > gpurun_out/zs_$tag.json 2>/dev/null || exit 3
  python3 -c "import json;d=json.load(open('gpurun_out/zs_$tag.json'));r=d['roofline'];print('$tag z=$z', d['ms_per_step'], r['encode_ms'], r['decode_ms'])"
}
for r in 1 2; do
  for z in 6 5 4; do one s4_${z}_$r $z; done
  for z in 5 4 3.5; do one s8_${z}_$r $z --bits 8; done
done
