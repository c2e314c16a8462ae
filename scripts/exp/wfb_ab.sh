set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in default wfb32 wfb8; do
    L=""; [ $v != default ] && L=gpu_exp_libs/$v.so
    OMF_CODEC_LIB_EXPERIMENT=$L timeout -k 10 120 python3 bench.py --bits 8 --no-topk --no-cpu-baseline --no-extras > gpurun_out/wfb_${v}_$r.json 2>/dev/null || exit 3
    python3 -c "import json;d=json.load(open('gpurun_out/wfb_${v}_$r.json'));r=d['roofline'];print('$v', d['ms_per_step'], r['encode_ms'], r['decode_ms'])"
  done
done
