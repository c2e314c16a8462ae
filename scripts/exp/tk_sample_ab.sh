# Top-K sampler A/B: the default build against a variant library (tk_old.so: OMF_SAMPLE_HIST_LATE=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
one() {  # tag lib
  OMF_CODEC_LIB_EXPERIMENT=$2 timeout -k 10 120 python3 bench.py --codec topk --no-cpu-baseline --no-extras > gpurun_out/tks_$1.json 2>/dev/null || exit 3
  python3 -c "import json;d=json.load(open('gpurun_out/tks_$1.json'));r=d['roofline'];print('$1', d['ms_per_step'], r['avg_launch_ms'], r.get('decode_ms'), d.get('encoder_paths'))"
}
for r in 1 2 3; do
  one new_$r ""
  one old_$r gpu_exp_libs/tk_old.so
done
OMF_CODEC_LIB_EXPERIMENT=gpu_exp_libs/tk_ts.so timeout -k 10 120 python3 bench.py --codec topk --steps 3 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/ts2.out 2> gpurun_out/ts2.err || exit 4
grep SAMPLE_TS gpurun_out/ts2.out | tail -7
