set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for r in 1 2 3; do
  OMF_CODEC_LIB_EXPERIMENT=$PWD/scripts/exp/ab_old.so timeout -k 10 200 python3 scripts/exp/enc_time.py llama400m 4 >> gpurun_out/ab_fmt.txt 2>>gpurun_out/ab_fmt.err || exit 2
  timeout -k 10 200 python3 scripts/exp/enc_time.py llama400m 4 >> gpurun_out/ab_fmt.txt 2>>gpurun_out/ab_fmt.err || exit 2
done
cat gpurun_out/ab_fmt.txt
