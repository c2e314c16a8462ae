set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for st in ordered ring resident ordered ring; do
  timeout -k 10 200 python3 scripts/exp/enc_time.py llama400m 8 $st >> gpurun_out/s8_ab.txt 2>> gpurun_out/s8_ab.err || exit 2
done
cat gpurun_out/s8_ab.txt
