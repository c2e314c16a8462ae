set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh prof tk512 --codec topk > /dev/null || exit 2
OMF_CODEC_LIB_EXPERIMENT=gpu_exp_libs/tk1024.so bash scripts/gpu.sh prof tk1024 --codec topk > /dev/null || exit 3
