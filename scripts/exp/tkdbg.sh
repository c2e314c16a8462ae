export TMPDIR=/tmp; R=$(pwd)
for d in ${DBGS:-0 1 2 3}; do
OMF_TOPK_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/tk_dbg$d -o run -- python3 $R/scripts/exp/topk_prof.py > gpurun_out/tk_dbg$d.log 2>&1 || exit 1
python3 scripts/rocpd_stats.py $(find gpurun_out/tk_dbg$d -name "*.db" | head -1) gpurun_out/tk_dbg$d.csv > gpurun_out/tk_dbg$d.txt
grep bucket_sort gpurun_out/tk_dbg$d.txt
done
