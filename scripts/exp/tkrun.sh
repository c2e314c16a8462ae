export TMPDIR=/tmp; R=$(pwd); N=$1
timeout -k 10 300 python -u -m pytest tests -q -x --timeout 120 --timeout-method thread -m gpu -k "topk or Topk or TopK" > gpurun_out/tk_tests.log 2>&1; tail -30 gpurun_out/tk_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/tk_prof$N -o run -- python3 $R/scripts/exp/topk_prof.py > gpurun_out/tk_prof$N.log 2>&1 && python3 scripts/rocpd_stats.py $(find gpurun_out/tk_prof$N -name "*.db" | head -1) gpurun_out/tk_stats$N.csv; grep topk gpurun_out/tk_prof$N.log
