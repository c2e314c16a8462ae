#!/bin/bash
# One driver for the GPU-box runs (gpurun -- bash scripts/gpu.sh <task> [args]).  Every GPU step
# runs under its own time limit and the first failure ends the script (no retries).
#   tests [pytest -k expr]  the -m gpu suite (or a subset), one process
#   wire [tag]              host-inclusive wire timings -> gpurun_out/<tag>_wire.json
#   bench [tag] [args...]   bench.py line -> gpurun_out/<tag>_bench.json
#   prof [tag] [args...]    rocprofv3 --kernel-trace --stats of bench.py (args: e.g. --codec topk)
#   pmc [tag] [args...]     FETCH_SIZE / WRITE_SIZE passes of bench.py + pmc_traffic.json
#                           (PMC_CFG / PMC_BITS name the config when args change it)
#   sq [tag]                SQ counter passes of the ResNet-18 encoders -> gpurun_out/<tag>_sq.json
#   py <script> [args...]   any experiment script (its stdout -> gpurun_out/py.out)
#   measure [tag]           the round's profile set: rocprofv3 kernel stats of the QSGD and the Top-K
#                           bench lines, the two PMC passes at s = 4 (QSGD + Top-K) and at s = 8 (the int32
#                           wire) (-> profiles/pmc_traffic.json, stamped with the source digest; OMF_COMMIT
#                           names the commit), the bench lines at s = 4 and s = 8 (they read the fresh PMC
#                           file), the wire timings; copied into profiles/<tag>_*
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
task=${1:-tests}
shift || true
case "$task" in
  tests)
    K=()
    [ -n "$1" ] && K=(-k "$1")
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${K[@]}" \
      > gpurun_out/tests.log 2>&1
    rc=$?
    tail -n 40 gpurun_out/tests.log
    exit $rc
    ;;
  wire)
    T=${1:-r04}
    timeout -k 10 600 python3 -u scripts/wire_bench.py llama400m gpurun_out/${T}_wire.json \
      > gpurun_out/${T}_wire.out 2> gpurun_out/${T}_wire.err || { tail -20 gpurun_out/${T}_wire.err; exit 2; }
    cat gpurun_out/${T}_wire.json
    ;;
  bench)
    T=${1:-r04}
    shift || true
    timeout -k 10 600 python3 -u bench.py "$@" > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
      || { tail -20 gpurun_out/${T}_bench.err; exit 2; }
    cat gpurun_out/${T}_bench.json
    ;;
  prof)
    T=${1:-r04}
    shift || true
    rm -rf gpurun_out/${T}_prof
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${T}_prof" -o run \
      -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-extras "$@" \
      > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 2; }
    s=$(find gpurun_out/${T}_prof -name '*kernel_stats.csv' | head -n 1)
    [ -n "$s" ] && cp "$s" gpurun_out/${T}_kernel_stats.csv && cat gpurun_out/${T}_kernel_stats.csv
    ;;
  pmc)
    T=${1:-r04}_s${PMC_BITS:-4}
    shift || true
    for c in FETCH_SIZE WRITE_SIZE; do
      rm -rf gpurun_out/${T}_pmc_$c
      timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/${T}_pmc_$c" -o run \
        -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-extras "$@" \
        > gpurun_out/${T}_pmc_$c.log 2>&1 || { tail -20 gpurun_out/${T}_pmc_$c.log; exit 2; }
    done
    python3 scripts/pmc_traffic.py gpurun_out/${T}_pmc_FETCH_SIZE gpurun_out/${T}_pmc_WRITE_SIZE \
      gpurun_out/${T}_pmc_traffic.json ${PMC_CFG:-llama400m} ${PMC_BITS:-4} || exit 3
    cat gpurun_out/${T}_pmc_traffic.json
    ;;
  sq)
    # SQ counter passes (VALU work, wave-cycle split, LDS stalls), one pass per group: by default
    # over the ResNet-18 encoder A/B (scripts/exp/r18_ab.py: ring, grid, two-launch encoders and
    # the decoder); SQ_PROG=topk over the Llama-400M Top-K encode + decode (bench.py --codec topk)
    T=${1:-r04_r18}
    if [ "${SQ_PROG:-r18}" = topk ]; then
      PROG=("$R/bench.py" --codec topk --steps 5 --warmup 2 --no-cpu-baseline --no-extras); CFG=llama400m
    else
      PROG=("$R/scripts/exp/r18_ab.py" 3 1); CFG=resnet18
    fi
    i=0
    for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
               "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INSTS_SMEM" \
               "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ATOMIC_RETURN SQ_LDS_UNALIGNED_STALL"; do
      i=$((i+1))
      rm -rf gpurun_out/${T}_sq$i
      echo "sq pass $i: $grp"
      timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/gpurun_out/${T}_sq$i" -o run \
        -- python3 "${PROG[@]}" > gpurun_out/${T}_sq$i.log 2>&1 || { tail -20 gpurun_out/${T}_sq$i.log; exit 2; }
    done
    E=$(python3 -c "from omnifed_amd import shapes; print(sum(shapes.numel(s) for _, s in shapes.model_shapes('$CFG')))")
    python3 scripts/sq_summary.py gpurun_out/${T}_sq.json "$E" gpurun_out/${T}_sq1 gpurun_out/${T}_sq2 gpurun_out/${T}_sq3 || exit 3
    ;;
  py)
    S=$1
    shift || true
    timeout -k 10 900 python3 -u "$S" "$@" > gpurun_out/py.out 2> gpurun_out/py.err || { tail -30 gpurun_out/py.err; exit 2; }
    tail -c 20000 gpurun_out/py.out
    ;;
  measure)
    T=${1:-r04}
    bash scripts/gpu.sh prof ${T} > /dev/null || exit 2
    bash scripts/gpu.sh prof ${T}_topk --codec topk > /dev/null || exit 3
    bash scripts/gpu.sh prof ${T}_s8 --bits 8 --no-topk > /dev/null || exit 3
    rm -f gpurun_out/${T}_s4_pmc_traffic.json gpurun_out/${T}_s8_pmc_traffic.json
    bash scripts/gpu.sh pmc ${T} || exit 4
    cp gpurun_out/${T}_s4_pmc_traffic.json gpurun_out/${T}_s8_pmc_traffic.json
    PMC_BITS=8 bash scripts/gpu.sh pmc ${T} --bits 8 --no-topk || exit 4
    cp gpurun_out/${T}_s8_pmc_traffic.json profiles/pmc_traffic.json
    bash scripts/gpu.sh bench ${T} || exit 5
    bash scripts/gpu.sh bench ${T}_s8 --bits 8 --no-topk --no-cpu-baseline || exit 5
    cp gpurun_out/${T}_s8_bench.json profiles/${T}_s8_bench.json
    bash scripts/gpu.sh wire ${T} > /dev/null || exit 6
    cp gpurun_out/${T}_kernel_stats.csv profiles/${T}_kernel_stats.csv
    cp gpurun_out/${T}_topk_kernel_stats.csv profiles/${T}_topk_kernel_stats.csv
    cp gpurun_out/${T}_s8_kernel_stats.csv profiles/${T}_s8_kernel_stats.csv
    cp gpurun_out/${T}_bench.json profiles/${T}_bench.json
    cp gpurun_out/${T}_wire.json profiles/${T}_wire.json
    mkdir -p gpurun_out/profiles_copy && cp profiles/pmc_traffic.json profiles/${T}_* gpurun_out/profiles_copy/
    echo "measure ok"
    ;;
  *)
    echo "unknown task $task"; exit 64 ;;
esac
