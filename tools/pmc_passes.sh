#!/bin/bash
# SQ issue/wait counters and HBM bytes (FETCH_SIZE, WRITE_SIZE) of every
# kernel a command runs, one counter group per rocprofv3 pass, each pass
# under its own time limit; per-kernel summary via tools/pmc_kernels.py.
# usage: TAG=x CMD="python3 tools/step_kernels_bench.py" tools/pmc_passes.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for pass in ${PASSES:-sq fetch write}; do
  case $pass in
    sq) C="$SQ" ;;
    fetch) C="FETCH_SIZE" ;;
    write) C="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" ;;
  esac
  timeout -s KILL ${PASS_TIMEOUT:-150} rocprofv3 --pmc $C -d $OUT/$pass -o run --output-format csv -- $CMD \
      > $OUT/$pass.log 2>&1
  rc=$?; echo "pass $pass exit $rc"; [ $rc -ne 0 ] && exit $rc
  python3 tools/pmc_kernels.py $OUT/$pass --note "pass $pass" >> $OUT/summary.jsonl
done
exit 0
