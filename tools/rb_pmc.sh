#!/bin/bash
# SQ issue/wait counters and HBM bytes of the one-pass RB-SOR kernel
# at 512^3 (tools/relax_bench.py, 20 iterations). One counter group per
# rocprofv3 pass, each pass under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-rbpmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for v in ${VARIANTS:-default}; do
  for pass in sq fetch write; do
    case $pass in
      sq) C="$SQ" ;;
      fetch) C="FETCH_SIZE" ;;
      write) C="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" ;;
    esac
    METHODS=rbsor ITERS=20 timeout -s KILL 120 rocprofv3 --pmc $C \
        -d $OUT/v${v}_$pass -o run --output-format csv -- python3 tools/relax_bench.py \
        > $OUT/v${v}_$pass.log 2>&1
    rc=$?; echo "variant $v pass $pass exit $rc"; [ $rc -ne 0 ] && exit $rc
    python3 tools/pmc_kernels.py $OUT/v${v}_$pass --note "variant $v pass $pass" >> $OUT/summary.jsonl
  done
done
exit 0
