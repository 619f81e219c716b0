#!/bin/bash
# rocprofv3 kernel-trace + stats of a 512^3 bench, then separate PMC passes
# for FETCH_SIZE and WRITE_SIZE on the CG sweeps (MI355X_MICROARCH.md §HBM).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-p1}
N=${N:-512}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --n $N --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace exit $rc"; [ $rc -ne 0 ] && exit $rc
if [ -n "${NO_PMC}" ]; then exit 0; fi
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_cg[AB]" -d $OUT/fetch -o run --output-format csv -- \
    python3 bench.py --n $N --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_fetch.log 2>&1
rc=$?; echo "fetch exit $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_cg[AB]" -d $OUT/write -o run --output-format csv -- \
    python3 bench.py --n $N --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_write.log 2>&1
rc=$?; echo "write exit $rc"; exit $rc
