#!/bin/bash
# rocprofv3 kernel-trace + stats of the 1-GPU bench, then separate PMC passes
# for FETCH_SIZE and WRITE_SIZE on its kernels (MI355X_MICROARCH.md "HBM":
# counters in their own passes, no trace domains alongside --pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-p1}
N=${N:-512}
ARGS=${ARGS:-"--size $N --steps 1 --warmup 1 --no-cpu-baseline"}
# interior cells per launch the traffic is divided by (bench.py keys the
# profile on it): (N-2)^3 for the cavity; the convection case passes its own
CELLS=${CELLS:-$(( (N-2)*(N-2)*(N-2) ))}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace exit $rc"; [ $rc -ne 0 ] && exit $rc
if [ -z "${NO_PMC}" ]; then
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
    python3 bench.py $ARGS > $OUT/bench_fetch.log 2>&1
rc=$?; echo "fetch exit $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- \
    python3 bench.py $ARGS > $OUT/bench_write.log 2>&1
rc=$?; echo "write exit $rc"; [ $rc -ne 0 ] && exit $rc
fi
# the trace/PMC output dirs nest by host/pid; flatten the CSVs we summarise
for sub in trace fetch write; do
  f=$(find $OUT/$sub -name 'run_kernel_stats.csv' 2>/dev/null | head -n 1)
  [ -n "$f" ] && cp "$f" $OUT/$sub/run_kernel_stats.csv 2>/dev/null
  f=$(find $OUT/$sub -name 'run_counter_collection.csv' 2>/dev/null | head -n 1)
  [ -n "$f" ] && cp "$f" $OUT/$sub/run_counter_collection.csv 2>/dev/null
done
python3 tools/prof_summary.py $OUT --cells $CELLS --json $OUT/traffic.json > $OUT/summary.txt 2>&1
echo "summary exit $?"
exit 0
