#!/bin/bash
# Round-end evidence on one box: the whole GPU suite, smoke(), the rocprofv3
# kernel trace + FETCH/WRITE passes of the 512^3 bench (traffic.json keyed on
# the current kernel sources), then the bench at the driver's settings with
# that profile committed in-tree for roofline.traffic / measured_GBps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02b}
# PART=tests: the suite and smoke() only; PART=bench: the profile and the bench
# only (one gpurun call is capped at 20 minutes)
if [ "${PART:-all}" != "bench" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -2 gpurun_out/${TAG}_smoke.log; [ $rc -ne 0 ] && exit $rc
[ "${PART:-all}" = "tests" ] && exit 0
fi
[ -n "$NO_PROF" ] || { TAG=$TAG ARGS="--size 512 --steps 1 --warmup 1 --no-cpu-baseline --no-compare-cg-variant --no-plugin-step" bash tools/gpu_profile.sh || exit $?; \
  cp gpurun_out/prof_${TAG}/traffic.json profiles/${TAG}_traffic.json; }
# the bench at the driver's settings under a rocprofv3 kernel trace (no CPU
# baseline: its child processes stay out of the profiler), so the committed
# kernel statistics and that line come from one run on one box
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_benchtrace -o run \
    --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-plugin-step \
    > gpurun_out/${TAG}_bench_traced.json 2> gpurun_out/${TAG}_bench_traced.err
rc=$?; echo "traced bench exit $rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/${TAG}_benchtrace -name 'run_kernel_stats.csv' | head -n 1)
[ -n "$f" ] && cp "$f" gpurun_out/${TAG}_bench_kernel_stats.csv
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench exit $rc"; tail -c 1500 gpurun_out/${TAG}_bench.json; exit $rc
