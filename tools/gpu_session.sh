#!/bin/bash
# One GPU session: parity tests, smoke, bench. Stops at the first crash /
# timeout (exit codes other than 0 and pytest's 1 = "tests failed").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-s1}
BENCH_ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1"}
timeout -k 10 ${PYTEST_TIMEOUT:-400} python -m pytest tests -x -q -m gpu ${PYTEST_ARGS} > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; echo "pytest exit $rc" | tee -a gpurun_out/pytest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
rc=$?; echo "smoke exit $rc" | tee -a gpurun_out/smoke_${TAG}.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "${NO_BENCH}" ]; then exit 0; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.log 2>&1
rc=$?; echo "bench exit $rc" | tee -a gpurun_out/bench_${TAG}.log
exit $rc
