#!/bin/bash
# Predictor / corrector / CG-setup parity (the step tests) and per-kernel times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-pc}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_energy.py tests/test_gpu_slabs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/step_kernels_bench.py > gpurun_out/${TAG}.jsonl 2> gpurun_out/${TAG}.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/${TAG}.jsonl; exit $rc
