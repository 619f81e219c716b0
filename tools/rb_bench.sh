#!/bin/bash
# One-pass RB-SOR kernel: bitwise parity, then the per-iteration time at 512^3
# and 1024x1024x512 (BASELINE configs[4]'s grid).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-rb}
timeout -k 10 300 python -u -m pytest tests/test_gpu_rb_variants.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; [ $rc -ne 0 ] && exit $rc
METHODS=rbsor,jacobi ITERS=60 timeout -k 10 240 python tools/relax_bench.py >> gpurun_out/${TAG}_512.jsonl || exit $?
METHODS=rbsor ITERS=30 NX=1024 NY=1024 NZ=512 timeout -k 10 300 python tools/relax_bench.py >> gpurun_out/${TAG}_1024.jsonl || exit $?
cat gpurun_out/${TAG}_512.jsonl gpurun_out/${TAG}_1024.jsonl
