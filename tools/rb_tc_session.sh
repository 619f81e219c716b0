#!/bin/bash
# k_rb1 tile widths (CFD_HIP_RB1_TC = 64 / 32 / 16): bitwise parity of every
# width, then the per-iteration time of each at 512^3 and 1024x1024x512.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-rbtc}
timeout -k 10 400 python -u -m pytest tests/test_gpu_rb_variants.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
for tc in 64 32 16; do
  CFD_HIP_RB1_TC=$tc METHODS=rbsor ITERS=60 timeout -k 10 240 python tools/relax_bench.py | sed "s/^{/{\"tc\": $tc, /" >> gpurun_out/${TAG}_512.jsonl || exit $?
done
for tc in 64 32 16; do
  CFD_HIP_RB1_TC=$tc METHODS=rbsor ITERS=30 NX=1024 NY=1024 NZ=512 timeout -k 10 300 python tools/relax_bench.py | sed "s/^{/{\"tc\": $tc, /" >> gpurun_out/${TAG}_1024.jsonl || exit $?
done
cat gpurun_out/${TAG}_512.jsonl gpurun_out/${TAG}_1024.jsonl
