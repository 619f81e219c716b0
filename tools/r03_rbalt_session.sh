#!/bin/bash
# r03 A/B: k_rb1 / k_rb1m with odd iterations marching z downwards
# (CFD_HIP_RB1_ALT=1) against all-upward; bitwise relaxation suites under both
# first, then fixed-iteration RB-SOR at 512^3 and 1024^2 x 512, three rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03_rbalt
mkdir -p $O
for v in 1 0; do
  CFD_HIP_RB1_ALT=$v timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_energy.py tests/test_gpu_poisson_3d.py \
      tests/test_gpu_rb_variants.py tests/test_gpu_slabs.py tests/test_gpu_dirty_faces.py -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; echo "pytest alt=$v exit $rc"; tail -2 $O/pytest_$v.log; [ $rc -ne 0 ] && exit $rc
done
for round in 1 2 3; do
  for v in 0 1; do
    CFD_HIP_RB1_ALT=$v METHODS=rbsor ITERS=60 timeout -k 10 200 python3 tools/relax_bench.py | sed "s/^{/{\"alt\": $v, \"round\": $round, /" >> $O/rb.jsonl || exit 1
    CFD_HIP_RB1_ALT=$v METHODS=rbsor ITERS=30 NX=1024 NY=1024 NZ=512 timeout -k 10 200 python3 tools/relax_bench.py | sed "s/^{/{\"alt\": $v, \"round\": $round, /" >> $O/rb.jsonl || exit 1
  done
done
cat $O/rb.jsonl
