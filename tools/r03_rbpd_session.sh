#!/bin/bash
# r03 A/B: k_rb1 / k_rb1m with one more plane of loads in flight
# (CFD_HIP_RB1_PD=1: six-slot X ring, three-slot rhs ring) against the
# default; bitwise relaxation tests first, then fixed-iteration RB-SOR at
# 512^3 and 1024^2 x 512, two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03_rbpd
mkdir -p $O
CFD_HIP_RB1_PD=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_energy.py tests/test_gpu_poisson_3d.py \
    -x -q -k "relax or rb or redblack or energy or poisson" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for v in 0 1; do
    CFD_HIP_RB1_PD=$v METHODS=rbsor ITERS=60 timeout -k 10 200 python3 tools/relax_bench.py | sed "s/^{/{\"pd\": $v, \"round\": $round, /" >> $O/rb.jsonl || exit 1
    CFD_HIP_RB1_PD=$v METHODS=rbsor ITERS=30 NX=1024 NY=1024 NZ=512 timeout -k 10 200 python3 tools/relax_bench.py | sed "s/^{/{\"pd\": $v, \"round\": $round, /" >> $O/rb.jsonl || exit 1
  done
done
cat $O/rb.jsonl
