#!/bin/bash
# r03 A/B: k_rb1 / k_rb1m memory hints (CFD_HIP_RB1_FL: 15 = NT stores + NT
# rhs loads (default), 13 = no NT loads, 12 = no NT hints, 14 = NT loads only),
# fixed-iteration RB-SOR at 512^3 (k_rb1m) and 1024^2 x 512 (k_rb1), two
# interleaved rounds, then one FETCH_SIZE pass per variant at 512^3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03_rbfl
mkdir -p $O
for round in 1 2; do
  for v in 15 13 12 14; do
    CFD_HIP_RB1_FL=$v METHODS=rbsor ITERS=60 timeout -k 10 200 python3 tools/relax_bench.py | sed "s/^{/{\"fl\": $v, \"round\": $round, /" >> $O/rb.jsonl || exit 1
    CFD_HIP_RB1_FL=$v METHODS=rbsor ITERS=30 NX=1024 NY=1024 NZ=512 timeout -k 10 200 python3 tools/relax_bench.py | sed "s/^{/{\"fl\": $v, \"round\": $round, /" >> $O/rb.jsonl || exit 1
  done
done
cat $O/rb.jsonl
for v in 15 13 12; do
  CFD_HIP_RB1_FL=$v METHODS=rbsor ITERS=10 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${v} -o p --output-format csv -- python3 tools/relax_bench.py > /dev/null 2>&1 || exit $?
done
echo done
