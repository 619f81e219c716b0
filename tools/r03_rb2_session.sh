#!/bin/bash
# r03: two RB-SOR iterations per sweep (k_rb2) -- bitwise tests, then per-
# iteration kernel time against the one-iteration sweep, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_rb2
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rb_variants.py \
    tests/test_gpu_parity.py tests/test_gpu_energy.py tests/test_gpu_poisson_3d.py tests/test_gpu_config_parity.py \
    > $O/pytest_rb.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAILED|Error" $O/pytest_rb.log | head -30; exit 1; }
tail -2 $O/pytest_rb.log
for round in 1 2; do
  for s in 1 0; do
    CFD_HIP_RB2=$s N=512 ITERS=60 METHODS=rbsor timeout -k 10 120 python3 tools/relax_bench.py \
        | sed "s/^{/{\"rb2\": $s, \"round\": $round, /" >> $O/relax.jsonl || exit 1
    CFD_HIP_RB2=$s NX=1024 NY=1024 NZ=512 ITERS=30 METHODS=rbsor timeout -k 10 120 python3 tools/relax_bench.py \
        | sed "s/^{/{\"rb2\": $s, \"round\": $round, /" >> $O/relax.jsonl || exit 1
  done
done
cut -c1-160 $O/relax.jsonl
