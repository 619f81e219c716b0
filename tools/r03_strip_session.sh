#!/bin/bash
# r03: k_rb1 remainder strip A/B: bitwise tests, per-iteration kernel time at
# 512^3 and 1024^2 x 512 (interleaved), and the configs[4] line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_strip
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rb_variants.py \
    tests/test_gpu_parity.py tests/test_gpu_energy.py tests/test_gpu_poisson_3d.py \
    > $O/pytest_rb.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_rb.log; exit 1; }
tail -2 $O/pytest_rb.log
for round in 1 2; do
  for s in 1 0; do
    CFD_HIP_RB1_STRIP=$s N=512 ITERS=60 METHODS=rbsor timeout -k 10 120 python3 tools/relax_bench.py \
        | sed "s/^{/{\"strip\": $s, \"round\": $round, /" >> $O/relax.jsonl || exit 1
    CFD_HIP_RB1_STRIP=$s NX=1024 NY=1024 NZ=512 ITERS=30 METHODS=rbsor timeout -k 10 120 python3 tools/relax_bench.py \
        | sed "s/^{/{\"strip\": $s, \"round\": $round, /" >> $O/relax.jsonl || exit 1
  done
done
cat $O/relax.jsonl
timeout -k 10 200 python3 bench.py --case convection --steps 1 --warmup 0 > $O/conv.json 2> $O/conv.err \
    || { echo "conv failed"; tail -5 $O/conv.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/conv.json')); print(d['ms_per_step'], d['rbsor_iters_per_step'], d['rbsor_iter_ms'], d['roofline'])"
