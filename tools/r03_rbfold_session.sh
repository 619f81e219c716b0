#!/bin/bash
# Round-3: the GPU suite, then configs[4] at full size on one GPU with the
# Neumann shell folded into k_rb1 (default) and with the separate k_rx_shell.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_fold
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
for f in 1 0; do
  CFD_HIP_RB1_FOLD=$f timeout -k 10 200 python3 bench.py --case convection --size 1024 --steps 1 --warmup 0 \
      > $O/conv_fold$f.json 2> $O/conv_fold$f.err || { echo "conv fold=$f failed"; tail -5 $O/conv_fold$f.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/conv_fold$f.json')); print('fold=$f', d['ms_per_step'], d['rbsor_iters_per_step'], d['rbsor_iter_ms'], d['roofline']['avg_sweep_ms'])"
done
