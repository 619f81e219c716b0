#!/bin/bash
# GPU check of bench.py's live CG-form probe: the multi-rank rehearsal tests,
# then a 2-rank 512^3 line on the one device (ranks share it; timings are
# not the node's, the path is)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread \
  tests/test_gpu_bench.py -k rehearsal > gpurun_out/${TAG}_pytest_rehearsal.log 2>&1 || exit $?
CFD_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node=2 --rdzv-backend=c10d --rdzv-endpoint=127.0.0.1:0 --local-addr=127.0.0.1 \
  bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/${TAG}_bench_n2_512.json \
  2> gpurun_out/${TAG}_bench_n2_512.err
