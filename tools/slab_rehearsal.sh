#!/bin/bash
# Shared-GPU rehearsal of the Z-slab CG forms at 512^3 (run with
# CFD_BENCH_SHARED_GPU=1 on a one-GPU box: every rank on device 0, RCCL
# between ranks of one device, dot products through the device mailbox):
# bench.py at N ranks for textbook CG (cg_variant 0) and the single-reduction
# CG (1; fused slab form, and CFD_HIP_CCF_SLAB_FUSED=0 the r04 form). The
# ranks share one GPU, so the numbers compare the forms' total device work
# and synchronisation, not an 8-GPU node's xGMI. usage: TAG=r05h NS="2 4 8" TESTS=1 CFD_BENCH_SHARED_GPU=1 tools/slab_rehearsal.sh
set -o pipefail
O=gpurun_out/${TAG:-r05g}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
      tests/test_gpu_cg_single_reduction.py tests/test_gpu_rccl.py > $O/pytest.log 2>&1 || exit 1
fi
port=29611
for n in ${NS:-2}; do
  for form in cg0 cg1 cg1_unfused; do
    v=${form:2:1}; fz=1; [ "$form" = cg1_unfused ] && fz=0
    port=$((port + 1))
    CFD_HIP_CCF_SLAB_FUSED=$fz timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n \
        --steps 2 --warmup 1 --cg-variant $v --no-cpu-baseline --fixed-cg-iters 0 \
        --no-compare-cg-variant > $O/n${n}_$form.json 2> $O/n${n}_$form.err || exit 1
  done
done
