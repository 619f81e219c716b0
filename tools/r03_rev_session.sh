#!/bin/bash
# r03 A/B: CG sweep B marching z downwards (CFD_HIP_CGB_REV=1; sweep A marches
# upwards, so each sweep starts where the last one ended, in the Infinity Cache);
# 25-step trajectory) with H2 first, then the 512^3 bench kernels interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03_rev
mkdir -p $O
CFD_HIP_CGB_REV=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config_parity.py \
    tests/test_gpu_cg_small.py tests/test_gpu_slabs.py tests/test_gpu_cavity512.py tests/test_gpu_cg_single_reduction.py \
    -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2 3; do
  for v in 0 1; do
    CFD_HIP_CGB_REV=$v timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-compare-cg-variant > $O/bench_${v}_$round.json 2> $O/bench_${v}_$round.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/bench_${v}_$round.json')); print(json.dumps({'rev':$v,'round':$round,'value':d['value'],'cg_iter_ms':d['cg_iter_ms'],'sweeps':{k:v['avg_ms'] for k,v in d['kernels'].items()}}))" >> $O/ab.jsonl
  done
done
cat $O/ab.jsonl
