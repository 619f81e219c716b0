#!/bin/bash
# CG sweep variant A/B on one box: bitwise tests of the sweep variants, then
# the 512^3 cavity bench with each variant (VARIANTS, interleaved, ROUNDS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-swv}
VARIANTS=${VARIANTS:-"15 47"}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "sweep" -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -1 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-compare-cg-variant --sweep-variant $v > gpurun_out/${TAG}_b.json || exit $?
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/${TAG}_b.json').read().strip().splitlines()[-1])
print(json.dumps({'variant': $v, 'value': d['value'], 'cg_iter_ms': d['cg_iter_ms'], 'iters': d['cg_iters_per_step'], 'sweeps': {k: v['avg_ms'] for k, v in d['cg_sweeps'].items()}, 'frac': d['roofline']['frac']}))" >> gpurun_out/${TAG}.jsonl || exit $?
  done
done
cat gpurun_out/${TAG}.jsonl
