#!/bin/bash
# Sweep the CG-sweep tiling knobs at 512^3 (one process per configuration).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-t1}
for rows in ${ROWS:-4 8}; do
  for kc in ${KCS:-32 64 128}; do
    timeout -k 10 300 python bench.py --size ${N:-512} --steps ${STEPS:-1} --warmup 1 --no-cpu-baseline \
        --sweep-rows $rows --kchunk $kc > gpurun_out/sweep_${TAG}_r${rows}_k${kc}.log 2>&1
    rc=$?
    echo "rows=$rows kc=$kc rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_${TAG}_r${rows}_k${kc}.log').read().strip().splitlines()[-1]); print(d['value'], d['cg_iter_ms'], d['kernels']['cg_sweep_a']['avg_ms'], d['kernels']['cg_sweep_b']['avg_ms'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
