#!/bin/bash
# r03c: k_rb1 direction alternation (CFD_HIP_RB1_ALT, default 1) parity under
# both settings and its A/B, then the round evidence on the final sources
# (tools/round_session.sh: whole GPU suite, smoke, rocprofv3 trace + PMC,
# driver-settings bench), then the configs[4] line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03_rbalt
mkdir -p $O
CFD_HIP_RB1_ALT=0 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rb_variants.py tests/test_gpu_energy.py \
    tests/test_gpu_poisson_3d.py -x -q --timeout 200 --timeout-method thread > $O/pytest_0.log 2>&1
rc=$?; echo "pytest alt=0 exit $rc"; tail -2 $O/pytest_0.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2 3; do
  for v in 0 1; do
    CFD_HIP_RB1_ALT=$v METHODS=rbsor ITERS=60 timeout -k 10 200 python3 tools/relax_bench.py | sed "s/^{/{\"alt\": $v, \"round\": $round, /" >> $O/rb.jsonl || exit 1
    CFD_HIP_RB1_ALT=$v METHODS=rbsor ITERS=30 NX=1024 NY=1024 NZ=512 timeout -k 10 200 python3 tools/relax_bench.py | sed "s/^{/{\"alt\": $v, \"round\": $round, /" >> $O/rb.jsonl || exit 1
  done
done
cat $O/rb.jsonl
TAG=r03c bash tools/round_session.sh || exit $?
timeout -k 10 400 python3 bench.py --case convection --steps 1 --warmup 0 \
    > gpurun_out/r03c_convection.json 2> gpurun_out/r03c_convection.err || { echo "convection failed"; tail -5 gpurun_out/r03c_convection.err; exit 1; }
tail -c 600 gpurun_out/r03c_convection.json
