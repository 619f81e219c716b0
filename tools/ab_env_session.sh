#!/bin/bash
# A/B of an environment switch on one box: parity (TESTS) with the switch on,
# then tools/step_kernels_bench.py with it off / on, interleaved (2 rounds).
# usage: TAG=x ENVSW=CFD_HIP_PRED_LDS TESTS="tests/a.py" tools/ab_env_session.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-abe}
TESTS=${TESTS:-"tests/test_gpu_parity.py tests/test_gpu_energy.py"}
env $ENVSW=1 timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -1 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for on in 0 1; do
    env $ENVSW=$on timeout -k 10 240 python tools/step_kernels_bench.py | sed "s/^{/{\"$ENVSW\": $on, /" >> gpurun_out/${TAG}.jsonl || exit $?
  done
done
cat gpurun_out/${TAG}.jsonl
