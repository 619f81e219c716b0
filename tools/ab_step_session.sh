#!/bin/bash
# Predictor / corrector A/B over library builds on one box: parity of each
# build (step + energy tests), then tools/step_kernels_bench.py per build,
# interleaved over two rounds. LIBS = space-separated names under
# cfd_amd/lib_ab/ (libcfd_hip_<name>.so); "cur" = the in-tree build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-abs}
LIBS=${LIBS:-cur}
sel() { if [ "$1" = cur ]; then unset CFD_AMD_HIP_LIB; else export CFD_AMD_HIP_LIB=$PWD/cfd_amd/lib_ab/libcfd_hip_$1.so; fi; }
for b in $LIBS; do
  sel $b
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_energy.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_$b.log 2>&1
  rc=$?; echo "pytest $b exit $rc"; tail -1 gpurun_out/${TAG}_pytest_$b.log; [ $rc -ne 0 ] && exit $rc
done
for round in 1 2; do
  for b in $LIBS; do
    sel $b
    timeout -k 10 240 python tools/step_kernels_bench.py | sed "s/^{/{\"build\": \"$b\", /" >> gpurun_out/${TAG}.jsonl || exit $?
  done
done
cat gpurun_out/${TAG}.jsonl
