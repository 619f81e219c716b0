# RB-SOR quick check (one box): the bitwise relaxation tests (TESTS), then
# the RB-SOR iteration time at 512^3 and 1024^2 x 512 for each CFD_HIP_RB2
# mode in MODES (1: k_rb2, the product; 0: k_rb1 one iteration per sweep).
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
TAG=${TAG:-r04_rb2_quick}
TESTS=${TESTS:-tests/test_gpu_rb2.py}
MODES=${MODES:-1}
timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for m in $MODES; do
  for g in "512 512 512" "1024 1024 512"; do
    set -- $g
    CFD_HIP_RB2=$m NX=$1 NY=$2 NZ=$3 ITERS=200 METHODS=rbsor timeout -k 10 120 python tools/relax_bench.py >> gpurun_out/${TAG}.jsonl 2>>gpurun_out/${TAG}.err || exit 1
  done
done
cat gpurun_out/${TAG}.jsonl
