# k_rb2 quick check (one box): the bitwise k_rb2 tests, then the RB-SOR
# iteration time with the product form at 512^3 and 1024^2 x 512.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
TAG=${TAG:-r04_rb2_quick}
timeout -k 10 400 python -u -m pytest tests/test_gpu_rb2.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for g in "512 512 512" "1024 1024 512"; do
  set -- $g
  CFD_HIP_RB2=1 NX=$1 NY=$2 NZ=$3 ITERS=200 METHODS=rbsor timeout -k 10 120 python tools/relax_bench.py >> gpurun_out/${TAG}.jsonl 2>>gpurun_out/${TAG}.err || exit 1
done
cat gpurun_out/${TAG}.jsonl
