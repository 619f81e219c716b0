# k_rb2 A/B (one box): RB-SOR iteration time of k_rb1 (CFD_HIP_RB2=0), the
# certified two-iteration sweep (1) and its reference-arithmetic form (2) at
# 512^3 and 1024^2 x 512, then the configs[4] bench step with the default.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
for m in 0 1 2; do
  for g in "512 512 512" "1024 1024 512"; do
    set -- $g
    CFD_HIP_RB2_LOG=1 CFD_HIP_RB2=$m NX=$1 NY=$2 NZ=$3 ITERS=200 METHODS=rbsor timeout -k 10 120 python tools/relax_bench.py >> gpurun_out/r04_rb2_perf.jsonl 2>>gpurun_out/r04_rb2_perf.err || exit 1
    echo "rb2=$m $g done"
  done
done
[ -n "$NO_CONV" ] && exit 0
timeout -k 10 300 python bench.py --case convection --steps 1 --warmup 0 > gpurun_out/r04_conv_rb2.json 2> gpurun_out/r04_conv_rb2.err || exit 1
echo conv done
