# k_rb2 PMC (one box): SQ issue/wait counters and FETCH/WRITE per launch at
# 1024^2 x 512 for the tile maps CFD_HIP_RB2_XMAP = 0 / 1
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
export NX=1024 NY=1024 NZ=512 ITERS=40 METHODS=rbsor CFD_HIP_RB2=1
for x in 0 1; do
  export CFD_HIP_RB2_XMAP=$x
  TAG=r04_rb2_pmc_x$x PASSES="${PASSES:-sq fetch write}" CMD="python3 tools/relax_bench.py" bash tools/pmc_passes.sh || exit 1
done
