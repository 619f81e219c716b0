# configs[4] on one box: the rocprofv3 trace + FETCH/WRITE passes of the
# 1024^2 x 512 convection step (RB-SOR capped at 200 iterations: the per-launch
# traffic does not depend on the count), that traffic profile placed in
# profiles/ of this copy, then the full step (tol 1e-6, cap 20000) whose line
# reads it for roofline.traffic.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
TAG=${TAG:-conv}
CELLS=$((1022*1022*510)) TAG=$TAG ARGS="--case convection --steps 1 --warmup 0 --relax-max-iter 200 --allow-max-iter --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
cp gpurun_out/prof_${TAG}/traffic.json profiles/${TAG}_traffic.json || exit 1
timeout -k 10 600 python bench.py --case convection --steps 1 --warmup 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench exit $rc"; tail -c 2500 gpurun_out/${TAG}_bench.json; exit $rc
