export NX=1024 NY=1024 NZ=512 ITERS=100 METHODS=rbsor
TAG=r04_rb2_xmap SW=CFD_HIP_RB2_XMAP VALUES="0 1" CMD="python3 tools/relax_bench.py" ROUNDS=2 bash tools/ab.sh || exit 1
export CFD_HIP_RB2_XMAP=1
TAG=r04_rb2_kc SW=CFD_HIP_RB2_KC VALUES="64 128 32" CMD="python3 tools/relax_bench.py" ROUNDS=2 bash tools/ab.sh || exit 1
export NX=512 NY=512 NZ=512
TAG=r04_rb2_xmap512 SW=CFD_HIP_RB2_XMAP VALUES="0 1" CMD="python3 tools/relax_bench.py" ROUNDS=2 bash tools/ab.sh
