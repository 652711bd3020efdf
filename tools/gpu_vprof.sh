# verify config timings + kernel trace of the same run
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02h
timeout -k 10 300 python -u tools/bench_configs.py --only verify --out gpurun_out/r02h/verify_cfg.json > gpurun_out/r02h/verify_cfg.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02h/vprof -o vprof -- python -u tools/bench_configs.py --only verify --out gpurun_out/r02h/verify_cfg_prof.json > gpurun_out/r02h/vprof.log 2>&1
