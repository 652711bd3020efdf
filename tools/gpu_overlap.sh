set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ov
timeout -k 10 200 python -u tools/overlap_probe.py > gpurun_out/ov/overlap.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/ov/prof -o ov -- python -u tools/overlap_probe.py --steps 10 > gpurun_out/ov/overlap_prof.log 2>&1
