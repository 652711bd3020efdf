# HBM read bytes of the C5 launches (rocprofv3 --pmc FETCH_SIZE, one pass)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c5f
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/c5f/p" -o c5 -- python3 "$GRAFT_REPO_ROOT/tools/prof_pieces.py" 3 > "$GRAFT_REPO_ROOT/gpurun_out/c5f/p.log" 2>&1
