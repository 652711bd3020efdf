#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kb
timeout -k 10 300 env KB_SUSTAIN="${KB_SUSTAIN:-}" ./tools/bin/kbench "${1:-1048576}" "${2:-20}" > gpurun_out/kb/kbench_${3:-x}.log 2>&1; rc=$?
cat gpurun_out/kb/kbench_${3:-x}.log; exit $rc
