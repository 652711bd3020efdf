set -e
mkdir -p gpurun_out/r02h
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "verify" > gpurun_out/r02h/verify_tests.log 2>&1
timeout -k 10 200 python -u tools/verify_latency.py > gpurun_out/r02h/verify_latency.log 2>&1
