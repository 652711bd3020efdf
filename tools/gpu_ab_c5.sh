# interleaved C5 A/B over lib/ab/*.so (Zipf 1.1 and 1.0), per-wave probe, then the GPU suite
set -e
mkdir -p gpurun_out/ab
timeout -k 10 200 python -u tools/ab_c5.py --s 1.1 --reps 7 > gpurun_out/ab/ab_s11.log 2>&1
timeout -k 10 200 python -u tools/ab_c5.py --s 1.0 --reps 7 > gpurun_out/ab/ab_s10.log 2>&1
PPROBE_DUMP=gpurun_out/ab/stamps_s11.npy timeout -k 10 200 python -u tools/pprobe.py --s 1.1 > gpurun_out/ab/pprobe_s11.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/gpu_tests.log 2>&1
