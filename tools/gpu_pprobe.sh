set -e
mkdir -p gpurun_out/pp
timeout -k 10 200 python -u tools/pprobe.py --s 1.1 > gpurun_out/pp/pprobe_s11.log 2>&1
PPROBE_DUMP=gpurun_out/pp/stamps_s11.npy timeout -k 10 200 python -u tools/pprobe.py --s 1.1 > gpurun_out/pp/pprobe_s11b.log 2>&1
