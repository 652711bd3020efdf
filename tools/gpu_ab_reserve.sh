set -e
mkdir -p gpurun_out/r02h
timeout -k 10 400 python -u tools/ab_reserve.py --reserve 0,4,8,12,16,24 --reps 8 > gpurun_out/r02h/ab_reserve2.log 2>&1
timeout -k 10 400 python -u tools/ab_reserve.py --reserve 0,8,16 --reps 8 --n 2097152 > gpurun_out/r02h/ab_reserve_2m.log 2>&1
