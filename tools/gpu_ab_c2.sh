# interleaved braided-kernel A/B over lib/ab/*.so at several small batch sizes
set -e
mkdir -p gpurun_out/ab2
for n in 16384 65536 262144; do
  timeout -k 10 200 python -u tools/ab_c2.py --n $n --reps 5 > gpurun_out/ab2/ab_c2_$n.log 2>&1
done
