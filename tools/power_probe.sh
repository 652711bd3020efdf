#!/usr/bin/env bash
# Sample GPU power/clock from sysfs every ~20 ms while kbench runs long sustained loops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/power; mkdir -p $OUT
HW=""
for d in /sys/class/drm/card*/device/hwmon/hwmon*; do [ -e "$d/power1_average" ] || [ -e "$d/power1_input" ] && HW="$d" && break; done
DEV=$(dirname $(dirname "$HW" 2>/dev/null) 2>/dev/null)
{ echo "HW=$HW DEV=$DEV"; ls $HW 2>&1 | head -50; ls $DEV 2>&1 | grep -i -E "pp_dpm|gpu_metrics|power" ; } > $OUT/sysfs.txt
( while true; do
    t=$(date +%s.%N)
    p=$(cat $HW/power1_average 2>/dev/null || cat $HW/power1_input 2>/dev/null)
    sc=$(grep '\*' $DEV/pp_dpm_sclk 2>/dev/null | tr -d '\n')
    mc=$(grep '\*' $DEV/pp_dpm_mclk 2>/dev/null | tr -d '\n')
    fc=$(grep '\*' $DEV/pp_dpm_fclk 2>/dev/null | tr -d '\n')
    echo "$t $p | s:$sc | m:$mc | f:$fc"
    sleep 0.02
  done ) > $OUT/samples.txt 2>&1 &
SP=$!
KB_NS=${KB_NS:-3000} KB_SUSTAIN="${1:-braid_prod,braid_nolut,braid_skel,gprobe_G16_R6_al1_d1_256x1024}" timeout -k 10 200 ./tools/bin/kbench 1048576 2 > $OUT/kbench.log 2>&1
rc=$?
kill $SP 2>/dev/null
grep SUSTAIN $OUT/kbench.log | cut -c1-110
exit $rc
