ls /sys/class/drm/ 2>&1 | head -20
for c in /sys/class/drm/card*/device; do echo "== $c"; cat $c/pp_dpm_sclk 2>&1 | head -5; ls $c/hwmon/*/ 2>/dev/null | grep -i freq | head; cat $c/hwmon/*/freq1_input 2>&1 | head -2; cat $c/hwmon/*/power1_average 2>&1 | head -1; cat $c/gpu_metrics 2>/dev/null | wc -c; done 2>&1 | head -60
which amd-smi rocm-smi 2>&1
timeout 20 amd-smi metric -c -g 0 2>&1 | head -30
