#!/bin/bash
# Sync-schedule step times against the emulated N-rank ring (1 GPU):
#   bash scripts/emu_grid.sh "2 8" "50 100 200" "buckets sharded factors"
O=gpurun_out/emu_grid.log
mkdir -p gpurun_out
for N in $1; do for BW in $2; do for S in $3; do
  r=$(timeout -k 10 120 python bench.py --comm-emulate 10,$BW,$N --sync-schedule $S --steps 500 \
      --warmup 50 --no-eval --prewarm-ms 50 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | grep -o '[0-9.]*$') || exit 3
  echo "N=$N busbw=$BW sched=$S us_per_step=$(python -c "print(round(1000*$r,1))")" | tee -a $O
done; done; done
