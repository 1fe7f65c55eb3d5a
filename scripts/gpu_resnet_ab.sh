#!/bin/bash
# ResNet-18 bf16 B=32 kernel traces with and without the BN backward epilogue
# (same box) -> gpurun_out/prof_r16_{on,off}.txt
set -e
R=/root/repo
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for mode in on off; do
  v=1; [ $mode = off ] && v=0
  MTA_BN_BWD_EPILOGUE=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_r16_$mode -o p -- python $R/bench.py --model resnet18 --dtype bf16 --steps 10 --warmup 3 --no-eval --prewarm-ms 0 > $O/prof_r16_$mode.log 2>&1
  python $R/scripts/prof_summary.py $(ls $O/prof_r16_$mode/*/*.db $O/prof_r16_$mode/*.db 2>/dev/null | head -1) > $O/prof_r16_$mode.txt
done
