#!/bin/bash
# ResNet-18 fp32 step trace summarised into gpurun_out/prof_r32.txt
set -e
R=/root/repo
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_r32 -o p -- python $R/bench.py --model resnet18 --steps 10 --warmup 3 --no-eval --prewarm-ms 0 > $O/prof_r32.log 2>&1
python $R/scripts/prof_summary.py $(ls $O/prof_r32/*/*.db $O/prof_r32/*.db 2>/dev/null | head -1) > $O/prof_r32.txt
