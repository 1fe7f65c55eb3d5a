#!/bin/bash
# MNIST bf16 kernel trace -> gpurun_out/prof_m16.txt
set -e
R=/root/repo
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_m16 -o p -- python $R/bench.py --dtype bf16 --steps 200 --warmup 50 --no-eval --prewarm-ms 0 > $O/prof_m16.log 2>&1
python $R/scripts/prof_summary.py $(ls $O/prof_m16/*/*.db $O/prof_m16/*.db 2>/dev/null | head -1) > $O/prof_m16.txt
