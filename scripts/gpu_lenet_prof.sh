#!/bin/bash
# LeNet-5 fp32 kernel trace -> gpurun_out/prof_le.txt
set -e
R=/root/repo
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_le -o p -- python $R/bench.py --model lenet5 --steps 200 --warmup 50 --no-eval --prewarm-ms 0 > $O/prof_le.log 2>&1
python $R/scripts/prof_summary.py $(ls $O/prof_le/*/*.db $O/prof_le/*.db 2>/dev/null | head -1) > $O/prof_le.txt
