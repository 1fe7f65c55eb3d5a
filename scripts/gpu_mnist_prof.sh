#!/bin/bash
# MNIST step: bench lines (fp32, bf16) + kernel traces summarised into
# gpurun_out/prof_m{32,16}.txt.   gpurun -- 'bash scripts/gpu_mnist_prof.sh'
set -e
R=/root/repo
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-eval > $O/b_m32.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b_m32_driver.log 2>&1
timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-eval --dtype bf16 > $O/b_m16.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_m32 -o p -- python $R/bench.py --steps 200 --warmup 50 --no-eval --prewarm-ms 0 > $O/prof_m32.log 2>&1
python $R/scripts/prof_summary.py $(ls $O/prof_m32/*/*.db $O/prof_m32/*.db 2>/dev/null | head -1) > $O/prof_m32.txt
