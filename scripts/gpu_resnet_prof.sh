#!/bin/bash
# ResNet-18 step: bench lines (bf16 B=32/128, fp32 B=32) + kernel traces
# summarised into gpurun_out/prof_r{16,32}.txt.   gpurun -- 'bash scripts/gpu_resnet_prof.sh'
set -e
R=/root/repo
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 200 python bench.py --model resnet18 --dtype bf16 --steps 30 --warmup 10 > $O/b_r16.log 2>&1
timeout -k 10 200 python bench.py --model resnet18 --dtype bf16 --batch-size 128 --steps 30 --warmup 10 --no-eval > $O/b_r16_128.log 2>&1
timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 10 > $O/b_r32.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_r16 -o p -- python $R/bench.py --model resnet18 --dtype bf16 --steps 10 --warmup 3 --no-eval --prewarm-ms 0 > $O/prof_r16.log 2>&1
python $R/scripts/prof_summary.py $(ls $O/prof_r16/*/*.db $O/prof_r16/*.db 2>/dev/null | head -1) > $O/prof_r16.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_r32 -o p -- python $R/bench.py --model resnet18 --steps 10 --warmup 3 --no-eval --prewarm-ms 0 > $O/prof_r32.log 2>&1
python $R/scripts/prof_summary.py $(ls $O/prof_r32/*/*.db $O/prof_r32/*.db 2>/dev/null | head -1) > $O/prof_r32.txt
