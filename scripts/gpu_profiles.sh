#!/bin/bash
# Every BASELINE config's bench.py line plus a rocprofv3 kernel trace of each,
# on the gpurun box (summaries: scripts/prof_summary.py <db> -> profiles/).
#   gpurun --timeout 1100 -- 'bash scripts/gpu_profiles.sh'
set -e
cd /root/repo
O=/root/repo/gpurun_out
mkdir -p $O
timeout -k 10 300 python bench.py > $O/b_mnist32.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_mnist32_driver.log 2>&1
timeout -k 10 300 python bench.py --dtype bf16 > $O/b_mnist16.log 2>&1
timeout -k 10 300 python bench.py --model lenet5 > $O/b_lenet.log 2>&1
for B in 32 64 128; do
  timeout -k 10 300 python bench.py --model resnet18 --dtype bf16 --batch-size $B --steps 30 --warmup 10 > $O/b_rn$B.log 2>&1
done
timeout -k 10 300 python bench.py --model resnet18 --steps 30 --warmup 10 > $O/b_rn32_fp32.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_m32 -o p -- python /root/repo/bench.py --steps 200 --warmup 50 --no-eval --prewarm-ms 0 > $O/prof_m32.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_m16 -o p -- python /root/repo/bench.py --dtype bf16 --steps 200 --warmup 50 --no-eval --prewarm-ms 0 > $O/prof_m16.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_le -o p -- python /root/repo/bench.py --model lenet5 --steps 200 --warmup 50 --no-eval --prewarm-ms 0 > $O/prof_le.log 2>&1
for B in 32 64 128; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rn$B -o p -- python /root/repo/bench.py --model resnet18 --dtype bf16 --batch-size $B --steps 10 --warmup 3 --no-eval --prewarm-ms 0 > $O/prof_rn$B.log 2>&1
done
