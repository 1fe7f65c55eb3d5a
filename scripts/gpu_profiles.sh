set -e
cd /root/repo
O=/root/repo/gpurun_out
timeout -k 10 300 python bench.py > $O/b_mnist32.log 2>&1
timeout -k 10 300 python bench.py --dtype bf16 > $O/b_mnist16.log 2>&1
timeout -k 10 300 python bench.py --model lenet5 > $O/b_lenet.log 2>&1
timeout -k 10 300 python bench.py --model resnet18 --dtype bf16 --steps 100 --warmup 20 > $O/b_rn32.log 2>&1
timeout -k 10 300 python bench.py --model resnet18 --dtype bf16 --batch-size 64 --steps 50 --warmup 10 > $O/b_rn64.log 2>&1
timeout -k 10 300 python bench.py --model resnet18 --dtype bf16 --batch-size 128 --steps 30 --warmup 10 > $O/b_rn128.log 2>&1
timeout -k 10 300 python bench.py --model resnet18 --steps 30 --warmup 10 > $O/b_rn32_fp32.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_m32 -o p -- python /root/repo/bench.py --steps 200 --warmup 50 --no-eval > $O/prof_m32.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_m16 -o p -- python /root/repo/bench.py --dtype bf16 --steps 200 --warmup 50 --no-eval > $O/prof_m16.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_le -o p -- python /root/repo/bench.py --model lenet5 --steps 200 --warmup 50 --no-eval > $O/prof_le.log 2>&1
