set -e
cd /root/repo
O=/root/repo/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_generic_ops_gpu.py > $O/t0.log 2>&1
for B in 32 128; do
  timeout -k 10 300 python bench.py --model resnet18 --dtype bf16 --batch-size $B --steps 30 --warmup 10 > $O/b_rn$B.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rn128 -o p -- python /root/repo/bench.py --model resnet18 --dtype bf16 --batch-size 128 --steps 10 --warmup 3 --no-eval > $O/prof_rn128.log 2>&1
