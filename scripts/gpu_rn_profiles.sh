set -e
cd /root/repo
O=/root/repo/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_generic_ops_gpu.py -k "resume" > $O/t_resume.log 2>&1
for B in 32 64 128; do
  timeout -k 10 300 python bench.py --model resnet18 --dtype bf16 --batch-size $B --steps 30 --warmup 10 > $O/b_rn$B.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
for B in 32 64 128; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rn$B -o p -- python /root/repo/bench.py --model resnet18 --dtype bf16 --batch-size $B --steps 10 --warmup 3 --no-eval > $O/prof_rn$B.log 2>&1
done
