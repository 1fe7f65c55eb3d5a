#!/bin/bash
# Round-3 closing session: every GPU test, smoke, every BASELINE config's bench line, and the
# kernel traces committed under profiles/ (summaries in gpurun_out/prof_*.txt)
cd /root/repo
R=/root/repo
O=$R/gpurun_out
bash scripts/gpu_session.sh \
  "700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "60 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "120 python bench.py --steps 20 --warmup 5" \
  "120 python bench.py --steps 1000 --warmup 100 --no-eval" \
  "120 python bench.py --dtype bf16 --steps 20 --warmup 5" \
  "120 python bench.py --dtype bf16 --steps 1000 --warmup 100 --no-eval" \
  "120 python bench.py --model lenet5" \
  "120 python bench.py --model resnet18 --dtype bf16 --steps 30 --warmup 10" \
  "120 python bench.py --model resnet18 --dtype bf16 --batch-size 128 --steps 30 --warmup 10 --no-eval" \
  "120 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "200 bash scripts/gpu_mnist_prof.sh" \
  "200 bash scripts/gpu_mnist_prof16.sh" \
  "200 bash scripts/gpu_resnet_prof16.sh" \
  "200 bash scripts/gpu_resnet_prof32.sh" \
  "200 bash scripts/gpu_lenet_prof.sh"
