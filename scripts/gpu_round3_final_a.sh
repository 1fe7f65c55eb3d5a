#!/bin/bash
# Round-3 closing session, part A: every GPU test, smoke, every BASELINE config's bench line
cd /root/repo
bash scripts/gpu_session.sh \
  "700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "60 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "120 python bench.py --steps 20 --warmup 5" \
  "120 python bench.py --steps 1000 --warmup 100 --no-eval" \
  "120 python bench.py --dtype bf16 --steps 20 --warmup 5" \
  "120 python bench.py --dtype bf16 --steps 1000 --warmup 100 --no-eval" \
  "120 python bench.py --model lenet5" \
  "120 python bench.py --model resnet18 --dtype bf16 --steps 30 --warmup 10" \
  "120 python bench.py --model resnet18 --dtype bf16 --batch-size 128 --steps 30 --warmup 10 --no-eval" \
  "120 python bench.py --model resnet18 --steps 30 --warmup 10"
