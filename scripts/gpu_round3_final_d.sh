#!/bin/bash
# Round-3 closing, final build: every GPU test, smoke, the bench lines that changed
cd /root/repo
bash scripts/gpu_session.sh \
  "700 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread" \
  "60 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "120 python bench.py --steps 20 --warmup 5" \
  "120 python bench.py --model resnet18 --steps 30 --warmup 10" \
  "120 python bench.py --model resnet18 --dtype bf16 --steps 30 --warmup 10 --no-eval" \
  "200 bash scripts/gpu_resnet_prof32.sh"
