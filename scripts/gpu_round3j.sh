#!/bin/bash
cd /root/repo
bash scripts/gpu_session.sh \
  "200 python -u -m pytest tests/test_generic_ops_gpu.py -q --timeout 120 --timeout-method thread" \
  "200 python scripts/conv_lab.py --ops fwd,dgrad --layers 1,3,6,9 --reps 20"
