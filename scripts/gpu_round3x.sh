#!/bin/bash
# fp32 stem filter gradient (gather path): slice-cap sweep
cd /root/repo
bash scripts/gpu_session.sh \
  "90 python scripts/conv_lab.py --dtype fp32 --reps 10 --layers 0 --ops wgrad" \
  "90 env MTA_TILED_GCAP=256 python scripts/conv_lab.py --dtype fp32 --reps 10 --layers 0 --ops wgrad" \
  "90 env MTA_TILED_GCAP=512 python scripts/conv_lab.py --dtype fp32 --reps 10 --layers 0 --ops wgrad" \
  "90 env MTA_TILED_GCAP=1024 python scripts/conv_lab.py --dtype fp32 --reps 10 --layers 0 --ops wgrad" \
  "90 python -u -m pytest tests/test_generic_ops_gpu.py -q -x --timeout 120 --timeout-method thread -k conv_fwd_bwd"
