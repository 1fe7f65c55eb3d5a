#!/bin/bash
# fp32 tiled conv tile plan: 128-row tiles from M >= 32768 (default) vs never vs always
cd /root/repo
bash scripts/gpu_session.sh \
  "120 python scripts/conv_lab.py --dtype fp32 --reps 10" \
  "120 env MTA_TILED_M128=1000000000 python scripts/conv_lab.py --dtype fp32 --reps 10" \
  "120 env MTA_TILED_M128=12000 python scripts/conv_lab.py --dtype fp32 --reps 10" \
  "120 env MTA_TILED_M128=0 python scripts/conv_lab.py --dtype fp32 --reps 10"
