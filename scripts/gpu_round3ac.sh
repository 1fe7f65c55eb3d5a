#!/bin/bash
# fp32 filter gradient (vector path): slice-cap sweep
cd /root/repo
bash scripts/gpu_session.sh \
  "90 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops wgrad" \
  "90 env MTA_TILED_VCAP=128 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops wgrad" \
  "90 env MTA_TILED_VCAP=256 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops wgrad" \
  "90 env MTA_TILED_VCAP=128 MTA_TILED_WGSPLIT=4096 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops wgrad"
