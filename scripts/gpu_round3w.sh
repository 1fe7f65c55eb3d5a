#!/bin/bash
# fp32 tiled convs: split-K target sweep (forward / dgrad, filter gradient)
cd /root/repo
bash scripts/gpu_session.sh \
  "90 python scripts/conv_lab.py --dtype fp32 --reps 10" \
  "90 env MTA_TILED_KSPLIT=512 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops fwd,dgrad" \
  "90 env MTA_TILED_KSPLIT=768 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops fwd,dgrad" \
  "90 env MTA_TILED_KSPLIT=1536 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops fwd,dgrad" \
  "90 env MTA_TILED_KSPLIT=2048 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops fwd,dgrad" \
  "90 env MTA_TILED_WGSPLIT=1024 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops wgrad" \
  "90 env MTA_TILED_WGSPLIT=1536 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops wgrad" \
  "90 env MTA_TILED_WGSPLIT=3072 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops wgrad" \
  "90 env MTA_TILED_WGSPLIT=4096 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops wgrad"
