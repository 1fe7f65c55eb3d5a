#!/bin/bash
cd /root/repo
bash scripts/gpu_session.sh \
  "120 python scripts/bnb_route_diff.py --hw 32 --batch 32"
