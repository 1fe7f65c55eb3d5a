#!/bin/bash
# Round-3 closing session, part B: kernel traces (summaries in gpurun_out/prof_*.txt)
cd /root/repo
bash scripts/gpu_session.sh \
  "200 bash scripts/gpu_mnist_prof.sh" \
  "200 bash scripts/gpu_mnist_prof16.sh" \
  "200 bash scripts/gpu_resnet_prof16.sh" \
  "200 bash scripts/gpu_resnet_prof32.sh" \
  "200 bash scripts/gpu_lenet_prof.sh"
