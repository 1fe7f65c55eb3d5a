#!/bin/bash
# Counters of the conv2 kernels (scripts/wino_lab.py), one pass per set.
#   bash scripts/gpu_pmc_wino.sh [--only NAME]
set -e
cd /tmp && export TMPDIR=/tmp
R=/root/repo
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM -d $R/gpurun_out/pmcw1 -o p -- python $R/scripts/wino_lab.py --reps 20 "$@" > $R/gpurun_out/pmcw1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d $R/gpurun_out/pmcw2 -o p -- python $R/scripts/wino_lab.py --reps 20 "$@" > $R/gpurun_out/pmcw2.log 2>&1
python $R/scripts/pmc_summary.py $R/gpurun_out/pmcw1 $R/gpurun_out/pmcw2 > $R/gpurun_out/pmcw_summary.txt
