#!/bin/bash
# Hardware counters of the conv kernels (conv_lab layers), one rocprofv3 --pmc
# pass per counter set, each under its own hard kill (no trace domains with
# --pmc).  Summarise with scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2.
#   gpurun --timeout 400 -- 'bash scripts/gpu_pmc.sh [conv_lab args]'
set -e
ARGS=${*:---batch 32 --layers 1,3,6 --ops fwd --reps 5}
cd /tmp && export TMPDIR=/tmp
R=/root/repo
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -d $R/gpurun_out/pmc1 -o p -- python $R/scripts/conv_lab.py $ARGS > $R/gpurun_out/pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU FETCH_SIZE -d $R/gpurun_out/pmc2 -o p -- python $R/scripts/conv_lab.py $ARGS > $R/gpurun_out/pmc2.log 2>&1
