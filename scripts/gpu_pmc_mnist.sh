#!/bin/bash
# Hardware counters of the MNIST step kernels (bench.py, a few graph-replayed
# steps), one rocprofv3 --pmc pass per counter set under its own hard kill.
# Summarise: python scripts/pmc_summary.py gpurun_out/pmcm1 gpurun_out/pmcm2 gpurun_out/pmcm3
#   gpurun --timeout 400 -- 'bash scripts/gpu_pmc_mnist.sh [bench args]'
set -e
ARGS=${*:---steps 20 --warmup 5 --no-eval}
cd /tmp && export TMPDIR=/tmp
R=/root/repo
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM -d $R/gpurun_out/pmcm1 -o p -- python $R/bench.py $ARGS > $R/gpurun_out/pmcm1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES FETCH_SIZE -d $R/gpurun_out/pmcm2 -o p -- python $R/bench.py $ARGS > $R/gpurun_out/pmcm2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_TA_BUSY_sum SQ_WAVES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmcm3 -o p -- python $R/bench.py $ARGS > $R/gpurun_out/pmcm3.log 2>&1
