#!/bin/bash
# The one GPU-session runner (run it under gpurun from the repo root).  A
# session is a list of steps; each step runs under its own time limit with
# its log in gpurun_out/.  A step that fails normally (exit 1: a test
# failure) lets the next one run; a fault / abort / segfault / timeout (any
# other non-zero code) ends the session there.
#
#   bash scripts/gpu_session.sh STEP...        STEP = "<limit_s> <command>"
#   bash scripts/gpu_session.sh @FILE          steps from FILE, one per line
#                                              (scripts/sessions/*.steps; # comments)
# Step commands may use these macros:
#   prof NAME ARGS...   rocprofv3 --kernel-trace --stats of `python ARGS`,
#                       summary in gpurun_out/NAME.txt (scripts/prof_summary.py)
#   pmc NAME SET ARGS...  one rocprofv3 --pmc pass (counter SET below) of
#                       `python ARGS` into gpurun_out/NAME (scripts/pmc_summary.py)
#   emu N BW SCHED ARGS...  bench.py against an emulated N-rank ring at BW GB/s
#                       (10 us latency), one "N= busbw= sched= us_per_step=" line
#                       appended to gpurun_out/emu_grid.log
R=$(pwd)
O=$R/gpurun_out
mkdir -p "$O"

declare -A PMC=(
  [wave]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM"
  [lds]="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES FETCH_SIZE"
  [mem]="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_TA_BUSY_sum SQ_WAVES GRBM_GUI_ACTIVE"
)

prof() {
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp &&
   rocprofv3 --kernel-trace --stats -d "$O/$name" -o p -- python "$R/$1" "${@:2}") > "$O/$name.log" 2>&1 || return $?
  python "$R/scripts/prof_summary.py" $(ls "$O/$name"/*/*.db "$O/$name"/*.db 2>/dev/null | head -1) > "$O/$name.txt"
}

pmc() {
  local name=$1 set=$2; shift 2
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -s KILL 90 rocprofv3 --pmc ${PMC[$set]} -d "$O/$name" -o p -- python "$R/$1" "${@:2}") > "$O/$name.log" 2>&1
}

emu() {
  local n=$1 bw=$2 sched=$3; shift 3
  local r
  r=$(python bench.py --comm-emulate 10,$bw,$n --sync-schedule $sched --no-eval "$@" 2>/dev/null |
      grep -o '"ms_per_step": [0-9.]*' | grep -o '[0-9.]*$') || return 3
  echo "N=$n busbw=$bw sched=$sched us_per_step=$(python -c "print(round(1000*$r,1))") args=$*" | tee -a "$O/emu_grid.log"
}
export -f prof pmc emu
export R O
export PMC_WAVE="${PMC[wave]}" PMC_LDS="${PMC[lds]}" PMC_MEM="${PMC[mem]}"

specs=()
for a in "$@"; do
  if [[ $a == @* ]]; then
    while IFS= read -r line; do
      [[ -z ${line// } || $line == \#* ]] && continue
      specs+=("$line")
    done < "${a#@}"
  else
    specs+=("$a")
  fi
done

n=0
for spec in "${specs[@]}"; do
  n=$((n+1))
  lim=${spec%% *}; cmd=${spec#* }
  echo "=== step $n (limit ${lim}s): $cmd" | tee -a "$O/session.log"
  start=$(date +%s)
  timeout -k 10 "$lim" bash -c "$(declare -p PMC); $(declare -f prof pmc emu); $cmd" > "$O/step$n.log" 2>&1
  rc=$?
  echo "=== step $n rc=$rc ($(( $(date +%s) - start ))s)" | tee -a "$O/session.log"
  tail -n 25 "$O/step$n.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping after rc=$rc" | tee -a "$O/session.log"
    exit $rc
  fi
done
exit 0
