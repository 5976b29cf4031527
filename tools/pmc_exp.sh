#!/bin/bash
# PMC passes over an experiment script (one counter group per rocprofv3 run, kernel trace only):
#   tools/pmc_exp.sh <tag> python3 tools/exp_bwd.py
# -> gpurun_out/pmcx_<tag>_<pass>/..., summarised by tools/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
run() {  # run <name> <counters...>
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmcx_${tag}/pmc_$name -o run \
    -- "${CMD[@]}" > gpurun_out/pmcx_${tag}_$name.log 2>&1
}
CMD=("$@")
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
  SQ_BUSY_CYCLES SQ_WAIT_INST_ANY && \
run sq2 SQ_INSTS_VALU_TRANS_F32 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
  SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU && \
python3 tools/pmc_summary.py gpurun_out/pmcx_${tag} gpurun_out/pmcx_${tag}.csv
