#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 run, kernel-trace only).
# CONFIG=<bench config> (default headline).  Output: gpurun_out/pmc/<config>_<pass>/...
# counter_collection.csv per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-headline}
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-lane-occupancy --train-steps 1}
mkdir -p gpurun_out/pmc
run() {  # run <name> <counters...>
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc/${CONFIG}_$name \
    -o run -- python3 bench.py --config $CONFIG $ARGS > gpurun_out/pmc/${CONFIG}_$name.log 2>&1
}
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY \
  SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 && \
run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD \
  SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
