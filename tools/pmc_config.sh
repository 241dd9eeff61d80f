#!/bin/bash
# PMC passes (one counter group per run, each under its own hard limit) for one bench config,
# then the per-kernel summary.  Usage (repo root, on the GPU box):
#   bash tools/pmc_config.sh <config> <outdir> [extra bench.py args...]
set -eo pipefail
export TMPDIR=/tmp
C=$1
OUT=$2
shift 2
mkdir -p "$OUT"
pass() { name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o $name --output-format csv -- \
    python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate $EXTRA > "$OUT/$name.log" 2>&1
  echo "pmc c$C $name ok"
}
EXTRA="$*"
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass valu SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES
pass stall SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
# EVALS / STEPS (env): one launch's batch and filter steps per eval, for the derived per-eval figures
python3 tools/pmc_summary.py ${EVALS:+--evals $EVALS --steps ${STEPS:-599}} $(find "$OUT" -name "*counter_collection.csv") > "$OUT/pmc_summary.json"
echo "summary ok"
