#!/bin/bash
# PMC passes for the bench kernel (run on the GPU box via gpurun). One pass per counter
# group (rocprofv3 does not split passes); each under its own hard time limit.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate"
pass() { name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/pmc_$name" -o $name --output-format csv -- $B > "$OUT/pmc_$name.log" 2>&1; echo "pass $name rc=$?"; }
pass valu SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass stall SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE
