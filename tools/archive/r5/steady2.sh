#!/bin/bash
set -u
O=gpurun_out/r5/steady2
mkdir -p $O
bash tools/r5/steady.sh steady2 || exit $?
timeout -k 10 240 python tools/dbg_c4_steady.py > $O/dbg_c4.log 2>&1 || exit 7
echo ok
