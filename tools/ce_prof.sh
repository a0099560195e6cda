#!/bin/bash
mkdir -p gpurun_out/ce
timeout -k 10 300 python tools/ce_prof.py flat-1B 6 > gpurun_out/ce/ce_1B.txt 2>&1 || exit $?
cat gpurun_out/ce/ce_1B.txt
