#!/bin/bash
# K5 phase timers by size only (tools/k5_prof.py)
mkdir -p gpurun_out/k5
timeout -k 10 300 python tools/k5_prof.py > gpurun_out/k5/k5prof.txt 2>&1
