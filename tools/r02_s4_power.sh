#!/bin/bash
# Power / energy / clock of serial vs pipelined calls.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python3 -u tools/power_probe.py c3 8 2>&1 | tee gpurun_out/power_c3.log &&
timeout -k 10 240 python3 -u tools/power_probe.py c5 4 2>&1 | tee gpurun_out/power_c5.log
