#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 1000 python tools/perf_table.py > gpurun_out/r03/perf_table_r03.md 2>&1 || { tail -20 gpurun_out/r03/perf_table_r03.md; exit 1; }
grep -v '^<!--' gpurun_out/r03/perf_table_r03.md
