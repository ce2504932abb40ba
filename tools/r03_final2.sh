#!/bin/bash
# Round-3 re-measurement after the general-kernel changes: C3 profile (stats + PMC) and the per-config table
set -o pipefail
O=gpurun_out/r03/${FINAL_TAG:-final2}
mkdir -p $O
bash tools/profile.sh r03c3${FINAL_TAG:-b} --config C3 --docs 10000 > $O/profile_c3.log 2>&1 || { tail $O/profile_c3.log; exit 4; }
python tools/pmc_summary.py gpurun_out/r03c3${FINAL_TAG:-b} merge_large_kernel > $O/c3_pmc_summary.json || exit 5
find gpurun_out/r03c3${FINAL_TAG:-b}/trace -name "*kernel_stats.csv" -exec cp {} $O/c3_kernel_stats.csv \;
timeout -k 10 1000 python tools/perf_table.py > $O/perf_table.md 2>&1 || { tail -20 $O/perf_table.md; exit 1; }
grep -v '^<!--' $O/perf_table.md
python3 -c "
import json
s = json.load(open('$O/c3_pmc_summary.json'))
print({k: round(v, 4) if isinstance(v, float) else v for k, v in s.items() if k in ('avg_ns', 'hbm_traffic_bytes', 'SQ_WAIT_ANY', 'SQ_WAVE_CYCLES', 'SQ_LDS_BANK_CONFLICT', 'SQ_INSTS_LDS')})
"
