"""Per-call kernel durations from a rocprofv3 kernel_trace.csv: tools/ktrace.py <csv> [substring...]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pats = sys.argv[2:] or [""]
for r in rows:
    n = r["Kernel_Name"]
    if any(p in n for p in pats):
        print(f"{n[:52]:52s} grid {r['Grid_Size_X']:>9s} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000:10.1f} us "
              f"vgpr {r['VGPR_Count']} scratch {r['Scratch_Size']} lds {r['LDS_Block_Size']}")
