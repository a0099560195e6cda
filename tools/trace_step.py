"""Print one bench step's kernel timeline from a rocprofv3 kernel-trace CSV.
   python tools/trace_step.py gpurun_out/prof_TAG [min_us]"""
import csv
import glob
import sys

d = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
path = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_compensate_list" in r["Kernel_Name"]]
i0, i1 = idx[-2], idx[-1]
prev = None
small = 0.0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    us = (e - s) / 1e3
    if us >= min_us:
        print(f"{r['Kernel_Name'][:58]:58s} {us:9.2f} us  gap {((s - prev) / 1e3 if prev else 0):6.2f}  "
              f"vgpr {r['VGPR_Count']} lds {r['LDS_Block_Size']}")
    else:
        small += us
    prev = e
print(f"(kernels under {min_us} us: {small:.1f} us)  step span {(int(rows[i1]['Start_Timestamp']) - int(rows[i0]['Start_Timestamp'])) / 1e6:.3f} ms")
