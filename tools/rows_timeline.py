"""Kernel timeline of the last SpGEMM call in a rocprofv3 kernel trace (relative us).
usage: python tools/rows_timeline.py gpurun_out/TAG/stats"""
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last call: from the last k_rows_entries (or k_fz_maxlen) onwards
first = max(i for i, r in enumerate(rows) if "k_rows_entries" in r["Kernel_Name"] or "k_band_stats" in r["Kernel_Name"]
            or "k_tcount" in r["Kernel_Name"])
first = max(0, first - 4)
t0 = int(rows[first]["Start_Timestamp"])
for r in rows[first:]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f'{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {r["Kernel_Name"][:70]}')
