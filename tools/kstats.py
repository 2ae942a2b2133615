"""Per-kernel duration summary from a rocprofv3 rocpd sqlite file or a
kernel_stats.csv:  python tools/kstats.py <file> [name-filter]"""
import csv
import sqlite3
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = defaultdict(list)
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        q = ("select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d "
             "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
        for name, dur in c.execute(q):
            acc[name].append(dur)
    else:
        for r in csv.DictReader(open(path)):
            acc[r["Name"]].append(float(r["AverageNs"]))  # averages only
    rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
    for name, d in rows:
        if filt in name:
            print(f"{sum(d)/1e6:10.3f} ms  n={len(d):4d}  avg={sum(d)/len(d)/1e6:9.4f} ms  {name[:110]}")


if __name__ == "__main__":
    main()
