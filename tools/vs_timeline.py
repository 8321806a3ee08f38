"""Per-kernel timeline of the last N dispatches of a rocprofv3 --kernel-trace CSV (the *_kernel_trace.csv
file): start offset, duration, queue/stream, kernel name.  Usage: python tools/vs_timeline.py trace.csv [N]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    t0 = int(rows[0]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("gbv::", "")
        print("%9.3f %8.3f  q%-3s %-40s grid %s" % ((s - t0) / 1e6, (e - s) / 1e6, r.get("Queue_Id", r.get("Stream_Id", "?")), name[:40],
                                                  r.get("Grid_Size", r.get("Grid_Size_X", "?"))))


if __name__ == "__main__":
    main()
