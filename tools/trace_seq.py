"""One stateful batch's kernel sequence from a rocprofv3 --kernel-trace CSV
directory: each dispatch's gap to the previous one's end and its duration (us),
from the last batch's stage-A classify to the end (GPU box output only; kernels on
the LRU's own stream overlap ct_count: negative gaps).

  python3 tools/trace_seq.py <rocprofv3 -d directory>
"""
import csv
import glob
import sys


def main():
    f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    # the batch's first conntrack kernel: ct_prep, or ct_stale_agg after a stage A that wrote the records
    idx = [i for i, r in enumerate(rows) if "ct_prep" in r["Kernel_Name"] or "ct_stale_agg" in r["Kernel_Name"]][-1] - 1
    prev, first = None, None
    for r in rows[idx - 4:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "copyBuffer" in r["Kernel_Name"]:
            continue
        first = first or s
        gap = (s - prev) / 1000 if prev else 0
        print(f"{r['Kernel_Name'][:48]:48s} grid {r.get('Grid_Size', '?'):>10s} wg {r.get('Workgroup_Size', '?'):>5s} "
              f"gap {gap:7.1f} dur {(e - s) / 1000:7.1f}")
        prev = e
    print(f"span {(prev - first) / 1000:.1f} us")


if __name__ == "__main__":
    main()
