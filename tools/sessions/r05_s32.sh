#!/bin/bash
# Round 5, session 32: one stateful batch's kernel sequence with timestamps (gaps
# and durations), to see what the 43 us of ct_seg_fix is when no cut is active.
TAG=r05_s32
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tr" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 3 > "$O/tr.log" 2>&1 )
echo "== tr rc=$?"
python3 - "$O/tr" > "$O/sequence.txt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# the last batch: from the last ct_prep's preceding classify to the end
idx = [i for i, r in enumerate(rows) if "ct_prep" in r["Kernel_Name"]][-1] - 1
prev = None
for r in rows[idx - 4:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0
    print(f"{r['Kernel_Name'][:48]:48s} grid {r.get('Grid_Size', r.get('Grid_Size_X', '?')):>10s} "
          f"wg {r.get('Workgroup_Size', r.get('Workgroup_Size_X', '?')):>5s} gap {gap:7.1f} dur {(e - s) / 1000:7.1f} "
          f"vgpr {r.get('Arch_VGPR_Count', r.get('VGPR_Count', '?'))} lds {r.get('LDS_Block_Size', r.get('Lds_Size', '?'))} scr {r.get('Scratch_Size', '?')}")
    prev = e
PY
find "$O" -name "*kernel_trace.csv" -delete
exit 0
