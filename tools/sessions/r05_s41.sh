#!/bin/bash
# Round 5, session 41: the LRU's pass 0 (no histogram, three merge atomics a
# workgroup) on 128 workgroups instead of 32; LRU tests, per-pass durations.
TAG=r05_s41
source "$(dirname "$0")/../gpu_lib.sh"
pytest_gpu tests_ct 600 tests/test_gpu_conntrack.py
KEEP_GOING=1
for r in 1 2; do
  run ct_probe_$r 300 python tools/ct_probe.py --steps 6
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ct_prof" -o run \
    -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/ct_prof.log" 2>&1 )
echo "== ct_prof rc=$?"
python3 - "$O/ct_prof" > "$O/ev_passes.txt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "ct_ev_" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for i, r in enumerate(rows):
    print(i % 8, r["Kernel_Name"][:40], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
PY
find "$O" -name "*kernel_trace.csv" -delete
pytest_gpu tests_fw 600 tests/test_gpu_firewall.py
exit 0
