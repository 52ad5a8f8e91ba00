#!/bin/bash
# Round 6, session 16 (measurement build): where ct_count's time goes -- the
# kernel with its LDS atomics (0), without them (1), loads only (2); kernel trace each.
TAG=${TAG:-r06_s16}
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
for m in 0 1 2; do
  ( cd /tmp && PCN_IPT_DEBUG_CT_COUNT_DBG=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$m" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 6 > "$O/prof_$m.log" 2>&1 )
  echo "== prof_$m rc=$?"
  python3 tools/ktsum.py "$O/prof_$m" > "$O/prof_$m.txt" 2>&1 || true
  find "$O" -name "*kernel_trace.csv" -delete
done
exit 0
