#!/bin/bash
# Helpers for one GPU-box session script (source it; run the script through gpurun
# from the repo root).  Every GPU step runs under its own timeout; `run` ends the
# session at the first crash, abort or time limit (124/134/137/139) and, unless
# KEEP_GOING=1, at any failure.  Logs go to gpurun_out/$TAG/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${TAG:-s}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp

run() {   # run <name> <timeout s> <cmd...>: stdout+stderr -> $O/<name>.log
  local name=$1 t=$2
  shift 2
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(( $(date +%s) - t0 )) s)"
  tail -4 "$O/$name.log"
  case $rc in
    0) ;;
    124|134|137|139) echo "fatal rc=$rc in $name: stopping"; exit $rc ;;
    *) [ "${KEEP_GOING:-0}" = 1 ] || exit $rc ;;
  esac
}

pytest_gpu() {   # pytest_gpu <name> <timeout> <pytest args...>
  local name=$1 t=$2
  shift 2
  run "$name" "$t" python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "$@"
}

# PMC passes of the classify kernel, one counter group per rocprofv3 run:
# pmc <name> <cfg> <log2n> [hook]   -> $O/<name>/p1 (FETCH_SIZE), p2 (WRITE_SIZE)
pmc() {
  local name=$1 cfg=$2 log2n=$3 hook=${4:-xdp}
  mkdir -p "$O/$name"
  local k=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    k=$((k + 1))
    ( cd /tmp && CFG5_HOOK=$hook timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
        -d "$O/$name/p$k" -o run -- python3 "$R/tools/ablate.py" --child --lib "" --hit 0.5 --iters 5 \
        --log2n "$log2n" --cfg "$cfg" --jit 1 > "$O/$name/p$k.log" 2>&1 )
    local rc=$?
    echo "== pmc $name $grp rc=$rc"
    case $rc in 0) ;; *) tail -5 "$O/$name/p$k.log"; exit $rc ;; esac
  done
}

# kernel trace + stats of one ablate child: ktrace <name> <cfg> <log2n> [iters] [hook]
ktrace() {
  local name=$1 cfg=$2 log2n=$3 iters=${4:-50} hook=${5:-xdp}
  ( cd /tmp && CFG5_HOOK=$hook timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$O/$name" -o run -- python3 "$R/tools/ablate.py" --child --lib "" --hit 0.5 --iters "$iters" \
      --log2n "$log2n" --cfg "$cfg" --jit 1 > "$O/$name.log" 2>&1 )
  local rc=$?
  echo "== ktrace $name rc=$rc"
  tail -2 "$O/$name.log"
  case $rc in 0) ;; *) exit $rc ;; esac
}

# One PMC pass (any counters) of one ablate child, kernel trace only, then
# summarised on the box (tools/pmc_summary.py: per-dispatch averages of the
# classify kernel) and the raw CSVs dropped (they exceed gpurun's copy-back):
# pmcq <name> <cfg> <log2n> <hit> "<counters>" [jit defs] [hook]  -> $O/<name>.json
pmcq() {
  local name=$1 cfg=$2 log2n=$3 hit=$4 ctrs=$5 defs=${6:-} hook=${7:-xdp}
  mkdir -p "$O/$name"
  ( cd /tmp && SETTLE=0.05 PCN_IPT_JIT_DEFS="$defs" CFG5_HOOK=$hook timeout -s KILL 120 rocprofv3 --pmc $ctrs \
      --kernel-trace --output-format csv -d "$O/$name/p1" -o run -- python3 "$R/tools/ablate.py" --child --lib "" \
      --hit "$hit" --iters 5 --log2n "$log2n" --cfg "$cfg" --jit 1 > "$O/$name.log" 2>&1 )
  local rc=$?
  echo "== pmcq $name rc=$rc"
  case $rc in 0) ;; *) tail -5 "$O/$name.log"; exit $rc ;; esac
  python3 "$R/tools/pmc_summary.py" "$O/$name" --frames $((1 << log2n)) --out "$O/$name.json" > /dev/null && \
    rm -rf "$O/$name"
}

# HBM traffic of the classify kernel for bench.py's roofline.traffic:
# pmct <key> <cfg> <log2n> [hook] -> FETCH_SIZE and WRITE_SIZE passes, summarised on the
# box into $O/pmc_<key>.json and into profiles/pmc_traffic.json (copied to $O), raw CSVs dropped
pmct() {
  local key=$1 cfg=$2 log2n=$3 hook=${4:-xdp}
  local d="$O/pmc_$key"
  mkdir -p "$d"
  local k=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    k=$((k + 1))
    ( cd /tmp && CFG5_HOOK=$hook timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
        -d "$d/p$k" -o run -- python3 "$R/tools/ablate.py" --child --lib "" --hit 0.5 --iters 5 \
        --log2n "$log2n" --cfg "$cfg" --jit 1 > "$d.p$k.log" 2>&1 )
    local rc=$?
    echo "== pmct $key $grp rc=$rc"
    case $rc in 0) ;; *) tail -5 "$d.p$k.log"; exit $rc ;; esac
  done
  python3 "$R/tools/pmc_summary.py" "$d" --frames $((1 << log2n)) --out "$d.json" --traffic --key "$key" \
    --profile "profiles/$TAG/pmc_$key.json" > /dev/null && rm -rf "$d" && cp "$R/profiles/pmc_traffic.json" "$O/"
}

# One PMC pass over the stateful probe (tools/ct_probe.py), summarised per kernel:
# pmcct <name> "<counters>" "<kernel substrings...>" -> $O/<name>_<kernel>.json
pmcct() {
  local name=$1 ctrs=$2 kernels=$3
  mkdir -p "$O/$name"
  ( cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$O/$name/p1" -o run \
      -- python3 "$R/tools/ct_probe.py" --steps 3 > "$O/$name.log" 2>&1 )
  local rc=$?
  echo "== pmcct $name rc=$rc"
  case $rc in 0) ;; *) tail -5 "$O/$name.log"; exit $rc ;; esac
  for k in $kernels; do
    python3 "$R/tools/pmc_summary.py" "$O/$name" --kernel "$k" --frames $((1 << 24)) --out "$O/${name}_$k.json" > /dev/null
  done
  rm -rf "$O/$name"
}

# Counter calibration of one tools/gather_calib pattern: its own timing line, then a
# FETCH_SIZE pass and a TCC_EA0_RDREQ split pass, each summarised over the pattern's
# kernel (calib_*): calib <name> <pattern> <log2n> <kernel>  -> $O/calib_<name>{.log,_fetch.json,_rdreq.json}
calib() {
  local name=$1 pat=$2 log2n=$3 kern=$4
  run calib_$name 120 "$R/tools/gather_calib" "$pat" "$log2n" 10
  local k=0
  for grp in "FETCH_SIZE" "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"; do
    k=$((k + 1))
    mkdir -p "$O/calib_$name/p$k"
    ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
        -d "$O/calib_$name/p$k" -o run -- "$R/tools/gather_calib" "$pat" "$log2n" 4 > "$O/calib_$name/p$k.log" 2>&1 )
    local rc=$?
    echo "== calib $name pass $k rc=$rc"
    case $rc in 0) ;; *) tail -5 "$O/calib_$name/p$k.log"; exit $rc ;; esac
  done
  python3 "$R/tools/pmc_summary.py" "$O/calib_$name" --kernel "$kern" --frames $((1 << log2n)) \
    --out "$O/calib_${name}.json" > /dev/null && rm -rf "$O/calib_$name"
}
