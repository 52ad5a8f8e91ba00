#!/bin/bash
# Round 4: randomised GPU-vs-oracle parity sweeps on the final build (packed
# counter copies, the two-item deal for multi-block chains): stateless trials
# (pcn-iptables and the three pcn-firewall conntrack modes), then stateful ones.
TAG=r04_sweep
source "$(dirname "$0")/../gpu_lib.sh"
KEEP_GOING=1
run sweep 300 python -u tools/parity_sweep.py --seconds 200 --seed0 40000
run sweep_ct 300 python -u tools/parity_sweep.py --seconds 200 --seed0 50000 --stateful
exit 0
