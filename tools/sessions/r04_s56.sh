#!/bin/bash
# Round 4, sessions 5 + 6 in one box: the stateful walk change (tests + A/B),
# then the counter passes and config-3 / config-5 A/Bs of session 5.
bash "$(dirname "$0")/r04_s6.sh"; rc=$?
case $rc in 124|134|137|139) exit $rc ;; esac
exec_s5() { bash "$(dirname "$0")/r04_s5.sh"; }
exec_s5
