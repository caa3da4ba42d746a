#!/bin/bash
# sample socket power and GFX clock once a second for N seconds (read-only amd-smi query): tools/power_sample.sh N
for i in $(seq 1 ${1:-30}); do
  echo "t $(date +%s.%N | cut -c1-12) $(amd-smi metric -p -c 2>/dev/null | grep -E 'SOCKET_POWER|^ +CLK:' | head -3 | tr -s ' ' | tr '\n' ' ')"
  sleep 1
done
