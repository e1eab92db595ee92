#!/bin/bash
# Sample GPU 0's shader clock and socket power every ~0.5 s while a command
# runs (diagnostic: is a measurement power- or clock-limited?).
#   tools/smi_watch.sh OUT.log -- cmd args...
out=$1; shift; [ "$1" = "--" ] && shift
( while true; do
    echo "t=$(date +%s.%N)" >> "$out"
    rocm-smi -d 0 -g -P 2>/dev/null | grep -E "sclk|Power|power" >> "$out"
    sleep 0.5
  done ) &
w=$!
"$@"
rc=$?
kill $w 2>/dev/null
wait $w 2>/dev/null
exit $rc
