#!/bin/bash
# GPU-box: device time of the configs[1] batch at fixed per-phase window sizes.
cd "$(dirname "$0")/.." || exit 1
for x in 8388608 10000000 12000000 6000000; do
  echo "X=$x Y=8388608"; GNOC_WINDOW_PS_X=$x GNOC_WINDOW_PS_Y=8388608 timeout -k 10 100 python -u tools/window_trace.py 3 | tail -n 1 || exit 1
done
for y in 7000000 9500000; do
  echo "X=8388608 Y=$y"; GNOC_WINDOW_PS_X=8388608 GNOC_WINDOW_PS_Y=$y timeout -k 10 100 python -u tools/window_trace.py 3 | tail -n 1 || exit 1
done
