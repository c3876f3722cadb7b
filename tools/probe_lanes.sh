#!/bin/bash
# frame time vs the k_generate lane budget (diagnostic)
for L in 65536 262144 1048576 4194304 16777216; do
  echo "lanes=$L"; NGP_RENDER_LANES=$L TIMER_MASK=0 python tools/probe_render.py 1500 | grep "cap=  32"
done
