#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
TAIL=9 step dbg_none 300 python -u tools/dbg_graph_step2.py
TAIL=9 step dbg_zero 300 python -u tools/dbg_graph_step2.py zero
TAIL=9 PADDLE_AMD_ALLOCATOR=auto_growth step dbg_native 300 python -u tools/dbg_graph_step2.py
