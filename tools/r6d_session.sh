#!/bin/bash
# Round-4 session D: bisect the C2 loss (round-3 tree r3 vs HEAD with single changes reverted).
export VNAMES="r3 base noP3 noflag oldtp all" VROUNDS=3
bash tools/gpu_session.sh R6d variants
