#!/bin/bash
# Round-4 session B: trace-group tests, promotion-rate A/B at C2, trace-group sweep at R = 8 / 4,
# C2 / C5 bench lines with the stall breakdown, the C5 LDS-DMA ring A/B.
export VNAMES="promR promE" VROUNDS=4
export HPARTS="8 4" HROUNDS=2
export HSETS='--sets default;tg=2;tg=4;tg=2,a1s=2.0,a1l=2.4;tg=4,a1s=1.6,a1l=2.0;tg=2,prs=300,prl=400;tg=4,prs=200,prl=300;tg=4,a1s=1.6,a1l=2.0,prs=200,prl=300;tg=2,tsolo=6;tg=4,tsolo=6,a1s=1.6,a1l=2.0;tg=2,capS=16;tg=4,capS=16;tg=4,capS=8,prs=300,prl=400'
export C5V="base ring2 ring3c16 ring4c16"
bash tools/gpu_session.sh R6b tests variants hsweep bench c5b c5
