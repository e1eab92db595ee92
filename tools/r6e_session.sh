#!/bin/bash
# Round-4 session E: the C2 loss fixed? (r3 vs HEAD), trace-group sweep at R = 8 / 4 on the fixed kernel.
export VNAMES="r3 base" VROUNDS=3
export HPARTS="8 4" HROUNDS=2
export HSETS='--sets default;tg=2;tg=4;tg=2,tsolo=6;tg=4,tsolo=6;tg=4,tsolo=6,a1s=1.6,a1l=2.0;tg=4,tsolo=4,a1s=1.6,a1l=2.0;tg=4,prs=200,prl=300;tg=4,tsolo=6,prs=300,prl=300;tg=2,tsolo=6,a1s=2.0,a1l=2.4,prs=400,prl=400;tg=4,tsolo=6,a1s=1.6,a1l=2.0,trs=0.35,trl=0.3;tg=8,tsolo=4,a1s=1.4,a1l=1.8'
bash tools/gpu_session.sh R6e variants hsweep parts
