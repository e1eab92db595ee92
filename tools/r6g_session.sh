#!/bin/bash
# Round-4 session G: compile-time group sizes in k_trace; GPU tests; R = 8 / 4 sweep; parts.
export HPARTS="8 4" HROUNDS=2
export HSETS='--sets default;tg=2,tsolo=6;tg=4,tsolo=6;tg=4,tsolo=6,trs=0.35,trl=0.3;tg=4,tsolo=6,a1s=1.6,a1l=2.0,trs=0.35,trl=0.3;tg=4,tsolo=8,a1s=1.4,a1l=2.0,trs=0.4,trl=0.3;tg=2,tsolo=6,a1s=2.0,a1l=2.4,trs=0.3,trl=0.25;tg=4,tsolo=6,a1s=1.6,a1l=2.0,trs=0.35,trl=0.3,a2s=1.3;tg=4,tsolo=6,a1s=1.6,a1l=2.0,trs=0.35,trl=0.3,prs=300,prl=300;tg=4,tsolo=5,a1s=1.8,a1l=2.2,trs=0.3,trl=0.3'
bash tools/gpu_session.sh R6g tests hsweep parts
