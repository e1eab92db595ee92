#!/bin/bash
# Round-4 session J: schedule sweep around the R6i best, R = 8 / 4 / 2.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/R6j; mkdir -p $OUT
B="tg=4,tsolo=6,a1s=1.6,a1l=2.0,trs=0.35,trl=0.3"
timeout -k 10 800 python tools/heavy_sweep.py --parts 8 4 2 --rounds 2 --sets "default;$B,prs=300,prl=300;$B,prs=200,prl=200;$B,prs=400,prl=400;$B,prs=300,prl=300,p1=2;$B,prs=150,prl=300;tg=4,tsolo=6,a1s=1.8,a1l=2.2,trs=0.35,trl=0.3,prs=200,prl=250;tg=4,tsolo=5,a1s=1.6,a1l=2.0,trs=0.3,trl=0.25,prs=300,prl=300;$B,prs=300,prl=300,a2s=3.0;$B,prs=300,prl=300,trm=0.15,prm=400;$B,prs=300,prl=300,trm=0.25,prm=300,a1=1.6;$B,prs=300,prl=300,coop=16" > $OUT/hsweep.jsonl 2>&1
echo "session J rc=$?"
