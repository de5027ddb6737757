#!/bin/bash
# Roofline evidence for one workload on the GPU box (run from the repo root):
# kernel stats + PMC traffic (tools/profile_c2.sh), SQ VALU counts
# (tools/pmc_valu.sh), both summaries copied into profiles/ (so that the bench
# line below quotes them), then the bench line itself.
#   tools/evidence.sh TAG WORKLOAD [exact|closed] [shift|fft] [bench args...]
#   -> profiles/<round>_<wl>[c][fft]_pmc_{traffic,valu}_TAG.json,
#      gpurun_out/evidence_TAG/{<key>.json, kernel_stats_<key>.csv, pmc_valu_summary_<key>.txt}
#   <round> = $IC_ROUND (default r05)
set -o pipefail
TAG=${1:?tag}; WL=${2:?workload}; FM=${3:-exact}; DD=${4:-shift}; shift 4
RND=${IC_ROUND:-r05}
lc=$(echo $WL | tr A-Z a-z); [ "$FM" = closed ] && lc=${lc}c; [ "$DD" != shift ] && lc=${lc}${DD/_/}
OUT=gpurun_out/evidence_$TAG
mkdir -p $OUT
tools/profile_c2.sh ${TAG}_$lc $WL $FM $DD || exit 1
tools/pmc_valu.sh ${TAG}_$lc $WL $FM $DD || exit 1
cp gpurun_out/prof_${TAG}_$lc/pmc_traffic.json profiles/${RND}_${lc}_pmc_traffic_$TAG.json
cp gpurun_out/valu_${TAG}_$lc/pmc_valu.json profiles/${RND}_${lc}_pmc_valu_$TAG.json
cp gpurun_out/prof_${TAG}_$lc/kernel_stats.csv $OUT/kernel_stats_$lc.csv
cp gpurun_out/valu_${TAG}_$lc/summary.txt $OUT/pmc_valu_summary_$lc.txt
timeout -k 10 400 python3 bench.py --workload $WL --fit-mode $FM --dedisp $DD "$@" > $OUT/$lc.json 2> $OUT/$lc.err \
    || { tail -5 $OUT/$lc.err; exit 1; }
echo "evidence $WL $FM $DD done"
